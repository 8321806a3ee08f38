#!/bin/bash
# C1 / C3 65 536-set pass: hash-role launch forms (lane quads / pairs) and the signature half on
# quads beside the aggregation, against the default thread forms (same box).
set -o pipefail
O=gpurun_out/r05p; mkdir -p $O
run() { local tag=$1; shift; timeout -k 10 240 python -u tools/vs_probe.py --steps 9 "$@" > $O/$tag.txt 2>&1 || { echo "$tag failed"; tail -5 $O/$tag.txt; exit 1; }; grep "^C" $O/$tag.txt | sed "s/^/$tag: /"; }
run base
run hpair --tune hash_pair_max=65536
run vspre --tune vs_pre_max=65536
run vspreq --tune vs_pre_max=65536 --tune hash_quad_max=65536
run base2
