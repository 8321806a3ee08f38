#!/bin/bash
# C1 / C3 65 536-set passes (512 chunks) with each chunk's (-g1, sum) Miller value formed beside the
# per-set ones (gbv_tune vs_fs_maxc=1024) against the default (inside the chunk check), alternated.
set -o pipefail
O=gpurun_out/r05zd; mkdir -p $O
vs() { timeout -k 10 240 python -u tools/vs_probe.py --steps 9 "${@:2}" > $O/vs_$1.txt 2>&1 || { echo "vs $1 failed"; tail -5 $O/vs_$1.txt; exit 1; }; grep "^C" $O/vs_$1.txt | sed "s/^/$1: /"; }
vs base_a && vs fs_a --tune vs_fs_maxc=1024 && vs base_b && vs fs_b --tune vs_fs_maxc=1024
