#!/bin/bash
# Electra blocks (C4e, 16-block segments) at 2 and 3 passes in flight, alternated.
set -o pipefail
O=gpurun_out/r05y; mkdir -p $O
c4() { timeout -k 10 240 python -u tools/c4_probe.py --electra --depth $2 > $O/c4e_$1.txt 2>&1 || { echo "c4e $1 failed"; tail -5 $O/c4e_$1.txt; exit 1; }; grep "^C4" $O/c4e_$1.txt | sed "s/^/$1: /"; }
c4 d2a 2 && c4 d3a 3 && c4 d2b 2 && c4 d3b 3
