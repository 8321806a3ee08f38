#!/bin/bash
# Passes in flight (the verifier allows MAX_PASSES_IN_FLIGHT = 3): C1 / C3 65 536-set passes and the
# C4 64-block segments at 2 and 3, alternated.
set -o pipefail
O=gpurun_out/r05x; mkdir -p $O
vs() { timeout -k 10 240 python -u tools/vs_probe.py --steps 9 --depths $2 > $O/vs_$1.txt 2>&1 || { echo "vs $1 failed"; tail -5 $O/vs_$1.txt; exit 1; }; grep "^C" $O/vs_$1.txt | sed "s/^/$1: /"; }
c4() { timeout -k 10 240 python -u tools/c4_probe.py --depth $2 > $O/c4_$1.txt 2>&1 || { echo "c4 $1 failed"; tail -5 $O/c4_$1.txt; exit 1; }; grep "^C4" $O/c4_$1.txt | sed "s/^/$1: /"; }
vs a 2,3 && vs b 3,2 && c4 d2a 2 && c4 d3a 3 && c4 d2b 2 && c4 d3b 3
