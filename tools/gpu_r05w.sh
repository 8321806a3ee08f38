#!/bin/bash
# Same-box A/B of the merged line products in the thread-form Miller loops: the previous tree's
# (lodestar_amd/variants/libgbv_old.so) against the current one, alternated, C5 then C1 / C3.
set -o pipefail
O=gpurun_out/r05w; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
c5() { timeout -k 10 200 env LODESTAR_AMD_LIB=$2 python -u tools/c5_probe.py > $O/c5_$1.txt 2>&1 || { echo "c5 $1 failed"; tail -5 $O/c5_$1.txt; exit 1; }; grep "^C5" $O/c5_$1.txt | sed "s/^/$1: /"; }
vs() { timeout -k 10 200 env LODESTAR_AMD_LIB=$2 python -u tools/vs_probe.py --steps 9 > $O/vs_$1.txt 2>&1 || { echo "vs $1 failed"; tail -5 $O/vs_$1.txt; exit 1; }; grep "^C" $O/vs_$1.txt | sed "s/^/$1: /"; }
OLD=lodestar_amd/variants/libgbv_old.so; NEW=lodestar_amd/libgbv.so
c5 old1 $OLD && c5 new1 $NEW && c5 old2 $OLD && c5 new2 $NEW && vs old $OLD && vs new $NEW
