#!/bin/bash
# Failure-path pairing checks at one wave per SIMD (k_sm_fb.hip, GBV_FB_WPE=1, this tree) against
# two for all three (lodestar_amd/variants/libgbv_fb2.so); this tree: group check at one wave, run / set checks at two.
set -o pipefail
O=gpurun_out/r05t; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
c5() { timeout -k 10 200 env LODESTAR_AMD_LIB=$2 python -u tools/c5_probe.py > $O/c5_$1.txt 2>&1 || { echo "c5 $1 failed"; tail -5 $O/c5_$1.txt; exit 1; }; grep "^C5\|fb_\|group_check" $O/c5_$1.txt | sed "s/^/$1: /"; }
W2=lodestar_amd/variants/libgbv_fb2.so; W1=lodestar_amd/libgbv.so
c5 w2a $W2 && c5 w1a $W1 && c5 w2b $W2 && c5 w1b $W1
