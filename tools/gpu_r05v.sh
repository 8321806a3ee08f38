#!/bin/bash
# k_vs_hash_sig roles alternating by block (this tree) against hash blocks first
# (lodestar_amd/variants/libgbv_hs0.so): C3 GPU tests, then C1 / C3 alternated.
set -o pipefail
O=gpurun_out/r05v; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_c3.py tests/test_gpu_scale.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
vs() { timeout -k 10 200 env LODESTAR_AMD_LIB=$2 python -u tools/vs_probe.py --steps 9 > $O/vs_$1.txt 2>&1 || { echo "vs $1 failed"; tail -5 $O/vs_$1.txt; exit 1; }; grep "^C\|hash_sig" $O/vs_$1.txt | sed "s/^/$1: /"; }
A=lodestar_amd/variants/libgbv_hs0.so; B=lodestar_amd/libgbv.so
vs first_a $A && vs alt_a $B && vs first_b $A && vs alt_b $B
