#!/bin/bash
# Fp2 products as one out-of-line call with three inline Fp products (GBV_FP2_IMPL=0,
# lodestar_amd/variants/libgbv_fp2i0.so) against the default (Karatsuba over out-of-line Fp
# products): GPU parity on the variant, then the full bench alternated.
set -o pipefail
O=gpurun_out/r05zb; mkdir -p $O
V=lodestar_amd/variants/libgbv_fp2i0.so; B=lodestar_amd/libgbv.so
timeout -k 10 300 env LODESTAR_AMD_LIB=$V python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_i0.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_i0.log; exit 1; }
tail -1 $O/pytest_i0.log
b() { timeout -k 10 400 env LODESTAR_AMD_LIB=$2 python -u bench.py --no-cpu-baseline > $O/bench_$1.json 2> $O/bench_$1.err || { echo "bench $1 failed"; tail -5 $O/bench_$1.err; exit 1; }; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], 'C2', d['value'], 'frac', r['frac'], [(k['kernel'], k['ms']) for k in r['stage_kernels']], 'C1', d['c1']['throughput_value'], 'C3', d['c3']['value'], 'C4', d['c4']['value'], 'C5', d['c5']['value'])" $O/bench_$1.json $1; }
b base1 $B && b i0a $V && b base2 $B && b i0b $V
