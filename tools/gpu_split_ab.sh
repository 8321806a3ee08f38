#!/bin/bash
# Lone-call latency forms, same box: two lanes per set in k_sm_prepare<true> (GBV_PREPARE_SPLIT_MAX)
# and the cooperative cofactor clearing of few-message hashing (GBV_HASH_COOP_MAX), each on/off;
# parity on both, then the latency probe and a bench line per configuration.
set -o pipefail
OUT=gpurun_out/split
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_c5.py tests/test_gpu_single_thread.py tests/test_addon.py tests/test_ssz.py -m gpu > "$OUT/test.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/test.log"; exit 1; }
tail -1 "$OUT/test.log"
for v in off split coop both off split coop both; do
  case $v in
    off) export GBV_PREPARE_SPLIT_MAX=0 GBV_HASH_COOP_MAX=0 ;;
    split) export GBV_PREPARE_SPLIT_MAX=2048 GBV_HASH_COOP_MAX=0 ;;
    coop) export GBV_PREPARE_SPLIT_MAX=0 GBV_HASH_COOP_MAX=256 ;;
    both) export GBV_PREPARE_SPLIT_MAX=2048 GBV_HASH_COOP_MAX=256 ;;
  esac
  timeout -k 10 120 python3 -u tools/latency_probe.py > "$OUT/lat_$v.txt" 2>&1 || { echo "probe $v failed"; tail -20 "$OUT/lat_$v.txt"; exit 1; }
  timeout -k 10 240 python3 -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-signing-roots > "$OUT/$v.json" 2> "$OUT/$v.err" || { echo "bench $v failed"; tail -20 "$OUT/$v.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$v.json')); print('$v', round(d['value']/1e6,3), 'p50', d['p50_batch_latency_ms'], 'api', d.get('api_path_sets_per_s'))"
  grep "^call" "$OUT/lat_$v.txt" | sed -n 2,3p
done
