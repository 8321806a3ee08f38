#!/bin/bash
# Two-wave chunk check (k_sm_group_miller2 + k_sm_group_fe) vs the one-wave k_sm_group_pairing
# (GBV_GROUP_PAIRING_1W=1): parity on the new path, then latency probe and bench lines for both.
set -o pipefail
OUT=gpurun_out/gp2
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_c5.py tests/test_gpu_single_thread.py tests/test_addon.py -m gpu > "$OUT/test.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/test.log"; exit 1; }
tail -1 "$OUT/test.log"
for v in 1w 2w 1w 2w; do
  if [ "$v" = 1w ]; then export GBV_GROUP_PAIRING_1W=1; else unset GBV_GROUP_PAIRING_1W; fi
  timeout -k 10 120 python3 -u tools/latency_probe.py > "$OUT/lat_$v.txt" 2>&1 || { echo "probe $v failed"; tail -20 "$OUT/lat_$v.txt"; exit 1; }
  timeout -k 10 240 python3 -u bench.py --steps 6 --warmup 1 --no-cpu-baseline --no-signing-roots > "$OUT/$v.json" 2> "$OUT/$v.err" || { echo "bench $v failed"; tail -20 "$OUT/$v.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$v.json')); print('$v', round(d['value']/1e6,3), 'p50', d['p50_batch_latency_ms'], 'c1', d.get('c1',{}).get('value'), 'c4', d.get('c4',{}).get('value'))"
  grep "^call" "$OUT/lat_$v.txt" | head -3
done
