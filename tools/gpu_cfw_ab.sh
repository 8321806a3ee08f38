#!/bin/bash
# Wave-per-chunk chunk_finish for small segments (default) vs the thread-per-chunk kernel
# (GBV_CHUNK_FINISH_WAVE_MAX=0): same-message parity, then the lone-call latency.
set -o pipefail
OUT=gpurun_out/cfw
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_c5.py tests/test_gpu_single_thread.py -m gpu > "$OUT/test.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/test.log"; exit 1; }
tail -1 "$OUT/test.log"
for v in 0 32 0 32; do
  export GBV_CHUNK_FINISH_WAVE_MAX=$v
  timeout -k 10 120 python3 -u tools/latency_probe.py > "$OUT/lat_$v.txt" 2>&1 || { echo "probe $v failed"; tail -20 "$OUT/lat_$v.txt"; exit 1; }
  timeout -k 10 240 python3 -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-signing-roots > "$OUT/$v.json" 2> "$OUT/$v.err" || { echo "bench $v failed"; tail -20 "$OUT/$v.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$v.json')); print('$v', round(d['value']/1e6,3), 'p50', d['p50_batch_latency_ms'], 'c1', d['c1']['value'], 'c4', d['c4']['value'])"
  grep "^call" "$OUT/lat_$v.txt" | head -3
done
