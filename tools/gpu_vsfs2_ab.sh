#!/bin/bash
# chunk-count bound of the (-g1, sum) Miller value beside the per-set ones: 0 (small passes only)
# vs the default (256 chunks: C4 segments) vs 1024 (C1/C3 512-chunk passes too).
set -o pipefail
OUT=gpurun_out/vsfs2
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_c3.py tests/test_block_sets.py tests/test_gpu_scale.py -m gpu > "$OUT/test.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/test.log"; exit 1; }
tail -1 "$OUT/test.log"
for v in 0 256 1024 0 256 1024; do
  export GBV_VS_FS_MAXC=$v
  timeout -k 10 240 python3 -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-signing-roots > "$OUT/$v.json" 2> "$OUT/$v.err" || { echo "bench $v failed"; tail -20 "$OUT/$v.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$v.json')); print('$v', round(d['value']/1e6,3), 'c1', d['c1']['value'], d['c1'].get('throughput_value'), 'c3', d['c3']['value'], 'c4', d['c4']['value'], d['c4']['lone_block_latency_ms_p50'], d['c4']['roofline']['kernel_ms_per_pass'])"
done
