#!/bin/bash
# verifySignatureSets small passes: hash on its own stream + split signature roles (default) vs one
# k_vs_hash_sig launch (GBV_VS_SPLIT=0); parity, then the C1 lone-call latency and bench lines.
set -o pipefail
OUT=gpurun_out/vssplit
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_c3.py tests/test_block_sets.py tests/test_gpu_sharded.py tests/test_addon.py tests/test_reference_vectors.py tests/test_gpu_single_thread.py -m gpu > "$OUT/test.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/test.log"; exit 1; }
tail -1 "$OUT/test.log"
for v in 0 1 0 1; do
  export GBV_VS_SPLIT=$v
  timeout -k 10 120 python3 -u tools/latency_probe.py > "$OUT/lat_$v.txt" 2>&1 || { echo "probe $v failed"; tail -20 "$OUT/lat_$v.txt"; exit 1; }
  timeout -k 10 240 python3 -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-signing-roots > "$OUT/$v.json" 2> "$OUT/$v.err" || { echo "bench $v failed"; tail -20 "$OUT/$v.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$v.json')); print('$v', round(d['value']/1e6,3), 'p50', d['p50_batch_latency_ms'], 'c1', d['c1']['value'], d['c1']['latency_ms_p50'], d['c1'].get('throughput_value'), 'c3', d['c3']['value'], 'c4', d['c4']['value'], d['c4']['lone_block_latency_ms_p50'])"
  grep "^c1 call" "$OUT/lat_$v.txt" | sed -n 2,3p
done
