#!/bin/bash
# few-item per-set checks (and the lone-call chunk check) on two waves (default) vs one
# (GBV_GROUP_PAIRING_1W=1): parity, then the lone valid / one-invalid call latency.
set -o pipefail
OUT=gpurun_out/fbsplit
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_c5.py tests/test_gpu_single_thread.py tests/test_addon.py -m gpu > "$OUT/test.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/test.log"; exit 1; }
tail -1 "$OUT/test.log"
for v in 1 0 1 0; do
  export GBV_GROUP_PAIRING_1W=$v
  timeout -k 10 120 python3 -u tools/latency_probe.py > "$OUT/lat_$v.txt" 2>&1 || { echo "probe $v failed"; tail -20 "$OUT/lat_$v.txt"; exit 1; }
  echo "1w=$v"; grep "^bad call" "$OUT/lat_$v.txt" | sed -n 2,4p
done
