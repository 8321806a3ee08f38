#!/bin/bash
# Quick A/B on the GPU: fast parity subset, then a C2 bench line (no CPU leg, no signing roots).
# Usage (repo root, via gpurun): bash tools/gpu_ab.sh TAG [extra bench args]
set -o pipefail
TAG=${1:-ab}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_single_thread.py > "$OUT/test.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/test.log"; exit 1; }
tail -1 "$OUT/test.log"
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-signing-roots "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
python3 - "$OUT/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["roofline"]
print("C2 %.3fM sets/s  ms/step %.2f  p50 %.2f  prepare %.2f ms  frac %.3f" % (d["value"] / 1e6, d["ms_per_step"], d["p50_batch_latency_ms"], r["avg_launch_ms"], r["frac"]))
print("kernel ms/step", r.get("kernel_ms_per_step"))
for k in ("c1", "c3", "c4"):
    if k in d:
        print(k, d[k]["value"], d[k].get("throughput_value"), d[k]["roofline"].get("kernel_ms_per_pass"))
PY
