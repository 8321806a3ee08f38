#!/bin/bash
# GPU tests, then the bench (C2 + c1/c3/c4 lines) with the default Miller kernel and with an env
# variant (A/B).  Usage (via gpurun): bash tools/gpu_ab_vs.sh tag "ENV=val" [skip-tests]
set -o pipefail
TAG=${1:-ab}
VAR=${2:-GBV_VS_MILLER=thread}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -z "$3" ]; then
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
fi
timeout -k 10 300 python -u bench.py --steps 6 --no-cpu-baseline --no-signing-roots > "$OUT/bench_a.json" 2> "$OUT/bench_a.err" || { echo "bench A failed"; tail -30 "$OUT/bench_a.err"; exit 1; }
timeout -k 10 300 env $VAR python -u bench.py --steps 6 --no-cpu-baseline --no-signing-roots > "$OUT/bench_b.json" 2> "$OUT/bench_b.err" || { echo "bench B failed"; tail -30 "$OUT/bench_b.err"; exit 1; }
python3 - "$OUT" <<'PY'
import json, sys
for k in ("a", "b"):
    d = json.load(open(sys.argv[1] + "/bench_%s.json" % k))
    print(k, "C2 %.2fM" % (d["value"] / 1e6), "p50 %.1f" % d["p50_batch_latency_ms"],
          "C1 %.0f thr %.2fM" % (d["c1"]["value"], d["c1"]["throughput_value"] / 1e6), d["c1"]["roofline"]["kernel_ms_per_pass"],
          "C3 %.2fM" % (d["c3"]["value"] / 1e6), d["c3"]["roofline"]["kernel_ms_per_pass"],
          "C4 %.0fk" % (d["c4"]["value"] / 1e3), d["c4"]["roofline"]["kernel_ms_per_pass"])
PY
