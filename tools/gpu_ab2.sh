#!/bin/bash
# Same-box A/B of the default library and one variant: C2 bench lines only (no tests).
# Usage (repo root, via gpurun): bash tools/gpu_ab2.sh TAG VARIANT_SO
set -o pipefail
TAG=$1; VAR=$2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
summ() {
python3 - "$1" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["roofline"]
print("%s: C2 %.3fM sets/s  ms/step %.2f  p50 %.2f  prepare %.2f ms  frac %.3f  %s" % (sys.argv[1], d["value"] / 1e6, d["ms_per_step"], d["p50_batch_latency_ms"], r["avg_launch_ms"], r["frac"], r.get("kernel_ms_per_step")))
PY
}
for rep in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-signing-roots --no-extras > "$OUT/base$rep.json" 2> "$OUT/base$rep.err" || { echo "base bench failed"; tail -20 "$OUT/base$rep.err"; exit 1; }
summ "$OUT/base$rep.json"
LODESTAR_AMD_LIB=$VAR timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-signing-roots --no-extras > "$OUT/var$rep.json" 2> "$OUT/var$rep.err" || { echo "variant bench failed"; tail -20 "$OUT/var$rep.err"; exit 1; }
summ "$OUT/var$rep.json"
done
