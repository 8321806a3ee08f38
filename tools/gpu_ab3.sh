#!/bin/bash
# A/B/C of an env knob over the bench's verifySignatureSets lines (C1/C3/C4/C4e), then extra steps.
# Usage (via gpurun): bash tools/gpu_ab3.sh tag VAR val1 val2 val3
set -o pipefail
TAG=$1; VAR=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for val in "$@"; do
  timeout -k 10 300 env $VAR=$val python -u bench.py --steps 4 --no-cpu-baseline --no-signing-roots > "$OUT/bench_$val.json" 2> "$OUT/bench_$val.err" || { echo "bench $val failed"; tail -30 "$OUT/bench_$val.err"; exit 1; }
done
python3 - "$OUT" "$@" <<'PY'
import json, sys
for val in sys.argv[2:]:
    d = json.load(open(sys.argv[1] + "/bench_%s.json" % val))
    print(val, "C2 %.2fM" % (d["value"] / 1e6))
    for c in ("c1", "c3", "c4", "c4e"):
        x = d.get(c) or {}
        r = x.get("roofline", {})
        print("  %s %.0f" % (c, x.get("value", 0)), r.get("kernel"), r.get("frac"), r.get("kernel_ms_per_pass"))
PY
