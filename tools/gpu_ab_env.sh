#!/bin/bash
# Same-box A/B over environment settings: one C2 bench line (no tests, no extras) per setting.
# Usage (repo root, via gpurun): bash tools/gpu_ab_env.sh TAG "ENV=... [ENV2=...]" "..."  ("-" = defaults)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for setting in "$@"; do
  i=$((i + 1))
  envs=""; [ "$setting" != "-" ] && envs="$setting"
  env $envs timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-signing-roots ${AB_EXTRAS:---no-extras} ${AB_ARGS:-} > "$OUT/run$i.json" 2> "$OUT/run$i.err" || { echo "bench failed ($setting)"; tail -20 "$OUT/run$i.err"; exit 1; }
  python3 - "$OUT/run$i.json" "$setting" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["roofline"]
k = r.get("kernel_ms_per_step", {})
for c in ("c1", "c3", "c4"):
    if d.get(c):
        print("   %s %.0f sets/s (throughput %s) %s" % (c, d[c]["value"], d[c].get("throughput_value"), d[c]["roofline"].get("kernel_ms_per_pass")))
print("[%s] C2 %.3fM sets/s  ms/step %.2f  p50 %.2f  prepare %.2f  msm %.2f  miller %.2f  seg_check %.2f  hash %.2f" % (sys.argv[2], d["value"] / 1e6, d["ms_per_step"], d["p50_batch_latency_ms"], r["avg_launch_ms"], k.get("msm", 0), k.get("miller", 0), k.get("seg_check", 0), k.get("hash", 0)))
PY
done
