#!/bin/bash
# Same-box A/B of library variants, the GPU parity suite on the IN-TREE library first:
#   bash tools/gpu_ab4.sh TAG V1 [V2 ...]   (variants from tools/build_variant.sh; "base" = in-tree lib)
# Each variant's bench runs twice, interleaved (base V1 V2 .. base V1 V2 ..).
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/test_base.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/test_base.log"; exit 1; }
tail -1 "$OUT/test_base.log"
for v in base "$@" base "$@"; do
  if [ "$v" = base ]; then lib=""; else lib=lodestar_amd/variants/libgbv_$v.so; fi
  LODESTAR_AMD_LIB=$lib timeout -k 10 300 python3 -u bench.py --steps 8 --warmup 1 --no-cpu-baseline --no-signing-roots ${AB_ARGS:-} > "$OUT/$v.json" 2> "$OUT/$v.err" || { echo "bench $v failed"; tail -20 "$OUT/$v.err"; exit 1; }
  python3 - "$OUT/$v.json" "$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); g = lambda k: (d.get(k) or {}).get("value")
k = d["roofline"]["kernel_ms_per_step"]
print(sys.argv[2], "C2 %.3fM" % (d["value"] / 1e6), "frac", d["roofline"]["frac"], "ms/step", d["ms_per_step"], "prep", k["prepare"], "msm", k["msm"], "p50", d.get("p50_batch_latency_ms"),
      "c1", g("c1"), "c3", g("c3"), "c4", g("c4"), "c5", g("c5"), "api", d.get("api_path_sets_per_s"), "oneshot", (d.get("api_path") or {}).get("oneshot_sets_per_s"))
PY
done
