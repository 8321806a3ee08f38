#!/bin/bash
# Same-box A/B of configurations, each "name=variant[:bench args]" ("base" = the in-tree library, else
# lodestar_amd/variants/libgbv_<variant>.so from tools/build_variant.sh), bench runs interleaved twice,
# after the GPU parity suite on the in-tree library (skipped with NO_TESTS=1):
#   bash tools/gpu_ab5.sh TAG "base=base" "hq0=base:--tune hash_quad_max=0" "canon=canon3"
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/test_base.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/test_base.log"; exit 1; }
  tail -1 "$OUT/test_base.log"
fi
for rep in 1 2; do
  for cfg in "$@"; do
    name=${cfg%%=*}; rest=${cfg#*=}; var=${rest%%:*}; args=""
    [ "$rest" != "$var" ] && args=${rest#*:}
    if [ "$var" = base ]; then lib=""; else lib=lodestar_amd/variants/libgbv_$var.so; fi
    LODESTAR_AMD_LIB=$lib timeout -k 10 300 python3 -u bench.py --steps 8 --warmup 1 --no-cpu-baseline --no-signing-roots ${AB_ARGS:-} $args \
      > "$OUT/${name}_$rep.json" 2> "$OUT/${name}_$rep.err" || { echo "bench $name failed"; tail -20 "$OUT/${name}_$rep.err"; exit 1; }
    python3 - "$OUT/${name}_$rep.json" "$name" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); g = lambda k: (d.get(k) or {}).get("value")
st = {k["kernel"]: k["ms"] for k in d["roofline"]["last_step_kernels"]}
print("%-10s C2 %.3fM frac %.3f ms/step %.2f dec %.2f prep %.2f miller %.2f hash %.2f msm_runs %.2f | c1 %s c3 %s c4 %s c5 %s" % (
    sys.argv[2], d["value"] / 1e6, d["roofline"]["frac"], d["ms_per_step"], st.get("k_sig_decode", 0), st.get("k_sm_prepare<false>", 0),
    st.get("k_sm_miller", 0), st.get("k_hash_clear_quad", 0) + st.get("k_hash_msgs_pre", 0) + st.get("k_hash_msgs", 0), st.get("k_msm_runs", 0),
    g("c1"), g("c3"), g("c4"), g("c5")))
PY
  done
done
