#!/bin/bash
# Same-box A/B of library variants: bench (C2/C3/C4/C5 lines) and the lone-call latency probe.
#   bash tools/gpu_chain_ab.sh TAG V1 [V2 ...]   ("base" = in-tree lib)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
# full GPU parity suite on the in-tree library (the candidate default)
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/test_base.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/test_base.log"; exit 1; }
tail -n 1 "$OUT/test_base.log"
for v in base "$@"; do
  if [ "$v" = base ]; then lib=""; else lib=lodestar_amd/variants/libgbv_$v.so; fi
  LODESTAR_AMD_LIB=$lib timeout -k 10 200 python3 -u tools/latency_probe.py > "$OUT/lat_$v.log" 2>&1 || { echo "probe $v failed"; tail -20 "$OUT/lat_$v.log"; exit 1; }
  python3 - "$OUT/lat_$v.log" "$v" <<'PY'
import re, sys, statistics as st
rows = {}
for line in open(sys.argv[1]):
    m = re.match(r"(call|bad call|c1 call|c4 block|c4e block) ([\d.]+) ms", line)
    if m: rows.setdefault(m.group(1), []).append(float(m.group(2)))
print(sys.argv[2], "lat p50", {k: round(st.median(v[1:]), 2) for k, v in rows.items()})
PY
done
for v in base "$@" base "$@"; do
  if [ "$v" = base ]; then lib=""; else lib=lodestar_amd/variants/libgbv_$v.so; fi
  LODESTAR_AMD_LIB=$lib timeout -k 10 300 python3 -u bench.py --steps 8 --warmup 1 --no-cpu-baseline --no-signing-roots > "$OUT/$v.json" 2> "$OUT/$v.err" || { echo "bench $v failed"; tail -20 "$OUT/$v.err"; exit 1; }
  python3 - "$OUT/$v.json" "$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); g = lambda k: (d.get(k) or {}).get("value")
print(sys.argv[2], round(d["value"] / 1e6, 3), "p50", d.get("p50_batch_latency_ms"), "c1", g("c1"), "c3", g("c3"), "c4", g("c4"), "c4e", g("c4e"), "c5", g("c5"), "api", (d.get("api_path") or {}).get("value"))
PY
done
