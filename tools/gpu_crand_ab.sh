#!/bin/bash
# Same-box A/B of the lone-call prepare's cooperative r sig role (GBV_PREP_COOP_RAND), after the GPU suite.
# (profiles/r03_ab/ab_crand/ ran it as an on/off switch, before the knob became a pass-size bound.)
set -o pipefail
OUT=gpurun_out/ab_crand; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for v in 512 0 512 0; do  # GBV_PREP_COOP_RAND: the largest pass (sets) given the cooperative r sig; 0 = off
  GBV_PREP_COOP_RAND=$v timeout -k 10 120 python -u tools/latency_probe.py > $OUT/lat_$v.txt 2>&1 || { tail -20 $OUT/lat_$v.txt; exit 1; }
  python3 - $OUT/lat_$v.txt $v <<'PY'
import re, statistics, sys
t = open(sys.argv[1]).read().splitlines()
ms = lambda pre: [float(re.match(pre + r" ([0-9.]+) ms", l).group(1)) for l in t if re.match(pre + r" [0-9.]+ ms", l)]
prep = [float(re.search(r"'prepare': ([0-9.]+)", l).group(1)) for l in t if l.startswith("call ")]
print("coop_rand", sys.argv[2], "lone p50 %.2f" % statistics.median(ms("call")), "prepare p50 %.2f" % statistics.median(prep),
      "bad %s" % ms("bad call"), "fallback", [re.search(r"'fallback': ([0-9.]+)", l).group(1) for l in t if l.startswith("call ")][:6])
PY
done
