#!/bin/bash
# Same-box A/B of the small-pass cooperative signature roles (GBV_VS_PRE_COOP=0 turns them off), after the GPU suite.
set -o pipefail
OUT=gpurun_out/ab_vscoop; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for v in 256 0 256 0; do  # 256: on for passes of <= 256 sets
  GBV_VS_PRE_COOP=$v timeout -k 10 120 python -u tools/latency_probe.py > $OUT/lat_$v.txt 2>&1 || { tail -20 $OUT/lat_$v.txt; exit 1; }
  python3 - $OUT/lat_$v.txt $v <<'PY'
import re, statistics, sys
t = open(sys.argv[1]).read().splitlines()
ms = lambda pre: [float(re.match(pre + r" ([0-9.]+) ms", l).group(1)) for l in t if re.match(pre + r" [0-9.]+ ms", l)]
hs = [float(re.search(r"'hash_sig': ([0-9.]+)", l).group(1)) for l in t if l.startswith("c1 call")]
print("vs_pre_coop", sys.argv[2], "lone p50 %.2f" % statistics.median(ms("call")), "c1 %s" % ms("c1 call"), "c1 hash_sig %s" % hs,
      "c4 %.2f" % statistics.median(ms("c4 block")), "c4e %.2f" % statistics.median(ms("c4e block")))
PY
done
