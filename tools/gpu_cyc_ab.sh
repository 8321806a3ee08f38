#!/bin/bash
# Same-box A/B of a cooperative-engine change against a variant library (tools/build_variant.sh;
# round 4: the written-out cyclotomic squaring against -DGBV_COOP_CYC_HAND=0, the written-out line
# product against -DGBV_COOP_LINE_HAND=0): the one-wave microbenchmark, the GPU parity suite on the
# in-tree library, then lone-call latency and the small verifySignatureSets probe on both.
#   bash tools/gpu_cyc_ab.sh TAG VARIANT
set -o pipefail
TAG=${1:-cyc}
VAR=${2:-cycold}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 tools/ubench_coop > "$OUT/ubench_new.txt" 2>&1 || { echo "ubench failed"; exit 1; }
grep -E "cyc|FE|ML1|miller1" "$OUT/ubench_new.txt"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
for v in base $VAR base $VAR; do
  if [ $v = base ]; then L=""; else L=lodestar_amd/variants/libgbv_$v.so; fi
  LODESTAR_AMD_LIB=$L timeout -k 10 150 python3 -u tools/latency_probe.py > "$OUT/lat_$v.txt" 2>&1 || { echo "lat $v failed"; tail -20 "$OUT/lat_$v.txt"; exit 1; }
  LODESTAR_AMD_LIB=$L timeout -k 10 200 python3 -u tools/vs_probe.py --blocks 64 --inflight 1,2 > "$OUT/vs_$v.txt" 2>&1 || { echo "vs $v failed"; tail -20 "$OUT/vs_$v.txt"; exit 1; }
  echo "== $v"; tail -4 "$OUT/lat_$v.txt"; grep -v "^\[probe\]" "$OUT/vs_$v.txt"
done
