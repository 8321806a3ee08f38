#!/bin/bash
# Same-box A/B of library variants with a parity subset on the first one:
#   bash tools/gpu_variant_ab.sh TAG V1 [V2 ...]   (variants from tools/build_variant.sh; "base" = in-tree lib)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
LODESTAR_AMD_LIB=lodestar_amd/variants/libgbv_$1.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_c5.py > "$OUT/test_$1.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/test_$1.log"; exit 1; }
tail -1 "$OUT/test_$1.log"
for v in base "$@" base "$@"; do
  if [ "$v" = base ]; then lib=""; else lib=lodestar_amd/variants/libgbv_$v.so; fi
  LODESTAR_AMD_LIB=$lib timeout -k 10 240 python3 -u bench.py --steps 8 --warmup 1 --no-cpu-baseline --no-signing-roots > "$OUT/$v.json" 2> "$OUT/$v.err" || { echo "bench $v failed"; tail -20 "$OUT/$v.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$v.json')); k=d['roofline']['kernel_ms_per_step']; print('$v', round(d['value']/1e6,3), d['ms_per_step'], 'prep', k['prepare'], 'msm', k['msm'], 'c3', d.get('c3',{}).get('value'), 'c4', d.get('c4',{}).get('value'))"
done
