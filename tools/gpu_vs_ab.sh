#!/bin/bash
# Same-box A/B of library variants on the small verifySignatureSets probe (C4 shape: one 64-block
# pass, lone and 1-3 in flight, plus a lone block), with the verifySignatureSets parity subset on
# each variant first:
#   bash tools/gpu_vs_ab.sh TAG V1 [V2 ...]
# V: a variant from tools/build_variant.sh, "base" (the in-tree lib), or E:VAR=VALUE (the in-tree lib
# under that environment setting).
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run_with() {  # run_with V cmd...
  local v=$1; shift
  case "$v" in
    base) "$@" ;;
    E:*) env $(echo "${v#E:}" | tr , " ") "$@" ;;
    *) LODESTAR_AMD_LIB=lodestar_amd/variants/libgbv_$v.so "$@" ;;
  esac
}
for v in base "$@"; do
  run_with "$v" timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_block_sets.py > "$OUT/test_${v//[:=\/]/_}.log" 2>&1 || { echo "tests failed ($v)"; tail -30 "$OUT/test_${v//[:=\/]/_}.log"; exit 1; }
  echo "$v: $(tail -1 "$OUT/test_${v//[:=\/]/_}.log")"
done
for v in base "$@" base "$@"; do
  f="$OUT/${v//[:=\/]/_}"
  run_with "$v" timeout -k 10 200 python3 -u tools/vs_probe.py --blocks 64 --inflight 1,2,3 > "$f.txt" 2>&1 || { echo "probe $v failed"; tail -20 "$f.txt"; exit 1; }
  echo "== $v"; grep -v "^\[probe\]" "$f.txt"
done
