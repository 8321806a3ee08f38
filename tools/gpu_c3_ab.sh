#!/bin/bash
# Same-box A/B of the C3 pass (tools/c3_probe.py) over variants: "base", a tools/build_variant.sh
# name, or E:VAR=VALUE.  Usage (via gpurun): bash tools/gpu_c3_ab.sh TAG V1 [V2 ...]
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run_with() {
  local v=$1; shift
  case "$v" in
    base) "$@" ;;
    E:*) env $(echo "${v#E:}" | tr , " ") "$@" ;;
    *) LODESTAR_AMD_LIB=lodestar_amd/variants/libgbv_$v.so "$@" ;;
  esac
}
for v in base "$@" base "$@"; do
  f="$OUT/${v//[:=\/]/_}"
  run_with "$v" timeout -k 10 300 python3 -u tools/c3_probe.py > "$f.txt" 2> "$f.err" || { echo "probe $v failed"; tail -20 "$f.err"; exit 1; }
  echo "$v: $(cat "$f.txt")"
done
