#!/bin/bash
# Same-box A/B of the sharded verifySignatureSets path (bench.py --mode vs-shard at N = 1) and of the
# C2 line over variants ("base", a tools/build_variant.sh name, or E:VAR=VALUE[,VAR=VALUE]).
# Usage (via gpurun): bash tools/gpu_shard_ab.sh TAG V1 [V2 ...]   (SHARD_CALLS, default 64)
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
  f="$OUT/${v//[:=\/,]/_}"
  run_with "$v" timeout -k 10 300 python3 -u bench.py --mode vs-shard --shard-calls ${SHARD_CALLS:-64} --steps 10 --warmup 2 > "$f.shard.json" 2> "$f.shard.err" || { echo "vs-shard $v failed"; tail -20 "$f.shard.err"; exit 1; }
  run_with "$v" timeout -k 10 200 python3 -u bench.py --steps 8 --warmup 1 --no-cpu-baseline --no-extras --no-api --no-signing-roots > "$f.c2.json" 2> "$f.c2.err" || { echo "c2 $v failed"; tail -20 "$f.c2.err"; exit 1; }
  python3 - "$f" "$v" <<'PY'
import json, sys
f, v = sys.argv[1], sys.argv[2]
s = json.load(open(f + ".shard.json")); c = json.load(open(f + ".c2.json"))
print(v, "vs-shard", s["value"], "sets/s", s["ms_per_step"], "ms/step", s["parity"], "| C2", c["value"], c["ms_per_step"])
PY
done
