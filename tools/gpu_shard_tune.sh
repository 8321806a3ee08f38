#!/bin/bash
# One shard size (--shard-calls, default 64 = 8 192 sets) at depth 4 under several gbv_tune launch shapes:
#   bash tools/gpu_shard_tune.sh TAG CALLS "name|--tune a=1 --tune b=2" ...
set -o pipefail
OUT=gpurun_out/$1; CALLS=$2; shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in "$@"; do
  name=${cfg%%|*}; args=${cfg#*|}
  timeout -k 10 200 python3 -u bench.py --mode vs-shard --shard-calls $CALLS --shard-depth 4 --steps 24 --warmup 4 $args \
    > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "$name failed"; tail -20 "$OUT/$name.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$name.json')); print('%-12s %s sets/s, %.3f ms per pass, lone %.3f ms' % ('$name', d['value'], d['ms_per_step'], d['lone_pass_ms']))"
done
