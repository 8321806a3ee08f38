#!/bin/bash
# C5 replay (bench.py --mode replay: 1 % invalid, every boolean checked against the injection map) at one
# per-GPU batch size under several gbv_tune settings of the failure path:
#   bash tools/gpu_replay_tune.sh TAG SETS "name|--tune a=1" ...
set -o pipefail
OUT=gpurun_out/$1; SETS=$2; shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in "$@"; do
  name=${cfg%%|*}; args=${cfg#*|}
  timeout -k 10 300 python3 -u bench.py --mode replay --sets $SETS --steps 8 --warmup 1 --no-cpu-baseline --no-signing-roots --no-extras --no-api $args \
    > "$OUT/${name}_$SETS.json" 2> "$OUT/${name}_$SETS.err" || { echo "$name failed"; tail -20 "$OUT/${name}_$SETS.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/${name}_$SETS.json')); print('%-10s sets %8d: %.3f M sets/s, %.2f ms per step' % ('$name', $SETS, d['value'] / 1e6, d['ms_per_step']))"
done
