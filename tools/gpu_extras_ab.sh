#!/bin/bash
# Same-box A/B of gbv_tune settings on the secondary lines (C1 / C3 / C4 / C4e / C5), alternated twice:
#   bash tools/gpu_extras_ab.sh TAG "name|--tune a=1 ..." ...
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2; do
  for cfg in "$@"; do
    name=${cfg%%|*}; args=${cfg#*|}
    timeout -k 10 400 python3 -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-signing-roots --no-api --no-vs-shard $args \
      > "$OUT/${name}_$rep.json" 2> "$OUT/${name}_$rep.err" || { echo "$name failed"; tail -20 "$OUT/${name}_$rep.err"; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/${name}_$rep.json')); g=lambda k:(d.get(k) or {}).get('value')
print('%-8s C2 %.2f M  c1 %s  c3 %s  c4 %s  c4e %s  c5 %s' % ('$name', d['value']/1e6, g('c1'), g('c3'), g('c4'), g('c4e'), g('c5')))"
  done
done
