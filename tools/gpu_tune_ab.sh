#!/bin/bash
# Same-box A/B of gbv_tune settings on the C2 line (alternated twice):
#   bash tools/gpu_tune_ab.sh TAG "name|--tune a=1 ..." ...   (extra bench args in $AB_ARGS)
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2; do
  for cfg in "$@"; do
    name=${cfg%%|*}; args=${cfg#*|}
    timeout -k 10 300 python3 -u bench.py --steps 12 --warmup 2 --no-cpu-baseline --no-signing-roots --no-extras --no-api --no-vs-shard ${AB_ARGS:-} $args \
      > "$OUT/${name}_$rep.json" 2> "$OUT/${name}_$rep.err" || { echo "$name failed"; tail -20 "$OUT/${name}_$rep.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/${name}_$rep.json')); k=d['roofline']['kernel_ms_per_step']; print('%-10s C2 %.3f M  ms/step %.2f  prep %.2f  msm %.2f  p50 %s' % ('$name', d['value']/1e6, d['ms_per_step'], k['prepare'], k['msm'], d.get('p50_batch_latency_ms')))"
  done
done
