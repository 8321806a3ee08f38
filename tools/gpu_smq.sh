#!/bin/bash
# A/B of the same-message chunk Miller launch form (gbv_tune "sm_quad_max") on C5 at a small per-GPU
# batch and on the C2 headline batch:  bash tools/gpu_smq.sh TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_replay_tune.sh "$1" 131072 "fb16k|--tune fb_coop_max=16384" "q512|--tune fb_coop_max=16384 --tune sm_quad_max=512" \
  "q2k|--tune fb_coop_max=16384 --tune sm_quad_max=2048" "q8k|--tune fb_coop_max=16384 --tune sm_quad_max=8192" || exit 1
for q in 0 8192 0 8192; do
  timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 1 --no-cpu-baseline --no-signing-roots --no-extras --no-api --no-vs-shard \
    --tune sm_quad_max=$q > "$OUT/c2_q$q.json" 2> "$OUT/c2_q$q.err" || { echo "c2 $q failed"; tail -20 "$OUT/c2_q$q.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c2_q$q.json')); print('C2 sm_quad_max $q: %.3f M sets/s' % (d['value'] / 1e6))"
done
