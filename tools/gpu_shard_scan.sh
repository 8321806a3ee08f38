#!/bin/bash
# Per-pass time of one sharded verifySignatureSets call's shard at N = 1 (bench.py --mode vs-shard, an
# RCCL group of one): shard sizes of 8 192 .. 65 536 sets (--shard-calls 64 .. 512 calls of 128), with
# 2..4 shard passes in flight.  The multi-GPU projection of DESIGN.md section 6 reads these.
#   bash tools/gpu_shard_scan.sh TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
for calls in 64 128 256 512; do
  for d in 2 3 4; do
    timeout -k 10 200 python3 -u bench.py --mode vs-shard --shard-calls $calls --shard-depth $d --steps 24 --warmup 4 \
      > "$OUT/shard_${calls}_d$d.json" 2> "$OUT/shard_${calls}_d$d.err" || { echo "vs-shard $calls d$d failed"; tail -20 "$OUT/shard_${calls}_d$d.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/shard_${calls}_d$d.json')); print('calls $calls depth $d: %s sets/s, %.3f ms per pass, lone pass %.3f ms' % (d['value'], d['ms_per_step'], d['lone_pass_ms']))"
  done
done
