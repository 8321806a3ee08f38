#!/bin/bash
# Round-5 probes: C5 with the failure path's chunk checks one thread each (default) or one wave each
# (group_coop), and the streamed vs-shard pass at 16 384 / 32 768 / 65 536 sets per rank (the
# per-pass times of the N = 4 / 2 / 1 shares of one 65 536-set call).  Usage: bash tools/gpu_r05g.sh tag
set -o pipefail
TAG=${1:-r05g}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/c5_probe.py --steps 9 --depth 3 > "$OUT/c5_thread.txt" 2> "$OUT/c5_thread.err" || { echo "c5 failed"; tail -20 "$OUT/c5_thread.err"; exit 1; }
head -1 "$OUT/c5_thread.txt"
timeout -k 10 300 python -u tools/c5_probe.py --steps 9 --depth 3 --tune group_coop=1 > "$OUT/c5_coop.txt" 2> "$OUT/c5_coop.err" || { echo "c5 coop failed"; tail -20 "$OUT/c5_coop.err"; exit 1; }
head -1 "$OUT/c5_coop.txt"
for calls in 128 256 512; do
  timeout -k 10 300 python -u bench.py --mode vs-shard --shard-calls $calls --steps 16 --warmup 2 > "$OUT/vs_shard$calls.json" 2> "$OUT/vs_shard$calls.err" || { echo "vs-shard $calls failed"; tail -20 "$OUT/vs_shard$calls.err"; exit 1; }
  cat "$OUT/vs_shard$calls.json"
done
