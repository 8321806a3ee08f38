#!/bin/bash
# Round-5 session: GPU parity, the C5 probe, the verifySignatureSets Miller-form probe and the
# streamed vs-shard line at N = 1.  Usage (repo root, via gpurun): bash tools/gpu_r05.sh tag
set -o pipefail
TAG=${1:-r05}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_c5.sh "$TAG" || exit 1
timeout -k 10 400 python -u tools/vs_probe.py > "$OUT/vs.txt" 2> "$OUT/vs.err" || { echo "vs probe failed"; tail -20 "$OUT/vs.err"; exit 1; }
cat "$OUT/vs.txt"
timeout -k 10 300 python -u bench.py --mode vs-shard --shard-calls 64 --steps 24 --warmup 2 > "$OUT/vs_shard64.json" 2> "$OUT/vs_shard64.err" || { echo "vs-shard failed"; tail -20 "$OUT/vs_shard64.err"; exit 1; }
cat "$OUT/vs_shard64.json"
