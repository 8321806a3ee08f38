#!/bin/bash
# Kernel trace of streamed shard passes (bench.py --mode vs-shard, N = 1): does k_fp12_check (stream 6)
# run beside the next pass's kernels?  Output: gpurun_out/$TAG/trace (rocprofv3 kernel_trace.csv)
set -o pipefail
TAG=${1:-fp12trace}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o run -- python3 -u bench.py --mode vs-shard --shard-calls 64 --steps 16 --warmup 2 \
  > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "trace run failed"; tail -20 "$OUT/bench.err"; exit 1; }
find "$OUT/trace" -name '*kernel_trace.csv' -exec cp {} "$OUT/kernel_trace.csv" \;
python3 tools/fp12_overlap.py "$OUT/kernel_trace.csv" | tee "$OUT/overlap.txt"
