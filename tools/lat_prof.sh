#!/bin/bash
# Kernel trace of the lone-call latency probe (per-kernel durations of a lone 64-set same-message
# call, a lone C1 call, lone blocks): bash tools/lat_prof.sh TAG
set -o pipefail
TAG=${1:-lat}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 -u tools/latency_probe.py > "$OUT/probe.log" 2>&1 || { echo "probe failed"; tail -20 "$OUT/probe.log"; exit 1; }
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
find "$OUT/prof" -name '*kernel_trace.csv' -exec cp {} "$OUT/kernel_trace.csv" \;
cut -c1-150 "$OUT/kernel_stats.csv" | head -30
