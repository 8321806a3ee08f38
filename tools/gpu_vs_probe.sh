#!/bin/bash
# Small verifySignatureSets pass probe (C4 shape): lone-pass latency A/B and a kernel trace of the passes.
# Usage (via gpurun): bash tools/gpu_vs_probe.sh tag [env assignments for the B run...]
set -o pipefail
TAG=${1:-probe}
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 200 python3 -u tools/vs_probe.py --blocks 64 --inflight ${INFLIGHT:-1,2,3,4} > "$OUT/a.txt" 2>&1 || { tail -20 "$OUT/a.txt"; exit 1; }
grep -v "^\[probe\]" "$OUT/a.txt"
if [ $# -gt 0 ]; then
  env "$@" timeout -k 10 150 python3 -u tools/vs_probe.py --blocks 64 > "$OUT/b.txt" 2>&1 || { tail -20 "$OUT/b.txt"; exit 1; }
  echo "B ($*):"; tail -1 "$OUT/b.txt"
fi
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o run -- python3 -u tools/vs_probe.py --blocks 64 --reps 2 > "$OUT/trace.txt" 2>&1 || { tail -20 "$OUT/trace.txt"; exit 1; }
f=$(find "$OUT/trace" -name '*kernel_trace.csv' | head -1)
python3 tools/vs_timeline.py "$f" 30 > "$OUT/timeline.txt" && cat "$OUT/timeline.txt"
