#!/bin/bash
# C5 session: the GPU parity suite, then the C5 probe (1M-set stream, 1 % invalid, every boolean
# checked) with the last batch's per-kernel times.  Usage (repo root, via gpurun): bash tools/gpu_c5.sh tag [probe args]
set -o pipefail
TAG=${1:-c5}
shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -u tools/c5_probe.py --steps 9 --depth 3 "$@" > "$OUT/c5.txt" 2> "$OUT/c5.err" || { echo "c5 failed"; tail -20 "$OUT/c5.err"; exit 1; }
cat "$OUT/c5.txt"
