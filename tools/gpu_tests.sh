#!/bin/bash
# GPU parity tests + smoke only (no bench).  Usage (repo root, via gpurun): bash tools/gpu_tests.sh tag [pytest -k expr]
set -o pipefail
TAG=${1:-t}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
K=${2:+-k "$2"}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread $K > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -30 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
