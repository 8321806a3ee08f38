#!/bin/bash
# One GPU-box session: parity tests, smoke, a bench line and a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; the script stops at the first failure.
# Usage (from the repo root, via gpurun): bash tools/gpu_round.sh [tag] [bench args...]
set -o pipefail
TAG=${1:-r01}
shift || true
BENCH_ARGS=${*:-""}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[gpu_round] host: $(nproc) cpus, $(grep -m1 'model name' /proc/cpuinfo | cut -d: -f2)" | tee "$OUT/host.txt"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -30 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 600 python -u bench.py $BENCH_ARGS > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 -u bench.py $BENCH_ARGS --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err" || { echo "rocprof failed"; tail -30 "$OUT/prof_bench.err"; exit 1; }
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
cut -c1-220 "$OUT/kernel_stats.csv"
echo "[gpu_round] done"
