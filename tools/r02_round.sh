#!/bin/bash
# Round-2 GPU session: new parity tests (addon), full bench (C2 headline + C1/C3/C4 lines), a
# single-rank replay-mode run.  Each GPU step has its own limit; stop at the first failure.
set -o pipefail
TAG=${1:-r02}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_addon.py -m gpu -x -v --timeout 200 --timeout-method thread > "$OUT/pytest_addon.log" 2>&1 || { echo "addon test failed"; tail -30 "$OUT/pytest_addon.log"; exit 1; }
tail -2 "$OUT/pytest_addon.log"
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
tail -8 "$OUT/bench.err"
timeout -k 10 300 python -u bench.py --mode replay --steps 4 --no-cpu-baseline --no-signing-roots > "$OUT/replay.json" 2> "$OUT/replay.err" || { echo "replay failed"; tail -30 "$OUT/replay.err"; exit 1; }
tail -2 "$OUT/replay.err"
echo "[r02_round] done"
