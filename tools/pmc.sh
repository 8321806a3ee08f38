#!/bin/bash
# PMC passes over a short bench run at the bench's own sizes (C2 1M sets, C1/C3 65 536-set passes,
# C4 8 384-set pass, C4e, C5): one counter group per run, as the MI355X guide prescribes (FETCH_SIZE
# and WRITE_SIZE cannot share a pass; no trace domains next to --pmc).
# Usage (repo root, via gpurun): bash tools/pmc.sh [tag] [fetch|write|sq|all]  -> gpurun_out/pmc_<tag>/pmc.json
# (one pass per call keeps each gpurun call short; the summary is re-made over every pass present)
set -o pipefail
TAG=${1:-r05}
WHICH=${2:-all}
OUT=gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-api --no-signing-roots"
run_pass() {
  local name=$1; shift
  timeout -s KILL 500 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- python3 -u $BENCH \
    > "$OUT/$name.log" 2>&1 || { echo "pmc pass $name failed"; tail -20 "$OUT/$name.log"; exit 1; }
  echo "pass $name done"
}
if [ "$WHICH" = all ] || [ "$WHICH" = fetch ]; then run_pass fetch FETCH_SIZE; fi
if [ "$WHICH" = all ] || [ "$WHICH" = write ]; then run_pass write WRITE_SIZE; fi
if [ "$WHICH" = all ] || [ "$WHICH" = sq ]; then run_pass sq SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE; fi
python3 tools/pmc_parse.py "$OUT" "$OUT/pmc.json" "$TAG" && echo "pmc summary: $OUT/pmc.json"
