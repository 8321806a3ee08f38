#!/bin/bash
# PMC passes over a short bench run (one counter group per run, as the MI355X guide prescribes:
# FETCH_SIZE and WRITE_SIZE cannot share a pass; no trace domains next to --pmc).
# Usage (repo root, via gpurun): bash tools/pmc.sh [tag]  -> gpurun_out/pmc_<tag>/, profiles-ready JSON
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="bench.py --steps 1 --warmup 0 --sets 262144 --no-cpu-baseline --no-stream --no-api"
run_pass() {
  local name=$1; shift
  timeout -s KILL 400 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- python3 -u $BENCH \
    > "$OUT/$name.log" 2>&1 || { echo "pmc pass $name failed"; tail -20 "$OUT/$name.log"; exit 1; }
}
run_pass fetch FETCH_SIZE
run_pass write WRITE_SIZE
run_pass sq SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
python3 tools/pmc_parse.py "$OUT" "$OUT/pmc.json" && cat "$OUT/pmc.json"
