#!/bin/bash
# SQ counter pass (dynamic VALU instructions, active VALU cycles, wave cycles) over a short C2 bench run
# for the in-tree library and library variants (tools/build_variant.sh), one rocprofv3 --pmc run each:
#   bash tools/pmc_ab.sh TAG V1 [V2 ...]   ("base" = the in-tree lib)  -> gpurun_out/pmcab_<TAG>/<v>/pmc.json
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/pmcab_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-api --no-signing-roots --no-extras --no-vs-shard"
for v in base "$@"; do
  if [ "$v" = base ]; then lib=""; else lib=lodestar_amd/variants/libgbv_$v.so; fi
  mkdir -p "$OUT/$v"
  LODESTAR_AMD_LIB=$lib timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INST_CYCLES_VMEM --output-format csv -d "$OUT/$v/sq" -o run -- python3 -u $BENCH \
    > "$OUT/$v/sq.log" 2>&1 || { echo "pmc $v failed"; tail -20 "$OUT/$v/sq.log"; exit 1; }
  python3 tools/pmc_parse.py "$OUT/$v" "$OUT/$v/pmc.json" "$TAG-$v" > /dev/null && echo "pass $v done"
done
