#!/bin/bash
# PMC passes over the small verifySignatureSets probe (C4 shape, tools/vs_probe.py): one counter group
# per rocprofv3 run, as the MI355X guide prescribes.  Usage (via gpurun): bash tools/gpu_vs_pmc.sh tag
set -o pipefail
TAG=${1:-vspmc}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
PROBE="tools/vs_probe.py --blocks 64 --reps 2"
run_pass() {
  local name=$1; shift
  timeout -s KILL 200 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- python3 -u $PROBE \
    > "$OUT/$name.log" 2>&1 || { echo "pmc pass $name failed"; tail -20 "$OUT/$name.log"; exit 1; }
}
run_pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_IFETCH SQ_INSTS_SALU SQ_BUSY_CYCLES
run_pass fetch FETCH_SIZE
run_pass write WRITE_SIZE
python3 tools/pmc_parse.py "$OUT" "$OUT/pmc.json" && python3 - "$OUT/pmc.json" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in sorted(d.items()):
    if not k.startswith(("k_vs", "k_hash", "k_vs_chunk", "void k_vs")):
        continue
    w = v.get("SQ_WAVES", 0) or 1
    print("%-28s grid %7d dur %.3f ms  valu/wave %.0f  wave_cyc/wave %.0f  active_valu %.3f  wait_inst %.3f  ifetch/wave %.0f  fetch %.1f MB  write %.1f MB" % (
        k, v["grid_size"], v.get("duration_ms", 0), v.get("SQ_INSTS_VALU", 0) / w, v.get("SQ_WAVE_CYCLES", 0) / w,
        v.get("SQ_ACTIVE_INST_VALU", 0) / max(v.get("SQ_WAVE_CYCLES", 1), 1), v.get("SQ_WAIT_INST_ANY", 0) / max(v.get("SQ_WAVE_CYCLES", 1), 1),
        v.get("SQ_IFETCH", 0) / w, v.get("FETCH_SIZE", 0) / 1024, v.get("WRITE_SIZE", 0) / 1024))
EOF
