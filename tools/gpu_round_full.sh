#!/bin/bash
# GPU round session: parity tests, smoke, the default bench, the multi-GPU shard mode at N=1, a rocprofv3 kernel-trace
# summary, PMC passes and the lone-call latency probe.  Each GPU step has its own limit; the script
# stops at the first failure.   Usage (via gpurun): bash tools/r03_round.sh tag
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[gpu] host: $(nproc) cpus, $(grep -m1 'model name' /proc/cpuinfo | cut -d: -f2)" | tee "$OUT/host.txt"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -30 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
tail -12 "$OUT/bench.err"
timeout -k 10 300 python -u bench.py --mode vs-shard --steps 5 --warmup 1 > "$OUT/vs_shard.json" 2> "$OUT/vs_shard.err" || { echo "vs-shard failed"; tail -30 "$OUT/vs_shard.err"; exit 1; }
cat "$OUT/vs_shard.json"
timeout -k 10 120 python -u tools/latency_probe.py > "$OUT/latency_probe.txt" 2>&1 || { echo "latency probe failed"; tail -20 "$OUT/latency_probe.txt"; exit 1; }
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 -u bench.py --steps 6 --no-cpu-baseline --no-signing-roots --no-api > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err" || { echo "rocprof failed"; tail -30 "$OUT/prof_bench.err"; exit 1; }
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
cut -c1-160 "$OUT/kernel_stats.csv" | head -25
python3 - "$OUT" <<'PY'
import json, sys
for k in ("bench",):
    d = json.load(open(sys.argv[1] + "/%s.json" % k))
    print(k, "C2 %.2fM" % (d["value"] / 1e6), "p50 %.1f" % d["p50_batch_latency_ms"], "api", d.get("api_path_sets_per_s"))
    for c in ("c1", "c3", "c4", "c4e"):
        x = d.get(c) or {}
        r = x.get("roofline", {})
        print("  %s %.0f sets/s" % (c, x.get("value", 0)), r.get("kernel"), r.get("frac"), r.get("kernel_ms_per_pass"),
              x.get("lone_block_latency_ms_p50"), x.get("latency_ms_p50"))
    if d.get("c5"):
        print("  c5 %.2fM" % (d["c5"]["value"] / 1e6))
PY
echo "[gpu] done"
