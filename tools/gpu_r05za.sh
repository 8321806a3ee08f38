#!/bin/bash
# C4 inside the full bench (after C1 / C3 in the same process) at 2 and 3 passes in flight, alternated.
set -o pipefail
O=gpurun_out/r05za; mkdir -p $O
b() { timeout -k 10 400 python -u bench.py --no-cpu-baseline --c4-depth $2 > $O/bench_$1.json 2> $O/bench_$1.err || { echo "bench $1 failed"; tail -5 $O/bench_$1.err; exit 1; }; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'C2', d['value'], 'C4', d['c4']['value'], d['c4']['config'][:60], 'C3', d['c3']['value'])" $O/bench_$1.json $1; }
b d2a 2 && b d3a 3 && b d2b 2 && b d3b 3
