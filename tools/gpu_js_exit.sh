#!/bin/bash
# Diagnosis of the Node child's exit (bench.py's JS API line): one bench run keeps the child's inputs,
# then the child alone up to 6 times with the addon's SIGSEGV backtrace on (GBV_SEGV_TRACE=1); stops at
# the first non-zero exit.  Output under gpurun_out/$TAG.
set -o pipefail
TAG=${1:-jsexit}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
GBV_JS_INPUTS=/tmp/gbv_js_in timeout -k 10 400 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras --no-signing-roots --no-vs-shard \
  > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
grep "api path\|api stream (js)" "$OUT/bench.err"
for k in 1 2 3 4 5 6; do
  GBV_SEGV_TRACE=1 timeout -k 10 300 node addon/bench_api.js /tmp/gbv_js_in 1 > "$OUT/js_$k.out" 2> "$OUT/js_$k.err"
  rc=$?
  echo "run $k: exit $rc"
  if [ $rc -ne 0 ]; then tail -40 "$OUT/js_$k.err"; exit 1; fi
done
