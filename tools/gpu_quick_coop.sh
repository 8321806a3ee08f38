#!/bin/bash
# Quick GPU check of a cooperative-engine change: the one-wave microbenchmark, the GPU parity suite,
# then lone-call latency (tools/latency_probe.py) and the small verifySignatureSets probe for the
# in-tree library and each environment variant given (VAR=VALUE[,VAR2=VALUE2]).
#   bash tools/gpu_quick_coop.sh TAG [ENV_VARIANT ...]
set -o pipefail
TAG=${1:-coop}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 120 tools/ubench_coop > $OUT/ubench.txt 2>&1 && grep -E "cyc|FE|ML1|miller1|xabs" $OUT/ubench.txt || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for v in base "$@"; do
  f=$OUT/lat_${v//[:=,\/]/_}.txt; g=$OUT/vs_${v//[:=,\/]/_}.txt
  if [ $v = base ]; then E=""; else E=$(echo $v | tr , " "); fi
  env $E timeout -k 10 150 python3 -u tools/latency_probe.py > $f 2>&1 || { tail -20 $f; exit 1; }
  env $E timeout -k 10 200 python3 -u tools/vs_probe.py --blocks 64 --inflight 1,2 > $g 2>&1 || { tail -20 $g; exit 1; }
  echo "== $v"; python3 tools/lat_summary.py $f; grep -v "^\[probe\]" $g
done
