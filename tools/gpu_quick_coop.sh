set -o pipefail
OUT=gpurun_out/r04ad; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 120 tools/ubench_coop > $OUT/ubench.txt 2>&1 && grep -E "cyc|FE|ML1|miller1" $OUT/ubench.txt && \
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && tail -1 $OUT/pytest_gpu.log && \
timeout -k 10 150 python3 -u tools/latency_probe.py > $OUT/lat_base.txt 2>&1 && \
timeout -k 10 200 python3 -u tools/vs_probe.py --blocks 64 --inflight 1,2 > $OUT/vs_base.txt 2>&1 && grep -v "^\[probe\]" $OUT/vs_base.txt
