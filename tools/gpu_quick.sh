# quick GPU check: parity + scale tests, a C2 bench line with the C1/C3/C4 extras, then the PMC passes
set -o pipefail
TAG=${1:-quick}
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_single_thread.py > gpurun_out/quick_test.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 12 --warmup 1 --no-cpu-baseline --no-signing-roots > gpurun_out/quick_bench.json 2> gpurun_out/quick_bench.err &&
bash tools/pmc.sh $TAG > gpurun_out/pmc_$TAG.log 2>&1
