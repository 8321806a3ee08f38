# C5 failure path: parity tests, the replay bench (failure path on its own stream, then on the
# tail stream), then the default C2 bench line -- one GPU
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_c5.py tests/test_gpu_scale.py tests/test_gpu_parity.py > gpurun_out/c5_test.log 2>&1 &&
timeout -k 10 300 python -u bench.py --mode replay --steps 8 --warmup 1 --no-cpu-baseline --no-signing-roots > gpurun_out/c5_bench.json 2> gpurun_out/c5_bench.err &&
GBV_FB_STREAM=0 timeout -k 10 300 python -u bench.py --mode replay --steps 8 --warmup 1 --no-cpu-baseline --no-signing-roots > gpurun_out/c5_bench2.json 2> gpurun_out/c5_bench2.err &&
timeout -k 10 300 python -u bench.py --steps 12 --warmup 1 --no-cpu-baseline --no-signing-roots > gpurun_out/c2_bench.json 2> gpurun_out/c2_bench.err
