set -o pipefail
mkdir -p gpurun_out/lazy
export TMPDIR=/tmp
LODESTAR_AMD_LIB=lodestar_amd/variants/libgbv_lazy.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_single_thread.py tests/test_gpu_c3.py > gpurun_out/lazy/test.log 2>&1 || { echo tests failed; tail -30 gpurun_out/lazy/test.log; exit 1; }
tail -1 gpurun_out/lazy/test.log
bash tools/ab.sh base lazy base lazy
