#!/bin/bash
# Host-side sanitizer run (ASan/UBSan for the host C): no GPU needed.
#  1. the Node-API addon (addon/gbv_addon.c) with -fsanitize=address,undefined, linked against the
#     CPU stand-in of the C ABI (tests/native/gbv_stub.c, also sanitized), driven from Node through
#     every entry point, the pass slots, concurrent libuv work, close() with passes in flight and GC
#     finalisation (addon/test_addon_stub.js), then the JavaScript GpuBlsVerifier's CPU suite;
#  2. the device arithmetic compiled for the host (tests/native/hosttest.cpp, the code of
#     lodestar_amd/csrc) with the same sanitizers, under tests/test_host_arith.py;
#  3. the oracle's C port (oracle/c/blsport.c) under tests/test_cpu_port.py.
# Any sanitizer report fails the run (halt_on_error).  Usage: bash tools/sanitize_host.sh [outdir]
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-$ROOT/build_asan}
mkdir -p "$OUT/stub"
SAN="-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g -O1"
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
GCC_ASAN=$(gcc -print-file-name=libasan.so)
GCC_UBSAN=$(gcc -print-file-name=libubsan.so)

echo "[sanitize] stub libgbv + addon (gcc $SAN)"
gcc $SAN -fPIC -shared -pthread -Wall -Wextra -o "$OUT/stub/libgbv.so" "$ROOT/tests/native/gbv_stub.c"
gcc $SAN -fPIC -shared -pthread -Wall -Wextra -Wno-unused-parameter -I"${NODE_INC:-/usr/include/node}" \
    -o "$OUT/gbv_addon_asan.node" "$ROOT/addon/gbv_addon.c" -L"$OUT/stub" -lgbv -Wl,-rpath,"$OUT/stub"
# node itself is not instrumented: the runtimes come first through LD_PRELOAD
LD_PRELOAD="$GCC_ASAN $GCC_UBSAN" node --expose-gc "$ROOT/addon/test_addon_stub.js" "$OUT/gbv_addon_asan.node" | tee "$OUT/addon_stub.json"
LD_PRELOAD="$GCC_ASAN $GCC_UBSAN" node "$ROOT/addon/test_verifier.js" cpu | tee "$OUT/verifier_cpu.json"

echo "[sanitize] host build of the device arithmetic (hipcc --offload-host-only $SAN)"
CLANG_ASAN=$(find /opt/rocm/lib/llvm/lib/clang -name 'libclang_rt.asan-x86_64.so' | head -1)
hipcc --offload-host-only $SAN -fno-gpu-sanitize -fPIC -shared -o "$OUT/libhosttest.so" "$ROOT/tests/native/hosttest.cpp"
# (the ~130-pairing shared-accumulator and locate prototypes are left out here: minutes under ASan, and
# their Miller / exponentiation code is the same the other host tests run)
GBV_HOSTTEST_LIB="$OUT/libhosttest.so" LD_PRELOAD="$CLANG_ASAN" \
    python3 -m pytest -q -p no:cacheprovider "$ROOT/tests/test_host_arith.py" -k "not ragged_calls and not locate_one_invalid" 2>&1 | tail -3

echo "[sanitize] oracle C port (gcc $SAN)"
gcc $SAN -fPIC -shared -pthread -O1 -o "$OUT/libblsport.so" "$ROOT/oracle/c/blsport.c"
GBV_BLSPORT_LIB="$OUT/libblsport.so" LD_PRELOAD="$GCC_ASAN $GCC_UBSAN" \
    python3 -m pytest -q -p no:cacheprovider "$ROOT/tests/test_cpu_port.py" 2>&1 | tail -3
echo "[sanitize] clean"
