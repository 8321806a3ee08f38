// Arithmetic self-check of the inline-asm carry chains at different occupancies: every lane runs
// the same dependent chain of Fp products / sums from its own seed; the results are printed as
// hex and compared with Python big-int arithmetic by tools/hazard_check.py.  1 wave per SIMD
// (one block) exposes any missing VALU->SGPR->VALU wait state; many waves hide it.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../lodestar_amd/csrc/fp.h"
using namespace gbv;

__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1))) k_chain(Fp* out, int iters) {
  uint32_t t = blockIdx.x * 64 + threadIdx.x;
  Fp a = FP_ONE, b = FP_ONE;
  a.v[0] ^= t * 0x9E3779B9u;
  a.v[5] ^= t;
  b.v[3] ^= 0x12345u + t;
  a = fp_reduce_once(a);
  b = fp_reduce_once(b);
  for (int i = 0; i < iters; ++i) {
    a = fp_mul_inl(a, b);
    b = fp_add(b, a);
    a = fp_sub(a, b);
  }
  out[t] = a;
}

int main(int argc, char** argv) {
  int blocks = argc > 1 ? atoi(argv[1]) : 1;
  int iters = argc > 2 ? atoi(argv[2]) : 500;
  Fp* d;
  hipMalloc(&d, sizeof(Fp) * 64 * blocks);
  hipLaunchKernelGGL(k_chain, dim3(blocks), dim3(64), 0, 0, d, iters);
  std::vector<Fp> h(64 * blocks);
  hipMemcpy(h.data(), d, sizeof(Fp) * 64 * blocks, hipMemcpyDeviceToHost);
  for (int t = 0; t < 64 * blocks; t += (blocks > 1 ? 61 : 1)) {
    printf("%d ", t);
    for (int i = 11; i >= 0; --i) printf("%08x", h[t].v[i]);
    printf("\n");
  }
  return 0;
}
