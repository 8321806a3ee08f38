// Field-arithmetic throughput microbenchmark for gfx950: how many Montgomery Fp multiplications
// per second the device library's primitives sustain when nothing else is in the kernel.
// Fixes the achievable ceiling that the verification kernels are compared against.
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/ubench_fp tools/ubench_fp.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../lodestar_amd/csrc/curve.h"

using namespace gbv;
#define ITERS 256

// one dependent chain of inlined fp_mul per thread
__global__ void __launch_bounds__(256) k_fp_mul_1(Fp* out) {
  Fp a = FP_ONE, b = FP_ONE;
  a.v[0] += threadIdx.x;
  b.v[1] += blockIdx.x;
  for (int i = 0; i < ITERS; ++i) a = fp_mul_inl(a, b);
  out[blockIdx.x * blockDim.x + threadIdx.x] = a;
}

// two independent chains (ILP 2)
__global__ void __launch_bounds__(256) k_fp_mul_2(Fp* out) {
  Fp a = FP_ONE, b = FP_ONE, c = FP_ONE;
  a.v[0] += threadIdx.x;
  c.v[2] += threadIdx.x;
  b.v[1] += blockIdx.x;
  for (int i = 0; i < ITERS / 2; ++i) {
    a = fp_mul_inl(a, b);
    c = fp_mul_inl(c, b);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = fp_add(a, c);
}

// out-of-line fp_mul calls
__global__ void __launch_bounds__(256) k_fp_mul_call(Fp* out) {
  Fp a = FP_ONE, b = FP_ONE;
  a.v[0] += threadIdx.x;
  b.v[1] += blockIdx.x;
  for (int i = 0; i < ITERS; ++i) a = fp_mul(a, b);
  out[blockIdx.x * blockDim.x + threadIdx.x] = a;
}

// out-of-line fp2_mul calls (3 Fp products each)
__global__ void __launch_bounds__(256) k_fp2_mul_call(Fp* out) {
  Fp2 a = fp2_one(), b = fp2_one();
  a.c0.v[0] += threadIdx.x;
  b.c1.v[1] += blockIdx.x;
  for (int i = 0; i < ITERS / 3; ++i) a = fp2_mul(a, b);
  out[blockIdx.x * blockDim.x + threadIdx.x] = fp_add(a.c0, a.c1);
}

// realistic G2 work: 64-bit scalar multiplication (63 dbl + ~32 madd, ~1.94k FME)
__global__ void __launch_bounds__(256) k_g2_mul64(Fp* out) {
  G2A q{Fp2{FP_ONE, FP_ONE}, Fp2{FP_B1, FP_ONE}};
  q.x.c0.v[0] += threadIdx.x;
  q.y.c1.v[1] += blockIdx.x;
  uint64_t k = 0x9E3779B97F4A7C15ull * (blockIdx.x * blockDim.x + threadIdx.x + 1) | (1ull << 63);
  G2J r = g2_mul_u64(q, k);
  out[blockIdx.x * blockDim.x + threadIdx.x] = fp_add(r.x.c0, r.z.c1);
}

typedef void (*kfn)(Fp*);
static void run(const char* name, kfn f, Fp* out, int blocks, int threads, double muls_per_thread) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), 0, 0, out);
  hipDeviceSynchronize();
  hipEventRecord(a);
  const int reps = 5;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), 0, 0, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  double muls = (double)reps * blocks * threads * muls_per_thread;
  printf("%-14s blocks=%6d threads=%d  %8.3f ms  %7.1f G Fp-mul/s  %6.2f T u32-MAC/s (288 MAC/mul)\n", name, blocks, threads,
         ms, muls / (ms * 1e-3) / 1e9, muls * 288 / (ms * 1e-3) / 1e12);
  fflush(stdout);
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  printf("device %s CUs=%d clock=%d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
  Fp* out;
  hipMalloc(&out, sizeof(Fp) * 256 * 32768);
  for (int bl : {256, 512, 1024, 4096}) {
    run("fp_mul_inl x1", k_fp_mul_1, out, bl, 256, ITERS);
    run("fp_mul_inl x2", k_fp_mul_2, out, bl, 256, ITERS);
    run("fp_mul call", k_fp_mul_call, out, bl, 256, ITERS);
    run("fp2_mul call", k_fp2_mul_call, out, bl, 256, 3.0 * (ITERS / 3));
    run("g2_mul_u64", k_g2_mul64, out, bl / 8, 256, 1940.0);
  }
  return 0;
}
