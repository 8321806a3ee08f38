// Integer-VALU throughput microbenchmark for gfx950: fixes the roofline peak
// (u32xu32->u64 MAC/s) used by bench.py.  Each kernel runs 16 independent
// dependency chains per lane so the issue rate, not latency, is measured.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 4096
#define CHAINS 16

__global__ void k_mad_u64(uint64_t* out, uint32_t m) {
  uint64_t acc[CHAINS];
  for (int k = 0; k < CHAINS; ++k) acc[k] = threadIdx.x + k;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int k = 0; k < CHAINS; ++k) {
      uint64_t r;
      uint32_t lo = (uint32_t)acc[k];
      asm volatile("v_mad_u64_u32 %0, %4, %1, %2, %3" : "=v"(r) : "v"(lo), "v"(m), "v"(acc[k]), "s"(0ull) : "vcc");
      acc[k] = r;
    }
  }
  uint64_t s = 0;
  for (int k = 0; k < CHAINS; ++k) s ^= acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mul_lo(uint64_t* out, uint32_t m) {
  uint32_t acc[CHAINS];
  for (int k = 0; k < CHAINS; ++k) acc[k] = threadIdx.x + k;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int k = 0; k < CHAINS; ++k) {
      uint32_t r;
      asm volatile("v_mul_lo_u32 %0, %1, %2" : "=v"(r) : "v"(acc[k]), "v"(m));
      acc[k] = r;
    }
  }
  uint64_t s = 0;
  for (int k = 0; k < CHAINS; ++k) s ^= acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mul_hi(uint64_t* out, uint32_t m) {
  uint32_t acc[CHAINS];
  for (int k = 0; k < CHAINS; ++k) acc[k] = threadIdx.x + k;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int k = 0; k < CHAINS; ++k) {
      uint32_t r;
      asm volatile("v_mul_hi_u32 %0, %1, %2" : "=v"(r) : "v"(acc[k]), "v"(m));
      acc[k] = r;
    }
  }
  uint64_t s = 0;
  for (int k = 0; k < CHAINS; ++k) s ^= acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_addc(uint64_t* out, uint32_t m) {
  uint32_t acc[CHAINS];
  for (int k = 0; k < CHAINS; ++k) acc[k] = threadIdx.x + k;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int k = 0; k < CHAINS; ++k) {
      uint32_t r;
      asm volatile("v_add_co_u32 %0, vcc, %1, %2" : "=v"(r) : "v"(acc[k]), "v"(m) : "vcc");
      acc[k] = r;
    }
  }
  uint64_t s = 0;
  for (int k = 0; k < CHAINS; ++k) s ^= acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_fma_f64(uint64_t* out, uint32_t m) {
  double acc[CHAINS];
  double mm = 1.0000001 + m * 1e-30;
  for (int k = 0; k < CHAINS; ++k) acc[k] = threadIdx.x + k;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int k = 0; k < CHAINS; ++k) {
      double r;
      asm volatile("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(acc[k]), "v"(mm), "v"(acc[k]));
      acc[k] = r;
    }
  }
  double s = 0;
  for (int k = 0; k < CHAINS; ++k) s += acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}

__global__ void k_mad_u24(uint64_t* out, uint32_t m) {
  uint32_t acc[CHAINS];
  for (int k = 0; k < CHAINS; ++k) acc[k] = threadIdx.x + k;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int k = 0; k < CHAINS; ++k) {
      uint32_t r;
      asm volatile("v_mad_u32_u24 %0, %1, %2, %1" : "=v"(r) : "v"(acc[k]), "v"(m));
      acc[k] = r;
    }
  }
  uint64_t s = 0;
  for (int k = 0; k < CHAINS; ++k) s ^= acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef void (*kfn)(uint64_t*, uint32_t);
static void run(const char* name, kfn f, uint64_t* out, int blocks, int threads) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), 0, 0, out, 3u);
  hipDeviceSynchronize();
  hipEventRecord(a);
  const int reps = 5;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), 0, 0, out, 3u);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  double ops = (double)reps * blocks * threads * (double)ITERS * CHAINS;
  printf("%-10s blocks=%d threads=%d  %.3f ms  %.2f T lane-ops/s\n", name, blocks, threads, ms, ops / (ms * 1e-3) / 1e12);
}

int main() {
  hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
  printf("device %s CUs=%d clock=%d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
  uint64_t* out; hipMalloc(&out, 256 * 64 * 1024 * 8);
  for (int bl : {2048, 8192}) {
    run("mad_u64", k_mad_u64, out, bl, 256);
    run("mul_lo", k_mul_lo, out, bl, 256);
    run("mul_hi", k_mul_hi, out, bl, 256);
    run("add_co", k_addc, out, bl, 256);
    run("fma_f64", k_fma_f64, out, bl, 256);
    run("mad_u24", k_mad_u24, out, bl, 256);
  }
  return 0;
}
