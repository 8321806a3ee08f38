// gfx950 issue rates of the VALU ops of the 28-bit Montgomery product (fp.h mul28, g2_lazy.h mul28s):
// v_mad_u64_u32 vs v_mad_i64_i32, the 64-bit shifts and v_lshl_add_u64, each with CHAINS independent
// chains per lane (issue rate) and with ONE dependent chain per lane at 1 and 2 waves per SIMD (the
// k_sm_prepare occupancy: latency of a dependent accumulator chain).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 4096
#define DEP_REPS 32  // the low-occupancy runs repeat the kernel body (launch overhead out of the time)

#define DEF(NAME, ASM, T)                                                                 \
  template <int CH> __global__ void NAME(uint64_t* out, uint32_t m) {                     \
    T acc[CH];                                                                             \
    for (int k = 0; k < CH; ++k) acc[k] = threadIdx.x + k;                                 \
    for (int i = 0; i < ITERS * (CH <= 2 ? DEP_REPS : 1); ++i) {                            \
      _Pragma("unroll") for (int k = 0; k < CH; ++k) {                                     \
        T r;                                                                               \
        uint32_t lo = (uint32_t)acc[k];                                                    \
        ASM;                                                                               \
        acc[k] = r;                                                                        \
      }                                                                                    \
    }                                                                                      \
    uint64_t s = 0;                                                                        \
    for (int k = 0; k < CH; ++k) s ^= (uint64_t)acc[k];                                    \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                        \
  }
DEF(k_mad_u64, asm volatile("v_mad_u64_u32 %0, %4, %1, %2, %3" : "=v"(r) : "v"(lo), "v"(m), "v"(acc[k]), "s"(0ull) : "vcc"), uint64_t)
DEF(k_mad_i64, asm volatile("v_mad_i64_i32 %0, %4, %1, %2, %3" : "=v"(r) : "v"(lo), "v"(m), "v"(acc[k]), "s"(0ull) : "vcc"), int64_t)
DEF(k_add_u32, asm volatile("v_add_u32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(m)), uint32_t)
DEF(k_lshl_add64, asm volatile("v_lshl_add_u64 %0, %1, 2, %2" : "=v"(r) : "v"(acc[k]), "v"((uint64_t)m)), uint64_t)
DEF(k_ashr64, asm volatile("v_ashrrev_i64 %0, 28, %1" : "=v"(r) : "v"(acc[k] + m)), int64_t)
DEF(k_lshr64, asm volatile("v_lshrrev_b64 %0, 28, %1" : "=v"(r) : "v"(acc[k] + m)), uint64_t)

typedef void (*kfn)(uint64_t*, uint32_t);
static void run(const char* name, kfn f, uint64_t* out, int blocks, int threads, int chains) {
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
  double ops = (double)reps * blocks * threads * (double)ITERS * chains * (chains <= 2 ? DEP_REPS : 1);
  printf("%-12s chains=%2d waves=%6d  %8.3f ms  %6.2f T lane-ops/s\n", name, chains, blocks * threads / 64, ms, ops / (ms * 1e-3) / 1e12);
}

int main() {
  hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
  printf("device %s CUs=%d clock=%d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
  uint64_t* out; hipMalloc(&out, 256 * 64 * 1024 * 8);
  const int full = 8192, w1 = p.multiProcessorCount * 4, w2 = 2 * w1;  // blocks of 64 threads
  run("mad_u64", k_mad_u64<16>, out, full, 256, 16);
  run("mad_i64", k_mad_i64<16>, out, full, 256, 16);
  run("lshl_add64", k_lshl_add64<16>, out, full, 256, 16);
  run("ashr64", k_ashr64<16>, out, full, 256, 16);
  run("lshr64", k_lshr64<16>, out, full, 256, 16);
  for (int w : {w1, w2}) {
    run("mad_u64 dep", k_mad_u64<1>, out, w, 64, 1);
    run("mad_i64 dep", k_mad_i64<1>, out, w, 64, 1);
    run("mad_u64 x2", k_mad_u64<2>, out, w, 64, 2);
    run("mad_i64 x2", k_mad_i64<2>, out, w, 64, 2);
    run("mad_u64 x16", k_mad_u64<16>, out, w, 64, 16);
  }
  for (int k = 1; k <= 4; ++k) {
    run("add_u32 x16", k_add_u32<16>, out, k * w1, 64, 16);
    run("mad_u64 x16", k_mad_u64<16>, out, k * w1, 64, 16);
  }
  run("mad_u64 dep", k_mad_u64<1>, out, 4 * w1, 64, 1);
  run("mad_u64 x2", k_mad_u64<2>, out, 4 * w1, 64, 2);
  return 0;
}
