// Latency microbenchmark of the wave-cooperative Fp12 engine (coop.h) on one wave, against the
// thread-level primitives it replaces.  Fixes what one coop program costs in wall time.
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/ubench_coop tools/ubench_coop.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../lodestar_amd/csrc/coop.h"

using namespace gbv;

// one wave: ITER cooperative Fp12 products, in place
__device__ inline Fp seed_fp(unsigned k) {
  Fp a = FP_ONE;
  a.v[1] += k;
  return a;
}

__global__ void __launch_bounds__(64) k_coop_mul(Fp* out, int iters) {
  __shared__ coop::Slot ws[36 + coop::ZSLOTS];
  coop::load_consts();
  if (threadIdx.x < 24) coop::put(ws + threadIdx.x, seed_fp(threadIdx.x));
  __syncthreads();
  for (int i = 0; i < iters; ++i) coop::mul12(ws, 36, 0, 12, 0);
  if (threadIdx.x < 12) out[blockIdx.x * 12 + threadIdx.x] = coop::get(ws + threadIdx.x);
}

__global__ void __launch_bounds__(64) k_coop_cyc(Fp* out, int iters) {
  __shared__ coop::Slot ws[36 + coop::ZSLOTS];
  coop::load_consts();
  if (threadIdx.x < 24) coop::put(ws + threadIdx.x, seed_fp(threadIdx.x));
  __syncthreads();
  for (int i = 0; i < iters; ++i) coop::run(coop::FP12_CYC_SQR, coop::ws2(ws, 36, 0, 0));  // the interpreted program
  if (threadIdx.x < 12) out[blockIdx.x * 12 + threadIdx.x] = coop::get(ws + threadIdx.x);
}

// the squarings as exp_x runs them (coop::cyc_sqr_lane: written out, lane terms resolved once)
__global__ void __launch_bounds__(64) k_coop_cyc_hand(Fp* out, int iters) {
  __shared__ coop::Slot ws[36 + coop::ZSLOTS];
  coop::load_consts();
  if (threadIdx.x < 24) coop::put(ws + threadIdx.x, seed_fp(threadIdx.x));
  __syncthreads();
  const coop::CycLane x = coop::cyc_lane(ws, 36, 0, 0, threadIdx.x);
  for (int i = 0; i < iters; ++i) coop::cyc_sqr_lane(x);
  if (threadIdx.x < 12) out[blockIdx.x * 12 + threadIdx.x] = coop::get(ws + threadIdx.x);
}

// one wave: the final exponentiation alone
__global__ void __launch_bounds__(64) k_coop_fe(Fp* out, int iters) {
  __shared__ coop::Slot ws[coop::FINAL_EXP_WS];
  coop::load_consts();
  bool ok = false;
  for (int i = 0; i < iters; ++i) {
    if (threadIdx.x < 12) coop::put(ws + coop::E_F + threadIdx.x, seed_fp(threadIdx.x + i));
    __syncthreads();
    ok ^= coop::final_exp_is_one(ws);
  }
  if (threadIdx.x < 12) out[blockIdx.x * 12 + threadIdx.x] = coop::get(ws + coop::E_C + threadIdx.x);
  if (threadIdx.x == 0) out[0].v[0] += ok;
}

// one wave: [|x|] Q by the cooperative point steps (the cofactor clearing's chain)
__global__ void __launch_bounds__(64) k_coop_xabs(Fp* out, int iters) {
  __shared__ coop::Slot ws[coop::MILLER_WS];
  coop::load_consts();
  G2A Q{Fp2{FP_ONE, FP_ONE}, Fp2{FP_B1, FP_ONE}};
  for (int i = 0; i < iters; ++i) coop::mul_xabs_point(ws, Q);
  if (threadIdx.x < 12) out[blockIdx.x * 12 + threadIdx.x] = coop::get(ws + coop::M_PAIR + threadIdx.x);
}

// one wave, one lane: dependent Fp products (latency of the thread-level primitive)
__global__ void __launch_bounds__(64) k_fp_mul_lat(Fp* out, int iters) {
  Fp a = FP_ONE, b = FP_ONE;
  a.v[0] += threadIdx.x;
  b.v[1] += 1;
  for (int i = 0; i < iters; ++i) a = fp_mul(a, b);
  out[blockIdx.x * 64 + threadIdx.x] = a;
}

// one wave: dependent thread-level Fp12 products
__global__ void __launch_bounds__(64) k_fp12_mul_lat(Fp* out, int iters) {
  Fp12 a = fp12_one(), b = fp12_one();
  a.c0.c0.c0.v[0] += threadIdx.x;
  b.c1.c0.c1.v[1] += 1;
  for (int i = 0; i < iters; ++i) a = fp12_mul(a, b);
  out[blockIdx.x * 64 + threadIdx.x] = a.c0.c0.c0;
}

// one wave: cooperative Miller loop (1 pair) + final exponentiation, iters times
__global__ void __launch_bounds__(64) k_coop_pairing(Fp* out, int iters) {
  __shared__ coop::Slot ws[coop::MILLER_WS + coop::FINAL_EXP_WS];
  coop::load_consts();
  G1A P = g1_neg_generator();
  G2A Q{Fp2{FP_ONE, FP_ONE}, Fp2{FP_B1, FP_ONE}};
  bool ok = false;
  for (int i = 0; i < iters; ++i) {
    coop::miller_load_pair(ws, 0, P, Q);
    coop::miller_loop(ws, 1);
    coop::copy(ws + coop::MILLER_WS + coop::E_F, ws + coop::M_F, 12);
    ok ^= coop::final_exp_is_one(ws + coop::MILLER_WS);
  }
  if (threadIdx.x < 12) out[blockIdx.x * 12 + threadIdx.x] = coop::get(ws + threadIdx.x);
  if (threadIdx.x == 0) out[0].v[0] += ok;
}

__global__ void __launch_bounds__(64) k_coop_miller(Fp* out, int iters) {
  __shared__ coop::Slot ws[coop::MILLER_WS];
  coop::load_consts();
  G1A P = g1_neg_generator();
  G2A Q{Fp2{FP_ONE, FP_ONE}, Fp2{FP_B1, FP_ONE}};
  for (int i = 0; i < iters; ++i) {
    coop::miller_load_pair(ws, 0, P, Q);
    coop::miller_loop(ws, 1);
  }
  if (threadIdx.x < 12) out[blockIdx.x * 12 + threadIdx.x] = coop::get(ws + threadIdx.x);
}

// one lane: thread-level pieces that run on lane 0 inside the cooperative kernels
__global__ void __launch_bounds__(64) k_lane0_fp12_inv(Fp* out, int iters) {
  Fp12 a = fp12_one();
  a.c1.c0.c1.v[1] += threadIdx.x + 3;
  for (int i = 0; i < iters; ++i) a = fp12_inv(a);
  out[blockIdx.x * 64 + threadIdx.x] = a.c0.c0.c0;
}
__global__ void __launch_bounds__(64) k_lane0_fp_inv(Fp* out, int iters) {
  Fp a = FP_ONE;
  a.v[1] += threadIdx.x + 3;
  for (int i = 0; i < iters; ++i) a = fp_inv(a);
  out[blockIdx.x * 64 + threadIdx.x] = a;
}
__global__ void __launch_bounds__(64) k_thread_miller(Fp* out, int iters) {
  G1A P = g1_neg_generator();
  G2A Q{Fp2{FP_ONE, FP_ONE}, Fp2{FP_B1, FP_ONE}};
  Fp12 f = fp12_one();
  for (int i = 0; i < iters; ++i) f = fp12_mul(f, miller_loop_1(P, Q));
  out[blockIdx.x * 64 + threadIdx.x] = f.c0.c0.c0;
}

typedef void (*kfn)(Fp*, int);
static void run(const char* name, kfn f, Fp* out, int blocks, int iters, double fme_per_iter) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(f, dim3(blocks), dim3(64), 0, 0, out, 2);
  hipDeviceSynchronize();
  hipEventRecord(a);
  hipLaunchKernelGGL(f, dim3(blocks), dim3(64), 0, 0, out, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  printf("%-14s blocks=%5d iters=%5d  %8.3f ms  %8.2f us/iter  (%.0f FME/iter -> %.2f us/FME latency)\n", name, blocks, iters, ms,
         ms * 1e3 / iters, fme_per_iter, ms * 1e3 / iters / fme_per_iter);
  fflush(stdout);
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  printf("device %s CUs=%d\n", p.gcnArchName, p.multiProcessorCount);
  Fp* out;
  hipMalloc(&out, sizeof(Fp) * 64 * 4096);
  run("fp_mul lat", k_fp_mul_lat, out, 1, 2000, 1);
  run("fp12_mul lat", k_fp12_mul_lat, out, 1, 100, 54);
  run("coop mul12", k_coop_mul, out, 1, 200, 54);
  run("coop cyc_sqr", k_coop_cyc, out, 1, 200, 18);
  run("coop cyc hand", k_coop_cyc_hand, out, 1, 200, 18);
  run("coop FE", k_coop_fe, out, 1, 3, 8400);
  run("coop miller1", k_coop_miller, out, 1, 5, 6200);
  run("coop xabs", k_coop_xabs, out, 1, 5, 2000);
  run("coop ML1+FE", k_coop_pairing, out, 1, 3, 14600);
  run("fp12_inv lane", k_lane0_fp12_inv, out, 1, 5, 500);
  run("fp_inv lane", k_lane0_fp_inv, out, 1, 5, 460);
  run("thread miller1", k_thread_miller, out, 1, 2, 6200);
  run("thread miller1", k_thread_miller, out, 205, 2, 6200);
  run("coop miller1", k_coop_miller, out, 13117, 1, 6200);
  run("coop mul12", k_coop_mul, out, 1024, 200, 54);
  run("coop mul12", k_coop_mul, out, 4096, 100, 54);
  return 0;
}
