// Where a cooperative program's time goes: run_ni (coop.h) re-stated with s_memtime stamps around
// its phases -- record fetch, each product round, the partial sums, the output sums, the output
// stores -- run on one wave for a few programs, cycles per call averaged over the iterations.
// Diagnostic build only (the stamps cost a few percent); the product kernels never run this.
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/ubench_coop_phase tools/ubench_coop_phase.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../lodestar_amd/csrc/coop.h"

using namespace gbv;
using namespace gbv::coop;

constexpr int NPH = 10;  // 0 fetch, 1..6 rounds, 7 parts, 8 out sums, 9 out stores

__device__ inline uint64_t stamp() { return __builtin_amdgcn_s_memtime(); }

__device__ __noinline__ void run_stamped(const Prog* PP, uint32_t b0, uint32_t b1, uint32_t b2, uint32_t b3, uint64_t* acc) {
  const Prog& P = *PP;
  const Ws w{{b0, b1, b2, b3}};
  const int lane = (int)threadIdx.x;
  uint32_t rec[PROD_WORDS], rpart[SUM_WORDS], rout[SUM_WORDS];
  const bool have_part = lane < P.n_part, have_out = lane < P.n_out;
  const uint32_t* gpart = P.parts + SUM_WORDS * lane;
  const uint32_t* gout = P.outs + SUM_WORDS * lane;
  uint64_t t = stamp(), u;
  int p0 = 0;
  if (lane < P.round_end[0]) load_words(rec, P.prods + PROD_WORDS * lane);
  if (have_part) load_words(rpart, gpart);
  if (have_out) load_words(rout, gout);
  __builtin_amdgcn_s_waitcnt(0);
  u = stamp();
  acc[0] += u - t;
  t = u;
  for (int r = 0; r < P.n_rounds; ++r) {
    int p1 = P.round_end[r];
    const uint32_t am = __builtin_amdgcn_readfirstlane(P.amax[r]), bm = __builtin_amdgcn_readfirstlane(P.bmax[r]);
    if (p0 + lane < p1) prod_lane(rec, P.prods + PROD_WORDS * (p0 + lane), p0 + lane, w, am, bm);
    if (r + 1 < P.n_rounds && p1 + lane < P.round_end[r + 1]) load_words(rec, P.prods + PROD_WORDS * (p1 + lane));
    p0 = p1;
    barrier();
    u = stamp();
    acc[1 + r] += u - t;
    t = u;
  }
  const uint32_t pm = __builtin_amdgcn_readfirstlane(P.pmax), om = __builtin_amdgcn_readfirstlane(P.omax);
  if (have_part) ws_put(w, SRC_Z, P.round_end[P.n_rounds - 1] + lane, sum_lane(rpart, gpart, w, pm));
  if (P.n_part) barrier();
  u = stamp();
  acc[7] += u - t;
  t = u;
  Fp o;
  if (have_out) o = sum_lane(rout, gout, w, om);
  barrier();
  u = stamp();
  acc[8] += u - t;
  t = u;
  if (have_out) ws_put(w, P.out_dst[lane], P.out_idx[lane], o);
  barrier();
  u = stamp();
  acc[9] += u - t;
}

__device__ inline Fp seed_fp(unsigned k) {
  Fp a = FP_ONE;
  a.v[1] += k;
  return a;
}

// layout: f 0..11, t 12..17, p 18..19, l 20..25, Z from 26
__global__ void __launch_bounds__(64) k_phase(int which, int iters, uint64_t* out, uint64_t* total) {
  __shared__ Slot ws[26 + ZSLOTS];
  load_consts();
  if (threadIdx.x < 26) put(ws + threadIdx.x, seed_fp(threadIdx.x));
  __syncthreads();
  uint64_t acc[NPH] = {};
  const Prog* P;
  Ws w;
  switch (which) {
    case 0: P = &FP12_CYC_SQR; w = make_ws(ws, 26, 0, 0); break;
    case 1: P = &FP12_MUL; w = make_ws(ws, 26, 0, 0, 0); break;
    case 2: P = &FP12_MUL_LINE; w = make_ws(ws, 26, 0, 20, 0); break;
    case 3: P = &MILLER_SQR_DBL; w = make_ws(ws, 26, 0, 12, 18, 0, 12, 20); break;
    case 4: P = &G2_DBL_PT; w = make_ws(ws, 26, 12, 12); break;
    default: P = &G2_ADD_STEP; w = make_ws(ws, 26, 12, 0, 18, 12, 20); break;
  }
  uint64_t t0 = stamp();
  for (int i = 0; i < iters; ++i) run_stamped(P, w.b[0], w.b[1], w.b[2], w.b[3], acc);
  uint64_t t1 = stamp();
  if (threadIdx.x == 0) {
    for (int k = 0; k < NPH; ++k) out[k] = acc[k];
    total[0] = t1 - t0;
  }
}

int main() {
  uint64_t *out, *tot;
  hipMalloc(&out, NPH * sizeof(uint64_t));
  hipMalloc(&tot, sizeof(uint64_t));
  const char* names[] = {"FP12_CYC_SQR", "FP12_MUL", "FP12_MUL_LINE", "MILLER_SQR_DBL", "G2_DBL_PT", "G2_ADD_STEP"};
  const int iters = 1000;
  for (int which = 0; which < 6; ++which) {
    hipLaunchKernelGGL(k_phase, dim3(1), dim3(64), 0, 0, which, 4, out, tot);
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL(k_phase, dim3(1), dim3(64), 0, 0, which, iters, out, tot);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    uint64_t h[NPH], T;
    hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
    hipMemcpy(&T, tot, sizeof(T), hipMemcpyDeviceToHost);
    printf("%-15s %7.2f us/call  %7.0f cyc/call (clock %.2f GHz) | fetch %.0f", names[which], ms * 1e3 / iters, (double)T / iters,
           (double)T / (ms * 1e-3) / 1e9, (double)h[0] / iters);
    for (int r = 0; r < 6; ++r)
      if (h[1 + r]) printf("  r%d %.0f", r, (double)h[1 + r] / iters);
    printf("  parts %.0f  outs %.0f  store %.0f\n", (double)h[7] / iters, (double)h[8] / iters, (double)h[9] / iters);
    fflush(stdout);
  }
  return 0;
}
