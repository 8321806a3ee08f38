// Product / doubling-chain throughput on gfx950 at the verifier kernels' occupancies (1, 2 waves per
// SIMD, and full): the out-of-line canonical Fp product (fp.h fp_mul), the signed lazy product
// (g2_lazy.h mul28s), the squaring, and the G2 subgroup check's [|x|] Q chain in both forms.
// A/B of product variants: build twice with different -D flags (GBV_SAR28, GBV_G2_LAZY ...).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 [-D...] -o tools/ubench_prod tools/ubench_prod.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../lodestar_amd/csrc/curve.h"

using namespace gbv;
#define ITERS 512
#ifndef UB_W
#define UB_W 2
#endif

GBV_NI G2J g2_ladder_canon(G2A a, G2A b, uint32_t sa, uint32_t sb) { return ret_copy(jac_mul_2d_signed(a, b, sa, sb)); }
#define KATTR(W) __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(W, W)))
template <int W> __global__ void KATTR(W) k_fp_mul(Fp* out) {
  Fp a = FP_ONE, b = FP_ONE;
  a.v[0] += threadIdx.x;
  b.v[1] += blockIdx.x;
  for (int i = 0; i < ITERS; ++i) a = fp_mul(a, b);
  out[blockIdx.x * blockDim.x + threadIdx.x] = a;
}
template <int W> __global__ void KATTR(W) k_fp_sqr(Fp* out) {
  Fp a = FP_ONE;
  a.v[0] += threadIdx.x + blockIdx.x;
  for (int i = 0; i < ITERS; ++i) a = fp_sqr(a);
  out[blockIdx.x * blockDim.x + threadIdx.x] = a;
}
template <int W> __global__ void KATTR(W) k_mul28s(Fp* out) {
  S28 a = s28_from_fp(FP_ONE), b = s28_from_fp(FP_ONE);
  a.v[0] += threadIdx.x;
  b.v[1] += blockIdx.x;
  for (int i = 0; i < ITERS; ++i) a = mul28s(a, b);
  out[blockIdx.x * blockDim.x + threadIdx.x] = s28_to_fp(a);
}
// [|x|] Q (63 doublings + 5 additions, ~1150 products) in the lazy and the canonical form
template <int W, bool LAZY> __global__ void KATTR(W) k_xabs(Fp* out) {
  G2A q{Fp2{FP_ONE, FP_ONE}, Fp2{FP_B1, FP_ONE}};
  q.x.c0.v[0] += threadIdx.x;
  q.y.c1.v[1] += blockIdx.x;
  const G2J r = LAZY ? g2_mul_xabs_lazy(q) : g2_mul_xabs(q);
  out[blockIdx.x * blockDim.x + threadIdx.x] = fp_add(r.x.c0, r.z.c1);
}

// where the lazy doubling's time goes: 63 doublings from a fixed point, (0) s2j_dbl as it is, (1) the
// same without its s28_norm steps (wrong values, bounds unchecked: timing only), (2) the 16 products of a
// doubling alone, chained through their outputs with one add per product
template <int W, int V> __global__ void KATTR(W) k_dbl(Fp* out) {
  G2A q{Fp2{FP_ONE, FP_ONE}, Fp2{FP_B1, FP_ONE}};
  q.x.c0.v[0] += threadIdx.x;
  q.y.c1.v[1] += blockIdx.x;
  S2J s = s2j_from(jac_from_aff(q));
  if (V == 0) {
    s2j_dbl_n(&s, 63);
  } else if (V >= 100) {
#pragma nounroll
    for (int i = 0; i < 63; ++i) s = s2j_dbl_skip<V - 100>(s);
  } else {
    for (int i = 0; i < 63; ++i) {
      S28 t = s.x.c0;
#pragma unroll
      for (int k = 0; k < 16; ++k) t = mul28s(s28_add(t, s.y.c0), s.z.c1);
      s.x.c0 = t;
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s28_to_fp(s28_add(s.x.c0, s.y.c1));
}

// the G2 batch randomisation r Q (curve.h randomize_g2: tables with one inversion, then the 2-D ladder)
template <int W, bool LAZY> __global__ void KATTR(W) k_rand_g2(Fp* out) {
  G2A q{Fp2{FP_ONE, FP_ONE}, Fp2{FP_B1, FP_ONE}};
  q.x.c0.v[0] += threadIdx.x;
  q.y.c1.v[1] += blockIdx.x;
  const G2A e = g2_neg_psi2(q);
  const G2J a1 = jac_add_aff(jac_from_aff(q), e), a2 = jac_add_aff(jac_from_aff(q), G2A{e.x, fp2_neg(e.y)});
  const G2A t1{a1.x, a1.y}, t2{a2.x, a2.y};  // (not normalised: timing only)
  const uint64_t r = 0x9E3779B97F4A7C15ull * (blockIdx.x * blockDim.x + threadIdx.x + 1);
  const G2J R = LAZY ? g2_mul_2d_signed_lazy(t1, t2, (uint32_t)r, (uint32_t)(r >> 32))
                     : g2_ladder_canon(t1, t2, (uint32_t)r, (uint32_t)(r >> 32));
  out[blockIdx.x * blockDim.x + threadIdx.x] = fp_add(R.x.c0, R.z.c1);
}

typedef void (*kfn)(Fp*);
static void run(const char* name, kfn f, Fp* out, int waves, double prods_per_thread) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(f, dim3(waves), dim3(64), 0, 0, out);
  hipDeviceSynchronize();
  hipEventRecord(a);
  const int reps = 3;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(f, dim3(waves), dim3(64), 0, 0, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double prods = (double)reps * waves * 64 * prods_per_thread;
  printf("%-18s waves=%6d  %8.3f ms  %7.2f G products/s  frac %.3f (300 MAC/product of 37.0 T)\n", name, waves, ms,
         prods / (ms * 1e-3) / 1e9, prods * 300 / (ms * 1e-3) / 37.0e12);
  fflush(stdout);
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int simds = p.multiProcessorCount * 4;
  // every kernel of one binary at the same occupancy: device functions shared by kernels of different
  // waves_per_eu are compiled for the smallest register budget among them (spills in the others)
  printf("device %s CUs=%d  GBV_SAR28=%d  UB_W=%d\n", p.gcnArchName, p.multiProcessorCount, GBV_SAR28, UB_W);
  Fp* out;
  hipMalloc(&out, sizeof(Fp) * 64 * 8 * simds * 4);
  const int w = UB_W * simds;
  run("fp_mul", k_fp_mul<UB_W>, out, w, ITERS);
  run("fp_sqr", k_fp_sqr<UB_W>, out, w, ITERS);
  run("mul28s", k_mul28s<UB_W>, out, w, ITERS);
  const double xabs_prods = 63 * 16 + 5 * 29;
  run("xabs lazy", k_xabs<UB_W, true>, out, w, xabs_prods);
  run("xabs canon", k_xabs<UB_W, false>, out, w, xabs_prods);
  run("rand_g2 lazy", k_rand_g2<UB_W, true>, out, w, 31 * 16 + 31 * 29);
  run("rand_g2 canon", k_rand_g2<UB_W, false>, out, w, 31 * 16 + 31 * 29);
  run("dbl63 via s2j_dbl_n", k_dbl<UB_W, 0>, out, w, 63 * 16);
  run("dbl63 inline", k_dbl<UB_W, 100>, out, w, 63 * 16);
  run("dbl63 inline no norm", k_dbl<UB_W, 163>, out, w, 63 * 16);
  run("dbl63 prods only", k_dbl<UB_W, 2>, out, w, 63 * 16);
  return 0;
}
