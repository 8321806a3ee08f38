// verifySignatureSets per-set Miller values (k_vs_miller, k_vs_miller_pair[2]), in a translation unit
// of their own so that the product's accumulator chains can be set for them alone: these kernels run
// one wave per SIMD, where independent v_mad_u64_u32 chains issue back to back (fp.h
// GBV_MUL28_CHAINS; GBV_MILLER_CHAINS overrides for A/B builds).
#ifndef GBV_MILLER_CHAINS
#define GBV_MILLER_CHAINS 1
#endif
#define GBV_MUL28_CHAINS GBV_MILLER_CHAINS
#ifndef GBV_VS_MILLER_LDS
#define GBV_VS_MILLER_LDS 0  // 1: k_vs_miller_lds for the one-thread-per-set passes
#endif
#include <cstring>

#include "launch.h"
#include "kernel_common.h"
#include "pair.h"

namespace gbv {

// Miller value f_{|x|, H(m_i)}(r_i pk_i) of every set that decoded (P Jacobian: the lines carry a
// Z^3 factor that the final exponentiation removes).
// One wave per SIMD (512 registers, VGPRs + AGPRs): a C3 pass of 65 536 sets is 1024 waves, one per
// SIMD anyway, and the 576-byte accumulator, T, the line and the operands then stay in registers
// (at two waves per SIMD the accumulator lived in scratch: 775 KB of HBM traffic per set).
#define GBV_MILLER_ATTR __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1)))
__global__ void GBV_MILLER_ATTR k_vs_miller(uint32_t n, const uint8_t* __restrict__ status, const G1J* __restrict__ rP,
                                            const G2A* __restrict__ H, Fp12* __restrict__ F) {
  uint32_t i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n || status[i] != SET_OK) return;
  F[i] = miller_loop_1j(rP[i], H[i]);
}

// The same Miller value with the Fp12 accumulator in LDS (k_vs_miller_lds): 36 quads (16 B) per
// lane, quad-major -- quad q of lane l at fl[64 q + l], so every access is a bank-conflict-free
// ds_read_b128 / ds_write_b128 -- 36 KB per wave, four waves (one per SIMD) per CU.  k_vs_miller's
// accumulator lives in the frame, i.e. scratch: with the callees' frames ~3.8 KB per lane, ~1 MB per
// CU, far past L1 and the XCD's L2 share, so its read-modify-writes went to HBM (~340 KB per set).
// Here the frame holds no Fp12: the square and the line product stream f's Fp6 halves through
// registers and park their Karatsuba terms in f's own slots until the outputs are formed.
typedef uint32_t q4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) q4 LQ;
struct LF12 {
  LQ* p;  // this lane's quad 0
};
__device__ __forceinline__ void lds_fence() { __asm__ __volatile__("" ::: "memory"); }  // compiler-only: reload, do not forward
__device__ __forceinline__ Fp lf_get(const LF12& f, int k) {
  const q4 a = f.p[(3 * k) * 64], b = f.p[(3 * k + 1) * 64], c = f.p[(3 * k + 2) * 64];
  Fp r;
  r.v = u32x12{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w};
  return r;
}
__device__ __forceinline__ void lf_put(const LF12& f, int k, const Fp& x) {
  f.p[(3 * k) * 64] = q4{x.v[0], x.v[1], x.v[2], x.v[3]};
  f.p[(3 * k + 1) * 64] = q4{x.v[4], x.v[5], x.v[6], x.v[7]};
  f.p[(3 * k + 2) * 64] = q4{x.v[8], x.v[9], x.v[10], x.v[11]};
}
__device__ __forceinline__ Fp2 lf_get2(const LF12& f, int k) { return Fp2{lf_get(f, 2 * k), lf_get(f, 2 * k + 1)}; }
__device__ __forceinline__ void lf_put2(const LF12& f, int k, const Fp2& x) {
  lf_put(f, 2 * k, x.c0);
  lf_put(f, 2 * k + 1, x.c1);
}
__device__ __forceinline__ Fp6 lf_get6(const LF12& f, int h) { return Fp6{lf_get2(f, 3 * h), lf_get2(f, 3 * h + 1), lf_get2(f, 3 * h + 2)}; }
__device__ __forceinline__ void lf_put6(const LF12& f, int h, const Fp6& x) {
  lf_put2(f, 3 * h, x.c0);
  lf_put2(f, 3 * h + 1, x.c1);
  lf_put2(f, 3 * h + 2, x.c2);
}

// f = f^2: c1 = 2 a0 a1, c0 = (a0 + a1)(a0 + v a1) - t - v t (t = a0 a1)
__device__ __forceinline__ void lf_sqr(const LF12& f) {
  Fp6 s, u;
  {
    const Fp6 a0 = lf_get6(f, 0), a1 = lf_get6(f, 1);
    const Fp6 t = fp6_mul(a0, a1);
    s = fp6_add(a0, a1);
    u = fp6_add(a0, fp6_mul_v(a1));
    lf_put6(f, 1, fp6_add(t, t));
    lf_put6(f, 0, fp6_add(t, fp6_mul_v(t)));  // parked until the second product is done
  }
  lds_fence();
  const Fp6 m = fp6_mul(s, u);
  lf_put6(f, 0, fp6_sub(m, lf_get6(f, 0)));
}

// f *= line (c0 + c2 v) + (c3 v) w: c0 = a + v b, c1 = e - a - b with a = f0 (c0 + c2 v),
// b = f1 (c3 v), e = (f0 + f1)(c0 + (c2 + c3) v); a and b parked in f's slots while e is formed
__device__ __forceinline__ void lf_mul_line(const LF12& f, const Line& l) {
  Fp6 s;
  {
    const Fp6 f0 = lf_get6(f, 0), f1 = lf_get6(f, 1);
    s = fp6_add(f0, f1);
    lf_put6(f, 0, fp6_mul_by_01(f0, l.c0, l.c2));
    lf_put6(f, 1, fp6_mul_by_1(f1, l.c3));
  }
  lds_fence();
  const Fp6 e = fp6_mul_by_01(s, l.c0, fp2_add(l.c2, l.c3));
  const Fp6 a = lf_get6(f, 0), b = lf_get6(f, 1);
  lf_put6(f, 1, fp6_sub(fp6_sub(e, a), b));
  lf_put6(f, 0, fp6_add(a, fp6_mul_v(b)));
}

// Fp2-granular forms: every Fp2 operand is read from LDS where it is used (lds_fence keeps the
// compiler from merging the reads into long-lived registers), so only the partial results of the
// current Fp6 product are held.
template <class FA, class FB>
__device__ __forceinline__ Fp6 fp6_mul_fn(FA A, FB B) {
  const Fp2 t0 = fp2_mul(A(0), B(0));
  const Fp2 t1 = fp2_mul(A(1), B(1));
  const Fp2 t2 = fp2_mul(A(2), B(2));
  const Fp2 c0 = fp2_add(t0, fp2_mul_xi(fp2_sub(fp2_sub(fp2_mul(fp2_add(A(1), A(2)), fp2_add(B(1), B(2))), t1), t2)));
  const Fp2 c1 = fp2_add(fp2_sub(fp2_sub(fp2_mul(fp2_add(A(0), A(1)), fp2_add(B(0), B(1))), t0), t1), fp2_mul_xi(t2));
  const Fp2 c2 = fp2_add(fp2_sub(fp2_sub(fp2_mul(fp2_add(A(0), A(2)), fp2_add(B(0), B(2))), t0), t2), t1);
  return Fp6{c0, c1, c2};
}
__device__ __forceinline__ Fp2 lf_ld2(const LF12& f, int k) {
  lds_fence();
  return lf_get2(f, k);
}
__device__ __forceinline__ void lf_sqr_fine(const LF12& f) {
  auto A0 = [&](int k) { return lf_ld2(f, k); };
  auto A1 = [&](int k) { return lf_ld2(f, 3 + k); };
  const Fp6 t = fp6_mul_fn(A0, A1);
  auto S = [&](int k) { return fp2_add(lf_ld2(f, k), lf_ld2(f, 3 + k)); };
  auto U = [&](int k) { return k == 0 ? fp2_add(lf_ld2(f, 0), fp2_mul_xi(lf_ld2(f, 5))) : fp2_add(lf_ld2(f, k), lf_ld2(f, 2 + k)); };
  const Fp6 m = fp6_mul_fn(S, U);
  lf_put6(f, 1, fp6_add(t, t));
  lf_put6(f, 0, fp6_sub(fp6_sub(m, t), fp6_mul_v(t)));
}
__device__ __forceinline__ void lf_mul_line_fine(const LF12& f, const Line& l) {
  const Fp2 c23 = fp2_add(l.c2, l.c3);
  Fp6 e;
  {  // e = (f0 + f1)(c0 + c23 v)
    auto S = [&](int k) { return fp2_add(lf_ld2(f, k), lf_ld2(f, 3 + k)); };
    const Fp2 t0 = fp2_mul(S(0), l.c0), t1 = fp2_mul(S(1), c23);
    e.c1 = fp2_sub(fp2_sub(fp2_mul(fp2_add(S(0), S(1)), fp2_add(l.c0, c23)), t0), t1);
    e.c0 = fp2_add(t0, fp2_mul_xi(fp2_mul(S(2), c23)));
    e.c2 = fp2_add(t1, fp2_mul(S(2), l.c0));
  }
  Fp6 a;
  {  // a = f0 (c0 + c2 v)
    auto F0 = [&](int k) { return lf_ld2(f, k); };
    const Fp2 t0 = fp2_mul(F0(0), l.c0), t1 = fp2_mul(F0(1), l.c2);
    a.c1 = fp2_sub(fp2_sub(fp2_mul(fp2_add(F0(0), F0(1)), fp2_add(l.c0, l.c2)), t0), t1);
    a.c0 = fp2_add(t0, fp2_mul_xi(fp2_mul(F0(2), l.c2)));
    a.c2 = fp2_add(t1, fp2_mul(F0(2), l.c0));
  }
  lds_fence();
  lf_put6(f, 0, fp6_sub(e, a));  // f0 is dead: park e - a there
  // b = f1 (c3 v) = (xi f1.c2 c3, f1.c0 c3, f1.c1 c3); then c1 = (e - a) - b, c0 = a + v b
  const Fp6 b{fp2_mul_xi(fp2_mul(lf_ld2(f, 5), l.c3)), fp2_mul(lf_ld2(f, 3), l.c3), fp2_mul(lf_ld2(f, 4), l.c3)};
  lds_fence();
  lf_put6(f, 1, fp6_sub(lf_get6(f, 0), b));
  lf_put6(f, 0, fp6_add(a, fp6_mul_v(b)));
}
#ifndef GBV_LF_FINE
#define GBV_LF_FINE 1
#endif

__global__ void GBV_MILLER_ATTR k_vs_miller_lds(uint32_t n, const uint8_t* __restrict__ status, const G1J* __restrict__ rP,
                                                const G2A* __restrict__ H, Fp12* __restrict__ F) {
  __shared__ q4 fl[36 * 64];
  const uint32_t i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n || status[i] != SET_OK) return;  // no barriers below: each lane owns its quads
  const LF12 f{(LQ*)fl + threadIdx.x};
  const G1J p = rP[i];
  const Fp z3 = fp_mul(fp_sqr(p.z), p.z);
  const Fp nxz = fp_neg(fp_mul(p.x, p.z));
  const Fp py = p.y;
  G2Proj T{H[i].x, H[i].y, fp2_one()};
  lf_put6(f, 0, fp6_one());
  lf_put6(f, 1, fp6_zero());
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    if (b != 62) GBV_LF_FINE ? lf_sqr_fine(f) : lf_sqr(f);
    Line l = dbl_step(T, nxz, py);
    l.c0 = fp2_mul_fp(l.c0, z3);
    GBV_LF_FINE ? lf_mul_line_fine(f, l) : lf_mul_line(f, l);
    if ((X_ABS >> b) & 1ull) {
      const G2A Q = H[i];  // re-read (L2): not held in registers across the loop
      l = add_step(T, Q, nxz, py);
      l.c0 = fp2_mul_fp(l.c0, z3);
      GBV_LF_FINE ? lf_mul_line_fine(f, l) : lf_mul_line(f, l);
    }
  }
  Fp12 out;
  out.c0 = lf_get6(f, 0);
  out.c1 = fp6_neg(lf_get6(f, 1));  // conjugation for x < 0
  F[i] = out;
}

// The same Miller values on lane pairs (pair.h): set i on lanes 2(i mod 32), 2(i mod 32) + 1 of block
// i / 32; lane 0 of the pair writes c0 of the conjugated value, lane 1 c1.  Every lane runs the loop
// (the pair exchanges need both lanes); pairs past n or whose set did not decode write nothing.
__device__ __forceinline__ void vs_miller_pair_body(uint32_t n, const uint8_t* __restrict__ status, const G1J* __restrict__ rP,
                                                     const G2A* __restrict__ H, Fp12* __restrict__ F) {
  const bool h = (threadIdx.x & 1) != 0;
  const uint32_t i = blockIdx.x * 32 + (threadIdx.x >> 1);
  const bool act = i < n && status[i] == SET_OK;
  const uint32_t j = i < n ? i : n - 1;
  const G1J p = rP[j];
  PairP P;
  P.z3 = fp_mul(fp_sqr(p.z), p.z);
  P.nxz = fp_neg(fp_mul(p.x, p.z));
  P.y = p.y;
  const G2A Q = H[j];
  PairT T{Q.x, Q.y, fp2_one()};
  Fp6 M = fp6_sel(h, fp6_zero(), fp6_one());
  for (int b = 62; b >= 0; --b) {
    if (b != 62) pair_sqr(M, h);
    Line l = pair_dbl(T, P, h);
    pair_mul_line(M, l, h);
    if ((X_ABS >> b) & 1ull) {
      l = pair_add(T, Q, P, h);
      pair_mul_line(M, l, h);
    }
  }
  if (act) ((Fp6*)&F[i])[h ? 1 : 0] = h ? fp6_neg(M) : M;
}
// one wave per SIMD (no spills) and two waves per SIMD (the 256-register budget: some spills, but
// twice the waves to hide the product chains' latency); GBV_VS_MILLER selects (A/B)
__global__ void GBV_MILLER_ATTR k_vs_miller_pair(uint32_t n, const uint8_t* __restrict__ status, const G1J* __restrict__ rP,
                                                 const G2A* __restrict__ H, Fp12* __restrict__ F) {
  vs_miller_pair_body(n, status, rP, H, F);
}
__global__ void GBV_KERNEL_ATTR k_vs_miller_pair2(uint32_t n, const uint8_t* __restrict__ status, const G1J* __restrict__ rP,
                                                  const G2A* __restrict__ H, Fp12* __restrict__ F) {
  vs_miller_pair_body(n, status, rP, H, F);
}

void launch_vs_miller(LaunchCfg c, uint32_t n, const uint8_t* status, const G1J* rP, const G2A* H, Fp12* F) {
  if (n == 0) return;
  // Lane pairs for passes of up to PAIR_MAX sets (range-sync segments: the pairs halve each set's
  // latency and the pass has fewer waves than SIMDs), one thread per set above (C3-sized passes,
  // measured equal or better: profiles/r03e).  GBV_VS_MILLER=thread / pair / pair2 (two waves per
  // SIMD) / lds (accumulator in LDS) forces one form (A/B).
  constexpr uint32_t PAIR_MAX = 32768;
  static const char* sel = getenv("GBV_VS_MILLER");
  const bool thread = sel ? sel[0] == 't' : n > PAIR_MAX;
  static const bool pair2 = sel && !strcmp(sel, "pair2");
  const bool lds = sel ? !strcmp(sel, "lds") : (GBV_VS_MILLER_LDS && thread);
  if (lds) {
    hipLaunchKernelGGL(k_vs_miller_lds, dim3((n + 63) / 64), dim3(64), 0, c.stream, n, status, rP, H, F);
    debug_sync(c.stream, "k_vs_miller_lds");
  } else if (thread) {
    hipLaunchKernelGGL(k_vs_miller, dim3((n + 63) / 64), dim3(64), 0, c.stream, n, status, rP, H, F);
    debug_sync(c.stream, "k_vs_miller");
  } else if (pair2) {
    hipLaunchKernelGGL(k_vs_miller_pair2, dim3((n + 31) / 32), dim3(64), 0, c.stream, n, status, rP, H, F);
    debug_sync(c.stream, "k_vs_miller_pair2");
  } else {
    hipLaunchKernelGGL(k_vs_miller_pair, dim3((n + 31) / 32), dim3(64), 0, c.stream, n, status, rP, H, F);
    debug_sync(c.stream, "k_vs_miller_pair");
  }
}

}  // namespace gbv
