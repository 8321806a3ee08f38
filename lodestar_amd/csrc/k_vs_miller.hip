// verifySignatureSets per-set Miller values (k_vs_miller, k_vs_miller_pair, k_vs_miller_quad) in a
// translation unit of their own: these kernels run one wave per SIMD (512 registers, VGPRs + AGPRs).
#include "launch.h"
#include "kernel_common.h"
#include "pair.h"
#include "quad.h"

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
__global__ void GBV_MILLER_ATTR k_vs_miller_pair(uint32_t n, const uint8_t* __restrict__ status, const G1J* __restrict__ rP,
                                                 const G2A* __restrict__ H, Fp12* __restrict__ F) {
  vs_miller_pair_body(n, status, rP, H, F);
}

#ifndef GBV_MILLER_QUAD_WPE
#define GBV_MILLER_QUAD_WPE 1  // one wave per SIMD: 512 registers, far fewer frame spills (64-block pass Miller 6.2 -> 3.7 ms)
#endif
#define GBV_MILLER_QUAD_ATTR __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(GBV_MILLER_QUAD_WPE, GBV_MILLER_QUAD_WPE)))
// The same Miller values on lane quads (quad.h): set i on lanes 4(i mod 16) .. 4(i mod 16) + 3 of
// block i / 16; lane 2h + s writes Fp components 3s .. 3s + 2 of half h of the conjugated value.
// Every lane runs the loop (the quad exchanges need all four); quads past n or whose set did not
// decode write nothing.
// One quad's Miller value of (p, Q); lanes of inactive quads run the loop and write nothing.
__device__ __forceinline__ void quad_miller_store(const G1J& p, const G2A& Q, bool act, Fp12* __restrict__ Fi) {
  quad::Lane L;
  L.q = threadIdx.x & 3u;
  L.h = (L.q & 2u) != 0;
  L.s = (L.q & 1u) != 0;
  PairP P;
  P.z3 = fp_mul(fp_sqr(p.z), p.z);
  P.nxz = fp_neg(fp_mul(p.x, p.z));
  P.y = p.y;
  PairT T{Q.x, Q.y, fp2_one()};
  Fp6 M = fp6_sel(L.h, fp6_zero(), fp6_one());
  for (int b = 62; b >= 0; --b) {
    if (b != 62) quad::sqr(M, L);
    Line l = quad::dbl(T, P, L.q);
    quad::mul_line(M, l, L);
    if ((X_ABS >> b) & 1ull) {
      l = quad::add(T, Q, P, L.q);
      quad::mul_line(M, l, L);
    }
  }
  if (!act) return;
  if (L.h) M = fp6_neg(M);
  // this lane's three Fp of the half: s = 0 -> c0.c0, c0.c1, c1.c0; s = 1 -> c1.c1, c2.c0, c2.c1
  Fp* out = (Fp*)Fi + 6 * (L.h ? 1 : 0) + 3 * (L.s ? 1 : 0);
  out[0] = fp_sel(L.s, M.c1.c1, M.c0.c0);
  out[1] = fp_sel(L.s, M.c2.c0, M.c0.c1);
  out[2] = fp_sel(L.s, M.c2.c1, M.c1.c0);
}

__global__ void GBV_MILLER_QUAD_ATTR k_vs_miller_quad(uint32_t n, const uint8_t* __restrict__ status, const G1J* __restrict__ rP,
                                                 const G2A* __restrict__ H, Fp12* __restrict__ F) {
  const uint32_t i = blockIdx.x * 16 + (threadIdx.x >> 2);
  const bool act = i < n && status[i] == SET_OK;
  const uint32_t j = i < n ? i : n - 1;
  quad_miller_store(rP[j], H[j], act, &F[j]);
}

// Same-message chunk Miller values f_g = f_{|x|, H(m_g)}(P_g) on lane quads (k_sm_miller's latency
// form for segments of few chunks: a thread per chunk leaves such a launch a few waves long).
__global__ void GBV_MILLER_QUAD_ATTR k_sm_miller_quad(uint32_t g0, uint32_t G, const uint32_t* __restrict__ grp_msg,
                                                 const uint8_t* __restrict__ grp_state, const G1J* __restrict__ PgJ,
                                                 const G2A* __restrict__ H, Fp12* __restrict__ F) {
  const uint32_t k = blockIdx.x * 16 + (threadIdx.x >> 2);
  const uint32_t g = g0 + (k < G ? k : G - 1);
  const bool act = k < G && grp_state[g] == GRP_PENDING;
  quad_miller_store(PgJ[g], H[grp_msg[g]], act, &F[g]);
}
void launch_sm_miller_quad(LaunchCfg c, uint32_t g0, uint32_t G, const uint32_t* grp_msg, const uint8_t* grp_state, const G1J* PgJ,
                           const G2A* H, Fp12* F) {
  if (G == 0) return;
  GBV_LAUNCH("k_sm_miller_quad", k_sm_miller_quad, dim3((G + 15) / 16), dim3(64), c.stream, G, g0, G, grp_msg, grp_state, PgJ, H, F);
}

void launch_vs_miller(LaunchCfg c, uint32_t n, const uint8_t* status, const G1J* rP, const G2A* H, Fp12* F) {
  if (n == 0) return;
  // Lane quads for passes of up to vs_quad_max sets (range-sync segments, shards: the pass has fewer
  // waves than SIMDs, and four lanes per set quarter each set's latency's product count), lane pairs
  // up to vs_pair_max, one thread per set above (C3-sized passes, measured equal or better:
  // profiles/r03e; groups of 2 / 4 sets on one accumulator per thread measured slower: profiles/r05d).
  const Tuning& t = tuning();
  if (n > t.vs_pair_max) {
    GBV_LAUNCH("k_vs_miller", k_vs_miller, dim3((n + 63) / 64), dim3(64), c.stream, n, n, status, rP, H, F);
  } else if (n > t.vs_quad_max) {
    GBV_LAUNCH("k_vs_miller_pair", k_vs_miller_pair, dim3((n + 31) / 32), dim3(64), c.stream, n, n, status, rP, H, F);
  } else {
    GBV_LAUNCH("k_vs_miller_quad", k_vs_miller_quad, dim3((n + 15) / 16), dim3(64), c.stream, n, n, status, rP, H, F);
  }
}

}  // namespace gbv
