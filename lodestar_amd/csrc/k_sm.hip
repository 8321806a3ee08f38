// Same-message path kernels (verifySignatureSetsSameMessage).
#include "launch.h"
#include "kernel_common.h"

namespace gbv {

// ---- same-message path ------------------------------------------------------------------------
__global__ void GBV_KERNEL_ATTR k_sm_prepare(uint32_t base, uint32_t n, const uint32_t* __restrict__ idx, const uint8_t* __restrict__ sig96,
                                                   const G1A* __restrict__ table, const uint8_t* __restrict__ table_ok, uint32_t table_n,
                                                   Seed seed, uint32_t nonce, G2A* __restrict__ S_out, G2J* __restrict__ rS_out,
                                                   G1J* __restrict__ rP_out, uint8_t* __restrict__ status) {
  uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  uint32_t i = base + t;
  uint32_t k = idx[i];
  uint8_t st = SET_OK;
  if (k >= table_n || !table_ok[k]) st = SET_BAD_PK;
  G2A s;
  uint8_t ds = g2_decode(s, sig96 + 96ull * i, 96);
  if (ds != PT_OK || !g2_in_subgroup(s)) st = SET_BAD_SIG;
  status[i] = st;
  if (st != SET_OK) return;
  S_out[i] = s;
  uint64_t r = prf_scalar(seed, i, nonce);
  rS_out[i] = g2_mul_u64(s, r);
  rP_out[i] = g1_mul_u64(table[k], r);
}

// ---- wave-level helpers ---------------------------------------------------------------------
__device__ inline Fp shfl_down_fp(const Fp& a, unsigned d) {
  Fp r;
#pragma unroll
  for (int i = 0; i < 12; ++i) r.v[i] = __shfl_down((unsigned)a.v[i], d, 64);
  return r;
}
__device__ inline Fp2 shfl_down_fp(const Fp2& a, unsigned d) { return Fp2{shfl_down_fp(a.c0, d), shfl_down_fp(a.c1, d)}; }
template <class F> __device__ inline Jac<F> shfl_down_jac(const Jac<F>& a, unsigned d) {
  return Jac<F>{shfl_down_fp(a.x, d), shfl_down_fp(a.y, d), shfl_down_fp(a.z, d)};
}
__device__ inline Fp6 shfl_down_fp6(const Fp6& a, unsigned d) {
  return Fp6{shfl_down_fp(a.c0, d), shfl_down_fp(a.c1, d), shfl_down_fp(a.c2, d)};
}
__device__ inline Fp12 shfl_down_fp12(const Fp12& a, unsigned d) { return Fp12{shfl_down_fp6(a.c0, d), shfl_down_fp6(a.c1, d)}; }

GBV_NI G1J g1_add(G1J a, G1J b) { return jac_add(a, b); }
GBV_NI G2J g2_add(G2J a, G2J b) { return jac_add(a, b); }

// One wave per same-message chunk: P_g = sum r_i pk_i (G1, to affine) and S_g = sum r_i sig_i (G2,
// Jacobian) by a cross-lane tree.  A chunk holding a malformed / non-subgroup signature goes
// straight to the per-set retry, as aggregateWithRandomness throwing does (index.ts:406-409).
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2)))
k_sm_chunk_reduce(uint32_t g0, const uint32_t* __restrict__ grp_off, const uint8_t* __restrict__ status, const G2J* __restrict__ rS,
                  const G1J* __restrict__ rP, G1A* __restrict__ Pg, G2J* __restrict__ SgJ, uint8_t* __restrict__ grp_state,
                  uint32_t* __restrict__ n_fallback) {
  uint32_t g = g0 + blockIdx.x;
  unsigned lane = threadIdx.x;
  uint32_t b = grp_off[g], e = grp_off[g + 1];
  int bad = (b == e);
  for (uint32_t i = b + lane; i < e; i += 64) bad |= status[i] != SET_OK;
  if (__any(bad)) {
    if (lane == 0) {
      grp_state[g] = GRP_FALLBACK;
      atomicAdd(n_fallback, 1u);
    }
    return;
  }
  G1J p = jac_infinity<Fp>();
  G2J s = jac_infinity<Fp2>();
  for (uint32_t i = b + lane; i < e; i += 64) {
    p = g1_add(p, rP[i]);
    s = g2_add(s, rS[i]);
  }
  for (unsigned d = 32; d >= 1; d >>= 1) {
    G1J po = shfl_down_jac(p, d);
    G2J so = shfl_down_jac(s, d);
    if (lane < d) {
      p = g1_add(p, po);
      s = g2_add(s, so);
    }
  }
  if (lane == 0) {
    G1A pa;
    bool ok = jac_to_aff(pa, p);
    Pg[g] = pa;
    SgJ[g] = s;
    grp_state[g] = ok ? GRP_PENDING : GRP_FALLBACK;
    if (!ok) atomicAdd(n_fallback, 1u);
  }
}

// Per block of 64 chunks of a segment: product of the pending chunks' Miller values and sum of
// their S_g, by a cross-lane tree.  has[blk] = 0 when the block holds no pending chunk.
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2)))
k_sm_seg_reduce(uint32_t g0, uint32_t G, const uint8_t* __restrict__ grp_state, const Fp12* __restrict__ F, const G2J* __restrict__ SgJ,
                Fp12* __restrict__ Fpart, G2J* __restrict__ Spart, uint8_t* __restrict__ has) {
  unsigned lane = threadIdx.x;
  uint32_t g = g0 + blockIdx.x * 64 + lane;
  int any = g < g0 + G && grp_state[g] == GRP_PENDING;
  Fp12 f = any ? F[g] : fp12_one();
  G2J s = any ? SgJ[g] : jac_infinity<Fp2>();
  for (unsigned d = 32; d >= 1; d >>= 1) {
    Fp12 fo = shfl_down_fp12(f, d);
    G2J so = shfl_down_jac(s, d);
    int ao = __shfl_down(any, d, 64);
    if (lane < d && ao) {
      f = any ? fp12_mul(f, fo) : fo;
      s = g2_add(s, so);
      any = 1;
    }
  }
  if (lane == 0) {
    has[blockIdx.x] = (uint8_t)any;
    if (any) {
      Fpart[blockIdx.x] = f;
      Spart[blockIdx.x] = s;
    }
  }
}

// valid[i] for every set; sets of failed chunks are verified one by one (2-pair check each).
__global__ void GBV_KERNEL_ATTR k_sm_fallback(uint32_t n, const uint32_t* __restrict__ set_grp, const uint32_t* __restrict__ grp_msg,
                                                    const uint8_t* __restrict__ grp_state, const uint8_t* __restrict__ status,
                                                    const uint32_t* __restrict__ idx, const G1A* __restrict__ table,
                                                    const G2A* __restrict__ S, const G2A* __restrict__ H, uint8_t* __restrict__ valid,
                                                    int do_fallback) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t g = set_grp[i];
  uint8_t st = grp_state[g];
  if (st == GRP_OK) {
    valid[i] = 1;
    return;
  }
  if (!do_fallback) return;
  if (status[i] != SET_OK) {
    valid[i] = 0;
    return;
  }
  valid[i] = pairing_check_2(table[idx[i]], false, H[grp_msg[g]], g1_neg_generator(), false, S[i]) ? 1 : 0;
}


void launch_sm_prepare(LaunchCfg c, uint32_t base, uint32_t n, const uint32_t* idx, const uint8_t* sig96, const G1A* table, const uint8_t* table_ok,
                       uint32_t table_n, const Seed& seed, uint32_t nonce, G2A* S_out, G2J* rS_out, G1J* rP_out, uint8_t* status) {
  hipLaunchKernelGGL(k_sm_prepare, dim3(c.blocks), dim3(c.threads), 0, c.stream, base, n, idx, sig96, table, table_ok, table_n, seed, nonce,
                     S_out, rS_out, rP_out, status);
  debug_sync(c.stream, "k_sm_prepare");
}
void launch_sm_chunk_reduce(LaunchCfg c, uint32_t g0, const uint32_t* grp_off, const uint8_t* status, const G2J* rS, const G1J* rP,
                            G1A* Pg, G2J* SgJ, uint8_t* grp_state, uint32_t* n_fallback) {
  hipLaunchKernelGGL(k_sm_chunk_reduce, dim3(c.blocks), dim3(64), 0, c.stream, g0, grp_off, status, rS, rP, Pg, SgJ, grp_state, n_fallback);
  debug_sync(c.stream, "k_sm_chunk_reduce");
}
void launch_sm_seg_reduce(LaunchCfg c, uint32_t g0, uint32_t G, const uint8_t* grp_state, const Fp12* F, const G2J* SgJ, Fp12* Fpart,
                          G2J* Spart, uint8_t* has) {
  hipLaunchKernelGGL(k_sm_seg_reduce, dim3((G + 63) / 64), dim3(64), 0, c.stream, g0, G, grp_state, F, SgJ, Fpart, Spart, has);
  debug_sync(c.stream, "k_sm_seg_reduce");
}
void launch_sm_fallback(LaunchCfg c, uint32_t n, const uint32_t* set_grp, const uint32_t* grp_msg, const uint8_t* grp_state,
                        const uint8_t* status, const uint32_t* idx, const G1A* table, const G2A* S, const G2A* H, uint8_t* valid,
                        int do_fallback) {
  hipLaunchKernelGGL(k_sm_fallback, dim3(c.blocks), dim3(c.threads), 0, c.stream, n, set_grp, grp_msg, grp_state, status, idx, table, S,
                     H, valid, do_fallback);
  debug_sync(c.stream, "k_sm_fallback");
}
}  // namespace gbv
