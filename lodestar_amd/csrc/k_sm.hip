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

__global__ void GBV_KERNEL_ATTR k_sm_group_sum(uint32_t g0, uint32_t G, const uint32_t* __restrict__ grp_off, const uint8_t* __restrict__ status,
                                                     const G2J* __restrict__ rS, const G1J* __restrict__ rP, G1A* __restrict__ Pg,
                                                     G2A* __restrict__ Sg, uint8_t* __restrict__ grp_state) {
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  g += g0;
  uint32_t b = grp_off[g], e = grp_off[g + 1];
  bool bad = (b == e);
  for (uint32_t i = b; i < e; ++i) bad |= status[i] != SET_OK;
  if (bad) {
    grp_state[g] = GRP_FALLBACK;
    return;
  }
  G2J s = rS[b];
  G1J p = rP[b];
  for (uint32_t i = b + 1; i < e; ++i) {
    s = jac_add(s, rS[i]);
    p = jac_add(p, rP[i]);
  }
  G1A pa;
  G2A sa;
  bool ok = jac_to_aff(pa, p);
  ok &= jac_to_aff(sa, s);
  Pg[g] = pa;
  Sg[g] = sa;
  grp_state[g] = ok ? GRP_PENDING : GRP_FALLBACK;
}

__global__ void GBV_KERNEL_ATTR k_sm_group_pairing(uint32_t g0, uint32_t G, const uint32_t* __restrict__ grp_msg, const G1A* __restrict__ Pg,
                                                         const G2A* __restrict__ Sg, const G2A* __restrict__ H,
                                                         uint8_t* __restrict__ grp_state, uint32_t* __restrict__ n_fallback) {
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  g += g0;
  uint8_t st = grp_state[g];
  if (st == GRP_PENDING) {
    bool ok = pairing_check_2(Pg[g], false, H[grp_msg[g]], g1_neg_generator(), false, Sg[g]);
    st = ok ? GRP_OK : GRP_FALLBACK;
    grp_state[g] = st;
  }
  if (st == GRP_FALLBACK) atomicAdd(n_fallback, 1u);
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
void launch_sm_group_sum(LaunchCfg c, uint32_t g0, uint32_t G, const uint32_t* grp_off, const uint8_t* status, const G2J* rS, const G1J* rP, G1A* Pg,
                         G2A* Sg, uint8_t* grp_state) {
  hipLaunchKernelGGL(k_sm_group_sum, dim3(c.blocks), dim3(c.threads), 0, c.stream, g0, G, grp_off, status, rS, rP, Pg, Sg, grp_state);
  debug_sync(c.stream, "k_sm_group_sum");
}
void launch_sm_group_pairing(LaunchCfg c, uint32_t g0, uint32_t G, const uint32_t* grp_msg, const G1A* Pg, const G2A* Sg, const G2A* H,
                             uint8_t* grp_state, uint32_t* n_fallback) {
  hipLaunchKernelGGL(k_sm_group_pairing, dim3(c.blocks), dim3(c.threads), 0, c.stream, g0, G, grp_msg, Pg, Sg, H, grp_state, n_fallback);
  debug_sync(c.stream, "k_sm_group_pairing");
}
void launch_sm_fallback(LaunchCfg c, uint32_t n, const uint32_t* set_grp, const uint32_t* grp_msg, const uint8_t* grp_state,
                        const uint8_t* status, const uint32_t* idx, const G1A* table, const G2A* S, const G2A* H, uint8_t* valid,
                        int do_fallback) {
  hipLaunchKernelGGL(k_sm_fallback, dim3(c.blocks), dim3(c.threads), 0, c.stream, n, set_grp, grp_msg, grp_state, status, idx, table, S,
                     H, valid, do_fallback);
  debug_sync(c.stream, "k_sm_fallback");
}
}  // namespace gbv
