// Thread-serial pairing checks of the same-message failure path (k_sm_group_check, k_sm_fb_blocks,
// k_sm_fb_sets) in a translation unit of their own, so that each can take its own register budget:
// the chunk checks (~200 waves) run at one wave per SIMD (512 registers, VGPRs + AGPRs), 32-37 ->
// 25 ms per 1M-set C5 batch; the run / per-set checks (persistent grids) stay at two waves, which
// measured faster for them (57.8 against 63 ms at one wave; profiles/r05s, r05t).
#include "launch.h"
#include "kernel_common.h"

namespace gbv {

#define GBV_FB_ATTR __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(GBV_FB_WPE, GBV_FB_WPE)))
#define GBV_GRPCHK_ATTR __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(GBV_GRPCHK_WPE, GBV_GRPCHK_WPE)))

// Failure path of a segment with many chunks: one thread per pending chunk.  It reuses the chunk's
// Miller value F[g] = f(P_g, H(m_g)) from k_sm_miller, adds the (-g1, S_g) pair and runs the final
// exponentiation: verify(msg, aggPk, aggSig) of the chunk (maybeBatch.ts:34-38).  Thread-serial
// checks keep the lanes busy when thousands of chunks are pending; a handful of chunks takes the
// wave-cooperative k_sm_group_pairing instead (lower latency per chunk).
__global__ void GBV_GRPCHK_ATTR k_sm_group_check(uint32_t g0, uint32_t G, const Fp12* __restrict__ F, const G2J* __restrict__ SgJ,
                                                 const uint8_t* __restrict__ seg_ok, uint8_t* __restrict__ grp_state,
                                                 uint32_t* __restrict__ n_fallback) {
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (*seg_ok || g >= G) return;  // launched unconditionally: no host round trip
  g += g0;
  if (grp_state[g] != GRP_PENDING) return;
  G2A sa;
  Fp12 f = F[g];
  if (jac_to_aff(sa, SgJ[g])) f = fp12_mul(f, miller_loop_1(g1_neg_generator(), sa));
  bool ok = fp12_is_one(final_exponentiation(f));
  grp_state[g] = ok ? GRP_OK : GRP_FALLBACK;
  if (!ok) atomicAdd(n_fallback, 1u);
}

void launch_sm_group_check(LaunchCfg c, uint32_t g0, uint32_t G, const Fp12* F, const G2J* SgJ, const uint8_t* seg_ok, uint8_t* grp_state,
                           uint32_t* n_fallback) {
  GBV_LAUNCH("k_sm_group_check", k_sm_group_check, dim3((G + 63) / 64), dim3(64), c.stream, G, g0, G, F, SgJ, seg_ok, grp_state, n_fallback);
}

// ---- failure path of a chunk: see k_sm.hip (k_sm_fb_runs) ------------------------------------

// Persistent over the run list: one randomised check per run; failing runs append their sets.
__global__ void GBV_FB_ATTR k_sm_fb_blocks(const uint4* __restrict__ runs, const uint32_t* __restrict__ n_runs, uint32_t cap,
                                               const uint8_t* __restrict__ status, const uint32_t* __restrict__ grp_msg,
                                               const G2J* __restrict__ Sh, const G1J* __restrict__ Ph, const G2A* __restrict__ H,
                                               uint8_t* __restrict__ valid, uint32_t* __restrict__ set_list, uint32_t* __restrict__ n_list,
                                               uint32_t coop_max) {
  uint32_t cnt = min(*n_runs, cap);
  if (cnt <= coop_max) return;  // k_sm_fb_blocks_coop has them
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < cnt; k += gridDim.x * blockDim.x) {
    uint4 r = runs[k];
    bool any = false;
    for (uint32_t i = r.x; i < r.y; ++i) any |= status[i] == SET_OK;
    bool ok = true;
    if (any) {
      G1A pa;
      G2A sa;
      bool p_fin = jac_to_aff(pa, Ph[r.x]);
      bool s_fin = jac_to_aff(sa, Sh[r.x]);
      ok = p_fin && pairing_check_2(pa, false, H[grp_msg[r.z]], g1_neg_generator(), !s_fin, sa);
    }
    for (uint32_t i = r.x; i < r.y; ++i) {
      if (status[i] != SET_OK) {
        valid[i] = 0;
      } else if (ok) {
        valid[i] = 1;
      } else {
        set_list[atomicAdd(n_list, 1u)] = i;
      }
    }
  }
}

// Persistent over the listed sets: verify(msg, pk_i, sig_i) each (2-pair check).
__global__ void GBV_FB_ATTR k_sm_fb_sets(const uint32_t* __restrict__ set_list, const uint32_t* __restrict__ n_list,
                                             const uint32_t* __restrict__ set_grp, const uint32_t* __restrict__ grp_msg,
                                             const uint32_t* __restrict__ idx, const G1A* __restrict__ table, const G2A* __restrict__ S,
                                             const G2A* __restrict__ H, uint8_t* __restrict__ valid, uint32_t coop_max) {
  uint32_t cnt = *n_list;
  if (cnt <= coop_max) return;  // k_sm_fb_sets_coop has them
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < cnt; k += gridDim.x * blockDim.x) {
    uint32_t i = set_list[k];
    valid[i] = pairing_check_2(table[idx[i]], false, H[grp_msg[set_grp[i]]], g1_neg_generator(), false, S[i]) ? 1 : 0;
  }
}

void launch_sm_fb_blocks(LaunchCfg c, const uint4* runs, const uint32_t* n_runs, uint32_t cap, const uint8_t* status, const uint32_t* grp_msg,
                         const G2J* Sh, const G1J* Ph, const G2A* H, uint8_t* valid, uint32_t* set_list, uint32_t* n_list, uint32_t coop_max) {
  GBV_LAUNCH("k_sm_fb_blocks", k_sm_fb_blocks, dim3(c.blocks), dim3(64), c.stream, 0, runs, n_runs, cap, status, grp_msg, Sh, Ph, H, valid, set_list,
             n_list, coop_max);
}
void launch_sm_fb_sets(LaunchCfg c, const uint32_t* set_list, const uint32_t* n_list, const uint32_t* set_grp, const uint32_t* grp_msg,
                       const uint32_t* idx, const G1A* table, const G2A* S, const G2A* H, uint8_t* valid, uint32_t coop_max) {
  GBV_LAUNCH("k_sm_fb_sets", k_sm_fb_sets, dim3(c.blocks), dim3(64), c.stream, 0, set_list, n_list, set_grp, grp_msg, idx, table, S, H, valid, coop_max);
}

}  // namespace gbv
