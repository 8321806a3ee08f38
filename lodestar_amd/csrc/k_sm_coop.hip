// Same-message path kernels built on the wave-cooperative pairing arithmetic (coop.h): one
// workgroup = one wave = one pairing job.  Kept in their own translation unit so their small
// register budget (one Fp product per lane) is not merged with the thread-per-set kernels'.
#include <cstdlib>

#include "launch.h"
#include "kernel_common.h"
#include "coop.h"
#include "quad.h"
#include "quad_g2.h"

namespace gbv {

GBV_NI G2J g2_add_j(G2J a, G2J b) { return jac_add(a, b); }
__device__ __forceinline__ G2J quad_g2_add(const G2J& a, const G2J& b, uint32_t q) { return quad::g2_add(a, b, q); }
#define g2_add g2_add_j

__device__ inline Fp shfl_down_fp_c(const Fp& a, unsigned d) {
  Fp r;
#pragma unroll
  for (int i = 0; i < 12; ++i) r.v[i] = __shfl_down((unsigned)a.v[i], d, 64);
  return r;
}

// One wave per segment: the randomised chunk equations of the whole segment are folded into one
// check  prod_g e(P_g, H(m_g)) * e(-g1, sum_g S_g) == 1  with ONE final exponentiation.  Every
// set carries its own random 64-bit scalar, so this is blst's verifyMultipleAggregateSignatures
// over the segment's sets: it passes iff every chunk would pass its own aggregate check, except
// with probability ~2^-64 (the bound each chunk check has).  Pass -> every pending chunk is
// valid; fail -> seg_ok = 0 and the host runs the per-chunk checks, then the per-set retries.
// The Miller loop and the final exponentiation share one workspace (M_F == E_F): the (-g1, S)
// Miller value is formed first, the partial products are multiplied into it, then the final
// exponentiation runs in place -- 224 slots (28 KB of LDS) per wave.
constexpr int SEG_WS = coop::MILLER_WS > coop::FINAL_EXP_WS ? coop::MILLER_WS : coop::FINAL_EXP_WS;
static_assert(coop::M_F == coop::E_F, "shared Miller / final-exponentiation workspace");
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) k_sm_seg_check(uint32_t g0, uint32_t G, uint32_t nb, const Fp12* __restrict__ Fpart,
                                                     const G2J* __restrict__ Spart, const uint8_t* __restrict__ has,
                                                     uint8_t* __restrict__ grp_state, uint8_t* __restrict__ seg_ok,
                                                     Fp12* __restrict__ miller_out, const G2J* __restrict__ S_extra) {
  GBV_TAIL_WAVE_PRIO();
  __shared__ coop::Slot ws[SEG_WS];
  __shared__ int flags[2];
  __shared__ Fp stage[6];  // the (-g1, S) pair, staged by lane 0
  unsigned lane = threadIdx.x;
  coop::load_consts();
  // S = S_extra (the segment's sum r_i sig_i from the bucket MSM, k_msm.hip, when the chunks carry
  // none) + the partial sums; flags[0]: any partial present
  if (lane == 0) {
    G2J s = S_extra ? S_extra[0] : jac_infinity<Fp2>();
    int any = 0;
    for (uint32_t k = 0; k < nb; ++k)
      if (has[k]) {
        s = g2_add(s, Spart[k]);
        any = 1;
      }
    G2A sa;
    flags[0] = any;
    flags[1] = any && jac_to_aff(sa, s) ? 1 : 0;
    if (flags[1]) {
      G1A ng = g1_neg_generator();
      stage[0] = ng.x;
      stage[1] = ng.y;
      stage[2] = sa.x.c0;
      stage[3] = sa.x.c1;
      stage[4] = sa.y.c0;
      stage[5] = sa.y.c1;
    }
  }
  coop::barrier();
  int ok = 1;
  if (flags[0]) {
    if (flags[1]) {
      const Fp* st = stage;
      coop::miller_load_pair(ws, 0, G1A{st[0], st[1]}, G2A{Fp2{st[2], st[3]}, Fp2{st[4], st[5]}});
      coop::miller_loop(ws, 1);
    } else {
      coop::set_one12(ws + coop::E_F);
    }
    for (uint32_t k = 0; k < nb; ++k) {  // F *= the (<= 4) final partials, one after another
      if (!has[k]) continue;
      if (lane < 12) coop::put(ws + coop::E_TMP + lane, ((const Fp*)&Fpart[k])[lane]);
      coop::barrier();
      coop::mul12(ws, coop::E_Z, coop::E_F, coop::E_TMP, coop::E_F);
    }
    if (!miller_out) ok = coop::final_exp_is_one(ws) ? 1 : 0;
  }
  if (miller_out) {  // shard mode: hand out the Miller product, the caller combines shards
    if (lane < 12) ((Fp*)miller_out)[lane] = flags[0] ? coop::get(ws + coop::E_F + lane) : (lane == 0 ? FP_ONE : fp_zero());
    if (lane == 0) seg_ok[0] = (uint8_t)flags[0];
    return;
  }
  if (lane == 0) seg_ok[0] = (uint8_t)ok;
  if (!ok) return;
  for (uint32_t g = g0 + lane; g < g0 + G; g += 64)
    if (grp_state[g] == GRP_PENDING) grp_state[g] = GRP_OK;
}

// Failure path of a segment: each pending chunk on its own, e(P_g, H(m_g)) e(-g1, S_g) == 1
// (verify(msg, aggPk, aggSig) of the chunk, maybeBatch.ts:34-38); one wave per chunk.
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) k_sm_group_pairing(uint32_t g0, const uint32_t* __restrict__ grp_msg, const G1J* __restrict__ PgJ,
                                                         const G2J* __restrict__ SgJ, const G2A* __restrict__ H, const uint8_t* __restrict__ seg_ok,
                                                         uint8_t* __restrict__ grp_state, uint32_t* __restrict__ n_fallback) {
  __shared__ coop::Slot ws[SEG_WS];
  __shared__ Fp sa_lds[6];
  __shared__ int sa_ok;
  uint32_t g = g0 + blockIdx.x;
  if (*seg_ok || grp_state[g] != GRP_PENDING) return;  // launched unconditionally: no host round trip
  unsigned lane = threadIdx.x;
  coop::load_consts();
  if (lane == 0) {
    G2A sa;
    G1A pa;
    sa_ok = jac_to_aff(sa, SgJ[g]) && jac_to_aff(pa, PgJ[g]) ? 1 : 0;
    sa_lds[0] = sa.x.c0;
    sa_lds[1] = sa.x.c1;
    sa_lds[2] = sa.y.c0;
    sa_lds[3] = sa.y.c1;
    sa_lds[4] = pa.x;
    sa_lds[5] = pa.y;
  }
  coop::barrier();
  bool ok = false;
  if (sa_ok) {
    coop::miller_load_pair(ws, 0, G1A{sa_lds[4], sa_lds[5]}, H[grp_msg[g]]);
    coop::miller_load_pair(ws, 1, g1_neg_generator(), G2A{Fp2{sa_lds[0], sa_lds[1]}, Fp2{sa_lds[2], sa_lds[3]}});
    coop::miller_loop(ws, 2);
    ok = coop::final_exp_is_one(ws);
  }
  if (lane == 0) {
    grp_state[g] = ok ? GRP_OK : GRP_FALLBACK;
    if (!ok) atomicAdd(n_fallback, 1u);
  }
}

// The same check with its two Miller loops on two waves (latency: a lone gossip call ends here).
// Block (g, j) forms the Miller value of pair j of chunk g -- j = 0: (P_g, H(m_g)), j = 1:
// (-g1, S_g) -- so the chain is one Miller loop (Fp12 square + one line per bit) instead of the
// 2-pair loop's square + two lines; k_sm_group_fe multiplies the two values and exponentiates.
// pair_ok[2g + j] = 0 when the pair's point is at infinity (the chunk then goes to the per-set path,
// as k_sm_group_pairing does).
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2)))
k_sm_group_miller2(uint32_t g0, const uint32_t* __restrict__ grp_msg, const G1J* __restrict__ PgJ, const G2J* __restrict__ SgJ,
                   const G2A* __restrict__ H, const uint8_t* __restrict__ seg_ok, const uint8_t* __restrict__ grp_state,
                   Fp12* __restrict__ Fpair, uint8_t* __restrict__ pair_ok) {
  __shared__ coop::Slot ws[coop::MILLER_WS];
  __shared__ Fp st[4];
  __shared__ int ok;
  const uint32_t g = g0 + blockIdx.x, j = blockIdx.y;
  if (*seg_ok || grp_state[g] != GRP_PENDING) return;  // launched unconditionally: no host round trip
  const unsigned lane = threadIdx.x;
  coop::load_consts();
  if (lane == 0) {
    if (j == 0) {
      G1A pa;
      ok = jac_to_aff(pa, PgJ[g]) ? 1 : 0;
      st[0] = pa.x;
      st[1] = pa.y;
    } else {
      G2A sa;
      ok = jac_to_aff(sa, SgJ[g]) ? 1 : 0;
      st[0] = sa.x.c0;
      st[1] = sa.x.c1;
      st[2] = sa.y.c0;
      st[3] = sa.y.c1;
    }
    pair_ok[2 * g + j] = (uint8_t)ok;
  }
  coop::barrier();
  if (!ok) return;
  if (j == 0)
    coop::miller_load_pair(ws, 0, G1A{st[0], st[1]}, H[grp_msg[g]]);
  else
    coop::miller_load_pair(ws, 0, g1_neg_generator(), G2A{Fp2{st[0], st[1]}, Fp2{st[2], st[3]}});
  coop::miller_loop(ws, 1);
  if (lane < 12) ((Fp*)&Fpair[2 * g + j])[lane] = coop::get(ws + coop::M_F + lane);
}

__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2)))
k_sm_group_fe(uint32_t g0, const uint8_t* __restrict__ seg_ok, const Fp12* __restrict__ Fpair, const uint8_t* __restrict__ pair_ok,
              uint8_t* __restrict__ grp_state, uint32_t* __restrict__ n_fallback) {
  __shared__ coop::Slot ws[coop::FINAL_EXP_WS];
  const uint32_t g = g0 + blockIdx.x;
  if (*seg_ok || grp_state[g] != GRP_PENDING) return;
  const unsigned lane = threadIdx.x;
  bool ok = false;
  if (pair_ok[2 * g] && pair_ok[2 * g + 1]) {
    coop::load_consts();
    if (lane < 12) {
      coop::put(ws + coop::E_F + lane, ((const Fp*)&Fpair[2 * g])[lane]);
      coop::put(ws + coop::E_TMP + lane, ((const Fp*)&Fpair[2 * g + 1])[lane]);
    }
    coop::barrier();
    coop::mul12(ws, coop::E_Z, coop::E_F, coop::E_TMP, coop::E_F);
    ok = coop::final_exp_is_one(ws);
  }
  if (lane == 0) {
    grp_state[g] = ok ? GRP_OK : GRP_FALLBACK;
    if (!ok) atomicAdd(n_fallback, 1u);
  }
}



// e(P, Q) * e(-g1, S) == 1 by one wave (S = infinity drops the second pair).  Arguments must be
// wave-uniform (the callers stage them in LDS).
__device__ inline bool coop_pair_check(coop::Slot* ws, const G1A& P, const G2A& Q, bool s_inf, const G2A& S) {
  coop::miller_load_pair(ws, 0, P, Q);
  int np = 1;
  if (!s_inf) {
    coop::miller_load_pair(ws, 1, g1_neg_generator(), S);
    np = 2;
  }
  coop::miller_loop(ws, np);
  return coop::final_exp_is_one(ws);
}

// Failure path for few items (<= FB_COOP_MAX): the run checks and per-set checks of
// k_sm_fb_blocks / k_sm_fb_sets with one wave per item, for latency.  Both variants are launched;
// the one that does not own the item count exits at once.
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2)))
k_sm_fb_blocks_coop(const uint4* __restrict__ runs, const uint32_t* __restrict__ n_runs, uint32_t cap, const uint8_t* __restrict__ status,
                    const uint32_t* __restrict__ grp_msg, const G2J* __restrict__ Sh, const G1J* __restrict__ Ph, const G2A* __restrict__ H,
                    uint8_t* __restrict__ valid, uint32_t* __restrict__ set_list, uint32_t* __restrict__ n_list, int direct_ok,
                    uint32_t coop_max) {
  __shared__ coop::Slot ws[SEG_WS];
  __shared__ Fp st[6];
  __shared__ int flags[3];
  uint32_t cnt = min(*n_runs, cap);
  if (cnt > coop_max) return;
  unsigned lane = threadIdx.x;
  if (direct_ok && cnt * FB_RUN_MAX <= coop_max) {  // few sets in all: straight to the per-set checks
    for (uint32_t k = blockIdx.x; k < cnt; k += gridDim.x) {
      const uint4 r = runs[k];
      if (lane == 0)
        for (uint32_t i = r.x; i < r.y; ++i) {
          if (status[i] != SET_OK)
            valid[i] = 0;
          else
            set_list[atomicAdd(n_list, 1u)] = i;
        }
    }
    return;
  }
  if (blockIdx.x < cnt) coop::load_consts();
  for (uint32_t k = blockIdx.x; k < cnt; k += gridDim.x) {
    uint4 r = runs[k];
    if (lane == 0) {
      bool any = false;
      for (uint32_t i = r.x; i < r.y; ++i) any |= status[i] == SET_OK;
      G1A pa = G1A{fp_zero(), fp_zero()};
      G2A sa = G2A{fp2_zero(), fp2_zero()};
      flags[0] = any;
      flags[1] = any && jac_to_aff(pa, Ph[r.x]);
      flags[2] = any && jac_to_aff(sa, Sh[r.x]);
      st[0] = pa.x;
      st[1] = pa.y;
      st[2] = sa.x.c0;
      st[3] = sa.x.c1;
      st[4] = sa.y.c0;
      st[5] = sa.y.c1;
    }
    coop::barrier();
    bool ok = true;
    if (flags[0]) {
      ok = false;
      if (flags[1])
        ok = coop_pair_check(ws, G1A{st[0], st[1]}, H[grp_msg[r.z]], !flags[2], G2A{Fp2{st[2], st[3]}, Fp2{st[4], st[5]}});
    }
    if (lane == 0)
      for (uint32_t i = r.x; i < r.y; ++i) {
        if (status[i] != SET_OK)
          valid[i] = 0;
        else if (ok)
          valid[i] = 1;
        else
          set_list[atomicAdd(n_list, 1u)] = i;
      }
    coop::barrier();
  }
}

__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2)))
k_sm_fb_sets_coop(const uint32_t* __restrict__ set_list, const uint32_t* __restrict__ n_list, const uint32_t* __restrict__ set_grp,
                  const uint32_t* __restrict__ grp_msg, const uint32_t* __restrict__ idx, const G1A* __restrict__ table,
                  const G2A* __restrict__ S, const G2A* __restrict__ H, uint8_t* __restrict__ valid, uint32_t coop_max) {
  __shared__ coop::Slot ws[SEG_WS];
  uint32_t cnt = *n_list;
  if (cnt > coop_max) return;
  if (blockIdx.x < cnt) coop::load_consts();
  for (uint32_t k = blockIdx.x; k < cnt; k += gridDim.x) {
    uint32_t i = set_list[k];
    bool ok = coop_pair_check(ws, table[idx[i]], H[grp_msg[set_grp[i]]], false, S[i]);
    if (threadIdx.x == 0) valid[i] = ok ? 1 : 0;
    coop::barrier();
  }
}

// k_sm_fb_sets_coop with each check's two Miller loops on two waves (block (k, j): pair j of item
// k, both points affine and finite as there), then product + final exponentiation by one wave.
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2)))
k_sm_fb_sets_miller2(const uint32_t* __restrict__ set_list, const uint32_t* __restrict__ n_list, const uint32_t* __restrict__ set_grp,
                     const uint32_t* __restrict__ grp_msg, const uint32_t* __restrict__ idx, const G1A* __restrict__ table,
                     const G2A* __restrict__ S, const G2A* __restrict__ H, Fp12* __restrict__ Fpair, uint32_t coop_max) {
  __shared__ coop::Slot ws[coop::MILLER_WS];
  const uint32_t cnt = *n_list;
  if (cnt > coop_max) return;
  if (blockIdx.x < cnt) coop::load_consts();
  const uint32_t j = blockIdx.y;
  for (uint32_t k = blockIdx.x; k < cnt; k += gridDim.x) {
    const uint32_t i = set_list[k];
    if (j == 0)
      coop::miller_load_pair(ws, 0, table[idx[i]], H[grp_msg[set_grp[i]]]);
    else
      coop::miller_load_pair(ws, 0, g1_neg_generator(), S[i]);
    coop::miller_loop(ws, 1);
    if (threadIdx.x < 12) ((Fp*)&Fpair[2 * k + j])[threadIdx.x] = coop::get(ws + coop::M_F + threadIdx.x);
    coop::barrier();
  }
}
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2)))
k_sm_fb_sets_fe(const uint32_t* __restrict__ set_list, const uint32_t* __restrict__ n_list, const Fp12* __restrict__ Fpair,
                uint8_t* __restrict__ valid, uint32_t coop_max) {
  __shared__ coop::Slot ws[coop::FINAL_EXP_WS];
  const uint32_t cnt = *n_list;
  if (cnt > coop_max) return;
  if (blockIdx.x < cnt) coop::load_consts();
  const unsigned lane = threadIdx.x;
  for (uint32_t k = blockIdx.x; k < cnt; k += gridDim.x) {
    if (lane < 12) {
      coop::put(ws + coop::E_F + lane, ((const Fp*)&Fpair[2 * k])[lane]);
      coop::put(ws + coop::E_TMP + lane, ((const Fp*)&Fpair[2 * k + 1])[lane]);
    }
    coop::barrier();
    coop::mul12(ws, coop::E_Z, coop::E_F, coop::E_TMP, coop::E_F);
    const bool ok = coop::final_exp_is_one(ws);
    if (lane == 0) valid[set_list[k]] = ok ? 1 : 0;
    coop::barrier();
  }
}

void launch_sm_fb_blocks_coop(LaunchCfg c, const uint4* runs, const uint32_t* n_runs, uint32_t cap, const uint8_t* status,
                              const uint32_t* grp_msg, const G2J* Sh, const G1J* Ph, const G2A* H, uint8_t* valid, uint32_t* set_list,
                              uint32_t* n_list, uint32_t cm) {
  GBV_LAUNCH("k_sm_fb_blocks_coop", k_sm_fb_blocks_coop, dim3(std::max(cm, 1u)), dim3(64), c.stream, 0, runs, n_runs, cap, status, grp_msg, Sh, Ph, H,
             valid, set_list, n_list, 1, cm);
}
void launch_sm_fb_sets_coop(LaunchCfg c, const uint32_t* set_list, const uint32_t* n_list, const uint32_t* set_grp, const uint32_t* grp_msg,
                            const uint32_t* idx, const G1A* table, const G2A* S, const G2A* H, uint8_t* valid, Fp12* Fpair, uint32_t cm) {
  const uint32_t gx = std::max(cm, 1u);
  if (Fpair) {  // 2 * FB_COOP_CAP Fp12 of scratch
    GBV_LAUNCH("k_sm_fb_sets_miller2", k_sm_fb_sets_miller2, dim3(gx, 2), dim3(64), c.stream, 0, set_list, n_list, set_grp, grp_msg, idx, table, S, H, Fpair, cm);
    GBV_LAUNCH("k_sm_fb_sets_fe", k_sm_fb_sets_fe, dim3(gx), dim3(64), c.stream, 0, set_list, n_list, Fpair, valid, cm);
    return;
  }
  GBV_LAUNCH("k_sm_fb_sets_coop", k_sm_fb_sets_coop, dim3(gx), dim3(64), c.stream, 0, set_list, n_list, set_grp, grp_msg, idx, table, S, H, valid, cm);
}

// One level of a segment's reduction on lane quads: block b combines items k = 64 b + j + 16 m
// (quad j, m < 4) that are active (k < n, act[k] == act_val) into the product of their Fp12 values and
// the sum of their G2 points -- per quad three quad::mul12 / quad::g2_add at most, then a 4-level
// tree -- where the thread form ran a 6-level tree of one-lane fp12_mul + G2 additions (~580
// product latencies against ~180).  has_out[b] = 0 when the block holds no active item.
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2)))
k_seg_reduce_quad(uint32_t n, const uint8_t* __restrict__ act, uint8_t act_val, const Fp12* __restrict__ Fin, const G2J* __restrict__ Sin,
                  Fp12* __restrict__ Fout, G2J* __restrict__ Sout, uint8_t* __restrict__ has_out) {
  GBV_TAIL_WAVE_PRIO();
  const unsigned lane = threadIdx.x;
  quad::Lane L;
  L.q = lane & 3u;
  L.h = (L.q & 2u) != 0;
  L.s = (L.q & 1u) != 0;
  const uint32_t j = lane >> 2, hf = L.h ? 1u : 0u;
  Fp6 M = fp6_zero();
  G2J S = jac_infinity<Fp2>();
  int has = 0;
  for (uint32_t m = 0; m < 4; ++m) {  // quad-uniform
    const uint32_t k = blockIdx.x * 64 + j + 16 * m;
    if (k >= n || act[k] != act_val) continue;
    const Fp6 G = ((const Fp6*)&Fin[k])[hf];
    const G2J P = Sin[k];
    if (has) {
      quad::mul12(M, G, L);
      S = quad_g2_add(S, P, L.q);
    } else {
      M = G;
      S = P;
      has = 1;
    }
  }
  for (unsigned d = 8; d >= 1; d >>= 1) {
    Fp6 O;
    G2J T;
    Fp* od = (Fp*)&O;
    const Fp* md = (const Fp*)&M;
    for (int k = 0; k < 6; ++k) od[k] = shfl_down_fp_c(md[k], 4 * d);
    Fp* td = (Fp*)&T;
    const Fp* sd = (const Fp*)&S;
    for (int k = 0; k < 6; ++k) td[k] = shfl_down_fp_c(sd[k], 4 * d);
    const int ho = __shfl_down(has, 4 * d, 64);
    if (j < d && ho) {
      if (has) {
        quad::mul12(M, O, L);
        S = quad_g2_add(S, T, L.q);
      } else {
        M = O;
        S = T;
        has = 1;
      }
    }
  }
  if (lane == 0) has_out[blockIdx.x] = (uint8_t)has;
  if (!has || j != 0) return;
  if (!L.s) ((Fp6*)&Fout[blockIdx.x])[hf] = M;  // lane 0: c0, lane 2: c1
  if (L.q == 0) Sout[blockIdx.x] = S;
}

uint32_t launch_seg_reduce_quad(hipStream_t s, uint32_t g0, uint32_t G, const uint8_t* grp_state, const Fp12* F, const G2J* SgJ, Fp12* Fpart,
                                G2J* Spart, uint8_t* has, uint32_t* n_out) {
  uint32_t n = (G + 63) / 64;
  GBV_LAUNCH("k_seg_reduce_quad", k_seg_reduce_quad, dim3(n), dim3(64), s, G, G, grp_state + g0, (uint8_t)GRP_PENDING, F + g0, SgJ + g0, Fpart, Spart, has);
  uint32_t off = 0;
  while (n > 4) {
    const uint32_t m = (n + 63) / 64;
    GBV_LAUNCH("k_seg_reduce_quad", k_seg_reduce_quad, dim3(m), dim3(64), s, n, n, has + off, (uint8_t)1, Fpart + off, Spart + off, Fpart + off + n,
               Spart + off + n, has + off + n);
    off += n;
    n = m;
  }
  *n_out = n;
  return off;
}

void launch_sm_seg_check(LaunchCfg c, uint32_t g0, uint32_t G, uint8_t* grp_state, const Fp12* F, const G2J* SgJ, Fp12* Fpart, G2J* Spart,
                         uint8_t* has, uint8_t* seg_ok, Fp12* miller_out, const G2J* S_extra) {
  uint32_t nb = 0;
  const uint32_t off = launch_seg_reduce_quad(c.stream, g0, G, grp_state, F, SgJ, Fpart, Spart, has, &nb);
  GBV_LAUNCH("k_sm_seg_check", k_sm_seg_check, dim3(1), dim3(64), c.stream, G, g0, G, nb, Fpart + off, Spart + off, has + off, grp_state, seg_ok, miller_out, S_extra);
}
void launch_sm_group_pairing(LaunchCfg c, uint32_t g0, uint32_t G, const uint32_t* grp_msg, const G1J* PgJ, const G2J* SgJ, const G2A* H,
                             const uint8_t* seg_ok, uint8_t* grp_state, uint32_t* n_fallback, Fp12* Fpair, uint8_t* pair_ok) {
  if (!Fpair) {
    GBV_LAUNCH("k_sm_group_pairing", k_sm_group_pairing, dim3(G), dim3(64), c.stream, G, g0, grp_msg, PgJ, SgJ, H, seg_ok, grp_state, n_fallback);
    return;
  }
  GBV_LAUNCH("k_sm_group_miller2", k_sm_group_miller2, dim3(G, 2), dim3(64), c.stream, G, g0, grp_msg, PgJ, SgJ, H, seg_ok, grp_state, Fpair, pair_ok);
  GBV_LAUNCH("k_sm_group_fe", k_sm_group_fe, dim3(G), dim3(64), c.stream, G, g0, seg_ok, Fpair, pair_ok, grp_state, n_fallback);
}
// Product of k Fp12 Miller partials (one per shard / GPU) and ONE final exponentiation == 1?
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2)))
k_fp12_check(uint32_t k, const Fp12* __restrict__ parts, uint8_t* __restrict__ out) {
  __shared__ coop::Slot ws[coop::FINAL_EXP_WS];
  unsigned lane = threadIdx.x;
  coop::load_consts();
  coop::set_one12(ws + coop::E_F);
  for (uint32_t j = 0; j < k; ++j) {
    if (lane < 12) coop::put(ws + coop::E_TMP + lane, ((const Fp*)&parts[j])[lane]);
    coop::barrier();
    coop::mul12(ws, coop::E_Z, coop::E_F, coop::E_TMP, coop::E_F);
  }
  bool ok = coop::final_exp_is_one(ws);
  if (lane == 0) out[0] = ok ? 1 : 0;
}

// Lane-quad reductions over a chunk's sets b .. e - 1 (all with status OK), one wave: quad j takes
// sets b + j, b + j + 16, ... in a row, then a 4-level tree over the 16 quads.
//   quad_chunk_f12: the product of the sets' Miller values (quad::mul12: 15 product latencies a
//     level where one lane's fp12_mul costs 54), staged into the workspace slot ws + slot;
//   quad_chunk_g2sum: the sum of their r_i sig_i (quad::g2_add, 11 product rounds where one lane's
//     addition has 43 products), returned on every lane of quad 0.
__device__ inline void quad_chunk_f12(const Fp12* __restrict__ f, uint32_t b, uint32_t e, coop::Slot* ws, int slot, Fp* stage) {
  const unsigned lane = threadIdx.x;
  quad::Lane L;
  L.q = lane & 3u;
  L.h = (L.q & 2u) != 0;
  L.s = (L.q & 1u) != 0;
  const uint32_t j = lane >> 2, hf = L.h ? 1u : 0u;
  Fp6 M = fp6_zero();
  int has = 0;
  for (uint32_t i = b + j; i < e; i += 16) {  // quad-uniform trip count
    const Fp6 G = ((const Fp6*)&f[i])[hf];
    if (has) {
      quad::mul12(M, G, L);
    } else {
      M = G;
      has = 1;
    }
  }
  for (unsigned d = 8; d >= 1; d >>= 1) {
    Fp6 O;
    Fp* od = (Fp*)&O;
    const Fp* md = (const Fp*)&M;
    for (int k = 0; k < 6; ++k) od[k] = shfl_down_fp_c(md[k], 4 * d);
    const int ho = __shfl_down(has, 4 * d, 64);
    if (j < d && ho) {  // quad-uniform
      if (has) {
        quad::mul12(M, O, L);
      } else {
        M = O;
        has = 1;
      }
    }
  }
  for (int half = 0; half < 2; ++half) {  // lane 0 holds c0 (Fp 0..5), lane 2 c1 (Fp 6..11)
    if (lane == 2u * half)
      for (int k = 0; k < 6; ++k) stage[k] = ((const Fp*)&M)[k];
    __syncthreads();
    if (lane < 6) coop::put(ws + slot + 6 * half + lane, stage[lane]);
    __syncthreads();
  }
}

__device__ inline G2J quad_chunk_g2sum(const G2J* __restrict__ rS, uint32_t b, uint32_t e) {
  const unsigned lane = threadIdx.x;
  const uint32_t q = lane & 3u, j = lane >> 2;
  G2J S = jac_infinity<Fp2>();
  int has = 0;
  for (uint32_t i = b + j; i < e; i += 16) {
    const G2J P = rS[i];
    if (has) {
      S = quad_g2_add(S, P, q);
    } else {
      S = P;
      has = 1;
    }
  }
  for (unsigned d = 8; d >= 1; d >>= 1) {
    G2J O;
    Fp* od = (Fp*)&O;
    const Fp* sd = (const Fp*)&S;
    for (int k = 0; k < 6; ++k) od[k] = shfl_down_fp_c(sd[k], 4 * d);
    const int ho = __shfl_down(has, 4 * d, 64);
    if (j < d && ho) {
      if (has) {
        S = quad_g2_add(S, O, q);
      } else {
        S = O;
        has = 1;
      }
    }
  }
  return S;
}

// verifySignatureSets chunks (<= 255 sets each, chunkifyMaximizeChunkSize; (begin, end) pairs): one wave per chunk
// multiplies its sets' Miller values and sums r_i sig_i (lane-quad trees), then runs the
// (-g1, sum) pair and the final exponentiation cooperatively (maybeBatch.ts:17-26).
// With Fs (small passes): the (-g1, sum) Miller value was formed beside the per-set ones by
// k_vs_chunk_s_miller (fs_flag 1; 2: the sum is infinity, no pair), so this kernel only multiplies.
constexpr int CHUNK_PROD_SLOT = coop::MILLER_WS;  // 12 slots the Miller loop does not touch
static_assert(CHUNK_PROD_SLOT + 12 <= SEG_WS, "chunk product slot inside the workspace");
template <bool FS>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2)))
k_vs_chunk_coop(const uint32_t* __restrict__ chunk_be, const uint8_t* __restrict__ status, const Fp12* __restrict__ f,
                const G2J* __restrict__ rS, uint8_t* __restrict__ chunk_valid, const Fp12* __restrict__ Fs,
                const uint8_t* __restrict__ fs_flag) {
  __shared__ coop::Slot ws[SEG_WS];
  __shared__ int flags[2];
  __shared__ Fp stage[6];
  unsigned lane = threadIdx.x;
  uint32_t c = blockIdx.x;
  uint32_t b = chunk_be[2 * c], e = chunk_be[2 * c + 1];
  int bad = b == e;
  for (uint32_t i = b + lane; i < e; i += 64) bad |= status[i] != SET_OK;
  if (__any(bad)) {
    if (lane == 0) chunk_valid[c] = 0;
    return;
  }
  coop::load_consts();
  if (FS) {
    quad_chunk_f12(f, b, e, ws, coop::E_F, stage);
    if (fs_flag[c] == 1 && lane < 12) coop::put(ws + coop::E_TMP + lane, ((const Fp*)&Fs[c])[lane]);
    coop::barrier();
    if (fs_flag[c] == 1) coop::mul12(ws, coop::E_Z, coop::E_F, coop::E_TMP, coop::E_F);
    bool ok = fs_flag[c] != 0 && coop::final_exp_is_one(ws);
    if (lane == 0) chunk_valid[c] = ok ? 1 : 0;
    return;
  }
  const G2J s = quad_chunk_g2sum(rS, b, e);
  if (lane == 0) {
    G2A sa;
    flags[0] = jac_to_aff(sa, s) ? 1 : 0;
    G1A ng = g1_neg_generator();
    stage[0] = ng.x;
    stage[1] = ng.y;
    stage[2] = sa.x.c0;
    stage[3] = sa.x.c1;
    stage[4] = sa.y.c0;
    stage[5] = sa.y.c1;
  }
  coop::barrier();
  const bool pair = flags[0] != 0;
  G1A ng;
  G2A sa;
  if (pair) {
    ng = G1A{stage[0], stage[1]};
    sa = G2A{Fp2{stage[2], stage[3]}, Fp2{stage[4], stage[5]}};
  }
  __syncthreads();
  // the product first, parked above the Miller workspace (stage is reused), then the (-g1, S) Miller
  // value into E_F (shared Miller / final-exp workspace) and F = f_(-g1, S) * prod f_i
  quad_chunk_f12(f, b, e, ws, pair ? CHUNK_PROD_SLOT : coop::E_F, stage);
  if (pair) {
    coop::miller_load_pair(ws, 0, ng, sa);
    coop::miller_loop(ws, 1);
    coop::barrier();
    if (lane < 12) coop::put(ws + coop::E_TMP + lane, coop::get(ws + CHUNK_PROD_SLOT + lane));
    coop::barrier();
    coop::mul12(ws, coop::E_Z, coop::E_F, coop::E_TMP, coop::E_F);
  }
  coop::barrier();
  bool ok = coop::final_exp_is_one(ws);
  if (lane == 0) chunk_valid[c] = ok ? 1 : 0;
}

// Chunk c's sum of r_i sig_i and the Miller value of (-g1, sum), one wave per chunk, on its own stream
// beside k_vs_miller_coop (small passes), so that k_vs_chunk_coop's critical path loses that Miller
// loop (fs_flag: 0 the chunk holds a rejected set, 1 Fs[c] set, 2 the sum is infinity).  A kernel of
// its own: the serial G2 additions would otherwise raise k_vs_miller_coop's register budget.
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2)))
k_vs_chunk_s_miller(const uint8_t* __restrict__ status, const uint32_t* __restrict__ chunk_be, const G2J* __restrict__ rS,
                    Fp12* __restrict__ Fs, uint8_t* __restrict__ fs_flag) {
  __shared__ coop::Slot ws[coop::MILLER_WS];
  __shared__ Fp stage[4];
  __shared__ int ok;
  const unsigned lane = threadIdx.x;
  const uint32_t c = blockIdx.x;
  const uint32_t b = chunk_be[2 * c], e = chunk_be[2 * c + 1];
  int bad = b == e;
  for (uint32_t i = b + lane; i < e; i += 64) bad |= status[i] != SET_OK;
  if (__any(bad)) {
    if (lane == 0) fs_flag[c] = 0;
    return;
  }
  const G2J s = quad_chunk_g2sum(rS, b, e);
  coop::load_consts();
  if (lane == 0) {
    G2A sa;
    ok = jac_to_aff(sa, s) ? 1 : 0;
    stage[0] = sa.x.c0;
    stage[1] = sa.x.c1;
    stage[2] = sa.y.c0;
    stage[3] = sa.y.c1;
    fs_flag[c] = ok ? 1 : 2;
  }
  coop::barrier();
  if (!ok) return;
  coop::miller_load_pair(ws, 0, g1_neg_generator(), G2A{Fp2{stage[0], stage[1]}, Fp2{stage[2], stage[3]}});
  coop::miller_loop(ws, 1);
  if (lane < 12) ((Fp*)&Fs[c])[lane] = coop::get(ws + coop::M_F + lane);
}

// Miller value f_{|x|, H(m_i)}(r_i pk_i) of one set per wave (latency: small verifySignatureSets
// passes; k_vs_miller runs one thread per set for large ones).  Same value up to an Fp factor as the
// thread version (the final exponentiation removes it): P is made affine by lane 0 first.
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2)))
k_vs_miller_coop(const uint8_t* __restrict__ status, const G1J* __restrict__ rP, const G2A* __restrict__ H, Fp12* __restrict__ F) {
  __shared__ coop::Slot ws[coop::MILLER_WS];
  __shared__ Fp stage[2];
  __shared__ int ok;
  const unsigned lane = threadIdx.x;
  const uint32_t i = blockIdx.x;
  if (status[i] != SET_OK) return;
  coop::load_consts();
  if (lane == 0) {
    G1A pa;
    ok = jac_to_aff(pa, rP[i]) ? 1 : 0;
    stage[0] = pa.x;
    stage[1] = pa.y;
  }
  coop::barrier();
  if (!ok) {  // r_i pk_i at infinity cannot happen for a valid key (r_i != 0 mod r); F = 1 keeps the product defined
    if (lane < 12) ((Fp*)&F[i])[lane] = lane == 0 ? FP_ONE : fp_zero();
    return;
  }
  coop::miller_load_pair(ws, 0, G1A{stage[0], stage[1]}, H[i]);
  coop::miller_loop(ws, 1);
  if (lane < 12) ((Fp*)&F[i])[lane] = coop::get(ws + coop::M_F + lane);
}

void launch_vs_chunk_s_miller(hipStream_t s, uint32_t C, const uint8_t* status, const uint32_t* chunk_be, const G2J* rS, Fp12* Fs,
                              uint8_t* fs_flag) {
  GBV_LAUNCH("k_vs_chunk_s_miller", k_vs_chunk_s_miller, dim3(C), dim3(64), s, C, status, chunk_be, rS, Fs, fs_flag);
}
void launch_vs_miller_coop(hipStream_t s, uint32_t n, const uint8_t* status, const G1J* rP, const G2A* H, Fp12* F) {
  GBV_LAUNCH("k_vs_miller_coop", k_vs_miller_coop, dim3(n), dim3(64), s, n, status, rP, H, F);
}

void launch_fp12_check(LaunchCfg c, uint32_t k, const Fp12* parts, uint8_t* out) {
  GBV_LAUNCH("k_fp12_check", k_fp12_check, dim3(1), dim3(64), c.stream, k, k, parts, out);
}
void launch_vs_chunk_coop(LaunchCfg c, uint32_t C, const uint32_t* chunk_be, const uint8_t* status, const Fp12* f, const G2J* rS,
                          uint8_t* chunk_valid, const Fp12* Fs, const uint8_t* fs_flag) {
  if (Fs)
    GBV_LAUNCH("k_vs_chunk_coop<true>", k_vs_chunk_coop<true>, dim3(C), dim3(64), c.stream, C, chunk_be, status, f, rS, chunk_valid, Fs, fs_flag);
  else
    GBV_LAUNCH("k_vs_chunk_coop<false>", k_vs_chunk_coop<false>, dim3(C), dim3(64), c.stream, C, chunk_be, status, f, rS, chunk_valid, Fs, fs_flag);
}
// hash_to_G2's cofactor clearing for few messages (launch_hash_msgs' latency form, n <= GBV_HASH_COOP_MAX):
// h_eff P = [x^2 - x - 1] P + [x - 1] psi(P) + psi^2(2P) as quad_g2.h g2_clear_cofactor, with both
// [|x|] multiplications on wave 0's written-out cooperative point steps (coop::mul_xabs_point, ~0.42 ms a
// chain against ~0.85 ms on a lane quad) and the rest -- affine forms, psi maps, additions -- on one lane
// quad of each wave (wave 1's quad forms psi(P) and psi^2(2P) - psi(P) - P beside chain 1).
__global__ void __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(1)))
k_hash_clear_coop(const G2J* __restrict__ Qpre, G2A* __restrict__ H) {
  __shared__ coop::Slot ws[coop::MILLER_WS];
  __shared__ G2A sa;
  __shared__ G2J s_t1, s_psi, s_u;
  __shared__ int ok, ok2;
  const uint32_t m = blockIdx.x;
  const unsigned lane = threadIdx.x & 63u, wv = threadIdx.x >> 6, q = lane & 3u;
  const G2J p = Qpre[m];
  if (wv == 0) {
    coop::load_consts();
    if (lane < 4) {
      G2A a;
      const bool okp = quad::g2_to_aff(a, p, q);
      if (q == 0) sa = a, ok = okp ? 1 : 0;
    }
    coop::barrier();
    if (ok) coop::mul_xabs_point(ws, sa);
  } else if (lane < 4) {
    const G2J psi = quad::g2_psi(p, q);
    G2J u = quad_g2_add(quad::g2_psi(quad::g2_psi(quad::g2_dbl(p, q), q), q), jac_neg(psi), q);
    u = quad_g2_add(u, jac_neg(p), q);
    if (q == 0) s_psi = psi, s_u = u;
  }
  __syncthreads();  // [|x|] P in ws; psi(P), u in LDS
  if (wv == 0 && lane < 4 && ok) {
    const G2J t1 = jac_neg(coop::point_jac(ws));  // [x] P
    G2A a;
    const bool o2 = quad::g2_to_aff(a, quad_g2_add(t1, s_psi, q), q);  // t2 = [x] P + psi(P)
    if (q == 0) s_t1 = t1, sa = a, ok2 = o2 ? 1 : 0;
  }
  __syncthreads();
  if (wv == 0) {
    if (ok && ok2) coop::mul_xabs_point(ws, sa);
  } else if (lane < 4 && ok) {
    const G2J u = quad_g2_add(s_u, jac_neg(s_t1), q);  // u - [x] P
    if (q == 0) s_u = u;
  }
  __syncthreads();  // [|x|] t2 in ws; u - [x] P in LDS
  if (wv == 0 && lane < 4) {
    // P at infinity clears to infinity; t2 at infinity: [x] t2 is infinity too
    const G2J r = !ok ? quad::g2_clear_cofactor(p, q) : ok2 ? quad_g2_add(jac_neg(coop::point_jac(ws)), s_u, q) : s_u;
    G2A a;
    quad::g2_to_aff(a, r, q);
    if (q == 0) H[m] = a;
  }
}
void launch_hash_clear_coop(hipStream_t s, uint32_t n, const G2J* Qpre, G2A* H) {
  GBV_LAUNCH("k_hash_clear_coop", k_hash_clear_coop, dim3(n), dim3(128), s, n, Qpre, H);
}
}  // namespace gbv
