// Same-message path kernels (verifySignatureSetsSameMessage).
#include <cstdlib>

#include "launch.h"
#include "kernel_common.h"


namespace gbv {

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

GBV_NI G1J g1_add(G1J a, G1J b) { return jac_add(a, b); }
GBV_NI G2J g2_add(G2J a, G2J b) { return jac_add(a, b); }
// ---- same-message path ------------------------------------------------------------------------
constexpr unsigned SCAN_W = 8;  // lanes per scan group (power of two, <= 64)

// Per set: Signature.fromBytes(sig, true) (decode + subgroup), then the randomised terms
// r_i sig_i, r_i pk_i of aggregateWithRandomness (jobItem.ts:73).  Each group of SCAN_W lanes
// then sums its terms per chunk with a segmented suffix scan (log2(SCAN_W) levels of point
// additions) and the first lane of every chunk segment in the group writes the segment's sum at
// its own set index; k_sm_chunk_finish adds the <= ceil(len/SCAN_W)+1 segment sums of a chunk.
//
// The signatures were decoded by k_sig_decode (k_dec.hip, its own kernel at a higher occupancy):
// status[i] holds the decode code and S_out[i] the point, so this kernel starts at the subgroup check.
template <bool WITH_G2>
__global__ void GBV_KERNEL_ATTR k_sm_prepare(uint32_t base, uint32_t n, const uint32_t* __restrict__ idx, const uint8_t* __restrict__ sig96,
                                             const uint32_t* __restrict__ set_grp, const G1A* __restrict__ table,
                                             const uint8_t* __restrict__ table_ok, uint32_t table_n, const uint4* __restrict__ comb,
                                             const uint8_t* __restrict__ comb_ok, Seed seed, uint32_t nonce, G2A* __restrict__ S_out,
                                             G2J* __restrict__ Sh_out, G1J* __restrict__ Ph_out, uint8_t* __restrict__ status) {
  unsigned lane = threadIdx.x;
  uint32_t t = blockIdx.x * 64 + lane;
  bool act = t < n;
  uint32_t i = base + t;
  uint32_t key = act ? set_grp[i] : 0xffffffffu;
  G2J rs = jac_infinity<Fp2>();
  G1J rp = jac_infinity<Fp>();
  if (act) {
    uint32_t k = idx[i];
    uint8_t st = SET_OK;
    if (k >= table_n || !table_ok[k]) st = SET_BAD_PK;
    G2A s;
    const uint8_t ds = status[i];
    if (ds == PT_OK) s = S_out[i];
    if (ds != PT_OK || !g2_in_subgroup(s)) st = SET_BAD_SIG;
    status[i] = st;
    if (st == SET_OK) {
      uint64_t r = prf_scalar(seed, i, nonce);
      if (comb && comb_ok[k]) {  // r pk from the validator's comb table (curve.h comb_mul)
        rp = comb_mul(comb + (size_t)k * (COMB_ENTRIES * COMB_U4), (uint32_t)r, (uint32_t)(r >> 32));
        if (WITH_G2 && !randomize_g2(s, r, &rs)) {  // unreachable for subgroup points: both terms with plain r
          rs = g2_mul_u64(s, r);
          rp = g1_mul_u64(table[k], r);
        }
      } else if (WITH_G2) {
        G1A pk = table[k];
        if (!randomize_pair(pk, s, r, &rp, &rs)) {  // unreachable for subgroup points; plain 64-bit r then
          rs = g2_mul_u64(s, r);
          rp = g1_mul_u64(pk, r);
        }
      } else {
        G1A pk = table[k];
        if (!randomize_g1(pk, r, &rp)) rp = g1_mul_u64(pk, r);
      }
    }
  }
  // segmented suffix scan inside each group of SCAN_W lanes (3 levels: the whole wave pays every
  // level, so fewer levels = less work here; k_sm_chunk_finish adds the group sums of a chunk)
  for (unsigned d = 1; d < SCAN_W; d <<= 1) {
    G1J po = shfl_down_jac(rp, d);
    uint32_t ko = __shfl_down(key, d, 64);
    bool take = (lane & (SCAN_W - 1)) + d < SCAN_W && ko == key;
    if (WITH_G2) {
      G2J so = shfl_down_jac(rs, d);
      if (take) rs = g2_add(rs, so);
    }
    if (take) rp = jac_add(rp, po);  // inline: an out-of-line G1 addition copies both points through scratch
  }
  uint32_t kprev = __shfl_up(key, 1, 64);
  if (act && ((lane & (SCAN_W - 1)) == 0 || kprev != key)) {
    if (WITH_G2) Sh_out[i] = rs;
    Ph_out[i] = rp;
  }
}

// After k_sm_prep_roles_quad (k_vs.hip): per set the verdict -- pubkey slot, decode code, the
// cooperative subgroup check (sub_ok) -- merged as k_sm_prepare merges it (a bad signature outranks a
// bad key), the set's r pk / r sig (Ph / Sh at its own index) kept only when it is valid, then the
// 8-set segmented scan with the sums written at the run heads (in place: every lane reads its own
// terms before the scan).
__global__ void GBV_KERNEL_ATTR k_sm_prep_scan(uint32_t base, uint32_t n, const uint32_t* __restrict__ idx,
                                               const uint32_t* __restrict__ set_grp, const uint8_t* __restrict__ table_ok,
                                               uint32_t table_n, const uint8_t* __restrict__ sub_ok, uint8_t* __restrict__ status,
                                               G2J* __restrict__ Sh, G1J* __restrict__ Ph) {
  const unsigned lane = threadIdx.x;
  const uint32_t t = blockIdx.x * 64 + lane;
  const bool act = t < n;
  const uint32_t i = base + t;
  const uint32_t key = act ? set_grp[i] : 0xffffffffu;
  G2J rs = jac_infinity<Fp2>();
  G1J rp = jac_infinity<Fp>();
  if (act) {
    const uint32_t k = idx[i];
    uint8_t st = (k >= table_n || !table_ok[k]) ? SET_BAD_PK : SET_OK;
    if (status[i] != PT_OK || !sub_ok[i]) st = SET_BAD_SIG;
    status[i] = st;
    if (st == SET_OK) {
      rs = Sh[i];
      rp = Ph[i];
    }
  }
  for (unsigned d = 1; d < SCAN_W; d <<= 1) {
    G1J po = shfl_down_jac(rp, d);
    uint32_t ko = __shfl_down(key, d, 64);
    bool take = (lane & (SCAN_W - 1)) + d < SCAN_W && ko == key;
    G2J so = shfl_down_jac(rs, d);
    if (take) rs = g2_add(rs, so);
    if (take) rp = jac_add(rp, po);
  }
  uint32_t kprev = __shfl_up(key, 1, 64);
  if (act && ((lane & (SCAN_W - 1)) == 0 || kprev != key)) {
    Sh[i] = rs;
    Ph[i] = rp;
  }
}

// The G2 half of k_sm_prepare for a segment whose fast check used the bucket MSM (k_msm.hip) and
// FAILED (or holds a chunk bound for the per-set path): the failure path needs the per-set
// r_i sig_i group sums (Sh) and the chunk sums S_g after all.  Same r_i (prf_scalar of the same seed/nonce/index), same 8-lane scan, so Sh/S_g are
// exactly what k_sm_prepare<true> would have written.  Exits at once when the segment passed.
__global__ void GBV_KERNEL_ATTR k_sm_redo_g2(uint32_t base, uint32_t n, const uint32_t* __restrict__ set_grp,
                                             const uint8_t* __restrict__ status, const G2A* __restrict__ S, Seed seed, uint32_t nonce,
                                             const uint8_t* __restrict__ seg_ok, const uint32_t* __restrict__ n_fallback,
                                             G2J* __restrict__ Sh_out) {
  // a passing segment still needs the per-set terms when one of its chunks went to the per-set
  // path (malformed / non-subgroup signature): the run checks read Sh (k_sm_fb_blocks*)
  if (*seg_ok && *n_fallback == 0) return;
  unsigned lane = threadIdx.x;
  uint32_t t = blockIdx.x * 64 + lane;
  bool act = t < n;
  uint32_t i = base + t;
  uint32_t key = act ? set_grp[i] : 0xffffffffu;
  G2J rs = jac_infinity<Fp2>();
  if (act && status[i] == SET_OK) {
    G2A s = S[i];
    uint64_t r = prf_scalar(seed, i, nonce);
    if (!randomize_g2(s, r, &rs)) rs = g2_mul_u64(s, r);
  }
  for (unsigned d = 1; d < SCAN_W; d <<= 1) {
    G2J so = shfl_down_jac(rs, d);
    uint32_t ko = __shfl_down(key, d, 64);
    if ((lane & (SCAN_W - 1)) + d < SCAN_W && ko == key) rs = g2_add(rs, so);
  }
  uint32_t kprev = __shfl_up(key, 1, 64);
  if (act && ((lane & (SCAN_W - 1)) == 0 || kprev != key)) Sh_out[i] = rs;
}

// S_g of every pending chunk of a failed MSM segment from the Sh written by k_sm_redo_g2.
__global__ void GBV_KERNEL_ATTR k_sm_chunk_finish_s(uint32_t g0, uint32_t G, uint32_t s0, const uint32_t* __restrict__ grp_off,
                                                    const uint8_t* __restrict__ grp_state, const G2J* __restrict__ Sh,
                                                    const uint8_t* __restrict__ seg_ok, G2J* __restrict__ SgJ) {
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (*seg_ok || g >= G) return;
  g += g0;
  if (grp_state[g] != GRP_PENDING) return;
  uint32_t b = grp_off[g], e = grp_off[g + 1];
  G2J s = Sh[b];
  for (uint32_t q = s0 + ((b - s0) / SCAN_W + 1) * SCAN_W; q < e; q += SCAN_W) s = g2_add(s, Sh[q]);
  SgJ[g] = s;
}

// Per chunk (one thread): P_g = sum r_i pk_i, S_g = sum r_i sig_i from the segment sums at the
// chunk start and at every SCAN_W-set group boundary inside it.  P_g stays Jacobian: the Miller loop
// takes Jacobian P (lines scaled by Z^3, which the final exponentiation removes).  The sums hold the
// chunk's decodable, in-group sets only (k_sm_prepare leaves a rejected set's terms at infinity): a
// malformed / non-subgroup signature is false on its own, and the chunk's check then decides the
// others -- the booleans of the reference's per-set retry after aggregateWithRandomness throws
// (index.ts:406-409, jobItem.ts:93-125).  A chunk without any such set is done: all false.
__global__ void GBV_KERNEL_ATTR k_sm_chunk_finish(uint32_t g0, uint32_t G, uint32_t s0, const uint32_t* __restrict__ grp_off,
                                                  const uint8_t* __restrict__ status, const G2J* __restrict__ Sh,
                                                  const G1J* __restrict__ Ph, G1J* __restrict__ PgJ, G2J* __restrict__ SgJ,
                                                  uint8_t* __restrict__ grp_state, uint32_t* __restrict__ n_fallback) {
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  g += g0;
  uint32_t b = grp_off[g], e = grp_off[g + 1];
  bool any = false;
  for (uint32_t i = b; i < e; ++i) any |= status[i] == SET_OK;
  if (!any) {  // no set to verify (every one malformed / outside the group / without a usable key): all false
    grp_state[g] = GRP_OK;
    return;
  }
  bool bad = false;
  {
    G1J p = Ph[b];
    G2J s = Sh ? Sh[b] : jac_infinity<Fp2>();  // Sh == nullptr: the segment's G2 sum is the MSM's
    for (uint32_t q = s0 + ((b - s0) / SCAN_W + 1) * SCAN_W; q < e; q += SCAN_W) {
      p = g1_add(p, Ph[q]);
      if (Sh) s = g2_add(s, Sh[q]);
    }
    bad = jac_is_inf(p);
    PgJ[g] = p;
    SgJ[g] = s;
  }
  grp_state[g] = bad ? GRP_FALLBACK : GRP_PENDING;
  if (bad) atomicAdd(n_fallback, 1u);
}

// The same with one wave per chunk (segments of few chunks: a lone gossip call): lane k adds in the
// k-th group sum of the chunk by a cross-lane tree (log2 of the group count levels instead of a
// serial chain of group additions).  Same sums, same grp_state / n_fallback as k_sm_chunk_finish.
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2)))
k_sm_chunk_finish_wave(uint32_t g0, uint32_t s0, const uint32_t* __restrict__ grp_off, const uint8_t* __restrict__ status,
                       const G2J* __restrict__ Sh, const G1J* __restrict__ Ph, G1J* __restrict__ PgJ, G2J* __restrict__ SgJ,
                       uint8_t* __restrict__ grp_state, uint32_t* __restrict__ n_fallback) {
  const uint32_t g = g0 + blockIdx.x;
  const unsigned lane = threadIdx.x;
  const uint32_t b = grp_off[g], e = grp_off[g + 1];
  int any_ok = 0;
  for (uint32_t i = b + lane; i < e; i += 64) any_ok |= status[i] == SET_OK;
  if (!__any(any_ok)) {  // nothing to verify: all false (as k_sm_chunk_finish)
    if (lane == 0) grp_state[g] = GRP_OK;
    return;
  }
  int bad = 0;
  // group starts: the chunk start, then every SCAN_W-set boundary of the segment inside the chunk
  // (lane k takes groups k, k + 64, ...: any chunk length)
  int any = 0;
  G1J p = jac_infinity<Fp>();
  G2J s = jac_infinity<Fp2>();
  for (uint32_t k = lane; !bad; k += 64) {
    const uint32_t q = k == 0 ? b : s0 + ((b - s0) / SCAN_W + k) * SCAN_W;
    if (q >= e) break;
    p = any ? g1_add(p, Ph[q]) : Ph[q];
    if (Sh) s = any ? g2_add(s, Sh[q]) : Sh[q];
    any = 1;
  }
  for (unsigned d = 32; d >= 1; d >>= 1) {
    G1J po = shfl_down_jac(p, d);
    G2J so = shfl_down_jac(s, d);
    int ao = __shfl_down(any, d, 64);
    if (lane < d && ao) {
      p = any ? g1_add(p, po) : po;
      if (Sh) s = any ? g2_add(s, so) : so;
      any = 1;
    }
  }
  if (lane == 0) {
    if (!bad) {
      bad = jac_is_inf(p);
      PgJ[g] = p;
      SgJ[g] = s;
    }
    grp_state[g] = bad ? GRP_FALLBACK : GRP_PENDING;
    if (bad) atomicAdd(n_fallback, 1u);
  }
}

// Miller value f_g = f_{|x|, H(m_g)}(P_g) of every pending chunk, one thread per chunk: the
// chunk count (~1/80 of the sets) is small, so these waves take few slots beside k_sm_prepare.
__global__ void GBV_KERNEL_ATTR k_sm_miller(uint32_t g0, uint32_t G, const uint32_t* __restrict__ grp_msg, const uint8_t* __restrict__ grp_state,
                                            const G1J* __restrict__ PgJ, const G2A* __restrict__ H, Fp12* __restrict__ F) {
  GBV_TAIL_WAVE_PRIO();
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  g += g0;
  if (grp_state[g] != GRP_PENDING) return;
  F[g] = miller_loop_1j(PgJ[g], H[grp_msg[g]]);
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
  if (st == GRP_OK) {  // the chunk's check held for its decodable, in-group sets (k_sm_chunk_finish)
    valid[i] = status[i] == SET_OK ? 1 : 0;
    return;
  }
  if (!do_fallback) return;
  if (status[i] != SET_OK) {
    valid[i] = 0;
    return;
  }
  valid[i] = pairing_check_2(table[idx[i]], false, H[grp_msg[g]], g1_neg_generator(), false, S[i]) ? 1 : 0;
}


// ---- failure path of a chunk: 8-set block checks, then per-set checks ---------------------------
// The per-set retry of a failing chunk (jobItem.ts:93-125) only has to find the invalid sets.  The
// runs of a chunk inside each 8-set scan group already have their randomised sums (Sh/Ph at the run
// head, written by k_sm_prepare), so each run is first checked as one randomised batch
// e(sum r pk, H) e(-g1, sum r sig) == 1: a passing run proves its sets valid (up to the 2^-64 batch
// bound), and only the sets of failing runs pay a 2-pair check of their own.  Both levels work on
// compacted lists (atomic append), so the few failing sets do not drag whole waves with them.

// One thread per 8-set window of a segment (windows aligned like k_sm_prepare's scan groups):
// append the window's runs that belong to failed chunks.
__global__ void GBV_KERNEL_ATTR k_sm_fb_runs(uint32_t s0, uint32_t n, const uint32_t* __restrict__ set_grp,
                                             const uint8_t* __restrict__ grp_state, uint4* __restrict__ runs,
                                             uint32_t* __restrict__ n_runs, uint32_t cap) {
  uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  if (8ull * w >= n) return;
  uint32_t i = s0 + 8 * w, i1 = s0 + min(n, 8 * w + SCAN_W);
  while (i < i1) {
    uint32_t g = set_grp[i], j = i + 1;
    while (j < i1 && set_grp[j] == g) ++j;
    if (grp_state[g] == GRP_FALLBACK) {
      uint32_t k = atomicAdd(n_runs, 1u);
      if (k < cap) runs[k] = make_uint4(i, j, g, 0);
    }
    i = j;
  }
}

void launch_sm_fb_runs(LaunchCfg c, uint32_t s0, uint32_t n, const uint32_t* set_grp, const uint8_t* grp_state, uint4* runs, uint32_t* n_runs,
                       uint32_t cap) {
  uint32_t windows = (n + SCAN_W - 1) / SCAN_W;
  GBV_LAUNCH("k_sm_fb_runs", k_sm_fb_runs, dim3((windows + 63) / 64), dim3(64), c.stream, n, s0, n, set_grp, grp_state, runs, n_runs, cap);
}
void launch_sm_prepare(LaunchCfg c, uint32_t base, uint32_t n, const uint32_t* idx, const uint8_t* sig96, const uint32_t* set_grp,
                       const G1A* table, const uint8_t* table_ok, uint32_t table_n, const uint4* comb, const uint8_t* comb_ok,
                       const Seed& seed, uint32_t nonce, G2A* S_out, G2J* Sh, G1J* Ph, uint8_t* status, uint8_t* scratch8) {
  // Sh == nullptr: G1 terms only (the segment's G2 sum comes from the bucket MSM); comb == nullptr:
  // no comb tables (gbv_tune "comb" 0, or not built), the ladder forms r pk
  const dim3 grid((n + 63) / 64);
  launch_sig_decode(c.stream, base, n, sig96, S_out, status);  // decompression first, at a higher occupancy (k_dec.hip)
  if (Sh && n <= tuning().prepare_split_max) {
    // latency, few sets: the subgroup checks and the randomisation on lane quads side by side, then
    // the verdicts and the scan
    launch_sm_prep_roles_quad(c.stream, base, n, idx, table, table_ok, table_n, comb, comb_ok, seed, nonce, S_out, status, scratch8, Sh, Ph);
    GBV_LAUNCH("k_sm_prep_scan", k_sm_prep_scan, grid, dim3(64), c.stream, n, base, n, idx, set_grp, table_ok, table_n, scratch8, status, Sh, Ph);
  } else if (Sh) {
    GBV_LAUNCH("k_sm_prepare<true>", k_sm_prepare<true>, grid, dim3(64), c.stream, n, base, n, idx, sig96, set_grp, table, table_ok, table_n,
               comb, comb_ok, seed, nonce, S_out, Sh, Ph, status);
  } else {
    GBV_LAUNCH("k_sm_prepare<false>", k_sm_prepare<false>, grid, dim3(64), c.stream, n, base, n, idx, sig96, set_grp, table, table_ok,
               table_n, comb, comb_ok, seed, nonce, S_out, Sh, Ph, status);
  }
}
void launch_sm_redo_g2(LaunchCfg c, uint32_t base, uint32_t n, const uint32_t* set_grp, const uint8_t* status, const G2A* S, const Seed& seed,
                       uint32_t nonce, const uint8_t* seg_ok, const uint32_t* n_fallback, G2J* Sh) {
  GBV_LAUNCH("k_sm_redo_g2", k_sm_redo_g2, dim3((n + 63) / 64), dim3(64), c.stream, n, base, n, set_grp, status, S, seed, nonce, seg_ok, n_fallback, Sh);
}
void launch_sm_chunk_finish_s(LaunchCfg c, uint32_t g0, uint32_t G, uint32_t s0, const uint32_t* grp_off, const uint8_t* grp_state,
                              const G2J* Sh, const uint8_t* seg_ok, G2J* SgJ) {
  GBV_LAUNCH("k_sm_chunk_finish_s", k_sm_chunk_finish_s, dim3((G + 63) / 64), dim3(64), c.stream, G, g0, G, s0, grp_off, grp_state, Sh, seg_ok, SgJ);
}
void launch_sm_chunk_finish(LaunchCfg c, uint32_t g0, uint32_t G, uint32_t s0, const uint32_t* grp_off, const uint8_t* status, const G2J* Sh,
                            const G1J* Ph, G1J* PgJ, G2J* SgJ, uint8_t* grp_state, uint32_t* n_fallback) {
  if (G <= tuning().chunk_finish_wave_max)  // latency (a lone call): a wave per chunk, tree over its group sums
    GBV_LAUNCH("k_sm_chunk_finish_wave", k_sm_chunk_finish_wave, dim3(G), dim3(64), c.stream, G, g0, s0, grp_off, status, Sh, Ph, PgJ, SgJ,
               grp_state, n_fallback);
  else
    GBV_LAUNCH("k_sm_chunk_finish", k_sm_chunk_finish, dim3((G + 63) / 64), dim3(64), c.stream, G, g0, G, s0, grp_off, status, Sh, Ph, PgJ, SgJ, grp_state, n_fallback);
}
void launch_sm_miller(LaunchCfg c, uint32_t g0, uint32_t G, const uint32_t* grp_msg, const uint8_t* grp_state, const G1J* PgJ, const G2A* H,
                      Fp12* F) {
  if (G <= tuning().sm_quad_max.load(std::memory_order_relaxed)) {
    launch_sm_miller_quad(c, g0, G, grp_msg, grp_state, PgJ, H, F);
    return;
  }
  GBV_LAUNCH("k_sm_miller", k_sm_miller, dim3((G + 63) / 64), dim3(64), c.stream, G, g0, G, grp_msg, grp_state, PgJ, H, F);
}
void launch_sm_fallback(LaunchCfg c, uint32_t n, const uint32_t* set_grp, const uint32_t* grp_msg, const uint8_t* grp_state,
                        const uint8_t* status, const uint32_t* idx, const G1A* table, const G2A* S, const G2A* H, uint8_t* valid,
                        int do_fallback) {
  GBV_LAUNCH("k_sm_fallback", k_sm_fallback, dim3(c.blocks), dim3(c.threads), c.stream, n, n, set_grp, grp_msg, grp_state, status, idx, table, S, H,
             valid, do_fallback);
}
}  // namespace gbv
