// Same-message path kernels (verifySignatureSetsSameMessage).
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
__device__ inline Fp6 shfl_down_fp6(const Fp6& a, unsigned d) {
  return Fp6{shfl_down_fp(a.c0, d), shfl_down_fp(a.c1, d), shfl_down_fp(a.c2, d)};
}
__device__ inline Fp12 shfl_down_fp12(const Fp12& a, unsigned d) { return Fp12{shfl_down_fp6(a.c0, d), shfl_down_fp6(a.c1, d)}; }

GBV_NI G1J g1_add(G1J a, G1J b) { return jac_add(a, b); }
GBV_NI G2J g2_add(G2J a, G2J b) { return jac_add(a, b); }
// ---- same-message path ------------------------------------------------------------------------
constexpr unsigned SCAN_W = 8;  // lanes per scan group (power of two, <= 64)

// Per set: Signature.fromBytes(sig, true) (decode + subgroup), then the randomised terms
// r_i sig_i, r_i pk_i of aggregateWithRandomness (jobItem.ts:73).  Each group of SCAN_W lanes
// then sums its terms per chunk with a segmented suffix scan (log2(SCAN_W) levels of point
// additions) and the first lane of every chunk segment in the group writes the segment's sum at
// its own set index; k_sm_chunk_finish adds the <= ceil(len/SCAN_W)+1 segment sums of a chunk.
__global__ void GBV_KERNEL_ATTR k_sm_prepare(uint32_t base, uint32_t n, const uint32_t* __restrict__ idx, const uint8_t* __restrict__ sig96,
                                             const uint32_t* __restrict__ set_grp, const G1A* __restrict__ table,
                                             const uint8_t* __restrict__ table_ok, uint32_t table_n, Seed seed, uint32_t nonce,
                                             G2A* __restrict__ S_out, G2J* __restrict__ Sh_out, G1J* __restrict__ Ph_out,
                                             uint8_t* __restrict__ status) {
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
    uint8_t ds = g2_decode(s, sig96 + 96ull * i, 96);
    if (ds != PT_OK || !g2_in_subgroup(s)) st = SET_BAD_SIG;
    status[i] = st;
    if (st == SET_OK) {
      S_out[i] = s;
      uint64_t r = prf_scalar(seed, i, nonce);
      G1A pk = table[k];
      if (!randomize_pair(pk, s, r, &rp, &rs)) {  // unreachable for subgroup points; plain 64-bit r then
        rs = g2_mul_u64(s, r);
        rp = g1_mul_u64(pk, r);
      }
    }
  }
  // segmented suffix scan inside each group of SCAN_W lanes (3 levels: the whole wave pays every
  // level, so fewer levels = less work here; k_sm_chunk_finish adds the group sums of a chunk)
  for (unsigned d = 1; d < SCAN_W; d <<= 1) {
    G2J so = shfl_down_jac(rs, d);
    G1J po = shfl_down_jac(rp, d);
    uint32_t ko = __shfl_down(key, d, 64);
    if ((lane & (SCAN_W - 1)) + d < SCAN_W && ko == key) {
      rs = g2_add(rs, so);
      rp = g1_add(rp, po);
    }
  }
  uint32_t kprev = __shfl_up(key, 1, 64);
  if (act && ((lane & (SCAN_W - 1)) == 0 || kprev != key)) {
    Sh_out[i] = rs;
    Ph_out[i] = rp;
  }
}

// Per chunk (one thread): P_g = sum r_i pk_i, S_g = sum r_i sig_i from the segment sums at the
// chunk start and at every SCAN_W-set group boundary inside it.  P_g stays Jacobian: the Miller loop
// takes Jacobian P (lines scaled by Z^3, which the final exponentiation removes).  A chunk holding
// a malformed / non-subgroup signature goes straight to the per-set retry, as
// aggregateWithRandomness throwing does (index.ts:406-409).
__global__ void GBV_KERNEL_ATTR k_sm_chunk_finish(uint32_t g0, uint32_t G, uint32_t s0, const uint32_t* __restrict__ grp_off,
                                                  const uint8_t* __restrict__ status, const G2J* __restrict__ Sh,
                                                  const G1J* __restrict__ Ph, G1J* __restrict__ PgJ, G2J* __restrict__ SgJ,
                                                  uint8_t* __restrict__ grp_state, uint32_t* __restrict__ n_fallback) {
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  g += g0;
  uint32_t b = grp_off[g], e = grp_off[g + 1];
  bool bad = (b == e);
  for (uint32_t i = b; i < e; ++i) bad |= status[i] != SET_OK;
  if (!bad) {
    G1J p = Ph[b];
    G2J s = Sh[b];
    for (uint32_t q = s0 + ((b - s0) / SCAN_W + 1) * SCAN_W; q < e; q += SCAN_W) {
      p = g1_add(p, Ph[q]);
      s = g2_add(s, Sh[q]);
    }
    bad = jac_is_inf(p);
    PgJ[g] = p;
    SgJ[g] = s;
  }
  grp_state[g] = bad ? GRP_FALLBACK : GRP_PENDING;
  if (bad) atomicAdd(n_fallback, 1u);
}

// Miller value f_g = f_{|x|, H(m_g)}(P_g) of every pending chunk, one thread per chunk: the
// chunk count (~1/80 of the sets) is small, so these waves take few slots beside k_sm_prepare.
__global__ void GBV_KERNEL_ATTR k_sm_miller(uint32_t g0, uint32_t G, const uint32_t* __restrict__ grp_msg, const uint8_t* __restrict__ grp_state,
                                            const G1J* __restrict__ PgJ, const G2A* __restrict__ H, Fp12* __restrict__ F) {
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  g += g0;
  if (grp_state[g] != GRP_PENDING) return;
  F[g] = miller_loop_1j(PgJ[g], H[grp_msg[g]]);
}


// Cross-lane tree: lane 0 ends with the product of the lanes' f and the sum of their s (lanes
// with any == 0 hold nothing).
__device__ inline void wave_reduce_fs(Fp12& f, G2J& s, int& any) {
  unsigned lane = threadIdx.x;
  for (unsigned d = 32; d >= 1; d >>= 1) {
    Fp12 fo = shfl_down_fp12(f, d);
    G2J so = shfl_down_jac(s, d);
    int ao = __shfl_down(any, d, 64);
    if (lane < d && ao) {
      f = any ? fp12_mul(f, fo) : fo;
      s = any ? g2_add(s, so) : so;
      any = 1;
    }
  }
}

// Per block of 64 chunks of a segment: product of the pending chunks' Miller values and sum of
// their S_g.  has[blk] = 0 when the block holds no pending chunk.
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2)))
k_sm_seg_reduce(uint32_t g0, uint32_t G, const uint8_t* __restrict__ grp_state, const Fp12* __restrict__ F, const G2J* __restrict__ SgJ,
                Fp12* __restrict__ Fpart, G2J* __restrict__ Spart, uint8_t* __restrict__ has) {
  uint32_t g = g0 + blockIdx.x * 64 + threadIdx.x;
  int any = g < g0 + G && grp_state[g] == GRP_PENDING;
  Fp12 f = any ? F[g] : fp12_one();
  G2J s = any ? SgJ[g] : jac_infinity<Fp2>();
  wave_reduce_fs(f, s, any);
  if (threadIdx.x == 0) {
    has[blockIdx.x] = (uint8_t)any;
    if (any) {
      Fpart[blockIdx.x] = f;
      Spart[blockIdx.x] = s;
    }
  }
}

// Next level of the same reduction: 64 partials per block -> one.
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2)))
k_sm_part_reduce(uint32_t n, const uint8_t* __restrict__ has_in, const Fp12* __restrict__ Fin, const G2J* __restrict__ Sin,
                 Fp12* __restrict__ Fout, G2J* __restrict__ Sout, uint8_t* __restrict__ has_out) {
  uint32_t k = blockIdx.x * 64 + threadIdx.x;
  int any = k < n && has_in[k];
  Fp12 f = any ? Fin[k] : fp12_one();
  G2J s = any ? Sin[k] : jac_infinity<Fp2>();
  wave_reduce_fs(f, s, any);
  if (threadIdx.x == 0) {
    has_out[blockIdx.x] = (uint8_t)any;
    if (any) {
      Fout[blockIdx.x] = f;
      Sout[blockIdx.x] = s;
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


void launch_sm_prepare(LaunchCfg c, uint32_t base, uint32_t n, const uint32_t* idx, const uint8_t* sig96, const uint32_t* set_grp,
                       const G1A* table, const uint8_t* table_ok, uint32_t table_n, const Seed& seed, uint32_t nonce, G2A* S_out, G2J* Sh,
                       G1J* Ph, uint8_t* status) {
  hipLaunchKernelGGL(k_sm_prepare, dim3((n + 63) / 64), dim3(64), 0, c.stream, base, n, idx, sig96, set_grp, table, table_ok, table_n, seed,
                     nonce, S_out, Sh, Ph, status);
  debug_sync(c.stream, "k_sm_prepare");
}
void launch_sm_chunk_finish(LaunchCfg c, uint32_t g0, uint32_t G, uint32_t s0, const uint32_t* grp_off, const uint8_t* status, const G2J* Sh,
                            const G1J* Ph, G1J* PgJ, G2J* SgJ, uint8_t* grp_state, uint32_t* n_fallback) {
  hipLaunchKernelGGL(k_sm_chunk_finish, dim3((G + 63) / 64), dim3(64), 0, c.stream, g0, G, s0, grp_off, status, Sh, Ph, PgJ, SgJ, grp_state,
                     n_fallback);
  debug_sync(c.stream, "k_sm_chunk_finish");
}
void launch_sm_miller(LaunchCfg c, uint32_t g0, uint32_t G, const uint32_t* grp_msg, const uint8_t* grp_state, const G1J* PgJ, const G2A* H,
                      Fp12* F) {
  hipLaunchKernelGGL(k_sm_miller, dim3((G + 63) / 64), dim3(64), 0, c.stream, g0, G, grp_msg, grp_state, PgJ, H, F);
  debug_sync(c.stream, "k_sm_miller");
}
// Reduces the segment's pending chunks to <= 4 partials (levels of 64); returns the offset of
// the final level inside Fpart / Spart / has and its length in *n_out.
uint32_t launch_sm_seg_reduce(LaunchCfg c, uint32_t g0, uint32_t G, const uint8_t* grp_state, const Fp12* F, const G2J* SgJ, Fp12* Fpart,
                              G2J* Spart, uint8_t* has, uint32_t* n_out) {
  uint32_t n = (G + 63) / 64;
  hipLaunchKernelGGL(k_sm_seg_reduce, dim3(n), dim3(64), 0, c.stream, g0, G, grp_state, F, SgJ, Fpart, Spart, has);
  debug_sync(c.stream, "k_sm_seg_reduce");
  uint32_t off = 0;
  while (n > 4) {
    uint32_t m = (n + 63) / 64;
    hipLaunchKernelGGL(k_sm_part_reduce, dim3(m), dim3(64), 0, c.stream, n, has + off, Fpart + off, Spart + off, Fpart + off + n,
                       Spart + off + n, has + off + n);
    debug_sync(c.stream, "k_sm_part_reduce");
    off += n;
    n = m;
  }
  *n_out = n;
  return off;
}
void launch_sm_fallback(LaunchCfg c, uint32_t n, const uint32_t* set_grp, const uint32_t* grp_msg, const uint8_t* grp_state,
                        const uint8_t* status, const uint32_t* idx, const G1A* table, const G2A* S, const G2A* H, uint8_t* valid,
                        int do_fallback) {
  hipLaunchKernelGGL(k_sm_fallback, dim3(c.blocks), dim3(c.threads), 0, c.stream, n, set_grp, grp_msg, grp_state, status, idx, table, S,
                     H, valid, do_fallback);
  debug_sync(c.stream, "k_sm_fallback");
}
}  // namespace gbv
