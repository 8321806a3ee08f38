// Bucket (Pippenger) multi-scalar multiplication for the G2 half of a large same-message segment.
//
// aggregateWithRandomness (multithread/jobItem.ts:73) needs, per chunk, sum r_i pk_i (paired with
// that chunk's H(m)) and sum r_i sig_i.  The segment check only pairs (-g1, S) with
// S = sum over ALL the segment's pending chunks of r_i sig_i, so the G2 terms need not be formed per
// set: one MSM over the segment's affine signatures replaces the per-set 32-step G2 ladders
// (~1.5k Fp products per set) with ~4 mixed additions per set plus a fixed bucket reduction.
//
// Scalars: r_i = a_i - b_i x^2 with a_i, b_i odd, |a_i|, |b_i| < 2^32 (curve.h randomize_pair), so
// r_i sig_i = a_i sig_i + b_i E(sig_i), E = -psi^2.  Each of the 2 points of a set takes its scalar
// magnitude in MSM_WINDOWS = 2 unsigned 16-bit digits and its sign on the point (negate y).
// Entries (local set index, point, sign) are counting-sorted by key = window * 2^16 + digit, each
// key's bucket is summed by one thread (mixed additions, complete formulas), then
// sum_w 2^(16 w) sum_d d B_{w,d} is formed by slices of 16 buckets (running sums + one 16-bit
// scalar multiple of the slice total) and a tree sum.  The segment's failure path does not use
// the MSM: k_sm_redo_g2 recomputes the per-set terms with the same r_i (k_sm.hip).
#include <cstdlib>

#include "launch.h"
#include "kernel_common.h"

namespace gbv {

GBV_NI G2J msm_add(G2J a, G2J b) { return jac_add(a, b); }
GBV_NI G2J msm_dbl(G2J a) { return jac_dbl(a); }

__device__ inline bool msm_member(uint32_t i, const uint32_t* set_grp, const uint8_t* status, const uint8_t* grp_state) {
  return status[i] == SET_OK && grp_state[set_grp[i]] == GRP_PENDING;
}

// One thread per set: count (SCATTER = false) or place (SCATTER = true) its <= 4 bucket entries.
template <bool SCATTER>
__global__ void __launch_bounds__(64) k_msm_entries(uint32_t s0, uint32_t n, const uint32_t* __restrict__ set_grp,
                                                     const uint8_t* __restrict__ status, const uint8_t* __restrict__ grp_state, Seed seed,
                                                     uint32_t nonce, uint32_t* __restrict__ cnt_or_cur, uint32_t* __restrict__ ent) {
  uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  uint32_t i = s0 + t;
  if (!msm_member(i, set_grp, status, grp_state)) return;
  uint64_t r = prf_scalar(seed, i, nonce);
#pragma unroll
  for (uint32_t h = 0; h < 2; ++h) {
    bool neg;
    uint32_t mag = scalar_half_mag(h ? (uint32_t)(r >> 32) : (uint32_t)r, &neg);
#pragma unroll
    for (uint32_t w = 0; w < MSM_WINDOWS; ++w) {
      uint32_t d = (mag >> (MSM_C * w)) & ((1u << MSM_C) - 1);
      if (!d) continue;
      uint32_t key = (w << MSM_C) | d;
      uint32_t pos = atomicAdd(&cnt_or_cur[key], 1u);
      if (SCATTER) ent[pos] = (t << 2) | (h << 1) | (neg ? 1u : 0u);
    }
  }
}

__global__ void __launch_bounds__(256) k_msm_zero(uint32_t* __restrict__ cnt) { cnt[blockIdx.x * 256 + threadIdx.x] = 0; }

// Exclusive scan of the MSM_KEYS bucket counts in 64-thread workgroups (a single large workgroup
// can wait a long time for a free CU beside k_sm_prepare's waves): wave sums, a one-wave scan of
// the wave sums, then per-wave exclusive scans plus their offsets.
__device__ inline uint32_t wave_incl_scan(uint32_t v) {
  unsigned lane = threadIdx.x;
  for (unsigned d = 1; d < 64; d <<= 1) {
    uint32_t o = __shfl_up(v, d, 64);
    if (lane >= d) v += o;
  }
  return v;
}
__global__ void __launch_bounds__(64) k_msm_scan_blocks(const uint32_t* __restrict__ cnt, uint32_t* __restrict__ bsum) {
  uint32_t v = wave_incl_scan(cnt[blockIdx.x * 64 + threadIdx.x]);
  if (threadIdx.x == 63) bsum[blockIdx.x] = v;
}
__global__ void __launch_bounds__(64) k_msm_scan_top(uint32_t nb, uint32_t* __restrict__ bsum) {
  // exclusive scan of nb block sums (nb a multiple of 64), one wave, 64-element tiles
  uint32_t carry = 0;
  for (uint32_t t = 0; t < nb; t += 64) {
    uint32_t x = bsum[t + threadIdx.x];
    uint32_t inc = wave_incl_scan(x);
    bsum[t + threadIdx.x] = carry + inc - x;
    carry += __shfl(inc, 63, 64);
  }
}
__global__ void __launch_bounds__(64) k_msm_scan_apply(const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ bsum,
                                                       uint32_t* __restrict__ off, uint32_t* __restrict__ cur) {
  uint32_t k = blockIdx.x * 64 + threadIdx.x;
  uint32_t c = cnt[k];
  uint32_t e = bsum[blockIdx.x] + wave_incl_scan(c) - c;
  off[k] = e;
  cur[k] = e;
}

__device__ inline G2A msm_entry_point(uint32_t v, uint32_t s0, const G2A* __restrict__ S) {
  G2A q = S[s0 + (v >> 2)];
  if (v & 2u) q = g2_neg_psi2(q);
  if (v & 1u) q.y = fp2_neg(q.y);
  return q;
}

// One thread per run of MSM_RUN consecutive sorted entries, so every lane does the same number of
// additions whatever the bucket sizes (window-0 digits are all odd: half those buckets are empty,
// the others hold twice the mean).  A bucket lying inside the run is written to B directly; a
// bucket continuing from the previous run goes to head[t], one continuing into the next run to
// tail[t], and k_msm_fixup adds the pieces.
__global__ void GBV_KERNEL_ATTR k_msm_runs(uint32_t s0, const uint32_t* __restrict__ off, const uint32_t* __restrict__ end,
                                           const uint32_t* __restrict__ ent, const G2A* __restrict__ S, G2J* __restrict__ B,
                                           G2J* __restrict__ head, G2J* __restrict__ tail) {
  const uint32_t E = end[MSM_KEYS - 1];  // total entries (the last key's end)
  uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t p = t * MSM_RUN;
  if (p >= E) return;
  uint32_t pe = min(p + MSM_RUN, E), r0 = p;
  // bucket holding entry p: the largest key with off[key] <= p (then end[key] = off[key+1] > p)
  uint32_t lo = 0, hi = MSM_KEYS - 1;
  while (lo < hi) {
    uint32_t mid = (lo + hi + 1) >> 1;
    if (off[mid] <= p) lo = mid; else hi = mid - 1;
  }
  uint32_t k = lo, kend = end[k];
  G2J acc = jac_infinity<Fp2>();
  for (; p < pe; ++p) {
    acc = jac_add_aff(acc, msm_entry_point(ent[p], s0, S));
    if (p + 1 == kend || p + 1 == pe) {
      bool starts_here = off[k] >= r0, ends_here = kend <= pe;
      if (starts_here && ends_here) B[k] = acc;
      else if (!starts_here) head[t] = acc;
      else tail[t] = acc;
      acc = jac_infinity<Fp2>();
      if (p + 1 < pe) {
        do { ++k; } while (end[k] == off[k]);
        kend = end[k];
      }
    }
  }
}

// One thread per bucket: empty buckets become infinity, buckets split over runs t0..t1 are
// tail[t0] + head[t0+1] + ... + head[t1].
__global__ void GBV_KERNEL_ATTR k_msm_fixup(const uint32_t* __restrict__ off, const uint32_t* __restrict__ end,
                                            const G2J* __restrict__ head, const G2J* __restrict__ tail, G2J* __restrict__ B) {
  uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= MSM_KEYS) return;
  uint32_t b = off[k], e = end[k];
  if (b == e) {
    B[k] = jac_infinity<Fp2>();
    return;
  }
  uint32_t t0 = b / MSM_RUN, t1 = (e - 1) / MSM_RUN;
  if (t0 == t1) return;
  G2J acc = tail[t0];
  for (uint32_t t = t0 + 1; t <= t1; ++t) acc = msm_add(acc, head[t]);
  B[k] = acc;
}

// One thread per slice of MSM_SLICE buckets of one window:
//   part = 2^(16 w) (sum_{q>=1} q B_{d0+q} + d0 sum_q B_{d0+q}),  d0 = slice * MSM_SLICE.
__global__ void GBV_KERNEL_ATTR k_msm_slices(const G2J* __restrict__ B, G2J* __restrict__ part) {
  GBV_TAIL_WAVE_PRIO();
  constexpr uint32_t PER_WIN = (1u << MSM_C) / MSM_SLICE;
  uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= MSM_PARTS) return;
  uint32_t w = j / PER_WIN, d0 = (j % PER_WIN) * MSM_SLICE;
  const G2J* b = B + (w << MSM_C) + d0;
  G2J T = jac_infinity<Fp2>(), A = jac_infinity<Fp2>();
  for (int q = MSM_SLICE - 1; q >= 1; --q) {
    T = msm_add(T, b[q]);
    A = msm_add(A, T);
  }
  T = msm_add(T, b[0]);
  // d0 T by double-and-add over the 16 bits of d0 (lanes differ in d0: the add is masked, not skipped)
  G2J M = jac_infinity<Fp2>();
  for (int k = MSM_C - 1; k >= 0; --k) {
    M = msm_dbl(M);
    if ((d0 >> k) & 1u) M = msm_add(M, T);
  }
  G2J R = msm_add(A, M);
  if (w) {
    for (uint32_t k = 0; k < MSM_C * w; ++k) R = msm_dbl(R);
  }
  part[j] = R;
}

__device__ inline Fp shfl_down_fp_m(const Fp& a, unsigned d) {
  Fp r;
#pragma unroll
  for (int i = 0; i < 12; ++i) r.v[i] = __shfl_down((unsigned)a.v[i], d, 64);
  return r;
}

// Tree sum of 64 points per workgroup: out[blk] = sum in[blk*64 .. blk*64+63] (< n).
__global__ void GBV_KERNEL_ATTR k_msm_sum64(uint32_t n, const G2J* __restrict__ in, G2J* __restrict__ out) {
  GBV_TAIL_WAVE_PRIO();
  uint32_t k = blockIdx.x * 64 + threadIdx.x;
  G2J s = k < n ? in[k] : jac_infinity<Fp2>();
  for (unsigned d = 32; d >= 1; d >>= 1) {
    G2J o;
    o.x = Fp2{shfl_down_fp_m(s.x.c0, d), shfl_down_fp_m(s.x.c1, d)};
    o.y = Fp2{shfl_down_fp_m(s.y.c0, d), shfl_down_fp_m(s.y.c1, d)};
    o.z = Fp2{shfl_down_fp_m(s.z.c0, d), shfl_down_fp_m(s.z.c1, d)};
    if (threadIdx.x < d) s = msm_add(s, o);
  }
  if (threadIdx.x == 0) out[blockIdx.x] = s;
}

void launch_msm_g2_buckets(hipStream_t s, uint32_t s0, uint32_t n, const uint32_t* set_grp, const uint8_t* status, const uint8_t* grp_state,
                           const G2A* S, const Seed& seed, uint32_t nonce, uint32_t* cnt, uint32_t* off, uint32_t* cur, uint32_t* ent,
                           G2J* buckets, G2J* head, G2J* tail) {
  static_assert(MSM_KEYS % 4096 == 0 && MSM_PARTS % 64 == 0, "MSM shape");
  GBV_LAUNCH("k_msm_zero", k_msm_zero, dim3(MSM_KEYS / 256), dim3(256), s, 0, cnt);
  unsigned eb = (n + 63) / 64;
  GBV_LAUNCH("k_msm_entries<false>", k_msm_entries<false>, dim3(eb), dim3(64), s, n, s0, n, set_grp, status, grp_state, seed, nonce, cnt, ent);
  // block sums live in the (not yet used) bucket area
  uint32_t* bsum = reinterpret_cast<uint32_t*>(buckets);
  GBV_LAUNCH("k_msm_scan_blocks", k_msm_scan_blocks, dim3(MSM_KEYS / 64), dim3(64), s, 0, cnt, bsum);
  GBV_LAUNCH("k_msm_scan_top", k_msm_scan_top, dim3(1), dim3(64), s, 0, MSM_KEYS / 64, bsum);
  GBV_LAUNCH("k_msm_scan_apply", k_msm_scan_apply, dim3(MSM_KEYS / 64), dim3(64), s, 0, cnt, bsum, off, cur);
  GBV_LAUNCH("k_msm_entries<true>", k_msm_entries<true>, dim3(eb), dim3(64), s, n, s0, n, set_grp, status, grp_state, seed, nonce, cur, ent);
  const uint32_t runs = (uint32_t)((4ull * n + MSM_RUN - 1) / MSM_RUN);  // upper bound; runs past the end exit
  GBV_LAUNCH("k_msm_runs", k_msm_runs, dim3((runs + 63) / 64), dim3(64), s, n, s0, off, cur, ent, S, buckets, head, tail);
  GBV_LAUNCH("k_msm_fixup", k_msm_fixup, dim3(MSM_KEYS / 64), dim3(64), s, 0, off, cur, head, tail, buckets);
}

void launch_msm_g2_reduce(hipStream_t s, const G2J* buckets, G2J* part, G2J* total) {
  GBV_LAUNCH("k_msm_slices", k_msm_slices, dim3(MSM_PARTS / 64), dim3(64), s, 0, buckets, part);
  // MSM_PARTS -> MSM_PARTS/64 -> ... -> 1
  uint32_t m = MSM_PARTS;
  G2J* src = part;
  G2J* dst = part + MSM_PARTS;
  while (m > 1) {
    uint32_t nb = (m + 63) / 64;
    G2J* o = nb == 1 ? total : dst;
    GBV_LAUNCH("k_msm_sum64", k_msm_sum64, dim3(nb), dim3(64), s, m, m, src, o);
    src = o;
    dst = o + nb;
    m = nb;
  }
}

}  // namespace gbv
