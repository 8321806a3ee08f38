// Distinct-message path kernels (verifySignatureSets, maybeBatch.ts:15-45), batched over many calls.
#include <cstring>

#include "launch.h"
#include "kernel_common.h"
#include "quad_g2.h"

namespace gbv {

GBV_NI G1J vs_g1_add(G1J a, G1J b) { return jac_add(a, b); }
// The gather loops' mixed addition is inline: out of line, the G1J result returned through the caller's
// frame was a 192-byte scratch write (and read) per member -- k_vs_agg_big's 3.9 MB of writes per 8 192
// members in PMC.
GBV_HD G1J vs_g1_add_aff(const G1J& a, const G1A& b) { return jac_add_aff(a, b); }

__device__ inline Fp vs_shfl_down(const Fp& a, unsigned d) {
  Fp r;
#pragma unroll
  for (int i = 0; i < 12; ++i) r.v[i] = __shfl_down((unsigned)a.v[i], d, 64);
  return r;
}

// aggregatePublicKeys over one set's validator indices (bls/utils.ts:5-20, jobItem.ts:55-62):
// AGG_LANES lanes per aggregate set, 64 / AGG_LANES sets per wave.  Lane j of a set gathers table
// entries j, j + AGG_LANES, ... (each lane reads its own 128-byte affine record) and adds them
// serially, then a log2(AGG_LANES)-level cross-lane tree (ds_bpermute shuffles inside the lane
// group) sums the group.  For a 128-member committee: 16 mixed additions + 3 full additions of
// latency per set, and every lane of the wave busy for all but the short tree.  The sum stays
// Jacobian: the randomisation (randomize_pair_jac) normalises its tables with the one inversion it
// does anyway, so no per-set inversion is spent here.
constexpr unsigned AGG_LANES = 8;
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2)))
k_vs_agg(uint32_t n_agg, const uint32_t* __restrict__ agg_list, const uint32_t* __restrict__ set_off, const uint32_t* __restrict__ arena,
         const G1A* __restrict__ table, const uint8_t* __restrict__ table_ok, G1J* __restrict__ pk_out, uint8_t* __restrict__ pk_st) {
  const unsigned lane = threadIdx.x, sub = lane % AGG_LANES;
  const uint32_t a = blockIdx.x * (64 / AGG_LANES) + lane / AGG_LANES;
  const bool act = a < n_agg;
  const uint32_t s = act ? agg_list[a] : 0;
  const uint32_t b = act ? set_off[s] : 0, e = act ? set_off[s + 1] : 0;
  G1J acc = jac_infinity<Fp>();
  int bad = 0;
  uint32_t j = b + sub;
  if (j < e) {  // the first member starts the sum: no addition to infinity
    uint32_t k = arena[j];
    bad |= table_ok[k] ? 0 : 1;
    acc = jac_from_aff(table[k]);
    j += AGG_LANES;
  }
  for (; j < e; j += AGG_LANES) {
    uint32_t k = arena[j];
    bad |= table_ok[k] ? 0 : 1;
    acc = vs_g1_add_aff(acc, table[k]);
  }
  for (unsigned d = AGG_LANES / 2; d >= 1; d >>= 1) {
    G1J o{vs_shfl_down(acc.x, d), vs_shfl_down(acc.y, d), vs_shfl_down(acc.z, d)};
    int ob = __shfl_down(bad, d, 64);
    if (sub < d) {
      acc = vs_g1_add(acc, o);
      bad |= ob;
    }
  }
  if (act && sub == 0) {
    pk_out[s] = acc;
    // an infinity aggregate fails verification in blst; an invalid table slot never verifies
    pk_st[s] = (bad || jac_is_inf(acc)) ? SET_BAD_PK : SET_OK;
  }
}

// aggregatePublicKeys of LARGE sets (electra attestations: committee_bits name up to 64 committees,
// so one aggregate holds thousands to tens of thousands of validators; epochCache.ts:953-973) by
// slices of tuning().agg_slice members (vs_fill): one 256-thread workgroup per slice.  Thread t reads index words
// begin + t, begin + t + 256, ... (consecutive threads, consecutive words: coalesced) and gathers the
// 128-byte table records; each thread sums its few records with mixed additions, a 6-level shuffle
// tree sums each wave and the 4 wave sums meet in LDS.  part[w] is the slice's Jacobian sum,
// part_bad[w] flags an unusable table slot.  k_vs_agg_big_fin then sums each set's slices.
constexpr unsigned AGG_BIG_TPB = 256;
__global__ void __launch_bounds__(AGG_BIG_TPB) k_vs_agg_big(const uint4* __restrict__ slices, const uint32_t* __restrict__ arena,
                                                            const G1A* __restrict__ table, const uint8_t* __restrict__ table_ok,
                                                            G1J* __restrict__ part, uint8_t* __restrict__ part_bad) {
  __shared__ G1J wsum[AGG_BIG_TPB / 64];
  __shared__ int wbad[AGG_BIG_TPB / 64];
  const uint4 sl = slices[blockIdx.x];  // (begin, end) of the slice in the arena
  const unsigned t = threadIdx.x, lane = t & 63, w = t >> 6;
  G1J acc = jac_infinity<Fp>();
  int bad = 0;
  uint32_t j = sl.x + t;
  if (j < sl.y) {
    const uint32_t k = arena[j];
    bad |= table_ok[k] ? 0 : 1;
    acc = jac_from_aff(table[k]);
    j += AGG_BIG_TPB;
  }
  for (; j < sl.y; j += AGG_BIG_TPB) {
    const uint32_t k = arena[j];
    bad |= table_ok[k] ? 0 : 1;
    acc = vs_g1_add_aff(acc, table[k]);
  }
  for (unsigned d = 32; d >= 1; d >>= 1) {
    G1J o{vs_shfl_down(acc.x, d), vs_shfl_down(acc.y, d), vs_shfl_down(acc.z, d)};
    bad |= __shfl_down(bad, d, 64);
    if (lane < d) acc = vs_g1_add(acc, o);
  }
  if (lane == 0) {
    wsum[w] = acc;
    wbad[w] = bad;
  }
  __syncthreads();
  if (t == 0) {
    for (unsigned q = 1; q < AGG_BIG_TPB / 64; ++q) {
      acc = vs_g1_add(acc, wsum[q]);
      bad |= wbad[q];
    }
    part[blockIdx.x] = acc;
    part_bad[blockIdx.x] = (uint8_t)bad;
  }
}

// One wave per large set: sum of its slice partials (lane-strided, then the shuffle tree).
// big = (set, first slice, slice count).
__global__ void __launch_bounds__(64) k_vs_agg_big_fin(uint32_t n_big, const uint4* __restrict__ big, const G1J* __restrict__ part,
                                                       const uint8_t* __restrict__ part_bad, G1J* __restrict__ pk_out,
                                                       uint8_t* __restrict__ pk_st) {
  const uint4 b = big[blockIdx.x];
  const unsigned lane = threadIdx.x;
  G1J acc = jac_infinity<Fp>();
  int bad = 0;
  for (uint32_t q = lane; q < b.z; q += 64) {
    acc = vs_g1_add(acc, part[b.y + q]);
    bad |= part_bad[b.y + q];
  }
  for (unsigned d = 32; d >= 1; d >>= 1) {
    G1J o{vs_shfl_down(acc.x, d), vs_shfl_down(acc.y, d), vs_shfl_down(acc.z, d)};
    bad |= __shfl_down(bad, d, 64);
    if (lane < d) acc = vs_g1_add(acc, o);
  }
  if (lane == 0) {
    pk_out[b.x] = acc;
    pk_st[b.x] = (bad || jac_is_inf(acc)) ? SET_BAD_PK : SET_OK;
  }
}

// Two block roles in one launch (wave-uniform, no divergence): blocks [0, nb) hash the signing
// roots; blocks [nb, 2 nb) decode and group-check the signatures (Signature.fromBytes(sig, true),
// maybeBatch.ts:23), fetch the pubkey (table slot, the k_vs_agg result, or a raw key validated like
// PublicKey.fromBytes(pk, true), blsToExecutionChange.ts:31) and form r_i pk_i and r_i sig_i.
// The two roles are independent, so hashing (the longest per-set chain) overlaps the rest.
//
// split (small passes, the hash then runs on its own stream): the signature role is itself two
// block roles side by side -- blocks [nb, nb + nsig) decode and group-check (status), blocks
// [nb + nsig, nb + 2 nsig) decode and randomise (rP, rS, written whatever the checks say: every
// consumer reads them only for sets whose status is SET_OK).
__global__ void GBV_KERNEL_ATTR k_vs_hash_sig(uint32_t n, uint32_t nb, uint32_t pair, uint32_t split, const uint8_t* __restrict__ msgs32,
                                              const uint32_t* __restrict__ set_off, const uint32_t* __restrict__ arena,
                                              const uint8_t* __restrict__ raw_flag, const uint8_t* __restrict__ raw_pk48,
                                              const uint8_t* __restrict__ sig, uint32_t sig_stride, const uint32_t* __restrict__ sig_len,
                                              const G1A* __restrict__ table, const uint8_t* __restrict__ table_ok,
                                              const G1J* __restrict__ pk_agg, const uint8_t* __restrict__ pk_st, Seed seed, uint32_t nonce,
                                              G2A* __restrict__ H, G1J* __restrict__ rP_out, G2J* __restrict__ rS_out,
                                              uint8_t* __restrict__ status) {
  if (blockIdx.x < nb) {
    if (pair) {  // few sets: lane pairs (hash_to_g2_lane_pair), nb = ceil(2n / 64)
      uint32_t i = (blockIdx.x * 64 + threadIdx.x) >> 1;
      bool act = i < n;
      uint32_t w[8] = {};
      if (act) load_msg_words(w, msgs32 + 32ull * i);
      G2A h;
      if (hash_to_g2_lane_pair(w, act, &h)) H[i] = h;
      return;
    }
    uint32_t i = blockIdx.x * 64 + threadIdx.x;
    if (i >= n) return;
    uint32_t w[8];
    load_msg_words(w, msgs32 + 32ull * i);
    H[i] = hash_to_g2(w);
    return;
  }
  const uint32_t nsig = (n + 63) / 64;
  uint32_t blk = blockIdx.x - nb;
  const bool rand_only = split && blk >= nsig, check_only = split && blk < nsig;
  if (rand_only) blk -= nsig;
  uint32_t i = blk * 64 + threadIdx.x;
  if (i >= n) return;
  uint8_t st = SET_OK;
  G1J pk;
  if (raw_flag[i]) {
    G1A a;
    uint8_t ds = g1_decompress(a, raw_pk48 + 48ull * i);
    if (ds != PT_OK || (!rand_only && !g1_in_subgroup(a))) st = SET_BAD_PK;
    pk = jac_from_aff(a);
  } else {
    uint32_t b = set_off[i], e = set_off[i + 1];
    if (e - b == 1) {
      uint32_t k = arena[b];
      pk = jac_from_aff(table[k]);
      if (!table_ok[k]) st = SET_BAD_PK;
    } else if (e == b) {
      st = SET_BAD_PK;  // empty aggregate: its call is rejected on the host, never verified
    } else {
      pk = pk_agg[i];
      if (pk_st[i] != SET_OK) st = SET_BAD_PK;
    }
  }
  G2A s;
  uint8_t ds = g2_decode(s, sig + (size_t)sig_stride * i, sig_len[i]);
  if (ds != PT_OK || (!rand_only && !g2_in_subgroup(s))) st = SET_BAD_SIG;
  if (!rand_only) status[i] = st;
  if (check_only || st != SET_OK) return;
  uint64_t r = prf_scalar(seed, i, nonce);
  G1J rp;
  G2J rs;
  if (!randomize_pair_jac(pk, s, r, &rp, &rs)) {  // unreachable for subgroup points; plain 64-bit r then
    G1A pa;
    jac_to_aff(pa, pk);
    rs = g2_mul_u64(s, r);
    rp = g1_mul_u64(pa, r);
  }
  rP_out[i] = rp;
  rS_out[i] = rs;
}

// Small passes, latency form ("pre" mode, gbv_vs.hip): the signature work that needs no pubkey runs
// on its own stream beside the pubkey aggregation -- k_vs_sig_decode decodes each signature, then the
// quad roles below check it and form r_i sig_i (the same r_i = a - b x^2 split as randomize_pair_jac)
// -- and k_vs_pk_rand_quad, after the aggregation and these, takes the pubkey, merges its verdict and
// forms r_i pk_i.  The aggregation (an Electra block's committee sums: ~3.7 ms) then no longer sits in
// front of the signature chain.
// The same two roles on lane quads (quad_g2.h), one quad per set and role: blocks [0, nq) check,
// blocks [nq, 2 nq) randomise, 16 sets per block.  The signatures were decoded by k_vs_sig_decode (one
// thread each: the square root is two Fp exponentiations in a row, nothing for a quad to share); the
// subgroup check's 63 doublings and r_i sig_i's 31-step ladder run their products four at a time.
__global__ void GBV_QUAD_ATTR k_vs_sig_pre_quad(uint32_t n, const G2A* __restrict__ Sd, const uint8_t* __restrict__ dec_st, Seed seed,
                                                  uint32_t nonce, G2J* __restrict__ rS_out, uint8_t* __restrict__ status,
                                                  uint8_t* __restrict__ sig_st) {
  const uint32_t nq = (n + 15) / 16;
  uint32_t blk = blockIdx.x;
  const bool rand = blk >= nq;
  if (rand) blk -= nq;
  const uint32_t q = threadIdx.x & 3u;
  const uint32_t i = blk * 16 + (threadIdx.x >> 2);
  if (i >= n) return;  // whole quads
  const uint8_t ds = dec_st[i];
  G2A s{fp2_zero(), fp2_zero()};
  if (ds == PT_OK) s = Sd[i];
  if (!rand) {
    const uint8_t st = (ds != PT_OK || !quad::g2_in_subgroup(s, q)) ? SET_BAD_SIG : SET_OK;
    if (q == 0) {
      status[i] = st;
      sig_st[i] = st;
    }
    return;
  }
  if (ds != PT_OK) return;
  const uint64_t r = prf_scalar(seed, i, nonce);
  G2J rs;
  if (!quad::g2_randomize(s, r, &rs, q)) rs = g2_mul_u64(s, r);  // unreachable for subgroup points
  quad::store_split<6>((Fp*)&rS_out[i], (const Fp*)&rs, q);
}

// Same-message latency prepare (segments <= prepare_split_max sets, after k_sig_decode) on lane quads:
// blocks [0, nq) run the G2 subgroup checks (sub_ok[i]), blocks [nq, 2 nq) the randomisation
// (Sh[i] = r_i sig_i by quad_g2.h's ladder, Ph[i] = r_i pk_i from the comb table or the G1 ladder),
// one quad per set and role, 16 sets per block: the point chains four lanes wide (round 3 ran them on
// the cooperative interpreter, one wave per set: prepare 2.8-3.0 -> 2.35 ms).  k_sm_prep_scan merges the
// verdicts.
__global__ void GBV_QUAD_ATTR k_sm_prep_roles_quad(uint32_t base, uint32_t n, const uint32_t* __restrict__ idx, const G1A* __restrict__ table,
                                                   const uint8_t* __restrict__ table_ok, uint32_t table_n, const uint4* __restrict__ comb,
                                                   const uint8_t* __restrict__ comb_ok, Seed seed, uint32_t nonce, const G2A* __restrict__ S,
                                                   const uint8_t* __restrict__ status, uint8_t* __restrict__ sub_ok, G2J* __restrict__ Sh,
                                                   G1J* __restrict__ Ph) {
  const uint32_t nq = (n + 15) / 16;
  uint32_t blk = blockIdx.x;
  const bool rand = blk >= nq;
  if (rand) blk -= nq;
  const uint32_t q = threadIdx.x & 3u;
  const uint32_t t = blk * 16 + (threadIdx.x >> 2);
  if (t >= n) return;  // whole quads
  const uint32_t i = base + t;
  if (!rand) {
    const bool ok = status[i] == PT_OK && quad::g2_in_subgroup(S[i], q);
    if (q == 0) sub_ok[i] = ok ? 1 : 0;
    return;
  }
  const uint32_t k = idx[i];
  if (!(status[i] == PT_OK && k < table_n && table_ok[k])) {  // discarded by k_sm_prep_scan
    if (q == 0) {
      Sh[i] = jac_infinity<Fp2>();
      Ph[i] = jac_infinity<Fp>();
    }
    return;
  }
  const uint64_t r = prf_scalar(seed, i, nonce);
  G2J rs;
  if (!quad::g2_randomize(S[i], r, &rs, q)) rs = g2_mul_u64(S[i], r);  // unreachable for subgroup points (the check role decides)
  quad::store_split<6>((Fp*)&Sh[i], (const Fp*)&rs, q);
  if (q == 0) {
    G1J rp;
    if (comb && comb_ok[k])
      rp = comb_mul(comb + (size_t)k * (COMB_ENTRIES * COMB_U4), (uint32_t)r, (uint32_t)(r >> 32));
    else if (!randomize_g1(table[k], r, &rp))  // a table key is in the subgroup: the 2-D ladder cannot fail
      rp = jac_infinity<Fp>();
    Ph[i] = rp;
  }
}

void launch_sm_prep_roles_quad(hipStream_t s, uint32_t base, uint32_t n, const uint32_t* idx, const G1A* table, const uint8_t* table_ok,
                               uint32_t table_n, const uint4* comb, const uint8_t* comb_ok, const Seed& seed, uint32_t nonce, const G2A* S,
                               const uint8_t* status, uint8_t* sub_ok, G2J* Sh, G1J* Ph) {
  GBV_LAUNCH("k_sm_prep_roles_quad", k_sm_prep_roles_quad, dim3(2 * ((n + 15) / 16)), dim3(64), s, n, base, n, idx, table, table_ok, table_n, comb, comb_ok, seed, nonce, S, status, sub_ok, Sh, Ph);
}

// The pubkey half on lane quads (stream A, after the aggregation and the signature roles): a rejected
// signature's verdict stands (it wins over a bad pubkey, as in k_vs_hash_sig); otherwise the pubkey's
// verdict is merged and r_i pk_i formed by quad_g2.h's G1 ladder (3 + 5 product rounds a step against
// 18 products), the same pubkey fetch on every lane of the quad.  Raw pubkeys
// (PublicKey.fromBytes(pk, true)) are decoded and group-checked here.
__global__ void GBV_QUAD_ATTR k_vs_pk_rand_quad(uint32_t n, const uint32_t* __restrict__ set_off, const uint32_t* __restrict__ arena,
                                                  const uint8_t* __restrict__ raw_flag, const uint8_t* __restrict__ raw_pk48,
                                                  const G1A* __restrict__ table, const uint8_t* __restrict__ table_ok,
                                                  const G1J* __restrict__ pk_agg, const uint8_t* __restrict__ pk_st, Seed seed, uint32_t nonce,
                                                  G1J* __restrict__ rP_out, uint8_t* __restrict__ status) {
  const uint32_t q = threadIdx.x & 3u;
  const uint32_t i = blockIdx.x * 16 + (threadIdx.x >> 2);
  if (i >= n || status[i] != SET_OK) return;  // whole quads
  bool ok = true, jac = false;
  G1A pa{fp_zero(), fp_zero()};
  G1J pj;
  if (raw_flag[i]) {
    ok = g1_decompress(pa, raw_pk48 + 48ull * i) == PT_OK && g1_in_subgroup(pa);
  } else {
    const uint32_t b = set_off[i], e = set_off[i + 1];
    if (e - b == 1) {
      const uint32_t k = arena[b];
      pa = table[k];
      ok = table_ok[k] != 0;
    } else if (e == b) {
      ok = false;
    } else {
      pj = pk_agg[i];
      jac = true;
      ok = pk_st[i] == SET_OK;
    }
  }
  if (ok && jac) ok = jac_to_aff(pa, pj);
  if (!ok) {
    if (q == 0) status[i] = SET_BAD_PK;
    return;
  }
  const uint64_t r = prf_scalar(seed, i, nonce);
  G1J rp;
  if (!quad::g1_randomize(pa, r, &rp, q)) rp = g1_mul_u64(pa, r);
  quad::store_split<3>((Fp*)&rP_out[i], (const Fp*)&rp, q);
}

// Signature.fromBytes(sig, true) (maybeBatch.ts:23; the "BLS deserializing signatures" perf id,
// test/perf/bls/bls.test.ts:89-100): decode + subgroup check, and the recompressed encoding of
// every accepted point (byte-identical to the input for canonical compressed signatures).
__global__ void GBV_KERNEL_ATTR k_sig_validate(uint32_t n, const uint8_t* __restrict__ sig, uint32_t sig_len, uint8_t* __restrict__ status,
                                               uint8_t* __restrict__ out96) {
  uint32_t i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  G2A s;
  uint8_t st = g2_decode(s, sig + (size_t)sig_len * i, sig_len);
  if (st == PT_OK && !g2_in_subgroup(s)) st = PT_NOT_IN_GROUP;
  status[i] = st;
  if (st == PT_OK)
    g2_compress(out96 + 96ull * i, s, false);
  else
    g2_compress(out96 + 96ull * i, s, true);  // infinity encoding as the placeholder of a rejected input
}

// aggregateSignatures(Signature.fromBytes(sig_i, validate)) (singleThread.ts:54-57): stage 1, one
// thread per signature decodes (+ subgroup check), a 6-level shuffle tree sums the wave, lane 0
// writes the block's Jacobian partial; any rejected input raises *bad.
GBV_NI G2J vs_g2_add(G2J a, G2J b) { return jac_add(a, b); }
__device__ inline Fp2 vs_shfl_down2(const Fp2& a, unsigned d) { return Fp2{vs_shfl_down(a.c0, d), vs_shfl_down(a.c1, d)}; }
__device__ inline G2J wave_sum_g2(G2J acc) {
  for (unsigned d = 32; d > 0; d >>= 1) {
    G2J o{vs_shfl_down2(acc.x, d), vs_shfl_down2(acc.y, d), vs_shfl_down2(acc.z, d)};
    acc = vs_g2_add(acc, o);
  }
  return acc;
}

__global__ void GBV_KERNEL_ATTR k_sig_aggregate(uint32_t n, const uint8_t* __restrict__ sig, uint32_t sig_len, int validate,
                                                G2J* __restrict__ part, uint32_t* __restrict__ bad) {
  uint32_t i = blockIdx.x * 64 + threadIdx.x;
  G2J acc = jac_infinity<Fp2>();
  if (i < n) {
    G2A s;
    uint8_t st = g2_decode(s, sig + (size_t)sig_len * i, sig_len);
    if (validate && st == PT_OK && !g2_in_subgroup(s)) st = PT_NOT_IN_GROUP;
    bool reject = st != PT_OK && (validate || st != PT_INFINITY);
    if (reject) atomicOr(bad, 1u);
    else if (st == PT_OK) acc = jac_from_aff(s);
  }
  acc = wave_sum_g2(acc);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

// stage 2: one wave sums the nb block partials and writes the compressed aggregate.
__global__ void __launch_bounds__(64) k_sig_aggregate_final(uint32_t nb, const G2J* __restrict__ part, uint8_t* __restrict__ out96) {
  G2J acc = jac_infinity<Fp2>();
  for (uint32_t b = threadIdx.x; b < nb; b += 64) acc = vs_g2_add(acc, part[b]);
  acc = wave_sum_g2(acc);
  if (threadIdx.x == 0) {
    G2A a;
    bool fin = jac_to_aff(a, acc);
    g2_compress(out96, a, !fin);
  }
}

void launch_sig_aggregate(hipStream_t s, uint32_t n, const uint8_t* sig, uint32_t sig_len, int validate, G2J* part, uint32_t* bad,
                          uint8_t* out96) {
  uint32_t nb = (n + 63) / 64;
  hipLaunchKernelGGL(k_sig_aggregate, dim3(nb), dim3(64), 0, s, n, sig, sig_len, validate, part, bad);
  debug_sync(s, "k_sig_aggregate");
  hipLaunchKernelGGL(k_sig_aggregate_final, dim3(1), dim3(64), 0, s, nb, part, out96);
  debug_sync(s, "k_sig_aggregate_final");
}

void launch_vs_agg(LaunchCfg c, const uint32_t* agg_list, const uint32_t* set_off, const uint32_t* arena, const G1A* table,
                   const uint8_t* table_ok, G1J* pk_out, uint8_t* pk_st) {
  const uint32_t n_agg = c.blocks;  // c.blocks carries the aggregate-set count
  GBV_LAUNCH("k_vs_agg", k_vs_agg, dim3((n_agg + 64 / AGG_LANES - 1) / (64 / AGG_LANES)), dim3(64), c.stream, n_agg, n_agg, agg_list, set_off, arena, table, table_ok, pk_out, pk_st);
}

void launch_vs_agg_big(hipStream_t s, uint32_t n_slices, const uint4* slices, uint32_t n_big, const uint4* big, const uint32_t* arena,
                       const G1A* table, const uint8_t* table_ok, G1J* part, uint8_t* part_bad, G1J* pk_out, uint8_t* pk_st) {
  if (!n_big) return;
  GBV_LAUNCH("k_vs_agg_big", k_vs_agg_big, dim3(n_slices), dim3(AGG_BIG_TPB), s, n_slices, slices, arena, table, table_ok, part, part_bad);
  GBV_LAUNCH("k_vs_agg_big_fin", k_vs_agg_big_fin, dim3(n_big), dim3(64), s, n_big, n_big, big, part, part_bad, pk_out, pk_st);
}

void launch_vs_hash_sig(hipStream_t s, uint32_t n, const uint8_t* msgs32, const uint32_t* set_off, const uint32_t* arena,
                        const uint8_t* raw_flag, const uint8_t* raw_pk48, const uint8_t* sig, uint32_t sig_stride, const uint32_t* sig_len,
                        const G1A* table, const uint8_t* table_ok, const G1J* pk_agg, const uint8_t* pk_st, const Seed& seed,
                        uint32_t nonce, G2A* H, G1J* rP, G2J* rS, uint8_t* status, bool split) {
  const uint32_t pair = n <= tuning().hash_pair_max ? 1u : 0u;
  const uint32_t nsig = (n + 63) / 64;
  const uint32_t nb = split ? 0u : pair ? (2 * n + 63) / 64 : (n + 63) / 64;  // split: the caller hashes
  GBV_LAUNCH("k_vs_hash_sig", k_vs_hash_sig, dim3(nb + (split ? 2 : 1) * nsig), dim3(64), s, n, n, nb, pair, split ? 1u : 0u, msgs32, set_off, arena, raw_flag, raw_pk48, sig, sig_stride, sig_len, table, table_ok, pk_agg, pk_st, seed, nonce, H, rP, rS, status);
}

void launch_vs_sig_pre(hipStream_t s, uint32_t n, const uint8_t* sig, uint32_t sig_stride, const uint32_t* sig_len, const Seed& seed,
                       uint32_t nonce, G2J* rS, uint8_t* status, uint8_t* sig_st, G2A* Sd, uint8_t* dec_st) {
  launch_vs_sig_decode(s, n, sig, sig_stride, sig_len, Sd, dec_st);
  GBV_LAUNCH("k_vs_sig_pre_quad", k_vs_sig_pre_quad, dim3(2 * ((n + 15) / 16)), dim3(64), s, n, n, Sd, dec_st, seed, nonce, rS, status, sig_st);
}
void launch_vs_pk_rand(hipStream_t s, uint32_t n, const uint32_t* set_off, const uint32_t* arena, const uint8_t* raw_flag,
                       const uint8_t* raw_pk48, const G1A* table, const uint8_t* table_ok, const G1J* pk_agg, const uint8_t* pk_st,
                       const Seed& seed, uint32_t nonce, G1J* rP, uint8_t* status) {
  GBV_LAUNCH("k_vs_pk_rand_quad", k_vs_pk_rand_quad, dim3((n + 15) / 16), dim3(64), s, n, n, set_off, arena, raw_flag, raw_pk48, table, table_ok, pk_agg, pk_st, seed, nonce, rP, status);
}

void launch_sig_validate(LaunchCfg c, uint32_t n, const uint8_t* sig, uint32_t sig_len, uint8_t* status, uint8_t* out96) {
  hipLaunchKernelGGL(k_sig_validate, dim3(c.blocks), dim3(64), 0, c.stream, n, sig, sig_len, status, out96);
  debug_sync(c.stream, "k_sig_validate");
}
}  // namespace gbv
