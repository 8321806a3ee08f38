// gfx950 kernels of the signature-set verifier.  One thread owns one signature set (or one
// chunk / one message) and keeps its field elements in VGPRs; the kernels of one call run back to
// back on the context's HIP stream.
//
// Reference mapping:
//   k_hash_msgs         hash_to_G2 inside blst verify / verifyMultipleAggregateSignatures
//   k_sm_prepare        aggregateWithRandomness per set: Signature.fromBytes(sig, true) + r_i*pk, r_i*sig
//                       (multithread/jobItem.ts:73)
//   k_sm_group_sum      sum_i r_i pk_i, sum_i r_i sig_i per same-message chunk
//   k_sm_group_pairing  verify(msg, aggPk, aggSig) of the chunk (worker.ts:29-107 -> maybeBatch n = 1)
//   k_sm_fallback       retry each set individually (jobItem.ts:93-125)
//   k_vs_prepare        per-set part of verifyMultipleAggregateSignatures (+ aggregatePublicKeys
//                       of index lists, bls/utils.ts:5-20)
//   k_vs_chunk          per-chunk multi-pairing product + one final exponentiation (maybeBatch.ts:17-26)
#pragma once
#include "hash_to_curve.h"
#include "pairing.h"

namespace gbv {

struct Seed { uint32_t w[8]; };

enum : uint8_t { SET_OK = 0, SET_BAD_SIG = 1, SET_BAD_PK = 2 };
enum : uint8_t { GRP_PENDING = 0, GRP_FALLBACK = 1, GRP_OK = 2 };

// Per-set random 64-bit scalar r_i = SHA-256(seed || i || nonce)[0..8), forced non-zero.
// blst draws 64-bit random scalars for the same purpose; only the booleans are compared.
__device__ inline uint64_t prf_scalar(const Seed& s, uint32_t i, uint32_t nonce) {
  uint32_t st[8];
  sha256_init(st);
  uint32_t blk[16];
  for (int k = 0; k < 8; ++k) blk[k] = s.w[k];
  blk[8] = i;
  blk[9] = nonce;
  blk[10] = 0x80000000u;
  for (int k = 11; k < 15; ++k) blk[k] = 0;
  blk[15] = 40u * 8u;
  sha256_compress(st, blk);
  uint64_t r = ((uint64_t)st[0] << 32) | st[1];
  return r ? r : 1ull;
}

__device__ inline void load_msg_words(uint32_t w[8], const uint8_t* m) {
  for (int i = 0; i < 8; ++i)
    w[i] = ((uint32_t)m[4 * i] << 24) | ((uint32_t)m[4 * i + 1] << 16) | ((uint32_t)m[4 * i + 2] << 8) | m[4 * i + 3];
}

// ---- hashing ----------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_hash_msgs(const uint8_t* __restrict__ msgs32, uint32_t n, G2A* __restrict__ H) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t w[8];
  load_msg_words(w, msgs32 + 32ull * i);
  H[i] = hash_to_g2(w);
}

// ---- same-message path ------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_sm_prepare(uint32_t n, const uint32_t* __restrict__ idx, const uint8_t* __restrict__ sig96,
                                                   const G1A* __restrict__ table, const uint8_t* __restrict__ table_ok, uint32_t table_n,
                                                   Seed seed, uint32_t nonce, G2A* __restrict__ S_out, G2J* __restrict__ rS_out,
                                                   G1J* __restrict__ rP_out, uint8_t* __restrict__ status) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
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
  rS_out[i] = jac_mul_u64(s, r);
  rP_out[i] = jac_mul_u64(table[k], r);
}

__global__ void __launch_bounds__(64) k_sm_group_sum(uint32_t G, const uint32_t* __restrict__ grp_off, const uint8_t* __restrict__ status,
                                                     const G2J* __restrict__ rS, const G1J* __restrict__ rP, G1A* __restrict__ Pg,
                                                     G2A* __restrict__ Sg, uint8_t* __restrict__ grp_state) {
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
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

__global__ void __launch_bounds__(64) k_sm_group_pairing(uint32_t G, const uint32_t* __restrict__ grp_msg, const G1A* __restrict__ Pg,
                                                         const G2A* __restrict__ Sg, const G2A* __restrict__ H,
                                                         uint8_t* __restrict__ grp_state, uint32_t* __restrict__ n_fallback) {
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  uint8_t st = grp_state[g];
  if (st == GRP_PENDING) {
    bool ok = pairing_check_2(Pg[g], false, H[grp_msg[g]], g1_neg_generator(), false, Sg[g]);
    st = ok ? GRP_OK : GRP_FALLBACK;
    grp_state[g] = st;
  }
  if (st == GRP_FALLBACK) atomicAdd(n_fallback, 1u);
}

// valid[i] for every set; sets of failed chunks are verified one by one (2-pair check each).
__global__ void __launch_bounds__(64) k_sm_fallback(uint32_t n, const uint32_t* __restrict__ set_grp, const uint32_t* __restrict__ grp_msg,
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

// ---- pubkey table -------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_pk_decompress(uint32_t n, const uint8_t* __restrict__ pk48, int validate,
                                                      G1A* __restrict__ table, uint8_t* __restrict__ table_ok,
                                                      uint8_t* __restrict__ status) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  G1A a;
  uint8_t st = g1_decompress(a, pk48 + 48ull * i);
  if (st == PT_OK && validate && !g1_in_subgroup(a)) st = PT_NOT_IN_GROUP;
  if (st != PT_OK) {
    a.x = fp_zero();
    a.y = fp_zero();
  }
  table[i] = a;
  table_ok[i] = st == PT_OK;
  status[i] = st;
}

__global__ void k_pk_replicate(G1A* __restrict__ table, uint8_t* __restrict__ table_ok, uint32_t src_first, uint32_t src_n,
                               uint32_t dst_first, uint32_t n) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t s = src_first + (i % src_n);
  table[dst_first + i] = table[s];
  table_ok[dst_first + i] = table_ok[s];
}

// aggregatePublicKeys over an index list: one 256-thread block, strided partial sums + LDS tree.
__global__ void __launch_bounds__(256) k_aggregate(const uint32_t* __restrict__ idx, uint32_t k, const G1A* __restrict__ table,
                                                   const uint8_t* __restrict__ table_ok, uint8_t* __restrict__ out48,
                                                   uint32_t* __restrict__ bad) {
  __shared__ G1J part[256];
  uint32_t t = threadIdx.x;
  G1J acc = jac_infinity<Fp>();
  for (uint32_t i = t; i < k; i += 256) {
    uint32_t j = idx[i];
    if (!table_ok[j]) atomicOr(bad, 1u);
    acc = jac_add_aff(acc, table[j]);
  }
  part[t] = acc;
  __syncthreads();
  for (uint32_t s = 128; s > 0; s >>= 1) {
    if (t < s) part[t] = jac_add(part[t], part[t + s]);
    __syncthreads();
  }
  if (t == 0) {
    G1A a;
    bool finite = jac_to_aff(a, part[0]);
    g1_compress(out48, a, !finite);
  }
}

// ---- distinct-message path (verifySignatureSets) ------------------------------------------------
__global__ void __launch_bounds__(64) k_vs_prepare(uint32_t n, const uint32_t* __restrict__ set_idx_off, const uint32_t* __restrict__ idx,
                                                   const uint8_t* __restrict__ raw_flag, const uint8_t* __restrict__ raw_pk48,
                                                   const uint8_t* __restrict__ msgs32, const uint8_t* __restrict__ sig, uint32_t sig_stride,
                                                   const uint32_t* __restrict__ sig_len, const G1A* __restrict__ table,
                                                   const uint8_t* __restrict__ table_ok, Seed seed, uint32_t nonce,
                                                   Fp12* __restrict__ f_out, G2J* __restrict__ rS_out, uint8_t* __restrict__ status) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t st = SET_OK;
  // public key: raw (validated like PublicKey.fromBytes(pk, true)) or aggregate of table entries
  G1A pk;
  bool pk_inf = false;
  if (raw_flag[i]) {
    uint8_t ds = g1_decompress(pk, raw_pk48 + 48ull * i);
    if (ds != PT_OK || !g1_in_subgroup(pk)) st = SET_BAD_PK;
  } else {
    uint32_t b = set_idx_off[i], e = set_idx_off[i + 1];
    G1J acc = jac_infinity<Fp>();
    for (uint32_t j = b; j < e; ++j) {
      uint32_t k = idx[j];
      if (!table_ok[k]) st = SET_BAD_PK;
      acc = jac_add_aff(acc, table[k]);
    }
    pk_inf = !jac_to_aff(pk, acc);
  }
  if (pk_inf) st = SET_BAD_PK;  // verify with an infinity pubkey fails in blst
  G2A s;
  uint8_t ds = g2_decode(s, sig + (size_t)sig_stride * i, sig_len[i]);
  if (ds != PT_OK || !g2_in_subgroup(s)) st = SET_BAD_SIG;
  status[i] = st;
  if (st != SET_OK) return;
  uint64_t r = prf_scalar(seed, i, nonce);
  G1A rp;
  jac_to_aff(rp, jac_mul_u64(pk, r));
  rS_out[i] = jac_mul_u64(s, r);
  uint32_t w[8];
  load_msg_words(w, msgs32 + 32ull * i);
  G2A h = hash_to_g2(w);
  f_out[i] = miller_loop_1(rp, h);
}

__global__ void __launch_bounds__(64) k_vs_chunk(uint32_t C, const uint32_t* __restrict__ chunk_off, const uint8_t* __restrict__ status,
                                                 const Fp12* __restrict__ f, const G2J* __restrict__ rS, uint8_t* __restrict__ chunk_valid) {
  uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  uint32_t b = chunk_off[c], e = chunk_off[c + 1];
  bool ok = b < e;
  for (uint32_t i = b; i < e; ++i) ok &= status[i] == SET_OK;
  if (!ok) {
    chunk_valid[c] = 0;
    return;
  }
  Fp12 acc = f[b];
  G2J s = rS[b];
  for (uint32_t i = b + 1; i < e; ++i) {
    acc = fp12_mul(acc, f[i]);
    s = jac_add(s, rS[i]);
  }
  G2A sa;
  if (!jac_to_aff(sa, s)) {
    chunk_valid[c] = 0;
    return;
  }
  acc = fp12_mul(acc, miller_loop_1(g1_neg_generator(), sa));
  chunk_valid[c] = fp12_is_one(final_exponentiation(acc)) ? 1 : 0;
}

// ---- utilities (synthetic workloads, tests) -----------------------------------------------------
__device__ inline void load_scalar_be32(uint32_t k[8], const uint8_t* b) {
  for (int i = 0; i < 8; ++i) {
    const uint8_t* q = b + 28 - 4 * i;
    k[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
}

__global__ void __launch_bounds__(64) k_util_sk_to_pk(uint32_t n, const uint8_t* __restrict__ sk32, uint8_t* __restrict__ pk48) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t k[8];
  load_scalar_be32(k, sk32 + 32ull * i);
  G1A g{G1_GEN_X, G1_GEN_Y};
  G1A a;
  bool fin = jac_to_aff(a, jac_mul_u256(g, k));
  g1_compress(pk48 + 48ull * i, a, !fin);
}

__global__ void __launch_bounds__(64) k_util_sign(uint32_t n, const uint8_t* __restrict__ sk32, const uint32_t* __restrict__ grp,
                                                  const G2A* __restrict__ H, uint8_t* __restrict__ sig96) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t k[8];
  load_scalar_be32(k, sk32 + 32ull * i);
  G2A a;
  bool fin = jac_to_aff(a, jac_mul_u256(H[grp[i]], k));
  g2_compress(sig96 + 96ull * i, a, !fin);
}

__global__ void __launch_bounds__(64) k_util_g2_out(uint32_t n, const G2A* __restrict__ H, uint8_t* __restrict__ out192) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t* o = out192 + 192ull * i;
  fp_store_be48(o, fp_from_mont(H[i].x.c1));
  fp_store_be48(o + 48, fp_from_mont(H[i].x.c0));
  fp_store_be48(o + 96, fp_from_mont(H[i].y.c1));
  fp_store_be48(o + 144, fp_from_mont(H[i].y.c0));
}

}  // namespace gbv
