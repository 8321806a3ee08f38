// SHA-256 (FIPS 180-4) for the device: the general compression used by hash_to_G2's
// expand_message_xmd, and the 64-byte digest that every SSZ Merkle node is (hash(left || right)),
// with the constant padding block of a 64-byte message folded into the round constants.
#pragma once
#include "fp_types.h"

namespace gbv {

// ---- SHA-256 --------------------------------------------------------------------------------
GBV_HD uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

GBV_HD void sha256_init(uint32_t s[8]) {
  s[0] = 0x6a09e667u; s[1] = 0xbb67ae85u; s[2] = 0x3c6ef372u; s[3] = 0xa54ff53au;
  s[4] = 0x510e527fu; s[5] = 0x9b05688cu; s[6] = 0x1f83d9abu; s[7] = 0x5be0cd19u;
}

static constexpr uint32_t SHA256_K[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

// One compression of a 64-byte block given as 16 big-endian words.
GBV_NI void sha256_compress(uint32_t s[8], const uint32_t blk[16]) {
  uint32_t w[16];
  for (int i = 0; i < 16; ++i) w[i] = blk[i];
  uint32_t a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
      uint32_t s0 = rotr32(w15, 7) ^ rotr32(w15, 18) ^ (w15 >> 3);
      uint32_t s1 = rotr32(w2, 17) ^ rotr32(w2, 19) ^ (w2 >> 10);
      wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
      w[i & 15] = wi;
    }
    uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = h + S1 + ch + SHA256_K[i] + wi;
    uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
    uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint32_t t2 = S0 + mj;
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  s[0] += a; s[1] += b; s[2] += c; s[3] += d; s[4] += e; s[5] += f; s[6] += g; s[7] += h;
}

// ---- SSZ nodes: SHA-256 of exactly 64 bytes ---------------------------------------------------
// persistent-merkle-tree's hasher.digest64(a, b) = sha256(a || b) (@chainsafe/as-sha256 0.5.0,
// yarn.lock:360; call site light-client/src/utils/verifyMerkleBranch.ts:23).  A 64-byte message has
// a second block that never changes (0x80, zeros, bit length 512), so its whole message schedule is a
// compile-time constant: SHA256_PAD64_KW[i] = K[i] + W_pad[i], and that block costs rounds only.
typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));

struct Sha256Kw { uint32_t v[64]; };
constexpr uint32_t sha256_rotr_c(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
constexpr Sha256Kw sha256_pad64_kw() {
  uint32_t w[64] = {};
  w[0] = 0x80000000u;
  w[15] = 512u;
  for (int i = 16; i < 64; ++i) {
    uint32_t s0 = sha256_rotr_c(w[i - 15], 7) ^ sha256_rotr_c(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = sha256_rotr_c(w[i - 2], 17) ^ sha256_rotr_c(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  Sha256Kw r = {};
  for (int i = 0; i < 64; ++i) r.v[i] = SHA256_K[i] + w[i];
  return r;
}
static constexpr Sha256Kw SHA256_PAD64_KW = sha256_pad64_kw();

// Three-input bit functions as single gfx950 VOP3 ops (v_bitop3_b32; truth tables in the
// a=0xF0 / b=0xCC / c=0xAA convention).  Only symmetric functions go through bitop3, so the operand
// order of the table cannot matter; the host-test build uses the plain expressions.
GBV_HD uint32_t xor3_32(uint32_t a, uint32_t b, uint32_t c) {
#ifdef __HIP_DEVICE_COMPILE__
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
  return a ^ b ^ c;
#endif
}
GBV_HD uint32_t maj32(uint32_t a, uint32_t b, uint32_t c) {
#ifdef __HIP_DEVICE_COMPILE__
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
#else
  return (a & b) | (a & c) | (b & c);
#endif
}

// 64 rounds over state s.  kw(i) supplies K[i] + W[i]; the message schedule (if any) is the caller's.
template <class KW> GBV_HD void sha256_rounds(uint32_t s[8], KW kw) {
  uint32_t a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    uint32_t S1 = xor3_32(rotr32(e, 6), rotr32(e, 11), rotr32(e, 25));
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = h + S1 + ch + kw(i);
    uint32_t t2 = xor3_32(rotr32(a, 2), rotr32(a, 13), rotr32(a, 22)) + maj32(a, b, c);
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  s[0] += a; s[1] += b; s[2] += c; s[3] += d; s[4] += e; s[5] += f; s[6] += g; s[7] += h;
}

// sha256(m) for a 64-byte m given as 16 big-endian words; returns the digest as 8 big-endian words.
GBV_HD u32x8 sha256_digest64_inl(u32x16 m) {
  uint32_t w[64];
#pragma unroll
  for (int i = 0; i < 16; ++i) w[i] = m[i];
#pragma unroll
  for (int i = 16; i < 64; ++i) {
    uint32_t w15 = w[i - 15], w2 = w[i - 2];
    uint32_t s0 = xor3_32(rotr32(w15, 7), rotr32(w15, 18), w15 >> 3);
    uint32_t s1 = xor3_32(rotr32(w2, 17), rotr32(w2, 19), w2 >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t s[8];
  sha256_init(s);
  sha256_rounds(s, [&](int i) { return SHA256_K[i] + w[i]; });
  sha256_rounds(s, [](int i) { return SHA256_PAD64_KW.v[i]; });
  u32x8 r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = s[i];
  return r;
}

// Out of line: one copy of the ~2.4k-instruction body serves every node of a tree walk.
GBV_NI u32x8 sha256_digest64(u32x16 m) { return sha256_digest64_inl(m); }

GBV_HD u32x16 sha256_cat(u32x8 l, u32x8 r) {
  u32x16 m;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    m[i] = l[i];
    m[8 + i] = r[i];
  }
  return m;
}
GBV_HD u32x8 sha256_node(u32x8 l, u32x8 r) { return sha256_digest64(sha256_cat(l, r)); }

}  // namespace gbv
