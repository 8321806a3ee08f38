// RFC 9380 hash_to_curve for G2, suite BLS12381G2_XMD:SHA-256_SSWU_RO_, with the Ethereum POP DST
// "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_" (what blst's verify / verifyMultipleAggregateSignatures
// hash messages with).  Messages on this path are always 32-byte signing roots
// (state-transition/src/util/signingRoot.ts:7-13), so expand_message_xmd is laid out for 32 bytes.
#pragma once
#include "curve.h"

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

// DST' = DST || I2OSP(len(DST), 1) = 44 bytes = 11 big-endian words
static constexpr uint32_t DST_PRIME_W[11] = {
    0x424c535fu, 0x5349475fu, 0x424c5331u, 0x32333831u, 0x47325f58u, 0x4d443a53u,
    0x48412d32u, 0x35365f53u, 0x5357555fu, 0x524f5f50u, 0x4f505f2bu};

// expand_message_xmd(msg32, DST_POP, 256) -> 64 big-endian words (b_1 .. b_8)
GBV_HD void expand_message_xmd_32(uint32_t out[64], const uint32_t msg[8]) {
  uint32_t blk[16];
  uint32_t s[8];
  // b_0 = H(Z_pad(64) || msg || I2OSP(256, 2) || 0x00 || DST')  -- 143 bytes, 3 blocks
  sha256_init(s);
  for (int i = 0; i < 16; ++i) blk[i] = 0;
  sha256_compress(s, blk);
  // block 1: msg (32B) || 01 00 00 || DST'[0..28]
  for (int i = 0; i < 8; ++i) blk[i] = msg[i];
  // bytes 32..35 = 0x01 0x00 0x00 DST'[0]
  blk[8] = 0x01000000u | (DST_PRIME_W[0] >> 24);
  for (int i = 9; i < 16; ++i) blk[i] = (DST_PRIME_W[i - 9] << 8) | (DST_PRIME_W[i - 8] >> 24);
  sha256_compress(s, blk);
  // block 2: DST'[29..43] (15 bytes) || 0x80 || 0... || bitlen 143*8
  // DST' bytes 29..43: word 7 bytes 1..3, words 8..10
  blk[0] = (DST_PRIME_W[7] << 8) | (DST_PRIME_W[8] >> 24);
  blk[1] = (DST_PRIME_W[8] << 8) | (DST_PRIME_W[9] >> 24);
  blk[2] = (DST_PRIME_W[9] << 8) | (DST_PRIME_W[10] >> 24);
  blk[3] = (DST_PRIME_W[10] << 8) | 0x80u;
  for (int i = 4; i < 15; ++i) blk[i] = 0;
  blk[15] = 143u * 8u;
  sha256_compress(s, blk);
  uint32_t b0[8];
  for (int i = 0; i < 8; ++i) b0[i] = s[i];
  // b_i = H((b_0 ^ b_{i-1}) || I2OSP(i, 1) || DST')  -- 77 bytes, 2 blocks
  uint32_t prev[8];
  for (int i = 0; i < 8; ++i) prev[i] = 0;
  for (int idx = 1; idx <= 8; ++idx) {
    sha256_init(s);
    for (int i = 0; i < 8; ++i) blk[i] = b0[i] ^ prev[i];
    blk[8] = ((uint32_t)idx << 24) | (DST_PRIME_W[0] >> 8);
    for (int i = 9; i < 16; ++i) blk[i] = (DST_PRIME_W[i - 9] << 24) | (DST_PRIME_W[i - 8] >> 8);
    sha256_compress(s, blk);
    // second block: DST' bytes 31..43 (13 bytes) || 0x80 || 0 || bitlen 77*8
    blk[0] = (DST_PRIME_W[7] << 24) | (DST_PRIME_W[8] >> 8);
    blk[1] = (DST_PRIME_W[8] << 24) | (DST_PRIME_W[9] >> 8);
    blk[2] = (DST_PRIME_W[9] << 24) | (DST_PRIME_W[10] >> 8);
    blk[3] = (DST_PRIME_W[10] << 24) | 0x00800000u;
    for (int i = 4; i < 15; ++i) blk[i] = 0;
    blk[15] = 77u * 8u;
    sha256_compress(s, blk);
    for (int i = 0; i < 8; ++i) {
      prev[i] = s[i];
      out[(idx - 1) * 8 + i] = s[i];
    }
  }
}

// 64 big-endian bytes (16 words) -> Fp (Montgomery), value mod p
GBV_HD Fp fp_from_be64_words(const uint32_t w[16]) {
  Fp hi = fp_zero(), lo = fp_zero();
  for (int i = 0; i < 8; ++i) {
    hi.v[i] = w[7 - i];
    lo.v[i] = w[15 - i];
  }
  return fp_add(fp_mul(hi, R2_SHL256_RAW), fp_mul(lo, R2_RAW));
}

// ---- simplified SWU onto E2': y^2 = x^3 + A'x + B', A' = 240i, B' = 1012(1+i), Z = -(2+i) ----
GBV_NI G2A map_to_curve_sswu(Fp2 u) {
  Fp2 u2 = fp2_sqr(u);
  Fp2 zu2 = fp2_mul(SSWU_Z, u2);
  Fp2 tv1 = fp2_add(fp2_sqr(zu2), zu2);
  bool exc = fp2_is_zero(tv1);
  Fp2 x1 = fp2_mul(SSWU_MINUS_B_OVER_A, fp2_add(fp2_one(), fp2_inv(tv1)));
  x1 = fp2_sel(exc, SSWU_B_OVER_ZA, x1);
  Fp2 gx1 = fp2_add(fp2_mul(fp2_add(fp2_sqr(x1), SSWU_A), x1), SSWU_B);
  Fp2 x2 = fp2_mul(zu2, x1);
  Fp2 gx2 = fp2_add(fp2_mul(fp2_add(fp2_sqr(x2), SSWU_A), x2), SSWU_B);
  Fp2 y1, y2;
  bool ok1 = fp2_sqrt(y1, gx1);
  fp2_sqrt(y2, gx2);
  Fp2 x = fp2_sel(ok1, x1, x2);
  Fp2 y = fp2_sel(ok1, y1, y2);
  if (fp2_sgn0(u) != fp2_sgn0(y)) y = fp2_neg(y);
  return G2A{x, y};
}

// 3-isogeny E2' -> E2 (RFC 9380 E.3), output in Jacobian coordinates (no inversion):
//   Z = xd*yd, X = xn*xd*yd^2, Y = y*yn*xd^3*yd^2
GBV_NI G2J iso_map(G2A p) {
  const Fp2& x = p.x;
  Fp2 xn = fp2_add(fp2_mul(fp2_add(fp2_mul(fp2_add(fp2_mul(ISO_XNUM_3, x), ISO_XNUM_2), x), ISO_XNUM_1), x), ISO_XNUM_0);
  Fp2 xd = fp2_add(fp2_mul(fp2_add(x, ISO_XDEN_1), x), ISO_XDEN_0);
  Fp2 yn = fp2_add(fp2_mul(fp2_add(fp2_mul(fp2_add(fp2_mul(ISO_YNUM_3, x), ISO_YNUM_2), x), ISO_YNUM_1), x), ISO_YNUM_0);
  Fp2 yd = fp2_add(fp2_mul(fp2_add(fp2_mul(fp2_add(x, ISO_YDEN_2), x), ISO_YDEN_1), x), ISO_YDEN_0);
  Fp2 yd2 = fp2_sqr(yd);
  Fp2 xd2 = fp2_sqr(xd);
  G2J r;
  r.z = fp2_mul(xd, yd);
  r.x = fp2_mul(fp2_mul(xn, xd), yd2);
  r.y = fp2_mul(fp2_mul(fp2_mul(p.y, yn), fp2_mul(xd2, xd)), yd2);
  return r;
}

// RFC 9380 G.3 clear_cofactor: h_eff P = [x^2-x-1]P + [x-1]psi(P) + psi^2(2P)
GBV_NI G2J clear_cofactor_g2(G2J p) {
  G2J t1 = jac_neg(g2_mul_xabs_jac(p));         // [x] P
  G2J t2 = g2_psi_jac(p);                         // psi(P)
  G2J t3 = g2_psi_jac(g2_psi_jac(jac_dbl(p)));    // psi^2(2P)
  t3 = jac_add(t3, jac_neg(t2));
  t2 = jac_add(t1, t2);
  t2 = jac_neg(g2_mul_xabs_jac(t2));             // [x] t2
  t3 = jac_add(t3, t2);
  t3 = jac_add(t3, jac_neg(t1));
  return jac_add(t3, jac_neg(p));
}

// hash_to_G2(msg32) as an affine point (Montgomery).  msg given as 8 big-endian words.
GBV_NI G2A hash_to_g2(const uint32_t* msg) {
  uint32_t u[64];
  expand_message_xmd_32(u, msg);
  Fp2 u0{fp_from_be64_words(u), fp_from_be64_words(u + 16)};
  Fp2 u1{fp_from_be64_words(u + 32), fp_from_be64_words(u + 48)};
  G2J q0 = iso_map(map_to_curve_sswu(u0));
  G2J q1 = iso_map(map_to_curve_sswu(u1));
  G2J q = clear_cofactor_g2(jac_add(q0, q1));
  G2A out;
  jac_to_aff(out, q);
  return out;
}

}  // namespace gbv
