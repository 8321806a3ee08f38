// RFC 9380 hash_to_curve for G2, suite BLS12381G2_XMD:SHA-256_SSWU_RO_, with the Ethereum POP DST
// "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_" (what blst's verify / verifyMultipleAggregateSignatures
// hash messages with).  Messages on this path are always 32-byte signing roots
// (state-transition/src/util/signingRoot.ts:7-13), so expand_message_xmd is laid out for 32 bytes.
#pragma once
#include "curve.h"
#include "sha256.h"

namespace gbv {

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
  // ONE norm exponentiation decides which of g(x1), g(x2) is the square and yields the norm root
  // of that one: n1 = N(g(x1)); a1 = n1^((p+1)/4) is sqrt(n1) if n1 is a residue (then g(x1) is a
  // square in Fp2), else sqrt(-n1); and g(x2) = Z^3 u^6 g(x1) gives
  // sqrt(N(g(x2))) = N(u)^3 sqrt(-N(Z)^3) a1.  Then one fp2_sqrt_with_norm_root -- two Fp
  // exponentiations per map instead of four.
  Fp n1 = fp2_norm(gx1);
  Fp a1 = fp_pow_sched(n1, SCHED_SQRT_NSQ, SCHED_SQRT_IDX, SCHED_SQRT_STEPS);
  bool sq1 = fp_eq(fp_sqr(a1), n1);
  Fp nu = fp2_norm(u);
  Fp a2 = fp_mul(fp_mul(fp_mul(fp_sqr(nu), nu), SSWU_SQRT_MINUS_NZ3), a1);
  Fp2 x = fp2_sel(sq1, x1, x2);
  Fp2 y;
  fp2_sqrt_with_norm_root(y, fp2_sel(sq1, gx1, gx2), fp_sel(sq1, a1, a2));
  if (fp2_sgn0(u) != fp2_sgn0(y)) y = fp2_neg(y);
  return ret_copy(G2A{x, y});
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
  return ret_copy(r);
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
  G2J r = jac_add(t3, jac_neg(p));
  return ret_copy(r);
}

// hash_to_field: u_j = expand_message_xmd(msg)[64 j .. 64 j + 64) as Fp2 (j = 0, 1)
GBV_HD Fp2 hash_to_field_fp2(const uint32_t* msg, int j) {
  uint32_t u[64];
  expand_message_xmd_32(u, msg);
  return Fp2{fp_from_be64_words(u + 32 * j), fp_from_be64_words(u + 32 * j + 16)};
}

// Q(u) = iso_map(map_to_curve(u)); the two halves of hash_to_G2 are independent
GBV_NI G2J hash_map_iso(Fp2 u) { return iso_map(map_to_curve_sswu(u)); }

// clear_cofactor(Q0 + Q1) as an affine point
GBV_NI G2A hash_finish(G2J q0, G2J q1) {
  G2J q = clear_cofactor_g2(jac_add(q0, q1));
  G2A out;
  jac_to_aff(out, q);
  return ret_copy(out);
}

// hash_to_G2(msg32) as an affine point (Montgomery).  msg given as 8 big-endian words.
GBV_NI G2A hash_to_g2(const uint32_t* msg) {
  uint32_t u[64];
  expand_message_xmd_32(u, msg);
  Fp2 u0{fp_from_be64_words(u), fp_from_be64_words(u + 16)};
  Fp2 u1{fp_from_be64_words(u + 32), fp_from_be64_words(u + 48)};
  return hash_finish(hash_map_iso(u0), hash_map_iso(u1));
}

}  // namespace gbv
