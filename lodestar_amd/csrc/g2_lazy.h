// Signed lazy 28-bit limbs for the G2 subgroup check's chain of 63 doublings ([|x|] Q, curve.h
// g2_in_subgroup; blst's POINTonE2_in_G2 inside Signature.fromBytes(sig, true), jobItem.ts:73).
//
// The canonical form (12 x 32-bit limbs, fp.h) pays, per Fp product, the repacking into the product's
// 28-bit limbs and back plus a final conditional subtraction (~130 of fp_mul's ~607 instructions), and
// per addition a modular carry chain with a compare and a select (~33 instructions).  Here a chain of
// doublings stays in the product's own limb form:
//   * an element is 14 SIGNED 28-bit-radix limbs (int32 each, value sum_i v_i 2^(28 i)), not canonical:
//     any integer congruent to the element mod p;
//   * add / sub / small multiples are limbwise (14 instructions, no carry, no modular reduction: a
//     difference is simply negative limbs);
//   * mul28s is the 28-bit Montgomery product (fp.h mul28_inl) on signed limbs: every a_i b_j is one
//     v_mad_i64_i32 into a signed 64-bit column accumulator, the m_i p_j one v_mad_u64_u32 as before,
//     the column carry an arithmetic shift.  Output: limbs 0..12 in [0, 2^28), the top limb signed;
//     |out| < |a b| / 2^392 + p;
//   * s28_norm moves each limb's carry one limb up (all limbs in parallel): limbs back in [-8, 2^28 + 8).
// Bounds (stated at every step of s2j_dbl, checked by the host build on every call -- GBV_HOST_TEST --
// and at the extremes by tests/test_host_arith.py): a product column holds 14 a_i b_j terms and 14
// m_i p_j < 2^56, so |a_i| |b_j| <= 2^59 keeps it inside int64; limbs stay inside int32; values stay
// below 64 p (a doubling maps inputs below 64 p to outputs below 55 p, a mixed addition too; product
// outputs stay below 8 p there).  The chain converts back to the canonical form once, at its end.
#pragma once
#if defined(GBV_HOST_TEST)
#include <cstdio>
#include <cstdlib>
#endif

namespace gbv {

typedef int32_t i32x14 __attribute__((ext_vector_type(14)));
struct S28 { i32x14 v; };
struct S2 { S28 c0, c1; };
struct S2J { S2 x, y, z; };

#if defined(GBV_HOST_TEST)
// host build: every lazy operation is recomputed in 64 bits and every product column in 128 bits; an
// out-of-range intermediate aborts the test process
inline void s28_check(bool ok, const char* what) {
  if (!ok) {
    fprintf(stderr, "g2_lazy bound violated: %s\n", what);
    abort();
  }
}
inline long long g_s28_max_col_bits = 0;  // widest product column seen (bits of |column|), for the tests
#define S28_LIMB_OP(r, expr)                                                   \
  do {                                                                        \
    const long long t_ = (long long)(expr);                                   \
    s28_check(t_ >= -2147483648LL && t_ <= 2147483647LL, "limb outside int32"); \
    (r) = (int32_t)t_;                                                        \
  } while (0)
#else
#define S28_LIMB_OP(r, expr) (r) = (int32_t)(expr)
#endif

GBV_HD S28 s28_from_fp(const Fp& a) {  // canonical (or any value < 2^384): limbs in [0, 2^28)
  const F28 t = fp_to28(a);
  S28 r;
#pragma unroll
  for (int i = 0; i < 14; ++i) r.v[i] = (int32_t)t.v[i];
  return r;
}

GBV_HD S28 s28_add(const S28& a, const S28& b) {
  S28 r;
#pragma unroll
  for (int i = 0; i < 14; ++i) S28_LIMB_OP(r.v[i], (long long)a.v[i] + b.v[i]);
  return r;
}
GBV_HD S28 s28_sub(const S28& a, const S28& b) {
  S28 r;
#pragma unroll
  for (int i = 0; i < 14; ++i) S28_LIMB_OP(r.v[i], (long long)a.v[i] - b.v[i]);
  return r;
}
template <int K> GBV_HD S28 s28_mulk(const S28& a) {  // K a, limbwise (K = 2, 3, 8: shifts / shift-adds)
  S28 r;
#pragma unroll
  for (int i = 0; i < 14; ++i) S28_LIMB_OP(r.v[i], (long long)a.v[i] * K);
  return r;
}
// a - K b, limbwise
template <int K> GBV_HD S28 s28_sub_k(const S28& a, const S28& b) {
  S28 r;
#pragma unroll
  for (int i = 0; i < 14; ++i) S28_LIMB_OP(r.v[i], (long long)a.v[i] - (long long)K * b.v[i]);
  return r;
}

// One carry step on every limb at once: limb i keeps its low 28 bits plus limb i-1's carry
// (arithmetic shift).  The value is unchanged; limbs of |x| < 2^31 come back in [-8, 2^28 + 8).
GBV_HD S28 s28_norm(const S28& x) {
  S28 r;
  r.v[0] = x.v[0] & (int32_t)M28;
#pragma unroll
  for (int i = 1; i < 13; ++i) r.v[i] = (x.v[i] & (int32_t)M28) + (x.v[i - 1] >> 28);
  S28_LIMB_OP(r.v[13], (long long)x.v[13] + (x.v[12] >> 28));
  return r;
}

// a b 2^-392 mod p on signed limbs (fp.h mul28_inl's column scan): |a_i| |b_j| <= 2^59.
GBV_HD S28 mul28s_inl(const S28& a, const S28& b) {
#if defined(GBV_HOST_TEST)
  ++g_fme_count;
  for (int i = 0; i < 14; ++i)
    for (int j = 0; j < 14; ++j)
      s28_check((long double)std::llabs((long long)a.v[i]) * (long double)std::llabs((long long)b.v[j]) <= 576460752303423488.0L * 1.0001L,
                "product operand limbs |a_i| |b_j| > 2^59 (1 + 1e-4)");
  __int128 wide = 0;
#endif
  uint32_t m[14];
  int32_t r[14];
  int64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 27; ++k) {
#pragma unroll
    for (int i = 0; i < 14; ++i) {
      const int j = k - i;
      if (j >= 0 && j < 14) {
        acc += (int64_t)a.v[i] * (int64_t)b.v[j];
#if defined(GBV_HOST_TEST)
        wide += (__int128)a.v[i] * b.v[j];
#endif
      }
    }
#pragma unroll
    for (int i = 0; i < 14; ++i) {
      const int j = k - i;
      if (i < k && j >= 0 && j < 14) {
        acc += (int64_t)((uint64_t)m[i] * P28[j]);
#if defined(GBV_HOST_TEST)
        wide += (__int128)((uint64_t)m[i] * P28[j]);
#endif
      }
    }
    int64_t s = acc;
    if (k < 14) {
      m[k] = ((uint32_t)s * NP28) & M28;
      s += (int64_t)((uint64_t)m[k] * P28[0]);
#if defined(GBV_HOST_TEST)
      wide += (__int128)((uint64_t)m[k] * P28[0]);
#endif
    } else {
      r[k - 14] = (int32_t)((uint32_t)s & M28);
    }
#if defined(GBV_HOST_TEST)
    s28_check(wide == (__int128)s, "product column outside int64");
    {
      const __int128 w = wide < 0 ? -wide : wide;
      long long bits = 0;
      while (bits < 127 && (w >> bits) != 0) ++bits;
      if (bits > g_s28_max_col_bits) g_s28_max_col_bits = bits;
    }
    wide >>= 28;
#endif
    acc = sar28(s);  // arithmetic: floor (two 32-bit ops, fp.h)
  }
  r[13] = (int32_t)acc;
#if defined(GBV_HOST_TEST)
  s28_check(wide == (__int128)acc && wide >= -2147483648LL && wide <= 2147483647LL, "product top limb outside int32");
#endif
  S28 o;
#pragma unroll
  for (int i = 0; i < 14; ++i) o.v[i] = r[i];
  return o;
}

// Out of line: the doubling's 16 products share one copy (the instruction cache; fp.h fp_mul).
GBV_NI S28 mul28s(S28 a, S28 b) { return mul28s_inl(a, b); }



// Canonical Fp of a lazy value (|value| < 256 p): W = value + 256 p > 0, carried to 28-bit limbs, then
// W - q p with q = floor(top / (P28[13] + 1)) <= W / p leaves W' < 2 p; one conditional subtraction.
GBV_HD Fp s28_to_fp(const S28& x) {
  int64_t c = 0;
  uint32_t w[14];
#pragma unroll
  for (int i = 0; i < 14; ++i) {
    c += (int64_t)x.v[i] + 256ll * (int64_t)P28[i];
    w[i] = i < 13 ? (uint32_t)(c & M28) : (uint32_t)c;
    c >>= 28;
  }
  const uint32_t q = w[13] / (P28[13] + 1u);
  int64_t b = 0;
  F28 t;
#pragma unroll
  for (int i = 0; i < 14; ++i) {
    b += (int64_t)w[i] - (int64_t)((uint64_t)q * P28[i]);
    t.v[i] = i < 13 ? (uint32_t)(b & M28) : (uint32_t)b;
    b >>= 28;
  }
  return fp_reduce_once(fp_from28(t));
}

GBV_HD S2 s2_from(const Fp2& a) { return S2{s28_from_fp(a.c0), s28_from_fp(a.c1)}; }
GBV_HD Fp2 s2_to(const S2& a) { return Fp2{s28_to_fp(a.c0), s28_to_fp(a.c1)}; }
GBV_HD S2J s2j_from(const G2J& p) { return S2J{s2_from(p.x), s2_from(p.y), s2_from(p.z)}; }
GBV_HD G2J s2j_to(const S2J& p) { return G2J{s2_to(p.x), s2_to(p.y), s2_to(p.z)}; }

GBV_HD S2 s2_add(const S2& a, const S2& b) { return S2{s28_add(a.c0, b.c0), s28_add(a.c1, b.c1)}; }
GBV_HD S2 s2_sub(const S2& a, const S2& b) { return S2{s28_sub(a.c0, b.c0), s28_sub(a.c1, b.c1)}; }
GBV_HD S2 s2_norm(const S2& a) { return S2{s28_norm(a.c0), s28_norm(a.c1)}; }
template <int K> GBV_HD S2 s2_mulk(const S2& a) { return S2{s28_mulk<K>(a.c0), s28_mulk<K>(a.c1)}; }
template <int K> GBV_HD S2 s2_sub_k(const S2& a, const S2& b) { return S2{s28_sub_k<K>(a.c0, b.c0), s28_sub_k<K>(a.c1, b.c1)}; }

// Karatsuba over i^2 = -1.  a, b normalized (limbs in [-8, 2^28 + 8)): the sums' limbs below 2^29,
// products of them below 2^58.  Out: c0 = t0 - t1 with limbs in (-2^28, 2^28), c1 = t2 - t0 - t1 in
// (-2^29, 2^28).
GBV_HD S2 s2_mul(const S2& a, const S2& b) {
  const S28 t0 = mul28s(a.c0, b.c0);
  const S28 t1 = mul28s(a.c1, b.c1);
  const S28 t2 = mul28s(s28_add(a.c0, a.c1), s28_add(b.c0, b.c1));
  return S2{s28_sub(t0, t1), s28_sub(s28_sub(t2, t0), t1)};
}

// (a0 + a1)(a0 - a1) + (2 a0) a1 i.  For limbs of a in [-2^29, 2^29): the operands' limbs below 2^30
// and 2^29 (a product below 2^59).  Out: product outputs, limbs 0..12 in [0, 2^28).
GBV_HD S2 s2_sqr(const S2& a) {
  const S28 c0 = mul28s(s28_add(a.c0, a.c1), s28_sub(a.c0, a.c1));
  const S28 c1 = mul28s(s28_mulk<2>(a.c0), a.c1);
  return S2{c0, c1};
}

// dbl-2009-l (curve.h jac_dbl, the same X3, Y3, Z3 mod p) on the lazy form.  In: x, y, z normalized,
// values below 64 p.  Out: the same.  L = 2^28; limb ranges at each step on the right.
GBV_HD S2J s2j_dbl(const S2J& p) {
  S2J r;
  const S2 YZ = s2_mul(p.y, p.z);                    // c0 (-L, L), c1 (-2L, L)
  r.z = s2_norm(s2_mulk<2>(YZ));                     // (-4L, 2L) -> normalized
  const S2 B = s2_sqr(p.y);                          // [0, L)
  const S2 A = s2_sqr(p.x);                          // [0, L)
  const S2 T = s2_sqr(s2_add(p.x, B));               // x + B in [-8, 2L + 8): operands < 4L and < 2L
  const S2 C = s2_sqr(B);                            // [0, L)
  const S2 D = s2_norm(s2_mulk<2>(s2_sub(s2_sub(T, A), C)));  // 2 (T - A - C) in (-4L, 2L) -> normalized
  const S2 E = s2_norm(s2_mulk<3>(A));               // 3 A in [0, 3L) -> normalized
  const S2 F = s2_sqr(E);                            // [0, L)
  r.x = s2_norm(s2_sub_k<2>(F, D));                  // F - 2 D in (-2L - 16, L + 16) -> normalized
  const S2 EDX = s2_mul(E, s2_sub(D, r.x));          // D - X3 in (-L - 16, L + 16); c0 (-L, L), c1 (-2L, L)
  r.y = s2_norm(s2_sub_k<8>(s2_norm(EDX), C));       // norm(EDX) in [-2, L), minus 8 C: (-8L + 6, L) -> normalized
  return r;
}

#if defined(GBV_UBENCH)
// tools/ubench_prod.hip only: s2j_dbl with the normalisations of mask SKIP left out (wrong values,
// bounds unchecked; timing of the norm steps).  Bits: 1 Z3, 2 D, 4 E, 8 X3, 16 EDX, 32 Y3.
template <int SKIP> GBV_HD S2 nrm(const S2& a, int bit) { return (SKIP & bit) ? a : s2_norm(a); }
template <int SKIP> GBV_HD S2J s2j_dbl_skip(const S2J& p) {
  S2J r;
  const S2 YZ = s2_mul(p.y, p.z);
  r.z = nrm<SKIP>(s2_mulk<2>(YZ), 1);
  const S2 B = s2_sqr(p.y);
  const S2 A = s2_sqr(p.x);
  const S2 T = s2_sqr(s2_add(p.x, B));
  const S2 C = s2_sqr(B);
  const S2 D = nrm<SKIP>(s2_mulk<2>(s2_sub(s2_sub(T, A), C)), 2);
  const S2 E = nrm<SKIP>(s2_mulk<3>(A), 4);
  const S2 F = s2_sqr(E);
  r.x = nrm<SKIP>(s2_sub_k<2>(F, D), 8);
  const S2 EDX = s2_mul(E, s2_sub(D, r.x));
  r.y = nrm<SKIP>(s2_sub_k<8>(nrm<SKIP>(EDX, 16), C), 32);
  return r;
}
#endif

// r <- [2^k] r, k >= 1 doublings on the lazy form (one copy of the doubling in the code)
GBV_NI void s2j_dbl_n(S2J* r, int k) {
  S2J t = *r;
#pragma nounroll
  for (int i = 0; i < k; ++i) t = s2j_dbl(t);
  *r = t;
}

GBV_NI G2J g2_madd(G2J p, G2A q) { return ret_copy(jac_add_aff(p, q)); }

// *r <- *r + q (madd-2007-bl, curve.h jac_add_aff: the same X3, Y3, Z3 mod p) on the lazy form; q
// affine (its S2 form), not infinity.  In / out normalized, values below 64 p.  No exceptional cases here:
// for *r = +-q (H = 0 mod p) the formula gives Z3 = 2 Z1 H = 0 mod p, and every later doubling
// (Z3 = 2 Y Z) and addition (Z3 = 2 Z1 H) keeps Z = 0 mod p, so the chain's caller sees Z = 0 at the end
// and recomputes on the canonical form, which handles the case (g2_mul_xabs_lazy).  Ordered to keep few
// values live (the finished Z3 goes to memory first).
GBV_NI void s2j_madd(S2J* rp, const S2* q) {
  const S2 Z1 = rp->z;
  const S2 Z1Z1 = s2_sqr(Z1);                                     // [0, L)
  const S2 H = s2_norm(s2_sub(s2_mul(q[0], Z1Z1), rp->x));       // U2 - X1: (-3L, L) -> normalized
  const S2 S2v = s2_mul(q[1], s2_mul(Z1, Z1Z1));                  // Y2 Z1^3: sums (-3L, 2L) x 2L
  const S2 R = s2_norm(s2_mulk<2>(s2_sub(S2v, rp->y)));          // 2 (S2 - Y1): (-6L, 2L) -> normalized
  const S2 HH = s2_sqr(H);                                        // [0, L)
  rp->z = s2_norm(s2_sub(s2_sub(s2_sqr(s2_add(Z1, H)), Z1Z1), HH));  // (Z1 + H)^2 - Z1Z1 - HH: (-2L, L)
  const S2 J = s2_norm(s2_mulk<4>(s2_mul(H, HH)));                // J = H I = 4 H HH: 4 (-2L, L) -> normalized
  const S2 YJ = s2_mul(rp->y, J);                                 // (-2L, L)
  const S2 V = s2_norm(s2_mulk<4>(s2_mul(rp->x, HH)));            // V = X1 I = 4 X1 HH -> normalized
  const S2 X3 = s2_norm(s2_sub_k<2>(s2_sub(s2_sqr(R), J), V));    // r^2 - J - 2V: (-3L - 16, L + 16)
  rp->x = X3;
  rp->y = s2_norm(s2_sub_k<2>(s2_mul(R, s2_sub(V, X3)), YJ));     // (-2L, L) - 2 (-2L, L): (-4L, 5L)
}

GBV_HD S2 s2_neg(const S2& a) { return S2{s28_sub(S28{}, a.c0), s28_sub(S28{}, a.c1)}; }
GBV_HD S28 s28_sel(bool c, const S28& a, const S28& b) {
  S28 r;
#pragma unroll
  for (int i = 0; i < 14; ++i) r.v[i] = c ? a.v[i] : b.v[i];
  return r;
}
GBV_HD S2 s2_sel(bool c, const S2& a, const S2& b) { return S2{s28_sel(c, a.c0, b.c0), s28_sel(c, a.c1, b.c1)}; }

// sum_i 2^i (d_i S) for the signed digit pairs of (sa, sb) -- curve.h jac_mul_2d_signed_tab, the batch
// scalar r = a - b x^2 applied through the endomorphism -- on the lazy form: 31 doublings and 31 mixed
// additions of +-S1 or +-S2 (affine, canonical, not infinity; held in the S2 form, a digit's sign
// applied to y limbwise).  Same point as the canonical ladder; when Z = 0 mod p at the end (an addition
// met R = +-S, impossible for points of the prime-order subgroup) the canonical ladder recomputes it.
GBV_NI G2J g2_mul_2d_signed_lazy(G2A S1, G2A S2v, uint32_t sa, uint32_t sb) {
  const S2 t1x = s2_from(S1.x), t1y = s2_from(S1.y), t2x = s2_from(S2v.x), t2y = s2_from(S2v.y);
  S2 q[2];
  auto pick = [&](int i) {
    const bool s = (sa >> i) & 1u, t = (sb >> i) & 1u;
    q[0] = s2_sel(s == t, t1x, t2x);
    const S2 y = s2_sel(s == t, t1y, t2y);
    q[1] = s2_sel(s, y, s2_neg(y));
  };
  pick(31);
  S2J R{q[0], q[1], S2{s28_from_fp(FP_ONE), S28{}}};
#pragma nounroll
  for (int i = 30; i >= 0; --i) {
    R = s2j_dbl(R);
    pick(i);
    s2j_madd(&R, q);
  }
  G2J r = s2j_to(R);
  if (fp2_is_zero(r.z)) r = jac_mul_2d_signed(S1, S2v, sa, sb);
  return ret_copy(r);
}

// [|x|] q, |x| = 0xd201000000010000: the runs of doublings between its set bits (62, 60, 57, 48, 16) and
// the five mixed additions, all on the lazy form.  Same point as jac_mul_xabs(q): when Z = 0 mod p at the
// end (an addition met *r = +-q, possible only for points of small order outside G2) the canonical chain
// recomputes it.
GBV_NI G2J g2_mul_xabs_lazy(G2A q) {
  static_assert(X_ABS == 0xd201000000010000ull, "run lengths below follow |x|");
  const S2 qs[2] = {s2_from(q.x), s2_from(q.y)};
  S2J s{qs[0], qs[1], S2{s28_from_fp(FP_ONE), s28_from_fp(fp_zero())}};
  const int runs[5] = {1, 2, 3, 9, 32};  // doublings before each addition
#pragma nounroll
  for (int k = 0; k < 5; ++k) {
    s2j_dbl_n(&s, runs[k]);
    s2j_madd(&s, qs);
  }
  s2j_dbl_n(&s, 16);
  G2J r = s2j_to(s);
  if (fp2_is_zero(r.z)) r = g2_mul_xabs(q);
  return ret_copy(r);
}

}  // namespace gbv
