// G1 (y^2 = x^3 + 4 over Fp) and G2 (y^2 = x^3 + 4(1+i) over Fp2): Jacobian arithmetic
// (a = 0: dbl-2009-l, madd-2007-bl, add-2007-bl), ZCash decoding with blst's accept/reject rules,
// Scott's endomorphism subgroup tests, and 64-bit scalar multiplication.
#pragma once
#include "fp2.h"

namespace gbv {

// ---- overloads so the point code is written once for both fields --------------------------
GBV_HD Fp f_add(const Fp& a, const Fp& b) { return fp_add(a, b); }
GBV_HD Fp f_sub(const Fp& a, const Fp& b) { return fp_sub(a, b); }
GBV_HD Fp f_neg(const Fp& a) { return fp_neg(a); }
GBV_HD Fp f_dbl(const Fp& a) { return fp_dbl(a); }
GBV_HD Fp f_mul(const Fp& a, const Fp& b) { return fp_mul(a, b); }
GBV_HD Fp f_sqr(const Fp& a) { return fp_sqr(a); }
GBV_HD Fp f_add_lazy(const Fp& a, const Fp& b) { return fp_add_lazy(a, b); }  // feeds products only
GBV_HD bool f_is_zero(const Fp& a) { return fp_is_zero(a); }
GBV_HD bool f_eq(const Fp& a, const Fp& b) { return fp_eq(a, b); }
GBV_HD Fp f_sel(bool c, const Fp& a, const Fp& b) { return fp_sel(c, a, b); }
GBV_HD Fp f_inv(const Fp& a) { return fp_inv(a); }
GBV_HD void f_one(Fp& r) { r = FP_ONE; }
GBV_HD void f_zero(Fp& r) { r = fp_zero(); }

GBV_HD Fp2 f_add(const Fp2& a, const Fp2& b) { return fp2_add(a, b); }
GBV_HD Fp2 f_sub(const Fp2& a, const Fp2& b) { return fp2_sub(a, b); }
GBV_HD Fp2 f_neg(const Fp2& a) { return fp2_neg(a); }
GBV_HD Fp2 f_dbl(const Fp2& a) { return fp2_dbl(a); }
GBV_HD Fp2 f_mul(const Fp2& a, const Fp2& b) { return fp2_mul(a, b); }
GBV_HD Fp2 f_sqr(const Fp2& a) { return fp2_sqr(a); }
GBV_HD Fp2 f_add_lazy(const Fp2& a, const Fp2& b) { return fp2_add_lazy(a, b); }
GBV_HD bool f_is_zero(const Fp2& a) { return fp2_is_zero(a); }
GBV_HD bool f_eq(const Fp2& a, const Fp2& b) { return fp2_eq(a, b); }
GBV_HD Fp2 f_sel(bool c, const Fp2& a, const Fp2& b) { return fp2_sel(c, a, b); }
GBV_HD Fp2 f_inv(const Fp2& a) { return fp2_inv(a); }
GBV_HD void f_one(Fp2& r) { r = fp2_one(); }
GBV_HD void f_zero(Fp2& r) { r = fp2_zero(); }

template <class F> struct Jac { F x, y, z; };   // infinity <=> z == 0
template <class F> struct Aff { F x, y; };      // infinity tracked by the caller

using G1J = Jac<Fp>;
using G1A = Aff<Fp>;
using G2J = Jac<Fp2>;
using G2A = Aff<Fp2>;

template <class F> GBV_HD Jac<F> jac_infinity() {
  Jac<F> r;
  f_one(r.x);
  f_one(r.y);
  f_zero(r.z);
  return r;
}

template <class F> GBV_HD Jac<F> jac_from_aff(const Aff<F>& a) {
  Jac<F> r;
  r.x = a.x;
  r.y = a.y;
  f_one(r.z);
  return r;
}

template <class F> GBV_HD bool jac_is_inf(const Jac<F>& p) { return f_is_zero(p.z); }

template <class F> GBV_HD Jac<F> jac_sel(bool c, const Jac<F>& a, const Jac<F>& b) {
  return Jac<F>{f_sel(c, a.x, b.x), f_sel(c, a.y, b.y), f_sel(c, a.z, b.z)};
}

template <class F> GBV_HD Jac<F> jac_neg(const Jac<F>& p) { return Jac<F>{p.x, f_neg(p.y), p.z}; }

// dbl-2009-l, 2M + 5S.  Complete for a = 0 (2-torsion and infinity give z3 = 0).
// Z3 first so that Z dies early: over Fp2 the live set then stays at five elements (120 VGPRs)
// plus one product's operands, inside the registers an out-of-line Fp product leaves untouched.
template <class F> GBV_HD Jac<F> jac_dbl(const Jac<F>& p) {
  Jac<F> r;
  r.z = f_dbl(f_mul(p.y, p.z));
  F B = f_sqr(p.y);
  F A = f_sqr(p.x);
  F C = f_sqr(B);
  F D = f_dbl(f_sub(f_sub(f_sqr(f_add_lazy(p.x, B)), A), C));
  F E = f_add_lazy(f_add_lazy(A, A), A);  // < 3p: feeds the two products below only
  F Fv = f_sqr(E);
  r.x = f_sub(Fv, f_dbl(D));
  F C8 = f_dbl(f_dbl(f_dbl(C)));
  r.y = f_sub(f_mul(E, f_sub(D, r.x)), C8);
  return r;
}

// madd-2007-bl (q affine, not infinity), 7M + 4S, with the exceptional cases handled.
template <class F> GBV_HD Jac<F> jac_add_aff(const Jac<F>& p, const Aff<F>& q) {
  F Z1Z1 = f_sqr(p.z);
  F U2 = f_mul(q.x, Z1Z1);
  F S2 = f_mul(q.y, f_mul(p.z, Z1Z1));
  F H = f_sub(U2, p.x);
  F rr = f_dbl(f_sub(S2, p.y));
  bool p_inf = f_is_zero(p.z);
  if (f_is_zero(H) && !p_inf) {  // same x: doubling or inverse points (rare, divergent)
    if (f_is_zero(rr)) return jac_dbl(p);
    return jac_infinity<F>();
  }
  F HH = f_sqr(H);
  F I = f_dbl(f_dbl(HH));
  F J = f_mul(H, I);
  F V = f_mul(p.x, I);
  Jac<F> r;
  r.x = f_sub(f_sub(f_sqr(rr), J), f_dbl(V));
  r.y = f_sub(f_mul(rr, f_sub(V, r.x)), f_dbl(f_mul(p.y, J)));
  r.z = f_sub(f_sub(f_sqr(f_add_lazy(p.z, H)), Z1Z1), HH);
  return jac_sel(p_inf, jac_from_aff(q), r);
}

// add-2007-bl, 11M + 5S, complete via the same exceptional-case handling.
template <class F> GBV_HD Jac<F> jac_add(const Jac<F>& p, const Jac<F>& q) {
  bool p_inf = f_is_zero(p.z);
  bool q_inf = f_is_zero(q.z);
  F Z1Z1 = f_sqr(p.z);
  F Z2Z2 = f_sqr(q.z);
  F U1 = f_mul(p.x, Z2Z2);
  F U2 = f_mul(q.x, Z1Z1);
  F S1 = f_mul(p.y, f_mul(q.z, Z2Z2));
  F S2 = f_mul(q.y, f_mul(p.z, Z1Z1));
  F H = f_sub(U2, U1);
  F rr = f_dbl(f_sub(S2, S1));
  if (f_is_zero(H) && !p_inf && !q_inf) {
    if (f_is_zero(rr)) return jac_dbl(p);
    return jac_infinity<F>();
  }
  F I = f_sqr(f_dbl(H));
  F J = f_mul(H, I);
  F V = f_mul(U1, I);
  Jac<F> r;
  r.x = f_sub(f_sub(f_sqr(rr), J), f_dbl(V));
  r.y = f_sub(f_mul(rr, f_sub(V, r.x)), f_dbl(f_mul(S1, J)));
  r.z = f_mul(f_sub(f_sub(f_sqr(f_add(p.z, q.z)), Z1Z1), Z2Z2), H);
  r = jac_sel(q_inf, p, r);
  return jac_sel(p_inf, q, r);
}

// returns false for infinity
template <class F> GBV_HD bool jac_to_aff(Aff<F>& out, const Jac<F>& p) {
  F zi = f_inv(p.z);
  F zi2 = f_sqr(zi);
  out.x = f_mul(p.x, zi2);
  out.y = f_mul(p.y, f_mul(zi2, zi));
  return !f_is_zero(p.z);
}

// p == q (q affine, not infinity)?
template <class F> GBV_HD bool jac_eq_aff(const Jac<F>& p, const Aff<F>& q) {
  F z2 = f_sqr(p.z);
  bool ex = f_eq(p.x, f_mul(q.x, z2));
  bool ey = f_eq(p.y, f_mul(q.y, f_mul(z2, p.z)));
  return ex && ey && !f_is_zero(p.z);
}

// [k] q for a 64-bit k (left-to-right double-and-add, q affine, not infinity)
template <class F> GBV_HD Jac<F> jac_mul_u64(const Aff<F>& q, uint64_t k) {
  Jac<F> r = jac_infinity<F>();
  if (k == 0) return r;
  int top = 63;
  while (((k >> top) & 1ull) == 0) --top;
  r = jac_from_aff(q);
  for (int i = top - 1; i >= 0; --i) {
    r = jac_dbl(r);
    if ((k >> i) & 1ull) r = jac_add_aff(r, q);
  }
  return r;
}

// [k] q for a 256-bit scalar given as 8 little-endian words (utility signing / key derivation)
template <class F> GBV_HD Jac<F> jac_mul_u256(const Aff<F>& q, const uint32_t k[8]) {
  Jac<F> r = jac_infinity<F>();
  for (int i = 255; i >= 0; --i) {
    r = jac_dbl(r);
    if ((k[i >> 5] >> (i & 31)) & 1u) r = jac_add_aff(r, q);
  }
  return r;
}

// [|x|] q, |x| = 0xd201000000010000 (fixed public scalar: uniform control flow)
template <class F> GBV_HD Jac<F> jac_mul_xabs(const Aff<F>& q) {
  Jac<F> r = jac_from_aff(q);
  for (int i = 62; i >= 0; --i) {
    r = jac_dbl(r);
    if ((X_ABS >> i) & 1ull) r = jac_add_aff(r, q);
  }
  return r;
}

template <class F> GBV_HD Jac<F> jac_mul_xabs_jac(const Jac<F>& q) {
  Jac<F> r = q;
  for (int i = 62; i >= 0; --i) {
    r = jac_dbl(r);
    if ((X_ABS >> i) & 1ull) r = jac_add(r, q);
  }
  return r;
}

// An out-of-line function that returns a named aggregate builds it in the caller's return slot
// (NRVO), i.e. in memory: the loop-carried point of a scalar multiplication was stored in full
// after every step (288 B per G2 doubling -- ~18 KB of the ~22 KB/set of scratch writes of
// k_sm_prepare went to the 63 doublings of the G2 subgroup check).  ret_copy() keeps the loop
// variable an ordinary (register) local and writes the return slot once.
template <class T> GBV_HD T ret_copy(const T& v) {
  T out = v;
  return out;
}

// Out-of-line scalar multiplications (coarse: the point crosses the call once).
GBV_NI G1J g1_mul_u64(G1A q, uint64_t k) { G1J r = jac_mul_u64(q, k); return ret_copy(r); }
GBV_NI G2J g2_mul_u64(G2A q, uint64_t k) { G2J r = jac_mul_u64(q, k); return ret_copy(r); }
GBV_NI G2J g2_mul_xabs(G2A q) { G2J r = jac_mul_xabs(q); return ret_copy(r); }

GBV_NI G2J g2_mul_xabs_jac(G2J q) { G2J r = jac_mul_xabs_jac(q); return ret_copy(r); }
GBV_NI G1J g1_mul_u256(G1A q, const uint32_t* k) { G1J r = jac_mul_u256(q, k); return ret_copy(r); }
GBV_NI G2J g2_mul_u256(G2A q, const uint32_t* k) { G2J r = jac_mul_u256(q, k); return ret_copy(r); }

// ---- curve constants & decoding -------------------------------------------------------------
enum : uint8_t {
  PT_OK = 0,
  PT_BAD_ENCODING = 1,
  PT_NOT_ON_CURVE = 2,
  PT_NOT_IN_GROUP = 3,
  PT_INFINITY = 4,
};

GBV_HD bool bytes_zero(const uint8_t* b, int n) {
  uint32_t acc = 0;
  for (int i = 0; i < n; ++i) acc |= b[i];
  return acc == 0;
}

// blst POINTonE1_Uncompress_Z (PublicKey.fromBytes): 48 bytes -> affine (Montgomery).
// Returns PT_INFINITY for the canonical infinity encoding.
GBV_HD uint8_t g1_decompress(G1A& out, const uint8_t* in) {
  uint8_t in0 = in[0];
  if ((in0 & 0x80) == 0) return PT_BAD_ENCODING;
  if (in0 & 0x40) {
    if ((in0 & 0x3f) == 0 && bytes_zero(in + 1, 47)) return PT_INFINITY;
    return PT_BAD_ENCODING;
  }
  Fp xr = fp_load_be48(in, true);
  if (!fp_raw_is_canonical(xr)) return PT_BAD_ENCODING;
  Fp x = fp_to_mont(xr);
  Fp y2 = fp_add(fp_mul(fp_sqr(x), x), FP_B1);
  Fp y = fp_sqrt_candidate(y2);
  if (!fp_eq(fp_sqr(y), y2)) return PT_NOT_ON_CURVE;
  bool want_large = (in0 & 0x20) != 0;
  if (fp_is_lexi_large(y) != want_large) y = fp_neg(y);
  out.x = x;
  out.y = y;
  if (fp_is_zero(x)) return PT_NOT_IN_GROUP;
  return PT_OK;
}

GBV_HD void g1_compress(uint8_t* out, const G1A& a, bool inf) {
  if (inf) {
    out[0] = 0xc0;
    for (int i = 1; i < 48; ++i) out[i] = 0;
    return;
  }
  fp_store_be48(out, fp_from_mont(a.x));
  out[0] |= 0x80;
  if (fp_is_lexi_large(a.y)) out[0] |= 0x20;
}

GBV_HD bool g2_on_curve(const G2A& a) {
  Fp2 y2 = fp2_sqr(a.y);
  Fp2 rhs = fp2_add(fp2_mul(fp2_sqr(a.x), a.x), FP2_B2);
  return fp2_eq(y2, rhs);
}

// blst POINTonE2_Uncompress_Z (96 bytes) / POINTonE2_Deserialize_Z (192 bytes).
GBV_HD uint8_t g2_decode(G2A& out, const uint8_t* in, uint32_t len) {
  uint8_t in0 = in[0];
  if (len == 96) {
    if ((in0 & 0x80) == 0) return PT_BAD_ENCODING;
    if (in0 & 0x40) {
      if ((in0 & 0x3f) == 0 && bytes_zero(in + 1, 95)) return PT_INFINITY;
      return PT_BAD_ENCODING;
    }
    Fp x1r = fp_load_be48(in, true);
    Fp x0r = fp_load_be48(in + 48, false);
    if (!fp_raw_is_canonical(x1r) || !fp_raw_is_canonical(x0r)) return PT_BAD_ENCODING;
    Fp2 x{fp_to_mont(x0r), fp_to_mont(x1r)};
    Fp2 y2 = fp2_add(fp2_mul(fp2_sqr(x), x), FP2_B2);
    Fp2 y;
    if (!fp2_sqrt(y, y2)) return PT_NOT_ON_CURVE;
    bool want_large = (in0 & 0x20) != 0;
    if (fp2_is_lexi_large(y) != want_large) y = fp2_neg(y);
    out.x = x;
    out.y = y;
    if (fp2_is_zero(x)) return PT_NOT_IN_GROUP;
    return PT_OK;
  }
  if (len == 192) {
    if (in0 & 0x80) return PT_BAD_ENCODING;
    if (in0 & 0xe0) {
      if ((in0 & 0x40) && (in0 & 0x3f) == 0 && bytes_zero(in + 1, 191)) return PT_INFINITY;
      return PT_BAD_ENCODING;
    }
    Fp r[4];
    for (int i = 0; i < 4; ++i) {
      r[i] = fp_load_be48(in + 48 * i, false);
      if (!fp_raw_is_canonical(r[i])) return PT_BAD_ENCODING;
    }
    out.x = Fp2{fp_to_mont(r[1]), fp_to_mont(r[0])};
    out.y = Fp2{fp_to_mont(r[3]), fp_to_mont(r[2])};
    if (!g2_on_curve(out)) return PT_NOT_ON_CURVE;
    if (fp2_is_zero(out.x)) return PT_NOT_IN_GROUP;
    return PT_OK;
  }
  return PT_BAD_ENCODING;
}

GBV_HD void g2_compress(uint8_t* out, const G2A& a, bool inf) {
  if (inf) {
    out[0] = 0xc0;
    for (int i = 1; i < 96; ++i) out[i] = 0;
    return;
  }
  fp_store_be48(out, fp_from_mont(a.x.c1));
  fp_store_be48(out + 48, fp_from_mont(a.x.c0));
  out[0] |= 0x80;
  if (fp2_is_lexi_large(a.y)) out[0] |= 0x20;
}

// psi(x, y) = (conj(x) PSI_X, conj(y) PSI_Y)
GBV_HD G2A g2_psi(const G2A& a) {
  return G2A{fp2_mul(fp2_conj(a.x), PSI_X), fp2_mul(fp2_conj(a.y), PSI_Y)};
}

GBV_HD G2J g2_psi_jac(const G2J& a) {
  return G2J{fp2_mul(fp2_conj(a.x), PSI_X), fp2_mul(fp2_conj(a.y), PSI_Y), fp2_conj(a.z)};
}

// G1 membership (Scott 2021): (beta x, y) == [-x^2] P.  P affine, not infinity.
GBV_NI bool g1_in_subgroup(G1A p) {
  G1J t = jac_mul_xabs(p);           // [|x|] P
  t = jac_mul_xabs_jac(t);           // [x^2] P
  t = jac_neg(t);                    // [-x^2] P
  G1A phi{fp_mul(p.x, FP_BETA), p.y};
  return jac_eq_aff(t, phi);
}

// ---- randomised batch scalars (aggregateWithRandomness / verifyMultipleAggregateSignatures) ----
// The batch scalar of a set is r = a - b x^2 (mod r) with
//   a = sum_{i<32} (2 s_i - 1) 2^i,  b = sum_{i<32} (2 t_i - 1) 2^i   (s = bits 0..31, t = 32..63 of
// a random 64-bit word).  (a, b) -> r is injective (|a|, |b| < 2^32, x^2 ~ 2^127), so r takes 2^64
// distinct values: the same 2^-64 soundness bound as blst's 64-bit random scalars; only booleans
// are compared with the reference, never the scalars.  Both groups have a cheap endomorphism with
// eigenvalue -x^2:  G1: phi(x, y) = (beta x, y);  G2: -psi^2(x, y) = (c x, y)  (psi^2 = [x^2]).
// So r P = a P + b phi(P): a 32-step joint signed-digit ladder whose every digit pair adds one of
// +-(P + phi P), +-(P - phi P) -- no zero digits, so no lane of a wave idles on a skipped add.

// R = sum_i 2^i (d_i S) for the digit pairs of (sa, sb); S1 = P + E(P), S2 = P - E(P), affine.
template <class F> GBV_HD Jac<F> jac_mul_2d_signed(const Aff<F>& S1, const Aff<F>& S2, uint32_t sa, uint32_t sb) {
  auto pick = [&](int i) {
    bool s = (sa >> i) & 1u, t = (sb >> i) & 1u;
    Aff<F> T{f_sel(s == t, S1.x, S2.x), f_sel(s == t, S1.y, S2.y)};
    T.y = f_sel(s, T.y, f_neg(T.y));
    return T;
  };
  Jac<F> R = jac_from_aff(pick(31));
  for (int i = 30; i >= 0; --i) {
    R = jac_dbl(R);
    R = jac_add_aff(R, pick(i));
  }
  return R;
}

}  // namespace gbv
#include "g2_lazy.h"
namespace gbv {

// G2 membership (Scott 2021): psi(Q) == [x] Q = -[|x|] Q.  Q affine, not infinity.  [|x|] Q on the
// signed lazy 28-bit form (g2_lazy.h; the canonical chain g2_mul_xabs gives the same point).
#ifndef GBV_G2_LAZY
#define GBV_G2_LAZY 1  // 0: the canonical chain (A/B builds only, tools/build_variant.sh)
#endif
GBV_NI bool g2_in_subgroup(G2A q) {
  G2J xq = jac_neg(GBV_G2_LAZY ? g2_mul_xabs_lazy(q) : g2_mul_xabs(q));
  return jac_eq_aff(xq, g2_psi(q));
}

GBV_HD G1A g1_phi(const G1A& p) { return G1A{fp_mul(p.x, FP_BETA), p.y}; }
GBV_HD G2A g2_neg_psi2(const G2A& q) { return G2A{fp2_mul_fp(q.x, PSI2_C1), q.y}; }

template <class F> GBV_HD Aff<F> aff_from_jac_inv(const Jac<F>& p, const F& zinv) {
  F z2 = f_sqr(zinv);
  return Aff<F>{f_mul(p.x, z2), f_mul(p.y, f_mul(z2, zinv))};
}

// Ladder tables S1 = P + E(P), S2 = P - E(P) live in a per-lane table object: registers on the
// host / in the generic path, LDS in k_sm_prepare (the two affine G2 points are 96 VGPRs that
// would otherwise be spilled to scratch around every out-of-line Fp product of the ladder).
template <class A> struct RegTab2 {
  A t[2];
  GBV_HD A load(int k) const { return k ? t[1] : t[0]; }
  GBV_HD void store(int k, const A& a) { t[k] = a; }
};

template <class F, class Tab> GBV_HD Jac<F> jac_mul_2d_signed_tab(const Tab& tab, uint32_t sa, uint32_t sb) {
  auto pick = [&](int i) {
    bool s = (sa >> i) & 1u, t = (sb >> i) & 1u;
    Aff<F> T = tab.load(s == t ? 0 : 1);
    T.y = f_sel(s, T.y, f_neg(T.y));
    return T;
  };
  Jac<F> R = jac_from_aff(pick(31));
  for (int i = 30; i >= 0; --i) {
    R = jac_dbl(R);
    R = jac_add_aff(R, pick(i));
  }
  return R;
}

// [r] P and [r] Q for the same batch scalar r (digits r64).  The four ladder tables
// P +- phi(P), Q +- (-psi^2 Q) are made affine with ONE shared Fp inversion (Montgomery's trick
// over z1 z2 N(Z1 Z2)).  Returns false only for points of small order (P = +-phi(P) etc.), which
// subgroup-checked inputs never are; the caller then re-verifies that set unrandomised.
template <class Tab1, class Tab2> GBV_HD bool randomize_pair_tab(const G1A& P, const G2A& Q, uint64_t r64, G1J* rP, G2J* rQ, Tab1& t1,
                                                                 Tab2& t2) {
  G1A ph = g1_phi(P);
  G2A qh = g2_neg_psi2(Q);
  G1J a1 = jac_add_aff(jac_from_aff(P), ph);
  G1J a2 = jac_add_aff(jac_from_aff(P), G1A{ph.x, fp_neg(ph.y)});
  G2J b1 = jac_add_aff(jac_from_aff(Q), qh);
  G2J b2 = jac_add_aff(jac_from_aff(Q), G2A{qh.x, fp2_neg(qh.y)});
  Fp2 W = fp2_mul(b1.z, b2.z);
  Fp nW = fp_add(fp_sqr(W.c0), fp_sqr(W.c1));
  Fp u = fp_mul(a1.z, a2.z);
  Fp tot = fp_mul(u, nW);
  if (fp_is_zero(tot)) return false;
  Fp inv = fp_inv(tot);
  Fp inv_u = fp_mul(inv, nW);
  Fp inv_nW = fp_mul(inv, u);
  Fp2 Winv = fp2_mul_fp(fp2_conj(W), inv_nW);
  t1.store(0, aff_from_jac_inv(a1, fp_mul(a2.z, inv_u)));
  t1.store(1, aff_from_jac_inv(a2, fp_mul(a1.z, inv_u)));
  t2.store(0, aff_from_jac_inv(b1, fp2_mul(b2.z, Winv)));
  t2.store(1, aff_from_jac_inv(b2, fp2_mul(b1.z, Winv)));
  uint32_t sa = (uint32_t)r64, sb = (uint32_t)(r64 >> 32);
  *rP = jac_mul_2d_signed_tab<Fp>(t1, sa, sb);
  *rQ = GBV_G2_LAZY ? g2_mul_2d_signed_lazy(t2.load(0), t2.load(1), sa, sb) : jac_mul_2d_signed_tab<Fp2>(t2, sa, sb);
  return true;
}

GBV_NI bool randomize_pair(G1A P, G2A Q, uint64_t r64, G1J* rP, G2J* rQ) {
  RegTab2<G1A> t1;
  RegTab2<G2A> t2;
  return randomize_pair_tab(P, Q, r64, rP, rQ, t1, t2);
}

// randomize_pair with P in Jacobian coordinates (an aggregate pubkey straight from the gather-sum,
// never normalised): phi(X : Y : Z) = (beta X : Y : Z), so P +- phi(P) are two full additions and
// the tables are normalised by the same single shared inversion -- no inversion for P itself.
GBV_NI bool randomize_pair_jac(G1J P, G2A Q, uint64_t r64, G1J* rP, G2J* rQ) {
  G1J ph{fp_mul(P.x, FP_BETA), P.y, P.z};
  G2A qh = g2_neg_psi2(Q);
  G1J a1 = jac_add(P, ph);
  G1J a2 = jac_add(P, jac_neg(ph));
  G2J b1 = jac_add_aff(jac_from_aff(Q), qh);
  G2J b2 = jac_add_aff(jac_from_aff(Q), G2A{qh.x, fp2_neg(qh.y)});
  Fp2 W = fp2_mul(b1.z, b2.z);
  Fp nW = fp_add(fp_sqr(W.c0), fp_sqr(W.c1));
  Fp u = fp_mul(a1.z, a2.z);
  Fp tot = fp_mul(u, nW);
  if (fp_is_zero(tot)) return false;
  Fp inv = fp_inv(tot);
  Fp inv_u = fp_mul(inv, nW);
  Fp inv_nW = fp_mul(inv, u);
  Fp2 Winv = fp2_mul_fp(fp2_conj(W), inv_nW);
  RegTab2<G1A> t1;
  RegTab2<G2A> t2;
  t1.store(0, aff_from_jac_inv(a1, fp_mul(a2.z, inv_u)));
  t1.store(1, aff_from_jac_inv(a2, fp_mul(a1.z, inv_u)));
  t2.store(0, aff_from_jac_inv(b1, fp2_mul(b2.z, Winv)));
  t2.store(1, aff_from_jac_inv(b2, fp2_mul(b1.z, Winv)));
  uint32_t sa = (uint32_t)r64, sb = (uint32_t)(r64 >> 32);
  *rP = jac_mul_2d_signed_tab<Fp>(t1, sa, sb);
  *rQ = GBV_G2_LAZY ? g2_mul_2d_signed_lazy(t2.load(0), t2.load(1), sa, sb) : jac_mul_2d_signed_tab<Fp2>(t2, sa, sb);
  return true;
}

// [r] P in one group only (same r = a - b x^2 as randomize_pair): the same-message path's G1 term
// when the G2 sum of a large segment comes from the bucket MSM (k_msm.hip), and the G2 term when
// a failing segment needs its per-set r_i sig_i after all.  E(P) = phi(P) or -psi^2(P).
// the signed 2-D ladder over a two-entry table: G1 on the canonical form, G2 on the lazy form (g2_lazy.h)
template <class Tab> GBV_HD G1J mul_2d_tab(const Tab& t, const G1A*, uint32_t sa, uint32_t sb) { return jac_mul_2d_signed_tab<Fp>(t, sa, sb); }
template <class Tab> GBV_HD G2J mul_2d_tab(const Tab& t, const G2A*, uint32_t sa, uint32_t sb) {
  return GBV_G2_LAZY ? g2_mul_2d_signed_lazy(t.load(0), t.load(1), sa, sb) : jac_mul_2d_signed_tab<Fp2>(t, sa, sb);
}

template <class F> GBV_HD bool randomize_one(const Aff<F>& P, const Aff<F>& E, uint64_t r64, Jac<F>* rP) {
  Jac<F> a1 = jac_add_aff(jac_from_aff(P), E);
  Jac<F> a2 = jac_add_aff(jac_from_aff(P), Aff<F>{E.x, f_neg(E.y)});
  F z = f_mul(a1.z, a2.z);
  if (f_is_zero(z)) return false;
  F inv = f_inv(z);
  RegTab2<Aff<F>> t;
  t.store(0, aff_from_jac_inv(a1, f_mul(a2.z, inv)));
  t.store(1, aff_from_jac_inv(a2, f_mul(a1.z, inv)));
  *rP = mul_2d_tab(t, (const Aff<F>*)nullptr, (uint32_t)r64, (uint32_t)(r64 >> 32));
  return true;
}
GBV_NI bool randomize_g1(G1A P, uint64_t r64, G1J* rP) { return randomize_one<Fp>(P, g1_phi(P), r64, rP); }
GBV_NI bool randomize_g2(G2A Q, uint64_t r64, G2J* rQ) { return randomize_one<Fp2>(Q, g2_neg_psi2(Q), r64, rQ); }

// ---- per-validator comb tables for r pk (the same-message path's G1 term) ---------------------
// r P = a P + b phi(P) with the signed digits of randomize_pair (a_i = 2 s_i - 1, b_i = 2 t_i - 1,
// 32 each).  An 8-row comb over the 64 digits -- column i (0..7) holds digits 8j + i (j = 0..3) of
// a and of b --
//   r P = sum_{i<8} 2^i G_i,   G_i = sum_{j<4} 2^{8j} (a_{8j+i} P + b_{8j+i} phi(P)),
// so G_i is one of the 256 signed sums of the bases B = (P, 2^8 P, 2^16 P, 2^24 P, phi of those).
// The table keeps the 128 with a positive B_7 coefficient (the others are their negatives), affine:
// entry e has sign +B_b iff bit b of e is set (b < 7).  Evaluation is 7 doublings + 7 mixed
// additions (~126 Fp products) against the 31 + 31 ladder steps and table inversion of
// randomize_g1 (~593).  The table is built once per validator (k_comb_* in k_table.hip), 12 KB
// each: index2pubkey laid out for HBM capacity instead of recomputed per signature.
constexpr int COMB_ENTRIES = 128;
constexpr int COMB_U4 = 6;  // one entry: x, y limbs (96 bytes) = six 16-byte words

GBV_HD uint32_t comb_digits(uint32_t sa, uint32_t sb, int i) {
  uint32_t d = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    d |= ((sa >> (8 * j + i)) & 1u) << j;
    d |= ((sb >> (8 * j + i)) & 1u) << (4 + j);
  }
  return d;
}

GBV_HD G1A comb_entry_load(const uint4* p) {
  G1A a;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    uint4 x = p[q], y = p[3 + q];
    a.x.v[4 * q] = x.x, a.x.v[4 * q + 1] = x.y, a.x.v[4 * q + 2] = x.z, a.x.v[4 * q + 3] = x.w;
    a.y.v[4 * q] = y.x, a.y.v[4 * q + 1] = y.y, a.y.v[4 * q + 2] = y.z, a.y.v[4 * q + 3] = y.w;
  }
  return a;
}

GBV_HD void comb_entry_store(uint4* p, const G1A& a) {
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    p[q] = uint4{a.x.v[4 * q], a.x.v[4 * q + 1], a.x.v[4 * q + 2], a.x.v[4 * q + 3]};
    p[3 + q] = uint4{a.y.v[4 * q], a.y.v[4 * q + 1], a.y.v[4 * q + 2], a.y.v[4 * q + 3]};
  }
}

GBV_HD G1A comb_pick(const uint4* tab, uint32_t sa, uint32_t sb, int i) {
  const uint32_t d = comb_digits(sa, sb, i);
  const bool pos = (d >> 7) & 1u;
  G1A t = comb_entry_load(tab + COMB_U4 * ((pos ? d : ~d) & 127u));
  t.y = fp_sel(pos, t.y, fp_neg(t.y));
  return t;
}

// One comb column: R = 2 R + G_c.  Out of line, and the driver below is a plain sequence of calls:
// with the evaluation written as one loop, the gfx950 backend (ROCm 7.2) software-pipelines the
// next column's table loads across the loop back-edge and miscompiles the loop-carried 12-limb
// values (tests/test_gpu_scale.py::test_comb_tables_match_ladder caught it); a call per column
// keeps every load and its use inside one straight-line body.
// The running point stays in comb_mul's frame and each column updates it in place (one 192-byte
// store per column; by value it was an argument copy plus a returned copy).
GBV_NI void comb_step_to(G1J* R, const uint4* tab, uint32_t sa, uint32_t sb, int c) {
  const G1A t = comb_pick(tab, sa, sb, c);
  *R = jac_add_aff(jac_dbl(*R), t);
}

// [r] P from P's comb table (r = a - b x^2 of the digit word, exactly randomize_g1's scalar)
GBV_NI G1J comb_mul(const uint4* tab, uint32_t sa, uint32_t sb) {
  G1J R = jac_from_aff(comb_pick(tab, sa, sb, 7));
  comb_step_to(&R, tab, sa, sb, 6);
  comb_step_to(&R, tab, sa, sb, 5);
  comb_step_to(&R, tab, sa, sb, 4);
  comb_step_to(&R, tab, sa, sb, 3);
  comb_step_to(&R, tab, sa, sb, 2);
  comb_step_to(&R, tab, sa, sb, 1);
  comb_step_to(&R, tab, sa, sb, 0);
  return ret_copy(R);
}

// The comb bases B[0..7] (affine) and D = 2 P, with one shared inversion.  P affine, in G1.
GBV_HD void comb_bases(const G1A& P, G1A B[8], G1A& D) {
  G1J J[4];  // 2P, 2^8 P, 2^16 P, 2^24 P
  G1J t = jac_dbl(jac_from_aff(P));
  J[0] = t;
  for (int k = 1; k < 4; ++k) {
    for (int q = 0; q < (k == 1 ? 7 : 8); ++q) t = jac_dbl(t);
    J[k] = t;
  }
  Fp p01 = fp_mul(J[0].z, J[1].z), p012 = fp_mul(p01, J[2].z);
  Fp inv = fp_inv(fp_mul(p012, J[3].z));
  Fp i3 = fp_mul(inv, p012);
  inv = fp_mul(inv, J[3].z);  // (z0 z1 z2)^-1
  Fp i2 = fp_mul(inv, p01);
  inv = fp_mul(inv, J[2].z);  // (z0 z1)^-1
  Fp i1 = fp_mul(inv, J[0].z), i0 = fp_mul(inv, J[1].z);
  D = aff_from_jac_inv(J[0], i0);
  B[0] = P;
  B[1] = aff_from_jac_inv(J[1], i1);
  B[2] = aff_from_jac_inv(J[2], i2);
  B[3] = aff_from_jac_inv(J[3], i3);
  for (int j = 0; j < 4; ++j) B[4 + j] = g1_phi(B[j]);
}

// entry e of the table, Jacobian (bit b of e: sign of B_b for b < 7; B_7 positive)
GBV_HD G1J comb_entry_jac(const G1A B[8], uint32_t e) {
  G1J R = jac_from_aff(B[7]);
  for (int b = 6; b >= 0; --b) {
    G1A t = B[b];
    t.y = fp_sel((e >> b) & 1u, t.y, fp_neg(t.y));
    R = jac_add_aff(R, t);
  }
  return R;
}

// Batch-scalar halves for the bucket MSM: r P = a P + b E(P) with a = 2 sa - (2^32 - 1),
// b = 2 sb - (2^32 - 1) (odd, |a|, |b| < 2^32).  Returns |a| or |b| and the sign.
GBV_HD uint32_t scalar_half_mag(uint32_t s, bool* neg) {
  // 2s - (2^32-1) >= 0  <=>  s >= 2^31
  *neg = s < 0x80000000u;
  return *neg ? (0xffffffffu - 2u * s) : (2u * s - 0xffffffffu);
}

}  // namespace gbv

