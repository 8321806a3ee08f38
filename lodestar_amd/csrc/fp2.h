// Fp2 = Fp[i]/(i^2 + 1).  Karatsuba multiplication and complex squaring, inlined into the caller
// over the out-of-line Fp product (fp.h fp_mul); halvings and the twist constant by additions.
#pragma once
#include "fp.h"

namespace gbv {

GBV_HD Fp2 fp2_zero() { return Fp2{fp_zero(), fp_zero()}; }
GBV_HD Fp2 fp2_one() { return Fp2{FP_ONE, fp_zero()}; }
GBV_HD Fp2 fp2_make(const Fp& a, const Fp& b) { return Fp2{a, b}; }
GBV_HD bool fp2_is_zero(const Fp2& a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
GBV_HD bool fp2_eq(const Fp2& a, const Fp2& b) { return fp_eq(a.c0, b.c0) && fp_eq(a.c1, b.c1); }
GBV_HD Fp2 fp2_sel(bool c, const Fp2& a, const Fp2& b) { return Fp2{fp_sel(c, a.c0, b.c0), fp_sel(c, a.c1, b.c1)}; }
GBV_HD Fp2 fp2_add(const Fp2& a, const Fp2& b) { return Fp2{fp_add(a.c0, b.c0), fp_add(a.c1, b.c1)}; }
GBV_HD Fp2 fp2_sub(const Fp2& a, const Fp2& b) { return Fp2{fp_sub(a.c0, b.c0), fp_sub(a.c1, b.c1)}; }
GBV_HD Fp2 fp2_neg(const Fp2& a) { return Fp2{fp_neg(a.c0), fp_neg(a.c1)}; }
GBV_HD Fp2 fp2_dbl(const Fp2& a) { return Fp2{fp_dbl(a.c0), fp_dbl(a.c1)}; }
GBV_HD Fp2 fp2_conj(const Fp2& a) { return Fp2{a.c0, fp_neg(a.c1)}; }
// (a0 + a1 i)(1 + i) = (a0 - a1) + (a0 + a1) i
GBV_HD Fp2 fp2_mul_xi(const Fp2& a) { return Fp2{fp_sub(a.c0, a.c1), fp_add(a.c0, a.c1)}; }

// Karatsuba over out-of-line Fp products: the Fp2 layer is inlined into its caller and only the
// 70-VGPR Fp product is a call, so occupancy (not in-thread ILP) hides the mad latency.  (One call
// per Fp2 product with the three Fp products inline measured far slower: C2 21.3 -> 16.1 M, round 5.)
// Inputs may be lazy (components below 4 p, fp_add_lazy): the Karatsuba sums and the (a0 - a1)
// of the square are formed without reduction; outputs are canonical.
GBV_HD Fp2 fp2_mul(const Fp2& a, const Fp2& b) {
  Fp t0 = fp_mul(a.c0, b.c0);
  Fp t1 = fp_mul(a.c1, b.c1);
  Fp t2 = fp_mul(fp_add_lazy(a.c0, a.c1), fp_add_lazy(b.c0, b.c1));
  return Fp2{fp_sub(t0, t1), fp_sub(fp_sub(t2, t0), t1)};
}

GBV_HD Fp2 fp2_sqr(const Fp2& a) {
  Fp t0 = fp_mul(fp_add_lazy(a.c0, a.c1), fp_sub_lazy4(a.c0, a.c1));
  Fp t1 = fp_mul(a.c0, a.c1);
  return Fp2{t0, fp_dbl(t1)};
}

GBV_HD Fp2 fp2_add_lazy(const Fp2& a, const Fp2& b) { return Fp2{fp_add_lazy(a.c0, b.c0), fp_add_lazy(a.c1, b.c1)}; }
// a / 2 (canonical a): two halvings, no product
GBV_HD Fp2 fp2_half(const Fp2& a) { return Fp2{fp_half(a.c0), fp_half(a.c1)}; }
// 12 (1 + i) c = 3 b' c (b' = 4 (1 + i), the twist's constant) by additions, no product
GBV_HD Fp2 fp2_mul_3b(const Fp2& c) {
  Fp2 x = fp2_mul_xi(c);
  Fp2 x4 = fp2_dbl(fp2_dbl(x));
  return fp2_add(fp2_dbl(x4), x4);
}


GBV_HD Fp2 fp2_mul_fp(const Fp2& a, const Fp& s) { return Fp2{fp_mul(a.c0, s), fp_mul(a.c1, s)}; }

GBV_HD Fp2 fp2_inv(const Fp2& a) {
  Fp n = fp_add(fp_sqr(a.c0), fp_sqr(a.c1));
  Fp ni = fp_inv(n);
  return Fp2{fp_mul(a.c0, ni), fp_neg(fp_mul(a.c1, ni))};
}

// RFC 9380 sgn0 for Fp2 (canonical values)
GBV_HD uint32_t fp2_sgn0(const Fp2& a) {
  Fp c0 = fp_from_mont(a.c0);
  Fp c1 = fp_from_mont(a.c1);
  uint32_t sign0 = c0.v[0] & 1u;
  uint32_t zero0 = fp_is_zero(c0) ? 1u : 0u;
  uint32_t sign1 = c1.v[0] & 1u;
  return sign0 | (zero0 & sign1);
}

// ZCash "lexicographically largest" (c1 first, then c0) -- blst sgn0_pty_mod_384x sign bit.
GBV_HD bool fp2_is_lexi_large(const Fp2& a) {
  bool c1_zero = fp_is_zero(a.c1);
  bool l1 = fp_is_lexi_large(a.c1);
  bool l0 = fp_is_lexi_large(a.c0);
  return c1_zero ? l0 : l1;
}

// Square root in Fp2 with uniform cost (two Fp exponentiations, no data-dependent branch):
//   alpha = sqrt(a0^2 + a1^2);  delta = (a0 + alpha)/2 (or (a0 - alpha)/2 if that is 0);
//   t = delta^((p-3)/4);  x0 = t*delta;  if x0*t == 1: root = (x0, a1 t / 2) else (-a1 t / 2, x0).
// Returns true iff a is a square (root^2 == a).  Prototype: tests/test_algorithm_prototypes.py.
// fp2_sqrt_with_norm_root is the second half, for callers that already hold a square root alpha
// (either sign) of the norm a0^2 + a1^2.
GBV_HD bool fp2_sqrt_with_norm_root(Fp2& root, const Fp2& a, const Fp& alpha) {
  Fp delta = fp_half(fp_add(a.c0, alpha));
  Fp delta2 = fp_half(fp_sub(a.c0, alpha));
  delta = fp_sel(fp_is_zero(delta), delta2, delta);
  Fp t = fp_pow_sched(delta, SCHED_SQRT_M3_NSQ, SCHED_SQRT_M3_IDX, SCHED_SQRT_M3_STEPS);
  Fp x0 = fp_mul(t, delta);
  bool qr = fp_eq(fp_mul(x0, t), FP_ONE);
  Fp h = fp_half(fp_mul(a.c1, t));
  root.c0 = fp_sel(qr, x0, fp_neg(h));
  root.c1 = fp_sel(qr, h, x0);
  return fp2_eq(fp2_sqr(root), a);
}

GBV_HD Fp fp2_norm(const Fp2& a) { return fp_add(fp_sqr(a.c0), fp_sqr(a.c1)); }

GBV_HD bool fp2_sqrt(Fp2& root, const Fp2& a) {
  Fp alpha = fp_pow_sched(fp2_norm(a), SCHED_SQRT_NSQ, SCHED_SQRT_IDX, SCHED_SQRT_STEPS);
  return fp2_sqrt_with_norm_root(root, a, alpha);
}

// Frobenius / psi helpers -------------------------------------------------------------------
GBV_HD Fp2 fp2_frob(const Fp2& a) { return fp2_conj(a); }

}  // namespace gbv
