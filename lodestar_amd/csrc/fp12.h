// Fp6 = Fp2[v]/(v^3 - xi), Fp12 = Fp6[w]/(w^2 - v), xi = 1 + i.
// Sparse line multiplication for the Miller loop and the final exponentiation
// (easy part by Frobenius, hard part by the x-chain 3(p^4-p^2+1)/r = (x-1)^2 (x+p)(x^2+p^2-1) + 3).
#pragma once
#include "fp2.h"

namespace gbv {

GBV_HD Fp6 fp6_zero() { return Fp6{fp2_zero(), fp2_zero(), fp2_zero()}; }
GBV_HD Fp6 fp6_one() { return Fp6{fp2_one(), fp2_zero(), fp2_zero()}; }
GBV_HD Fp6 fp6_add(const Fp6& a, const Fp6& b) { return Fp6{fp2_add(a.c0, b.c0), fp2_add(a.c1, b.c1), fp2_add(a.c2, b.c2)}; }
GBV_HD Fp6 fp6_sub(const Fp6& a, const Fp6& b) { return Fp6{fp2_sub(a.c0, b.c0), fp2_sub(a.c1, b.c1), fp2_sub(a.c2, b.c2)}; }
GBV_HD Fp6 fp6_neg(const Fp6& a) { return Fp6{fp2_neg(a.c0), fp2_neg(a.c1), fp2_neg(a.c2)}; }
GBV_HD bool fp6_eq(const Fp6& a, const Fp6& b) { return fp2_eq(a.c0, b.c0) && fp2_eq(a.c1, b.c1) && fp2_eq(a.c2, b.c2); }
// multiply by v: (c0, c1, c2) -> (xi c2, c0, c1)
GBV_HD Fp6 fp6_mul_v(const Fp6& a) { return Fp6{fp2_mul_xi(a.c2), a.c0, a.c1}; }

GBV_HD Fp6 fp6_mul(const Fp6& a, const Fp6& b) {
  Fp2 t0 = fp2_mul(a.c0, b.c0);
  Fp2 t1 = fp2_mul(a.c1, b.c1);
  Fp2 t2 = fp2_mul(a.c2, b.c2);
  Fp2 c0 = fp2_add(t0, fp2_mul_xi(fp2_sub(fp2_sub(fp2_mul(fp2_add(a.c1, a.c2), fp2_add(b.c1, b.c2)), t1), t2)));
  Fp2 c1 = fp2_add(fp2_sub(fp2_sub(fp2_mul(fp2_add(a.c0, a.c1), fp2_add(b.c0, b.c1)), t0), t1), fp2_mul_xi(t2));
  Fp2 c2 = fp2_add(fp2_sub(fp2_sub(fp2_mul(fp2_add(a.c0, a.c2), fp2_add(b.c0, b.c2)), t0), t2), t1);
  return Fp6{c0, c1, c2};
}

// (f0, f1, f2) * (a, b, 0)
GBV_HD Fp6 fp6_mul_by_01(const Fp6& f, const Fp2& a, const Fp2& b) {
  Fp2 t0 = fp2_mul(f.c0, a);
  Fp2 t1 = fp2_mul(f.c1, b);
  Fp2 c1 = fp2_sub(fp2_sub(fp2_mul(fp2_add(f.c0, f.c1), fp2_add(a, b)), t0), t1);
  Fp2 c0 = fp2_add(t0, fp2_mul_xi(fp2_mul(f.c2, b)));
  Fp2 c2 = fp2_add(t1, fp2_mul(f.c2, a));
  return Fp6{c0, c1, c2};
}

// (f0, f1, f2) * (0, c, 0) = (xi f2 c, f0 c, f1 c)
GBV_HD Fp6 fp6_mul_by_1(const Fp6& f, const Fp2& c) {
  return Fp6{fp2_mul_xi(fp2_mul(f.c2, c)), fp2_mul(f.c0, c), fp2_mul(f.c1, c)};
}

GBV_HD Fp6 fp6_inv(const Fp6& a) {
  Fp2 t0 = fp2_sub(fp2_sqr(a.c0), fp2_mul_xi(fp2_mul(a.c1, a.c2)));
  Fp2 t1 = fp2_sub(fp2_mul_xi(fp2_sqr(a.c2)), fp2_mul(a.c0, a.c1));
  Fp2 t2 = fp2_sub(fp2_sqr(a.c1), fp2_mul(a.c0, a.c2));
  Fp2 d = fp2_add(fp2_mul(a.c0, t0), fp2_mul_xi(fp2_add(fp2_mul(a.c2, t1), fp2_mul(a.c1, t2))));
  Fp2 di = fp2_inv(d);
  return Fp6{fp2_mul(t0, di), fp2_mul(t1, di), fp2_mul(t2, di)};
}

// ---- Fp12 ----------------------------------------------------------------------------------
// Miller-loop line: (c0 + c2 v) + (c3 v) w, coefficients at w^0, w^2, w^3
struct Line { Fp2 c0, c2, c3; };

GBV_HD Fp12 fp12_one() { return Fp12{fp6_one(), fp6_zero()}; }
GBV_HD bool fp12_eq(const Fp12& a, const Fp12& b) { return fp6_eq(a.c0, b.c0) && fp6_eq(a.c1, b.c1); }
GBV_HD bool fp12_is_one(const Fp12& a) { return fp12_eq(a, fp12_one()); }
GBV_HD Fp12 fp12_conj(const Fp12& a) { return Fp12{a.c0, fp6_neg(a.c1)}; }

// Out-of-line Fp12 operations take pointers and write through an output pointer (which may alias
// an input: every function reads what it needs before it writes).  An Fp12 is 144 VGPRs, so it
// lives in the caller's frame either way; passed by value, each call also copied its arguments
// and result through fresh frame slots, and the final exponentiation's frames alone reached
// 24 KB of scratch per lane.  The value-returning wrappers below keep call sites unchanged.
GBV_NI void fp12_mul_to(Fp12* r, const Fp12* a, const Fp12* b) {
  Fp6 t0 = fp6_mul(a->c0, b->c0);
  Fp6 t1 = fp6_mul(a->c1, b->c1);
  Fp6 c1 = fp6_sub(fp6_sub(fp6_mul(fp6_add(a->c0, a->c1), fp6_add(b->c0, b->c1)), t0), t1);
  r->c0 = fp6_add(t0, fp6_mul_v(t1));
  r->c1 = c1;
}

GBV_NI void fp12_sqr_to(Fp12* r, const Fp12* a) {
  Fp6 t = fp6_mul(a->c0, a->c1);
  Fp6 c0 = fp6_sub(fp6_sub(fp6_mul(fp6_add(a->c0, a->c1), fp6_add(a->c0, fp6_mul_v(a->c1))), t), fp6_mul_v(t));
  r->c0 = c0;
  r->c1 = fp6_add(t, t);
}

// f *= line, line = (c0 + c2 v) + (c3 v) w  (coefficients at w^0, w^2, w^3)
GBV_NI void fp12_mul_line_to(Fp12* f, const Line* l) {
  Fp6 a = fp6_mul_by_01(f->c0, l->c0, l->c2);
  Fp6 b = fp6_mul_by_1(f->c1, l->c3);
  Fp6 e = fp6_mul_by_01(fp6_add(f->c0, f->c1), l->c0, fp2_add(l->c2, l->c3));
  f->c1 = fp6_sub(fp6_sub(e, a), b);
  f->c0 = fp6_add(a, fp6_mul_v(b));
}

GBV_NI void fp12_inv_to(Fp12* r, const Fp12* a) {
  Fp6 d = fp6_sub(fp6_mul(a->c0, a->c0), fp6_mul_v(fp6_mul(a->c1, a->c1)));
  Fp6 di = fp6_inv(d);
  Fp6 c1 = fp6_neg(fp6_mul(a->c1, di));
  r->c0 = fp6_mul(a->c0, di);
  r->c1 = c1;
}

// Frobenius: every output coefficient depends on the same coefficient of the input only.
GBV_NI void fp12_frob_to(Fp12* r, const Fp12* a) {
  r->c0.c0 = fp2_conj(a->c0.c0);
  r->c0.c1 = fp2_mul(fp2_conj(a->c0.c1), FROB_V1);
  r->c0.c2 = fp2_mul(fp2_conj(a->c0.c2), FROB_V2);
  r->c1.c0 = fp2_mul(fp2_conj(a->c1.c0), FROB_W);
  r->c1.c1 = fp2_mul(fp2_conj(a->c1.c1), FROB_V1W);
  r->c1.c2 = fp2_mul(fp2_conj(a->c1.c2), FROB_V2W);
}

GBV_HD void fp12_conj_to(Fp12* r, const Fp12* a) {
  r->c0 = a->c0;
  r->c1 = fp6_neg(a->c1);
}

// Granger-Scott squaring for a in the cyclotomic subgroup (after the easy part of the final
// exponentiation): Fp12 = Fp4^3 over Fp4 = Fp2[y]/(y^2 - xi), y = w^3, so a^2 is three Fp4
// squarings -- 6 Fp2 products (18 Fp) instead of fp12_sqr's 12 (36 Fp).  Same formula as the
// coop engine's FP12_CYC_SQR program (tools/gen_coop.py f12cyc_sqr).
GBV_HD void fp4_sqr(Fp2& t0, Fp2& t1, const Fp2& x, const Fp2& y) {
  Fp2 tmp = fp2_mul(x, y);
  t0 = fp2_sub(fp2_sub(fp2_mul(fp2_add(x, y), fp2_add(fp2_mul_xi(y), x)), tmp), fp2_mul_xi(tmp));
  t1 = fp2_dbl(tmp);
}
GBV_HD Fp2 cyc_3t_minus_2z(const Fp2& t, const Fp2& z) { return fp2_add(fp2_dbl(fp2_sub(t, z)), t); }
GBV_HD Fp2 cyc_3t_plus_2z(const Fp2& t, const Fp2& z) { return fp2_add(fp2_dbl(fp2_add(t, z)), t); }
GBV_NI void fp12_cyc_sqr_to(Fp12* r, const Fp12* a) {
  // coefficient names of the Fp4 view: z0 = c0.c0, z4 = c0.c1, z3 = c0.c2, z2 = c1.c0, z1 = c1.c1, z5 = c1.c2
  Fp2 t0, t1, t2, t3, t4, t5;
  fp4_sqr(t0, t1, a->c0.c0, a->c1.c1);
  Fp2 n0 = cyc_3t_minus_2z(t0, a->c0.c0);
  Fp2 n1 = cyc_3t_plus_2z(t1, a->c1.c1);
  r->c0.c0 = n0;
  r->c1.c1 = n1;
  fp4_sqr(t2, t3, a->c1.c0, a->c0.c2);
  fp4_sqr(t4, t5, a->c0.c1, a->c1.c2);
  Fp2 n2 = cyc_3t_plus_2z(fp2_mul_xi(t5), a->c1.c0);
  Fp2 n3 = cyc_3t_minus_2z(t4, a->c0.c2);
  Fp2 n4 = cyc_3t_minus_2z(t2, a->c0.c1);
  Fp2 n5 = cyc_3t_plus_2z(t3, a->c1.c2);
  r->c1.c0 = n2;
  r->c0.c2 = n3;
  r->c0.c1 = n4;
  r->c1.c2 = n5;
}

// r = a^x (x < 0: a^|x| by cyclotomic squarings, then conjugate), a in the cyclotomic subgroup
GBV_NI void fp12_exp_x_to(Fp12* r, const Fp12* a) {
  Fp12 base = *a;
  Fp12 acc = base;
  for (int i = 62; i >= 0; --i) {
    fp12_cyc_sqr_to(&acc, &acc);
    if ((X_ABS >> i) & 1ull) fp12_mul_to(&acc, &acc, &base);
  }
  fp12_conj_to(r, &acc);
}

// r = f^(3 (p^12 - 1)/r).  Equal to 1 iff f^((p^12-1)/r) == 1 (gcd(3, r) = 1).
GBV_NI void final_exponentiation_to(Fp12* out, const Fp12* f) {
  Fp12 t, a, b, c;
  fp12_inv_to(&a, f);
  fp12_conj_to(&t, f);
  fp12_mul_to(&t, &t, &a);                              // t = f^(p^6 - 1)
  fp12_frob_to(&a, &t);
  fp12_frob_to(&a, &a);
  fp12_mul_to(&t, &a, &t);                              // t ^= (p^2 + 1): cyclotomic from here on
  fp12_exp_x_to(&a, &t);
  fp12_conj_to(&b, &t);
  fp12_mul_to(&a, &a, &b);                              // a = t^(x-1)
  fp12_exp_x_to(&b, &a);
  fp12_conj_to(&c, &a);
  fp12_mul_to(&a, &b, &c);                              // a = t^((x-1)^2)
  fp12_exp_x_to(&b, &a);
  fp12_frob_to(&c, &a);
  fp12_mul_to(&b, &b, &c);                              // b = a^(x+p)
  fp12_exp_x_to(&c, &b);
  fp12_exp_x_to(&c, &c);
  fp12_frob_to(&a, &b);
  fp12_frob_to(&a, &a);
  fp12_mul_to(&c, &c, &a);
  fp12_conj_to(&a, &b);
  fp12_mul_to(&c, &c, &a);                              // c = b^(x^2+p^2-1)
  fp12_cyc_sqr_to(&a, &t);
  fp12_mul_to(&a, &a, &t);                              // t^3
  fp12_mul_to(out, &c, &a);
}

// value-returning forms (the frame holds the result; no argument copies)
GBV_HD Fp12 fp12_mul(const Fp12& a, const Fp12& b) { Fp12 r; fp12_mul_to(&r, &a, &b); return r; }
GBV_HD Fp12 fp12_sqr(const Fp12& a) { Fp12 r; fp12_sqr_to(&r, &a); return r; }
GBV_HD Fp12 fp12_cyc_sqr(const Fp12& a) { Fp12 r; fp12_cyc_sqr_to(&r, &a); return r; }
GBV_HD Fp12 fp12_inv(const Fp12& a) { Fp12 r; fp12_inv_to(&r, &a); return r; }
GBV_HD Fp12 fp12_frob(const Fp12& a) { Fp12 r; fp12_frob_to(&r, &a); return r; }
GBV_HD Fp12 fp12_exp_x(const Fp12& a) { Fp12 r; fp12_exp_x_to(&r, &a); return r; }
GBV_HD Fp12 final_exponentiation(const Fp12& f) { Fp12 r; final_exponentiation_to(&r, &f); return r; }
GBV_HD Fp12 fp12_mul_line(const Fp12& f, const Fp2& c0, const Fp2& c2, const Fp2& c3) {
  Fp12 r = f;
  Line l{c0, c2, c3};
  fp12_mul_line_to(&r, &l);
  return r;
}

}  // namespace gbv
