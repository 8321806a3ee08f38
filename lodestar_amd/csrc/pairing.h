// Optimal-ate Miller loop over |x| = 0xd201000000010000 with T in homogeneous projective
// coordinates on the twist, sparse lines (w^0, w^2, w^3), conjugation for x < 0.
// Formulas and line shapes follow tests/test_algorithm_prototypes.py (dbl_step / add_step),
// which checks them against the oracle's affine pairing.
#pragma once
#include "fp12.h"
#include "curve.h"

namespace gbv {

struct G2Proj { Fp2 x, y, z; };

// Doubling step; P given as (-xP, yP).  The halvings and 3 b' C by additions: 27 Fp products.
GBV_HD Line dbl_step(G2Proj& T, const Fp& neg_xP, const Fp& yP) {
  Fp2 A = fp2_half(fp2_mul(T.x, T.y));
  Fp2 B = fp2_sqr(T.y);
  Fp2 C = fp2_sqr(T.z);
  Fp2 E = fp2_mul_3b(C);
  Fp2 F = fp2_add(fp2_dbl(E), E);
  Fp2 X3 = fp2_mul(A, fp2_sub(B, F));
  Fp2 G = fp2_half(fp2_add(B, F));
  Fp2 E2 = fp2_sqr(E);
  Fp2 Y3 = fp2_sub(fp2_sqr(G), fp2_add(fp2_dbl(E2), E2));
  Fp2 H = fp2_sub(fp2_sqr(fp2_add(T.y, T.z)), fp2_add(B, C));
  Fp2 Z3 = fp2_mul(B, H);
  Fp2 X2 = fp2_sqr(T.x);
  Line l;
  l.c0 = fp2_sub(B, E);
  l.c2 = fp2_mul_fp(fp2_add(fp2_dbl(X2), X2), neg_xP);
  l.c3 = fp2_mul_fp(H, yP);
  T.x = X3;
  T.y = Y3;
  T.z = Z3;
  return l;
}

// Mixed addition step T += Q (Q affine)
GBV_HD Line add_step(G2Proj& T, const G2A& Q, const Fp& neg_xP, const Fp& yP) {
  Fp2 theta = fp2_sub(T.y, fp2_mul(Q.y, T.z));
  Fp2 lam = fp2_sub(T.x, fp2_mul(Q.x, T.z));
  Fp2 C = fp2_sqr(theta);
  Fp2 D = fp2_sqr(lam);
  Fp2 E = fp2_mul(D, lam);
  Fp2 F = fp2_mul(T.z, C);
  Fp2 G = fp2_mul(T.x, D);
  Fp2 H = fp2_sub(fp2_add(E, F), fp2_dbl(G));
  Fp2 X3 = fp2_mul(lam, H);
  Fp2 Y3 = fp2_sub(fp2_mul(theta, fp2_sub(G, H)), fp2_mul(T.y, E));
  Fp2 Z3 = fp2_mul(T.z, E);
  Line l;
  l.c0 = fp2_sub(fp2_mul(theta, Q.x), fp2_mul(lam, Q.y));
  l.c2 = fp2_mul_fp(theta, neg_xP);
  l.c3 = fp2_mul_fp(lam, yP);
  T.x = X3;
  T.y = Y3;
  T.z = Z3;
  return l;
}

// The accumulator f lives in the frame and is updated in place through the pointer-taking Fp12
// calls (fp12.h); the two G2 points T_j stay in VGPRs.

// prod_{j<2} f_{|x|, Q_j}(P_j), conjugated.  A pair whose P or Q is infinity contributes 1.
GBV_NI void miller_loop_2_to(Fp12* out, G1A P0, bool inf0, G2A Q0, G1A P1, bool inf1, G2A Q1) {
  Fp nx0 = fp_neg(P0.x), nx1 = fp_neg(P1.x);
  G2Proj T0{Q0.x, Q0.y, fp2_one()};
  G2Proj T1{Q1.x, Q1.y, fp2_one()};
  Fp12 f = fp12_one();
  Line l;
  for (int i = 62; i >= 0; --i) {
    if (i != 62) fp12_sqr_to(&f, &f);
    l = dbl_step(T0, nx0, P0.y);
    if (!inf0) fp12_mul_line_to(&f, &l);
    l = dbl_step(T1, nx1, P1.y);
    if (!inf1) fp12_mul_line_to(&f, &l);
    if ((X_ABS >> i) & 1ull) {
      l = add_step(T0, Q0, nx0, P0.y);
      if (!inf0) fp12_mul_line_to(&f, &l);
      l = add_step(T1, Q1, nx1, P1.y);
      if (!inf1) fp12_mul_line_to(&f, &l);
    }
  }
  fp12_conj_to(out, &f);
}

// single pair
GBV_NI void miller_loop_1_to(Fp12* out, G1A P0, G2A Q0) {
  Fp nx0 = fp_neg(P0.x);
  G2Proj T0{Q0.x, Q0.y, fp2_one()};
  Fp12 f = fp12_one();
  Line l;
  for (int i = 62; i >= 0; --i) {
    if (i != 62) fp12_sqr_to(&f, &f);
    l = dbl_step(T0, nx0, P0.y);
    fp12_mul_line_to(&f, &l);
    if ((X_ABS >> i) & 1ull) {
      l = add_step(T0, Q0, nx0, P0.y);
      fp12_mul_line_to(&f, &l);
    }
  }
  fp12_conj_to(out, &f);
}

// single pair with P in Jacobian coordinates (X : Y : Z), Z != 0: every line is the affine line
// times Z^3 (c0 * Z^3, c2 from -X Z, c3 from Y), an Fp factor the final exponentiation removes,
// so no inversion is needed to get P affine.
GBV_NI void miller_loop_1j_to(Fp12* out, G1J P, G2A Q0) {
  Fp z2 = fp_sqr(P.z);
  Fp z3 = fp_mul(z2, P.z);
  Fp nxz = fp_neg(fp_mul(P.x, P.z));
  G2Proj T0{Q0.x, Q0.y, fp2_one()};
  Fp12 f = fp12_one();
  Line l;
  for (int i = 62; i >= 0; --i) {
    l = dbl_step(T0, nxz, P.y);
    l.c0 = fp2_mul_fp(l.c0, z3);
    if (i != 62) fp12_sqr_to(&f, &f);
    fp12_mul_line_to(&f, &l);
    if ((X_ABS >> i) & 1ull) {
      l = add_step(T0, Q0, nxz, P.y);
      l.c0 = fp2_mul_fp(l.c0, z3);
      fp12_mul_line_to(&f, &l);
    }
  }
  fp12_conj_to(out, &f);
}

GBV_HD Fp12 miller_loop_2(const G1A& P0, bool inf0, const G2A& Q0, const G1A& P1, bool inf1, const G2A& Q1) {
  Fp12 r;
  miller_loop_2_to(&r, P0, inf0, Q0, P1, inf1, Q1);
  return r;
}
GBV_HD Fp12 miller_loop_1(const G1A& P0, const G2A& Q0) { Fp12 r; miller_loop_1_to(&r, P0, Q0); return r; }
GBV_HD Fp12 miller_loop_1j(const G1J& P, const G2A& Q0) { Fp12 r; miller_loop_1j_to(&r, P, Q0); return r; }

// e(P0, Q0) * e(P1, Q1) == 1 ?
GBV_HD bool pairing_check_2(const G1A& P0, bool inf0, const G2A& Q0, const G1A& P1, bool inf1, const G2A& Q1) {
  Fp12 f;
  miller_loop_2_to(&f, P0, inf0, Q0, P1, inf1, Q1);
  final_exponentiation_to(&f, &f);
  return fp12_is_one(f);
}

GBV_HD G1A g1_neg_generator() { return G1A{G1_GEN_X, G1_GEN_NEG_Y}; }

}  // namespace gbv
