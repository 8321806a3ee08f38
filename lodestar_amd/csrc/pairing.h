// Optimal-ate Miller loop over |x| = 0xd201000000010000 with T in homogeneous projective
// coordinates on the twist, sparse lines (w^0, w^2, w^3), conjugation for x < 0.
// Formulas and line shapes follow tests/test_algorithm_prototypes.py (dbl_step / add_step),
// which checks them against the oracle's affine pairing.
#pragma once
#include "fp12.h"
#include "curve.h"

namespace gbv {

struct G2Proj { Fp2 x, y, z; };

struct Line { Fp2 c0, c2, c3; };

// Doubling step; P given as (-xP, yP)
GBV_HD Line dbl_step(G2Proj& T, const Fp& neg_xP, const Fp& yP) {
  Fp2 A = fp2_mul_fp(fp2_mul(T.x, T.y), FP_INV2);
  Fp2 B = fp2_sqr(T.y);
  Fp2 C = fp2_sqr(T.z);
  Fp2 E = fp2_mul(C, FP2_3B2);
  Fp2 F = fp2_add(fp2_dbl(E), E);
  Fp2 X3 = fp2_mul(A, fp2_sub(B, F));
  Fp2 G = fp2_mul_fp(fp2_add(B, F), FP_INV2);
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

// prod_{j<2} f_{|x|, Q_j}(P_j), conjugated.  A pair whose P or Q is infinity contributes 1.
GBV_NI Fp12 miller_loop_2(G1A P0, bool inf0, G2A Q0, G1A P1, bool inf1, G2A Q1) {
  Fp nx0 = fp_neg(P0.x), nx1 = fp_neg(P1.x);
  G2Proj T0{Q0.x, Q0.y, fp2_one()};
  G2Proj T1{Q1.x, Q1.y, fp2_one()};
  Fp12 f = fp12_one();
  for (int i = 62; i >= 0; --i) {
    if (i != 62) f = fp12_sqr(f);
    Line l0 = dbl_step(T0, nx0, P0.y);
    if (!inf0) f = fp12_mul_line(f, l0.c0, l0.c2, l0.c3);
    Line l1 = dbl_step(T1, nx1, P1.y);
    if (!inf1) f = fp12_mul_line(f, l1.c0, l1.c2, l1.c3);
    if ((X_ABS >> i) & 1ull) {
      l0 = add_step(T0, Q0, nx0, P0.y);
      if (!inf0) f = fp12_mul_line(f, l0.c0, l0.c2, l0.c3);
      l1 = add_step(T1, Q1, nx1, P1.y);
      if (!inf1) f = fp12_mul_line(f, l1.c0, l1.c2, l1.c3);
    }
  }
  return fp12_conj(f);
}

// single pair
GBV_NI Fp12 miller_loop_1(G1A P0, G2A Q0) {
  Fp nx0 = fp_neg(P0.x);
  G2Proj T0{Q0.x, Q0.y, fp2_one()};
  Fp12 f = fp12_one();
  for (int i = 62; i >= 0; --i) {
    if (i != 62) f = fp12_sqr(f);
    Line l0 = dbl_step(T0, nx0, P0.y);
    f = fp12_mul_line(f, l0.c0, l0.c2, l0.c3);
    if ((X_ABS >> i) & 1ull) {
      l0 = add_step(T0, Q0, nx0, P0.y);
      f = fp12_mul_line(f, l0.c0, l0.c2, l0.c3);
    }
  }
  return fp12_conj(f);
}

// single pair with P in Jacobian coordinates (X : Y : Z), Z != 0: every line is the affine line
// times Z^3 (c0 * Z^3, c2 from -X Z, c3 from Y), an Fp factor the final exponentiation removes,
// so no inversion is needed to get P affine.
GBV_NI Fp12 miller_loop_1j(G1J P, G2A Q0) {
  Fp z2 = fp_sqr(P.z);
  Fp z3 = fp_mul(z2, P.z);
  Fp nxz = fp_neg(fp_mul(P.x, P.z));
  G2Proj T0{Q0.x, Q0.y, fp2_one()};
  Fp12 f = fp12_one();
  for (int i = 62; i >= 0; --i) {
    if (i != 62) f = fp12_sqr(f);
    Line l0 = dbl_step(T0, nxz, P.y);
    f = fp12_mul_line(f, fp2_mul_fp(l0.c0, z3), l0.c2, l0.c3);
    if ((X_ABS >> i) & 1ull) {
      l0 = add_step(T0, Q0, nxz, P.y);
      f = fp12_mul_line(f, fp2_mul_fp(l0.c0, z3), l0.c2, l0.c3);
    }
  }
  return fp12_conj(f);
}

// e(P0, Q0) * e(P1, Q1) == 1 ?
GBV_HD bool pairing_check_2(const G1A& P0, bool inf0, const G2A& Q0, const G1A& P1, bool inf1, const G2A& Q1) {
  Fp12 f = miller_loop_2(P0, inf0, Q0, P1, inf1, Q1);
  return fp12_is_one(final_exponentiation(f));
}

GBV_HD G1A g1_neg_generator() { return G1A{G1_GEN_X, G1_GEN_NEG_Y}; }

}  // namespace gbv
