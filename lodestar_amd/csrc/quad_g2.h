// G2 point arithmetic on a lane quad (quad.h's product rounds): one point, the same on the four lanes
// of a DPP quad, each step a few rounds of four Fp products (lane j runs product j of the round and
// the four results are broadcast by quad_perm moves).  For the per-set G2 chains of small passes --
// hash_to_G2's cofactor clearing, the signature's subgroup check, r_i sig_i -- whose thread form
// leaves most of the chip idle on a range-sync segment.
//   doubling (dbl-2009-l, 2M + 5S = 16 products)           4 rounds   (16 products on one lane)
//   mixed addition (madd-2007-bl, 7M + 4S = 29 products)   9 rounds
//   addition (add-2007-bl, 11M + 5S = 43 products)        11 rounds
// Same formulas and exceptional-case handling as curve.h's jac_dbl / jac_add_aff / jac_add (branches
// on values every lane of the quad holds alike, so a quad never diverges), hence the same Jacobian
// triples bit for bit.
#pragma once
#include "curve.h"
#include "quad.h"

namespace gbv {
namespace quad {

#define QLZA fp_add_lazy
#define QLZS fp_sub_lazy4
#define R4(...) round4(r, q, __VA_ARGS__)

__device__ __forceinline__ G2J g2_dbl(const G2J& p, uint32_t q) {
  const Fp2 &x = p.x, &y = p.y, &z = p.z;
  Fp r[4];
  R4(QLZA(y.c0, y.c1), QLZS(y.c0, y.c1), y.c0, y.c1, QLZA(x.c0, x.c1), QLZS(x.c0, x.c1), x.c0, x.c1);
  const Fp2 B = sq(r[0], r[1]), A = sq(r[2], r[3]);
  const Fp2 E = fp2_add(fp2_dbl(A), A), u = fp2_add(x, B);
  R4(QLZA(B.c0, B.c1), QLZS(B.c0, B.c1), B.c0, B.c1, QLZA(u.c0, u.c1), QLZS(u.c0, u.c1), u.c0, u.c1);
  const Fp2 C = sq(r[0], r[1]), U2 = sq(r[2], r[3]);
  R4(QLZA(E.c0, E.c1), QLZS(E.c0, E.c1), E.c0, E.c1, y.c0, z.c0, y.c1, z.c1);
  const Fp2 F = sq(r[0], r[1]);
  const Fp yz0 = r[2], yz1 = r[3];
  const Fp2 D = fp2_dbl(fp2_sub(fp2_sub(U2, A), C));
  G2J o;
  o.x = fp2_sub(F, fp2_dbl(D));
  const Fp2 W = fp2_sub(D, o.x);
  R4(QLZA(y.c0, y.c1), QLZA(z.c0, z.c1), E.c0, W.c0, E.c1, W.c1, QLZA(E.c0, E.c1), QLZA(W.c0, W.c1));
  o.z = fp2_dbl(kara(yz0, yz1, r[0]));
  o.y = fp2_sub(kara(r[1], r[2], r[3]), fp2_dbl(fp2_dbl(fp2_dbl(C))));
  return o;
}

// p + a (a affine, not infinity), madd-2007-bl with jac_add_aff's exceptional cases
__device__ __forceinline__ G2J g2_madd(const G2J& p, const G2A& a, uint32_t q) {
  const Fp2 &x1 = p.x, &y1 = p.y, &z1 = p.z;
  const Fp zero = fp_zero();
  Fp r[4];
  R4(QLZA(z1.c0, z1.c1), QLZS(z1.c0, z1.c1), z1.c0, z1.c1, zero, zero, zero, zero);
  const Fp2 ZZ = sq(r[0], r[1]);
  // U2 = x2 ZZ, T = z1 ZZ
  R4(a.x.c0, ZZ.c0, a.x.c1, ZZ.c1, QLZA(a.x.c0, a.x.c1), QLZA(ZZ.c0, ZZ.c1), z1.c0, ZZ.c0);
  const Fp2 U2 = kara(r[0], r[1], r[2]);
  const Fp t0 = r[3];
  const Fp2 H = fp2_sub(U2, x1);
  R4(z1.c1, ZZ.c1, QLZA(z1.c0, z1.c1), QLZA(ZZ.c0, ZZ.c1), QLZA(H.c0, H.c1), QLZS(H.c0, H.c1), H.c0, H.c1);
  const Fp2 T = kara(t0, r[0], r[1]), HH = sq(r[2], r[3]);
  // S2 = y2 T, (z1 + H)^2
  const Fp2 zH = fp2_add(z1, H);
  R4(a.y.c0, T.c0, a.y.c1, T.c1, QLZA(a.y.c0, a.y.c1), QLZA(T.c0, T.c1), QLZA(zH.c0, zH.c1), QLZS(zH.c0, zH.c1));
  const Fp2 S2 = kara(r[0], r[1], r[2]);
  const Fp zh0 = r[3];
  const Fp2 rr = fp2_dbl(fp2_sub(S2, y1));
  const bool p_inf = fp2_is_zero(z1);
  if (fp2_is_zero(H) && !p_inf) {  // same x: doubling or inverse points (rare; quad-uniform)
    if (fp2_is_zero(rr)) return g2_dbl(p, q);
    return jac_infinity<Fp2>();
  }
  const Fp2 I = fp2_dbl(fp2_dbl(HH));
  R4(zH.c0, zH.c1, QLZA(rr.c0, rr.c1), QLZS(rr.c0, rr.c1), rr.c0, rr.c1, H.c0, I.c0);
  const Fp2 ZH2 = sq(zh0, r[0]), R2 = sq(r[1], r[2]);
  const Fp j0 = r[3];
  R4(H.c1, I.c1, QLZA(H.c0, H.c1), QLZA(I.c0, I.c1), x1.c0, I.c0, x1.c1, I.c1);
  const Fp2 J = kara(j0, r[0], r[1]);
  const Fp v0 = r[2], v1 = r[3];
  R4(QLZA(x1.c0, x1.c1), QLZA(I.c0, I.c1), y1.c0, J.c0, y1.c1, J.c1, QLZA(y1.c0, y1.c1), QLZA(J.c0, J.c1));
  const Fp2 V = kara(v0, v1, r[0]), YJ = kara(r[1], r[2], r[3]);
  G2J o;
  o.x = fp2_sub(fp2_sub(R2, J), fp2_dbl(V));
  const Fp2 W = fp2_sub(V, o.x);
  R4(rr.c0, W.c0, rr.c1, W.c1, QLZA(rr.c0, rr.c1), QLZA(W.c0, W.c1), zero, zero);
  o.y = fp2_sub(kara(r[0], r[1], r[2]), fp2_dbl(YJ));
  o.z = fp2_sub(fp2_sub(ZH2, ZZ), HH);
  return jac_sel(p_inf, jac_from_aff(a), o);
}

// p + a (both Jacobian), add-2007-bl with jac_add's exceptional cases
__device__ __forceinline__ G2J g2_add(const G2J& p, const G2J& a, uint32_t q) {
  const Fp2 &x1 = p.x, &y1 = p.y, &z1 = p.z, &x2 = a.x, &y2 = a.y, &z2 = a.z;
  const bool p_inf = fp2_is_zero(z1), a_inf = fp2_is_zero(z2);
  const Fp zero = fp_zero();
  Fp r[4];
  R4(QLZA(z1.c0, z1.c1), QLZS(z1.c0, z1.c1), z1.c0, z1.c1, QLZA(z2.c0, z2.c1), QLZS(z2.c0, z2.c1), z2.c0, z2.c1);
  const Fp2 Z1Z1 = sq(r[0], r[1]), Z2Z2 = sq(r[2], r[3]);
  // U1 = x1 Z2Z2, U2 = x2 Z1Z1, T2 = z2 Z2Z2, T1 = z1 Z1Z1
  R4(x1.c0, Z2Z2.c0, x1.c1, Z2Z2.c1, QLZA(x1.c0, x1.c1), QLZA(Z2Z2.c0, Z2Z2.c1), x2.c0, Z1Z1.c0);
  const Fp2 U1 = kara(r[0], r[1], r[2]);
  const Fp u20 = r[3];
  R4(x2.c1, Z1Z1.c1, QLZA(x2.c0, x2.c1), QLZA(Z1Z1.c0, Z1Z1.c1), z2.c0, Z2Z2.c0, z2.c1, Z2Z2.c1);
  const Fp2 U2 = kara(u20, r[0], r[1]);
  const Fp t20 = r[2], t21 = r[3];
  R4(QLZA(z2.c0, z2.c1), QLZA(Z2Z2.c0, Z2Z2.c1), z1.c0, Z1Z1.c0, z1.c1, Z1Z1.c1, QLZA(z1.c0, z1.c1), QLZA(Z1Z1.c0, Z1Z1.c1));
  const Fp2 T2 = kara(t20, t21, r[0]), T1 = kara(r[1], r[2], r[3]);
  const Fp2 H = fp2_sub(U2, U1), H2 = fp2_dbl(H);
  // S1 = y1 T2, S2 = y2 T1, I = (2H)^2
  R4(y1.c0, T2.c0, y1.c1, T2.c1, QLZA(y1.c0, y1.c1), QLZA(T2.c0, T2.c1), y2.c0, T1.c0);
  const Fp2 S1 = kara(r[0], r[1], r[2]);
  const Fp s20 = r[3];
  R4(y2.c1, T1.c1, QLZA(y2.c0, y2.c1), QLZA(T1.c0, T1.c1), QLZA(H2.c0, H2.c1), QLZS(H2.c0, H2.c1), H2.c0, H2.c1);
  const Fp2 S2 = kara(s20, r[0], r[1]), I = sq(r[2], r[3]);
  const Fp2 rr = fp2_dbl(fp2_sub(S2, S1));
  if (fp2_is_zero(H) && !p_inf && !a_inf) {  // quad-uniform, rare
    if (fp2_is_zero(rr)) return g2_dbl(p, q);
    return jac_infinity<Fp2>();
  }
  // rr^2, J = H I, V = U1 I
  R4(QLZA(rr.c0, rr.c1), QLZS(rr.c0, rr.c1), rr.c0, rr.c1, H.c0, I.c0, H.c1, I.c1);
  const Fp2 R2 = sq(r[0], r[1]);
  const Fp j0 = r[2], j1 = r[3];
  R4(QLZA(H.c0, H.c1), QLZA(I.c0, I.c1), U1.c0, I.c0, U1.c1, I.c1, QLZA(U1.c0, U1.c1), QLZA(I.c0, I.c1));
  const Fp2 J = kara(j0, j1, r[0]), V = kara(r[1], r[2], r[3]);
  G2J o;
  o.x = fp2_sub(fp2_sub(R2, J), fp2_dbl(V));
  const Fp2 W = fp2_sub(V, o.x);
  // rr W, S1 J, (z1 + z2)^2
  const Fp2 zs = fp2_add(z1, z2);
  R4(rr.c0, W.c0, rr.c1, W.c1, QLZA(rr.c0, rr.c1), QLZA(W.c0, W.c1), S1.c0, J.c0);
  const Fp2 RW = kara(r[0], r[1], r[2]);
  const Fp sj0 = r[3];
  R4(S1.c1, J.c1, QLZA(S1.c0, S1.c1), QLZA(J.c0, J.c1), QLZA(zs.c0, zs.c1), QLZS(zs.c0, zs.c1), zs.c0, zs.c1);
  o.y = fp2_sub(RW, fp2_dbl(kara(sj0, r[0], r[1])));
  const Fp2 K = fp2_sub(fp2_sub(sq(r[2], r[3]), Z1Z1), Z2Z2);
  R4(K.c0, H.c0, K.c1, H.c1, QLZA(K.c0, K.c1), QLZA(H.c0, H.c1), zero, zero);
  o.z = kara(r[0], r[1], r[2]);
  o = jac_sel(a_inf, p, o);
  return jac_sel(p_inf, a, o);
}

// psi(X : Y : Z) = (conj(X) PSI_X : conj(Y) PSI_Y : conj(Z)); PSI_X = k i, so conj(X) PSI_X = (X1 k, X0 k)
__device__ __forceinline__ G2J g2_psi(const G2J& p, uint32_t q) {
  const Fp zero = fp_zero();
  const Fp k = PSI_X.c1;
  const Fp2 yc = fp2_conj(p.y);
  Fp r[4];
  R4(p.x.c1, k, p.x.c0, k, yc.c0, PSI_Y.c0, yc.c1, PSI_Y.c1);
  G2J o;
  o.x = Fp2{r[0], r[1]};
  const Fp y0 = r[2], y1 = r[3];
  R4(QLZA(yc.c0, yc.c1), QLZA(PSI_Y.c0, PSI_Y.c1), zero, zero, zero, zero, zero, zero);
  o.y = kara(y0, y1, r[0]);
  o.z = fp2_conj(p.z);
  return o;
}

// [|x|] p (p Jacobian): curve.h jac_mul_xabs_jac
__device__ __noinline__ G2J g2_mul_xabs_jac(G2J p, uint32_t q) {
  G2J r = p;
  for (int i = 62; i >= 0; --i) {
    r = g2_dbl(r, q);
    if ((X_ABS >> i) & 1ull) r = g2_add(r, p, q);
  }
  return r;
}

// [|x|] a (a affine): curve.h jac_mul_xabs
__device__ __noinline__ G2J g2_mul_xabs(G2A a, uint32_t q) {
  G2J r = jac_from_aff(a);
  for (int i = 62; i >= 0; --i) {
    r = g2_dbl(r, q);
    if ((X_ABS >> i) & 1ull) r = g2_madd(r, a, q);
  }
  return r;
}

// RFC 9380 G.3 clear_cofactor, as hash_to_curve.h clear_cofactor_g2
__device__ __noinline__ G2J g2_clear_cofactor(G2J p, uint32_t q) {
  const G2J t1 = jac_neg(g2_mul_xabs_jac(p, q));        // [x] P
  G2J t2 = g2_psi(p, q);                                 // psi(P)
  G2J t3 = g2_psi(g2_psi(g2_dbl(p, q), q), q);           // psi^2(2P)
  t3 = g2_add(t3, jac_neg(t2), q);
  t2 = g2_add(t1, t2, q);
  t2 = jac_neg(g2_mul_xabs_jac(t2, q));                  // [x] t2
  t3 = g2_add(t3, t2, q);
  t3 = g2_add(t3, jac_neg(t1), q);
  return g2_add(t3, jac_neg(p), q);
}

// p == a (a affine, not infinity): curve.h jac_eq_aff
__device__ __forceinline__ bool g2_eq_aff(const G2J& p, const G2A& a, uint32_t q) {
  const Fp zero = fp_zero();
  const Fp2& z = p.z;
  Fp r[4];
  R4(QLZA(z.c0, z.c1), QLZS(z.c0, z.c1), z.c0, z.c1, zero, zero, zero, zero);
  const Fp2 z2 = sq(r[0], r[1]);
  R4(a.x.c0, z2.c0, a.x.c1, z2.c1, QLZA(a.x.c0, a.x.c1), QLZA(z2.c0, z2.c1), z2.c0, z.c0);
  const bool ex = fp2_eq(p.x, kara(r[0], r[1], r[2]));
  const Fp w0 = r[3];
  R4(z2.c1, z.c1, QLZA(z2.c0, z2.c1), QLZA(z.c0, z.c1), zero, zero, zero, zero);
  const Fp2 z3 = kara(w0, r[0], r[1]);
  R4(a.y.c0, z3.c0, a.y.c1, z3.c1, QLZA(a.y.c0, a.y.c1), QLZA(z3.c0, z3.c1), zero, zero);
  const bool ey = fp2_eq(p.y, kara(r[0], r[1], r[2]));
  return ex && ey && !fp2_is_zero(z);
}

// G2 membership (curve.h g2_in_subgroup): psi(Q) == -[|x|] Q
__device__ __forceinline__ bool g2_in_subgroup(const G2A& a, uint32_t q) {
  return g2_eq_aff(jac_neg(g2_mul_xabs(a, q)), gbv::g2_psi(a), q);
}

// affine form (curve.h jac_to_aff; the Fp inversion on every lane, the products on the quad)
__device__ __forceinline__ bool g2_to_aff(G2A& out, const G2J& p, uint32_t q) {
  const Fp zero = fp_zero();
  const Fp2& z = p.z;
  Fp r[4];
  R4(z.c0, z.c0, z.c1, z.c1, zero, zero, zero, zero);
  const Fp ni = fp_inv(fp_add(r[0], r[1]));
  R4(z.c0, ni, z.c1, ni, zero, zero, zero, zero);
  const Fp2 zi{r[0], fp_neg(r[1])};
  R4(QLZA(zi.c0, zi.c1), QLZS(zi.c0, zi.c1), zi.c0, zi.c1, zero, zero, zero, zero);
  const Fp2 zi2 = sq(r[0], r[1]);
  R4(zi2.c0, zi.c0, zi2.c1, zi.c1, QLZA(zi2.c0, zi2.c1), QLZA(zi.c0, zi.c1), p.x.c0, zi2.c0);
  const Fp2 zi3 = kara(r[0], r[1], r[2]);
  const Fp x0 = r[3];
  R4(p.x.c1, zi2.c1, QLZA(p.x.c0, p.x.c1), QLZA(zi2.c0, zi2.c1), p.y.c0, zi3.c0, p.y.c1, zi3.c1);
  out.x = kara(x0, r[0], r[1]);
  const Fp y0 = r[2], y1 = r[3];
  R4(QLZA(p.y.c0, p.y.c1), QLZA(zi3.c0, zi3.c1), zero, zero, zero, zero, zero, zero);
  out.y = kara(y0, y1, r[0]);
  return !fp2_is_zero(z);
}

// randomize_g2 (curve.h randomize_one with E = -psi^2): r Q = a Q + b E(Q) by the signed-digit ladder
// over the affine tables Q + E(Q), Q - E(Q).  Returns false for the small-order cases.
__device__ __noinline__ bool g2_randomize(G2A Q, uint64_t r64, G2J* out, uint32_t qd) {
  const uint32_t q = qd;
  const G2A E = g2_neg_psi2(Q);
  const G2J a1 = g2_madd(jac_from_aff(Q), E, q);
  const G2J a2 = g2_madd(jac_from_aff(Q), G2A{E.x, fp2_neg(E.y)}, q);
  const Fp zero = fp_zero();
  Fp r[4];
  // z = a1.z a2.z, its inverse, then each table point's z^-1 = (other z) z^-1
  R4(a1.z.c0, a2.z.c0, a1.z.c1, a2.z.c1, QLZA(a1.z.c0, a1.z.c1), QLZA(a2.z.c0, a2.z.c1), zero, zero);
  const Fp2 z = kara(r[0], r[1], r[2]);
  if (fp2_is_zero(z)) return false;
  R4(z.c0, z.c0, z.c1, z.c1, zero, zero, zero, zero);
  const Fp ni = fp_inv(fp_add(r[0], r[1]));
  R4(z.c0, ni, z.c1, ni, zero, zero, zero, zero);
  const Fp2 zinv{r[0], fp_neg(r[1])};
  R4(a2.z.c0, zinv.c0, a2.z.c1, zinv.c1, QLZA(a2.z.c0, a2.z.c1), QLZA(zinv.c0, zinv.c1), a1.z.c0, zinv.c0);
  const Fp2 i1 = kara(r[0], r[1], r[2]);
  const Fp w0 = r[3];
  R4(a1.z.c1, zinv.c1, QLZA(a1.z.c0, a1.z.c1), QLZA(zinv.c0, zinv.c1), QLZA(i1.c0, i1.c1), QLZS(i1.c0, i1.c1), i1.c0, i1.c1);
  const Fp2 i2 = kara(w0, r[0], r[1]);
  const Fp2 i1s = sq(r[2], r[3]);
  // table point k: (x i_k^2, y i_k^3)
  R4(QLZA(i2.c0, i2.c1), QLZS(i2.c0, i2.c1), i2.c0, i2.c1, i1s.c0, i1.c0, i1s.c1, i1.c1);
  const Fp2 i2s = sq(r[0], r[1]);
  const Fp c0 = r[2], c1 = r[3];
  R4(QLZA(i1s.c0, i1s.c1), QLZA(i1.c0, i1.c1), i2s.c0, i2.c0, i2s.c1, i2.c1, QLZA(i2s.c0, i2s.c1), QLZA(i2.c0, i2.c1));
  const Fp2 i1c = kara(c0, c1, r[0]), i2c = kara(r[1], r[2], r[3]);
  G2A t[2];
  R4(a1.x.c0, i1s.c0, a1.x.c1, i1s.c1, QLZA(a1.x.c0, a1.x.c1), QLZA(i1s.c0, i1s.c1), a1.y.c0, i1c.c0);
  t[0].x = kara(r[0], r[1], r[2]);
  const Fp e0 = r[3];
  R4(a1.y.c1, i1c.c1, QLZA(a1.y.c0, a1.y.c1), QLZA(i1c.c0, i1c.c1), a2.x.c0, i2s.c0, a2.x.c1, i2s.c1);
  t[0].y = kara(e0, r[0], r[1]);
  const Fp f0 = r[2], f1 = r[3];
  R4(QLZA(a2.x.c0, a2.x.c1), QLZA(i2s.c0, i2s.c1), a2.y.c0, i2c.c0, a2.y.c1, i2c.c1, QLZA(a2.y.c0, a2.y.c1), QLZA(i2c.c0, i2c.c1));
  t[1].x = kara(f0, f1, r[0]);
  t[1].y = kara(r[1], r[2], r[3]);
  const uint32_t sa = (uint32_t)r64, sb = (uint32_t)(r64 >> 32);
  auto pick = [&](int i) {
    const bool s = (sa >> i) & 1u, u = (sb >> i) & 1u;
    G2A T{fp2_sel(s == u, t[0].x, t[1].x), fp2_sel(s == u, t[0].y, t[1].y)};
    T.y = fp2_sel(s, T.y, fp2_neg(T.y));
    return T;
  };
  G2J R = jac_from_aff(pick(31));
  for (int i = 30; i >= 0; --i) {
    R = g2_dbl(R, q);
    R = g2_madd(R, pick(i), q);
  }
  *out = R;
  return true;
}

// ---- G1 (Fp coordinates): the same formulas, products one Fp each ----------------------------------
__device__ __forceinline__ G1J g1_dbl(const G1J& p, uint32_t q) {
  const Fp zero = fp_zero();
  Fp r[4];
  R4(p.y, p.y, p.x, p.x, zero, zero, zero, zero);
  const Fp B = r[0], A = r[1];
  const Fp E = fp_add(fp_dbl(A), A), u = fp_add(p.x, B);
  R4(B, B, u, u, E, E, zero, zero);
  const Fp C = r[0], F = r[2];
  const Fp D = fp_dbl(fp_sub(fp_sub(r[1], A), C));
  G1J o;
  o.x = fp_sub(F, fp_dbl(D));
  R4(E, fp_sub(D, o.x), p.y, p.z, zero, zero, zero, zero);
  o.y = fp_sub(r[0], fp_dbl(fp_dbl(fp_dbl(C))));
  o.z = fp_dbl(r[1]);
  return o;
}

__device__ __forceinline__ G1J g1_madd(const G1J& p, const G1A& a, uint32_t q) {
  const Fp zero = fp_zero();
  Fp r[4];
  R4(p.z, p.z, zero, zero, zero, zero, zero, zero);
  const Fp ZZ = r[0];
  R4(a.x, ZZ, p.z, ZZ, zero, zero, zero, zero);
  const Fp H = fp_sub(r[0], p.x), T = r[1];
  const Fp zH = fp_add(p.z, H);
  R4(a.y, T, H, H, zH, zH, zero, zero);
  const Fp HH = r[1], ZH2 = r[2];
  const Fp rr = fp_dbl(fp_sub(r[0], p.y));
  const bool p_inf = fp_is_zero(p.z);
  if (fp_is_zero(H) && !p_inf) {  // quad-uniform, rare
    if (fp_is_zero(rr)) return g1_dbl(p, q);
    return jac_infinity<Fp>();
  }
  const Fp I = fp_dbl(fp_dbl(HH));
  R4(rr, rr, H, I, p.x, I, zero, zero);
  const Fp J = r[1], V = r[2];
  G1J o;
  o.x = fp_sub(fp_sub(r[0], J), fp_dbl(V));
  R4(rr, fp_sub(V, o.x), p.y, J, zero, zero, zero, zero);
  o.y = fp_sub(r[0], fp_dbl(r[1]));
  o.z = fp_sub(fp_sub(ZH2, ZZ), HH);
  return jac_sel(p_inf, jac_from_aff(a), o);
}

// randomize_g1 (curve.h randomize_one with E = phi): the same ladder as g2_randomize over G1
__device__ __noinline__ bool g1_randomize(G1A P, uint64_t r64, G1J* out, uint32_t qd) {
  const uint32_t q = qd;
  const G1A E = g1_phi(P);
  const G1J a1 = g1_madd(jac_from_aff(P), E, q);
  const G1J a2 = g1_madd(jac_from_aff(P), G1A{E.x, fp_neg(E.y)}, q);
  const Fp zero = fp_zero();
  Fp r[4];
  R4(a1.z, a2.z, zero, zero, zero, zero, zero, zero);
  if (fp_is_zero(r[0])) return false;
  const Fp inv = fp_inv(r[0]);
  R4(a2.z, inv, a1.z, inv, zero, zero, zero, zero);
  const Fp i1 = r[0], i2 = r[1];
  R4(i1, i1, i2, i2, zero, zero, zero, zero);
  const Fp s1 = r[0], s2 = r[1];
  R4(s1, i1, s2, i2, a1.x, s1, a2.x, s2);
  G1A t[2];
  t[0].x = r[2];
  t[1].x = r[3];
  R4(a1.y, r[0], a2.y, r[1], zero, zero, zero, zero);
  t[0].y = r[0];
  t[1].y = r[1];
  const uint32_t sa = (uint32_t)r64, sb = (uint32_t)(r64 >> 32);
  auto pick = [&](int i) {
    const bool s = (sa >> i) & 1u, u = (sb >> i) & 1u;
    G1A T{fp_sel(s == u, t[0].x, t[1].x), fp_sel(s == u, t[0].y, t[1].y)};
    T.y = fp_sel(s, T.y, fp_neg(T.y));
    return T;
  };
  G1J R = jac_from_aff(pick(31));
  for (int i = 30; i >= 0; --i) {
    R = g1_dbl(R, q);
    R = g1_madd(R, pick(i), q);
  }
  *out = R;
  return true;
}

#undef R4
#undef QLZA
#undef QLZS

}  // namespace quad
}  // namespace gbv
