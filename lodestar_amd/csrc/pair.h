// Lane-pair Miller loop: one signature set's f_{|x|, Q}(P) on TWO lanes (2j, 2j+1) of a wave.
//
// The thread-per-set Miller loop (pairing.h miller_loop_1j_to) keeps a 576-byte Fp12 accumulator,
// the G2 point T and the line in one lane: ~370 live dwords, so the accumulator lives in scratch and
// every Fp12 step streams it through memory (775 KB of HBM traffic per set measured).
// Here lane h of the pair owns one Fp6 half of f = c0 + c1 w (h = 0: c0, h = 1: c1) and every step
// is split into rounds of Fp products with per-lane operands -- the same instruction stream on both
// lanes, operands picked by v_cndmask -- and partial results cross the pair by one DPP quad_perm
// swap per dword (no LDS, no memory):
//   f^2        lane 0: t = c0 c1, lane 1: u = (c0 + c1)(c0 + v c1); c0' = u - t - v t, c1' = 2 t
//              (one Fp6 product per lane: 18 Fp products instead of 36 in a row)
//   f * line   line = A + B w, A = (l0, l2, 0), B = (0, l3, 0); lane h forms c_h A (15) and c_h B (9);
//              c0' = c0 A + v c1 B, c1' = c0 B + c1 A (24 per lane instead of 39 in a row)
//   doubling   27 Fp products in two rounds (6 + 8 per lane), 3b' C and the halvings by additions
//   addition   43 Fp products in four rounds (3 + 7 + 6 + 6 per lane)
// Per loop: ~3.76 k product rounds per lane instead of 7.24 k products in one lane, i.e. twice the
// lanes for about half the latency and a quarter of the live state per lane.  Formulas: the same
// dbl_step / add_step as pairing.h (tests/test_algorithm_prototypes.py checks them against the
// oracle); P Jacobian, lines scaled by Z^3 (removed by the final exponentiation).
#pragma once
#include "pairing.h"

namespace gbv {

#if defined(__HIP_DEVICE_COMPILE__)
// swap with the other lane of the pair: DPP quad_perm [1,0,3,2]
__device__ __forceinline__ uint32_t pair_swap_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true);
}
#else
__device__ inline uint32_t pair_swap_u32(uint32_t v) { return v; }  // host pass: parsed, never emitted
#endif

__device__ __forceinline__ Fp pswap(const Fp& a) {
  Fp r;
#pragma unroll
  for (int i = 0; i < 12; ++i) r.v[i] = pair_swap_u32(a.v[i]);
  return r;
}
__device__ __forceinline__ Fp2 pswap(const Fp2& a) { return Fp2{pswap(a.c0), pswap(a.c1)}; }
__device__ __forceinline__ Fp6 pswap(const Fp6& a) { return Fp6{pswap(a.c0), pswap(a.c1), pswap(a.c2)}; }

// one product per lane: lane 0 (h = false) a0 b0, lane 1 a1 b1
__device__ __forceinline__ Fp pm(bool h, const Fp& a0, const Fp& b0, const Fp& a1, const Fp& b1) {
  return fp_mul(fp_sel(h, a1, a0), fp_sel(h, b1, b0));
}
__device__ __forceinline__ Fp6 fp6_sel(bool c, const Fp6& a, const Fp6& b) {
  return Fp6{fp2_sel(c, a.c0, b.c0), fp2_sel(c, a.c1, b.c1), fp2_sel(c, a.c2, b.c2)};
}
// Karatsuba recombination of (a0 b0, a1 b1, (a0 + a1)(b0 + b1))
__device__ __forceinline__ Fp2 kara(const Fp& t0, const Fp& t1, const Fp& t2) { return Fp2{fp_sub(t0, t1), fp_sub(fp_sub(t2, t0), t1)}; }
#define LZA fp_add_lazy
#define LZS fp_sub_lazy4

struct PairT { Fp2 x, y, z; };  // T in homogeneous projective coordinates, the same on both lanes
struct PairP { Fp nxz, y, z3; };  // P = (X : Y : Z) Jacobian: -X Z, Y, Z^3, the same on both lanes

// f <- f^2 (M = this lane's half of f)
__device__ __forceinline__ void pair_sqr(Fp6& M, bool h) {
  Fp6 O = pswap(M);
  // lane 0 (M = c0, O = c1): X = c0, Y = c1.  lane 1 (M = c1, O = c0): X = c0 + c1, Y = c0 + v c1.
  Fp6 X = fp6_sel(h, fp6_add(O, M), M);
  Fp6 Y = fp6_sel(h, fp6_add(O, fp6_mul_v(M)), O);
  Fp6 R = fp6_mul(X, Y);
  Fp6 Ro = pswap(R);
  // lane 0: c0' = u - t - v t with t = R, u = Ro; lane 1: c1' = 2 t with t = Ro
  M = fp6_sel(h, fp6_add(Ro, Ro), fp6_sub(Ro, fp6_add(R, fp6_mul_v(R))));
}

// f <- f * (A + B w), A = (l0, l2, 0), B = (0, l3, 0)
__device__ __forceinline__ void pair_mul_line(Fp6& M, const Line& l, bool h) {
  Fp6 X1 = fp6_mul_by_01(M, l.c0, l.c2);  // c_h A
  Fp6 X2 = fp6_mul_by_1(M, l.c3);         // c_h B
  Fp6 X2o = pswap(X2);                    // lane 0: c1 B, lane 1: c0 B
  M = fp6_add(X1, fp6_sel(h, X2o, fp6_mul_v(X2o)));
}

// Doubling step T <- 2T and its line through P (dbl_step, pairing.h), on the pair.
__device__ __forceinline__ Line pair_dbl(PairT& T, const PairP& P, bool h) {
  const Fp2 &x = T.x, &y = T.y, &z = T.z;
  const Fp2 s = fp2_add(y, z);
  // round 1 -- lane 0: x^2 (2), x y (3), one spare; lane 1: y^2 (2), z^2 (2), (y + z)^2 (2)
  Fp k0 = pm(h, LZA(x.c0, x.c1), LZS(x.c0, x.c1), LZA(y.c0, y.c1), LZS(y.c0, y.c1));
  Fp k1 = pm(h, x.c0, x.c1, y.c0, y.c1);
  Fp k2 = pm(h, x.c0, y.c0, LZA(s.c0, s.c1), LZS(s.c0, s.c1));
  Fp k3 = pm(h, x.c1, y.c1, s.c0, s.c1);
  Fp k4 = pm(h, LZA(x.c0, x.c1), LZA(y.c0, y.c1), LZA(z.c0, z.c1), LZS(z.c0, z.c1));
  Fp k5 = pm(h, x.c0, x.c0, z.c0, z.c1);
  // lane 0: X2 = (k0, 2 k1), xy = kara(k2, k3, k4); lane 1: B = (k0, 2 k1), S = (k2, 2 k3), C = (k4, 2 k5)
  const Fp2 sq01{k0, fp_dbl(k1)};
  const Fp2 xy = kara(k2, k3, k4);
  const Fp2 S{k2, fp_dbl(k3)}, C1{k4, fp_dbl(k5)};
  // exchange: lane 0 gets B, C; lane 1 gets X2
  const Fp2 w1 = pswap(sq01);
  const Fp2 w2 = pswap(C1);
  const Fp2 B = fp2_sel(h, sq01, w1), C = fp2_sel(h, C1, w2), X2 = fp2_sel(h, w1, sq01);
  const Fp2 E = fp2_mul_3b(C), F = fp2_add(fp2_dbl(E), E);
  const Fp2 A = fp2_half(xy);                         // lane 0 only
  const Fp2 BmF = fp2_sub(B, F), G = fp2_half(fp2_add(B, F));
  const Fp2 H = fp2_sub(S, fp2_add(B, C));            // lane 1 only
  const Fp2 L0 = fp2_sub(B, E), X2x3 = fp2_add(fp2_dbl(X2), X2);
  // round 2 -- lane 0: X3 = A (B - F) (3), E^2 (2), G^2 (2), c2.re (1);
  //            lane 1: Z3 = B H (3), c0 = (B - E) z^3 (2), c3 = H y (2), c2.im (1)
  Fp q0 = pm(h, A.c0, BmF.c0, B.c0, H.c0);
  Fp q1 = pm(h, A.c1, BmF.c1, B.c1, H.c1);
  Fp q2 = pm(h, LZA(A.c0, A.c1), LZA(BmF.c0, BmF.c1), LZA(B.c0, B.c1), LZA(H.c0, H.c1));
  Fp q3 = pm(h, LZA(E.c0, E.c1), LZS(E.c0, E.c1), L0.c0, P.z3);
  Fp q4 = pm(h, E.c0, E.c1, L0.c1, P.z3);
  Fp q5 = pm(h, LZA(G.c0, G.c1), LZS(G.c0, G.c1), H.c0, P.y);
  Fp q6 = pm(h, G.c0, G.c1, H.c1, P.y);
  Fp q7 = pm(h, X2x3.c0, P.nxz, X2x3.c1, P.nxz);
  const Fp2 K = kara(q0, q1, q2);  // lane 0: X3, lane 1: Z3
  const Fp2 E2{q3, fp_dbl(q4)}, G2{q5, fp_dbl(q6)};
  const Fp2 Y3 = fp2_sub(G2, fp2_add(fp2_dbl(E2), E2));  // lane 0
  const Fp2 c0{q3, q4}, c3{q5, q6};                      // lane 1
  // exchange: lane 0 sends X3, Y3, c2.re; lane 1 sends Z3, c0, c3, c2.im
  const Fp2 v1 = pswap(K);
  const Fp2 v2 = pswap(fp2_sel(h, c0, Y3));
  const Fp2 v3 = pswap(c3);
  const Fp v4 = pswap(q7);
  T.x = fp2_sel(h, v1, K);
  T.y = fp2_sel(h, v2, Y3);
  T.z = fp2_sel(h, K, v1);
  Line l;
  l.c0 = fp2_sel(h, c0, v2);
  l.c3 = fp2_sel(h, c3, v3);
  l.c2 = Fp2{fp_sel(h, v4, q7), fp_sel(h, q7, v4)};
  return l;
}

// Mixed addition step T <- T + Q (Q affine) and its line through P (add_step, pairing.h).
__device__ __forceinline__ Line pair_add(PairT& T, const G2A& Q, const PairP& P, bool h) {
  const Fp2 &x = T.x, &y = T.y, &z = T.z;
  // round 1 -- lane 0: Qy z, lane 1: Qx z
  const Fp2 Qs = fp2_sel(h, Q.x, Q.y);
  Fp a0 = fp_mul(Qs.c0, z.c0);
  Fp a1 = fp_mul(Qs.c1, z.c1);
  Fp a2 = fp_mul(LZA(Qs.c0, Qs.c1), LZA(z.c0, z.c1));
  const Fp2 Qz = kara(a0, a1, a2);
  const Fp2 tl = fp2_sub(fp2_sel(h, x, y), Qz);  // lane 0: theta = y - Qy z, lane 1: lam = x - Qx z
  const Fp2 tlo = pswap(tl);
  const Fp2 th = fp2_sel(h, tlo, tl), lm = fp2_sel(h, tl, tlo);
  // round 2 -- lane 0: C = theta^2, theta Qx, c2 = theta (-X Z); lane 1: D = lam^2, lam Qy, c3 = lam Y
  const Fp2 Qo = fp2_sel(h, Q.y, Q.x);
  const Fp so = fp_sel(h, P.y, P.nxz);
  Fp b0 = fp_mul(LZA(tl.c0, tl.c1), LZS(tl.c0, tl.c1));
  Fp b1 = fp_mul(tl.c0, tl.c1);
  Fp b2 = fp_mul(tl.c0, Qo.c0);
  Fp b3 = fp_mul(tl.c1, Qo.c1);
  Fp b4 = fp_mul(LZA(tl.c0, tl.c1), LZA(Qo.c0, Qo.c1));
  Fp b5 = fp_mul(tl.c0, so);
  Fp b6 = fp_mul(tl.c1, so);
  const Fp2 sq{b0, fp_dbl(b1)}, tq = kara(b2, b3, b4), cc{b5, b6};
  const Fp2 sqo = pswap(sq), tqo = pswap(tq), cco = pswap(cc);
  const Fp2 C = fp2_sel(h, sqo, sq), D = fp2_sel(h, sq, sqo);
  const Fp2 L0 = fp2_sel(h, fp2_sub(tqo, tq), fp2_sub(tq, tqo));  // theta Qx - lam Qy
  Line l;
  l.c2 = fp2_sel(h, cco, cc);
  l.c3 = fp2_sel(h, cc, cco);
  // round 3 -- lane 0: E = D lam (3), F = z C (3); lane 1: G = x D (3), c0 = L0 z^3 (2), one spare
  Fp d0 = pm(h, D.c0, lm.c0, x.c0, D.c0);
  Fp d1 = pm(h, D.c1, lm.c1, x.c1, D.c1);
  Fp d2 = pm(h, LZA(D.c0, D.c1), LZA(lm.c0, lm.c1), LZA(x.c0, x.c1), LZA(D.c0, D.c1));
  Fp d3 = pm(h, z.c0, C.c0, L0.c0, P.z3);
  Fp d4 = pm(h, z.c1, C.c1, L0.c1, P.z3);
  Fp d5 = pm(h, LZA(z.c0, z.c1), LZA(C.c0, C.c1), L0.c0, P.z3);
  const Fp2 EG = kara(d0, d1, d2);                 // lane 0: E, lane 1: G
  const Fp2 Fc = fp2_sel(h, Fp2{d3, d4}, kara(d3, d4, d5));  // lane 0: F, lane 1: c0
  const Fp2 EGo = pswap(EG), Fco = pswap(Fc);
  const Fp2 E = fp2_sel(h, EGo, EG), G = fp2_sel(h, EG, EGo), Fz = fp2_sel(h, Fco, Fc);
  l.c0 = fp2_sel(h, Fc, Fco);
  const Fp2 Hh = fp2_sub(fp2_add(E, Fz), fp2_dbl(G));
  const Fp2 GH = fp2_sub(G, Hh);
  // round 4 -- lane 0: X3 = lam H (3), theta (G - H) (3); lane 1: y E (3), Z3 = z E (3)
  const Fp2 u = fp2_sel(h, y, lm), v = fp2_sel(h, E, Hh), w = fp2_sel(h, z, th), t = fp2_sel(h, E, GH);
  Fp e0 = fp_mul(u.c0, v.c0);
  Fp e1 = fp_mul(u.c1, v.c1);
  Fp e2 = fp_mul(LZA(u.c0, u.c1), LZA(v.c0, v.c1));
  Fp e3 = fp_mul(w.c0, t.c0);
  Fp e4 = fp_mul(w.c1, t.c1);
  Fp e5 = fp_mul(LZA(w.c0, w.c1), LZA(t.c0, t.c1));
  const Fp2 K1 = kara(e0, e1, e2);  // lane 0: X3, lane 1: y E
  const Fp2 K2 = kara(e3, e4, e5);  // lane 0: theta (G - H), lane 1: Z3
  const Fp2 K1o = pswap(K1), K2o = pswap(K2);
  const Fp2 yE = fp2_sel(h, K1, K1o), W = fp2_sel(h, K2o, K2);
  T.x = fp2_sel(h, K1o, K1);
  T.z = fp2_sel(h, K2, K2o);
  T.y = fp2_sub(W, yE);
  return l;
}
#undef LZA
#undef LZS

}  // namespace gbv
