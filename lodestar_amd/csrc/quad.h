// Quad-lane Miller loop: one signature set's f_{|x|, Q}(P) on the FOUR lanes of a DPP quad (lanes
// 4j .. 4j+3 of a wave), for passes too small to fill the chip with a lane pair per set (pair.h):
// range-sync segments, per-GPU shards of one call.
//
// Lane q = 2h + s of the quad: the lanes h = 0 hold c0 of f = c0 + c1 w, the lanes h = 1 hold c1
// (pair.h's split, each half on two lanes), and the G2 point T, the line, P and Q are on all four.
// Every step is a sequence of product rounds: in a round each lane runs ONE product with operands
// picked by v_cndmask from candidates all lanes form alike, then the results cross the quad by DPP
// quad_perm moves (one v_mov_b32_dpp per dword; no LDS, no memory):
//   f^2        the half pair's Fp6 product (t = c0 c1 on h = 0, u = (c0 + c1)(c0 + v c1) on h = 1)
//              as 6 Fp2 products, 3 per lane; c0' = u - t - v t, c1' = 2 t
//   f * line   line = A + B w, A = (l0, l2, 0), B = (0, l3, 0): c_h A and c_h B, 8 Fp2 products, 4
//              per lane; c0' = c0 A + v c1 B, c1' = c0 B + c1 A
//   doubling   27 Fp products in 3 + 4 rounds of 4 (T on all lanes: broadcasts of all four results)
//   addition   43 Fp products in 2 + 4 + 3 + 3 rounds of 4
// Per Miller bit a lane runs 28 Fp products (56 on a lane pair, 111 on one lane), with the per-lane
// state of the pair form (an Fp6 half, T, P, Q).  Formulas: pairing.h dbl_step / add_step and pair.h
// (tests/test_algorithm_prototypes.py checks them against the oracle); all results canonical, so
// the Miller value equals the thread and pair forms' bit for bit.
#pragma once
#include "pair.h"

namespace gbv {
namespace quad {

// quad_perm controls: broadcast of quad lane J = J * 0x55; the partner in the half pair [1,0,3,2];
// the same lane of the other half [2,3,0,1]
constexpr int SWAP_S = 0xB1, SWAP_H = 0x4E;

#if defined(__HIP_DEVICE_COMPILE__)
template <int CTRL> __device__ __forceinline__ uint32_t dpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}
#else
template <int CTRL> __device__ inline uint32_t dpp(uint32_t v) { return v; }  // host pass: parsed, never emitted
#endif

template <int CTRL> __device__ __forceinline__ Fp dpp(const Fp& a) {
  Fp r;
#pragma unroll
  for (int i = 0; i < 12; ++i) r.v[i] = dpp<CTRL>(a.v[i]);
  return r;
}
template <int CTRL> __device__ __forceinline__ Fp2 dpp(const Fp2& a) { return Fp2{dpp<CTRL>(a.c0), dpp<CTRL>(a.c1)}; }
template <int CTRL> __device__ __forceinline__ Fp6 dpp(const Fp6& a) { return Fp6{dpp<CTRL>(a.c0), dpp<CTRL>(a.c1), dpp<CTRL>(a.c2)}; }
template <int CTRL, class F> __device__ __forceinline__ Jac<F> dpp(const Jac<F>& a) {
  return Jac<F>{dpp<CTRL>(a.x), dpp<CTRL>(a.y), dpp<CTRL>(a.z)};
}

struct Lane {
  uint32_t q;  // lane in the quad
  bool h, s;   // q = 2h + s
};

__device__ __forceinline__ Fp sel4(uint32_t q, const Fp& x0, const Fp& x1, const Fp& x2, const Fp& x3) {
  return fp_sel((q & 2u) != 0, fp_sel((q & 1u) != 0, x3, x2), fp_sel((q & 1u) != 0, x1, x0));
}

// Store of a value every quad lane holds: lane j writes Fp words j, j + 4, ... (n_fp Fp in all)
template <int NFP> __device__ __forceinline__ void store_split(Fp* out, const Fp* v, uint32_t q) {
#pragma unroll
  for (int k = 0; k < NFP; k += 4) {
    if (k + 3 < NFP) {
      out[k + q] = sel4(q, v[k], v[k + 1], v[k + 2], v[k + 3]);
    } else {
      const Fp a = v[k], b = k + 1 < NFP ? v[k + 1] : v[k], c = k + 2 < NFP ? v[k + 2] : v[k];
      if (k + q < (uint32_t)NFP) out[k + q] = sel4(q, a, b, c, c);
    }
  }
}

// One round of four Fp products on the quad: lane j runs a_j b_j; every lane returns all four.
__device__ __forceinline__ void round4(Fp r[4], uint32_t q, const Fp& a0, const Fp& b0, const Fp& a1, const Fp& b1, const Fp& a2,
                                       const Fp& b2, const Fp& a3, const Fp& b3) {
  const Fp x = fp_mul(sel4(q, a0, a1, a2, a3), sel4(q, b0, b1, b2, b3));
  r[0] = dpp<0x00>(x);
  r[1] = dpp<0x55>(x);
  r[2] = dpp<0xAA>(x);
  r[3] = dpp<0xFF>(x);
}

#define QLZA fp_add_lazy
#define QLZS fp_sub_lazy4
__device__ __forceinline__ Fp2 sq(const Fp& t0, const Fp& t1) { return Fp2{t0, fp_dbl(t1)}; }  // ((a0+a1)(a0-a1), a0 a1)

// Doubling step T <- 2T and its line through P (pair_dbl's products, spread over the quad).
__device__ __forceinline__ Line dbl(PairT& T, const PairP& P, uint32_t q) {
  const Fp2 &x = T.x, &y = T.y, &z = T.z;
  const Fp zero = fp_zero();
  Fp r[4];
  // round 1: x y (3), y^2 (2), z^2 (2), x^2 (2), (y + z)^2 (2)
  round4(r, q, x.c0, y.c0, x.c1, y.c1, QLZA(x.c0, x.c1), QLZA(y.c0, y.c1), QLZA(y.c0, y.c1), QLZS(y.c0, y.c1));
  const Fp2 xy = kara(r[0], r[1], r[2]);
  const Fp b_re = r[3];
  round4(r, q, y.c0, y.c1, QLZA(z.c0, z.c1), QLZS(z.c0, z.c1), z.c0, z.c1, QLZA(x.c0, x.c1), QLZS(x.c0, x.c1));
  const Fp2 B{b_re, fp_dbl(r[0])};
  const Fp2 C = sq(r[1], r[2]);
  const Fp x2_re = r[3];
  const Fp2 s = fp2_add(y, z);
  round4(r, q, x.c0, x.c1, QLZA(s.c0, s.c1), QLZS(s.c0, s.c1), s.c0, s.c1, zero, zero);
  const Fp2 X2{x2_re, fp_dbl(r[0])};
  const Fp2 S = sq(r[1], r[2]);
  const Fp2 E = fp2_mul_3b(C), F = fp2_add(fp2_dbl(E), E);
  const Fp2 A = fp2_half(xy);
  const Fp2 BmF = fp2_sub(B, F), G = fp2_half(fp2_add(B, F));
  const Fp2 H = fp2_sub(S, fp2_add(B, C));
  const Fp2 L0 = fp2_sub(B, E), X2x3 = fp2_add(fp2_dbl(X2), X2);
  // round 2: X3 = A (B - F) (3), E^2 (2), G^2 (2), Z3 = B H (3), c0 = (B - E) z^3 (2), c3 = H y (2),
  // c2 = 3 X^2 (-x z) (2)
  round4(r, q, A.c0, BmF.c0, A.c1, BmF.c1, QLZA(A.c0, A.c1), QLZA(BmF.c0, BmF.c1), QLZA(E.c0, E.c1), QLZS(E.c0, E.c1));
  T.x = kara(r[0], r[1], r[2]);
  const Fp e2_re = r[3];
  round4(r, q, E.c0, E.c1, QLZA(G.c0, G.c1), QLZS(G.c0, G.c1), G.c0, G.c1, B.c0, H.c0);
  const Fp2 E2{e2_re, fp_dbl(r[0])};
  T.y = fp2_sub(sq(r[1], r[2]), fp2_add(fp2_dbl(E2), E2));
  const Fp bh0 = r[3];
  Line l;
  round4(r, q, B.c1, H.c1, QLZA(B.c0, B.c1), QLZA(H.c0, H.c1), L0.c0, P.z3, L0.c1, P.z3);
  T.z = kara(bh0, r[0], r[1]);
  l.c0 = Fp2{r[2], r[3]};
  round4(r, q, H.c0, P.y, H.c1, P.y, X2x3.c0, P.nxz, X2x3.c1, P.nxz);
  l.c3 = Fp2{r[0], r[1]};
  l.c2 = Fp2{r[2], r[3]};
  return l;
}

// Mixed addition step T <- T + Q (Q affine) and its line through P (pair_add's products).
__device__ __forceinline__ Line add(PairT& T, const G2A& Q, const PairP& P, uint32_t q) {
  const Fp2 &x = T.x, &y = T.y, &z = T.z;
  const Fp zero = fp_zero();
  Fp r[4];
  // round 1: Qy z (3), Qx z (3)
  round4(r, q, Q.y.c0, z.c0, Q.y.c1, z.c1, QLZA(Q.y.c0, Q.y.c1), QLZA(z.c0, z.c1), Q.x.c0, z.c0);
  const Fp2 th = fp2_sub(y, kara(r[0], r[1], r[2]));
  const Fp qxz0 = r[3];
  round4(r, q, Q.x.c1, z.c1, QLZA(Q.x.c0, Q.x.c1), QLZA(z.c0, z.c1), zero, zero, zero, zero);
  const Fp2 lm = fp2_sub(x, kara(qxz0, r[0], r[1]));
  // round 2: C = th^2 (2), D = lm^2 (2), th Qx (3), lm Qy (3), c2 = th (-x z) (2), c3 = lm y (2)
  round4(r, q, QLZA(th.c0, th.c1), QLZS(th.c0, th.c1), th.c0, th.c1, QLZA(lm.c0, lm.c1), QLZS(lm.c0, lm.c1), lm.c0, lm.c1);
  const Fp2 C = sq(r[0], r[1]), D = sq(r[2], r[3]);
  round4(r, q, th.c0, Q.x.c0, th.c1, Q.x.c1, QLZA(th.c0, th.c1), QLZA(Q.x.c0, Q.x.c1), lm.c0, Q.y.c0);
  const Fp2 thQx = kara(r[0], r[1], r[2]);
  const Fp lqy0 = r[3];
  Line l;
  round4(r, q, lm.c1, Q.y.c1, QLZA(lm.c0, lm.c1), QLZA(Q.y.c0, Q.y.c1), th.c0, P.nxz, th.c1, P.nxz);
  const Fp2 L0 = fp2_sub(thQx, kara(lqy0, r[0], r[1]));
  l.c2 = Fp2{r[2], r[3]};
  // c3 = lm y with the first two products of round 3: E = D lm (3), F = z C (3), G = x D (3),
  // c0 = L0 z^3 (2)
  round4(r, q, lm.c0, P.y, lm.c1, P.y, D.c0, lm.c0, D.c1, lm.c1);
  l.c3 = Fp2{r[0], r[1]};
  const Fp dl0 = r[2], dl1 = r[3];
  round4(r, q, QLZA(D.c0, D.c1), QLZA(lm.c0, lm.c1), z.c0, C.c0, z.c1, C.c1, QLZA(z.c0, z.c1), QLZA(C.c0, C.c1));
  const Fp2 E = kara(dl0, dl1, r[0]);
  const Fp2 Fz = kara(r[1], r[2], r[3]);
  round4(r, q, x.c0, D.c0, x.c1, D.c1, QLZA(x.c0, x.c1), QLZA(D.c0, D.c1), L0.c0, P.z3);
  const Fp2 G = kara(r[0], r[1], r[2]);
  const Fp c00 = r[3];
  const Fp2 Hh = fp2_sub(fp2_add(E, Fz), fp2_dbl(G));
  const Fp2 GH = fp2_sub(G, Hh);
  // the last product of round 3 with round 4: X3 = lm H (3), th (G - H) (3), y E (3), Z3 = z E (3)
  round4(r, q, L0.c1, P.z3, lm.c0, Hh.c0, lm.c1, Hh.c1, QLZA(lm.c0, lm.c1), QLZA(Hh.c0, Hh.c1));
  l.c0 = Fp2{c00, r[0]};
  const Fp2 X3 = kara(r[1], r[2], r[3]);
  round4(r, q, th.c0, GH.c0, th.c1, GH.c1, QLZA(th.c0, th.c1), QLZA(GH.c0, GH.c1), y.c0, E.c0);
  const Fp2 thGH = kara(r[0], r[1], r[2]);
  const Fp ye0 = r[3];
  round4(r, q, y.c1, E.c1, QLZA(y.c0, y.c1), QLZA(E.c0, E.c1), z.c0, E.c0, z.c1, E.c1);
  T.y = fp2_sub(thGH, kara(ye0, r[0], r[1]));
  const Fp ze0 = r[2], ze1 = r[3];
  round4(r, q, QLZA(z.c0, z.c1), QLZA(E.c0, E.c1), zero, zero, zero, zero, zero, zero);
  T.z = kara(ze0, ze1, r[0]);
  T.x = X3;
  return l;
}
#undef QLZA
#undef QLZS

// Fp6 Karatsuba recombination of k = (a0 b0, a1 b1, a2 b2, (a1+a2)(b1+b2), (a0+a1)(b0+b1), (a0+a2)(b0+b2))
__device__ __forceinline__ Fp6 fp6_kara(const Fp2& k0, const Fp2& k1, const Fp2& k2, const Fp2& k3, const Fp2& k4, const Fp2& k5) {
  return Fp6{fp2_add(k0, fp2_mul_xi(fp2_sub(fp2_sub(k3, k1), k2))), fp2_add(fp2_sub(fp2_sub(k4, k0), k1), fp2_mul_xi(k2)),
             fp2_add(fp2_sub(fp2_sub(k5, k0), k2), k1)};
}

// f <- f^2 (M = this lane's half of f)
__device__ __forceinline__ void sqr(Fp6& M, const Lane& L) {
  const Fp6 O = dpp<SWAP_H>(M);
  // h = 0 (M = c0, O = c1): X = c0, Y = c1.  h = 1 (M = c1, O = c0): X = c0 + c1, Y = c0 + v c1.
  const Fp6 X = fp6_sel(L.h, fp6_add(O, M), M);
  const Fp6 Y = fp6_sel(L.h, fp6_add(O, fp6_mul_v(M)), O);
  // s = 0: X0 Y0, X1 Y1, X2 Y2; s = 1: (X1+X2)(Y1+Y2), (X0+X1)(Y0+Y1), (X0+X2)(Y0+Y2)
  const Fp2 k0 = fp2_mul(fp2_sel(L.s, fp2_add_lazy(X.c1, X.c2), X.c0), fp2_sel(L.s, fp2_add_lazy(Y.c1, Y.c2), Y.c0));
  const Fp2 k1 = fp2_mul(fp2_sel(L.s, fp2_add_lazy(X.c0, X.c1), X.c1), fp2_sel(L.s, fp2_add_lazy(Y.c0, Y.c1), Y.c1));
  const Fp2 k2 = fp2_mul(fp2_sel(L.s, fp2_add_lazy(X.c0, X.c2), X.c2), fp2_sel(L.s, fp2_add_lazy(Y.c0, Y.c2), Y.c2));
  const Fp2 o0 = dpp<SWAP_S>(k0), o1 = dpp<SWAP_S>(k1), o2 = dpp<SWAP_S>(k2);
  const Fp6 R = fp6_kara(fp2_sel(L.s, o0, k0), fp2_sel(L.s, o1, k1), fp2_sel(L.s, o2, k2), fp2_sel(L.s, k0, o0), fp2_sel(L.s, k1, o1),
                         fp2_sel(L.s, k2, o2));
  const Fp6 Ro = dpp<SWAP_H>(R);
  // h = 0: c0' = u - t - v t (t = R, u = Ro); h = 1: c1' = 2 t (t = Ro)
  M = fp6_sel(L.h, fp6_add(Ro, Ro), fp6_sub(Ro, fp6_add(R, fp6_mul_v(R))));
}

// f <- f g (M, G: this lane's halves of f and g).  t_h = f_h g_h on the lanes of half h (the Fp6
// Karatsuba products split by s, as in sqr), u = (f0 + f1)(g0 + g1) with its six Fp2 products spread
// over the four lanes and broadcast; then c0 = t0 + v t1, c1 = u - t0 - t1.  15 Fp products a lane
// (54 on one lane); the same canonical value as fp12_mul.
__device__ __forceinline__ void mul12(Fp6& M, const Fp6& G, const Lane& L) {
  const Fp2 k0 = fp2_mul(fp2_sel(L.s, fp2_add_lazy(M.c1, M.c2), M.c0), fp2_sel(L.s, fp2_add_lazy(G.c1, G.c2), G.c0));
  const Fp2 k1 = fp2_mul(fp2_sel(L.s, fp2_add_lazy(M.c0, M.c1), M.c1), fp2_sel(L.s, fp2_add_lazy(G.c0, G.c1), G.c1));
  const Fp2 k2 = fp2_mul(fp2_sel(L.s, fp2_add_lazy(M.c0, M.c2), M.c2), fp2_sel(L.s, fp2_add_lazy(G.c0, G.c2), G.c2));
  const Fp2 o0 = dpp<SWAP_S>(k0), o1 = dpp<SWAP_S>(k1), o2 = dpp<SWAP_S>(k2);
  const Fp6 T = fp6_kara(fp2_sel(L.s, o0, k0), fp2_sel(L.s, o1, k1), fp2_sel(L.s, o2, k2), fp2_sel(L.s, k0, o0), fp2_sel(L.s, k1, o1),
                         fp2_sel(L.s, k2, o2));
  const Fp6 X = fp6_add(M, dpp<SWAP_H>(M)), Y = fp6_add(G, dpp<SWAP_H>(G));  // f0 + f1, g0 + g1 on every lane
  // u's products: lane q runs product q, lanes 0, 1 also product q + 4 (lanes 2, 3 repeat theirs)
  //   0: X0 Y0, 1: X1 Y1, 2: X2 Y2, 3: (X1 + X2)(Y1 + Y2), 4: (X0 + X1)(Y0 + Y1), 5: (X0 + X2)(Y0 + Y2)
  const bool hi = (L.q & 2u) != 0, lo = (L.q & 1u) != 0;
  const Fp2 a0 = fp2_sel(hi, fp2_sel(lo, fp2_add_lazy(X.c1, X.c2), X.c2), fp2_sel(lo, X.c1, X.c0));
  const Fp2 b0 = fp2_sel(hi, fp2_sel(lo, fp2_add_lazy(Y.c1, Y.c2), Y.c2), fp2_sel(lo, Y.c1, Y.c0));
  const Fp2 a1 = fp2_sel(lo, fp2_add_lazy(X.c0, X.c2), fp2_add_lazy(X.c0, X.c1));
  const Fp2 b1 = fp2_sel(lo, fp2_add_lazy(Y.c0, Y.c2), fp2_add_lazy(Y.c0, Y.c1));
  const Fp2 pa = fp2_mul(a0, b0), pb = fp2_mul(a1, b1);
  const Fp6 U = fp6_kara(dpp<0x00>(pa), dpp<0x55>(pa), dpp<0xAA>(pa), dpp<0xFF>(pa), dpp<0x00>(pb), dpp<0x55>(pb));
  const Fp6 To = dpp<SWAP_H>(T);
  // h = 0: c0 = t0 + v t1 (T = t0, To = t1); h = 1: c1 = u - t0 - t1
  M = fp6_sel(L.h, fp6_sub(fp6_sub(U, To), T), fp6_add(T, fp6_mul_v(To)));
}

// f <- f * (A + B w), A = (l0, l2, 0), B = (0, l3, 0)
__device__ __forceinline__ void mul_line(Fp6& M, const Line& l, const Lane& L) {
  // c_h A = (p0 + xi p3, p2 - p0 - p1, p1 + p4), c_h B = (xi p5, p6, p7);
  // s = 0: p0 = M0 l0, p1 = M1 l2, p2 = (M0 + M1)(l0 + l2), p3 = M2 l2;
  // s = 1: p4 = M2 l0, p5 = M2 l3, p6 = M0 l3, p7 = M1 l3
  const Fp2 a = fp2_mul(fp2_sel(L.s, M.c2, M.c0), l.c0);
  const Fp2 b = fp2_mul(fp2_sel(L.s, M.c2, M.c1), fp2_sel(L.s, l.c3, l.c2));
  const Fp2 c = fp2_mul(fp2_sel(L.s, M.c0, fp2_add_lazy(M.c0, M.c1)), fp2_sel(L.s, l.c3, fp2_add_lazy(l.c0, l.c2)));
  const Fp2 d = fp2_mul(fp2_sel(L.s, M.c1, M.c2), fp2_sel(L.s, l.c3, l.c2));
  const Fp2 ao = dpp<SWAP_S>(a), bo = dpp<SWAP_S>(b), co = dpp<SWAP_S>(c), dd = dpp<SWAP_S>(d);
  const Fp2 p0 = fp2_sel(L.s, ao, a), p1 = fp2_sel(L.s, bo, b), p2 = fp2_sel(L.s, co, c), p3 = fp2_sel(L.s, dd, d);
  const Fp2 p4 = fp2_sel(L.s, a, ao), p5 = fp2_sel(L.s, b, bo), p6 = fp2_sel(L.s, c, co), p7 = fp2_sel(L.s, d, dd);
  const Fp6 X1{fp2_add(p0, fp2_mul_xi(p3)), fp2_sub(fp2_sub(p2, p0), p1), fp2_add(p1, p4)};
  const Fp6 X2o = dpp<SWAP_H>(Fp6{fp2_mul_xi(p5), p6, p7});  // h = 0: c1 B, h = 1: c0 B
  M = fp6_add(X1, fp6_sel(L.h, X2o, fp6_mul_v(X2o)));
}

}  // namespace quad
}  // namespace gbv
