// Lazy Fp / Fp2 arithmetic in the 28-bit limb form of the product (fp.h: F28), for long chains of
// point doublings (the G2 subgroup check's [|x|]Q: 63 doublings per signature).
//
// The 12 x 32-bit form pays, per Fp product, the repacking into 28-bit limbs and back plus a final
// conditional subtraction (128 of 607 instructions), and a full modular add/sub (carry chain +
// compare + select) per addition.  Here the values stay in 28-bit limbs between products:
//   * add       a + b limb by limb (14 adds, no carry);
//   * sub       a + K - b limb by limb, K a multiple of p whose limbs are raised by borrowing so
//               that every limb of K is >= the matching limb of b (no negative limb ever appears);
//   * norm      carry propagation (limbs < 2^28 except the top one) before a value is multiplied;
//   * wred      subtract q p, q from the top limb, bringing a normalized value below 1.01 p.
// Values are congruent mod p, never canonical; each call site below states the bound (in units of
// p) of what it produces, and every product input is normalized with value < 64 p, so each column
// of mul28 stays below 2^63 and its output below 1.01 p + (a b / 2^392) (fp.h).  Canonical
// values come back through l_to_fp (wred, repack, one conditional subtraction).
#pragma once
#include "fp2.h"

namespace gbv {

// k p in 28-bit limbs with limbs 0..12 raised into [2^s - 2^(s-28), 2^s + 2^28) by borrowing
// 2^(s-28) from the limb above (the value is unchanged); the top limb keeps the rest.
struct K28 { uint32_t v[14]; };
constexpr K28 kp28(uint32_t k, int s) {
  K28 r{};
  uint64_t c = 0;
  for (int i = 0; i < 14; ++i) {
    const uint64_t t = (uint64_t)k * P28[i] + c;
    r.v[i] = i < 13 ? (uint32_t)(t & 0xFFFFFFFull) : (uint32_t)t;
    c = t >> 28;
  }
  for (int i = 0; i < 13; ++i) {
    r.v[i] += 1u << s;
    r.v[i + 1] -= 1u << (s - 28);
  }
  return r;
}

// the constants the doubling uses (kp28(k, s): value k p, limbs >= 2^s - 2^(s-28))
constexpr K28 K2P_28 = kp28(2, 28);    // covers a normalized subtrahend < 2 p
constexpr K28 K4P_28 = kp28(4, 28);
constexpr K28 K12P_28 = kp28(12, 28);
constexpr K28 K4P_29 = kp28(4, 29);    // covers a sum of two normalized values < 4 p
constexpr K28 K24P_29 = kp28(24, 29);  // covers 2 x (normalized < 12 p)

struct L2 { F28 c0, c1; };
struct L2J { L2 x, y, z; };

GBV_HD F28 l_add(const F28& a, const F28& b) {
  F28 r;
#pragma unroll
  for (int i = 0; i < 14; ++i) r.v[i] = a.v[i] + b.v[i];
  return r;
}

GBV_HD F28 l_subk(const F28& a, const F28& b, const K28 k) {
  F28 r;
#pragma unroll
  for (int i = 0; i < 14; ++i) r.v[i] = a.v[i] + k.v[i] - b.v[i];
  return r;
}

GBV_HD F28 l_norm(const F28& a) {
  F28 r = a;
#pragma unroll
  for (int i = 0; i < 13; ++i) {
    r.v[i + 1] += r.v[i] >> 28;
    r.v[i] &= M28;
  }
  return r;
}

// normalized a (top limb t < 2^28) -> a - q p with q = floor(t / (P28[13] + 1)) <= floor(a / p):
// the result is >= 0 and below (P28[13] + q + 1) 2^364 < 1.01 p for q < 2^10.  Normalized out.
GBV_HD F28 l_wred(const F28& a) {
  const uint32_t q = a.v[13] / (P28[13] + 1u);
  F28 r;
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < 13; ++i) {
    const int64_t t = (int64_t)a.v[i] - (int64_t)((uint64_t)q * P28[i]) + c;
    r.v[i] = (uint32_t)t & M28;
    c = t >> 28;  // arithmetic: floor
  }
  r.v[13] = (uint32_t)((int64_t)a.v[13] - (int64_t)q * P28[13] + c);
  return r;
}

GBV_HD L2 l2_add(const L2& a, const L2& b) { return L2{l_add(a.c0, b.c0), l_add(a.c1, b.c1)}; }
GBV_HD L2 l2_subk(const L2& a, const L2& b, const K28 k) { return L2{l_subk(a.c0, b.c0, k), l_subk(a.c1, b.c1, k)}; }
GBV_HD L2 l2_norm(const L2& a) { return L2{l_norm(a.c0), l_norm(a.c1)}; }
GBV_HD L2 l2_wred(const L2& a) { return L2{l_wred(a.c0), l_wred(a.c1)}; }

// Karatsuba product.  a, b normalized with values va, vb < 16 p: t0, t1 < 1.13 p, t2 < 1.5 p;
// c0 = t0 + 2p - t1 < 3.2 p, c1 = t2 + 4p - t0 - t1 < 5.5 p, both normalized.
GBV_HD L2 l2_mul(const L2& a, const L2& b) {
  const F28 t0 = mul28(a.c0, b.c0);
  const F28 t1 = mul28(a.c1, b.c1);
  const F28 t2 = mul28(l_add(a.c0, a.c1), l_add(b.c0, b.c1));
  return L2{l_norm(l_subk(t0, t1, K2P_28)), l_norm(l_subk(t2, l_add(t0, t1), K4P_29))};
}

// (a0 + a1)(a0 - a1) + 2 a0 a1 i.  a normalized with value va <= K's multiple of p (the caller
// passes K covering a.c1): outputs normalized, < 1 p + (2 va)(va + k) p / 2520 (R / p ~ 2520).
GBV_HD L2 l2_sqr(const L2& a, const K28 k) {
  const F28 c0 = mul28(l_add(a.c0, a.c1), l_subk(a.c0, a.c1, k));
  const F28 c1 = mul28(l_add(a.c0, a.c0), a.c1);
  return L2{c0, c1};
}

GBV_HD L2 l2_from(const Fp2& a) { return L2{fp_to28(a.c0), fp_to28(a.c1)}; }
GBV_HD Fp l_to_fp(const F28& a) { return fp_reduce_once(fp_from28(l_wred(a))); }  // a normalized
GBV_HD Fp2 l2_to(const L2& a) { return Fp2{l_to_fp(a.c0), l_to_fp(a.c1)}; }

// dbl-2009-l (as jac_dbl in curve.h) over L2.  In: x, y, z normalized < 2 p.  Out: the same.
// Bounds (units of p) at each step are in the comments; products of inputs < 16 p are < 1.13 p.
GBV_HD L2J l2j_dbl(const L2J& p) {
  L2J r;
  const L2 yz = l2_mul(p.y, p.z);                         // < 3.2 / 5.5
  r.z = l2_wred(l2_norm(l2_add(yz, yz)));                 // < 11 -> < 1.01
  const L2 B = l2_sqr(p.y, K2P_28);                       // < 1.01
  const L2 A = l2_sqr(p.x, K2P_28);                       // < 1.01
  const L2 C = l2_sqr(B, K2P_28);                         // < 1.01
  const L2 T = l2_sqr(l2_norm(l2_add(p.x, B)), K4P_28);   // x + B < 3.02 -> T < 1.03
  const L2 D = l2_norm(l2_add(l2_subk(T, l2_add(A, C), K4P_29), l2_subk(T, l2_add(A, C), K4P_29)));  // < 10.1
  const L2 E = l2_norm(l2_add(l2_add(A, A), A));          // < 3.03
  const L2 Fv = l2_sqr(E, K4P_28);                        // < 1.03
  r.x = l2_wred(l2_norm(l2_subk(Fv, l2_add(D, D), K24P_29)));  // 2D < 20.2: < 25.1 -> < 1.01
  const L2 DX = l2_norm(l2_subk(D, r.x, K2P_28));         // < 12.1
  const L2 EDX = l2_mul(E, DX);                           // < 3.2 / 5.5
  const L2 C8 = l2_norm(l2_add(l2_add(l2_add(C, C), l2_add(C, C)), l2_add(l2_add(C, C), l2_add(C, C))));  // < 8.1
  r.y = l2_wred(l2_norm(l2_subk(EDX, C8, K12P_28)));      // < 17.6 -> < 1.01
  return r;
}

}  // namespace gbv
