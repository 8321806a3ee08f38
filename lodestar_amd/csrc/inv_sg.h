// Fp inversion by Bernstein-Yang "safegcd" divsteps, variable time (the inputs are public: signature
// and pubkey coordinates, pairing values), in batches of 62 divsteps.
//
// Why: the branch-free binary extended GCD it replaces runs ~768 fixed steps of ~190 VALU ops, ~330 us
// on one lane (profiles/ubench/r02_ubench_coop_v5.txt "fp_inv lane"), and sits on every latency path
// several times: the affine conversions of the cofactor clearing, of the pairing-check inputs and of
// the randomisation tables, the Fp12 inversion of the final exponentiation.  Here each batch works on
// the low 64 bits of f and g only (divsteps_62_var: shifts over runs of zeros, one table-free 4- or
// 6-bit inverse per step), and applies the resulting 2x2 transition matrix (entries below 2^62) to the
// full numbers once, as 7 signed limbs of 62 bits.  d and e track the inverse modulo p with one
// Montgomery-style correction per batch (the matrix divides by 2^62).
//
// The algorithm: D. J. Bernstein, B.-Y. Yang, "Fast constant-time gcd computation and modular
// inversion" (2019), in its variable-time form with eta = -delta and 62-step batches.  Checked against
// the oracle by tests/test_host_arith.py (the same code compiled for the host).
//
// Attribution.  divsteps_62_var, update_de_62, update_fg_62 and the limb-length reduction of
// inv_var below follow libsecp256k1's src/modinv64_impl.h (secp256k1_modinv64_divsteps_62_var,
// _update_de_62, _update_fg_62, _modinv64_var), re-parameterised for BLS12-381's p (7 signed
// 62-bit limbs, p^-1 mod 2^62) and for device code.  That file is distributed under the MIT license:
//
//   Copyright (c) 2020 Peter Dettman
//   Copyright (c) 2013 Pieter Wuille and the libsecp256k1 contributors
//
//   Permission is hereby granted, free of charge, to any person obtaining a copy of this software
//   and associated documentation files (the "Software"), to deal in the Software without
//   restriction, including without limitation the rights to use, copy, modify, merge, publish,
//   distribute, sublicense, and/or sell copies of the Software, and to permit persons to whom the
//   Software is furnished to do so, subject to the following conditions:
//
//   The above copyright notice and this permission notice shall be included in all copies or
//   substantial portions of the Software.
//
//   THE SOFTWARE IS PROVIDED "AS IS", WITHOUT WARRANTY OF ANY KIND, EXPRESS OR IMPLIED, INCLUDING
//   BUT NOT LIMITED TO THE WARRANTIES OF MERCHANTABILITY, FITNESS FOR A PARTICULAR PURPOSE AND
//   NONINFRINGEMENT. IN NO EVENT SHALL THE AUTHORS OR COPYRIGHT HOLDERS BE LIABLE FOR ANY CLAIM,
//   DAMAGES OR OTHER LIABILITY, WHETHER IN AN ACTION OF CONTRACT, TORT OR OTHERWISE, ARISING FROM,
//   OUT OF OR IN CONNECTION WITH THE SOFTWARE OR THE USE OR OTHER DEALINGS IN THE SOFTWARE.
#pragma once
#include "fp_types.h"
#include "bls_constants.h"

namespace gbv {
namespace sg {

constexpr int NL = 7;  // 7 x 62 = 434 bits > 381 + sign
constexpr int64_t M62 = (int64_t)(UINT64_MAX >> 2);
typedef __int128 i128;

struct S62 { int64_t v[NL]; };
struct T2 { int64_t u, v, q, r; };

// p in 62-bit limbs, and p^-1 mod 2^62
constexpr S62 P62 = {{0x39feffffffffaaabll, 0x3aaffffac54ffffell, 0x330d2a0f6b0f6241ll, 0x1dd2e13ce144afd9ll, 0x1ba7b6434bacd764ll,
                      0x447a8e5ff9a692cll, 0x1a0ll}};
constexpr uint64_t PINV62 = 0x360c000300030003ull;

GBV_HD int ctz64(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return (int)__builtin_ctzll(x);
#else
  return __builtin_ctzll(x);
#endif
}

// 62 divsteps on the low bits of f (odd) and g; returns the new eta, the transition matrix in t
// (scaled by 2^62: [u v; q r] applied to (f, g) gives 2^62 (f', g')).
GBV_HD int64_t divsteps_62_var(int64_t eta, uint64_t f0, uint64_t g0, T2* t) {
  uint64_t u = 1, v = 0, q = 0, r = 1;
  uint64_t f = f0, g = g0, m, w;
  int i = 62, limit, zeros;
  for (;;) {
    zeros = ctz64(g | (UINT64_MAX << i));  // runs of zero bits: one shift for the whole run
    g >>= zeros;
    u <<= zeros;
    v <<= zeros;
    eta -= zeros;
    i -= zeros;
    if (i == 0) break;
    if (eta < 0) {  // swap (f, g) = (g, -f) and the matrix rows
      uint64_t tmp;
      eta = -eta;
      tmp = f; f = g; g = 0 - tmp;
      tmp = u; u = q; q = 0 - tmp;
      tmp = v; v = r; r = 0 - tmp;
      limit = ((int)eta + 1) > i ? i : ((int)eta + 1);
      m = (UINT64_MAX >> (64 - limit)) & 63u;
      w = (f * g * (f * f - 2)) & m;  // -g / f mod 2^min(limit, 6)
    } else {
      limit = ((int)eta + 1) > i ? i : ((int)eta + 1);
      m = (UINT64_MAX >> (64 - limit)) & 15u;
      w = f + (((f + 1) & 4) << 1);   // 1 / f mod 16
      w = ((0 - w) * g) & m;          // -g / f mod 2^min(limit, 4)
    }
    g += f * w;
    q += u * w;
    r += v * w;
  }
  t->u = (int64_t)u;
  t->v = (int64_t)v;
  t->q = (int64_t)q;
  t->r = (int64_t)r;
  return eta;
}

// (d, e) <- [u v; q r] (d, e) / 2^62 mod p (a multiple of p added to make the low 62 bits vanish)
GBV_HD void update_de_62(S62& d, S62& e, const T2& t) {
  const int64_t u = t.u, v = t.v, q = t.q, r = t.r;
  const int64_t sd = d.v[NL - 1] >> 63, se = e.v[NL - 1] >> 63;
  int64_t md = (u & sd) + (v & se);
  int64_t me = (q & sd) + (r & se);
  i128 cd = (i128)u * d.v[0] + (i128)v * e.v[0];
  i128 ce = (i128)q * d.v[0] + (i128)r * e.v[0];
  md -= (int64_t)((PINV62 * (uint64_t)cd + (uint64_t)md) & (uint64_t)M62);
  me -= (int64_t)((PINV62 * (uint64_t)ce + (uint64_t)me) & (uint64_t)M62);
  cd += (i128)P62.v[0] * md;
  ce += (i128)P62.v[0] * me;
  cd >>= 62;
  ce >>= 62;
#pragma unroll
  for (int i = 1; i < NL; ++i) {
    cd += (i128)u * d.v[i] + (i128)v * e.v[i];
    ce += (i128)q * d.v[i] + (i128)r * e.v[i];
    cd += (i128)P62.v[i] * md;
    ce += (i128)P62.v[i] * me;
    d.v[i - 1] = (int64_t)cd & M62;
    cd >>= 62;
    e.v[i - 1] = (int64_t)ce & M62;
    ce >>= 62;
  }
  d.v[NL - 1] = (int64_t)cd;
  e.v[NL - 1] = (int64_t)ce;
}

// (f, g) <- [u v; q r] (f, g) / 2^62 over the first len limbs (exact: the low 62 bits are zero)
GBV_HD void update_fg_62(int len, S62& f, S62& g, const T2& t) {
  const int64_t u = t.u, v = t.v, q = t.q, r = t.r;
  i128 cf = (i128)u * f.v[0] + (i128)v * g.v[0];
  i128 cg = (i128)q * f.v[0] + (i128)r * g.v[0];
  cf >>= 62;
  cg >>= 62;
  for (int i = 1; i < len; ++i) {
    cf += (i128)u * f.v[i] + (i128)v * g.v[i];
    cg += (i128)q * f.v[i] + (i128)r * g.v[i];
    f.v[i - 1] = (int64_t)cf & M62;
    cf >>= 62;
    g.v[i - 1] = (int64_t)cg & M62;
    cg >>= 62;
  }
  f.v[len - 1] = (int64_t)cf;
  g.v[len - 1] = (int64_t)cg;
}

// r in (-2p, p) -> r * sign(sign) mod p in [0, p)
GBV_HD void normalize_62(S62& r, int64_t sign) {
  int64_t ca = r.v[NL - 1] >> 63;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.v[i] += P62.v[i] & ca;
  const int64_t cn = sign >> 63;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.v[i] = (r.v[i] ^ cn) - cn;
#pragma unroll
  for (int i = 0; i < NL - 1; ++i) {
    r.v[i + 1] += r.v[i] >> 62;
    r.v[i] &= M62;
  }
  ca = r.v[NL - 1] >> 63;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.v[i] += P62.v[i] & ca;
#pragma unroll
  for (int i = 0; i < NL - 1; ++i) {
    r.v[i + 1] += r.v[i] >> 62;
    r.v[i] &= M62;
  }
}

GBV_HD S62 from_fp(const Fp& a) {
  S62 s;
#pragma unroll
  for (int j = 0; j < NL; ++j) {
    const int b = 62 * j, w = b >> 5, o = b & 31;
    uint64_t x = 0;
    if (w < 12) x = (uint64_t)a.v[w] >> o;
    if (w + 1 < 12) x |= (uint64_t)a.v[w + 1] << (32 - o);
    if (w + 2 < 12 && 64 - o < 62) x |= (uint64_t)a.v[w + 2] << (64 - o);
    s.v[j] = (int64_t)(x & (uint64_t)M62);
  }
  return s;
}

GBV_HD Fp to_fp(const S62& s) {  // limbs in [0, 2^62), value < 2^384
  Fp a;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const int b = 32 * i, j = b / 62, o = b % 62;
    uint64_t x = (uint64_t)s.v[j] >> o;
    if (j + 1 < NL && 62 - o < 32) x |= (uint64_t)s.v[j + 1] << (62 - o);
    a.v[i] = (uint32_t)x;
  }
  return a;
}

// x^-1 mod p for the canonical integer x (0 -> 0)
GBV_HD Fp inv_raw(const Fp& x) {
  uint32_t nz = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) nz |= x.v[i];
  if (!nz) return x;
  S62 d = {{0, 0, 0, 0, 0, 0, 0}}, e = {{1, 0, 0, 0, 0, 0, 0}}, f = P62, g = from_fp(x);
  int len = NL;
  int64_t eta = -1;
  for (int guard = 0; guard < 64; ++guard) {  // ~12-15 batches for 381 bits; the guard never binds
    T2 t;
    eta = divsteps_62_var(eta, (uint64_t)f.v[0], (uint64_t)g.v[0], &t);
    update_de_62(d, e, t);
    update_fg_62(len, f, g, t);
    if (g.v[0] == 0) {
      int64_t cond = 0;
      for (int j = 1; j < len; ++j) cond |= g.v[j];
      if (cond == 0) break;
    }
    const int64_t fn = f.v[len - 1], gn = g.v[len - 1];
    int64_t cond = ((int64_t)len - 2) >> 63;
    cond |= fn ^ (fn >> 63);
    cond |= gn ^ (gn >> 63);
    if (cond == 0) {  // both top limbs are 0 or -1: drop a limb
      f.v[len - 2] |= (int64_t)((uint64_t)fn << 62);
      g.v[len - 2] |= (int64_t)((uint64_t)gn << 62);
      --len;
    }
  }
  normalize_62(d, f.v[len - 1]);  // f = +-1 now
  return to_fp(d);
}

}  // namespace sg
}  // namespace gbv
