// Fp arithmetic for BLS12-381 on the gfx950 integer VALU.
//
// One thread owns one element: 12 x 32-bit limbs in VGPRs, Montgomery form.  Multiplication is
// CIOS Montgomery with the "no final carry" shortcut (top limb of p < 2^31), so every
// limb product is one v_mad_u64_u32 (u32 x u32 + u64 -> u64) -- measured full-rate on MI355X
// (tools/ubench_int.hip).  There is no floating point anywhere in this library.
//
// The blst operations this replaces: mul_fp / sqr_fp / add_fp / sub_fp /
// sqrt_fp / reciprocal_fp inside @chainsafe/blst 2.1.0 (yarn.lock:446-457).
#pragma once
#include "fp_types.h"
#include "bls_constants.h"
#include "fp_asm.h"
#include "inv_sg.h"

namespace gbv {

GBV_HD Fp fp_zero() {
  Fp r;
#pragma unroll
  for (int i = 0; i < 12; ++i) r.v[i] = 0;
  return r;
}

GBV_HD bool fp_is_zero(const Fp& a) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) acc |= a.v[i];
  return acc == 0;
}

GBV_HD bool fp_eq(const Fp& a, const Fp& b) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) acc |= a.v[i] ^ b.v[i];
  return acc == 0;
}

// r = c ? a : b  (branch-free select; the compiler emits v_cndmask)
GBV_HD Fp fp_sel(bool c, const Fp& a, const Fp& b) {
  Fp r;
#pragma unroll
  for (int i = 0; i < 12; ++i) r.v[i] = c ? a.v[i] : b.v[i];
  return r;
}

// Raw 384-bit helpers ------------------------------------------------------------------------
// s = a - b, returns borrow (1 if a < b).  __builtin_subc/__builtin_addc lower to one
// v_sub_co/v_subb_co (v_add_co/v_addc_co) carry chain: 12 VALU ops per 384-bit add or subtract.
GBV_HD uint32_t raw_sub(Fp& s, const Fp& a, const Fp& b) {
  unsigned br = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) s.v[i] = __builtin_subc(a.v[i], b.v[i], br, &br);
  return br;
}

GBV_HD uint32_t raw_add(Fp& s, const Fp& a, const Fp& b) {
  unsigned c = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) s.v[i] = __builtin_addc(a.v[i], b.v[i], c, &c);
  return c;
}

#if defined(__HIP_DEVICE_COMPILE__)
// Device: each modular add/sub is one inline-asm carry chain (fp_asm.h).  Written this way the
// chain links issue back to back; compiled from C the gfx950 backend pads every VCC hand-off.
GBV_HD Fp fp_reduce_once(const Fp& x) {
  Fp r;
  const Fp p = P_RAW;
  GBV_ASM_REDUCE_ONCE(r, x, p);
  return r;
}

GBV_HD Fp fp_add(const Fp& a, const Fp& b) {
  Fp s, r;
  const Fp p = P_RAW;
  GBV_ASM_ADD_MOD(s, r, a, b, p);
  return r;
}

GBV_HD Fp fp_sub(const Fp& a, const Fp& b) {
  Fp d, m;
  const Fp p = P_RAW;
  GBV_ASM_SUB_MOD(d, m, a, b, p);
  return d;
}

GBV_HD Fp fp_neg(const Fp& a) { return fp_sub(fp_zero(), a); }
#else
// reduce x in [0, 2p) to [0, p)
GBV_HD Fp fp_reduce_once(const Fp& x) {
  Fp t;
  uint32_t br = raw_sub(t, x, P_RAW);
  return fp_sel(br != 0, x, t);
}

GBV_HD Fp fp_add(const Fp& a, const Fp& b) {
  Fp s;
  raw_add(s, a, b);  // < 2p < 2^382: no carry out
  return fp_reduce_once(s);
}

GBV_HD Fp fp_sub(const Fp& a, const Fp& b) {
  Fp d, t;
  uint32_t br = raw_sub(d, a, b);
  raw_add(t, d, P_RAW);
  return fp_sel(br != 0, t, d);
}

GBV_HD Fp fp_neg(const Fp& a) {
  Fp d;
  raw_sub(d, P_RAW, a);
  return fp_sel(fp_is_zero(a), a, d);
}
#endif

GBV_HD Fp fp_dbl(const Fp& a) { return fp_add(a, a); }

// m x mod p for canonical x and 2 <= m < 2^16 (the scaled terms of the cooperative programs: 3b
// multiples up to 144): r = m x as 13 limbs (one multiply-add chain), q = floor(r_top / (p_11 + 1))
// from r's top 45 bits in double precision -- exact for these magnitudes and at most one below
// floor(r / p) -- then r - q p < 2p and one conditional subtraction.  ~60 VALU ops against ~300 for
// a double-and-add chain of modular doublings.
GBV_HD Fp fp_mul_small(const Fp& x, uint32_t m) {
  uint32_t r[13];
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    c += (uint64_t)x.v[i] * m;
    r[i] = (uint32_t)c;
    c >>= 32;
  }
  r[12] = (uint32_t)c;
  const double top = (double)r[12] * 4294967296.0 + (double)r[11];
  const uint32_t q = (uint32_t)(top * (1.0 / 436277739.0));  // p_11 + 1 = 0x1a0111eb
  Fp d;
  uint64_t s = 0;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    s += (uint64_t)P_RAW.v[i] * q;
    d.v[i] = __builtin_subc(r[i], (uint32_t)s, br, &br);
    s >>= 32;
  }
  return fp_reduce_once(d);
}

// Lazy forms for values that only feed a product: the product takes any input below 2^384 (fp_to28)
// and its Montgomery output stays below 1.02 p for inputs below 7 p (7p x 7p / 2^392 < 0.02 p), so
// the conditional subtraction of a modular add/sub is skipped.  fp_sub_lazy4: a + 4p - b for b < 4p.
static constexpr Fp P4_RAW = {{0xfffeaaacu, 0xe7fbffffu, 0xc54ffffeu, 0x7aaffffau, 0xdac3d890u, 0x9cc34a83u, 0xce144afdu,
                               0x91dd2e13u, 0x0d2eb35du, 0x2c6e9ed9u, 0xe5ff9a69u, 0x680447a8u}};  // 4 p < 2^383
static constexpr Fp P2_RAW = {{0xffff5556u, 0x73fdffffu, 0x62a7ffffu, 0x3d57fffdu, 0xed61ec48u, 0xce61a541u, 0xe70a257eu,
                               0xc8ee9709u, 0x869759aeu, 0x96374f6cu, 0x72ffcd34u, 0x340223d4u}};  // 2 p
#if defined(__HIP_DEVICE_COMPILE__)
GBV_HD Fp fp_add_lazy(const Fp& a, const Fp& b) {
  Fp s;
  GBV_ASM_ADD_RAW(s, a, b);
  return s;
}
// x in [0, 8p) (a raw sum of up to 8 canonical values) -> [0, p): conditional subtractions of 4p, 2p, p
GBV_HD Fp fp_reduce8(const Fp& x) {
  Fp a, b, c;
  const Fp k4 = P4_RAW, k2 = P2_RAW, k1 = P_RAW;
  GBV_ASM_REDUCE_ONCE(a, x, k4);
  GBV_ASM_REDUCE_ONCE(b, a, k2);
  GBV_ASM_REDUCE_ONCE(c, b, k1);
  return c;
}
GBV_HD Fp fp_sub_lazy4(const Fp& a, const Fp& b) {
  Fp t, d;
  const Fp k = P4_RAW;
  GBV_ASM_SUB_RAW_K(t, d, a, b, k);
  return d;
}
// In-place forms for accumulators (the asm output is the input's registers: no copies at joins)
GBV_HD void fp_acc_lazy(Fp& acc, const Fp& b) { GBV_ASM_ACC_RAW(acc, b); }
GBV_HD void fp_reduce8_ip(Fp& x) {
  Fp t;
  const Fp k4 = P4_RAW, k2 = P2_RAW, k1 = P_RAW;
  GBV_ASM_REDUCE_IP(x, t, k4);
  GBV_ASM_REDUCE_IP(x, t, k2);
  GBV_ASM_REDUCE_IP(x, t, k1);
}
#else
GBV_HD Fp fp_add_lazy(const Fp& a, const Fp& b) {
  Fp s;
  raw_add(s, a, b);
  return s;
}
GBV_HD Fp fp_reduce8(const Fp& x) {
  Fp t, y = x;
  if (!raw_sub(t, y, P4_RAW)) y = t;
  if (!raw_sub(t, y, P2_RAW)) y = t;
  if (!raw_sub(t, y, P_RAW)) y = t;
  return y;
}
GBV_HD Fp fp_sub_lazy4(const Fp& a, const Fp& b) {
  Fp t, d;
  raw_add(t, a, P4_RAW);
  raw_sub(d, t, b);
  return d;
}
GBV_HD void fp_acc_lazy(Fp& acc, const Fp& b) { raw_add(acc, acc, b); }
GBV_HD void fp_reduce8_ip(Fp& x) { x = fp_reduce8(x); }
#endif

// ---- the product: 14 x 28-bit limbs, Montgomery radix R = 2^392 ---------------------------------
// An element is stored as 12 x 32-bit limbs (adds, subtracts and comparisons use the hardware carry
// chain), but multiplied as 14 limbs of 28 bits: a column of up to 14 a_i b_j and 14 m_i p_j
// products of 56 bits sums below 2^61, so each limb product is ONE v_mad_u64_u32 into a plain
// 64-bit accumulator -- no carry word, no carry instruction -- where the 32-bit FIPS form needs a
// v_addc per product to catch the 96-bit column's carry.  Counted on the gfx950 code: 479
// instructions per product against 673 (288 mad + 288 addc + 97) for 32-bit limbs.
// The output of mul28_inl is < 2p for inputs < 2p (4p^2 < R p); fp_mul_inl reduces it once.
// (Splitting a column into two accumulation chains measured no faster at 2 waves/SIMD.)
typedef uint32_t u32x14 __attribute__((ext_vector_type(14)));
struct F28 { u32x14 v; };
constexpr uint32_t M28 = 0xFFFFFFFu;

GBV_HD F28 fp_to28(const Fp& a) {  // the same integer in 28-bit limbs
  F28 r;
#pragma unroll
  for (int j = 0; j < 14; ++j) {
    const int w = (28 * j) >> 5, o = (28 * j) & 31;
    uint32_t v = a.v[w] >> o;
    if (o > 4 && w + 1 < 12) v |= a.v[w + 1] << (32 - o);
    r.v[j] = v & M28;
  }
  return r;
}

GBV_HD Fp fp_from28(const F28& z) {  // z < 2^384, limbs < 2^28
  Fp r;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const int j = (32 * i) / 28, o = (32 * i) % 28;
    uint32_t v = z.v[j] >> o;
    if (j + 1 < 14) v |= z.v[j + 1] << (28 - o);
    if (j + 2 < 14 && 56 - o < 32) v |= z.v[j + 2] << (56 - o);
    r.v[i] = v;
  }
  return r;
}

// Column carry of the product scans: s >> 28 (arithmetic; unsigned columns stay below 2^63).  The 64-bit
// shift issues at half the rate of v_mad_u64_u32 in isolation (tools/ubench_int2.hip: 19.3 vs 36.6 T
// lane-ops/s), but inside the product it is on the carry chain beside the column's mads, and the
// two-instruction form (v_alignbit_b32 + v_ashrrev_i32, GBV_SAR28=1) measured slower there.
// (The halves go through an ext_vector bit cast: rebuilt with shifts and ors, the backend adds a zero
// move and two 64-bit adds per column.)
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
#ifndef GBV_SAR28
#define GBV_SAR28 0  // 1: the two 32-bit ops below -- measured SLOWER than the 64-bit shift in the product
#endif              // (tools/ubench_prod.hip, profiles/r06f: mul28s 68.8 -> 66.0 G/s at 2 waves per SIMD)
GBV_HD int64_t sar28(int64_t s) {
#if defined(__HIP_DEVICE_COMPILE__) && GBV_SAR28
  const u32x2 w = __builtin_bit_cast(u32x2, s);
  u32x2 r;
  r.x = __builtin_amdgcn_alignbit(w.y, w.x, 28);
  r.y = (uint32_t)((int32_t)w.y >> 28);
  return __builtin_bit_cast(int64_t, r);
#else
  return s >> 28;
#endif
}

#if defined(GBV_HOST_TEST)
// Host build only (tests/native/hosttest.cpp): every Fp product is counted, so the algorithmic work
// per signature set that bench.py's roofline uses is measured on the code, not estimated.
inline unsigned long long g_fme_count = 0;
#endif

// a b 2^-392 mod p (< 2p) by product scanning: column k of a*b and of m*p in one 64-bit
// accumulator, m_k from the column's low 28 bits for k < 14, output limb k-14 for k >= 14.  (Two or
// four independent accumulators per column were measured, in C and as generated asm: LLVM
// reassociates the C form back into one chain, and the asm form issued no faster)
GBV_HD F28 mul28_inl(const F28& a, const F28& b) {
#if defined(GBV_HOST_TEST)
  ++g_fme_count;
#endif
  uint32_t m[14], r[14];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 27; ++k) {
#pragma unroll
    for (int i = 0; i < 14; ++i) {
      const int j = k - i;
      if (j >= 0 && j < 14) acc += (uint64_t)a.v[i] * b.v[j];
    }
#pragma unroll
    for (int i = 0; i < 14; ++i) {
      const int j = k - i;
      if (i < k && j >= 0 && j < 14) acc += (uint64_t)m[i] * P28[j];
    }
    uint64_t s = acc;
    if (k < 14) {
      m[k] = ((uint32_t)s * NP28) & M28;
      s += (uint64_t)m[k] * P28[0];
    } else {
      r[k - 14] = (uint32_t)s & M28;
    }
    acc = (uint64_t)sar28((int64_t)s);
  }
  r[13] = (uint32_t)acc;
  F28 o;
#pragma unroll
  for (int i = 0; i < 14; ++i) o.v[i] = r[i];
  return o;
}

// a^2 2^-392 mod p (< 2p): the same column scan with the 91 cross products a_i (2 a_j), i < j, and
// the 14 squares a_i^2 -- 105 limb products instead of 196.  Column bound: 7 cross products
// < 2^57, one square < 2^56, 14 m_i p_j < 2^56 and the carried 2^36: below 2^62.
GBV_HD F28 sqr28_inl(const F28& a) {
#if defined(GBV_HOST_TEST)
  ++g_fme_count;
#endif
  uint32_t d[14], m[14], r[14];
#pragma unroll
  for (int i = 0; i < 14; ++i) d[i] = a.v[i] << 1;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 27; ++k) {
#pragma unroll
    for (int i = 0; i < 14; ++i) {
      const int j = k - i;
      if (i < j && j < 14) acc += (uint64_t)a.v[i] * d[j];
    }
    if ((k & 1) == 0 && (k >> 1) < 14) acc += (uint64_t)a.v[k >> 1] * a.v[k >> 1];
#pragma unroll
    for (int i = 0; i < 14; ++i) {
      const int j = k - i;
      if (i < k && j >= 0 && j < 14) acc += (uint64_t)m[i] * P28[j];
    }
    uint64_t s = acc;
    if (k < 14) {
      m[k] = ((uint32_t)s * NP28) & M28;
      s += (uint64_t)m[k] * P28[0];
    } else {
      r[k - 14] = (uint32_t)s & M28;
    }
    acc = (uint64_t)sar28((int64_t)s);
  }
  r[13] = (uint32_t)acc;
  F28 o;
#pragma unroll
  for (int i = 0; i < 14; ++i) o.v[i] = r[i];
  return o;
}

// Montgomery product a b R^-1 mod p, R = 2^392.  Inputs < p, output < p.
GBV_HD Fp fp_mul_inl(const Fp& a, const Fp& b) { return fp_reduce_once(fp_from28(mul28_inl(fp_to28(a), fp_to28(b)))); }
GBV_HD Fp fp_sqr_inl(const Fp& a) { return fp_reduce_once(fp_from28(sqr28_inl(fp_to28(a)))); }

// Out-of-line versions: keep the hot loops of the big kernels inside the instruction cache.
GBV_NI Fp fp_mul(Fp a, Fp b) { return fp_mul_inl(a, b); }
GBV_NI Fp fp_sqr(Fp a) { return fp_sqr_inl(a); }

GBV_HD Fp fp_to_mont(const Fp& raw) { return fp_mul(raw, R2_RAW); }

GBV_HD Fp fp_from_mont(const Fp& a) {
  Fp one = fp_zero();
  one.v[0] = 1;
  return fp_mul(a, one);
}

// Exponentiations stay in the 28-bit limb form from the first product to the last: every step is
// a bare mul28 (479 instructions, no repacking, no final reduction -- the values stay < 2p).
GBV_NI F28 mul28(F28 a, F28 b) { return mul28_inl(a, b); }
GBV_NI F28 sqr28(F28 a) { return sqr28_inl(a); }
GBV_HD F28 f28_sel(bool c, const F28& a, const F28& b) {
  F28 r;
#pragma unroll
  for (int i = 0; i < 14; ++i) r.v[i] = c ? a.v[i] : b.v[i];
  return r;
}

// a^e for a fixed public exponent (12 little-endian words, top bit index nbits-1).
// Square-and-multiply; the branch is on the public exponent so all lanes agree.
GBV_NI Fp fp_pow(Fp a, const uint32_t* e, int nbits) {
  const F28 x = fp_to28(a);
  F28 r = x;
  for (int i = nbits - 2; i >= 0; --i) {
    r = sqr28(r);
    if ((e[i >> 5] >> (i & 31)) & 1) r = mul28(r, x);
  }
  return fp_reduce_once(fp_from28(r));
}

// a^e for a fixed public exponent given as a sliding-window schedule (tools/gen_constants.py
// c_sched): table of odd powers a^1..a^15, ~76 multiplications for a 379-bit exponent instead of
// ~228 by square-and-multiply.  The table index is wave-uniform; picked with selects.
GBV_NI Fp fp_pow_sched(Fp a, const uint8_t* nsq, const uint8_t* idx, int steps) {
  F28 t[8];
  t[0] = fp_to28(a);
  const F28 a2 = sqr28(t[0]);
#pragma unroll
  for (int j = 1; j < 8; ++j) t[j] = mul28(t[j - 1], a2);
  auto pick = [&](uint32_t k) {
    F28 s = t[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) s = f28_sel(k == (uint32_t)j, t[j], s);
    return s;
  };
  F28 r = pick(idx[0]);
  for (int s = 1; s < steps; ++s) {
    for (int q = 0; q < nsq[s]; ++q) r = sqr28(r);
    if (idx[s] != 255) r = mul28(r, pick(idx[s]));
  }
  return fp_reduce_once(fp_from28(r));
}

GBV_HD Fp fp_inv_pow(const Fp& a) { return fp_pow(a, EXP_INV, EXP_INV_BITS); }  // 0 -> 0

// x / 2 mod p (x < p): (x + (x odd ? p : 0)) >> 1, the sum < 2p < 2^382 never carries out
GBV_HD Fp fp_half(const Fp& x) {
  Fp t;
  raw_add(t, x, P_RAW);
  t = fp_sel(x.v[0] & 1u, t, x);
  Fp r;
#pragma unroll
  for (int i = 0; i < 11; ++i) r.v[i] = (t.v[i] >> 1) | (t.v[i + 1] << 31);
  r.v[11] = t.v[11] >> 1;
  return r;
}

// Inverse by safegcd divsteps (inv_sg.h): (a R)^-1 R^3 R^-1 = a^-1 R.  0 -> 0.
GBV_NI Fp fp_inv(Fp a) {
  return fp_mul(sg::inv_raw(a), R3_RAW);
}

// Canonical (non-Montgomery) value comparisons used by sign rules ----------------------------
// true iff canonical(a) > (p-1)/2
GBV_HD bool fp_is_lexi_large(const Fp& a_mont) {
  Fp c = fp_from_mont(a_mont);
  Fp t;
  uint32_t br = raw_sub(t, P_HALF_RAW, c);  // borrow iff half < c
  return br != 0;
}

GBV_HD uint32_t fp_parity(const Fp& a_mont) { return fp_from_mont(a_mont).v[0] & 1u; }

// Big-endian 48-byte decoding/encoding -------------------------------------------------------
// Loads 48 big-endian bytes (optionally masking the top 3 flag bits) into raw limbs.
GBV_HD Fp fp_load_be48(const uint8_t* b, bool mask_flags) {
  Fp r;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const uint8_t* q = b + 44 - 4 * i;
    r.v[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | (uint32_t)q[3];
  }
  if (mask_flags) r.v[11] &= 0x1fffffffu;
  return r;
}

GBV_HD void fp_store_be48(uint8_t* b, const Fp& raw) {
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    uint8_t* q = b + 44 - 4 * i;
    uint32_t w = raw.v[i];
    q[0] = (uint8_t)(w >> 24);
    q[1] = (uint8_t)(w >> 16);
    q[2] = (uint8_t)(w >> 8);
    q[3] = (uint8_t)w;
  }
}

// raw < p ?
GBV_HD bool fp_raw_is_canonical(const Fp& raw) {
  Fp t;
  return raw_sub(t, raw, P_RAW) != 0;
}

// Square root candidate a^((p+1)/4); caller checks r^2 == a.
GBV_HD Fp fp_sqrt_candidate(const Fp& a) { return fp_pow_sched(a, SCHED_SQRT_NSQ, SCHED_SQRT_IDX, SCHED_SQRT_STEPS); }

}  // namespace gbv
