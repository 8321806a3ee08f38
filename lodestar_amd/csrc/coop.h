// Wave-cooperative Fp12 arithmetic and pairing drivers for the latency-bound parts of
// verification (per-chunk Miller values, the shared final exponentiation, per-chunk retries).
//
// One workgroup = one wave (64 lanes) = one pairing job.  Field elements live in a per-wave LDS
// workspace (Ws); a program from coop_tables.h (tools/gen_coop.py) runs as
//   product rounds : lane k computes Z[k] = (sum of its A terms) * (sum of its B terms)
//   partial sums   : lane j sums <= 6 terms of a long output into Z
//   outputs        : lane o computes output coordinate o, then every lane stores after a barrier
// so an Fp12 product costs ~1 Fp product of latency instead of 54.  The same drivers compile for
// the host (GBV_HOST_TEST: the 64 lanes run one after another) and are checked against the
// oracle in tests/test_host_arith.py; tests/test_coop_tables.py checks the programs themselves.
#pragma once
#include "pairing.h"

#if defined(GBV_HOST_TEST)
#define GBV_COOP_TABLE static const
#else
#define GBV_COOP_TABLE __constant__ const
#endif

namespace gbv {
namespace coop {

struct Term { uint8_t src, idx; int16_t coef; };
// Fixed-size per-lane records (tools/gen_coop.py): product k = prods[20k .. 20k+19]
// (A terms 0..9, B terms 10..19), partial j = parts[8j ..] -> Z[n_prod + j], output o = outs[8o ..]
// -> operand out_dst[o], coordinate out_idx[o].  Padding terms have coef 0.
struct Prog {
  uint8_t n_rounds, n_part, n_out;
  uint16_t round_end[6];
  const Term* prods;
  const Term* parts;
  const Term* outs;
  const uint8_t* out_dst;
  const uint8_t* out_idx;
};
constexpr int OPW = 10;
enum { SRC_Z = 6, SRC_C = 7 };

}  // namespace coop
}  // namespace gbv

#include "coop_tables.h"

namespace gbv {
namespace coop {

constexpr int LANES = 64;
constexpr int ZSLOTS = 128;

// LDS-typed pointers so workspace accesses compile to ds_read/ds_write (a generic pointer would
// give flat instructions, which wait on both the vector-memory and LDS counters).
#if defined(GBV_HOST_TEST)
typedef Fp LFp;
#define GBV_LDS(p) (p)
#else
typedef __attribute__((address_space(3))) Fp LFp;
#define GBV_LDS(p) ((LFp*)(p))
#endif

GBV_HD Fp ld(const LFp* p) {
  Fp r;
  r.v = p->v;
  return r;
}
GBV_HD void st(LFp* p, const Fp& a) { p->v = a.v; }

// Per-wave workspace: mem[] is LDS on the device; operand k of a program lives at mem + op[k].
struct Ws {
  LFp* mem;
  uint16_t op[6];
  uint16_t z;
};

GBV_HD Term term_of(uint32_t u) { return Term{(uint8_t)u, (uint8_t)(u >> 8), (int16_t)(u >> 16)}; }

// Copy n (multiple of 4) terms into registers with 16-byte loads: one memory latency per record.
template <int N> GBV_HD void load_terms(uint32_t (&r)[N], const Term* t) {
  static_assert(N % 4 == 0, "records are whole 16-byte units");
  const uint4* q = (const uint4*)t;
#pragma unroll
  for (int i = 0; i < N / 4; ++i) {
    uint4 x = q[i];
    r[4 * i] = x.x;
    r[4 * i + 1] = x.y;
    r[4 * i + 2] = x.z;
    r[4 * i + 3] = x.w;
  }
}

GBV_HD Fp ws_get(const Ws& w, Term t) {
  if (t.src == SRC_C) return CONSTS[t.idx];
  uint32_t base = t.src == SRC_Z ? w.z : t.src == 0 ? w.op[0] : t.src == 1 ? w.op[1] : t.src == 2 ? w.op[2]
                 : t.src == 3 ? w.op[3] : t.src == 4 ? w.op[4] : w.op[5];
  return ld(w.mem + base + t.idx);
}

// c * v for a small integer c >= 2 (rare: scaled terms of the doubling/cyclotomic formulas)
GBV_NI Fp scale_small(Fp v, int c) {
  Fp s = v;
  bool have = false;
  while (c) {
    if (c & 1) {
      s = have ? fp_add(s, v) : v;
      have = true;
    }
    c >>= 1;
    if (c) v = fp_dbl(v);
  }
  return s;
}

// p - s for s < p, without reduction (s = 0 gives p, which every consumer below accepts: it only
// ever enters fp_add next to a value < p).
GBV_HD Fp fp_neg_raw(const Fp& s) {
  Fp d;
  raw_sub(d, P_RAW, s);
  return d;
}

// sum of coef * value over N packed terms: all N operand loads are issued first, then each term is
// conditionally negated / zeroed with selects and added -- no divergent branch per term (a lane's
// term count and signs differ from its neighbours').
template <int N> GBV_HD Fp lin_eval(const Ws& w, const uint32_t* r) {
  Fp v[N];
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = ws_get(w, term_of(r[i]));
  Fp acc = fp_zero();
#pragma unroll
  for (int i = 0; i < N; ++i) {
    int c = (int16_t)(r[i] >> 16);
    int m = c < 0 ? -c : c;
    Fp s = v[i];
    if (m > 1) s = scale_small(s, m);  // rare (doubling / cyclotomic constants)
    Fp t = fp_sel(c < 0, fp_neg_raw(s), s);
    t = fp_sel(c == 0, fp_zero(), t);
    acc = fp_add(acc, t);
  }
  return acc;
}

GBV_HD void prod_lane(const uint32_t (&r)[2 * OPW], int k, const Ws& w) {
  Fp x = lin_eval<OPW>(w, r);
  Fp y = lin_eval<OPW>(w, r + OPW);
  st(w.mem + w.z + k, fp_mul(x, y));
}

GBV_HD void part_lane(const Prog& P, const uint32_t (&r)[8], int j, const Ws& w) {
  st(w.mem + w.z + P.round_end[P.n_rounds - 1] + j, lin_eval<8>(w, r));
}

#if defined(GBV_HOST_TEST)
inline unsigned lane_id() { return 0; }
inline void barrier() {}

// Host: the lanes of each phase run one after another.
inline void run(const Prog& P, const Ws& w) {
  int p0 = 0;
  uint32_t rec[2 * OPW], r8[8];
  for (int r = 0; r < P.n_rounds; ++r) {
    for (int k = p0; k < P.round_end[r]; ++k) {
      load_terms(rec, P.prods + 2 * OPW * k);
      prod_lane(rec, k, w);
    }
    p0 = P.round_end[r];
  }
  for (int j = 0; j < P.n_part; ++j) {
    load_terms(r8, P.parts + 8 * j);
    part_lane(P, r8, j, w);
  }
  Fp o[LANES];
  for (int k = 0; k < P.n_out; ++k) {
    load_terms(r8, P.outs + 8 * k);
    o[k] = lin_eval<8>(w, r8);
  }
  for (int k = 0; k < P.n_out; ++k) st(w.mem + w.op[P.out_dst[k]] + P.out_idx[k], o[k]);
}
#define COOP_LANES(l) for (unsigned l = 0; l < (unsigned)LANES; ++l)
#define COOP_LANE0 if (true)
#else
__device__ inline unsigned lane_id() { return threadIdx.x; }
__device__ inline void barrier() { __syncthreads(); }

// All of a lane's records for this program are fetched up front (one memory latency), the next
// round's while the current round computes.
__device__ __noinline__ void run_ni(const Prog* PP, LFp* mem, uint32_t op01, uint32_t op23, uint32_t op45, uint32_t z) {
  const Prog& P = *PP;
  const Ws w{mem, {(uint16_t)op01, (uint16_t)(op01 >> 16), (uint16_t)op23, (uint16_t)(op23 >> 16), (uint16_t)op45, (uint16_t)(op45 >> 16)},
             (uint16_t)z};
  const int lane = (int)threadIdx.x;
  uint32_t rec[2 * OPW], rpart[8], rout[8];
  bool have_part = lane < P.n_part, have_out = lane < P.n_out;
  int p0 = 0;
  if (lane < P.round_end[0]) load_terms(rec, P.prods + 2 * OPW * lane);
  if (have_part) load_terms(rpart, P.parts + 8 * lane);
  if (have_out) load_terms(rout, P.outs + 8 * lane);
  for (int r = 0; r < P.n_rounds; ++r) {
    int p1 = P.round_end[r];
    if (p0 + lane < p1) prod_lane(rec, p0 + lane, w);  // every round has <= 64 products
    if (r + 1 < P.n_rounds && p1 + lane < P.round_end[r + 1]) load_terms(rec, P.prods + 2 * OPW * (p1 + lane));
    p0 = p1;
    __syncthreads();
  }
  if (have_part) part_lane(P, rpart, lane, w);
  if (P.n_part) __syncthreads();
  Fp o;
  if (have_out) o = lin_eval<8>(w, rout);
  __syncthreads();
  if (have_out) st(w.mem + w.op[P.out_dst[lane]] + P.out_idx[lane], o);
  __syncthreads();
}
// One out-of-line copy of the interpreter serves every call site (the drivers make hundreds).
__device__ inline void run(const Prog& P, const Ws& w) {
  run_ni(&P, w.mem, w.op[0] | ((uint32_t)w.op[1] << 16), w.op[2] | ((uint32_t)w.op[3] << 16), w.op[4] | ((uint32_t)w.op[5] << 16), w.z);
}
#define COOP_LANES(l) for (unsigned l = threadIdx.x; l == threadIdx.x; l = ~0u)
#define COOP_LANE0 if (threadIdx.x == 0)
#endif

// ---- operand helpers (lane-parallel, end with a barrier) ------------------------------------
GBV_HD void set_one12(Fp* fg) {
  LFp* f = GBV_LDS(fg);
  COOP_LANES(l) if (l < 12) st(f + l, l == 0 ? FP_ONE : fp_zero());
  barrier();
}
GBV_HD void copy(Fp* dstg, const Fp* srcg, unsigned n) {
  LFp* dst = GBV_LDS(dstg);
  const LFp* src = GBV_LDS(srcg);
  COOP_LANES(l) if (l < n) st(dst + l, ld(src + l));
  barrier();
}
GBV_HD void conj12(Fp* fg) {  // negate the w-odd half (coordinates 6..11)
  LFp* f = GBV_LDS(fg);
  COOP_LANES(l) if (l >= 6 && l < 12) st(f + l, fp_neg(ld(f + l)));
  barrier();
}
GBV_HD bool is_one12(const Fp* f) {
  bool ok = true;
  for (int i = 0; i < 12; ++i) ok = ok && fp_eq(f[i], i == 0 ? FP_ONE : fp_zero());
  return ok;
}

GBV_HD Ws ws2(Fp* mem, uint16_t z, uint16_t a, uint16_t b) { return Ws{GBV_LDS(mem), {a, b, 0, 0, 0, 0}, z}; }
GBV_HD Ws ws3(Fp* mem, uint16_t z, uint16_t a, uint16_t b, uint16_t c) { return Ws{GBV_LDS(mem), {a, b, c, 0, 0, 0}, z}; }

GBV_HD void mul12(Fp* mem, uint16_t z, uint16_t a, uint16_t b, uint16_t c) { run(FP12_MUL, ws3(mem, z, a, b, c)); }
GBV_HD void cyc_sqr12(Fp* mem, uint16_t z, uint16_t a, uint16_t c) { run(FP12_CYC_SQR, ws2(mem, z, a, c)); }
GBV_HD void frob12(Fp* mem, uint16_t z, int n, uint16_t a, uint16_t c) { run(n == 1 ? FP12_FROB1 : FP12_FROB2, ws2(mem, z, a, c)); }

// ---- Miller loop over up to 2 pairs ---------------------------------------------------------
// Workspace layout (Fp offsets), MILLER_WS Fp in total:
//   F 0..11 | L 12..17 | per pair j: T 18+12j (6), Q 24+12j (4), P 28+12j (2: -xP, yP) | Z 42..169
constexpr uint16_t M_F = 0, M_L = 12, M_PAIR = 18, M_Z = 42;
constexpr int MILLER_WS = M_Z + ZSLOTS;

// Load pair j: P affine G1, Q affine G2 (neither infinity).  Lane-parallel, ends with a barrier.
GBV_HD void miller_load_pair(Fp* mem, int j, const G1A& P, const G2A& Q) {
  LFp* b = GBV_LDS(mem + M_PAIR + 12 * j);
  COOP_LANES(l) {
    if (l < 12) {
      Fp v;
      switch (l) {
        case 0: v = Q.x.c0; break;
        case 1: v = Q.x.c1; break;
        case 2: v = Q.y.c0; break;
        case 3: v = Q.y.c1; break;
        case 4: v = FP_ONE; break;
        case 5: v = fp_zero(); break;
        case 6: v = Q.x.c0; break;
        case 7: v = Q.x.c1; break;
        case 8: v = Q.y.c0; break;
        case 9: v = Q.y.c1; break;
        case 10: v = fp_neg(P.x); break;
        default: v = P.y; break;
      }
      st(b + l, v);
    }
  }
  barrier();
}

// F = prod_j f_{|x|, Q_j}(P_j), conjugated (x < 0).  Pairs must be loaded first.
GBV_HD void miller_loop(Fp* mem, int npairs) {
  set_one12(mem + M_F);
  for (int i = 62; i >= 0; --i) {
    if (i != 62) run(FP12_SQR, ws2(mem, M_Z, M_F, M_F));
    for (int j = 0; j < npairs; ++j) {
      uint16_t t = M_PAIR + 12 * j;
      run(G2_DBL_STEP, Ws{GBV_LDS(mem), {t, (uint16_t)(t + 10), t, M_L, 0, 0}, M_Z});
      run(FP12_MUL_LINE, ws3(mem, M_Z, M_F, M_L, M_F));
    }
    if ((X_ABS >> i) & 1ull) {
      for (int j = 0; j < npairs; ++j) {
        uint16_t t = M_PAIR + 12 * j;
        run(G2_ADD_STEP, Ws{GBV_LDS(mem), {t, (uint16_t)(t + 6), (uint16_t)(t + 10), t, M_L, 0}, M_Z});
        run(FP12_MUL_LINE, ws3(mem, M_Z, M_F, M_L, M_F));
      }
    }
  }
  conj12(mem + M_F);
}

// ---- final exponentiation: f^(3 (p^12 - 1)/r) == 1 ? -----------------------------------------
// Workspace (Fp offsets): F 0..11 (input, clobbered) | INV 12 | T 24 | A 36 | B 48 | C 60 |
// TMP 72 | TMP2 84 | Z 96..223
constexpr uint16_t E_F = 0, E_INV = 12, E_T = 24, E_A = 36, E_B = 48, E_C = 60, E_TMP = 72, E_TMP2 = 84, E_Z = 96;
constexpr int FINAL_EXP_WS = E_Z + ZSLOTS;

GBV_HD Fp12 load12(const Fp* f) {
  Fp12 r;
  Fp* d = (Fp*)&r;
  for (int i = 0; i < 12; ++i) d[i] = f[i];
  return r;
}
GBV_HD void store12(Fp* f, const Fp12& a) {
  const Fp* s = (const Fp*)&a;
  for (int i = 0; i < 12; ++i) f[i] = s[i];
}

// r = a^x (a in the cyclotomic subgroup)
GBV_HD void exp_x(Fp* mem, uint16_t a, uint16_t r) {
  copy(mem + r, mem + a, 12);
  for (int i = 62; i >= 0; --i) {
    cyc_sqr12(mem, E_Z, r, r);
    if ((X_ABS >> i) & 1ull) mul12(mem, E_Z, r, a, r);
  }
  conj12(mem + r);
}

// f (at mem + E_F) -> returns f^(3 (p^12-1)/r) == 1 (same value on every lane)
GBV_HD bool final_exp_is_one(Fp* mem) {
  COOP_LANE0 store12(mem + E_INV, fp12_inv(load12(mem + E_F)));  // one scalar inversion
  barrier();
  conj12(mem + E_F);
  mul12(mem, E_Z, E_F, E_INV, E_T);       // t = f^(p^6 - 1)
  frob12(mem, E_Z, 2, E_T, E_TMP);
  mul12(mem, E_Z, E_TMP, E_T, E_T);       // t = t^(p^2 + 1)
  exp_x(mem, E_T, E_A);
  copy(mem + E_TMP, mem + E_T, 12);
  conj12(mem + E_TMP);
  mul12(mem, E_Z, E_A, E_TMP, E_A);       // a = t^(x - 1)
  exp_x(mem, E_A, E_TMP);
  conj12(mem + E_A);
  mul12(mem, E_Z, E_TMP, E_A, E_A);       // a = a^(x - 1)
  exp_x(mem, E_A, E_TMP);
  frob12(mem, E_Z, 1, E_A, E_TMP2);
  mul12(mem, E_Z, E_TMP, E_TMP2, E_B);    // b = a^(x + p)
  exp_x(mem, E_B, E_TMP);
  exp_x(mem, E_TMP, E_C);
  frob12(mem, E_Z, 2, E_B, E_TMP);
  mul12(mem, E_Z, E_C, E_TMP, E_C);
  conj12(mem + E_B);
  mul12(mem, E_Z, E_C, E_B, E_C);         // c = b^(x^2 + p^2 - 1)
  cyc_sqr12(mem, E_Z, E_T, E_TMP);
  mul12(mem, E_Z, E_TMP, E_T, E_TMP);     // t^3
  mul12(mem, E_Z, E_C, E_TMP, E_C);
  return is_one12(mem + E_C);
}

}  // namespace coop
}  // namespace gbv
