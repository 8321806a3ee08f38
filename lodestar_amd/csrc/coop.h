// Wave-cooperative Fp12 arithmetic and pairing drivers for the latency-bound parts of
// verification (per-chunk Miller values, the shared final exponentiation, per-chunk retries).
//
// One workgroup = one wave (64 lanes) = one pairing job.  Field elements live in a per-wave LDS
// workspace of Slots -- each Fp stored next to its negation, so a signed term of a linear
// combination is ONE LDS load and ONE modular add; a program from coop_tables.h
// (tools/gen_coop.py) runs as
//   product rounds : lane k computes Z[k] = (sum of its A terms) * (sum of its B terms)
//   partial sums   : lane j sums <= 6 terms of a long output into Z
//   outputs        : lane o computes output coordinate o, then every lane stores after a barrier
// with term lists of their true length (records carry the counts; positive terms first), so an
// Fp12 multiplication costs about one Fp product plus a few dozen adds of latency instead of 54
// products.  The Miller loop's line products and the final exponentiation's cyclotomic squarings
// are written out instead (mul_line, cyc_sqr: two phases, no records).  The same drivers compile for the host (GBV_HOST_TEST: the 64 lanes run one after
// another) and are checked against the oracle in tests/test_host_arith.py;
// tests/test_coop_tables.py checks the programs themselves.
#pragma once
#include "pairing.h"

#if defined(GBV_HOST_TEST)
#define GBV_COOP_TABLE static const
#else
#define GBV_COOP_TABLE __constant__ const
#endif

namespace gbv {
namespace coop {

// Per-lane records (tools/gen_coop.py): a product record is PROD_WORDS u32 -- header
// (npos_A | nneg_A << 8 | npos_B << 16 | nneg_B << 24), OPW A terms, OPW B terms, scaled-term
// counts (nsc_A | nsc_B << 8), padding -- a partial-sum / output record is SUM_WORDS u32 -- header
// (npos | nneg << 8 | nsc << 16), SUM_TERMS terms.  A term is src (bits 0-2) | neg << 4 | idx << 8 |
// magnitude << 16.  Unit terms come first (+1 then -1: the sign is the position), the rare scaled
// terms (|coefficient| > 1, sign in bit 4) last.
struct Prog {
  uint8_t n_rounds, n_part, n_out;
  uint16_t round_end[6];
  uint8_t amax[6], bmax[6];  // per round: the largest unit-term count of the A / B operands
  uint8_t pmax, omax;        // the same for the partial sums and the outputs
  const uint32_t* prods;
  const uint32_t* parts;
  const uint32_t* outs;
  const uint8_t* out_dst;
  const uint8_t* out_idx;
};
constexpr int OPW = 10;
constexpr int PROD_WORDS = 24;
constexpr int SUM_WORDS = 12, SUM_TERMS = 11;
enum { SRC_Z = 6, SRC_C = 7 };
constexpr int N_CONSTS_MAX = 16;

}  // namespace coop
}  // namespace gbv

#include "coop_tables.h"

namespace gbv {
namespace coop {

constexpr int LANES = 64;
constexpr int ZSLOTS = 128;

// A workspace slot: the value and its negation (p - v, and 0 for 0).
struct Slot {
  Fp v, n;
};

// LDS-typed pointers so workspace accesses compile to ds_read/ds_write (a generic pointer would
// give flat instructions, which wait on both the vector-memory and LDS counters).
#if defined(GBV_HOST_TEST)
typedef Slot LSlot;
#define GBV_LDS(p) (p)
#else
typedef __attribute__((address_space(3))) Slot LSlot;
#define GBV_LDS(p) ((LSlot*)(p))
#endif

GBV_HD Fp get(const LSlot* s) {
  Fp r;
  r.v = s->v.v;
  return r;
}
GBV_HD Fp get_signed(const LSlot* s, bool neg) {
  Fp r;
  r.v = neg ? s->n.v : s->v.v;
  return r;
}
GBV_HD void put(LSlot* s, const Fp& a) {
  s->v.v = a.v;
  s->n.v = fp_neg(a).v;
}
GBV_HD void put_pair(LSlot* s, const Fp& a, const Fp& na) {
  s->v.v = a.v;
  s->n.v = na.v;
}
#if !defined(GBV_HOST_TEST)
// generic-pointer forms for callers holding a plain Slot* into __shared__ memory
__device__ inline Fp get(const Slot* s) { return get(GBV_LDS(s)); }
__device__ inline void put(Slot* s, const Fp& a) { put(GBV_LDS(s), a); }
#endif

// The constant pool, in LDS so that every term source is a workspace load.
#if defined(GBV_HOST_TEST)
inline Slot g_consts[N_CONSTS_MAX];
#define GBV_CONSTS_LDS (g_consts)
#else
__shared__ Slot g_consts[N_CONSTS_MAX];
#define GBV_CONSTS_LDS GBV_LDS(g_consts)
#endif

// Per-wave workspace addressing.  Operand k of a program lives at workspace slot op[k], the
// program's scratch Z at slot z, the constant pool in g_consts.
#if defined(GBV_HOST_TEST)
struct Ws {
  LSlot* mem;
  uint16_t op[6];
  uint16_t z;
};
inline Ws make_ws(Slot* mem, uint16_t z, uint16_t o0, uint16_t o1 = 0, uint16_t o2 = 0, uint16_t o3 = 0, uint16_t o4 = 0,
                  uint16_t o5 = 0) {
  return Ws{mem, {o0, o1, o2, o3, o4, o5}, z};
}
inline LSlot* ws_slot(const Ws& w, uint32_t src, uint32_t idx) {
  if (src == SRC_C) return GBV_CONSTS_LDS + idx;
  return w.mem + (src == SRC_Z ? w.z : w.op[src]) + idx;
}
inline Fp term_load(const Ws& w, uint32_t t, uint32_t neg) {
  const LSlot* s = ws_slot(w, t & 7, (t >> 8) & 0xFF);
  return neg ? s->n : s->v;
}
inline void ws_put(const Ws& w, uint32_t src, uint32_t idx, const Fp& a) { put(ws_slot(w, src, idx), a); }
#else
// Device: every source is an absolute LDS address in 64-byte units (a Slot is two units: the value,
// then its negation), packed as 16-bit bases -- op0|op1, op2|op3, op4|op5, Z|consts -- so a term's
// address is two selects, a shift and an add, and the load reads exactly one Fp.
typedef __attribute__((address_space(3))) Fp LFp;
struct Ws {
  uint32_t b[4];
};
__device__ inline uint32_t lds_unit(const LSlot* p) { return (uint32_t)(size_t)p >> 6; }
__device__ inline Ws make_ws(Slot* mem, uint16_t z, uint16_t o0, uint16_t o1 = 0, uint16_t o2 = 0, uint16_t o3 = 0, uint16_t o4 = 0,
                             uint16_t o5 = 0) {
  const uint32_t m = lds_unit(GBV_LDS(mem));
  auto u = [m](uint16_t o) { return m + 2u * o; };
  return Ws{{u(o0) | u(o1) << 16, u(o2) | u(o3) << 16, u(o4) | u(o5) << 16, u(z) | lds_unit(GBV_CONSTS_LDS) << 16}};
}
// branch-free: a term's source differs per lane, and a select chain written as ?: compiled to
// exec-mask branches around every term
__device__ inline uint32_t ws_unit(const Ws& w, uint32_t src, uint32_t idx) {
  const uint32_t m1 = 0u - ((src >> 1) & 1u), m2 = 0u - ((src >> 2) & 1u);
  const uint32_t w01 = w.b[0] ^ ((w.b[0] ^ w.b[1]) & m1);
  const uint32_t w23 = w.b[2] ^ ((w.b[2] ^ w.b[3]) & m1);
  const uint32_t word = w01 ^ ((w01 ^ w23) & m2);
  return ((word >> ((src & 1u) << 4)) & 0xFFFFu) + 2u * idx;
}
__device__ inline Fp term_load(const Ws& w, uint32_t t, uint32_t neg) {
  const LFp* q = (const LFp*)(size_t)((ws_unit(w, t & 7, (t >> 8) & 0xFF) + neg) << 6);
  Fp r;
  r.v = q->v;
  return r;
}
__device__ inline void ws_put(const Ws& w, uint32_t src, uint32_t idx, const Fp& a) {
  LFp* q = (LFp*)(size_t)(ws_unit(w, src, idx) << 6);
  q[0].v = a.v;
  q[1].v = fp_neg(a).v;
}
#endif

// Signed sum of a record's terms: the nu unit terms (+1, or -1 with the neg bit of the term word)
// of r[0 .. N) -- each one slot load of the value or its stored negation -- then the nsc scaled terms
// (|c| > 1: doubling / cyclotomic coefficients) that follow them, read from the record in memory (rg)
// and multiplied in by fp_mul_small.  No calls: the interpreter keeps its registers across the whole
// program.
//
// The unit-term loop runs `umax` times on every lane -- the phase's largest unit count, from the
// program (wave-uniform: scalar branches only) -- and a lane's words past its own nu are masked to the
// zero constant (ZERO_TERM) by one select each.  So all the loads of an operand issue back to back
// and their latencies overlap, and the adds follow without per-term branches.  The adds are raw
// 384-bit sums (every slot holds a canonical value; a sum of up to 8 stays below 8p < 2^384): one
// 12-limb carry chain per term, reduced (fp_reduce8) after the 8th term and where a canonical value is
// needed -- before the scaled terms, and for CANON results (sums stored back into the workspace).  A
// product operand may stay below 8p: fp_mul_inl takes it (64 p^2 < 2^392 p keeps the Montgomery
// output below 2p, reduced once).
#ifndef GBV_COOP_LAZY
#define GBV_COOP_LAZY 1  // 0: modular adds throughout (A/B)
#endif
// unit term i of a record held in registers: resolved from the term word and the bindings
struct RecLoad {
  const Ws& w;
  const uint32_t* r;
  uint32_t nu;
  GBV_HD Fp operator()(int i) const {
    const uint32_t t = (uint32_t)i < nu ? r[i] : ZERO_TERM;
    return term_load(w, t, (t >> 4) & 1);
  }
};
template <int N, bool CANON, class Load>
GBV_HD Fp lin_sum(const Load& load, const Ws& w, uint32_t umax, uint32_t nu, uint32_t nsc, const uint32_t* rg) {
  // groups of G terms: the G loads issue together, then their adds (G x 12 VGPRs in flight)
  constexpr int G = 4;
  Fp acc = fp_zero();
#pragma unroll
  for (int g = 0; g < N; g += G) {
    Fp v[G];
#pragma unroll
    for (int q = 0; q < G; ++q) {
      const int i = g + q;
      if (i < N && (uint32_t)i < umax) v[q] = load(i);
    }
#pragma unroll
    for (int q = 0; q < G; ++q) {
      const int i = g + q;
      if (i < N && (uint32_t)i < umax) {
        if (i == 0)
          acc = v[q];
        else if (GBV_COOP_LAZY)
          fp_acc_lazy(acc, v[q]);
        else
          acc = fp_add(acc, v[q]);
      }
      if (GBV_COOP_LAZY && i == 7 && N > 8 && umax > 8) fp_reduce8_ip(acc);
    }
  }
  if (GBV_COOP_LAZY && umax > 1 && (CANON || nsc)) fp_reduce8_ip(acc);
  for (uint32_t j = 0; j < nsc; ++j) {
    const uint32_t t = rg[nu + j], m = t >> 16;
    const Fp s = fp_mul_small(term_load(w, t, (t >> 4) & 1), m);
    acc = (nu == 0 && j == 0) ? s : fp_add(acc, s);
  }
  return acc;
}
template <int N, bool CANON>
GBV_HD Fp lin_eval(const Ws& w, const uint32_t* r, uint32_t umax, uint32_t nu, uint32_t nsc, const uint32_t* rg) {
  return lin_sum<N, CANON>(RecLoad{w, r, nu}, w, umax, nu, nsc, rg);
}

// Copy n (multiple of 4) words into registers with 16-byte loads: one memory latency per record.
template <int N> GBV_HD void load_words(uint32_t (&r)[N], const uint32_t* t) {
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

// product k: Z[k] = A * B (rg: the record in memory, for the scaled terms; amax / bmax: the round's
// unit-term trip counts)
GBV_HD void prod_lane(const uint32_t (&r)[PROD_WORDS], const uint32_t* rg, int k, const Ws& w, uint32_t amax, uint32_t bmax) {
  const uint32_t h = r[0], hs = r[1 + 2 * OPW];
  Fp x = lin_eval<OPW, false>(w, r + 1, amax, (h & 0xFF) + ((h >> 8) & 0xFF), hs & 0xFF, rg + 1);
  Fp y = lin_eval<OPW, false>(w, r + 1 + OPW, bmax, ((h >> 16) & 0xFF) + (h >> 24), (hs >> 8) & 0xFF, rg + 1 + OPW);
  ws_put(w, SRC_Z, (uint32_t)k, fp_mul_inl(x, y));
}

GBV_HD Fp sum_lane(const uint32_t (&r)[SUM_WORDS], const uint32_t* rg, const Ws& w, uint32_t umax) {
  return lin_eval<SUM_TERMS, true>(w, r + 1, umax, (r[0] & 0xFF) + ((r[0] >> 8) & 0xFF), (r[0] >> 16) & 0xFF, rg + 1);
}

#if defined(GBV_HOST_TEST)
inline unsigned lane_id() { return 0; }
inline void barrier() {}
inline void load_consts() {
  for (int i = 0; i < N_CONSTS_MAX && i < N_CONSTS; ++i) put(g_consts + i, CONSTS[i]);
}

// Host: the lanes of each phase run one after another.
inline void run(const Prog& P, const Ws& w) {
  int p0 = 0;
  uint32_t rec[PROD_WORDS], r8[SUM_WORDS];
  for (int r = 0; r < P.n_rounds; ++r) {
    for (int k = p0; k < P.round_end[r]; ++k) {
      load_words(rec, P.prods + PROD_WORDS * k);
      prod_lane(rec, P.prods + PROD_WORDS * k, k, w, P.amax[r], P.bmax[r]);
    }
    p0 = P.round_end[r];
  }
  for (int j = 0; j < P.n_part; ++j) {
    load_words(r8, P.parts + SUM_WORDS * j);
    ws_put(w, SRC_Z, P.round_end[P.n_rounds - 1] + j, sum_lane(r8, P.parts + SUM_WORDS * j, w, P.pmax));
  }
  Fp o[LANES];
  for (int k = 0; k < P.n_out; ++k) {
    load_words(r8, P.outs + SUM_WORDS * k);
    o[k] = sum_lane(r8, P.outs + SUM_WORDS * k, w, P.omax);
  }
  for (int k = 0; k < P.n_out; ++k) ws_put(w, P.out_dst[k], P.out_idx[k], o[k]);
}
#define COOP_LANES(l) for (unsigned l = 0; l < (unsigned)LANES; ++l)
#define COOP_LANE0 if (true)
#else
__device__ inline unsigned lane_id() { return threadIdx.x & 63u; }  // a job is one wave; a block may hold several
// A coop job is ONE wave: its phases synchronise at wavefront scope -- the workgroup-scope fences
// of __syncthreads (prior LDS writes complete and visible, later reads not hoisted) around a wave
// barrier instead of s_barrier.  For the one-wave workgroups this is what __syncthreads compiles to
// anyway; it also lets a workgroup hold a second wave doing other work, which
// meets the coop wave only at explicit __syncthreads.
__device__ inline void barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
// Every kernel that runs programs calls this first (lane-parallel copy of the constant pool).
__device__ inline void load_consts() {
  if (threadIdx.x < N_CONSTS) put(GBV_CONSTS_LDS + threadIdx.x, CONSTS[threadIdx.x]);
  barrier();
}

// All of a lane's records for this program are fetched up front (one memory latency), the next
// round's while the current round computes.
__device__ __forceinline__ void run_body(const Prog* PP, uint32_t b0, uint32_t b1, uint32_t b2, uint32_t b3) {
  const Prog& P = *PP;
  const Ws w{{b0, b1, b2, b3}};
  const int lane = (int)(threadIdx.x & 63u);
  uint32_t rec[PROD_WORDS], rpart[SUM_WORDS], rout[SUM_WORDS];
  const bool have_part = lane < P.n_part, have_out = lane < P.n_out;
  const uint32_t* gpart = P.parts + SUM_WORDS * lane;
  const uint32_t* gout = P.outs + SUM_WORDS * lane;
  int p0 = 0;
  if (lane < P.round_end[0]) load_words(rec, P.prods + PROD_WORDS * lane);
  if (have_part) load_words(rpart, gpart);
  if (have_out) load_words(rout, gout);
  for (int r = 0; r < P.n_rounds; ++r) {
    int p1 = P.round_end[r];
    // the round's unit-term trip counts, wave-uniform (scalar registers: the term loops branch on them
    // without exec-mask juggling)
    const uint32_t am = __builtin_amdgcn_readfirstlane(P.amax[r]), bm = __builtin_amdgcn_readfirstlane(P.bmax[r]);
    if (p0 + lane < p1) prod_lane(rec, P.prods + PROD_WORDS * (p0 + lane), p0 + lane, w, am, bm);  // every round has <= 64 products
    if (r + 1 < P.n_rounds && p1 + lane < P.round_end[r + 1]) load_words(rec, P.prods + PROD_WORDS * (p1 + lane));
    p0 = p1;
    barrier();
  }
  const uint32_t pm = __builtin_amdgcn_readfirstlane(P.pmax), om = __builtin_amdgcn_readfirstlane(P.omax);
  if (have_part) ws_put(w, SRC_Z, P.round_end[P.n_rounds - 1] + lane, sum_lane(rpart, gpart, w, pm));
  if (P.n_part) barrier();
  Fp o;
  if (have_out) o = sum_lane(rout, gout, w, om);
  barrier();
  if (have_out) ws_put(w, P.out_dst[lane], P.out_idx[lane], o);
  barrier();
}
// One out-of-line copy of the interpreter serves every call site (the drivers make hundreds).
__device__ __noinline__ void run_ni(const Prog* PP, uint32_t b0, uint32_t b1, uint32_t b2, uint32_t b3) { run_body(PP, b0, b1, b2, b3); }
__device__ inline void run(const Prog& P, const Ws& w) { run_ni(&P, w.b[0], w.b[1], w.b[2], w.b[3]); }

#define COOP_LANES(l) for (unsigned l = threadIdx.x & 63u; l == (threadIdx.x & 63u); l = ~0u)
#define COOP_LANE0 if ((threadIdx.x & 63u) == 0)
#endif

// ---- operand helpers (lane-parallel, end with a barrier) ------------------------------------
GBV_HD void set_one12(Slot* fg) {
  LSlot* f = GBV_LDS(fg);
  COOP_LANES(l) if (l < 12) put(f + l, l == 0 ? FP_ONE : fp_zero());
  barrier();
}
GBV_HD void copy(Slot* dstg, const Slot* srcg, unsigned n) {
  LSlot* dst = GBV_LDS(dstg);
  const LSlot* src = GBV_LDS(srcg);
  COOP_LANES(l) if (l < n) put_pair(dst + l, get_signed(src + l, false), get_signed(src + l, true));
  barrier();
}
GBV_HD void conj12(Slot* fg) {  // negate the w-odd half (coordinates 6..11): swap value and negation
  LSlot* f = GBV_LDS(fg);
  COOP_LANES(l) if (l >= 6 && l < 12) {
    Fp a = get_signed(f + l, false), na = get_signed(f + l, true);
    put_pair(f + l, na, a);
  }
  barrier();
}
// Fp12 <-> 12 consecutive slots
GBV_HD Fp12 load12(const Slot* fg) {
  const LSlot* f = GBV_LDS(fg);
  Fp12 r;
  Fp* d = (Fp*)&r;
  for (int i = 0; i < 12; ++i) d[i] = get(f + i);
  return r;
}
GBV_HD void store12(Slot* fg, const Fp12& a) {
  LSlot* f = GBV_LDS(fg);
  const Fp* s = (const Fp*)&a;
  for (int i = 0; i < 12; ++i) put(f + i, s[i]);
}
GBV_HD bool is_one12(const Slot* fg) {
  const LSlot* f = GBV_LDS(fg);
  bool ok = true;
  for (int i = 0; i < 12; ++i) ok = ok && fp_eq(get(f + i), i == 0 ? FP_ONE : fp_zero());
  return ok;
}

GBV_HD Ws ws2(Slot* mem, uint16_t z, uint16_t a, uint16_t b) { return make_ws(mem, z, a, b); }
GBV_HD Ws ws3(Slot* mem, uint16_t z, uint16_t a, uint16_t b, uint16_t c) { return make_ws(mem, z, a, b, c); }

GBV_HD void frob12(Slot* mem, uint16_t z, int n, uint16_t a, uint16_t c) { run(n == 1 ? FP12_FROB1 : FP12_FROB2, ws2(mem, z, a, c)); }

// ---- written-out programs: lane descriptors resolved once, no records -------------------------
// The hottest programs (the Miller loop's line products, the exponentiations' cyclotomic squarings)
// as fixed two-phase code: product lanes, a barrier, output lanes.  A lane's term addresses (value or
// stored negation, the zero constant for padding) are resolved once per loop into registers.
#if defined(GBV_HOST_TEST)
typedef const Fp* CAddr;
inline CAddr caddr(const LSlot* s, uint32_t neg) { return neg ? &s->n : &s->v; }
inline Fp cload(CAddr a) { return *a; }
#else
typedef uint32_t CAddr;  // LDS byte address of a value or its stored negation
__device__ inline CAddr caddr(const LSlot* s, uint32_t neg) { return (uint32_t)(size_t)s + (neg << 6); }
__device__ inline Fp cload(CAddr a) {
  Fp r;
  r.v = ((const LFp*)(size_t)a)->v;
  return r;
}
#endif

// Sparse line product c = f l, l = c0 + c2 w^2 + c3 w^3 (slots l: c0 0 1 | c2 2 3 | c3 4 5; the lines
// of G2_DBL_STEP / G2_ADD_STEP / MILLER_SQR_DBL).  Over Fp2[w]/(w^6 - xi) -- f_k at slot 2k for even
// k, 2k + 5 for odd -- the w^m coefficient of f l is f_m c0 + [xi] f_(m-2) c2 + [xi] f_(m-3) c3 (xi
// where the index wraps): 18 Fp2 products, each Karatsuba (P0 = f0 c0, P1 = f1 c1, P2 = (f0 + f1)
// (c0 + c1)), one Fp product per lane on 54 lanes; then 12 output lanes of <= 9 unit terms --
// (P0 - P1, P2 - P0 - P1), or (2 P0 - P2, P2 - 2 P1) for a xi-twisted product.  Against the
// interpreted FP12_MUL_LINE (39 products, 24 partial sums, 318 terms): one phase fewer and ~220 terms.
// The unit terms of component c of a Karatsuba Fp2 product (P0 = a0 b0, P1 = a1 b1, P2 = (a0 + a1)
// (b0 + b1) at P): (P0 - P1, P2 - P0 - P1), or times xi (2 P0 - P2, P2 - 2 P1); a plain real part has
// two terms, the third the zero constant.
struct Terms3 {
  CAddr t[3];
};
GBV_HD Terms3 kara_terms(const LSlot* P, uint32_t c, bool tw, CAddr zero) {
  Terms3 r;
  r.t[0] = c ? caddr(P + 2, 0) : caddr(P, 0);
  r.t[1] = c ? caddr(P + 1, 1) : tw ? caddr(P, 0) : caddr(P + 1, 1);
  r.t[2] = c ? (tw ? caddr(P + 1, 1) : caddr(P, 1)) : tw ? caddr(P + 2, 1) : zero;
  return r;
}
struct LineLane {
  CAddr a[2], b[2];  // product lane (l < 54)
  CAddr o[9];        // output lane (l < 12)
  LSlot *dz, *dout;
};
GBV_HD LineLane line_lane(Slot* memg, uint16_t zo, uint16_t fo, uint16_t lo, uint16_t co, uint32_t l) {
  LSlot* mem = GBV_LDS(memg);
  const LSlot *f = mem + fo, *ln = mem + lo, *zs = mem + zo;
  const CAddr zero = caddr(GBV_CONSTS_LDS, 0);
  LineLane x;
  x.a[0] = x.a[1] = x.b[0] = x.b[1] = zero;
  for (int i = 0; i < 9; ++i) x.o[i] = zero;
  x.dz = mem + zo + (l < 54 ? l : 0);
  x.dout = mem + co + (l < 12 ? l : 0);
  if (l < 54) {
    const uint32_t t = l / 3, r = l - 3 * t, m = t / 3, s = t - 3 * m;
    const uint32_t sh = s == 0 ? 0 : s + 1;  // w-degree of the line coefficient: 0, 2, 3
    const uint32_t k = (m + 6 - sh) % 6;
    const LSlot* fk = f + (k & 1 ? k + 5 : k);
    const LSlot* lc = ln + 2 * s;
    if (r < 2) {
      x.a[0] = caddr(fk + r, 0), x.b[0] = caddr(lc + r, 0);
    } else {
      x.a[0] = caddr(fk, 0), x.a[1] = caddr(fk + 1, 0), x.b[0] = caddr(lc, 0), x.b[1] = caddr(lc + 1, 0);
    }
  }
  if (l < 12) {
    const uint32_t sp = l >> 1, c = l & 1, m = sp < 3 ? 2 * sp : 2 * (sp - 3) + 1;
#pragma unroll
    for (uint32_t s = 0; s < 3; ++s) {  // fixed register positions: no dynamically indexed arrays
      const Terms3 t = kara_terms(zs + 3 * (3 * m + s), c, m < (s == 0 ? 0u : s + 1), zero);
      x.o[3 * s] = t.t[0], x.o[3 * s + 1] = t.t[1], x.o[3 * s + 2] = t.t[2];
    }
  }
  return x;
}
GBV_HD void line_prod(const LineLane& x) {
  Fp a = cload(x.a[0]), b = cload(x.b[0]);
  const Fp a1 = cload(x.a[1]), b1 = cload(x.b[1]);
  fp_acc_lazy(a, a1);
  fp_acc_lazy(b, b1);
  put(x.dz, fp_mul_inl(a, b));
}
GBV_HD void line_out(const LineLane& x) {
  Fp v[9];
  for (int i = 0; i < 9; ++i) v[i] = cload(x.o[i]);
  Fp u = v[0];
  for (int i = 1; i < 6; ++i) fp_acc_lazy(u, v[i]);
  fp_reduce8_ip(u);  // < 6p
  for (int i = 6; i < 9; ++i) fp_acc_lazy(u, v[i]);
  fp_reduce8_ip(u);  // < 4p
  put(x.dout, u);
}
#if defined(GBV_HOST_TEST)
inline void mul_line(Slot* mem, uint16_t zo, uint16_t fo, uint16_t lo, uint16_t co) {
  for (uint32_t l = 0; l < 54; ++l) line_prod(line_lane(mem, zo, fo, lo, co, l));
  for (uint32_t l = 0; l < 12; ++l) line_out(line_lane(mem, zo, fo, lo, co, l));
}
#else
__device__ __forceinline__ void mul_line_lane(const LineLane& x) {
  const uint32_t l = lane_id();
  if (l < 54) line_prod(x);
  barrier();
  if (l < 12) line_out(x);
  barrier();
}
#endif

// One Miller-loop bit written out: f^2 (optional) and the doubling step of T with its line, the
// same maps as MILLER_SQR_DBL / G2_DBL_STEP (tools/gen_coop.py dbl_step_into: T' = 4 [2]T
// homogeneous; line (B - E, 3 X^2 (-xP), H yP)).  Round 1: the doubling's 11 products d0..d10 (XY
// Karatsuba, Y^2, Z^2, (Y + Z)^2, X^2) on lanes 0..10 and f^2's first 53 products on lanes 11..63;
// round 2: the doubling's 14 products r0..r13, whose operands are small multiples of round-1 products
// (3b' = 12 xi, so 36, 72, 3456 ...: unit terms plus k times a sum, fp_mul_small), and f^2's last 4;
// then 24 output lanes: f^2 (<= 9 unit terms), T', the line.  f^2 over Fp2[w]/(w^6 - xi): the
// w^m coefficient sums f_i f_j over i + j = m mod 6 (xi where it wraps): 15 cross products
// (2 f_i) f_j (Karatsuba, 3 products) and 6 squares (2 products), 57 in all.  Z: d at 0..10, the
// square's products at 11..67, r at 68..81.
struct SqrDblLane {
  CAddr a[4], b[4];                    // round 1
  CAddr a2[4], av[3], b2[4], bv[3];    // round 2: operand = unit terms + k (sum of v terms)
  uint32_t ak, bk;
  CAddr o[12], ov[2];                  // output: unit terms + k (sum of v terms)
  uint32_t ok;
  LSlot *dz1, *dz2, *dout;
};
constexpr uint32_t SD_F2 = 11, SD_R2 = 68;
// the operands of the square's product k (< 57): unit terms only
GBV_HD void sqr_prod_terms(CAddr (&a)[4], CAddr (&b)[4], const LSlot* f, uint32_t k, CAddr zero) {
  const bool cross = k < 45;
  const uint32_t c = k / 3, rc = k - 3 * c, sq = (k - 45) >> 1, rs = (k - 45) & 1;
  uint32_t ci = 0, cj = 0, n = 0;
#pragma unroll
  for (uint32_t i = 0; i < 6; ++i)
#pragma unroll
    for (uint32_t j = i + 1; j < 6; ++j, ++n)
      if (n == c) ci = i, cj = j;
  const uint32_t i = cross ? ci : sq;
  const LSlot* A = f + (i & 1 ? i + 5 : i);
  const LSlot* B = f + (cj & 1 ? cj + 5 : cj);
  const CAddr a0 = caddr(A, 0), a1 = caddr(A + 1, 0), b0 = caddr(B, 0), b1 = caddr(B + 1, 0);
  for (int q = 0; q < 4; ++q) a[q] = b[q] = zero;
  if (cross) {  // (2 f_i) f_j
    a[0] = a[1] = rc == 1 ? a1 : a0;
    a[2] = a[3] = rc == 2 ? a1 : zero;
    b[0] = rc == 1 ? b1 : b0;
    b[1] = rc == 2 ? b1 : zero;
  } else {  // f_i^2 = ((a0 + a1)(a0 - a1), a0 (2 a1))
    a[0] = a0;
    a[1] = rs ? zero : a1;
    b[0] = rs ? a1 : a0;
    b[1] = rs ? a1 : caddr(A + 1, 1);
  }
}
GBV_HD SqrDblLane sqr_dbl_lane(Slot* memg, uint16_t zo, uint16_t fo, uint16_t to, uint16_t po, uint16_t lo, uint32_t l) {
  LSlot* mem = GBV_LDS(memg);
  const LSlot *f = mem + fo, *T = mem + to, *P = mem + po, *zs = mem + zo;
  const CAddr zero = caddr(GBV_CONSTS_LDS, 0);
  SqrDblLane x;
  for (int q = 0; q < 4; ++q) x.a[q] = x.b[q] = x.a2[q] = x.b2[q] = zero;
  for (int q = 0; q < 3; ++q) x.av[q] = x.bv[q] = zero;
  for (int q = 0; q < 12; ++q) x.o[q] = zero;
  x.ov[0] = x.ov[1] = zero;
  x.ak = x.bk = x.ok = 1;
  x.dz1 = mem + zo + (l < 64 ? l : 0);
  x.dz2 = mem + zo + (l < 14 ? SD_R2 + l : l < 18 ? l + SD_F2 + 39 : 0);
  x.dout = l < 12 ? mem + fo + l : l < 18 ? mem + to + (l - 12) : l < 24 ? mem + lo + (l - 18) : mem + zo;
  auto t = [&](uint32_t i, uint32_t neg) { return caddr(T + i, neg); };  // x0 x1 y0 y1 z0 z1
  auto d = [&](uint32_t i, uint32_t neg) { return caddr(zs + i, neg); };
  // round 1
  if (l < 11) {
    switch (l) {
      case 0: x.a[0] = t(0, 0), x.b[0] = t(2, 0); break;
      case 1: x.a[0] = t(1, 0), x.b[0] = t(3, 0); break;
      case 2: x.a[0] = t(0, 0), x.a[1] = t(1, 0), x.b[0] = t(2, 0), x.b[1] = t(3, 0); break;
      case 3: x.a[0] = t(2, 0), x.a[1] = t(3, 0), x.b[0] = t(2, 0), x.b[1] = t(3, 1); break;
      case 4: x.a[0] = t(2, 0), x.b[0] = x.b[1] = t(3, 0); break;
      case 5: x.a[0] = t(4, 0), x.a[1] = t(5, 0), x.b[0] = t(4, 0), x.b[1] = t(5, 1); break;
      case 6: x.a[0] = t(4, 0), x.b[0] = x.b[1] = t(5, 0); break;
      case 7:
        x.a[0] = t(2, 0), x.a[1] = t(4, 0), x.a[2] = t(3, 0), x.a[3] = t(5, 0);
        x.b[0] = t(2, 0), x.b[1] = t(4, 0), x.b[2] = t(3, 1), x.b[3] = t(5, 1);
        break;
      case 8:
        x.a[0] = t(2, 0), x.a[1] = t(4, 0);
        x.b[0] = x.b[2] = t(3, 0), x.b[1] = x.b[3] = t(5, 0);
        break;
      case 9: x.a[0] = t(0, 0), x.a[1] = t(1, 0), x.b[0] = t(0, 0), x.b[1] = t(1, 1); break;
      default: x.a[0] = t(0, 0), x.b[0] = x.b[1] = t(1, 0); break;
    }
  } else if (l < 64) {
    sqr_prod_terms(x.a, x.b, f, l - SD_F2, zero);
  }
  // round 2
  if (l < 14) {
    switch (l) {
      case 0: x.a2[0] = x.a2[1] = d(0, 0), x.a2[2] = x.a2[3] = d(1, 1), x.b2[0] = d(3, 0), x.bv[0] = d(6, 0), x.bv[1] = d(5, 1), x.bk = 36; break;
      case 1: x.av[0] = d(2, 0), x.av[1] = d(0, 1), x.av[2] = d(1, 1), x.ak = 2, x.b2[0] = d(4, 0), x.bv[0] = d(5, 1), x.bv[1] = d(6, 1), x.bk = 36; break;
      case 2: x.av[0] = d(2, 0), x.av[1] = x.av[2] = d(1, 1), x.ak = 2, x.b2[0] = d(3, 0), x.b2[1] = d(4, 0), x.bv[0] = d(5, 1), x.bk = 72; break;
      case 3: x.a2[0] = d(3, 0), x.a2[1] = d(4, 0), x.av[0] = d(5, 0), x.ak = 72, x.b2[0] = d(3, 0), x.b2[1] = d(4, 1), x.bv[0] = d(6, 1), x.bk = 72; break;
      case 4: x.a2[0] = d(3, 0), x.av[0] = d(5, 0), x.av[1] = d(6, 1), x.ak = 36, x.b2[0] = x.b2[1] = d(4, 0), x.bv[0] = d(5, 0), x.bv[1] = d(6, 0), x.bk = 72; break;
      case 5: x.av[0] = d(5, 0), x.ak = 3456, x.b2[0] = x.b2[1] = d(6, 1); break;
      case 6: x.av[0] = d(5, 0), x.av[1] = d(6, 1), x.ak = 3456, x.b2[0] = d(5, 0), x.b2[1] = d(6, 0); break;
      case 7: x.a2[0] = x.a2[1] = x.a2[2] = x.a2[3] = d(3, 0), x.b2[0] = d(7, 0), x.b2[1] = d(3, 1), x.b2[2] = d(5, 1); break;
      case 8: x.a2[0] = x.a2[1] = x.a2[2] = x.a2[3] = d(4, 0), x.b2[0] = d(8, 0), x.b2[1] = d(4, 1), x.b2[2] = d(6, 1); break;
      case 9:
        x.av[0] = d(3, 0), x.av[1] = d(4, 0), x.ak = 4;
        x.b2[0] = d(7, 0), x.b2[1] = d(8, 0), x.b2[2] = d(3, 1), x.b2[3] = d(4, 1), x.bv[0] = d(5, 1), x.bv[1] = d(6, 1);
        break;
      case 10: x.a2[0] = x.a2[1] = x.a2[2] = d(9, 0), x.b2[0] = caddr(P, 0); break;
      case 11: x.a2[0] = x.a2[1] = x.a2[2] = d(10, 0), x.b2[0] = caddr(P, 0); break;
      case 12: x.a2[0] = d(7, 0), x.a2[1] = d(3, 1), x.a2[2] = d(5, 1), x.b2[0] = caddr(P + 1, 0); break;
      default: x.a2[0] = d(8, 0), x.a2[1] = d(4, 1), x.a2[2] = d(6, 1), x.b2[0] = caddr(P + 1, 0); break;
    }
  } else if (l < 18) {
    sqr_prod_terms(x.a2, x.b2, f, l + 39, zero);
  }
  // outputs
  if (l < 12) {
    const uint32_t sp = l >> 1, c = l & 1, m = sp < 3 ? 2 * sp : 2 * (sp - 3) + 1;
    uint32_t q = 0;
#pragma unroll
    for (uint32_t i = 0; i < 6; ++i) {
      const uint32_t j = (m + 6 - i) % 6;
      const bool use = i <= j, tw = i + j >= 6;
      Terms3 tt;
      if (i < j) {
        const uint32_t cp = i * (11 - i) / 2 + (j - i - 1);  // cross pair index
        tt = kara_terms(zs + SD_F2 + 3 * cp, c, tw, zero);
      } else {  // f_i^2 = (S0, S1), times xi: (S0 - S1, S0 + S1)
        const LSlot* S = zs + SD_F2 + 45 + 2 * i;
        tt.t[0] = c ? caddr(S + 1, 0) : caddr(S, 0);
        tt.t[1] = tw ? (c ? caddr(S, 0) : caddr(S + 1, 1)) : zero;
        tt.t[2] = zero;
      }
#pragma unroll
      for (uint32_t qq = 0; qq < 4; ++qq)
        if (use && q == qq) x.o[3 * qq] = tt.t[0], x.o[3 * qq + 1] = tt.t[1], x.o[3 * qq + 2] = tt.t[2];
      q += use ? 1 : 0;
    }
  } else if (l < 24) {
    const LSlot* R = zs + SD_R2;
    auto r = [&](uint32_t i, uint32_t neg) { return caddr(R + i, neg); };
    switch (l - 12) {
      case 0: x.o[0] = r(0, 0), x.o[1] = r(1, 1); break;                   // X' = 2A (B - F)
      case 1: x.o[0] = r(2, 0), x.o[1] = r(0, 1), x.o[2] = r(1, 1); break;
      case 2: x.o[0] = r(3, 0), x.o[1] = r(5, 1); break;                   // Y' = (B + F)^2 - 12 E^2
      case 3: x.o[0] = r(4, 0), x.o[1] = r(6, 1); break;
      case 4: x.o[0] = r(7, 0), x.o[1] = r(8, 1); break;                   // Z' = 4 B H
      case 5: x.o[0] = r(9, 0), x.o[1] = r(7, 1), x.o[2] = r(8, 1); break;
      case 6: x.o[0] = d(3, 0), x.ov[0] = d(6, 0), x.ov[1] = d(5, 1), x.ok = 12; break;  // B - E
      case 7: x.o[0] = d(4, 0), x.ov[0] = d(5, 1), x.ov[1] = d(6, 1), x.ok = 12; break;
      case 8: x.o[0] = r(10, 0); break;                                    // 3 X^2 (-xP)
      case 9: x.o[0] = r(11, 0); break;
      case 10: x.o[0] = r(12, 0); break;                                   // H yP
      default: x.o[0] = r(13, 0); break;
    }
  }
  return x;
}
GBV_HD Fp sd_sum4(const CAddr (&u)[4]) {
  Fp s = cload(u[0]);
  const Fp s1 = cload(u[1]), s2 = cload(u[2]), s3 = cload(u[3]);
  fp_acc_lazy(s, s1);
  fp_acc_lazy(s, s2);
  fp_acc_lazy(s, s3);
  return s;  // < 4p
}
// unit terms + k (sum of v terms): < 5p, a product operand
GBV_HD Fp sd_operand(const CAddr (&u)[4], const CAddr (&v)[3], uint32_t k) {
  Fp w = cload(v[0]);
  const Fp w1 = cload(v[1]), w2 = cload(v[2]);
  Fp s = sd_sum4(u);
  fp_acc_lazy(w, w1);
  fp_acc_lazy(w, w2);
  fp_reduce8_ip(w);
  fp_acc_lazy(s, fp_mul_small(w, k));
  return s;
}
GBV_HD void sd_round1(const SqrDblLane& x) { put(x.dz1, fp_mul_inl(sd_sum4(x.a), sd_sum4(x.b))); }
GBV_HD void sd_round2(const SqrDblLane& x) { put(x.dz2, fp_mul_inl(sd_operand(x.a2, x.av, x.ak), sd_operand(x.b2, x.bv, x.bk))); }
GBV_HD void sd_out(const SqrDblLane& x) {
  Fp v[12];
  for (int i = 0; i < 12; ++i) v[i] = cload(x.o[i]);
  Fp w = cload(x.ov[0]);
  const Fp w1 = cload(x.ov[1]);
  Fp u = v[0];
  for (int i = 1; i < 6; ++i) fp_acc_lazy(u, v[i]);
  fp_reduce8_ip(u);
  for (int i = 6; i < 12; ++i) fp_acc_lazy(u, v[i]);
  fp_reduce8_ip(u);  // < 7p
  fp_acc_lazy(w, w1);
  fp_reduce8_ip(w);
  fp_acc_lazy(u, fp_mul_small(w, x.ok));
  fp_reduce8_ip(u);  // < 2p
  put(x.dout, u);
}
#if defined(GBV_HOST_TEST)
inline void sqr_dbl(Slot* mem, uint16_t zo, uint16_t fo, uint16_t to, uint16_t po, uint16_t lo, bool sqr) {
  for (uint32_t l = 0; l < 64; ++l)
    if (l < 11 || sqr) sd_round1(sqr_dbl_lane(mem, zo, fo, to, po, lo, l));
  for (uint32_t l = 0; l < 18; ++l)
    if (l < 14 || sqr) sd_round2(sqr_dbl_lane(mem, zo, fo, to, po, lo, l));
  for (uint32_t l = 0; l < 24; ++l)
    if (l >= 12 || sqr) sd_out(sqr_dbl_lane(mem, zo, fo, to, po, lo, l));
}
#else
__device__ __forceinline__ void sqr_dbl_run(const SqrDblLane& x, bool sqr) {
  const uint32_t l = lane_id();
  if (l < 11 || sqr) sd_round1(x);
  barrier();
  if (l < 14 || (sqr && l < 18)) sd_round2(x);
  barrier();
  if ((l >= 12 && l < 24) || (sqr && l < 12)) sd_out(x);
  barrier();
}
#endif

// General Fp12 product c = f g, schoolbook over Fp2[w]/(w^6 - xi): the w^m coefficient sums f_i
// g_(m-i) (xi where i > m), 36 Karatsuba Fp2 products = 108 Fp products, two per lane on 54 lanes (the
// two independent), then 12 output lanes of <= 18 unit terms.  Against the interpreted FP12_MUL
// (Karatsuba at every level: 54 products, partial sums, long outputs) one product more per lane and no
// partial-sum phase.  Z: product 3 (6 i + j) + r (r: P0 P1 P2 of f_i g_j) at Z + 0 .. 107.
struct MulLane {
  CAddr a[2][2], b[2][2];  // product lane (l < 54): two products, two terms per operand
  CAddr o[18];             // output lane (l < 12)
  LSlot *dz0, *dz1, *dout;
};
GBV_HD MulLane mul_lane(Slot* memg, uint16_t zo, uint16_t ao, uint16_t bo, uint16_t co, uint32_t l) {
  LSlot* mem = GBV_LDS(memg);
  const LSlot *f = mem + ao, *g = mem + bo, *zs = mem + zo;
  const CAddr zero = caddr(GBV_CONSTS_LDS, 0);
  MulLane x;
#pragma unroll
  for (uint32_t h = 0; h < 2; ++h) {
    const uint32_t P = l + 54 * h, t = P / 3, r = P - 3 * t, i = t / 6, j = t - 6 * i;
    const LSlot* F = f + (i & 1 ? i + 5 : i);
    const LSlot* G = g + (j & 1 ? j + 5 : j);
    x.a[h][0] = caddr(F + (r == 1 ? 1 : 0), 0);
    x.a[h][1] = r == 2 ? caddr(F + 1, 0) : zero;
    x.b[h][0] = caddr(G + (r == 1 ? 1 : 0), 0);
    x.b[h][1] = r == 2 ? caddr(G + 1, 0) : zero;
  }
  x.dz0 = mem + zo + (l < 54 ? l : 0);
  x.dz1 = mem + zo + (l < 54 ? l + 54 : 0);
  x.dout = mem + co + (l < 12 ? l : 0);
  const uint32_t sp = (l < 12 ? l : 0) >> 1, c = l & 1, m = sp < 3 ? 2 * sp : 2 * (sp - 3) + 1;
#pragma unroll
  for (uint32_t i = 0; i < 6; ++i) {
    const uint32_t j = (m + 6 - i) % 6;
    const Terms3 t = kara_terms(zs + 3 * (6 * i + j), c, i > m, zero);
    x.o[3 * i] = t.t[0], x.o[3 * i + 1] = t.t[1], x.o[3 * i + 2] = t.t[2];
  }
  return x;
}
GBV_HD void mul_prod(const MulLane& x) {
  Fp a0 = cload(x.a[0][0]), b0 = cload(x.b[0][0]), a1 = cload(x.a[1][0]), b1 = cload(x.b[1][0]);
  const Fp a01 = cload(x.a[0][1]), b01 = cload(x.b[0][1]), a11 = cload(x.a[1][1]), b11 = cload(x.b[1][1]);
  fp_acc_lazy(a0, a01);
  fp_acc_lazy(b0, b01);
  fp_acc_lazy(a1, a11);
  fp_acc_lazy(b1, b11);
  put(x.dz0, fp_mul_inl(a0, b0));
  put(x.dz1, fp_mul_inl(a1, b1));
}
GBV_HD void mul_out(const MulLane& x) {
  Fp v[18];
  for (int i = 0; i < 18; ++i) v[i] = cload(x.o[i]);
  Fp u = v[0];
  for (int i = 1; i < 6; ++i) fp_acc_lazy(u, v[i]);
  fp_reduce8_ip(u);
  for (int i = 6; i < 12; ++i) fp_acc_lazy(u, v[i]);
  fp_reduce8_ip(u);  // < 7p
  for (int i = 12; i < 18; ++i) fp_acc_lazy(u, v[i]);
  fp_reduce8_ip(u);
  put(x.dout, u);
}
#if defined(GBV_HOST_TEST)
inline void mul12(Slot* mem, uint16_t z, uint16_t a, uint16_t b, uint16_t c) {
  for (uint32_t l = 0; l < 54; ++l) mul_prod(mul_lane(mem, z, a, b, c, l));
  for (uint32_t l = 0; l < 12; ++l) mul_out(mul_lane(mem, z, a, b, c, l));
}
#else
__device__ __forceinline__ void mul12_lane(const MulLane& x) {
  const uint32_t l = lane_id();
  if (l < 54) mul_prod(x);
  barrier();
  if (l < 12) mul_out(x);
  barrier();
}
// c = a b (c may be a or b)
__device__ inline void mul12(Slot* mem, uint16_t z, uint16_t a, uint16_t b, uint16_t c) { mul12_lane(mul_lane(mem, z, a, b, c, lane_id())); }
#endif

// ---- cyclotomic squaring written out (the exponentiations' ~315 squarings) --------------------
// Granger-Scott: f in the cyclotomic subgroup as three Fp4 pairs (z0, z1), (z2, z3), (z4, z5) --
// slots (0 1 | 8 9), (6 7 | 4 5), (2 3 | 10 11) -- each pair's t0 = a^2 + xi b^2,
// t1 = (a + b)^2 - a^2 - b^2, and
//   z0' = 3 t0(z0,z1) - 2 z0   z1' = 3 t1(z0,z1) + 2 z1   z4' = 3 t0(z2,z3) - 2 z4
//   z5' = 3 t1(z2,z3) + 2 z5   z2' = 3 xi t1(z4,z5) + 2 z2   z3' = 3 t0(z4,z5) - 2 z3.
// An Fp2 square x^2 is two Fp products, P = (x0 + x1)(x0 - x1) and Q = x0 (2 x1): 18 products, one
// per lane, then 12 output lanes, each 3 (<= 6 signed products) +- 2 z_o.  Against the interpreted
// FP12_CYC_SQR (18 products, 12 partial sums with scaled terms read from the record, 12 outputs): no
// partial-sum phase, no scaled terms, no record reads, and a lane's term addresses resolved once
// per exponentiation.  The output lane of slot o reads input slot o only, so c may be a.
struct CycLane {
  CAddr a[4], b[4];  // product lane (l < 18): the terms of its two operands
  CAddr o[6], z;     // output lane (l < 12): its signed product terms, +-z_o
  LSlot *dz, *dout;
};
GBV_HD CycLane cyc_lane(Slot* memg, uint16_t zo, uint16_t ao, uint16_t co, uint32_t l) {
  LSlot* mem = GBV_LDS(memg);
  const LSlot* in = mem + ao;
  const LSlot* zs = mem + zo;
  const CAddr zero = caddr(GBV_CONSTS_LDS, 0);
  CycLane x;
  for (int i = 0; i < 4; ++i) x.a[i] = x.b[i] = zero;
  for (int i = 0; i < 6; ++i) x.o[i] = zero;
  x.z = zero;
  x.dz = mem + zo + (l < 18 ? l : 0);
  x.dout = mem + co + (l < 12 ? l : 0);
  if (l < 18) {
    const uint32_t k = l / 6, j = l - 6 * k;
    const uint32_t A = k == 0 ? 0 : k == 1 ? 6 : 2, B = k == 0 ? 8 : k == 1 ? 4 : 10;
    const CAddr x0 = caddr(in + A, 0), x1 = caddr(in + A + 1, 0), x2 = caddr(in + B, 0), x3 = caddr(in + B + 1, 0);
    const CAddr n1 = caddr(in + A + 1, 1), n3 = caddr(in + B + 1, 1);
    switch (j) {
      case 0: x.a[0] = x0, x.a[1] = x1, x.b[0] = x0, x.b[1] = n1; break;  // P(a)
      case 1: x.a[0] = x0, x.b[0] = x1, x.b[1] = x1; break;                // Q(a)
      case 2: x.a[0] = x2, x.a[1] = x3, x.b[0] = x2, x.b[1] = n3; break;  // P(b)
      case 3: x.a[0] = x2, x.b[0] = x3, x.b[1] = x3; break;                // Q(b)
      case 4:                                                              // P(a + b)
        x.a[0] = x0, x.a[1] = x2, x.a[2] = x1, x.a[3] = x3;
        x.b[0] = x0, x.b[1] = x2, x.b[2] = n1, x.b[3] = n3;
        break;
      default: x.a[0] = x0, x.a[1] = x2, x.b[0] = x1, x.b[1] = x3, x.b[2] = x1, x.b[3] = x3; break;  // Q(a + b)
    }
  }
  if (l < 12) {
    // slot pair s: z0 z4 z3 | z2 | z1 z5 -> t0 of pair s (minus 2z) | xi t1 of pair 2 | t1 of pair s - 4
    const uint32_t s = l >> 1, c = l & 1;
    const uint32_t k = s < 3 ? s : s == 3 ? 2 : s - 4;
    const LSlot* p = zs + 6 * k;  // P(a) Q(a) P(b) Q(b) P(a+b) Q(a+b)
    auto t = [&](int m, uint32_t neg) { return caddr(p + m, neg); };
    if (s < 3) {
      x.o[0] = c ? t(1, 0) : t(0, 0), x.o[1] = t(2, 0), x.o[2] = t(3, c ? 0 : 1);  // t0
    } else if (s == 3) {
      x.o[0] = t(4, 0), x.o[1] = t(0, 1), x.o[2] = t(2, 1);  // xi t1 = (t1.0 - t1.1, t1.0 + t1.1)
      x.o[3] = t(5, c ? 0 : 1), x.o[4] = t(1, c ? 1 : 0), x.o[5] = t(3, c ? 1 : 0);
    } else {
      x.o[0] = t(c ? 5 : 4, 0), x.o[1] = t(c ? 1 : 0, 1), x.o[2] = t(c ? 3 : 2, 1);  // t1
    }
    x.z = caddr(in + l, s < 3 ? 1 : 0);
  }
  return x;
}
GBV_HD void cyc_prod(const CycLane& x) {
  Fp a = cload(x.a[0]), b = cload(x.b[0]);
  const Fp a1 = cload(x.a[1]), a2 = cload(x.a[2]), a3 = cload(x.a[3]);
  const Fp b1 = cload(x.b[1]), b2 = cload(x.b[2]), b3 = cload(x.b[3]);
  fp_acc_lazy(a, a1);  // operands below 4p: the product takes them
  fp_acc_lazy(a, a2);
  fp_acc_lazy(a, a3);
  fp_acc_lazy(b, b1);
  fp_acc_lazy(b, b2);
  fp_acc_lazy(b, b3);
  put(x.dz, fp_mul_inl(a, b));
}
GBV_HD void cyc_out(const CycLane& x) {
  Fp u = cload(x.o[0]);
  Fp v[5];
  for (int i = 0; i < 5; ++i) v[i] = cload(x.o[1 + i]);
  const Fp z = cload(x.z);
  for (int i = 0; i < 5; ++i) fp_acc_lazy(u, v[i]);
  fp_reduce8_ip(u);  // < 6p -> canonical
  Fp r = u;
  fp_acc_lazy(r, u);
  fp_acc_lazy(r, u);
  fp_acc_lazy(r, z);
  fp_acc_lazy(r, z);
  fp_reduce8_ip(r);  // 3u +- 2z < 5p
  put(x.dout, r);
}
#if defined(GBV_HOST_TEST)
inline void cyc_sqr(Slot* mem, uint16_t zo, uint16_t ao, uint16_t co) {
  for (uint32_t l = 0; l < 18; ++l) cyc_prod(cyc_lane(mem, zo, ao, co, l));
  for (uint32_t l = 0; l < 12; ++l) cyc_out(cyc_lane(mem, zo, ao, co, l));
}
#else
__device__ __forceinline__ void cyc_sqr_lane(const CycLane& x) {
  const uint32_t l = lane_id();
  if (l < 18) cyc_prod(x);
  barrier();
  if (l < 12) cyc_out(x);
  barrier();
}
__device__ inline void cyc_sqr(Slot* mem, uint16_t zo, uint16_t ao, uint16_t co) { cyc_sqr_lane(cyc_lane(mem, zo, ao, co, lane_id())); }
#endif

// ---- Miller loop over up to 2 pairs ---------------------------------------------------------
// Workspace layout (slot offsets), MILLER_WS slots in total:
//   F 0..11 | L 12..17 | per pair j: T 18+12j (6), Q 24+12j (4), P 28+12j (2: -xP, yP) | Z 42..169
constexpr uint16_t M_F = 0, M_L = 12, M_PAIR = 18, M_Z = 42;
constexpr int MILLER_WS = M_Z + ZSLOTS;

// Load pair j: P affine G1, Q affine G2 (neither infinity).  Lane-parallel, ends with a barrier.
GBV_HD void miller_load_pair(Slot* mem, int j, const G1A& P, const G2A& Q) {
  LSlot* b = GBV_LDS(mem + M_PAIR + 12 * j);
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
      put(b + l, v);
    }
  }
  barrier();
}

// F = prod_j f_{|x|, Q_j}(P_j), conjugated (x < 0).  Pairs must be loaded first.
GBV_HD void miller_loop(Slot* mem, int npairs) {
#if defined(GBV_HOST_TEST)
  auto mline = [&]() { mul_line(mem, M_Z, M_F, M_L, M_F); };
  auto sqdbl = [&](int j) { sqr_dbl(mem, M_Z, M_F, M_PAIR + 12 * j, M_PAIR + 12 * j + 10, M_L, j == 0); };
#else
  // every lane's terms resolved once: f = f l, and per pair the bit's doubling (with f^2 for pair 0)
  const LineLane lx = line_lane(mem, M_Z, M_F, M_L, M_F, lane_id());
  const SqrDblLane d0 = sqr_dbl_lane(mem, M_Z, M_F, M_PAIR, M_PAIR + 10, M_L, lane_id());
  const SqrDblLane d1 = sqr_dbl_lane(mem, M_Z, M_F, M_PAIR + 12, M_PAIR + 22, M_L, lane_id());
  auto mline = [&]() { mul_line_lane(lx); };
  auto sqdbl = [&](int j) { sqr_dbl_run(j == 0 ? d0 : d1, j == 0); };
#endif
  set_one12(mem + M_F);
  for (int i = 62; i >= 0; --i) {
    for (int j = 0; j < npairs; ++j) {
      sqdbl(j);  // f^2 (pair 0, f = 1 on the first bit) and pair j's doubling step with its line
      mline();
    }
    if ((X_ABS >> i) & 1ull) {
      for (int j = 0; j < npairs; ++j) {
        uint16_t t = M_PAIR + 12 * j;
        run(G2_ADD_STEP, make_ws(mem, M_Z, t, (uint16_t)(t + 6), (uint16_t)(t + 10), t, M_L));
        mline();
      }
    }
  }
  conj12(mem + M_F);
}

// T (at M_PAIR) = 4 [2]T by the written-out doubling step (its line, through the P slots M_PAIR + 10,
// lands in M_L and is ignored; f is not touched).  The lane terms are resolved once per ladder.
#if defined(GBV_HOST_TEST)
struct DblPt {
  Slot* mem;
  void operator()() const { sqr_dbl(mem, M_Z, M_F, M_PAIR, M_PAIR + 10, M_L, false); }
};
inline DblPt dbl_point(Slot* mem) { return DblPt{mem}; }
#else
struct DblPt {
  SqrDblLane x;
  __device__ void operator()() const { sqr_dbl_run(x, false); }
};
__device__ inline DblPt dbl_point(Slot* mem) { return DblPt{sqr_dbl_lane(mem, M_Z, M_F, M_PAIR, M_PAIR + 10, M_L, lane_id())}; }
#endif

// [|x|] Q (Q affine, not infinity) by the Miller loop's point steps alone (the lines they also
// write to M_L are ignored): T ends at mem + M_PAIR in homogeneous projective coordinates
// (x = X/Z, y = Y/Z).  The mixed addition is incomplete only for T = +-Q, i.e. for Q of order
// dividing k -+ 1 with k < 2^64: a point of a small-order subgroup of E'(Fp2), never a hash output
// or a curve point that has a component in the order-r subgroup.
GBV_HD void mul_xabs_point(Slot* mem, const G2A& Q) {
  miller_load_pair(mem, 0, G1A{fp_zero(), fp_zero()}, Q);
  const uint16_t t = M_PAIR;
  const DblPt dbl = dbl_point(mem);
  for (int i = 62; i >= 0; --i) {
    dbl();
    if ((X_ABS >> i) & 1ull) run(G2_ADD_STEP, make_ws(mem, M_Z, t, (uint16_t)(t + 6), (uint16_t)(t + 10), t, M_L));
  }
}
// [a - b x^2] Q for the batch digits (sa, sb) -- the scalar of curve.h's jac_mul_2d_signed, by its
// signed joint ladder R = sum_i 2^i (+-Q +-E), E = -psi^2(Q) = [-x^2] Q -- on the cooperative point
// steps, with the two digits of a step added one after the other (+-Q, then +-E: affine points
// as they are, so no ladder table and no inversion): 31 doublings, 63 mixed additions.  T ends at
// mem + M_PAIR like mul_xabs_point's.  For Q in the order-r subgroup no addition meets T = +-(its
// operand): before a Q digit T = [2a + 2b lambda] Q with (a, b) != 0 -- never [+-1] Q -- and before an
// E digit T = [odd + even lambda] Q, never +-E (|a|, |b| < 2^33 and the lattice of (u, v) with
// u = v lambda mod r has no vector that short).  A point outside the subgroup gets a wrong multiple,
// and the subgroup check beside it rejects that set.  Workspace: Q at M_PAIR + 6, -Q, E, -E at
// M_PAIR + 12 / 16 / 20 (pair 1's slots).
GBV_HD void mul_2d_point(Slot* mem, const G2A& Q, const G2A& E, uint32_t sa, uint32_t sb) {
  const uint16_t t = M_PAIR, QP = t + 6, QN = t + 12, EP = t + 16, EN = t + 20;
  LSlot* b = GBV_LDS(mem + M_PAIR);
  COOP_LANES(l) {
    if (l < 24) {
      const G2A& p = (l >= 16) ? E : Q;
      Fp v;
      if (l == 4)
        v = FP_ONE;
      else if (l == 5 || l == 10 || l == 11)
        v = fp_zero();
      else {
        const uint32_t c = l < 4 ? l : l < 10 ? l - 6 : (l & 3);  // x.c0 x.c1 y.c0 y.c1
        v = c == 0 ? p.x.c0 : c == 1 ? p.x.c1 : c == 2 ? p.y.c0 : p.y.c1;
        const bool neg = c >= 2 && ((l < 4 && !((sa >> 31) & 1u)) || (l >= 12 && l < 16) || l >= 20);
        if (neg) v = fp_neg(v);
      }
      put(b + l, v);
    }
  }
  barrier();
  // T = +-Q (digit 31 of sa) is loaded; its E digit, then the 31 lower steps
  run(G2_ADD_STEP, make_ws(mem, M_Z, t, ((sb >> 31) & 1u) ? EP : EN, (uint16_t)(t + 10), t, M_L));
  const DblPt dbl = dbl_point(mem);
  for (int i = 30; i >= 0; --i) {
    dbl();
    run(G2_ADD_STEP, make_ws(mem, M_Z, t, ((sa >> i) & 1u) ? QP : QN, (uint16_t)(t + 10), t, M_L));
    run(G2_ADD_STEP, make_ws(mem, M_Z, t, ((sb >> i) & 1u) ? EP : EN, (uint16_t)(t + 10), t, M_L));
  }
}

// the point left by mul_xabs_point as a Jacobian point (X Z, Y Z^2, Z); one lane
GBV_HD G2J point_jac(const Slot* mem) {
  const LSlot* b = GBV_LDS(mem + M_PAIR);
  const Fp2 X{get(b + 0), get(b + 1)}, Y{get(b + 2), get(b + 3)}, Z{get(b + 4), get(b + 5)};
  return G2J{fp2_mul(X, Z), fp2_mul(Y, fp2_sqr(Z)), Z};
}

// ---- final exponentiation: f^(3 (p^12 - 1)/r) == 1 ? -----------------------------------------
// Workspace (slot offsets): F 0..11 (input, clobbered) | INV 12 | T 24 | A 36 | B 48 | C 60 |
// TMP 72 | TMP2 84 | Z 96..223
constexpr uint16_t E_F = 0, E_INV = 12, E_T = 24, E_A = 36, E_B = 48, E_C = 60, E_TMP = 72, E_TMP2 = 84, E_Z = 96;
constexpr int FINAL_EXP_WS = E_Z + ZSLOTS;

// r = a^x (a in the cyclotomic subgroup)
GBV_HD void exp_x(Slot* mem, uint16_t a, uint16_t r) {
  copy(mem + r, mem + a, 12);
#if defined(GBV_HOST_TEST)
  for (int i = 62; i >= 0; --i) {
    cyc_sqr(mem, E_Z, r, r);
    if ((X_ABS >> i) & 1ull) mul12(mem, E_Z, r, a, r);
  }
#else
  const CycLane x = cyc_lane(mem, E_Z, r, r, lane_id());
  const MulLane y = mul_lane(mem, E_Z, r, a, r, lane_id());
  for (int i = 62; i >= 0; --i) {
    cyc_sqr_lane(x);
    if ((X_ABS >> i) & 1ull) mul12_lane(y);
  }
#endif
  conj12(mem + r);
}

// f^-1 (E_F -> E_INV; E_T .. E_TMP are scratch) by norms down to Fp2, the products cooperative and
// one Fp2 inversion on lane 0: t = f conj(f) in Fp6, s = t^(p^2 + p^4) (two Frobenius maps), N = t s
// in Fp2, f^-1 = conj(f) s N^-1.  Against fp12_inv on one lane (~250 us: ~100 dependent thread-level
// Fp products around the Fp inversion) four cooperative products and the Fp2 inversion alone.
GBV_HD void inv12(Slot* mem) {
  copy(mem + E_TMP, mem + E_F, 12);
  conj12(mem + E_TMP);
  mul12(mem, E_Z, E_F, E_TMP, E_T);  // t
  frob12(mem, E_Z, 2, E_T, E_A);
  frob12(mem, E_Z, 2, E_A, E_B);
  mul12(mem, E_Z, E_A, E_B, E_C);    // s
  mul12(mem, E_Z, E_T, E_C, E_A);    // N (coordinates 0, 1; the rest 0)
  mul12(mem, E_Z, E_TMP, E_C, E_B);  // conj(f) s
  COOP_LANE0 {
    const Fp2 ni = fp2_inv(Fp2{get(GBV_LDS(mem + E_A)), get(GBV_LDS(mem + E_A + 1))});
    put(GBV_LDS(mem + E_A), ni.c0);
    put(GBV_LDS(mem + E_A + 1), ni.c1);
  }
  barrier();
  mul12(mem, E_Z, E_B, E_A, E_INV);
}

// f (at mem + E_F) -> returns f^(3 (p^12-1)/r) == 1 (same value on every lane)
GBV_HD bool final_exp_is_one(Slot* mem) {
  inv12(mem);
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
  cyc_sqr(mem, E_Z, E_T, E_TMP);
  mul12(mem, E_Z, E_TMP, E_T, E_TMP);     // t^3
  mul12(mem, E_Z, E_C, E_TMP, E_C);
  return is_one12(mem + E_C);
}

}  // namespace coop
}  // namespace gbv
