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
struct Prod { uint16_t a0, an, b0, bn; };
struct Part { uint16_t t0, tn, z; };
struct Out { uint16_t t0, tn; uint8_t dst, idx; };
struct Prog {
  uint8_t n_rounds, n_part, n_out;
  uint16_t round_end[6];
  const Prod* prods;
  const Part* parts;
  const Out* outs;
  const Term* terms;
};
enum { SRC_Z = 6, SRC_C = 7 };

}  // namespace coop
}  // namespace gbv

#include "coop_tables.h"

namespace gbv {
namespace coop {

constexpr int LANES = 64;
constexpr int ZSLOTS = 128;

// Per-wave workspace: mem[] is LDS on the device; operand k of a program lives at mem + op[k].
struct Ws {
  Fp* mem;
  uint16_t op[6];
  uint16_t z;
};

GBV_HD Fp ws_get(const Ws& w, uint8_t src, uint8_t idx) {
  if (src == SRC_C) return CONSTS[idx];
  uint32_t base = src == SRC_Z ? w.z : w.op[src];
  return w.mem[base + idx];
}

// sum of coef * value over a term list (coefficients are small integers: double-and-add)
GBV_HD Fp lin_eval(const Ws& w, const Term* t, int n) {
  Fp acc = fp_zero();
  for (int i = 0; i < n; ++i) {
    Term tt = t[i];
    Fp v = ws_get(w, tt.src, tt.idx);
    int c = tt.coef;
    bool neg = c < 0;
    if (neg) c = -c;
    Fp s;
    if (c == 1) {
      s = v;
    } else {
      bool have = false;
      while (c) {
        if (c & 1) {
          s = have ? fp_add(s, v) : v;
          have = true;
        }
        c >>= 1;
        if (c) v = fp_dbl(v);
      }
    }
    acc = i == 0 ? (neg ? fp_neg(s) : s) : (neg ? fp_sub(acc, s) : fp_add(acc, s));
  }
  return acc;
}

GBV_HD void prod_lane(const Prog& P, int k, const Ws& w) {
  Prod pr = P.prods[k];
  Fp x = lin_eval(w, P.terms + pr.a0, pr.an);
  Fp y = lin_eval(w, P.terms + pr.b0, pr.bn);
  w.mem[w.z + k] = fp_mul(x, y);
}

GBV_HD void part_lane(const Prog& P, int j, const Ws& w) {
  Part pt = P.parts[j];
  w.mem[w.z + pt.z] = lin_eval(w, P.terms + pt.t0, pt.tn);
}

GBV_HD Fp out_lane(const Prog& P, int o, const Ws& w) {
  Out ou = P.outs[o];
  return lin_eval(w, P.terms + ou.t0, ou.tn);
}

#if defined(GBV_HOST_TEST)
inline unsigned lane_id() { return 0; }
inline void barrier() {}

// Host: the lanes of each phase run one after another.
inline void run(const Prog& P, const Ws& w) {
  int p0 = 0;
  for (int r = 0; r < P.n_rounds; ++r) {
    for (int k = p0; k < P.round_end[r]; ++k) prod_lane(P, k, w);
    p0 = P.round_end[r];
  }
  for (int j = 0; j < P.n_part; ++j) part_lane(P, j, w);
  Fp o[LANES];
  for (int k = 0; k < P.n_out; ++k) o[k] = out_lane(P, k, w);
  for (int k = 0; k < P.n_out; ++k) w.mem[w.op[P.outs[k].dst] + P.outs[k].idx] = o[k];
}
#define COOP_LANES(l) for (unsigned l = 0; l < (unsigned)LANES; ++l)
#define COOP_LANE0 if (true)
#else
__device__ inline unsigned lane_id() { return threadIdx.x; }
__device__ inline void barrier() { __syncthreads(); }

__device__ inline void run(const Prog& P, const Ws& w) {
  const int lane = (int)threadIdx.x;
  int p0 = 0;
  for (int r = 0; r < P.n_rounds; ++r) {
    int p1 = P.round_end[r];
    if (p0 + lane < p1) prod_lane(P, p0 + lane, w);  // every round has <= 64 products
    p0 = p1;
    __syncthreads();
  }
  if (lane < P.n_part) {
    part_lane(P, lane, w);
  }
  if (P.n_part) __syncthreads();
  Fp o;
  bool have = lane < P.n_out;
  if (have) o = out_lane(P, lane, w);
  __syncthreads();
  if (have) w.mem[w.op[P.outs[lane].dst] + P.outs[lane].idx] = o;
  __syncthreads();
}
#define COOP_LANES(l) for (unsigned l = threadIdx.x; l == threadIdx.x; l = ~0u)
#define COOP_LANE0 if (threadIdx.x == 0)
#endif

// ---- operand helpers (lane-parallel, end with a barrier) ------------------------------------
GBV_HD void set_one12(Fp* f) {
  COOP_LANES(l) if (l < 12) f[l] = l == 0 ? FP_ONE : fp_zero();
  barrier();
}
GBV_HD void copy(Fp* dst, const Fp* src, unsigned n) {
  COOP_LANES(l) if (l < n) dst[l] = src[l];
  barrier();
}
GBV_HD void conj12(Fp* f) {  // negate the w-odd half (coordinates 6..11)
  COOP_LANES(l) if (l >= 6 && l < 12) f[l] = fp_neg(f[l]);
  barrier();
}
GBV_HD bool is_one12(const Fp* f) {
  bool ok = true;
  for (int i = 0; i < 12; ++i) ok = ok && fp_eq(f[i], i == 0 ? FP_ONE : fp_zero());
  return ok;
}

GBV_HD Ws ws2(Fp* mem, uint16_t z, uint16_t a, uint16_t b) { return Ws{mem, {a, b, 0, 0, 0, 0}, z}; }
GBV_HD Ws ws3(Fp* mem, uint16_t z, uint16_t a, uint16_t b, uint16_t c) { return Ws{mem, {a, b, c, 0, 0, 0}, z}; }

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
  Fp* b = mem + M_PAIR + 12 * j;
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
      b[l] = v;
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
      run(G2_DBL_STEP, Ws{mem, {t, (uint16_t)(t + 10), t, M_L, 0, 0}, M_Z});
      run(FP12_MUL_LINE, ws3(mem, M_Z, M_F, M_L, M_F));
    }
    if ((X_ABS >> i) & 1ull) {
      for (int j = 0; j < npairs; ++j) {
        uint16_t t = M_PAIR + 12 * j;
        run(G2_ADD_STEP, Ws{mem, {t, (uint16_t)(t + 6), (uint16_t)(t + 10), t, M_L, 0}, M_Z});
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
