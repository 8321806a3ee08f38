/*
 * blsport.c -- CPU port of the BLS12-381 same-message / signature-set verification path.
 * TEST/BENCH INFRASTRUCTURE ONLY (oracle/): used as bench.py's `cpu_baseline` ("port") and as a
 * second CPU checker in tests.  The product (lodestar_amd) never links or calls it.
 *
 * What it restates: the arithmetic @chainsafe/blst 2.1.0 performs for
 * BlsMultiThreadWorkerPool.verifySignatureSetsSameMessage (multithread/index.ts:212-236):
 * per set Signature.fromBytes(sig, true) (decompress + subgroup check) and the 64-bit random
 * scalar multiplications of aggregateWithRandomness (jobItem.ts:73), per chunk hash_to_G2 and the
 * 2-pair pairing check of verify() (maybeBatch.ts:34-38), per-set retry on failure
 * (jobItem.ts:93-125).  The thread pool shape mirrors the reference pool: N worker threads
 * pulling <=128-set chunks (multithread/index.ts:46,56; poolSize.ts:7).
 *
 * 6 x 64-bit limbs, Montgomery (R = 2^384), CIOS with unsigned __int128.  No assembly, no
 * external library: a "CPU stand-in, not blst" baseline.
 */
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef struct { uint64_t l[6]; } fp;
typedef struct { fp c0, c1; } fp2;
typedef struct { fp2 c0, c1, c2; } fp6;
typedef struct { fp6 c0, c1; } fp12;

static const fp P = {{0xb9feffffffffaaabULL, 0x1eabfffeb153ffffULL, 0x6730d2a0f6b0f624ULL,
                      0x64774b84f38512bfULL, 0x4b1ba7b6434bacd7ULL, 0x1a0111ea397fe69aULL}};
static const uint64_t NP0 = 0x89f3fffcfffcfffdULL; /* -p^-1 mod 2^64 */
static fp R1, R2, R2_256, INV2, B1M, NEG_G1Y, G1X_M;
static fp2 B2M, B2M3, PSI_X, PSI_Y, FROB_V1, FROB_V2, FROB_W, FROB_V1W, FROB_V2W;
static fp2 SSWU_A, SSWU_B, SSWU_Z, SSWU_NB_A, SSWU_B_ZA;
static fp2 ISO_XN[4], ISO_XD[3], ISO_YN[4], ISO_YD[4];
static uint64_t E_SQRT[6], E_SQRTM3[6], E_INV[6];
static const uint64_t X_ABS = 0xd201000000010000ULL;

/* ---------------- Fp ---------------- */
static inline int fp_is_zero(const fp* a) { return (a->l[0] | a->l[1] | a->l[2] | a->l[3] | a->l[4] | a->l[5]) == 0; }
static inline int fp_eq(const fp* a, const fp* b) { return memcmp(a, b, sizeof(fp)) == 0; }

static inline void fp_reduce(fp* r) {
  fp t;
  uint64_t br = 0;
  for (int i = 0; i < 6; ++i) {
    u128 d = (u128)r->l[i] - P.l[i] - br;
    t.l[i] = (uint64_t)d;
    br = (uint64_t)(d >> 127);
  }
  if (!br) *r = t;
}

static inline void fp_add(fp* r, const fp* a, const fp* b) {
  uint64_t c = 0;
  for (int i = 0; i < 6; ++i) {
    u128 s = (u128)a->l[i] + b->l[i] + c;
    r->l[i] = (uint64_t)s;
    c = (uint64_t)(s >> 64);
  }
  fp_reduce(r);
}

static inline void fp_sub(fp* r, const fp* a, const fp* b) {
  uint64_t br = 0;
  fp t;
  for (int i = 0; i < 6; ++i) {
    u128 d = (u128)a->l[i] - b->l[i] - br;
    t.l[i] = (uint64_t)d;
    br = (uint64_t)(d >> 127);
  }
  if (br) {
    uint64_t c = 0;
    for (int i = 0; i < 6; ++i) {
      u128 s = (u128)t.l[i] + P.l[i] + c;
      t.l[i] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
  }
  *r = t;
}

static inline void fp_neg(fp* r, const fp* a) {
  if (fp_is_zero(a)) { *r = *a; return; }
  fp z = {{0}};
  fp_sub(r, &z, a);
}

static inline void fp_dbl(fp* r, const fp* a) { fp_add(r, a, a); }

static void fp_mul(fp* r, const fp* a, const fp* b) {
  uint64_t t[6] = {0};
  for (int i = 0; i < 6; ++i) {
    u128 A = (u128)a->l[0] * b->l[i] + t[0];
    uint64_t m = (uint64_t)A * NP0;
    u128 C = (u128)m * P.l[0] + (uint64_t)A;
    A >>= 64;
    C >>= 64;
    for (int j = 1; j < 6; ++j) {
      A = (u128)a->l[j] * b->l[i] + t[j] + (uint64_t)A;
      C = (u128)m * P.l[j] + (uint64_t)A + (uint64_t)C;
      t[j - 1] = (uint64_t)C;
      A >>= 64;
      C >>= 64;
    }
    t[5] = (uint64_t)A + (uint64_t)C;
  }
  memcpy(r->l, t, sizeof t);
  fp_reduce(r);
}

static inline void fp_sqr(fp* r, const fp* a) { fp_mul(r, a, a); }

static void fp_pow(fp* r, const fp* a, const uint64_t* e) {
  int top = 383;
  while (top > 0 && !((e[top >> 6] >> (top & 63)) & 1)) --top;
  fp acc = *a, base = *a;
  for (int i = top - 1; i >= 0; --i) {
    fp_sqr(&acc, &acc);
    if ((e[i >> 6] >> (i & 63)) & 1) fp_mul(&acc, &acc, &base);
  }
  *r = acc;
}

static void fp_inv(fp* r, const fp* a) { fp_pow(r, a, E_INV); }

static void fp_from_raw(fp* r, const uint64_t v[6]) {
  fp t;
  memcpy(t.l, v, 48);
  fp_mul(r, &t, &R2);
}

static void fp_to_raw(uint64_t v[6], const fp* a) {
  fp one = {{1, 0, 0, 0, 0, 0}}, t;
  fp_mul(&t, a, &one);
  memcpy(v, t.l, 48);
}

static void be48_to_raw(uint64_t v[6], const uint8_t* b) {
  for (int i = 0; i < 6; ++i) {
    uint64_t w = 0;
    for (int k = 0; k < 8; ++k) w = (w << 8) | b[40 - 8 * i + k];
    v[i] = w;
  }
}

static void raw_to_be48(uint8_t* b, const uint64_t v[6]) {
  for (int i = 0; i < 6; ++i)
    for (int k = 0; k < 8; ++k) b[40 - 8 * i + k] = (uint8_t)(v[i] >> (56 - 8 * k));
}

static int raw_lt_p(const uint64_t v[6]) {
  for (int i = 5; i >= 0; --i) {
    if (v[i] < P.l[i]) return 1;
    if (v[i] > P.l[i]) return 0;
  }
  return 0;
}

static int fp_lexi_large(const fp* a) {
  uint64_t v[6], h[6];
  fp_to_raw(v, a);
  /* (p-1)/2 */
  uint64_t c = 0;
  for (int i = 5; i >= 0; --i) {
    uint64_t w = P.l[i];
    h[i] = (w >> 1) | (c << 63);
    c = w & 1;
  }
  for (int i = 5; i >= 0; --i) {
    if (v[i] > h[i]) return 1;
    if (v[i] < h[i]) return 0;
  }
  return 0;
}

/* ---------------- Fp2 ---------------- */
static inline void fp2_add(fp2* r, const fp2* a, const fp2* b) { fp_add(&r->c0, &a->c0, &b->c0); fp_add(&r->c1, &a->c1, &b->c1); }
static inline void fp2_sub(fp2* r, const fp2* a, const fp2* b) { fp_sub(&r->c0, &a->c0, &b->c0); fp_sub(&r->c1, &a->c1, &b->c1); }
static inline void fp2_neg(fp2* r, const fp2* a) { fp_neg(&r->c0, &a->c0); fp_neg(&r->c1, &a->c1); }
static inline void fp2_dbl(fp2* r, const fp2* a) { fp2_add(r, a, a); }
static inline int fp2_is_zero(const fp2* a) { return fp_is_zero(&a->c0) && fp_is_zero(&a->c1); }
static inline int fp2_eq(const fp2* a, const fp2* b) { return fp_eq(&a->c0, &b->c0) && fp_eq(&a->c1, &b->c1); }
static inline void fp2_conj(fp2* r, const fp2* a) { r->c0 = a->c0; fp_neg(&r->c1, &a->c1); }

static void fp2_mul(fp2* r, const fp2* a, const fp2* b) {
  fp t0, t1, s0, s1, t2;
  fp_mul(&t0, &a->c0, &b->c0);
  fp_mul(&t1, &a->c1, &b->c1);
  fp_add(&s0, &a->c0, &a->c1);
  fp_add(&s1, &b->c0, &b->c1);
  fp_mul(&t2, &s0, &s1);
  fp_sub(&r->c0, &t0, &t1);
  fp_sub(&t2, &t2, &t0);
  fp_sub(&r->c1, &t2, &t1);
}

static void fp2_sqr(fp2* r, const fp2* a) {
  fp s, d, t;
  fp_add(&s, &a->c0, &a->c1);
  fp_sub(&d, &a->c0, &a->c1);
  fp_mul(&t, &a->c0, &a->c1);
  fp_mul(&r->c0, &s, &d);
  fp_dbl(&r->c1, &t);
}

static inline void fp2_mul_fp(fp2* r, const fp2* a, const fp* s) { fp_mul(&r->c0, &a->c0, s); fp_mul(&r->c1, &a->c1, s); }
static inline void fp2_mul_xi(fp2* r, const fp2* a) {
  fp t0, t1;
  fp_sub(&t0, &a->c0, &a->c1);
  fp_add(&t1, &a->c0, &a->c1);
  r->c0 = t0;
  r->c1 = t1;
}

static void fp2_inv(fp2* r, const fp2* a) {
  fp n, t, ni;
  fp_sqr(&n, &a->c0);
  fp_sqr(&t, &a->c1);
  fp_add(&n, &n, &t);
  fp_inv(&ni, &n);
  fp_mul(&r->c0, &a->c0, &ni);
  fp_mul(&t, &a->c1, &ni);
  fp_neg(&r->c1, &t);
}

static int fp2_sqrt(fp2* root, const fp2* a) {
  fp n, t, alpha, delta, d2, x0, h, q;
  fp_sqr(&n, &a->c0);
  fp_sqr(&t, &a->c1);
  fp_add(&n, &n, &t);
  fp_pow(&alpha, &n, E_SQRT);
  fp_add(&t, &a->c0, &alpha);
  fp_mul(&delta, &t, &INV2);
  if (fp_is_zero(&delta)) {
    fp_sub(&t, &a->c0, &alpha);
    fp_mul(&d2, &t, &INV2);
    delta = d2;
  }
  fp_pow(&t, &delta, E_SQRTM3);
  fp_mul(&x0, &t, &delta);
  fp_mul(&q, &x0, &t);
  fp_mul(&h, &a->c1, &t);
  fp_mul(&h, &h, &INV2);
  if (fp_eq(&q, &R1)) {
    root->c0 = x0;
    root->c1 = h;
  } else {
    fp_neg(&root->c0, &h);
    root->c1 = x0;
  }
  fp2 chk;
  fp2_sqr(&chk, root);
  return fp2_eq(&chk, a);
}

static int fp2_lexi_large(const fp2* a) { return fp_is_zero(&a->c1) ? fp_lexi_large(&a->c0) : fp_lexi_large(&a->c1); }

static int fp2_sgn0(const fp2* a) {
  uint64_t v0[6], v1[6];
  fp_to_raw(v0, &a->c0);
  fp_to_raw(v1, &a->c1);
  int z0 = (v0[0] | v0[1] | v0[2] | v0[3] | v0[4] | v0[5]) == 0;
  return (int)(v0[0] & 1) | (z0 & (int)(v1[0] & 1));
}

/* ---------------- Fp6 / Fp12 ---------------- */
static void fp6_add(fp6* r, const fp6* a, const fp6* b) { fp2_add(&r->c0, &a->c0, &b->c0); fp2_add(&r->c1, &a->c1, &b->c1); fp2_add(&r->c2, &a->c2, &b->c2); }
static void fp6_sub(fp6* r, const fp6* a, const fp6* b) { fp2_sub(&r->c0, &a->c0, &b->c0); fp2_sub(&r->c1, &a->c1, &b->c1); fp2_sub(&r->c2, &a->c2, &b->c2); }
static void fp6_neg(fp6* r, const fp6* a) { fp2_neg(&r->c0, &a->c0); fp2_neg(&r->c1, &a->c1); fp2_neg(&r->c2, &a->c2); }
static void fp6_mul_v(fp6* r, const fp6* a) {
  fp2 t;
  fp2_mul_xi(&t, &a->c2);
  r->c2 = a->c1;
  r->c1 = a->c0;
  r->c0 = t;
}

static void fp6_mul(fp6* r, const fp6* a, const fp6* b) {
  fp2 t0, t1, t2, s, u, c0, c1, c2;
  fp2_mul(&t0, &a->c0, &b->c0);
  fp2_mul(&t1, &a->c1, &b->c1);
  fp2_mul(&t2, &a->c2, &b->c2);
  fp2_add(&s, &a->c1, &a->c2); fp2_add(&u, &b->c1, &b->c2); fp2_mul(&c0, &s, &u);
  fp2_sub(&c0, &c0, &t1); fp2_sub(&c0, &c0, &t2); fp2_mul_xi(&c0, &c0); fp2_add(&c0, &c0, &t0);
  fp2_add(&s, &a->c0, &a->c1); fp2_add(&u, &b->c0, &b->c1); fp2_mul(&c1, &s, &u);
  fp2_sub(&c1, &c1, &t0); fp2_sub(&c1, &c1, &t1); fp2_mul_xi(&s, &t2); fp2_add(&c1, &c1, &s);
  fp2_add(&s, &a->c0, &a->c2); fp2_add(&u, &b->c0, &b->c2); fp2_mul(&c2, &s, &u);
  fp2_sub(&c2, &c2, &t0); fp2_sub(&c2, &c2, &t2); fp2_add(&c2, &c2, &t1);
  r->c0 = c0; r->c1 = c1; r->c2 = c2;
}

static void fp6_mul_by_01(fp6* r, const fp6* f, const fp2* a, const fp2* b) {
  fp2 t0, t1, s, u, c0, c1, c2;
  fp2_mul(&t0, &f->c0, a);
  fp2_mul(&t1, &f->c1, b);
  fp2_add(&s, &f->c0, &f->c1); fp2_add(&u, a, b); fp2_mul(&c1, &s, &u);
  fp2_sub(&c1, &c1, &t0); fp2_sub(&c1, &c1, &t1);
  fp2_mul(&s, &f->c2, b); fp2_mul_xi(&s, &s); fp2_add(&c0, &t0, &s);
  fp2_mul(&s, &f->c2, a); fp2_add(&c2, &t1, &s);
  r->c0 = c0; r->c1 = c1; r->c2 = c2;
}

static void fp6_mul_by_1(fp6* r, const fp6* f, const fp2* c) {
  fp2 c0, c1, c2;
  fp2_mul(&c0, &f->c2, c); fp2_mul_xi(&c0, &c0);
  fp2_mul(&c1, &f->c0, c);
  fp2_mul(&c2, &f->c1, c);
  r->c0 = c0; r->c1 = c1; r->c2 = c2;
}

static void fp6_inv(fp6* r, const fp6* a) {
  fp2 t0, t1, t2, s, d, di;
  fp2_sqr(&t0, &a->c0); fp2_mul(&s, &a->c1, &a->c2); fp2_mul_xi(&s, &s); fp2_sub(&t0, &t0, &s);
  fp2_sqr(&t1, &a->c2); fp2_mul_xi(&t1, &t1); fp2_mul(&s, &a->c0, &a->c1); fp2_sub(&t1, &t1, &s);
  fp2_sqr(&t2, &a->c1); fp2_mul(&s, &a->c0, &a->c2); fp2_sub(&t2, &t2, &s);
  fp2_mul(&d, &a->c2, &t1); fp2_mul(&s, &a->c1, &t2); fp2_add(&d, &d, &s); fp2_mul_xi(&d, &d);
  fp2_mul(&s, &a->c0, &t0); fp2_add(&d, &d, &s);
  fp2_inv(&di, &d);
  fp2_mul(&r->c0, &t0, &di); fp2_mul(&r->c1, &t1, &di); fp2_mul(&r->c2, &t2, &di);
}

static void fp12_one(fp12* r) { memset(r, 0, sizeof *r); r->c0.c0.c0 = R1; }
static int fp12_is_one(const fp12* a) { fp12 o; fp12_one(&o); return memcmp(a, &o, sizeof o) == 0; }
static void fp12_conj(fp12* r, const fp12* a) { r->c0 = a->c0; fp6_neg(&r->c1, &a->c1); }

static void fp12_mul(fp12* r, const fp12* a, const fp12* b) {
  fp6 t0, t1, s, u, c1;
  fp6_mul(&t0, &a->c0, &b->c0);
  fp6_mul(&t1, &a->c1, &b->c1);
  fp6_add(&s, &a->c0, &a->c1); fp6_add(&u, &b->c0, &b->c1); fp6_mul(&c1, &s, &u);
  fp6_sub(&c1, &c1, &t0); fp6_sub(&c1, &c1, &t1);
  fp6_mul_v(&t1, &t1);
  fp6_add(&r->c0, &t0, &t1);
  r->c1 = c1;
}

static void fp12_sqr(fp12* r, const fp12* a) {
  fp6 t, s, u, c0;
  fp6_mul(&t, &a->c0, &a->c1);
  fp6_add(&s, &a->c0, &a->c1); fp6_mul_v(&u, &a->c1); fp6_add(&u, &a->c0, &u); fp6_mul(&c0, &s, &u);
  fp6_sub(&c0, &c0, &t); fp6_mul_v(&s, &t); fp6_sub(&c0, &c0, &s);
  r->c0 = c0;
  fp6_add(&r->c1, &t, &t);
}

static void fp12_mul_line(fp12* f, const fp2* c0, const fp2* c2, const fp2* c3) {
  fp6 a, b, e, s;
  fp2 c23;
  fp6_mul_by_01(&a, &f->c0, c0, c2);
  fp6_mul_by_1(&b, &f->c1, c3);
  fp6_add(&s, &f->c0, &f->c1); fp2_add(&c23, c2, c3); fp6_mul_by_01(&e, &s, c0, &c23);
  fp6_sub(&e, &e, &a); fp6_sub(&e, &e, &b);
  fp6_mul_v(&b, &b);
  fp6_add(&f->c0, &a, &b);
  f->c1 = e;
}

static void fp12_inv(fp12* r, const fp12* a) {
  fp6 d, t, di;
  fp6_mul(&d, &a->c0, &a->c0);
  fp6_mul(&t, &a->c1, &a->c1); fp6_mul_v(&t, &t); fp6_sub(&d, &d, &t);
  fp6_inv(&di, &d);
  fp6_mul(&r->c0, &a->c0, &di);
  fp6_mul(&t, &a->c1, &di); fp6_neg(&r->c1, &t);
}

static void fp12_frob(fp12* r, const fp12* a) {
  fp2 t;
  fp2_conj(&r->c0.c0, &a->c0.c0);
  fp2_conj(&t, &a->c0.c1); fp2_mul(&r->c0.c1, &t, &FROB_V1);
  fp2_conj(&t, &a->c0.c2); fp2_mul(&r->c0.c2, &t, &FROB_V2);
  fp2_conj(&t, &a->c1.c0); fp2_mul(&r->c1.c0, &t, &FROB_W);
  fp2_conj(&t, &a->c1.c1); fp2_mul(&r->c1.c1, &t, &FROB_V1W);
  fp2_conj(&t, &a->c1.c2); fp2_mul(&r->c1.c2, &t, &FROB_V2W);
}

static void fp12_exp_x(fp12* r, const fp12* a) {
  fp12 acc = *a;
  for (int i = 62; i >= 0; --i) {
    fp12_sqr(&acc, &acc);
    if ((X_ABS >> i) & 1) fp12_mul(&acc, &acc, a);
  }
  fp12_conj(r, &acc);
}

static void final_exp(fp12* r, const fp12* f) {
  fp12 t, u, a, b, c, t3;
  fp12_conj(&t, f); fp12_inv(&u, f); fp12_mul(&t, &t, &u);
  fp12_frob(&u, &t); fp12_frob(&u, &u); fp12_mul(&t, &u, &t);
  fp12_exp_x(&a, &t); fp12_conj(&u, &t); fp12_mul(&a, &a, &u);
  fp12_exp_x(&u, &a); fp12_conj(&c, &a); fp12_mul(&a, &u, &c);
  fp12_exp_x(&b, &a); fp12_frob(&u, &a); fp12_mul(&b, &b, &u);
  fp12_exp_x(&c, &b); fp12_exp_x(&c, &c); fp12_frob(&u, &b); fp12_frob(&u, &u); fp12_mul(&c, &c, &u);
  fp12_conj(&u, &b); fp12_mul(&c, &c, &u);
  fp12_sqr(&t3, &t); fp12_mul(&t3, &t3, &t);
  fp12_mul(r, &c, &t3);
}

/* ---------------- points ---------------- */
typedef struct { fp x, y, z; } g1j;
typedef struct { fp x, y; } g1a;
typedef struct { fp2 x, y, z; } g2j;
typedef struct { fp2 x, y; } g2a;


#define CURVE_FUNCS(PFX, F, T, A, ONE_INIT)                                                           \
  static void PFX##_dbl(T* r, const T* p) {                                                           \
    F a, b, c, d, e, f, t, z3;                                                                        \
    F##_sqr(&a, &p->x); F##_sqr(&b, &p->y); F##_sqr(&c, &b);                                          \
    F##_add(&t, &p->x, &b); F##_sqr(&t, &t); F##_sub(&t, &t, &a); F##_sub(&t, &t, &c); F##_dbl(&d, &t); \
    F##_dbl(&e, &a); F##_add(&e, &e, &a); F##_sqr(&f, &e);                                            \
    F##_mul(&z3, &p->y, &p->z); F##_dbl(&z3, &z3);                                                    \
    F##_dbl(&t, &d); F##_sub(&r->x, &f, &t);                                                          \
    F##_dbl(&c, &c); F##_dbl(&c, &c); F##_dbl(&c, &c);                                                \
    F##_sub(&t, &d, &r->x); F##_mul(&t, &e, &t); F##_sub(&r->y, &t, &c);                              \
    r->z = z3;                                                                                        \
  }                                                                                                   \
  static void PFX##_add_aff(T* r, const T* p, const A* q) {                                           \
    if (F##_is_zero(&p->z)) { r->x = q->x; r->y = q->y; ONE_INIT(r->z); return; }                     \
    F z1z1, u2, s2, h, rr, hh, i, j, v, t;                                                            \
    F##_sqr(&z1z1, &p->z); F##_mul(&u2, &q->x, &z1z1);                                                \
    F##_mul(&s2, &p->z, &z1z1); F##_mul(&s2, &q->y, &s2);                                             \
    F##_sub(&h, &u2, &p->x); F##_sub(&rr, &s2, &p->y); F##_dbl(&rr, &rr);                             \
    if (F##_is_zero(&h)) {                                                                            \
      if (F##_is_zero(&rr)) { PFX##_dbl(r, p); return; }                                              \
      memset(r, 0, sizeof *r); return;                                                                \
    }                                                                                                 \
    F##_sqr(&hh, &h); F##_dbl(&i, &hh); F##_dbl(&i, &i); F##_mul(&j, &h, &i); F##_mul(&v, &p->x, &i); \
    T o;                                                                                              \
    F##_sqr(&t, &rr); F##_sub(&t, &t, &j); F##_sub(&t, &t, &v); F##_sub(&o.x, &t, &v);                \
    F##_sub(&t, &v, &o.x); F##_mul(&t, &rr, &t); F##_mul(&v, &p->y, &j); F##_dbl(&v, &v);            \
    F##_sub(&o.y, &t, &v);                                                                            \
    F##_add(&t, &p->z, &h); F##_sqr(&t, &t); F##_sub(&t, &t, &z1z1); F##_sub(&o.z, &t, &hh);          \
    *r = o;                                                                                           \
  }                                                                                                   \
  static void PFX##_add(T* r, const T* p, const T* q) {                                               \
    if (F##_is_zero(&p->z)) { *r = *q; return; }                                                      \
    if (F##_is_zero(&q->z)) { *r = *p; return; }                                                      \
    F z1z1, z2z2, u1, u2, s1, s2, h, rr, i, j, v, t;                                                  \
    F##_sqr(&z1z1, &p->z); F##_sqr(&z2z2, &q->z);                                                     \
    F##_mul(&u1, &p->x, &z2z2); F##_mul(&u2, &q->x, &z1z1);                                           \
    F##_mul(&s1, &q->z, &z2z2); F##_mul(&s1, &p->y, &s1);                                             \
    F##_mul(&s2, &p->z, &z1z1); F##_mul(&s2, &q->y, &s2);                                             \
    F##_sub(&h, &u2, &u1); F##_sub(&rr, &s2, &s1); F##_dbl(&rr, &rr);                                 \
    if (F##_is_zero(&h)) {                                                                            \
      if (F##_is_zero(&rr)) { PFX##_dbl(r, p); return; }                                              \
      memset(r, 0, sizeof *r); return;                                                                \
    }                                                                                                 \
    F##_dbl(&i, &h); F##_sqr(&i, &i); F##_mul(&j, &h, &i); F##_mul(&v, &u1, &i);                      \
    T o;                                                                                              \
    F##_sqr(&t, &rr); F##_sub(&t, &t, &j); F##_sub(&t, &t, &v); F##_sub(&o.x, &t, &v);                \
    F##_sub(&t, &v, &o.x); F##_mul(&t, &rr, &t); F##_mul(&v, &s1, &j); F##_dbl(&v, &v);              \
    F##_sub(&o.y, &t, &v);                                                                            \
    F##_add(&t, &p->z, &q->z); F##_sqr(&t, &t); F##_sub(&t, &t, &z1z1); F##_sub(&t, &t, &z2z2);       \
    F##_mul(&o.z, &t, &h);                                                                            \
    *r = o;                                                                                           \
  }                                                                                                   \
  static int PFX##_to_aff(A* r, const T* p) {                                                         \
    if (F##_is_zero(&p->z)) return 0;                                                                 \
    F zi, zi2, t;                                                                                     \
    F##_inv(&zi, &p->z); F##_sqr(&zi2, &zi);                                                          \
    F##_mul(&r->x, &p->x, &zi2); F##_mul(&t, &zi2, &zi); F##_mul(&r->y, &p->y, &t);                 \
    return 1;                                                                                         \
  }                                                                                                   \
  static void PFX##_mul_u64(T* r, const A* q, uint64_t k) {                                          \
    memset(r, 0, sizeof *r);                                                                          \
    if (!k) return;                                                                                   \
    int top = 63;                                                                                     \
    while (!((k >> top) & 1)) --top;                                                                  \
    r->x = q->x; r->y = q->y; ONE_INIT(r->z);                                                         \
    for (int i = top - 1; i >= 0; --i) {                                                              \
      PFX##_dbl(r, r);                                                                                \
      if ((k >> i) & 1) PFX##_add_aff(r, r, q);                                                       \
    }                                                                                                 \
  }

#define FP_ONE_INIT(z) ((z) = R1)
#define FP2_ONE_INIT(z) ((z).c0 = R1, memset(&(z).c1, 0, sizeof(fp)))
CURVE_FUNCS(g1, fp, g1j, g1a, FP_ONE_INIT)
CURVE_FUNCS(g2, fp2, g2j, g2a, FP2_ONE_INIT)

static void g2_psi(g2a* r, const g2a* a) {
  fp2 t;
  fp2_conj(&t, &a->x); fp2_mul(&r->x, &t, &PSI_X);
  fp2_conj(&t, &a->y); fp2_mul(&r->y, &t, &PSI_Y);
}

static void g2_psi_j(g2j* r, const g2j* a) {
  fp2 t;
  fp2_conj(&t, &a->x); fp2_mul(&r->x, &t, &PSI_X);
  fp2_conj(&t, &a->y); fp2_mul(&r->y, &t, &PSI_Y);
  fp2_conj(&r->z, &a->z);
}

static void g2_mul_xabs_j(g2j* r, const g2j* q) {
  g2j acc = *q;
  for (int i = 62; i >= 0; --i) {
    g2_dbl(&acc, &acc);
    if ((X_ABS >> i) & 1) g2_add(&acc, &acc, q);
  }
  *r = acc;
}

static int g2_in_subgroup(const g2a* q) {
  g2j x;
  g2_mul_u64(&x, q, X_ABS);
  fp2_neg(&x.y, &x.y);
  g2a ps;
  g2_psi(&ps, q);
  if (fp2_is_zero(&x.z)) return 0;
  fp2 z2, z3, t;
  fp2_sqr(&z2, &x.z);
  fp2_mul(&z3, &z2, &x.z);
  fp2_mul(&t, &ps.x, &z2);
  if (!fp2_eq(&t, &x.x)) return 0;
  fp2_mul(&t, &ps.y, &z3);
  return fp2_eq(&t, &x.y);
}

/* returns 0 ok, nonzero invalid (blst POINTonE2_Uncompress_Z) */
static int g2_decompress(g2a* out, const uint8_t* in) {
  uint8_t in0 = in[0];
  if (!(in0 & 0x80)) return 1;
  if (in0 & 0x40) return 4; /* infinity (or bad encoding): invalid as a signature either way */
  uint8_t b[48];
  memcpy(b, in, 48);
  b[0] &= 0x1f;
  uint64_t r1[6], r0[6];
  be48_to_raw(r1, b);
  be48_to_raw(r0, in + 48);
  if (!raw_lt_p(r1) || !raw_lt_p(r0)) return 1;
  fp2 x, y, y2, t;
  fp_from_raw(&x.c0, r0);
  fp_from_raw(&x.c1, r1);
  fp2_sqr(&t, &x); fp2_mul(&t, &t, &x); fp2_add(&y2, &t, &B2M);
  if (!fp2_sqrt(&y, &y2)) return 2;
  if (fp2_lexi_large(&y) != !!(in0 & 0x20)) fp2_neg(&y, &y);
  if (fp2_is_zero(&x)) return 3;
  out->x = x;
  out->y = y;
  return 0;
}

void port_init(void);

int port_g1_decompress(const uint8_t* in, uint8_t* out96) {
  port_init();
  uint8_t in0 = in[0];
  if (!(in0 & 0x80) || (in0 & 0x40)) return 1;
  uint8_t b[48];
  memcpy(b, in, 48);
  b[0] &= 0x1f;
  uint64_t r[6];
  be48_to_raw(r, b);
  if (!raw_lt_p(r)) return 1;
  fp x, y, y2, t;
  fp_from_raw(&x, r);
  fp_sqr(&t, &x); fp_mul(&t, &t, &x); fp_add(&y2, &t, &B1M);
  fp_pow(&y, &y2, E_SQRT);
  fp_sqr(&t, &y);
  if (!fp_eq(&t, &y2)) return 2;
  if (fp_lexi_large(&y) != !!(in0 & 0x20)) fp_neg(&y, &y);
  uint64_t v[6];
  fp_to_raw(v, &x); raw_to_be48(out96, v);
  fp_to_raw(v, &y); raw_to_be48(out96 + 48, v);
  return 0;
}

/* ---------------- hash to G2 ---------------- */
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5, 0xd807aa98, 0x12835b01,
    0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc,
    0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147,
    0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116, 0x1e376c08,
    0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3, 0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208,
    0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

static void sha256(uint8_t out[32], const uint8_t* msg, size_t len) {
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  size_t total = ((len + 9 + 63) / 64) * 64;
  uint8_t buf[256];
  memset(buf, 0, total);
  memcpy(buf, msg, len);
  buf[len] = 0x80;
  uint64_t bits = (uint64_t)len * 8;
  for (int i = 0; i < 8; ++i) buf[total - 1 - i] = (uint8_t)(bits >> (8 * i));
  for (size_t o = 0; o < total; o += 64) {
    uint32_t w[64];
    for (int i = 0; i < 16; ++i)
      w[i] = ((uint32_t)buf[o + 4 * i] << 24) | ((uint32_t)buf[o + 4 * i + 1] << 16) | ((uint32_t)buf[o + 4 * i + 2] << 8) | buf[o + 4 * i + 3];
    for (int i = 16; i < 64; ++i) {
      uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
      uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
      w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; ++i) {
      uint32_t t1 = hh + (ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
      uint32_t t2 = (ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
      hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
  }
  for (int i = 0; i < 8; ++i) {
    out[4 * i] = h[i] >> 24; out[4 * i + 1] = h[i] >> 16; out[4 * i + 2] = h[i] >> 8; out[4 * i + 3] = h[i];
  }
}

static const char DST[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_";

static void expand_xmd(uint8_t out[256], const uint8_t msg[32]) {
  uint8_t buf[200], b0[32], bi[32];
  size_t dl = 43;
  memset(buf, 0, 64);
  memcpy(buf + 64, msg, 32);
  buf[96] = 1; buf[97] = 0; buf[98] = 0;
  memcpy(buf + 99, DST, dl); buf[99 + dl] = (uint8_t)dl;
  sha256(b0, buf, 100 + dl);
  memset(bi, 0, 32);
  for (int i = 1; i <= 8; ++i) {
    for (int k = 0; k < 32; ++k) buf[k] = b0[k] ^ bi[k];
    buf[32] = (uint8_t)i;
    memcpy(buf + 33, DST, dl); buf[33 + dl] = (uint8_t)dl;
    sha256(bi, buf, 34 + dl);
    memcpy(out + 32 * (i - 1), bi, 32);
  }
}

static void fp_from_be64(fp* r, const uint8_t* b) {
  uint64_t hi[6] = {0}, lo[6] = {0};
  for (int i = 0; i < 4; ++i) {
    uint64_t w1 = 0, w2 = 0;
    for (int k = 0; k < 8; ++k) { w1 = (w1 << 8) | b[24 - 8 * i + k]; w2 = (w2 << 8) | b[56 - 8 * i + k]; }
    hi[i] = w1; lo[i] = w2;
  }
  fp h, l, t1, t2;
  memcpy(h.l, hi, 48); memcpy(l.l, lo, 48);
  fp_mul(&t1, &h, &R2_256);
  fp_mul(&t2, &l, &R2);
  fp_add(r, &t1, &t2);
}

static void map_sswu(g2a* out, const fp2* u) {
  fp2 u2, zu2, tv1, x1, gx1, x2, gx2, y1, y2, t, one;
  one.c0 = R1; memset(&one.c1, 0, sizeof(fp));
  fp2_sqr(&u2, u); fp2_mul(&zu2, &SSWU_Z, &u2);
  fp2_sqr(&tv1, &zu2); fp2_add(&tv1, &tv1, &zu2);
  if (fp2_is_zero(&tv1)) x1 = SSWU_B_ZA;
  else { fp2_inv(&t, &tv1); fp2_add(&t, &t, &one); fp2_mul(&x1, &SSWU_NB_A, &t); }
  fp2_sqr(&t, &x1); fp2_add(&t, &t, &SSWU_A); fp2_mul(&t, &t, &x1); fp2_add(&gx1, &t, &SSWU_B);
  fp2_mul(&x2, &zu2, &x1);
  fp2_sqr(&t, &x2); fp2_add(&t, &t, &SSWU_A); fp2_mul(&t, &t, &x2); fp2_add(&gx2, &t, &SSWU_B);
  if (fp2_sqrt(&y1, &gx1)) { out->x = x1; out->y = y1; }
  else { fp2_sqrt(&y2, &gx2); out->x = x2; out->y = y2; }
  if (fp2_sgn0(u) != fp2_sgn0(&out->y)) fp2_neg(&out->y, &out->y);
}

static void poly(fp2* r, const fp2* c, int n, const fp2* x) {
  fp2 acc = c[n - 1];
  for (int i = n - 2; i >= 0; --i) { fp2_mul(&acc, &acc, x); fp2_add(&acc, &acc, &c[i]); }
  *r = acc;
}

static void iso_map(g2j* r, const g2a* p) {
  fp2 xn, xd, yn, yd, yd2, xd2, t, one;
  one.c0 = R1; memset(&one.c1, 0, sizeof(fp));
  fp2 xdc[3] = {ISO_XD[0], ISO_XD[1], one};
  fp2 ydc[4] = {ISO_YD[0], ISO_YD[1], ISO_YD[2], one};
  poly(&xn, ISO_XN, 4, &p->x); poly(&xd, xdc, 3, &p->x); poly(&yn, ISO_YN, 4, &p->x); poly(&yd, ydc, 4, &p->x);
  fp2_sqr(&yd2, &yd); fp2_sqr(&xd2, &xd);
  fp2_mul(&r->z, &xd, &yd);
  fp2_mul(&t, &xn, &xd); fp2_mul(&r->x, &t, &yd2);
  fp2_mul(&t, &p->y, &yn); fp2_mul(&xd2, &xd2, &xd); fp2_mul(&t, &t, &xd2); fp2_mul(&r->y, &t, &yd2);
}

static void g2_neg_j(g2j* r, const g2j* p) { *r = *p; fp2_neg(&r->y, &p->y); }

static void hash_to_g2(g2a* out, const uint8_t msg[32]) {
  uint8_t u[256];
  expand_xmd(u, msg);
  fp2 u0, u1;
  fp_from_be64(&u0.c0, u); fp_from_be64(&u0.c1, u + 64); fp_from_be64(&u1.c0, u + 128); fp_from_be64(&u1.c1, u + 192);
  g2a m0, m1;
  g2j q0, q1, p, t1, t2, t3, t;
  map_sswu(&m0, &u0); map_sswu(&m1, &u1);
  iso_map(&q0, &m0); iso_map(&q1, &m1);
  g2_add(&p, &q0, &q1);
  g2_mul_xabs_j(&t1, &p); g2_neg_j(&t1, &t1);
  g2_psi_j(&t2, &p);
  g2_dbl(&t3, &p); g2_psi_j(&t3, &t3); g2_psi_j(&t3, &t3);
  g2_neg_j(&t, &t2); g2_add(&t3, &t3, &t);
  g2_add(&t2, &t1, &t2);
  g2_mul_xabs_j(&t2, &t2); g2_neg_j(&t2, &t2);
  g2_add(&t3, &t3, &t2);
  g2_neg_j(&t, &t1); g2_add(&t3, &t3, &t);
  g2_neg_j(&t, &p); g2_add(&t3, &t3, &t);
  g2_to_aff(out, &t3);
}

/* ---------------- pairing ---------------- */
typedef struct { fp2 x, y, z; } g2p;

static void dbl_step(g2p* T, fp2* c0, fp2* c2, fp2* c3, const fp* nxp, const fp* yp) {
  fp2 A, B, C, E, F, X3, G, Y3, H, Z3, X2, t;
  fp2_mul(&A, &T->x, &T->y); fp2_mul_fp(&A, &A, &INV2);
  fp2_sqr(&B, &T->y); fp2_sqr(&C, &T->z);
  fp2_mul(&E, &C, &B2M3);
  fp2_dbl(&F, &E); fp2_add(&F, &F, &E);
  fp2_sub(&t, &B, &F); fp2_mul(&X3, &A, &t);
  fp2_add(&G, &B, &F); fp2_mul_fp(&G, &G, &INV2);
  fp2_sqr(&t, &E); fp2_dbl(&Y3, &t); fp2_add(&t, &Y3, &t); fp2_sqr(&Y3, &G); fp2_sub(&Y3, &Y3, &t);
  fp2_add(&t, &T->y, &T->z); fp2_sqr(&t, &t); fp2_add(&H, &B, &C); fp2_sub(&H, &t, &H);
  fp2_mul(&Z3, &B, &H);
  fp2_sqr(&X2, &T->x);
  fp2_sub(c0, &B, &E);
  fp2_dbl(&t, &X2); fp2_add(&t, &t, &X2); fp2_mul_fp(c2, &t, nxp);
  fp2_mul_fp(c3, &H, yp);
  T->x = X3; T->y = Y3; T->z = Z3;
}

static void add_step(g2p* T, const g2a* Q, fp2* c0, fp2* c2, fp2* c3, const fp* nxp, const fp* yp) {
  fp2 th, la, C, D, E, F, G, H, t, u;
  fp2_mul(&t, &Q->y, &T->z); fp2_sub(&th, &T->y, &t);
  fp2_mul(&t, &Q->x, &T->z); fp2_sub(&la, &T->x, &t);
  fp2_sqr(&C, &th); fp2_sqr(&D, &la); fp2_mul(&E, &D, &la);
  fp2_mul(&F, &T->z, &C); fp2_mul(&G, &T->x, &D);
  fp2_add(&H, &E, &F); fp2_dbl(&t, &G); fp2_sub(&H, &H, &t);
  fp2 X3, Y3, Z3;
  fp2_mul(&X3, &la, &H);
  fp2_sub(&t, &G, &H); fp2_mul(&t, &th, &t); fp2_mul(&u, &T->y, &E); fp2_sub(&Y3, &t, &u);
  fp2_mul(&Z3, &T->z, &E);
  fp2_mul(&t, &th, &Q->x); fp2_mul(&u, &la, &Q->y); fp2_sub(c0, &t, &u);
  fp2_mul_fp(c2, &th, nxp);
  fp2_mul_fp(c3, &la, yp);
  T->x = X3; T->y = Y3; T->z = Z3;
}

static int pairing_check_2(const g1a* P0, const g2a* Q0, const g1a* P1, const g2a* Q1) {
  fp nx0, nx1;
  fp_neg(&nx0, &P0->x); fp_neg(&nx1, &P1->x);
  g2p T0 = {Q0->x, Q0->y, {R1, {{0}}}}, T1 = {Q1->x, Q1->y, {R1, {{0}}}};
  fp12 f;
  fp12_one(&f);
  fp2 c0, c2, c3;
  for (int i = 62; i >= 0; --i) {
    if (i != 62) fp12_sqr(&f, &f);
    dbl_step(&T0, &c0, &c2, &c3, &nx0, &P0->y); fp12_mul_line(&f, &c0, &c2, &c3);
    dbl_step(&T1, &c0, &c2, &c3, &nx1, &P1->y); fp12_mul_line(&f, &c0, &c2, &c3);
    if ((X_ABS >> i) & 1) {
      add_step(&T0, Q0, &c0, &c2, &c3, &nx0, &P0->y); fp12_mul_line(&f, &c0, &c2, &c3);
      add_step(&T1, Q1, &c0, &c2, &c3, &nx1, &P1->y); fp12_mul_line(&f, &c0, &c2, &c3);
    }
  }
  fp12_conj(&f, &f);
  fp12 e;
  final_exp(&e, &f);
  return fp12_is_one(&e);
}

/* ---------------- constants ---------------- */
static void raw_from_hex(uint64_t v[6], const char* h) {
  memset(v, 0, 48);
  size_t n = strlen(h);
  for (size_t i = 0; i < n; ++i) {
    char c = h[n - 1 - i];
    uint64_t d = (c >= '0' && c <= '9') ? (uint64_t)(c - '0') : (uint64_t)((c | 32) - 'a' + 10);
    v[i / 16] |= d << (4 * (i % 16));
  }
}
static void fp_hex(fp* r, const char* h) { uint64_t v[6]; raw_from_hex(v, h); fp_from_raw(r, v); }
static void fp_small(fp* r, uint64_t s, int neg) {
  uint64_t v[6] = {s, 0, 0, 0, 0, 0};
  fp_from_raw(r, v);
  if (neg) fp_neg(r, r);
}

static int g_init = 0;

static void fp2_pow_raw(fp2* r, const fp2* a, const uint64_t* e, int words) {
  fp2 acc;
  acc.c0 = R1; memset(&acc.c1, 0, sizeof(fp));
  for (int i = 64 * words - 1; i >= 0; --i) {
    fp2_sqr(&acc, &acc);
    if ((e[i >> 6] >> (i & 63)) & 1) fp2_mul(&acc, &acc, a);
  }
  *r = acc;
}

/* (p - k) / d as 6 words */
static void p_minus_div(uint64_t out[6], uint64_t k, uint64_t d, int plus) {
  u128 rem = 0;
  uint64_t t[6];
  /* t = p -/+ k */
  uint64_t c = k;
  for (int i = 0; i < 6; ++i) {
    if (plus) { u128 s = (u128)P.l[i] + c; t[i] = (uint64_t)s; c = (uint64_t)(s >> 64); }
    else { u128 s = (u128)P.l[i] - c; t[i] = (uint64_t)s; c = (uint64_t)(s >> 127); }
  }
  for (int i = 5; i >= 0; --i) {
    u128 cur = (rem << 64) | t[i];
    out[i] = (uint64_t)(cur / d);
    rem = cur % d;
  }
}

void port_init(void) {
  if (g_init) return;
  /* R^2 mod p by doubling R (R = 2^384 mod p) */
  fp one_raw = {{1, 0, 0, 0, 0, 0}};
  /* compute R1 = 2^384 mod p by repeated doubling of 1 (384 times) in raw space */
  fp x = one_raw;
  for (int i = 0; i < 384; ++i) fp_add(&x, &x, &x);
  R1 = x;
  for (int i = 0; i < 384; ++i) fp_add(&x, &x, &x);
  R2 = x; /* 2^768 mod p */
  fp y = R2;
  for (int i = 0; i < 256; ++i) fp_add(&y, &y, &y);
  R2_256 = y;
  p_minus_div(E_SQRT, 1, 4, 1);
  p_minus_div(E_SQRTM3, 3, 4, 0);
  p_minus_div(E_INV, 2, 1, 0);
  fp_small(&INV2, 2, 0); fp_inv(&INV2, &INV2);
  fp_small(&B1M, 4, 0);
  fp_small(&B2M.c0, 4, 0); B2M.c1 = B2M.c0;
  fp_small(&B2M3.c0, 12, 0); B2M3.c1 = B2M3.c0;
  fp_hex(&G1X_M, "17f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb");
  fp_hex(&NEG_G1Y, "08b3f481e3aaa0f1a09e30ed741d8ae4fcf5e095d5d00af600db18cb2c04b3edd03cc744a2888ae40caa232946c5e7e1");
  fp_neg(&NEG_G1Y, &NEG_G1Y);
  fp2 xi;
  fp_small(&xi.c0, 1, 0); xi.c1 = xi.c0;
  uint64_t e3[6], e6[6], e2[6], e23[6];
  p_minus_div(e3, 1, 3, 0);
  p_minus_div(e6, 1, 6, 0);
  p_minus_div(e2, 1, 2, 0);
  /* 2(p-1)/3 */
  { uint64_t c = 0; for (int i = 0; i < 6; ++i) { u128 s = (u128)e3[i] * 2 + c; e23[i] = (uint64_t)s; c = (uint64_t)(s >> 64); } }
  fp2_pow_raw(&FROB_V1, &xi, e3, 6);
  fp2_pow_raw(&FROB_V2, &xi, e23, 6);
  fp2_pow_raw(&FROB_W, &xi, e6, 6);
  fp2_mul(&FROB_V1W, &FROB_V1, &FROB_W);
  fp2_mul(&FROB_V2W, &FROB_V2, &FROB_W);
  fp2_inv(&PSI_X, &FROB_V1);
  fp2 t;
  fp2_pow_raw(&t, &xi, e2, 6);
  fp2_inv(&PSI_Y, &t);
  memset(&SSWU_A, 0, sizeof SSWU_A); fp_small(&SSWU_A.c1, 240, 0);
  fp_small(&SSWU_B.c0, 1012, 0); SSWU_B.c1 = SSWU_B.c0;
  fp_small(&SSWU_Z.c0, 2, 1); fp_small(&SSWU_Z.c1, 1, 1);
  fp2 ia, nb;
  fp2_inv(&ia, &SSWU_A); fp2_neg(&nb, &SSWU_B); fp2_mul(&SSWU_NB_A, &nb, &ia);
  fp2_mul(&t, &SSWU_Z, &SSWU_A); fp2_inv(&t, &t); fp2_mul(&SSWU_B_ZA, &SSWU_B, &t);
  const char* k10 = "5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97d6";
  const char* k11 = "11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71a";
  const char* k12a = "11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71e";
  const char* k12b = "8ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38d";
  const char* k13 = "171d6541fa38ccfaed6dea691f5fb614cb14b4e7f4e810aa22d6108f142b85757098e38d0f671c7188e2aaaaaaaa5ed1";
  fp_hex(&ISO_XN[0].c0, k10); ISO_XN[0].c1 = ISO_XN[0].c0;
  memset(&ISO_XN[1].c0, 0, sizeof(fp)); fp_hex(&ISO_XN[1].c1, k11);
  fp_hex(&ISO_XN[2].c0, k12a); fp_hex(&ISO_XN[2].c1, k12b);
  fp_hex(&ISO_XN[3].c0, k13); memset(&ISO_XN[3].c1, 0, sizeof(fp));
  memset(&ISO_XD[0].c0, 0, sizeof(fp)); fp_small(&ISO_XD[0].c1, 72, 1);
  fp_small(&ISO_XD[1].c0, 12, 0); fp_small(&ISO_XD[1].c1, 12, 1);
  const char* y0 = "1530477c7ab4113b59a4c18b076d11930f7da5d4a07f649bf54439d87d27e500fc8c25ebf8c92f6812cfc71c71c6d706";
  const char* y1 = "5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97be";
  const char* y2a = "11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71c";
  const char* y2b = "8ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38f";
  const char* y3 = "124c9ad43b6cf79bfbf7043de3811ad0761b0f37a1e26286b0e977c69aa274524e79097a56dc4bd9e1b371c71c718b10";
  fp_hex(&ISO_YN[0].c0, y0); ISO_YN[0].c1 = ISO_YN[0].c0;
  memset(&ISO_YN[1].c0, 0, sizeof(fp)); fp_hex(&ISO_YN[1].c1, y1);
  fp_hex(&ISO_YN[2].c0, y2a); fp_hex(&ISO_YN[2].c1, y2b);
  fp_hex(&ISO_YN[3].c0, y3); memset(&ISO_YN[3].c1, 0, sizeof(fp));
  fp_small(&ISO_YD[0].c0, 432, 1); fp_small(&ISO_YD[0].c1, 432, 1);
  memset(&ISO_YD[1].c0, 0, sizeof(fp)); fp_small(&ISO_YD[1].c1, 216, 1);
  fp_small(&ISO_YD[2].c0, 18, 0); fp_small(&ISO_YD[2].c1, 18, 1);
  g_init = 1;
}

/* ---------------- the verification path ---------------- */
static uint64_t splitmix(uint64_t* s) {
  uint64_t z = (*s += 0x9e3779b97f4a7c15ULL);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

static int load_g1_aff96(g1a* p, const uint8_t* b) {
  uint64_t v[6];
  be48_to_raw(v, b); fp_from_raw(&p->x, v);
  be48_to_raw(v, b + 48); fp_from_raw(&p->y, v);
  return 0;
}

/* verify(msg, pk, sig): per-set check used by the retry path */
static int verify_one(const g1a* pk, const g2a* h, const uint8_t* sig96) {
  g2a s;
  if (g2_decompress(&s, sig96)) return 0;
  if (!g2_in_subgroup(&s)) return 0;
  g1a ng = {G1X_M, NEG_G1Y};
  return pairing_check_2(pk, h, &ng, &s);
}

/* One same-message chunk (jobItemWorkReq sameMessage + worker verify + retry). */
static void chunk_same_message(const uint8_t* pk_aff, const uint8_t* sigs, size_t n, const uint8_t* msg, uint8_t* valid,
                               uint64_t* rng) {
  g2a h;
  hash_to_g2(&h, msg);
  g1j accp;
  g2j accs;
  memset(&accp, 0, sizeof accp);
  memset(&accs, 0, sizeof accs);
  int ok = n > 0;
  for (size_t i = 0; i < n && ok; ++i) {
    g2a s;
    if (g2_decompress(&s, sigs + 96 * i) || !g2_in_subgroup(&s)) { ok = 0; break; }
    g1a p;
    load_g1_aff96(&p, pk_aff + 96 * i);
    uint64_t r = 0;
    while (!r) r = splitmix(rng);
    g1j rp;
    g2j rs;
    g1_mul_u64(&rp, &p, r);
    g2_mul_u64(&rs, &s, r);
    g1_add(&accp, &accp, &rp);
    g2_add(&accs, &accs, &rs);
  }
  if (ok) {
    g1a pa;
    g2a sa;
    g1a ng = {G1X_M, NEG_G1Y};
    if (g1_to_aff(&pa, &accp) && g2_to_aff(&sa, &accs) && g2_in_subgroup(&sa))
      ok = pairing_check_2(&pa, &h, &ng, &sa);
    else
      ok = 0;
  }
  if (ok) {
    memset(valid, 1, n);
    return;
  }
  for (size_t i = 0; i < n; ++i) {
    g1a p;
    load_g1_aff96(&p, pk_aff + 96 * i);
    valid[i] = (uint8_t)verify_one(&p, &h, sigs + 96 * i);
  }
}

typedef struct {
  const uint32_t* chunk_off;
  const uint32_t* chunk_msg;
  size_t n_chunks;
  const uint8_t* pk_aff;
  const uint8_t* sigs;
  const uint8_t* msgs;
  uint8_t* valid;
  atomic_size_t next;
  uint64_t seed;
} job_t;

static void* worker(void* arg) {
  job_t* j = (job_t*)arg;
  uint64_t rng = j->seed ^ (uint64_t)(uintptr_t)&rng;
  for (;;) {
    size_t c = atomic_fetch_add(&j->next, 1);
    if (c >= j->n_chunks) break;
    uint32_t a = j->chunk_off[c], b = j->chunk_off[c + 1];
    chunk_same_message(j->pk_aff + 96ull * a, j->sigs + 96ull * a, b - a, j->msgs + 32ull * j->chunk_msg[c], j->valid + a, &rng);
  }
  return NULL;
}

/* Many verifySignatureSetsSameMessage calls on `nthreads` worker threads (pool shape).
 * call_off: n_calls+1 offsets; pk_aff: 96-byte affine pubkey (x||y, BE canonical) per set. */
int port_verify_same_message_batch(int nthreads, size_t n_calls, const uint32_t* call_off, const uint8_t* pk_aff,
                                   const uint8_t* sigs, const uint8_t* msgs, uint8_t* valid, uint64_t seed) {
  port_init();
  size_t cap = 16;
  size_t nc = 0;
  uint32_t* off = (uint32_t*)malloc(sizeof(uint32_t) * (cap + 1));
  uint32_t* cm = (uint32_t*)malloc(sizeof(uint32_t) * cap);
  for (size_t g = 0; g < n_calls; ++g) {
    uint32_t len = call_off[g + 1] - call_off[g];
    if (!len) continue;
    uint32_t cc = len / 128, per = len;
    if (cc > 1) per = (len + cc - 1) / cc;
    for (uint32_t s = 0; s < len; s += per) {
      if (nc + 1 >= cap) {
        cap *= 2;
        off = (uint32_t*)realloc(off, sizeof(uint32_t) * (cap + 1));
        cm = (uint32_t*)realloc(cm, sizeof(uint32_t) * cap);
      }
      off[nc] = call_off[g] + s;
      cm[nc] = (uint32_t)g;
      ++nc;
    }
  }
  off[nc] = n_calls ? call_off[n_calls] : 0;
  job_t j;
  j.chunk_off = off; j.chunk_msg = cm; j.n_chunks = nc; j.pk_aff = pk_aff; j.sigs = sigs; j.msgs = msgs; j.valid = valid;
  atomic_init(&j.next, 0);
  j.seed = seed;
  if (nthreads < 1) nthreads = 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
  for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, worker, &j);
  for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  free(th);
  free(off);
  free(cm);
  return 0;
}

/* single verify, for tests: pk48 compressed, msg32, sig96 */
int port_verify(const uint8_t* pk48, const uint8_t* msg32, const uint8_t* sig96) {
  port_init();
  uint8_t aff[96];
  if (port_g1_decompress(pk48, aff)) return 0;
  g1a p;
  load_g1_aff96(&p, aff);
  g2a h;
  hash_to_g2(&h, msg32);
  return verify_one(&p, &h, sig96);
}

/* hash_to_G2 (uncompressed 192-byte output: x.c1 x.c0 y.c1 y.c0) */
void port_hash_to_g2(const uint8_t* msg32, uint8_t* out192) {
  port_init();
  g2a h;
  hash_to_g2(&h, msg32);
  uint64_t v[6];
  fp_to_raw(v, &h.x.c1); raw_to_be48(out192, v);
  fp_to_raw(v, &h.x.c0); raw_to_be48(out192 + 48, v);
  fp_to_raw(v, &h.y.c1); raw_to_be48(out192 + 96, v);
  fp_to_raw(v, &h.y.c0); raw_to_be48(out192 + 144, v);
}

/* ---------------- verifySignatureSets (distinct messages, aggregate pubkeys) ----------------
 * BlsMultiThreadWorkerPool.verifySignatureSets (multithread/index.ts:157-207): every call is split
 * with chunkifyMaximizeChunkSize(128) into jobs; a job's sets get their aggregate pubkey
 * (aggregatePublicKeys, jobItem.ts:55-62), and the worker verifies the job as ONE randomised batch
 * (verifyMultipleAggregateSignatures, maybeBatch.ts:17-26): per set decompress + subgroup check,
 * 64-bit random r, hash_to_G2; then prod e(r_i pk_i, H(m_i)) * e(-g1, sum r_i sig_i) with a
 * multi-Miller loop sharing its Fp12 squarings, and one final exponentiation.  A call is the AND
 * over its jobs.  Workers pull jobs, as the pool's workers do. */
typedef struct {
  g2p T;
  g2a Q;
  fp nx, y;
} mpair;

static int multi_pairing_is_one(mpair* pr, size_t n) {
  fp12 f;
  fp12_one(&f);
  fp2 c0, c2, c3;
  for (int i = 62; i >= 0; --i) {
    if (i != 62) fp12_sqr(&f, &f);
    for (size_t j = 0; j < n; ++j) { dbl_step(&pr[j].T, &c0, &c2, &c3, &pr[j].nx, &pr[j].y); fp12_mul_line(&f, &c0, &c2, &c3); }
    if ((X_ABS >> i) & 1)
      for (size_t j = 0; j < n; ++j) { add_step(&pr[j].T, &pr[j].Q, &c0, &c2, &c3, &pr[j].nx, &pr[j].y); fp12_mul_line(&f, &c0, &c2, &c3); }
  }
  fp12_conj(&f, &f);
  fp12 e;
  final_exp(&e, &f);
  return fp12_is_one(&e);
}

/* one job: sets [a, b) -> 1 valid / 0 invalid */
static int vs_job(size_t a, size_t b, const uint32_t* pk_off, const uint32_t* pk_idx, const uint8_t* pk_aff, const uint8_t* msgs,
                  const uint8_t* sigs, uint64_t* rng) {
  size_t n = b - a;
  if (n == 0) return 0; /* verifySignatureSetsMaybeBatch([]) -> false */
  mpair* pr = (mpair*)malloc(sizeof(mpair) * (n + 1));
  g2j acc;
  memset(&acc, 0, sizeof acc);
  int ok = 1;
  for (size_t s = a; s < b && ok; ++s) {
    g1j agg;
    memset(&agg, 0, sizeof agg);
    for (uint32_t k = pk_off[s]; k < pk_off[s + 1]; ++k) {
      g1a p;
      load_g1_aff96(&p, pk_aff + 96ull * pk_idx[k]);
      g1_add_aff(&agg, &agg, &p);
    }
    g1a pk;
    g2a sg;
    if (!g1_to_aff(&pk, &agg) || g2_decompress(&sg, sigs + 96 * s) || !g2_in_subgroup(&sg)) { ok = 0; break; }
    uint64_t r = 0;
    while (!r) r = splitmix(rng);
    g1j rp;
    g2j rs;
    g1_mul_u64(&rp, &pk, r);
    g2_mul_u64(&rs, &sg, r);
    g2_add(&acc, &acc, &rs);
    g1a rpa;
    g1_to_aff(&rpa, &rp);
    mpair* m = &pr[s - a];
    hash_to_g2(&m->Q, msgs + 32 * s);
    m->T.x = m->Q.x; m->T.y = m->Q.y; m->T.z.c0 = R1; memset(&m->T.z.c1, 0, sizeof(fp));
    fp_neg(&m->nx, &rpa.x);
    m->y = rpa.y;
  }
  if (ok) {
    g2a sa;
    if (!g2_to_aff(&sa, &acc)) ok = 0;
    else {
      mpair* m = &pr[n];
      m->Q = sa;
      m->T.x = sa.x; m->T.y = sa.y; m->T.z.c0 = R1; memset(&m->T.z.c1, 0, sizeof(fp));
      fp_neg(&m->nx, &G1X_M);
      m->y = NEG_G1Y;
      ok = multi_pairing_is_one(pr, n + 1);
    }
  }
  free(pr);
  return ok;
}

typedef struct {
  const uint32_t* job_be; /* (begin, end) set range per job */
  const uint32_t *pk_off, *pk_idx;
  size_t n_jobs;
  const uint8_t *pk_aff, *msgs, *sigs;
  uint8_t* job_ok;
  atomic_size_t next;
  uint64_t seed;
} vsjob_t;

static void* vs_worker(void* arg) {
  vsjob_t* j = (vsjob_t*)arg;
  uint64_t rng = j->seed ^ (uint64_t)(uintptr_t)&rng;
  for (;;) {
    size_t c = atomic_fetch_add(&j->next, 1);
    if (c >= j->n_jobs) break;
    j->job_ok[c] = (uint8_t)vs_job(j->job_be[2 * c], j->job_be[2 * c + 1], j->pk_off, j->pk_idx, j->pk_aff, j->msgs, j->sigs, &rng);
  }
  return NULL;
}

/* n_calls verifySignatureSets calls on `nthreads` workers.  call_off: n_calls+1 set offsets; set s
 * aggregates the 96-byte affine pubkeys pk_aff[pk_idx[pk_off[s] .. pk_off[s+1])]; msgs 32 B and
 * sigs 96 B per set.  out[c] = AND over the call's <=128-set jobs (0 for an empty call). */
int port_verify_sets_batch(int nthreads, size_t n_calls, const uint32_t* call_off, const uint32_t* pk_off, const uint32_t* pk_idx,
                           const uint8_t* pk_aff, const uint8_t* msgs, const uint8_t* sigs, uint8_t* out, uint64_t seed) {
  port_init();
  size_t cap = 16, nj = 0;
  uint32_t* be = (uint32_t*)malloc(sizeof(uint32_t) * 2 * cap);
  uint32_t* jc = (uint32_t*)malloc(sizeof(uint32_t) * cap);
  for (size_t g = 0; g < n_calls; ++g) {
    uint32_t len = call_off[g + 1] - call_off[g];
    if (!len) continue;
    uint32_t cc = len / 128, per = len; /* chunkifyMaximizeChunkSize(call, 128) */
    if (cc > 1) per = (len + cc - 1) / cc;
    for (uint32_t s = 0; s < len; s += per) {
      if (nj == cap) {
        cap *= 2;
        be = (uint32_t*)realloc(be, sizeof(uint32_t) * 2 * cap);
        jc = (uint32_t*)realloc(jc, sizeof(uint32_t) * cap);
      }
      be[2 * nj] = call_off[g] + s;
      be[2 * nj + 1] = call_off[g] + (s + per < len ? s + per : len);
      jc[nj] = (uint32_t)g;
      ++nj;
    }
  }
  uint8_t* job_ok = (uint8_t*)malloc(nj + 1);
  vsjob_t j;
  memset(&j, 0, sizeof j);
  j.job_be = be; j.pk_off = pk_off; j.pk_idx = pk_idx; j.pk_aff = pk_aff; j.msgs = msgs; j.sigs = sigs;
  j.n_jobs = nj; j.job_ok = job_ok; j.seed = seed;
  atomic_init(&j.next, 0);
  if (nthreads < 1) nthreads = 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
  for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, vs_worker, &j);
  for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  for (size_t g = 0; g < n_calls; ++g) out[g] = call_off[g + 1] > call_off[g] ? 1 : 0;
  for (size_t k = 0; k < nj; ++k) out[jc[k]] &= job_ok[k];
  free(th);
  free(job_ok);
  free(be);
  free(jc);
  return 0;
}
