// Host build of the device arithmetic library (lodestar_amd/csrc/*.h) for CPU unit tests.
// This is NOT a product code path: it exists so the field/curve/pairing code can be checked
// against the Python oracle without a GPU.  Built by tests/native/build_hosttest.sh.
#define GBV_HOST_TEST 1
#include "../../lodestar_amd/csrc/pairing.h"
#include "../../lodestar_amd/csrc/hash_to_curve.h"
#include "../../lodestar_amd/csrc/coop.h"
#include "../../lodestar_amd/csrc/ssz.h"
#include "locate_proto.h"
#include <vector>

using namespace gbv;

static Fp load_mont(const uint8_t* be48) { return fp_to_mont(fp_load_be48(be48, false)); }
static void store_canon(uint8_t* be48, const Fp& a) { fp_store_be48(be48, fp_from_mont(a)); }
static void store_fp2(uint8_t* out, const Fp2& a) { store_canon(out, a.c0); store_canon(out + 48, a.c1); }
static Fp2 load_fp2(const uint8_t* in) { return Fp2{load_mont(in), load_mont(in + 48)}; }

extern "C" {
void ht_fp_mul(uint8_t* out, const uint8_t* a, const uint8_t* b) { store_canon(out, fp_mul(load_mont(a), load_mont(b))); }
// Lazy product inputs (fp.h fp_add_lazy / fp_sub_lazy4): raw 384-bit Montgomery-form operands, which
// may be >= p; op 0: (a + b) * c, op 1: (a + 4p - b) * c, op 2: a * b.  Output raw (must be < p).
void ht_fp_lazy(uint8_t* out, const uint8_t* a, const uint8_t* b, const uint8_t* c, int op) {
  const Fp x = fp_load_be48(a, false), y = fp_load_be48(b, false), z = fp_load_be48(c, false);
  Fp r = op == 0 ? fp_mul(fp_add_lazy(x, y), z) : op == 1 ? fp_mul(fp_sub_lazy4(x, y), z) : fp_mul(x, y);
  fp_store_be48(out, r);
}
void ht_fp_inv(uint8_t* out, const uint8_t* a) { store_canon(out, fp_inv(load_mont(a))); }
int ht_fp2_sqrt(uint8_t* out, const uint8_t* a) {
  Fp2 r;
  bool ok = fp2_sqrt(r, load_fp2(a));
  store_fp2(out, r);
  return ok;
}
void ht_fp2_mul(uint8_t* out, const uint8_t* a, const uint8_t* b) { store_fp2(out, fp2_mul(load_fp2(a), load_fp2(b))); }
// out: x.c0 x.c1 y.c0 y.c1 (canonical BE)
void ht_hash_to_g2(uint8_t* out, const uint8_t* msg32) {
  uint32_t w[8];
  for (int i = 0; i < 8; ++i) w[i] = ((uint32_t)msg32[4*i] << 24) | ((uint32_t)msg32[4*i+1] << 16) | ((uint32_t)msg32[4*i+2] << 8) | msg32[4*i+3];
  G2A q = hash_to_g2(w);
  store_fp2(out, q.x);
  store_fp2(out + 96, q.y);
}
void ht_expand(uint8_t* out256, const uint8_t* msg32) {
  uint32_t w[8], o[64];
  for (int i = 0; i < 8; ++i) w[i] = ((uint32_t)msg32[4*i] << 24) | ((uint32_t)msg32[4*i+1] << 16) | ((uint32_t)msg32[4*i+2] << 8) | msg32[4*i+3];
  expand_message_xmd_32(o, w);
  for (int i = 0; i < 64; ++i) { out256[4*i] = o[i] >> 24; out256[4*i+1] = o[i] >> 16; out256[4*i+2] = o[i] >> 8; out256[4*i+3] = o[i]; }
}
int ht_g2_decode(uint8_t* out, const uint8_t* in, uint32_t len) {
  G2A a;
  uint8_t st = g2_decode(a, in, len);
  if (st == PT_OK) { store_fp2(out, a.x); store_fp2(out + 96, a.y); }
  return st;
}
int ht_g2_in_subgroup(const uint8_t* xy) {
  G2A a{load_fp2(xy), load_fp2(xy + 96)};
  return g2_in_subgroup(a);
}
// The lazy G2 chain (g2_lazy.h) against the canonical one: [|x|] Q both ways, coordinates compared
// exactly (the same formulas mod p).  Returns 1 when equal; *max_col_bits: widest product column seen.
int ht_g2_mul_xabs_lazy_cmp(const uint8_t* xy, long long* max_col_bits) {
  G2A a{load_fp2(xy), load_fp2(xy + 96)};
  g_s28_max_col_bits = 0;
  const G2J lazy = g2_mul_xabs_lazy(a);
  const G2J ref = jac_mul_xabs(a);
  *max_col_bits = g_s28_max_col_bits;
  return fp2_eq(lazy.x, ref.x) && fp2_eq(lazy.y, ref.y) && fp2_eq(lazy.z, ref.z);
}
// One lazy doubling from adversarial limbs: x, y, z with low limbs drawn from {-8, 2^28 + 7, random in
// range} (mode bits select the extremes) and top limbs up to +-31 p's top limb (values below 32 p),
// checked against jac_dbl of their canonical values.  The host build aborts on any bound violation.
int ht_s2j_dbl_extreme(uint64_t seed, int mode, long long* max_col_bits) {
  uint64_t st = seed * 0x9E3779B97F4A7C15ull + 1;
  auto rnd = [&]() { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; };
  auto limb_of = [&](int i) -> int32_t {
    const int m = (mode >> (i % 3)) & 3;
    if (m == 1) return 268435456 + 7;
    if (m == 2) return -8;
    return (int32_t)(rnd() % (268435456ull + 16)) - 8;
  };
  S2J p;
  S28* f[6] = {&p.x.c0, &p.x.c1, &p.y.c0, &p.y.c1, &p.z.c0, &p.z.c1};
  for (int k = 0; k < 6; ++k) {
    for (int i = 0; i < 13; ++i) f[k]->v[i] = limb_of(i + k);
    const int32_t top = (int32_t)(rnd() % (2u * 60u * P28[13])) - (int32_t)(60u * P28[13]);
    f[k]->v[13] = top;
  }
  g_s28_max_col_bits = 0;
  S2J r = p;
  G2J want;
  if (mode & 64) {  // the mixed addition of q = 2^k G (canonical, affine) instead of the doubling
    uint32_t w[8] = {(uint32_t)seed, (uint32_t)mode, 1, 2, 3, 4, 5, 6};
    const G2A q = hash_to_g2(w);
    const S2 qs[2] = {s2_from(q.x), s2_from(q.y)};
    s2j_madd(&r, qs);
    want = jac_add_aff(s2j_to(p), q);
  } else {
    r = s2j_dbl(p);
    want = jac_dbl(s2j_to(p));
  }
  *max_col_bits = g_s28_max_col_bits;
  const G2J got = s2j_to(r);
  // the outputs stay normalized (limbs 0..12 in [-8, 2^28 + 8)) for the next doubling
  const S28* g[6] = {&r.x.c0, &r.x.c1, &r.y.c0, &r.y.c1, &r.z.c0, &r.z.c1};
  bool norm = true;
  for (int k = 0; k < 6; ++k)
    for (int i = 0; i < 13; ++i) norm = norm && g[k]->v[i] >= -8 && g[k]->v[i] < 268435456 + 8;
  return norm && fp2_eq(got.x, want.x) && fp2_eq(got.y, want.y) && fp2_eq(got.z, want.z);
}
// The lazy mixed addition at its exceptional inputs *r = q and *r = -q (Jacobian, scaled by a random
// lambda): the formula leaves Z = 0 mod p (which g2_mul_xabs_lazy turns into a canonical recomputation),
// and a doubling of such a point keeps Z = 0 mod p.  Returns 1 when both hold for both inputs.
int ht_s2j_madd_exceptional(uint64_t seed) {
  uint32_t w[8] = {(uint32_t)seed, 7, 7, 7, 7, 7, 7, 7};
  const G2A q = hash_to_g2(w);
  const S2 qs[2] = {s2_from(q.x), s2_from(q.y)};
  Fp2 lam{fp_to_mont(Fp{{(uint32_t)seed | 1u, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 1}}), FP_ONE};
  int ok = 1;
  for (int neg = 0; neg < 2; ++neg) {
    const Fp2 l2 = fp2_sqr(lam);
    G2J p{fp2_mul(q.x, l2), fp2_mul(neg ? fp2_neg(q.y) : q.y, fp2_mul(l2, lam)), lam};
    S2J s = s2j_from(p);
    s2j_madd(&s, qs);
    ok &= fp2_is_zero(s2j_to(s).z);
    s2j_dbl_n(&s, 3);
    ok &= fp2_is_zero(s2j_to(s).z);
  }
  return ok;
}
int ht_g1_decompress(uint8_t* out, const uint8_t* in) {
  G1A a;
  uint8_t st = g1_decompress(a, in);
  if (st == PT_OK) { store_canon(out, a.x); store_canon(out + 48, a.y); }
  return st;
}
int ht_g1_in_subgroup(const uint8_t* xy) {
  G1A a{load_mont(xy), load_mont(xy + 48)};
  return g1_in_subgroup(a);
}
// scalar mult by u64 for G2 (affine in/out)
int ht_g2_mul_u64(uint8_t* out, const uint8_t* xy, uint64_t k) {
  G2A a{load_fp2(xy), load_fp2(xy + 96)};
  G2A r;
  bool ok = jac_to_aff(r, jac_mul_u64(a, k));
  store_fp2(out, r.x); store_fp2(out + 96, r.y);
  return ok;
}
int ht_g1_mul_u64(uint8_t* out, const uint8_t* xy, uint64_t k) {
  G1A a{load_mont(xy), load_mont(xy + 48)};
  G1A r;
  bool ok = jac_to_aff(r, jac_mul_u64(a, k));
  store_canon(out, r.x); store_canon(out + 48, r.y);
  return ok;
}
// Miller loop (1 pair) + final exponentiation, Fp12 out as 12 canonical Fp in tower order
void ht_pairing(uint8_t* out, const uint8_t* p96, const uint8_t* q192) {
  G1A P{load_mont(p96), load_mont(p96 + 48)};
  G2A Q{load_fp2(q192), load_fp2(q192 + 96)};
  Fp12 f = final_exponentiation(miller_loop_1(P, Q));
  const Fp2* c[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
  for (int i = 0; i < 6; ++i) store_fp2(out + 96 * i, *c[i]);
}
// verify(pk48, msg32, sig) following the blst accept/reject rules
int ht_verify(const uint8_t* pk48, const uint8_t* msg32, const uint8_t* sig, uint32_t sig_len) {
  G1A pk;
  if (g1_decompress(pk, pk48) != PT_OK) return 0;
  G2A s;
  if (g2_decode(s, sig, sig_len) != PT_OK) return 0;
  if (!g2_in_subgroup(s)) return 0;
  uint32_t w[8];
  for (int i = 0; i < 8; ++i) w[i] = ((uint32_t)msg32[4*i] << 24) | ((uint32_t)msg32[4*i+1] << 16) | ((uint32_t)msg32[4*i+2] << 8) | msg32[4*i+3];
  G2A h = hash_to_g2(w);
  return pairing_check_2(pk, false, h, g1_neg_generator(), false, s);
}
// Wave-cooperative drivers (coop.h) run lane by lane: Miller loop over 1 or 2 pairs, then the
// final exponentiation; out = the FE value (12 canonical Fp, tower order); returns is_one.
int ht_coop_pairing(uint8_t* out, const uint8_t* p96, const uint8_t* q192, int npairs) {
  coop::load_consts();
  std::vector<coop::Slot> mem(coop::MILLER_WS + coop::FINAL_EXP_WS);
  for (int j = 0; j < npairs; ++j) {
    G1A P{load_mont(p96 + 96 * j), load_mont(p96 + 96 * j + 48)};
    G2A Q{load_fp2(q192 + 192 * j), load_fp2(q192 + 192 * j + 96)};
    coop::miller_load_pair(mem.data(), j, P, Q);
  }
  coop::miller_loop(mem.data(), npairs);
  coop::Slot* fe = mem.data() + coop::MILLER_WS;
  coop::copy(fe + coop::E_F, mem.data() + coop::M_F, 12);
  int ok = coop::final_exp_is_one(fe) ? 1 : 0;
  for (int i = 0; i < 12; ++i) store_canon(out + 48 * i, coop::get(fe + coop::E_C + i));
  return ok;
}
// The written-out cooperative Fp12 steps (coop.h) on one workspace, lanes in sequence: out = 4 Fp12
// (12 canonical BE Fp each, slot order): mul12(f, g), cyc_sqr(fc) (fc in the cyclotomic subgroup),
// inv12(f), mul_line(f, l) (l: c0, c2, c3 as 6 Fp)
void ht_coop_f12_ops(uint8_t* out, const uint8_t* f, const uint8_t* g, const uint8_t* fc, const uint8_t* l) {
  coop::load_consts();
  std::vector<coop::Slot> mem(coop::FINAL_EXP_WS);
  coop::Slot* w = mem.data();
  for (int i = 0; i < 12; ++i) {
    coop::put(w + coop::E_F + i, load_mont(f + 48 * i));
    coop::put(w + coop::E_TMP + i, load_mont(g + 48 * i));
    coop::put(w + coop::E_T + i, load_mont(fc + 48 * i));
  }
  for (int i = 0; i < 6; ++i) coop::put(w + coop::E_A + i, load_mont(l + 48 * i));
  coop::mul12(w, coop::E_Z, coop::E_F, coop::E_TMP, coop::E_B);
  coop::cyc_sqr(w, coop::E_Z, coop::E_T, coop::E_C);
  coop::mul_line(w, coop::E_Z, coop::E_F, coop::E_A, coop::E_TMP2);
  for (int i = 0; i < 12; ++i) {
    store_canon(out + 48 * i, coop::get(w + coop::E_B + i));
    store_canon(out + 576 + 48 * i, coop::get(w + coop::E_C + i));
    store_canon(out + 1728 + 48 * i, coop::get(w + coop::E_TMP2 + i));
  }
  coop::inv12(w);
  for (int i = 0; i < 12; ++i) store_canon(out + 1152 + 48 * i, coop::get(w + coop::E_INV + i));
}
// clear_cofactor_g2 with both [|x|] multiplications by the cooperative point steps
// (coop::mul_xabs_point on the written-out doubling; the device clears on lane quads, k_hash_clear_quad); in: affine point of E2, out: affine
void ht_coop_clear_cofactor(uint8_t* out, const uint8_t* xy) {
  coop::load_consts();
  std::vector<coop::Slot> mem(coop::MILLER_WS);
  const G2A a{load_fp2(xy), load_fp2(xy + 96)};
  const G2J p = jac_from_aff(a);
  coop::mul_xabs_point(mem.data(), a);
  const G2J t1 = jac_neg(coop::point_jac(mem.data()));
  G2J t2 = g2_psi_jac(p);
  G2J t3 = g2_psi_jac(g2_psi_jac(jac_dbl(p)));
  t3 = jac_add(t3, jac_neg(t2));
  t2 = jac_add(t1, t2);
  G2A b;
  jac_to_aff(b, t2);
  coop::mul_xabs_point(mem.data(), b);
  t2 = jac_neg(coop::point_jac(mem.data()));
  t3 = jac_add(t3, t2);
  t3 = jac_add(t3, jac_neg(t1));
  G2A o;
  jac_to_aff(o, jac_add(t3, jac_neg(p)));
  store_fp2(out, o.x);
  store_fp2(out + 96, o.y);
}
// [r] Q for the same batch scalar by the cooperative ladder (coop::mul_2d_point, as
// k_sm_prep_roles runs it); out: affine
void ht_coop_mul_2d(uint8_t* out, const uint8_t* q192, uint64_t r64) {
  coop::load_consts();
  std::vector<coop::Slot> mem(coop::MILLER_WS);
  const G2A Q{load_fp2(q192), load_fp2(q192 + 96)};
  coop::mul_2d_point(mem.data(), Q, g2_neg_psi2(Q), (uint32_t)r64, (uint32_t)(r64 >> 32));
  G2A o;
  jac_to_aff(o, coop::point_jac(mem.data()));
  store_fp2(out, o.x);
  store_fp2(out + 96, o.y);
}
// [r] P, [r] Q for the batch scalar r = a - b x^2 of the 64-bit digit word r64 (curve.h)
int ht_randomize(uint8_t* outp, uint8_t* outq, const uint8_t* p96, const uint8_t* q192, uint64_t r64) {
  G1A P{load_mont(p96), load_mont(p96 + 48)};
  G2A Q{load_fp2(q192), load_fp2(q192 + 96)};
  G1J rp;
  G2J rq;
  if (!randomize_pair(P, Q, r64, &rp, &rq)) return 0;
  G1A pa;
  G2A qa;
  jac_to_aff(pa, rp);
  jac_to_aff(qa, rq);
  store_canon(outp, pa.x); store_canon(outp + 48, pa.y);
  store_fp2(outq, qa.x); store_fp2(outq + 96, qa.y);
  return 1;
}
// randomize_pair_jac with P given in Jacobian coordinates scaled by z (X z^2, Y z^3, z)
int ht_randomize_jac(uint8_t* outp, uint8_t* outq, const uint8_t* p96, const uint8_t* q192, uint64_t r64, const uint8_t* z48) {
  G1A P{load_mont(p96), load_mont(p96 + 48)};
  G2A Q{load_fp2(q192), load_fp2(q192 + 96)};
  Fp z = load_mont(z48), z2 = fp_sqr(z);
  G1J PJ{fp_mul(P.x, z2), fp_mul(P.y, fp_mul(z2, z)), z};
  G1J rp;
  G2J rq;
  if (!randomize_pair_jac(PJ, Q, r64, &rp, &rq)) return 0;
  G1A pa;
  G2A qa;
  jac_to_aff(pa, rp);
  jac_to_aff(qa, rq);
  store_canon(outp, pa.x); store_canon(outp + 48, pa.y);
  store_fp2(outq, qa.x); store_fp2(outq + 96, qa.y);
  return 1;
}
// [r] P through a comb table built on the host (comb_bases + comb_entry_jac, one inversion per
// entry here; the device normalises a slot's 128 entries with one inversion) -- k_sm_prepare's
// comb path.  Also returns the Fp products of the evaluation alone (the per-set work).
int ht_comb_mul(uint8_t* outp, const uint8_t* p96, uint64_t r64, unsigned long long* fme) {
  G1A P{load_mont(p96), load_mont(p96 + 48)};
  G1A B[8], D;
  comb_bases(P, B, D);
  std::vector<uint4> tab(COMB_ENTRIES * COMB_U4);
  for (uint32_t e = 0; e < (uint32_t)COMB_ENTRIES; ++e) {
    G1J j = (e & 1u) ? jac_add_aff(comb_entry_jac(B, e & ~1u), D) : comb_entry_jac(B, e);
    G1A a;
    if (!jac_to_aff(a, j)) return 0;
    comb_entry_store(tab.data() + COMB_U4 * e, a);
  }
  g_fme_count = 0;
  G1J rp = comb_mul(tab.data(), (uint32_t)r64, (uint32_t)(r64 >> 32));
  *fme = g_fme_count;
  G1A pa;
  jac_to_aff(pa, rp);
  store_canon(outp, pa.x); store_canon(outp + 48, pa.y);
  return 1;
}
// k_comb_entries' wave normalisation replayed lane by lane (prefix / suffix products, one inversion):
// returns the number of entries that differ from per-entry normalisation (expected 0).
int ht_comb_wave_check(const uint8_t* p96) {
  G1A P{load_mont(p96), load_mont(p96 + 48)};
  G1A B[8], D;
  comb_bases(P, B, D);
  G1J J0[64], J1[64];
  Fp zz[64], pre[64], suf[64];
  for (int l = 0; l < 64; ++l) {
    J0[l] = comb_entry_jac(B, 2u * l);
    J1[l] = jac_add_aff(J0[l], D);
    zz[l] = fp_mul(J0[l].z, J1[l].z);
    pre[l] = suf[l] = zz[l];
  }
  for (int d = 1; d < 64; d <<= 1) {
    Fp po[64], so[64];
    for (int l = 0; l < 64; ++l) {
      po[l] = pre[l - d >= 0 ? l - d : l];
      so[l] = suf[l + d < 64 ? l + d : l];
    }
    for (int l = 0; l < 64; ++l) {
      if (l - d >= 0) pre[l] = fp_mul(pre[l], po[l]);
      if (l + d < 64) suf[l] = fp_mul(suf[l], so[l]);
    }
  }
  Fp inv = fp_inv(pre[63]);
  int bad = 0;
  for (int l = 0; l < 64; ++l) {
    Fp ex_pre = l > 0 ? pre[l - 1] : FP_ONE, ex_suf = l < 63 ? suf[l + 1] : FP_ONE;
    Fp izz = fp_mul(inv, fp_mul(ex_pre, ex_suf));
    G1A a0 = aff_from_jac_inv(J0[l], fp_mul(izz, J1[l].z)), a1 = aff_from_jac_inv(J1[l], fp_mul(izz, J0[l].z));
    G1A r0, r1;
    jac_to_aff(r0, J0[l]);
    jac_to_aff(r1, J1[l]);
    bad += !(fp_eq(a0.x, r0.x) && fp_eq(a0.y, r0.y)) + !(fp_eq(a1.x, r1.x) && fp_eq(a1.y, r1.y));
  }
  return bad;
}
// SSZ hashing (sha256.h / ssz.h): 64 bytes -> sha256, and the AttestationData signing root.
static u32x8 ht_chunk_be(const uint8_t* p) {
  u32x8 r;
  for (int i = 0; i < 8; ++i) r[i] = ((uint32_t)p[4*i] << 24) | ((uint32_t)p[4*i+1] << 16) | ((uint32_t)p[4*i+2] << 8) | p[4*i+3];
  return r;
}
static void ht_store_be(uint8_t* o, u32x8 r) {
  for (int i = 0; i < 8; ++i) { o[4*i] = r[i] >> 24; o[4*i+1] = r[i] >> 16; o[4*i+2] = r[i] >> 8; o[4*i+3] = r[i]; }
}
void ht_digest64(uint8_t* out32, const uint8_t* in64) { ht_store_be(out32, sha256_digest64(sha256_cat(ht_chunk_be(in64), ht_chunk_be(in64 + 32)))); }
void ht_att_signing_root(uint8_t* out32, const uint8_t* data128, const uint8_t* domain32) {
  uint32_t d[32];
  for (int i = 0; i < 32; ++i) d[i] = (uint32_t)data128[4*i] | ((uint32_t)data128[4*i+1] << 8) | ((uint32_t)data128[4*i+2] << 16) | ((uint32_t)data128[4*i+3] << 24);
  ht_store_be(out32, ssz_signing_root(ssz_attestation_data_root(d), ht_chunk_be(domain32)));
}
}

// ---- the failure path's locate (locate.h), as k_sm_group_check / k_sm_fb_blocks run it ------------
// n sets over one message H: pk_i affine (96 B each), sig_i affine (192 B each, x.c0 x.c1 y.c0 y.c1), batch
// scalars r64[i]; the per-set terms r_i pk_i / r_i sig_i by randomize_pair, the chunk check value D of
// their sums, then locate_one.  Returns the located index, LOC_NONE, or 0xfffffffe when D == 1.
extern "C" unsigned ht_locate(const uint8_t* pks96, const uint8_t* sigs192, const uint64_t* r64, unsigned n, const uint8_t* h192) {
  std::vector<G1J> Pset(n);
  std::vector<G2J> Sset(n);
  G1J P = jac_infinity<Fp>();
  G2J S = jac_infinity<Fp2>();
  const G2A H{load_fp2(h192), load_fp2(h192 + 96)};
  for (unsigned i = 0; i < n; ++i) {
    const G1A pk{load_mont(pks96 + 96 * i), load_mont(pks96 + 96 * i + 48)};
    const G2A sg{load_fp2(sigs192 + 192 * i), load_fp2(sigs192 + 192 * i + 96)};
    if (!randomize_pair(pk, sg, r64[i], &Pset[i], &Sset[i])) return 0xfffffffdu;
    P = jac_add(P, Pset[i]);
    S = jac_add(S, Sset[i]);
  }
  Fp12 D;
  if (!pair_value_to(&D, P, H, S)) return 0xfffffffcu;
  if (fp12_is_one(D)) return 0xfffffffeu;
  return locate_one(0, n, &D, H, Pset.data(), Sset.data());
}

// ---- Fp-product counts of the per-unit work of each kernel path (bench.py roofline numerators) ----
// Each returns the number of Fp multiplications/squarings (FME) one unit costs on the code path the
// device runs; inputs are the caller's valid points/messages (data-independent control flow except
// for the rare exceptional additions, which valid random inputs never hit).
extern "C" {
unsigned long long ht_count_hash_to_g2(const uint8_t* msg32) {
  uint32_t w[8];
  for (int i = 0; i < 8; ++i) w[i] = ((uint32_t)msg32[4*i] << 24) | ((uint32_t)msg32[4*i+1] << 16) | ((uint32_t)msg32[4*i+2] << 8) | msg32[4*i+3];
  g_fme_count = 0;
  (void)hash_to_g2(w);
  return g_fme_count;
}
// G2 decompress + subgroup check of a 96-byte signature (Signature.fromBytes(sig, true))
unsigned long long ht_count_sig_validate(const uint8_t* sig96) {
  G2A s;
  g_fme_count = 0;
  if (g2_decode(s, sig96, 96) == PT_OK) (void)g2_in_subgroup(s);
  return g_fme_count;
}
// G2 decompression alone (k_sig_decode / k_vs_sig_decode)
unsigned long long ht_count_g2_decode(const uint8_t* sig96) {
  G2A s;
  g_fme_count = 0;
  (void)g2_decode(s, sig96, 96);
  return g_fme_count;
}
// the two halves of hash_to_G2 as the small-pass kernels split them: which = 0 the two SSWU maps +
// isogenies and Q0 + Q1 (k_hash_msgs_pre), 1 the cofactor clearing and the affine form
// (k_hash_clear_quad / k_hash_clear_coop)
unsigned long long ht_count_hash_part(const uint8_t* msg32, int which) {
  uint32_t w[8];
  for (int i = 0; i < 8; ++i) w[i] = ((uint32_t)msg32[4*i] << 24) | ((uint32_t)msg32[4*i+1] << 16) | ((uint32_t)msg32[4*i+2] << 8) | msg32[4*i+3];
  G2J q = jac_add(hash_map_iso(hash_to_field_fp2(w, 0)), hash_map_iso(hash_to_field_fp2(w, 1)));
  g_fme_count = 0;
  if (which == 0) {
    (void)jac_add(hash_map_iso(hash_to_field_fp2(w, 0)), hash_map_iso(hash_to_field_fp2(w, 1)));
  } else {
    G2A out;
    (void)jac_to_aff(out, clear_cofactor_g2(q));
  }
  return g_fme_count;
}
// randomize_pair (r pk and r sig) / randomize_g1 (r pk only)
unsigned long long ht_count_randomize(const uint8_t* p96, const uint8_t* q192, uint64_t r64, int g1_only) {
  G1A P{load_mont(p96), load_mont(p96 + 48)};
  G2A Q{load_fp2(q192), load_fp2(q192 + 96)};
  G1J rp;
  G2J rq;
  G1J PJ = jac_from_aff(P);
  g_fme_count = 0;
  if (g1_only == 1) randomize_g1(P, r64, &rp);
  else if (g1_only == 2) randomize_pair_jac(PJ, Q, r64, &rp, &rq);
  else if (g1_only == 3) randomize_g2(Q, r64, &rq);
  else randomize_pair(P, Q, r64, &rp, &rq);
  return g_fme_count;
}
// Miller value with Jacobian P (k_vs_miller / k_sm_miller)
unsigned long long ht_count_miller_1j(const uint8_t* p96, const uint8_t* q192) {
  G1J P = jac_from_aff(G1A{load_mont(p96), load_mont(p96 + 48)});
  G2A Q{load_fp2(q192), load_fp2(q192 + 96)};
  g_fme_count = 0;
  (void)miller_loop_1j(P, Q);
  return g_fme_count;
}
// Measured and not adopted: a shared-accumulator Miller loop for k pairs,
// as a thread-per-group kernel (k_vs_miller_group) it cut the per-set Fp products (7256 -> 6134 /
// 5573 for k = 2 / 4) but ran slower on the device (fewer threads, a frame-resident state).  Kept
// here as the counted prototype.
// prod_{j<k} f_{|x|, Q_j}(P_j) over k <= K pairs (P_j Jacobian) with one shared accumulator: one
// Fp12 squaring per bit for all k pairs (a third of one pair's per-bit products is that squaring:
// 36 of ~109 FME), then each pair's doubling / addition line.  The product equals the product of the
// k single-pair values (same lines, same Z^3 factors), so a chunk check multiplying Miller values
// sees the same Fp12.
}  // extern "C"
template <int K = 4>
static void miller_loop_kj_to(Fp12* out, const G1J* P, const G2A* Q, int k) {
  Fp z3[K], nxz[K];
  G2Proj T[K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    if (j < k) {
      z3[j] = fp_mul(fp_sqr(P[j].z), P[j].z);
      nxz[j] = fp_neg(fp_mul(P[j].x, P[j].z));
      T[j] = G2Proj{Q[j].x, Q[j].y, fp2_one()};
    }
  }
  Fp12 f = fp12_one();
  Line l;
  for (int i = 62; i >= 0; --i) {
    if (i != 62) fp12_sqr_to(&f, &f);
#pragma unroll
    for (int j = 0; j < K; ++j) {
      if (j < k) {
        l = dbl_step(T[j], nxz[j], P[j].y);
        l.c0 = fp2_mul_fp(l.c0, z3[j]);
        fp12_mul_line_to(&f, &l);
      }
    }
    if ((X_ABS >> i) & 1ull) {
#pragma unroll
      for (int j = 0; j < K; ++j) {
        if (j < k) {
          l = add_step(T[j], Q[j], nxz[j], P[j].y);
          l.c0 = fp2_mul_fp(l.c0, z3[j]);
          fp12_mul_line_to(&f, &l);
        }
      }
    }
  }
  fp12_conj_to(out, &f);
}
extern "C" {

// The shared-accumulator loop against the product of per-pair Miller values: P_j =
// 2 (p_j) (Jacobian, Z != 1), Q_j affine; mode 0 = product of miller_loop_1j, 1 and 2 = miller_loop_kj_to
// (k <= 4).  out = the Fp12 (12 canonical Fp, tower order); returns the FME count.
unsigned long long ht_miller_group(uint8_t* out, const uint8_t* p96, const uint8_t* q192, int k, int mode) {
  G1J P[4];
  G2A Q[4];
  for (int j = 0; j < k; ++j) {
    P[j] = jac_dbl(jac_from_aff(G1A{load_mont(p96 + 96 * j), load_mont(p96 + 96 * j + 48)}));
    Q[j] = G2A{load_fp2(q192 + 192 * j), load_fp2(q192 + 192 * j + 96)};
  }
  g_fme_count = 0;
  Fp12 f;
  if (mode == 0) {
    f = fp12_one();
    for (int j = 0; j < k; ++j) {
      Fp12 g = miller_loop_1j(P[j], Q[j]);
      f = fp12_mul(f, g);
    }
  } else if (mode == 1) {
    miller_loop_kj_to<4>(&f, P, Q, k);
  } else {
    miller_loop_kj_to<4>(&f, P, Q, k);
  }
  const Fp2* c[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
  for (int i = 0; i < 6; ++i) store_fp2(out + 96 * i, *c[i]);
  return g_fme_count;
}
// A call of n sets as round 5's k_vs_miller_group<K> cut it: groups of K consecutive sets, the last one
// ragged (n mod K sets), each group's product on one shared accumulator; against the product of the n
// per-set values (miller_loop_1j).  P_j = 2 p_j (Jacobian, Z != 1).  Writes both Fp12 (576 bytes each).
void ht_miller_call_groups(uint8_t* want, uint8_t* got, const uint8_t* p96, const uint8_t* q192, int n, int K) {
  std::vector<G1J> P(n);
  std::vector<G2A> Q(n);
  for (int j = 0; j < n; ++j) {
    P[j] = jac_dbl(jac_from_aff(G1A{load_mont(p96 + 96 * j), load_mont(p96 + 96 * j + 48)}));
    Q[j] = G2A{load_fp2(q192 + 192 * j), load_fp2(q192 + 192 * j + 96)};
  }
  Fp12 a = fp12_one(), b = fp12_one();
  for (int j = 0; j < n; ++j) a = fp12_mul(a, miller_loop_1j(P[j], Q[j]));
  for (int j = 0; j < n; j += K) {
    const int k = n - j < K ? n - j : K;
    Fp12 g;
    if (K == 2)
      miller_loop_kj_to<2>(&g, &P[j], &Q[j], k);
    else
      miller_loop_kj_to<4>(&g, &P[j], &Q[j], k);
    b = fp12_mul(b, g);
  }
  const Fp12* f[2] = {&a, &b};
  uint8_t* o[2] = {want, got};
  for (int t = 0; t < 2; ++t) {
    const Fp2* c[6] = {&f[t]->c0.c0, &f[t]->c0.c1, &f[t]->c0.c2, &f[t]->c1.c0, &f[t]->c1.c1, &f[t]->c1.c2};
    for (int i = 0; i < 6; ++i) store_fp2(o[t] + 96 * i, *c[i]);
  }
}
// one mixed G1 addition (the gather-aggregate step), one full G1 addition (tree step),
// one Fp12 product, one Jacobian G2 addition, one final exponentiation
unsigned long long ht_count_op(int which, const uint8_t* p96, const uint8_t* q192) {
  G1A P{load_mont(p96), load_mont(p96 + 48)};
  G2A Q{load_fp2(q192), load_fp2(q192 + 96)};
  G1J J = jac_dbl(jac_from_aff(P));
  G2J JQ = jac_dbl(jac_from_aff(Q));
  Fp12 f = miller_loop_1(P, Q);
  g_fme_count = 0;
  switch (which) {
    case 0: (void)jac_add_aff(J, P); break;
    case 1: (void)jac_add(J, jac_dbl(J)); g_fme_count -= 0; break;
    case 2: (void)fp12_mul(f, f); break;
    case 3: (void)jac_add(JQ, jac_dbl(JQ)); break;
    case 4: (void)final_exponentiation(f); break;
    case 5: { G1A a; (void)jac_to_aff(a, J); break; }
    default: break;
  }
  return g_fme_count;
}
}
