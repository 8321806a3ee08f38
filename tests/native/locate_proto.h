// Prototype (test-only): locating the one invalid set of a failing same-message chunk from the
// per-set randomised terms, host-tested against the oracle (tests/native/hosttest.cpp ht_locate,
// tests/test_host_arith.py::test_locate_one_invalid_set).  Round 5 ran it on the GPU in three forms,
// all slower than the run / per-set checks it shortcuts (C5 6.3 M sets/s without it): inside the
// thread-per-chunk group check (3.3 M: half of each wave's lanes idle behind one ~50 k-product chain),
// as one wave per chunk on the cooperative steps (5.2 M: the engine's per-product overhead on a
// saturated device), and as compacted thread-per-chunk phases (5.4 M: ~6.5 k chains of ~30 k products
// cannot fill 1 024 SIMDs, where the ~65 k run checks do).  DESIGN.md 7.
#pragma once
#include "../../lodestar_amd/csrc/pairing.h"

namespace gbv {

GBV_NI G1J loc_g1_add(G1J a, G1J b) { return jac_add(a, b); }
GBV_NI G2J loc_g2_add(G2J a, G2J b) { return jac_add(a, b); }

// ---- locating the invalid set of a failing chunk or run --------------------------------------------
// With the batch scalars r_i of its check, a chunk (or 8-set run) of sets i = b .. e-1 checks
//   D = FE(prod_i e(r_i pk_i, H) e(-g1, r_i sig_i)) = prod_i E_i^{r_i},  E_i = e(pk_i, H) / e(g1, sig_i),
// and E_i = 1 exactly for a valid set.  When D != 1 because ONE set w is invalid, the position-weighted
// check D' = FE(prod_i e(w_i r_i pk_i, H) e(-g1, w_i r_i sig_i)), w_i = i - b + 1, equals D^{w_w} (D has
// order r, so the w <= e - b with D^w = D' is unique); the candidate is confirmed by its own term,
// X = FE(e(r_w pk_w, H) e(-g1, r_w sig_w)) == D -- then prod_{i != w} E_i^{r_i} = 1, which is the
// randomised batch check of the chunk without w (the same 2^-64 soundness as the chunk's own check),
// and w is invalid because D != 1.  No candidate, or X != D (two or more invalid sets), leaves the
// chunk to the run / per-set checks.  The reference retries every set of a failing chunk on its own
// (jobItem.ts:93-125); the booleans are the same, the work ~3 pairing checks instead of ~18.
// The weighted sums come from the per-set terms k_sm_prepare / k_sm_prep_scan / k_sm_redo_g2 keep
// (Pset, Sset: infinity for a rejected set): suffix sums T_i = sum_{j >= i} X_j, sum_i T_i =
// sum_j (j - b + 1) X_j, two additions per set.
constexpr uint32_t LOC_NONE = 0xffffffffu;

// FE(f(P, H) f(-g1, S)) with P Jacobian (its lines carry a Z^3 factor the final exponentiation removes)
// and S Jacobian; S at infinity drops its pair; false for P at infinity.
GBV_NI bool pair_value_to(Fp12* out, G1J P, G2A Hm, G2J S) {
  if (jac_is_inf(P)) return false;
  Fp12 f;
  miller_loop_1j_to(&f, P, Hm);
  G2A sa;
  if (jac_to_aff(sa, S)) {
    Fp12 h;
    miller_loop_1_to(&h, g1_neg_generator(), sa);
    fp12_mul_to(&f, &f, &h);
  }
  final_exponentiation_to(out, &f);
  return true;
}

GBV_NI void weighted_sums(uint32_t b, uint32_t e, const G1J* __restrict__ Pset, const G2J* __restrict__ Sset, G1J* Pw, G2J* Sw) {
  G1J tp = jac_infinity<Fp>(), ap = jac_infinity<Fp>();
  G2J ts = jac_infinity<Fp2>(), as = jac_infinity<Fp2>();
  for (uint32_t i = e; i-- > b;) {
    tp = loc_g1_add(tp, Pset[i]);
    ap = loc_g1_add(ap, tp);
    ts = loc_g2_add(ts, Sset[i]);
    as = loc_g2_add(as, ts);
  }
  *Pw = ap;
  *Sw = as;
}

// the w in [1, n] with D^w == Dw, or 0
GBV_NI uint32_t dlog_small(const Fp12* D, const Fp12* Dw, uint32_t n) {
  Fp12 y = *D;
  for (uint32_t w = 1; w <= n; ++w) {
    if (fp12_eq(y, *Dw)) return w;
    fp12_mul_to(&y, &y, D);
  }
  return 0;
}

// the one invalid set of [b, e) given its check value D != 1, or LOC_NONE
GBV_NI uint32_t locate_one(uint32_t b, uint32_t e, const Fp12* D, G2A Hm, const G1J* __restrict__ Pset, const G2J* __restrict__ Sset) {
  G1J Pw;
  G2J Sw;
  weighted_sums(b, e, Pset, Sset, &Pw, &Sw);
  Fp12 Dw;
  if (!pair_value_to(&Dw, Pw, Hm, Sw)) return LOC_NONE;
  const uint32_t w = dlog_small(D, &Dw, e - b);
  if (!w) return LOC_NONE;
  const uint32_t i = b + w - 1;
  Fp12 X;
  if (!pair_value_to(&X, Pset[i], Hm, Sset[i])) return LOC_NONE;
  return fp12_eq(X, *D) ? i : LOC_NONE;
}

}  // namespace gbv
