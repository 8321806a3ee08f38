// Host-side launchers of the gfx950 kernels (one translation unit per kernel family so the build
// parallelises; gbv.hip sequences them on the context stream).
#pragma once
#include <hip/hip_runtime.h>

#include <vector>
#include "curve.h"
#include "fp12.h"

namespace gbv {
struct Seed;
struct LaunchCfg { unsigned blocks; unsigned threads; hipStream_t stream; };

// Qpre (optional, n entries): Q0 + Q1 of the lane-pair maps ahead of the latency forms of the cofactor
// clearing (k_hash_clear_coop: one workgroup per message, n <= GBV_HASH_COOP_MAX; k_hash_clear_quad)
void launch_hash_msgs(LaunchCfg c, const uint8_t* msgs32, uint32_t n, G2A* H, G2J* Qpre = nullptr);
void launch_hash_clear_coop(hipStream_t s, uint32_t n, const G2J* Qpre, G2A* H);
void launch_util_g2_out(LaunchCfg c, uint32_t n, const G2A* H, uint8_t* out192);

// Signature.fromBytes decoding of sets [base, base + n): S[i] = the point, status[i] = GBV_PT_* (k_dec.hip)
void launch_sig_decode(hipStream_t s, uint32_t base, uint32_t n, const uint8_t* sig96, G2A* S, uint8_t* status);
void launch_vs_sig_decode(hipStream_t s, uint32_t n, const uint8_t* sig, uint32_t sig_stride, const uint32_t* sig_len, G2A* S,
                          uint8_t* dec_st);
void launch_sm_prepare(LaunchCfg c, uint32_t base, uint32_t n, const uint32_t* idx, const uint8_t* sig96, const uint32_t* set_grp,
                       const G1A* table, const uint8_t* table_ok, uint32_t table_n, const uint4* comb, const uint8_t* comb_ok,
                       const Seed& seed, uint32_t nonce, G2A* S_out, G2J* Sh, G1J* Ph, uint8_t* status, uint8_t* scratch8);
// few sets (k_sm_coop.hip): cooperative subgroup checks (one wave per set, verdict in sub_ok) beside
// the per-set randomisation (r sig / r pk into Sh / Ph at the set's index), after k_sig_decode
void launch_sm_prep_roles_quad(hipStream_t s, uint32_t base, uint32_t n, const uint32_t* idx, const G1A* table, const uint8_t* table_ok,
                               uint32_t table_n, const uint4* comb, const uint8_t* comb_ok, const Seed& seed, uint32_t nonce, const G2A* S,
                               const uint8_t* status, uint8_t* sub_ok, G2J* Sh, G1J* Ph);
void launch_sm_chunk_finish(LaunchCfg c, uint32_t g0, uint32_t G, uint32_t s0, const uint32_t* grp_off, const uint8_t* status, const G2J* Sh,
                            const G1J* Ph, G1J* PgJ, G2J* SgJ, uint8_t* grp_state, uint32_t* n_fallback);
void launch_sm_miller_quad(LaunchCfg c, uint32_t g0, uint32_t G, const uint32_t* grp_msg, const uint8_t* grp_state, const G1J* PgJ,
                           const G2A* H, Fp12* F);
void launch_sm_miller(LaunchCfg c, uint32_t g0, uint32_t G, const uint32_t* grp_msg, const uint8_t* grp_state, const G1J* PgJ, const G2A* H,
                      Fp12* F);
uint32_t launch_seg_reduce_quad(hipStream_t s, uint32_t g0, uint32_t G, const uint8_t* grp_state, const Fp12* F, const G2J* SgJ, Fp12* Fpart,
                                G2J* Spart, uint8_t* has, uint32_t* n_out);
void launch_sm_seg_check(LaunchCfg c, uint32_t g0, uint32_t G, uint8_t* grp_state, const Fp12* F, const G2J* SgJ, Fp12* Fpart, G2J* Spart,
                         uint8_t* has, uint8_t* seg_ok, Fp12* miller_out = nullptr, const G2J* S_extra = nullptr);
// runs when the segment check failed or any chunk went to the per-set path (n_fallback > 0)
void launch_sm_redo_g2(LaunchCfg c, uint32_t base, uint32_t n, const uint32_t* set_grp, const uint8_t* status, const G2A* S, const Seed& seed,
                       uint32_t nonce, const uint8_t* seg_ok, const uint32_t* n_fallback, G2J* Sh);
void launch_sm_chunk_finish_s(LaunchCfg c, uint32_t g0, uint32_t G, uint32_t s0, const uint32_t* grp_off, const uint8_t* grp_state,
                              const G2J* Sh, const uint8_t* seg_ok, G2J* SgJ);
// Bucket MSM of a same-message segment: total = sum over its sets with status OK in pending chunks
// of r_i sig_i (k_msm.hip).  Scratch: cnt/off/cur MSM_KEYS u32 each, ent 4 u32 per set, buckets
// MSM_KEYS G2J, part MSM_PARTS + 130 G2J.
#ifndef GBV_MSM_RUN
#define GBV_MSM_RUN 32
#endif
constexpr uint32_t MSM_RUN = GBV_MSM_RUN;  // sorted entries per thread of k_msm_runs (head/tail: 4n/MSM_RUN + 1 G2J each)
constexpr uint32_t MSM_C = 16, MSM_WINDOWS = 2, MSM_KEYS = MSM_WINDOWS << MSM_C, MSM_SLICE = 16, MSM_PARTS = MSM_KEYS / MSM_SLICE;
// throughput part (stream A): entries, counting sort, bucket sums
void launch_msm_g2_buckets(hipStream_t s, uint32_t s0, uint32_t n, const uint32_t* set_grp, const uint8_t* status, const uint8_t* grp_state,
                           const G2A* S, const Seed& seed, uint32_t nonce, uint32_t* cnt, uint32_t* off, uint32_t* cur, uint32_t* ent,
                           G2J* buckets, G2J* head, G2J* tail);
// latency part (tail stream): slice running sums and the tree sum into *total
void launch_msm_g2_reduce(hipStream_t s, const G2J* buckets, G2J* part, G2J* total);
void launch_fp12_check(LaunchCfg c, uint32_t k, const Fp12* parts, uint8_t* out);
// chunk_be: (begin, end) set range of each of the C chunks
void launch_vs_chunk_coop(LaunchCfg c, uint32_t C, const uint32_t* chunk_be, const uint8_t* status, const Fp12* f, const G2J* rS,
                          uint8_t* chunk_valid, const Fp12* Fs = nullptr, const uint8_t* fs_flag = nullptr);
void launch_sm_group_pairing(LaunchCfg c, uint32_t g0, uint32_t G, const uint32_t* grp_msg, const G1J* PgJ, const G2J* SgJ, const G2A* H,
                             const uint8_t* seg_ok, uint8_t* grp_state, uint32_t* n_fallback, Fp12* Fpair, uint8_t* pair_ok);
void launch_sm_fallback(LaunchCfg c, uint32_t n, const uint32_t* set_grp, const uint32_t* grp_msg, const uint8_t* grp_state,
                        const uint8_t* status, const uint32_t* idx, const G1A* table, const G2A* S, const G2A* H, uint8_t* valid,
                        int do_fallback);

// thread per pending chunk of a failed segment: the chunk's own check
void launch_sm_group_check(LaunchCfg c, uint32_t g0, uint32_t G, const Fp12* F, const G2J* SgJ, const uint8_t* seg_ok, uint8_t* grp_state,
                           uint32_t* n_fallback);
void launch_sm_fb_runs(LaunchCfg c, uint32_t s0, uint32_t n, const uint32_t* set_grp, const uint8_t* grp_state, uint4* runs, uint32_t* n_runs,
                       uint32_t cap);
void launch_sm_fb_blocks(LaunchCfg c, const uint4* runs, const uint32_t* n_runs, uint32_t cap, const uint8_t* status, const uint32_t* grp_msg,
                         const G2J* Sh, const G1J* Ph, const G2A* H, uint8_t* valid, uint32_t* set_list, uint32_t* n_list, uint32_t coop_max);
void launch_sm_fb_sets(LaunchCfg c, const uint32_t* set_list, const uint32_t* n_list, const uint32_t* set_grp, const uint32_t* grp_msg,
                       const uint32_t* idx, const G1A* table, const G2A* S, const G2A* H, uint8_t* valid, uint32_t coop_max);

void launch_sm_fb_blocks_coop(LaunchCfg c, const uint4* runs, const uint32_t* n_runs, uint32_t cap, const uint8_t* status,
                              const uint32_t* grp_msg, const G2J* Sh, const G1J* Ph, const G2A* H, uint8_t* valid, uint32_t* set_list,
                              uint32_t* n_list, uint32_t coop_max);
void launch_sm_fb_sets_coop(LaunchCfg c, const uint32_t* set_list, const uint32_t* n_list, const uint32_t* set_grp, const uint32_t* grp_msg,
                            const uint32_t* idx, const G1A* table, const G2A* S, const G2A* H, uint8_t* valid, Fp12* Fpair, uint32_t coop_max);

void launch_pk_decompress(LaunchCfg c, uint32_t n, const uint8_t* pk48, int validate, G1A* table, uint8_t* table_ok, uint8_t* status);
void launch_comb_build(hipStream_t s, uint32_t first, uint32_t n, const G1A* table, const uint8_t* table_ok, G1A* bases9, uint4* comb,
                       uint8_t* comb_ok);
void launch_util_g1_mul_rand(hipStream_t s, uint32_t n, const uint32_t* slots, const uint64_t* r64, const G1A* table, const uint4* comb,
                             int use_comb, uint8_t* out48);
void launch_comb_replicate(hipStream_t s, uint4* comb, uint8_t* comb_ok, uint32_t src_first, uint32_t src_n, uint32_t dst_first, uint32_t n);
void launch_pk_replicate(LaunchCfg c, G1A* table, uint8_t* table_ok, uint32_t src_first, uint32_t src_n, uint32_t dst_first, uint32_t n);
// idx == nullptr: entries 0..k-1 of table (serialized keys decompressed into scratch slots; slots
// with table_ok == 0 -- infinity keys -- are skipped rather than flagged)
void launch_aggregate(LaunchCfg c, const uint32_t* idx, uint32_t k, const G1A* table, const uint8_t* table_ok, uint8_t* out48,
                      uint32_t* bad);
void launch_util_sk_to_pk(LaunchCfg c, uint32_t n, const uint8_t* sk32, uint8_t* pk48);
void launch_util_sign(LaunchCfg c, uint32_t n, const uint8_t* sk32, const uint32_t* grp, const G2A* H, uint8_t* sig96);

// verifySignatureSets batches (k_vs.hip)
void launch_vs_agg(LaunchCfg c, const uint32_t* agg_list, const uint32_t* set_off, const uint32_t* arena, const G1A* table,
                   const uint8_t* table_ok, G1J* pk_out, uint8_t* pk_st);
// large aggregate sets (>= AGG_BIG_MIN members): slices (begin, end) of AGG_SLICE members, one
// 256-thread workgroup each, then one wave per set over its slices; big = (set, first slice, count)
constexpr uint32_t AGG_BIG_MIN = 1024;  // slice size: tuning().agg_slice
void launch_vs_agg_big(hipStream_t s, uint32_t n_slices, const uint4* slices, uint32_t n_big, const uint4* big, const uint32_t* arena,
                       const G1A* table, const uint8_t* table_ok, G1J* part, uint8_t* part_bad, G1J* pk_out, uint8_t* pk_st);
void launch_vs_hash_sig(hipStream_t s, uint32_t n, const uint8_t* msgs32, const uint32_t* set_off, const uint32_t* arena,
                        const uint8_t* raw_flag, const uint8_t* raw_pk48, const uint8_t* sig, uint32_t sig_stride, const uint32_t* sig_len,
                        const G1A* table, const uint8_t* table_ok, const G1J* pk_agg, const uint8_t* pk_st, const Seed& seed,
                        uint32_t nonce, G2A* H, G1J* rP, G2J* rS, uint8_t* status, bool split = false);
// the same per-set work in two halves for small passes: signatures (no pubkey needed) beside the
// aggregation, then the pubkeys (k_vs.hip)
void launch_vs_sig_pre(hipStream_t s, uint32_t n, const uint8_t* sig, uint32_t sig_stride, const uint32_t* sig_len, const Seed& seed,
                       uint32_t nonce, G2J* rS, uint8_t* status, uint8_t* sig_st, G2A* Sd, uint8_t* dec_st);
void launch_vs_pk_rand(hipStream_t s, uint32_t n, const uint32_t* set_off, const uint32_t* arena, const uint8_t* raw_flag,
                       const uint8_t* raw_pk48, const G1A* table, const uint8_t* table_ok, const G1J* pk_agg, const uint8_t* pk_st,
                       const Seed& seed, uint32_t nonce, G1J* rP, uint8_t* status);
void launch_vs_miller_coop(hipStream_t s, uint32_t n, const uint8_t* status, const G1J* rP, const G2A* H, Fp12* F);
void launch_vs_chunk_s_miller(hipStream_t s, uint32_t C, const uint8_t* status, const uint32_t* chunk_be, const G2J* rS, Fp12* Fs,
                              uint8_t* fs_flag);
void launch_vs_miller(LaunchCfg c, uint32_t n, const uint8_t* status, const G1J* rP, const G2A* H, Fp12* F);
void launch_sig_validate(LaunchCfg c, uint32_t n, const uint8_t* sig, uint32_t sig_len, uint8_t* status, uint8_t* out96);
void launch_sig_aggregate(hipStream_t s, uint32_t n, const uint8_t* sig, uint32_t sig_len, int validate, G2J* part, uint32_t* bad,
                          uint8_t* out96);

void launch_ssz_digest64(hipStream_t s, const uint8_t* in64, uint32_t n, uint8_t* out32);
void launch_ssz_signing_roots(hipStream_t s, const uint8_t* roots32, uint32_t n, const uint8_t* domains32, const uint32_t* dom_idx,
                              uint8_t* out32);
void launch_ssz_att_signing_roots(hipStream_t s, const uint8_t* data128, uint32_t n, const uint8_t* domains32, const uint32_t* dom_idx,
                                  uint8_t* out32);
}  // namespace gbv

namespace gbv {
// GBV_SYNC_DEBUG=1: synchronise after every launch and report the failing kernel by name.
void debug_sync(hipStream_t s, const char* kernel);

// Per-kernel device time of a pass (bench rooflines, gbv_last_ops): while an enqueue routine has set
// t_kprof (the context's "kprof" setting), every GBV_LAUNCH brackets its kernel with two HIP events
// on the kernel's own stream and records the kernel's name, its grid in work-items (rocprofv3's
// Grid_Size, so PMC rows can be matched to it) and the units of work it covers.
struct KRec {
  const char* name;
  uint32_t threads, units;
  hipEvent_t a, b;
};
struct KProf {
  std::vector<KRec> recs;
  std::vector<hipEvent_t> pool;  // created on first use, reused pass after pass
  size_t used = 0;
  void reset() { recs.clear(); used = 0; }
  void destroy() {
    for (hipEvent_t e : pool) (void)hipEventDestroy(e);
    pool.clear();
    reset();
  }
};
extern thread_local KProf* t_kprof;
void kprof_begin(hipStream_t s, const char* name, uint32_t threads, uint32_t units);
void kprof_end(hipStream_t s);
struct KScope {
  hipStream_t s;
  KScope(hipStream_t s_, const char* name, uint32_t threads, uint32_t units) : s(s_) { kprof_begin(s, name, threads, units); }
  ~KScope() { kprof_end(s); }
};
}  // namespace gbv

// hipLaunchKernelGGL + the kprof events + debug_sync.  NAME is the kernel's name as rocprofv3 prints
// it (template instances included), UNITS the sets / messages / chunks the launch covers.
#define GBV_LAUNCH(NAME, KERNEL, GRID, BLOCK, STREAM, UNITS, ...)                                              \
  do {                                                                                                       \
    const dim3 g_ = (GRID), b_ = (BLOCK);                                                                    \
    gbv::KScope ks_((STREAM), NAME, (uint32_t)(g_.x * g_.y * g_.z * b_.x * b_.y * b_.z), (uint32_t)(UNITS)); \
    hipLaunchKernelGGL(KERNEL, g_, b_, 0, (STREAM), __VA_ARGS__);                                            \
    gbv::debug_sync((STREAM), NAME);                                                                         \
  } while (0)
