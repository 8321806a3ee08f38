// Shared pieces of the gfx950 kernels of the signature-set verifier.  One thread owns one signature set (or one
// chunk / one message) and keeps its field elements in VGPRs; the kernels of one call run back to
// back on the context's HIP stream.
//
// Reference mapping:
//   k_hash_msgs         hash_to_G2 inside blst verify / verifyMultipleAggregateSignatures
//   k_sm_prepare        aggregateWithRandomness per set: Signature.fromBytes(sig, true) + r_i*pk, r_i*sig
//                       (multithread/jobItem.ts:73)
//   k_sm_prepare        also sums r_i pk_i, r_i sig_i per chunk within each wave (segmented scan)
//   k_sm_chunk_finish   sum_i r_i pk_i, sum_i r_i sig_i per same-message chunk from the wave sums
//   k_sm_miller         Miller value of (sum r_i pk_i, H(m)) per chunk (thread per chunk)
//   k_sm_seg_check      one randomised multi-pairing check over a segment of chunks
//   k_sm_group_pairing  verify(msg, aggPk, aggSig) of the chunk (worker.ts:29-107 -> maybeBatch n = 1),
//                       only for chunks of a failing segment
//   k_sm_fallback       retry each set individually (jobItem.ts:93-125)
//   k_vs_agg            aggregatePublicKeys of index lists (bls/utils.ts:5-20), one wave per set
//   k_vs_hash_sig       per-set part of verifyMultipleAggregateSignatures: hash_to_G2 | decode,
//                       subgroup check, randomisation (two block roles of one launch)
//   k_vs_miller         per-set Miller values
//   k_vs_chunk_coop     per-chunk multi-pairing product + one final exponentiation, one wave per chunk
//                       (maybeBatch.ts:17-26)
//   k_fp12_check        product of per-GPU Miller partials + one final exponentiation (multi-GPU)
#pragma once
#include <atomic>
#include "hash_to_curve.h"
#include "pairing.h"

// One wave per workgroup; the register budget is capped so that two waves share each SIMD
// (measured on MI355X, tools/ubench_fp.hip: 2 waves/SIMD beat 1 and 3 for the point kernels,
// whose live state -- a Jacobian G2 point plus its operand -- does not fit the 128 VGPRs of 4).
#ifndef GBV_WAVES_PER_EU
#define GBV_WAVES_PER_EU 2
#endif
#define GBV_KERNEL_ATTR __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(GBV_WAVES_PER_EU)))
// lane-quad point kernels of small passes (k_hash_msgs_quad, k_vs_sig_pre_quad, k_vs_pk_rand_quad)
#ifndef GBV_QUAD_WPE
#define GBV_QUAD_WPE 1  // 512 registers, fewer frame spills: 64-block pass 12.2 -> 11.75 ms, 2 in flight 9.3 -> 8.3-8.6 ms
#endif
// thread-serial pairing checks of the same-message failure path (k_sm_fb.hip)
#ifndef GBV_FB_WPE
#define GBV_FB_WPE 2  // 1 wave: k_sm_fb_blocks / _sets 57.8 -> 63 ms (profiles/r05s)
#endif
#ifndef GBV_GRPCHK_WPE
#define GBV_GRPCHK_WPE 1  // k_sm_group_check (~200 waves): 1 wave 31.8 -> 24-26 ms (profiles/r05s)
#endif
constexpr unsigned FB_GRID = 1024 * GBV_FB_WPE;  // persistent failure-path grids: GBV_FB_WPE waves per SIMD
#define GBV_QUAD_ATTR __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(GBV_QUAD_WPE, GBV_QUAD_WPE)))

// Tail kernels (chunk Miller values, MSM reduction, segment reduction and check) share SIMDs with
// the next batch's k_sm_prepare; GBV_TAIL_PRIO > 0 raises their waves' issue priority (s_setprio)
// so the tail of a batch finishes sooner.  0 = hardware default.
#ifndef GBV_TAIL_PRIO
#define GBV_TAIL_PRIO 0
#endif
#define GBV_TAIL_WAVE_PRIO() \
  do {                       \
    if (GBV_TAIL_PRIO > 0) __builtin_amdgcn_s_setprio(GBV_TAIL_PRIO); \
  } while (0)

namespace gbv {

struct Seed { uint32_t w[8]; };

enum : uint8_t { SET_OK = 0, SET_BAD_SIG = 1, SET_BAD_PK = 2 };
enum : uint8_t { GRP_PENDING = 0, GRP_FALLBACK = 1, GRP_OK = 2 };
// Failure-path item counts up to which one wave per item (k_sm_fb_*_coop, latency) beats one
// thread per item (k_sm_fb_blocks / k_sm_fb_sets, throughput).
constexpr uint32_t FB_COOP_MAX = 16384;  // default of gbv_tune "fb_coop_max" (131 072-set C5 batches +16 %, 1M unchanged: profiles/r06l)
constexpr uint32_t FB_COOP_CAP = 16384;  // its largest value (the per-batch scratch of the two-wave per-set checks)
// Sets per failure-path run (the 8-set scan windows of k_sm_prepare).  When the failing runs hold at
// most FB_COOP_MAX sets in all, k_sm_fb_blocks_coop skips the run checks and hands every set to the
// per-set stage: one pairing stage of latency instead of two.
constexpr uint32_t FB_RUN_MAX = 8;
// Message counts up to which hash_to_G2 runs on lane pairs (latency) instead of one lane each.
constexpr uint32_t HASH_PAIR_MAX = 4096;

// Launch-shape tunables (host side only, process-wide).  Defaults are the measured choices of
// DESIGN.md section 7; experiments change them through gbv_tune (tuning_set, by the names below), never
// through a beacon node's environment.  Only GBV_SYNC_DEBUG is read from the environment (tuning_load,
// first gbv_init): it synchronises after every launch, which changes timing, not results.
struct Tuning {  // relaxed atomics: gbv_tune may run beside another context's enqueue
  std::atomic<uint32_t> hash_pair_max{HASH_PAIR_MAX};  // hash on lane pairs up to this many messages
  std::atomic<uint32_t> hash_quad_max{16384};          // hash on lane quads up to this many messages
  std::atomic<uint32_t> hash_coop_max{128};            // latency form, cofactor clearing one workgroup per message (two waves each: past ~128 messages they crowd the signature work beside them)
  std::atomic<uint32_t> prepare_split_max{2048};       // same-message latency prepare up to this many sets
  std::atomic<uint32_t> chunk_finish_wave_max{32};     // chunk sums one wave per chunk up to this many
  std::atomic<uint32_t> vs_pre_max{16384};             // verifySignatureSets signature half (lane quads) beside the aggregation
  std::atomic<uint32_t> vs_fs_maxc{256};               // per-chunk (-g1, sum) Miller value beside the per-set ones
  std::atomic<uint32_t> vs_quad_max{16384};            // per-set Miller values on lane quads up to this many sets
  std::atomic<uint32_t> vs_pair_max{32768};            // ... on lane pairs up to this many (one lane per set above)
  std::atomic<uint32_t> agg_slice{8192};               // large aggregates: members per k_vs_agg_big workgroup (256 threads; profiles/r05l)
  std::atomic<uint32_t> fb_coop_max{FB_COOP_MAX};      // same-message failure path: run / per-set checks one wave each up to this many
  std::atomic<uint32_t> group_thread_min{512};         // ... chunk checks one thread each from this many chunks of a segment (one wave each below)
  std::atomic<uint32_t> sm_quad_max{8192};               // same-message chunk Miller values on lane quads up to this many chunks of a segment
  std::atomic<uint32_t> sync_debug{0};                 // GBV_SYNC_DEBUG: synchronise + report after every launch (debugging)
};
const Tuning& tuning();
void tuning_load();
bool tuning_set(const char* name, uint32_t value);  // false for an unknown name
// verifySignatureSets passes up to this many sets compute their Miller values one wave per set
// (cooperative, ~2.9 ms) instead of one thread per set (~16 ms of latency, far less VALU in total).
constexpr uint32_t VS_COOP_MILLER_MAX = 2048;

// Per-set random 64-bit scalar r_i = SHA-256(seed || i || nonce)[0..8), forced non-zero.
// blst draws 64-bit random scalars for the same purpose; only the booleans are compared.
__device__ inline uint64_t prf_scalar(const Seed& s, uint32_t i, uint32_t nonce) {
  uint32_t st[8];
  sha256_init(st);
  uint32_t blk[16];
  for (int k = 0; k < 8; ++k) blk[k] = s.w[k];
  blk[8] = i;
  blk[9] = nonce;
  blk[10] = 0x80000000u;
  for (int k = 11; k < 15; ++k) blk[k] = 0;
  blk[15] = 40u * 8u;
  sha256_compress(st, blk);
  uint64_t r = ((uint64_t)st[0] << 32) | st[1];
  return r ? r : 1ull;
}

// Lane-pair hash_to_G2 for latency (few messages): lanes 2m and 2m+1 map u_0 and u_1 of message m
// at the same time, the odd lane hands its point over (shuffles), the even lane clears the
// cofactor.  Every lane of the wave must call it (the shuffles); returns true on the even lane.
__device__ inline Fp shfl_fp(const Fp& a, int src) {
  Fp r;
#pragma unroll
  for (int i = 0; i < 12; ++i) r.v[i] = __shfl((unsigned)a.v[i], src, 64);
  return r;
}
__device__ inline bool hash_to_g2_lane_pair(const uint32_t w[8], bool active, G2A* out) {
  const int lane = (int)threadIdx.x, half = lane & 1;
  G2J q = jac_infinity<Fp2>();
  if (active) q = hash_map_iso(hash_to_field_fp2(w, half));
  Fp* f = (Fp*)&q;
  G2J o;
  Fp* g = (Fp*)&o;
#pragma unroll
  for (int i = 0; i < 6; ++i) g[i] = shfl_fp(f[i], lane | 1);
  if (!active || half) return false;
  *out = hash_finish(q, o);
  return true;
}

// The same lane pairs, stopping before the cofactor clearing: Q0 + Q1 (Jacobian) on the even lane
// (k_hash_clear_quad then clears the cofactor on a lane quad per message).
__device__ inline bool hash_to_g2_lane_pair_pre(const uint32_t w[8], bool active, G2J* out) {
  const int lane = (int)threadIdx.x, half = lane & 1;
  G2J q = jac_infinity<Fp2>();
  if (active) q = hash_map_iso(hash_to_field_fp2(w, half));
  Fp* f = (Fp*)&q;
  G2J o;
  Fp* g = (Fp*)&o;
#pragma unroll
  for (int i = 0; i < 6; ++i) g[i] = shfl_fp(f[i], lane | 1);
  if (!active || half) return false;
  *out = jac_add(q, o);
  return true;
}

__device__ inline void load_msg_words(uint32_t w[8], const uint8_t* m) {
  for (int i = 0; i < 8; ++i)
    w[i] = ((uint32_t)m[4 * i] << 24) | ((uint32_t)m[4 * i + 1] << 16) | ((uint32_t)m[4 * i + 2] << 8) | m[4 * i + 3];
}

}  // namespace gbv
