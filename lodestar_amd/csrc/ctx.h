// Host-side context of the C ABI (include/gbv.h), shared by the translation units that implement
// it: gbv.hip (context, pubkey table, same-message batches, signing roots, utilities) and gbv_vs.hip
// (verifySignatureSets batches, multi-GPU partials).
#pragma once
#include "../../include/gbv.h"
#include "launch.h"
#include "kernel_common.h"

#include <sys/random.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

namespace gbv {

constexpr uint32_t MAX_SIGNATURE_SETS_PER_JOB = 128;  // multithread/index.ts:56
constexpr int TPB = 64;

// chunkifyMaximizeChunkSize (multithread/utils.ts:4-18): returns chunk start offsets + end.
inline std::vector<uint32_t> chunk_offsets(uint32_t len, uint32_t min_per_chunk) {
  std::vector<uint32_t> off;
  uint32_t chunk_count = len / min_per_chunk;
  if (chunk_count <= 1) {
    off.push_back(0);
    off.push_back(len);
    return off;
  }
  uint32_t per_chunk = (len + chunk_count - 1) / chunk_count;
  for (uint32_t i = 0; i < len; i += per_chunk) off.push_back(i);
  off.push_back(len);
  return off;
}

inline unsigned blocks_for(size_t n, int tpb = TPB) { return (unsigned)((n + tpb - 1) / tpb); }

// Entries written by launch_seg_reduce_quad for n items: every level of 64-way
// reductions is stored until 4 or fewer partials remain (ceil(n/64) + ceil(ceil(n/64)/64) + ...).
inline size_t seg_reduce_scratch(size_t n) {
  size_t total = 0, m = (n + 63) / 64;
  total += m;
  while (m > 4) {
    m = (m + 63) / 64;
    total += m;
  }
  return total + 4;
}

inline Seed fresh_seed() {
  Seed s;
  size_t got = 0;
  while (got < sizeof(s.w)) {
    ssize_t r = getrandom((uint8_t*)s.w + got, sizeof(s.w) - got, 0);
    if (r > 0) got += (size_t)r;
  }
  return s;
}

template <class T> inline hipError_t dalloc(T** p, size_t count) {
  return hipMalloc((void**)p, std::max<size_t>(count, 1) * sizeof(T));
}

// Fp is a 12 x u32 ext_vector (64-byte slots in memory); the C ABI's Fp12 blobs are packed to
// 12 x 48 bytes of little-endian limbs.
inline void fp12_pack(uint8_t* out576, const Fp12& a) {
  const Fp* f = (const Fp*)&a;
  for (int i = 0; i < 12; ++i) memcpy(out576 + 48 * i, &f[i], 48);
}
inline Fp12 fp12_unpack(const uint8_t* in576) {
  Fp12 r;
  memset((void*)&r, 0, sizeof(r));
  Fp* f = (Fp*)&r;
  for (int i = 0; i < 12; ++i) memcpy(&f[i], in576 + 48 * i, 48);
  return r;
}
// "name grid_threads units ms" per kernel of a waited pass (gbv_last_ops); every event of the pass
// has completed once its done event has
inline std::string kprof_format(KProf& p) {
  std::string out;
  char line[160];
  for (const KRec& r : p.recs) {
    float ms = 0.f;
    if (hipEventSynchronize(r.b) != hipSuccess || hipEventElapsedTime(&ms, r.a, r.b) != hipSuccess) {
      (void)hipGetLastError();
      ms = -1.f;
    }
    snprintf(line, sizeof line, "%s %u %u %.4f\n", r.name, r.threads, r.units, ms);
    out += line;
  }
  return out;
}

// Sets t_kprof for the enqueue routine that holds it (nothing recorded when p is null).
struct KProfScope {
  explicit KProfScope(KProf* p) {
    if (p) p->reset();
    t_kprof = p;
  }
  ~KProfScope() { t_kprof = nullptr; }
};

inline Fp12 fp12_one_host() {
  Fp12 r;
  memset((void*)&r, 0, sizeof(r));
  r.c0.c0.c0 = FP_ONE;
  return r;
}

}  // namespace gbv

struct gbv_vs_batch;
struct gbv_sm_batch;

struct gbv_ctx {
  int device = 0;
  // stream A (per-set throughput kernels) at the lowest priority; the tail stream 2 (chunk-level
  // latency-bound work), the hash stream 4 and stream 5 at the highest.  Stream 5 carries the
  // signature half of small verifySignatureSets passes and, in the invalid-dense same-message regime,
  // every other batch's failure path (the hash then runs on stream A).  Five streams exist per context
  // (with stream 6 below) over GPU_MAX_HW_QUEUES=4 hardware queues, so the runtime maps two of them to
  // one queue; the same-message and verifySignatureSets paths keep at most four busy at once.
  hipStream_t stream = nullptr, stream2 = nullptr, stream4 = nullptr;
  hipStream_t stream5 = nullptr;
  // gbv_fp12_check: the multi-GPU exchange's final check, beside streamed shard passes.  Shard passes
  // use streams A, 2 / 4 and 5, so stream 6 shares a hardware queue with one of them: the check can
  // still queue behind that stream's kernels of the next pass.  Measured (kernel trace of 16 streamed
  // passes, profiles/r06/fp12trace/overlap.txt): 17 of 23 checks ran beside the next pass's kernels
  // (the others: the warm-up and lone passes, nothing queued), ~1.1 ms each.
  hipStream_t stream6 = nullptr;
  gbv::G1A* table = nullptr;
  uint8_t* table_ok = nullptr;
  size_t table_cap = 0;
  std::atomic<size_t> table_n{0};  // read without the lock (gbv_pubkeys_count), written under it
  // per-slot comb tables for r pk (curve.h comb_mul; 128 affine entries = 12 KB per slot), built on
  // append / replicate; comb_on = false (gbv_tune "comb" 0, or an allocation that failed) -> the ladder
  uint4* comb = nullptr;
  uint8_t* comb_ok = nullptr;
  size_t comb_cap = 0;
  bool comb_on = true;
  std::string err;
  uint32_t nonce = 0;
  uint32_t sm_submits = 0;  // batches submitted (statistics)
  // A failing MSM segment pays the per-set G2 terms after all (k_sm_redo_g2) on top of the MSM, so
  // after one the next MSM_COOLDOWN submits use the per-set ladders (invalid-dense streams, C5)
  uint32_t msm_cooldown = 0;
  // Per-context settings (defaults at gbv_init), changed only by gbv_tune ("msm_min", "msm_cooldown",
  // "segments"): segments of at least msm_min sets form their G2 sum with the bucket MSM (k_msm.hip;
  // 0 = never); a failing MSM segment starts a cooldown of msm_cooldown_len submits; a batch is cut
  // into at most `segments` pipeline segments (tests use several on small batches)
  uint32_t msm_min = 131072, msm_cooldown_len = 16, segments = 1;
  static constexpr int NK = 8;  // hash, prepare, chunk_reduce, miller, seg_check, group_pairing, fallback, msm
  float last_ms[NK] = {};
  int last_launches[NK] = {};
  uint32_t last_fallback_chunks = 0, last_failed_segments = 0;
  bool closed = false;
  // one-shot calls (gbv_verify_same_message[_multi], gbv_verify_sets[_multi], gbv_vs_partial)
  // reuse these device-resident batches, grown on demand: no hipMalloc / hipFree per call
  gbv_sm_batch* sm_scratch = nullptr;
  gbv_vs_batch* vs_scratch = nullptr;
  // small device/pinned scratch for the table / aggregate / fp12 entry points (grow-only)
  uint8_t* small_dev = nullptr;
  size_t small_dev_cap = 0;
  uint8_t* small_host = nullptr;  // pinned
  size_t small_host_cap = 0;
  // signing-root (SSZ) calls: grow-only device buffers [input, output, domains, domain indices]
  uint8_t* ssz_buf[4] = {};
  size_t ssz_cap[4] = {};
  hipEvent_t ssz_ev[2] = {};
  float last_ssz_ms = 0.f;
  float last_vs_ms[4] = {};  // agg, hash+sig, miller, chunk check of the last vs batch
  // per-kernel timing of every pass (gbv_tune "kprof"; off by default: two events per kernel) and the
  // last waited pass of each path (gbv_last_ops: 0 same-message, 1 verifySignatureSets / partials)
  bool kprof_on = false;
  std::string last_ops[2];
  // Every entry point holds this while it touches the context (its streams, table, counters), so
  // host threads may share a context: the Python verifier's worker threads and its event-loop
  // thread, the addon's libuv pool.  Recursive: a fill nests inside a one-shot call.  No entry point
  // holds it while it blocks on the device: the batch waits and the one-shot calls (which hold
  // their scratch batch's own mutex instead) wait on an event without it.
  std::recursive_mutex mu;
  // The one-shot calls' scratch batches, each owned by one call at a time.  Lock order: a scratch
  // mutex first, then mu.
  std::mutex sm_scratch_mu, vs_scratch_mu;
};

#define GBV_LOCK(c) std::lock_guard<std::recursive_mutex> gbv_lock_((c)->mu)

// Synchronise the context's streams, ignoring errors: an enqueue that failed midway leaves
// nothing queued that could still read buffers the caller is about to free or refill.
void ctx_drain(gbv_ctx* c);

int gbv_fail(gbv_ctx* c, int code, const std::string& msg);

#define HIP_CHECK(ctx, call)                                                                 \
  do {                                                                                       \
    hipError_t e_ = (call);                                                                  \
    if (e_ != hipSuccess)                                                                    \
      return gbv_fail(ctx, GBV_E_DEVICE, std::string(#call) + ": " + hipGetErrorString(e_)); \
  } while (0)

// HIP_CHECK for calls made after kernels were enqueued: drain the streams before returning
#define HIP_CHECK_DRAIN(ctx, call)                                                           \
  do {                                                                                       \
    hipError_t e_ = (call);                                                                  \
    if (e_ != hipSuccess) {                                                                  \
      ctx_drain(ctx);                                                                        \
      return gbv_fail(ctx, GBV_E_DEVICE, std::string(#call) + ": " + hipGetErrorString(e_)); \
    }                                                                                        \
  } while (0)

// grow-only small scratch (device / pinned host) owned by the context
int ctx_small_dev(gbv_ctx* c, size_t bytes, uint8_t** out);
int ctx_small_host(gbv_ctx* c, size_t bytes, uint8_t** out);
// released by gbv_destroy (defined in gbv_vs.hip)
void vs_batch_free(gbv_vs_batch* b);
