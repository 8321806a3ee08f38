// Host side of the C ABI (include/gbv.h): device memory, the HBM pubkey table, chunking exactly
// as the reference pool does it, kernel sequencing on one HIP stream per context.
#include "../../include/gbv.h"
#include "launch.h"
#include "kernel_common.h"

#include <sys/random.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

using namespace gbv;

namespace {

constexpr uint32_t MAX_SIGNATURE_SETS_PER_JOB = 128;  // multithread/index.ts:56
constexpr int TPB = 64;
constexpr unsigned FB_GRID = 2048;  // persistent failure-path grids: 2 waves per SIMD
// a failing segment with at least this many chunks checks them one thread each (throughput), below
// it one wave each (latency); see k_sm_group_check / k_sm_group_pairing
constexpr uint32_t GROUP_CHECK_THREAD_MIN = 512;
// segments of at most this many chunks skip the combined segment check (latency of small calls)
constexpr uint32_t DIRECT_CHUNK_MAX = 32;
// segments of at least this many sets form their G2 sum sum r_i sig_i with the bucket MSM
// (k_msm.hip) instead of per-set ladders; GBV_MSM_MIN overrides (0 = never)
constexpr uint32_t MSM_MIN_SETS = 131072;
constexpr uint32_t MSM_COOLDOWN = 16;

// chunkifyMaximizeChunkSize (multithread/utils.ts:4-18): returns chunk start offsets + end.
std::vector<uint32_t> chunk_offsets(uint32_t len, uint32_t min_per_chunk) {
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

unsigned blocks_for(size_t n, int tpb = TPB) { return (unsigned)((n + tpb - 1) / tpb); }

}  // namespace

struct gbv_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  G1A* table = nullptr;
  uint8_t* table_ok = nullptr;
  size_t table_cap = 0;
  size_t table_n = 0;
  std::string err;
  uint32_t nonce = 0;
  hipStream_t stream2 = nullptr, stream3 = nullptr, stream4 = nullptr;
  uint32_t sm_submits = 0;  // parity picks which of stream2/stream3 carries a batch's chunk tail
  // A failing MSM segment pays the per-set G2 terms after all (k_sm_redo_g2) on top of the MSM, so
  // after one the next MSM_COOLDOWN submits use the per-set ladders (invalid-dense streams, C5)
  uint32_t msm_cooldown = 0;
  std::vector<hipEvent_t> events;
  static constexpr int NK = 8;  // hash, prepare, chunk_reduce, miller, seg_check, group_pairing, fallback, msm
  float last_ms[NK] = {};
  int last_launches[NK] = {};
  uint32_t last_fallback_chunks = 0, last_failed_segments = 0;
  bool closed = false;
  // signing-root (SSZ) calls: grow-only device buffers [input, output, domains, domain indices]
  uint8_t* ssz_buf[4] = {};
  size_t ssz_cap[4] = {};
  hipEvent_t ssz_ev[2] = {};
  float last_ssz_ms = 0.f;
};

struct gbv_sm_batch {
  size_t n = 0, G = 0, n_calls = 0;
  std::vector<uint32_t> grp_off_host;
  uint32_t *idx = nullptr, *grp_off = nullptr, *grp_msg = nullptr, *set_grp = nullptr, *n_fallback = nullptr;
  uint8_t *sig = nullptr, *msgs = nullptr, *status = nullptr, *grp_state = nullptr, *valid = nullptr, *seg_ok = nullptr;
  uint8_t* seg_ok_host = nullptr;  // pinned
  uint8_t* valid_host = nullptr;   // pinned, n bytes: results of the last submitted verify
  uint32_t* nfb_host = nullptr;    // pinned: fallback chunk count of the last submitted verify
  size_t seg_cap = 0;
  std::vector<uint8_t> seg_direct = std::vector<uint8_t>(64);  // per segment: combined check skipped
  // in-flight state of the last gbv_sm_batch_submit
  bool in_flight = false;
  size_t n_seg = 0;
  // two event sets, one per tail stream (gbv_ctx::sm_submits parity): an event is only ever
  // recorded on one stream
  std::vector<hipEvent_t> evs[2];
  hipEvent_t dones[2] = {};
  int cur = 0;  // event set of the last submit
  G2A *H = nullptr, *S = nullptr;
  G2J *rS = nullptr, *SgJ = nullptr;
  Fp12* F = nullptr;
  Fp12* Fpart = nullptr;  // per 64-chunk block partials of a segment (reused segment after segment)
  G2J* Spart = nullptr;
  uint8_t* has = nullptr;
  G1J* rP = nullptr;
  G1J* PgJ = nullptr;
  // failure path lists: runs of failed chunks (head, end, chunk), then sets of failing runs
  uint4* fb_runs = nullptr;
  uint32_t* fb_list = nullptr;
  uint32_t* fb_cnt = nullptr;  // [runs, listed sets]
  size_t fb_cap = 0;
  // bucket MSM scratch (allocated on the first submit that uses it): two sets, by segment parity
  uint32_t *msm_cnt[2] = {}, *msm_off[2] = {}, *msm_cur[2] = {};
  G2J *msm_buckets[2] = {}, *msm_part[2] = {}, *msm_head[2] = {}, *msm_tail[2] = {};
  uint32_t* msm_ent = nullptr;  // 4 per set, segment s at 4 * s0
  G2J* msm_total = nullptr;     // one per segment
  std::vector<uint8_t> seg_msm = std::vector<uint8_t>(64);
};

static size_t msm_min_sets() { return getenv("GBV_MSM_MIN") ? (size_t)atol(getenv("GBV_MSM_MIN")) : MSM_MIN_SETS; }

template <class T> static hipError_t dalloc(T** p, size_t count);

static hipError_t msm_alloc(gbv_sm_batch* b) {
  hipError_t e = hipSuccess;
  auto chk = [&](hipError_t x) { if (x != hipSuccess && e == hipSuccess) e = x; };
  for (int k = 0; k < 2; ++k) {
    chk(dalloc(&b->msm_cnt[k], MSM_KEYS)); chk(dalloc(&b->msm_off[k], MSM_KEYS)); chk(dalloc(&b->msm_cur[k], MSM_KEYS));
    chk(dalloc(&b->msm_buckets[k], MSM_KEYS)); chk(dalloc(&b->msm_part[k], MSM_PARTS + 130));
    chk(dalloc(&b->msm_head[k], 4 * b->n / MSM_RUN + 64)); chk(dalloc(&b->msm_tail[k], 4 * b->n / MSM_RUN + 64));
  }
  chk(dalloc(&b->msm_ent, 4 * b->n)); chk(dalloc(&b->msm_total, b->seg_cap));
  return e;
}

static int fail(gbv_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

#define HIP_CHECK(ctx, call)                                                             \
  do {                                                                                   \
    hipError_t e_ = (call);                                                              \
    if (e_ != hipSuccess)                                                                \
      return fail(ctx, GBV_E_DEVICE, std::string(#call) + ": " + hipGetErrorString(e_)); \
  } while (0)

template <class T> static hipError_t dalloc(T** p, size_t count) {
  return hipMalloc((void**)p, std::max<size_t>(count, 1) * sizeof(T));
}

// Fp is a 12 x u32 ext_vector (64-byte slots in memory); the C ABI's Fp12 blobs are packed to
// 12 x 48 bytes of little-endian limbs.
static void fp12_pack(uint8_t* out576, const Fp12& a) {
  const Fp* f = (const Fp*)&a;
  for (int i = 0; i < 12; ++i) memcpy(out576 + 48 * i, &f[i], 48);
}
static Fp12 fp12_unpack(const uint8_t* in576) {
  Fp12 r;
  memset(&r, 0, sizeof(r));
  Fp* f = (Fp*)&r;
  for (int i = 0; i < 12; ++i) memcpy(&f[i], in576 + 48 * i, 48);
  return r;
}

static Fp12 fp12_one_host() {
  Fp12 r;
  memset(&r, 0, sizeof(r));
  r.c0.c0.c0 = FP_ONE;
  return r;
}

static Seed fresh_seed() {
  Seed s;
  size_t got = 0;
  while (got < sizeof(s.w)) {
    ssize_t r = getrandom((uint8_t*)s.w + got, sizeof(s.w) - got, 0);
    if (r > 0) got += (size_t)r;
  }
  return s;
}

namespace gbv {
void debug_sync(hipStream_t s, const char* kernel) {
  static int on = getenv("GBV_SYNC_DEBUG") ? atoi(getenv("GBV_SYNC_DEBUG")) : 0;
  if (!on) return;
  hipError_t e = hipStreamSynchronize(s);
  if (e == hipSuccess) e = hipGetLastError();
  fprintf(stderr, "[gbv] %s: %s\n", kernel, hipGetErrorString(e));
}
}  // namespace gbv

extern "C" {

int gbv_init(int device, gbv_ctx** out) {
  if (!out) return GBV_E_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return GBV_E_DEVICE;
  if (device < 0 || device >= ndev) return GBV_E_ARG;
  gbv_ctx* c = new gbv_ctx();
  c->device = device;
  // stream A (k_sm_prepare, throughput) at the lowest priority, the latency-bound chunk tails, hash
  // and MSM streams at the highest: their few waves then dispatch ahead of k_sm_prepare's
  int prio_lo = 0, prio_hi = 0;
  if (hipSetDevice(device) != hipSuccess || hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi) != hipSuccess ||
      hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, prio_lo) != hipSuccess) {
    delete c;
    return GBV_E_DEVICE;
  }
  if (hipStreamCreateWithPriority(&c->stream2, hipStreamNonBlocking, prio_hi) != hipSuccess ||
      hipStreamCreateWithPriority(&c->stream3, hipStreamNonBlocking, prio_hi) != hipSuccess ||
      hipStreamCreateWithPriority(&c->stream4, hipStreamNonBlocking, prio_hi) != hipSuccess) {
    hipStreamDestroy(c->stream);
    if (c->stream2) hipStreamDestroy(c->stream2);
  if (c->stream3) hipStreamDestroy(c->stream3);
  if (c->stream4) hipStreamDestroy(c->stream4);
    delete c;
    return GBV_E_DEVICE;
  }
  *out = c;
  return GBV_OK;
}

void gbv_destroy(gbv_ctx* c) {
  if (!c) return;
  hipSetDevice(c->device);
  if (c->stream) hipStreamSynchronize(c->stream);
  hipFree(c->table);
  hipFree(c->table_ok);
  for (auto* p : c->ssz_buf) hipFree(p);
  for (auto e : c->ssz_ev)
    if (e) hipEventDestroy(e);
  if (c->stream2) hipStreamSynchronize(c->stream2);
  if (c->stream3) hipStreamSynchronize(c->stream3);
  if (c->stream4) hipStreamSynchronize(c->stream4);
  for (auto& e : c->events) hipEventDestroy(e);
  if (c->stream) hipStreamDestroy(c->stream);
  if (c->stream2) hipStreamDestroy(c->stream2);
  if (c->stream3) hipStreamDestroy(c->stream3);
  if (c->stream4) hipStreamDestroy(c->stream4);
  delete c;
}

const char* gbv_last_error(gbv_ctx* c) { return c ? c->err.c_str() : "null context"; }

size_t gbv_pubkeys_count(gbv_ctx* c) { return c ? c->table_n : 0; }

static int table_reserve(gbv_ctx* c, size_t need) {
  if (need <= c->table_cap) return GBV_OK;
  size_t cap = std::max(need, c->table_cap * 2);
  G1A* t = nullptr;
  uint8_t* ok = nullptr;
  HIP_CHECK(c, dalloc(&t, cap));
  HIP_CHECK(c, dalloc(&ok, cap));
  HIP_CHECK(c, hipMemsetAsync(ok, 0, cap, c->stream));
  if (c->table_n) {
    HIP_CHECK(c, hipMemcpyAsync(t, c->table, c->table_n * sizeof(G1A), hipMemcpyDeviceToDevice, c->stream));
    HIP_CHECK(c, hipMemcpyAsync(ok, c->table_ok, c->table_n, hipMemcpyDeviceToDevice, c->stream));
  }
  HIP_CHECK(c, hipStreamSynchronize(c->stream));
  hipFree(c->table);
  hipFree(c->table_ok);
  c->table = t;
  c->table_ok = ok;
  c->table_cap = cap;
  return GBV_OK;
}

int gbv_pubkeys_append(gbv_ctx* c, uint32_t first, const uint8_t* pk48, size_t n, int validate, uint8_t* status) {
  if (!c) return GBV_E_ARG;
  if (c->closed) return GBV_E_CLOSED;
  if (n == 0) return GBV_OK;
  if (!pk48) return fail(c, GBV_E_ARG, "null pk48");
  HIP_CHECK(c, hipSetDevice(c->device));
  int rc = table_reserve(c, (size_t)first + n);
  if (rc) return rc;
  uint8_t *d_pk = nullptr, *d_st = nullptr;
  HIP_CHECK(c, dalloc(&d_pk, 48 * n));
  HIP_CHECK(c, dalloc(&d_st, n));
  HIP_CHECK(c, hipMemcpyAsync(d_pk, pk48, 48 * n, hipMemcpyHostToDevice, c->stream));
  launch_pk_decompress(LaunchCfg{blocks_for(n), TPB, c->stream}, (uint32_t)n, d_pk, validate,
                     c->table + first, c->table_ok + first, d_st);
  HIP_CHECK(c, hipGetLastError());
  if (status) HIP_CHECK(c, hipMemcpyAsync(status, d_st, n, hipMemcpyDeviceToHost, c->stream));
  HIP_CHECK(c, hipStreamSynchronize(c->stream));
  hipFree(d_pk);
  hipFree(d_st);
  c->table_n = std::max(c->table_n, (size_t)first + n);
  return GBV_OK;
}

int gbv_pubkeys_replicate(gbv_ctx* c, uint32_t src_first, uint32_t src_n, uint32_t dst_first, size_t n) {
  if (!c || src_n == 0 || (size_t)src_first + src_n > c->table_n) return fail(c, GBV_E_ARG, "bad replicate range");
  HIP_CHECK(c, hipSetDevice(c->device));
  int rc = table_reserve(c, (size_t)dst_first + n);
  if (rc) return rc;
  launch_pk_replicate(LaunchCfg{blocks_for(n, 256), 256, c->stream}, c->table, c->table_ok, src_first, src_n,
                     dst_first, (uint32_t)n);
  HIP_CHECK(c, hipGetLastError());
  HIP_CHECK(c, hipStreamSynchronize(c->stream));
  c->table_n = std::max(c->table_n, (size_t)dst_first + n);
  return GBV_OK;
}

int gbv_aggregate_pubkeys(gbv_ctx* c, const uint32_t* idx, size_t k, uint8_t out48[48]) {
  if (!c) return GBV_E_ARG;
  if (c->closed) return GBV_E_CLOSED;
  if (k == 0) return fail(c, GBV_E_EMPTY_AGGREGATE, "EMPTY_AGGREGATE_ARRAY");
  if (!idx || !out48) return fail(c, GBV_E_ARG, "null argument");
  for (size_t i = 0; i < k; ++i)
    if (idx[i] >= c->table_n) return fail(c, GBV_E_ARG, "validator index out of range");
  HIP_CHECK(c, hipSetDevice(c->device));
  uint32_t *d_idx = nullptr, *d_bad = nullptr;
  uint8_t* d_out = nullptr;
  HIP_CHECK(c, dalloc(&d_idx, k));
  HIP_CHECK(c, dalloc(&d_bad, 1));
  HIP_CHECK(c, dalloc(&d_out, 48));
  HIP_CHECK(c, hipMemcpyAsync(d_idx, idx, 4 * k, hipMemcpyHostToDevice, c->stream));
  HIP_CHECK(c, hipMemsetAsync(d_bad, 0, 4, c->stream));
  launch_aggregate(LaunchCfg{1, 256, c->stream}, d_idx, (uint32_t)k, c->table, c->table_ok, d_out, d_bad);
  HIP_CHECK(c, hipGetLastError());
  uint32_t bad = 0;
  HIP_CHECK(c, hipMemcpyAsync(out48, d_out, 48, hipMemcpyDeviceToHost, c->stream));
  HIP_CHECK(c, hipMemcpyAsync(&bad, d_bad, 4, hipMemcpyDeviceToHost, c->stream));
  HIP_CHECK(c, hipStreamSynchronize(c->stream));
  hipFree(d_idx);
  hipFree(d_bad);
  hipFree(d_out);
  if (bad) return fail(c, GBV_E_ARG, "aggregate over an invalid table entry");
  return GBV_OK;
}

// ---- same-message batches ------------------------------------------------------------------
void gbv_sm_batch_destroy(gbv_ctx* c, gbv_sm_batch* b) {
  (void)c;
  if (!b) return;
  hipFree(b->idx); hipFree(b->grp_off); hipFree(b->grp_msg); hipFree(b->set_grp); hipFree(b->n_fallback);
  hipFree(b->sig); hipFree(b->msgs); hipFree(b->status); hipFree(b->grp_state); hipFree(b->valid);
  hipFree(b->H); hipFree(b->S); hipFree(b->SgJ); hipFree(b->rS); hipFree(b->rP); hipFree(b->PgJ);
  if (b->in_flight && b->dones[b->cur]) hipEventSynchronize(b->dones[b->cur]);
  for (int k = 0; k < 2; ++k) {
    for (auto& e : b->evs[k]) hipEventDestroy(e);
    if (b->dones[k]) hipEventDestroy(b->dones[k]);
  }
  hipHostFree(b->valid_host);
  hipHostFree(b->nfb_host);
  hipFree(b->F); hipFree(b->seg_ok); hipHostFree(b->seg_ok_host);
  hipFree(b->Fpart); hipFree(b->Spart); hipFree(b->has);
  hipFree(b->fb_runs); hipFree(b->fb_list); hipFree(b->fb_cnt);
  for (int k = 0; k < 2; ++k) {
    hipFree(b->msm_cnt[k]); hipFree(b->msm_off[k]); hipFree(b->msm_cur[k]); hipFree(b->msm_buckets[k]); hipFree(b->msm_part[k]);
    hipFree(b->msm_head[k]); hipFree(b->msm_tail[k]);
  }
  hipFree(b->msm_ent); hipFree(b->msm_total);
  delete b;
}

int gbv_sm_batch_create(gbv_ctx* c, size_t n_calls, const uint32_t* call_off, const uint32_t* idx, const uint8_t* sigs96,
                        const uint8_t* msgs32, gbv_sm_batch** out) {
  if (!c || !out) return GBV_E_ARG;
  if (c->closed) return GBV_E_CLOSED;
  *out = nullptr;
  if (n_calls && (!call_off || !msgs32)) return fail(c, GBV_E_ARG, "null argument");
  size_t n = n_calls ? call_off[n_calls] : 0;
  if (n && (!idx || !sigs96)) return fail(c, GBV_E_ARG, "null argument");
  for (size_t g = 0; g < n_calls; ++g)
    if (call_off[g + 1] < call_off[g]) return fail(c, GBV_E_ARG, "call offsets not monotone");
  for (size_t i = 0; i < n; ++i)
    if (idx[i] >= c->table_n) return fail(c, GBV_E_ARG, "validator index out of range");
  // chunk every call exactly like verifySignatureSetsSameMessage (index.ts:218-219)
  std::vector<uint32_t> grp_off, grp_msg, set_grp(n);
  for (size_t g = 0; g < n_calls; ++g) {
    uint32_t len = call_off[g + 1] - call_off[g];
    if (len == 0) continue;
    std::vector<uint32_t> co = chunk_offsets(len, MAX_SIGNATURE_SETS_PER_JOB);
    for (size_t j = 0; j + 1 < co.size(); ++j) {
      uint32_t gid = (uint32_t)grp_msg.size();
      grp_off.push_back(call_off[g] + co[j]);
      grp_msg.push_back((uint32_t)g);
      for (uint32_t i = call_off[g] + co[j]; i < call_off[g] + co[j + 1]; ++i) set_grp[i] = gid;
    }
  }
  grp_off.push_back((uint32_t)n);
  size_t G = grp_msg.size();
  HIP_CHECK(c, hipSetDevice(c->device));
  gbv_sm_batch* b = new gbv_sm_batch();
  b->n = n;
  b->G = G;
  b->n_calls = n_calls;
  b->grp_off_host = grp_off;
  hipError_t e = hipSuccess;
  auto chk = [&](hipError_t x) { if (x != hipSuccess && e == hipSuccess) e = x; };
  chk(dalloc(&b->idx, n)); chk(dalloc(&b->sig, 96 * n)); chk(dalloc(&b->grp_off, G + 1)); chk(dalloc(&b->grp_msg, G));
  chk(dalloc(&b->set_grp, n)); chk(dalloc(&b->msgs, 32 * n_calls)); chk(dalloc(&b->n_fallback, 1));
  chk(dalloc(&b->status, n)); chk(dalloc(&b->grp_state, G)); chk(dalloc(&b->valid, n));
  chk(dalloc(&b->H, n_calls)); chk(dalloc(&b->S, n)); chk(dalloc(&b->rS, n)); chk(dalloc(&b->rP, n));
  chk(dalloc(&b->PgJ, G)); chk(dalloc(&b->SgJ, G)); chk(dalloc(&b->F, G));
  // block partials: one region per segment stream (two segments' reductions can be in flight)
  chk(dalloc(&b->Fpart, 2 * (G / 64 + G / 4096 + 4))); chk(dalloc(&b->Spart, 2 * (G / 64 + G / 4096 + 4)));
  chk(dalloc(&b->has, 2 * (G / 64 + G / 4096 + 4)));
  b->fb_cap = n / 8 + G + 64;  // runs: at most one per 8-set window plus one per chunk start
  chk(dalloc(&b->fb_runs, b->fb_cap)); chk(dalloc(&b->fb_list, n)); chk(dalloc(&b->fb_cnt, 2));
  b->seg_cap = 64;
  chk(dalloc(&b->seg_ok, b->seg_cap));
  chk(hipHostMalloc((void**)&b->seg_ok_host, b->seg_cap, hipHostMallocDefault));
  chk(hipHostMalloc((void**)&b->valid_host, std::max<size_t>(n, 1), hipHostMallocDefault));
  chk(hipHostMalloc((void**)&b->nfb_host, sizeof(uint32_t), hipHostMallocDefault));
  chk(hipEventCreateWithFlags(&b->dones[0], hipEventDisableTiming));
  chk(hipEventCreateWithFlags(&b->dones[1], hipEventDisableTiming));
  if (msm_min_sets() && n >= msm_min_sets()) chk(msm_alloc(b));
  if (e != hipSuccess) {
    gbv_sm_batch_destroy(c, b);
    return fail(c, GBV_E_OOM, std::string("hipMalloc: ") + hipGetErrorString(e));
  }
  if (n) {
    chk(hipMemcpyAsync(b->idx, idx, 4 * n, hipMemcpyHostToDevice, c->stream));
    chk(hipMemcpyAsync(b->sig, sigs96, 96 * n, hipMemcpyHostToDevice, c->stream));
    chk(hipMemcpyAsync(b->set_grp, set_grp.data(), 4 * n, hipMemcpyHostToDevice, c->stream));
  }
  chk(hipMemcpyAsync(b->grp_off, grp_off.data(), 4 * (G + 1), hipMemcpyHostToDevice, c->stream));
  if (G) chk(hipMemcpyAsync(b->grp_msg, grp_msg.data(), 4 * G, hipMemcpyHostToDevice, c->stream));
  if (n_calls) chk(hipMemcpyAsync(b->msgs, msgs32, 32 * n_calls, hipMemcpyHostToDevice, c->stream));
  chk(hipStreamSynchronize(c->stream));
  if (e != hipSuccess) {
    gbv_sm_batch_destroy(c, b);
    return fail(c, GBV_E_DEVICE, std::string("upload: ") + hipGetErrorString(e));
  }
  *out = b;
  return GBV_OK;
}

// Pipelined over segments of ~n/S sets (cut at chunk boundaries), all enqueued without a host
// round trip so consecutive submits overlap (the chunk-level tail of batch k runs beside the
// throughput-bound k_sm_prepare of batch k+1):
//   stream H      : k_hash_msgs
//   stream A      : k_sm_prepare(segment s)  -- throughput-bound, also forms per-wave chunk sums
//   streams B0/B1 : (segment s alternates) wait(prepare s, hash) k_sm_chunk_finish, k_sm_miller,
//                   k_sm_seg_reduce + k_sm_seg_check, k_sm_group_pairing (exits at once unless
//                   the segment check failed)
//   stream B0     : wait(all) k_sm_fallback (per-set retry of failed chunks only), copy-out
// Each segment ends in ONE randomised multi-pairing check over all its chunks; only a failing
// segment pays per-chunk checks and only a failing chunk pays per-set retries.
int gbv_sm_batch_submit(gbv_ctx* c, gbv_sm_batch* b) {
  if (!c || !b) return GBV_E_ARG;
  if (c->closed) return GBV_E_CLOSED;
  if (b->in_flight) return fail(c, GBV_E_ARG, "batch already in flight");
  HIP_CHECK(c, hipSetDevice(c->device));
  if (b->n == 0) return GBV_OK;
  Seed seed = fresh_seed();
  uint32_t nonce = c->nonce++;
  // consecutive batches put their chunk-level tails on different streams, so that the tail of
  // batch k and of batch k+1 overlap (each beside the next batch's k_sm_prepare on stream A)
  // GBV_FLIP=1: alternate the tail stream per batch (lets consecutive tails overlap, but together
  // with the MSM launches it stalled the device for seconds at a time on ROCm 7.2 -- off by default)
  static const bool use_flip = getenv("GBV_FLIP") != nullptr;
  const bool flip = use_flip && (c->sm_submits++ & 1) != 0;
  hipStream_t sa = c->stream, sh = c->stream4;
  hipStream_t sbs[2] = {flip ? c->stream3 : c->stream2, flip ? c->stream2 : c->stream3};
  const size_t max_seg = b->seg_cap;
  const size_t n_seg = getenv("GBV_SEGMENTS") ? (size_t)std::max(1, atoi(getenv("GBV_SEGMENTS"))) : 1;
  size_t sub_sets = std::max<size_t>((b->n + n_seg - 1) / n_seg, 16384);
  std::vector<uint32_t> gcut{0};
  {
    size_t next = sub_sets;
    for (size_t g = 1; g < b->G; ++g)
      if (b->grp_off_host[g] >= next && gcut.size() < max_seg) {
        gcut.push_back((uint32_t)g);
        next = b->grp_off_host[g] + sub_sets;
      }
  }
  gcut.push_back((uint32_t)b->G);
  size_t S = gcut.size() - 1;
  b->n_seg = S;
  const size_t msm_min = c->msm_cooldown ? 0 : msm_min_sets();
  if (c->msm_cooldown) --c->msm_cooldown;
  bool any_msm = false;
  for (size_t s = 0; s < S; ++s) {
    uint32_t G = gcut[s + 1] - gcut[s];
    size_t ns = b->grp_off_host[gcut[s + 1]] - b->grp_off_host[gcut[s]];
    b->seg_direct[s] = G <= DIRECT_CHUNK_MAX;
    b->seg_msm[s] = msm_min && ns >= msm_min && !b->seg_direct[s];
    any_msm |= b->seg_msm[s] != 0;
  }
  if (any_msm && !b->msm_ent) {  // normally allocated by gbv_sm_batch_create (no hipMalloc while work is queued)
    hipError_t e = msm_alloc(b);
    if (e != hipSuccess) return fail(c, GBV_E_OOM, std::string("hipMalloc (msm): ") + hipGetErrorString(e));
  }
  // events: [0,1] hash; per segment 13 (prep, finish, miller, check, group, msm, msm reduce done);
  // then [tail] 2 fallback
  constexpr size_t EPS = 13;
  size_t need = 2 + EPS * S + 2;
  b->cur = flip ? 1 : 0;
  std::vector<hipEvent_t>& evv = b->evs[b->cur];
  if (evv.size() < need) {
    size_t old = evv.size();
    evv.resize(need);
    for (size_t k = old; k < need; ++k) HIP_CHECK(c, hipEventCreateWithFlags(&evv[k], hipEventDefault));
  }
  hipEvent_t* ev = evv.data();
  const size_t part_stride = b->G / 64 + b->G / 4096 + 4;
  HIP_CHECK(c, hipMemsetAsync(b->n_fallback, 0, 4, sh));
  HIP_CHECK(c, hipMemsetAsync(b->fb_cnt, 0, 8, sh));
  hipEventRecord(ev[0], sh);
  launch_hash_msgs(LaunchCfg{blocks_for(b->n_calls), TPB, sh}, b->msgs, (uint32_t)b->n_calls, b->H);
  hipEventRecord(ev[1], sh);
  for (size_t s = 0; s < S; ++s) {
    hipEvent_t* e = ev + 2 + EPS * s;
    hipStream_t sb = sbs[s & 1];
    uint32_t g0 = gcut[s], G = gcut[s + 1] - gcut[s];
    uint32_t s0 = b->grp_off_host[g0], s1 = b->grp_off_host[gcut[s + 1]];
    const bool msm = b->seg_msm[s];
    G2J* Sh = msm ? nullptr : b->rS;  // MSM segment: k_sm_prepare forms the G1 terms only
    hipEventRecord(e[0], sa);
    launch_sm_prepare(LaunchCfg{0, 64, sa}, s0, s1 - s0, b->idx, b->sig, b->set_grp, c->table, c->table_ok, (uint32_t)c->table_n, seed,
                      nonce, b->S, Sh, b->rP, b->status);
    hipEventRecord(e[1], sa);
    // A segment of a few chunks (a lone gossip call) skips the combined check (seg_direct): each
    // chunk goes straight to its own one-wave check, which is the shorter dependency chain.
    // An MSM segment runs its chunk sums and the bucket MSM on stream A right after its
    // k_sm_prepare (the MSM's bucket pass then has the whole device instead of fighting the next
    // k_sm_prepare for CUs); the tail stream waits for them.  Other segments sum their chunks on
    // the tail stream.
    hipStream_t scf = msm ? sa : sb;
    if (!msm) HIP_CHECK(c, hipStreamWaitEvent(sb, e[1], 0));
    HIP_CHECK(c, hipStreamWaitEvent(scf, ev[1], 0));
    hipEventRecord(e[2], scf);
    launch_sm_chunk_finish(LaunchCfg{0, 64, scf}, g0, G, s0, b->grp_off, b->status, Sh, b->rP, b->PgJ, b->SgJ, b->grp_state,
                           b->n_fallback);
    hipEventRecord(e[3], scf);
    // the bucket pass runs on stream A (default) or, with GBV_MSM_STREAM=h, on the hash stream beside
    // the tail's Miller values
    static const bool msm_on_hash = getenv("GBV_MSM_STREAM") && getenv("GBV_MSM_STREAM")[0] == 'h';
    hipStream_t smsm = msm ? (msm_on_hash ? sh : sa) : scf;
    if (msm && msm_on_hash) HIP_CHECK(c, hipStreamWaitEvent(sh, e[3], 0));
    hipEventRecord(e[10], smsm);
    // segment s-2 shares this segment's bucket buffers: its reduction (tail stream) must be done
    if (msm && s >= 2 && b->seg_msm[s - 2]) HIP_CHECK(c, hipStreamWaitEvent(smsm, ev[2 + EPS * (s - 2) + 12], 0));
    if (msm)
      launch_msm_g2_buckets(smsm, s0, s1 - s0, b->set_grp, b->status, b->grp_state, b->S, seed, nonce, b->msm_cnt[s & 1], b->msm_off[s & 1],
                            b->msm_cur[s & 1], b->msm_ent + 4ull * s0, b->msm_buckets[s & 1], b->msm_head[s & 1], b->msm_tail[s & 1]);
    hipEventRecord(e[11], smsm);
    if (msm) HIP_CHECK(c, hipStreamWaitEvent(sb, e[3], 0));
    hipEventRecord(e[4], sb);
    if (!b->seg_direct[s]) launch_sm_miller(LaunchCfg{0, 64, sb}, g0, G, b->grp_msg, b->grp_state, b->PgJ, b->H, b->F);
    hipEventRecord(e[5], sb);
    if (msm) {  // the latency-bound bucket reduction overlaps the next k_sm_prepare
      HIP_CHECK(c, hipStreamWaitEvent(sb, e[11], 0));
      launch_msm_g2_reduce(sb, b->msm_buckets[s & 1], b->msm_part[s & 1], b->msm_total + s);
    }
    hipEventRecord(e[12], sb);
    hipEventRecord(e[6], sb);
    size_t po = (s & 1) * part_stride;
    if (b->seg_direct[s])
      HIP_CHECK(c, hipMemsetAsync(b->seg_ok + s, 0, 1, sb));
    else
      launch_sm_seg_check(LaunchCfg{1, 64, sb}, g0, G, b->grp_state, b->F, b->SgJ, b->Fpart + po, b->Spart + po, b->has + po,
                          b->seg_ok + s, nullptr, msm ? b->msm_total + s : nullptr);
    hipEventRecord(e[7], sb);
    hipEventRecord(e[8], sb);
    if (msm) {  // failure path of an MSM segment needs the per-set / per-chunk G2 sums (exit at once on pass)
      launch_sm_redo_g2(LaunchCfg{0, 64, sb}, s0, s1 - s0, b->set_grp, b->status, b->S, seed, nonce, b->seg_ok + s, b->rS);
      launch_sm_chunk_finish_s(LaunchCfg{0, 64, sb}, g0, G, s0, b->grp_off, b->grp_state, b->rS, b->seg_ok + s, b->SgJ);
    }
    if (G >= GROUP_CHECK_THREAD_MIN)
      launch_sm_group_check(LaunchCfg{0, 64, sb}, g0, G, b->F, b->SgJ, b->seg_ok + s, b->grp_state, b->n_fallback);
    else
      launch_sm_group_pairing(LaunchCfg{G, 64, sb}, g0, G, b->grp_msg, b->PgJ, b->SgJ, b->H, b->seg_ok + s, b->grp_state, b->n_fallback);
    hipEventRecord(e[9], sb);
  }
  hipEvent_t* ep = ev + 2 + EPS * S;
  // the tail runs on B0 after everything of this batch (B1's last segment included)
  if (S > 1) {
    size_t last_b1 = (S - 1) & 1 ? S - 1 : S - 2;  // last segment that ran on B1
    HIP_CHECK(c, hipStreamWaitEvent(sbs[0], ev[2 + EPS * last_b1 + 9], 0));
  }
  hipEventRecord(ep[0], sbs[0]);
  // valid = 1 for the sets of passing chunks; the sets of failed chunks go through 8-set run
  // checks and, for failing runs only, per-set checks (compacted lists, persistent grids)
  launch_sm_fallback(LaunchCfg{blocks_for(b->n), TPB, sbs[0]}, (uint32_t)b->n, b->set_grp, b->grp_msg, b->grp_state, b->status, b->idx,
                     c->table, b->S, b->H, b->valid, 0);
  for (size_t s = 0; s < S; ++s) {
    uint32_t s0 = b->grp_off_host[gcut[s]], s1 = b->grp_off_host[gcut[s + 1]];
    launch_sm_fb_runs(LaunchCfg{0, 64, sbs[0]}, s0, s1 - s0, b->set_grp, b->grp_state, b->fb_runs, b->fb_cnt, (uint32_t)b->fb_cap);
  }
  // few items: one wave each (latency); many: one thread each (throughput) -- one of each pair exits
  launch_sm_fb_blocks_coop(LaunchCfg{0, 64, sbs[0]}, b->fb_runs, b->fb_cnt, (uint32_t)b->fb_cap, b->status, b->grp_msg, b->rS, b->rP,
                           b->H, b->valid, b->fb_list, b->fb_cnt + 1);
  launch_sm_fb_blocks(LaunchCfg{FB_GRID, 64, sbs[0]}, b->fb_runs, b->fb_cnt, (uint32_t)b->fb_cap, b->status, b->grp_msg, b->rS, b->rP, b->H,
                      b->valid, b->fb_list, b->fb_cnt + 1);
  launch_sm_fb_sets_coop(LaunchCfg{0, 64, sbs[0]}, b->fb_list, b->fb_cnt + 1, b->set_grp, b->grp_msg, b->idx, c->table, b->S, b->H,
                         b->valid);
  launch_sm_fb_sets(LaunchCfg{FB_GRID, 64, sbs[0]}, b->fb_list, b->fb_cnt + 1, b->set_grp, b->grp_msg, b->idx, c->table, b->S, b->H,
                    b->valid);
  hipEventRecord(ep[1], sbs[0]);
  HIP_CHECK(c, hipMemcpyAsync(b->valid_host, b->valid, b->n, hipMemcpyDeviceToHost, sbs[0]));
  HIP_CHECK(c, hipMemcpyAsync(b->nfb_host, b->n_fallback, sizeof(uint32_t), hipMemcpyDeviceToHost, sbs[0]));
  HIP_CHECK(c, hipMemcpyAsync(b->seg_ok_host, b->seg_ok, S, hipMemcpyDeviceToHost, sbs[0]));
  HIP_CHECK(c, hipEventRecord(b->dones[b->cur], sbs[0]));
  HIP_CHECK(c, hipGetLastError());
  b->in_flight = true;
  return GBV_OK;
}

int gbv_sm_batch_wait(gbv_ctx* c, gbv_sm_batch* b, uint8_t* valid) {
  if (!c || !b) return GBV_E_ARG;
  if (b->n == 0) return GBV_OK;
  if (!b->in_flight) return fail(c, GBV_E_ARG, "batch not submitted");
  HIP_CHECK(c, hipSetDevice(c->device));
  b->in_flight = false;
  HIP_CHECK(c, hipEventSynchronize(b->dones[b->cur]));
  if (valid) memcpy(valid, b->valid_host, b->n);
  c->last_fallback_chunks = *b->nfb_host;
  c->last_failed_segments = 0;
  for (size_t s = 0; s < b->n_seg; ++s) {
    bool failed = !(b->seg_ok_host[s] || b->seg_direct[s]);
    c->last_failed_segments += failed ? 1 : 0;
    if (failed && b->seg_msm[s])
      c->msm_cooldown = getenv("GBV_MSM_COOLDOWN") ? (uint32_t)atoi(getenv("GBV_MSM_COOLDOWN")) : MSM_COOLDOWN;
  }
  for (auto& x : c->last_ms) x = 0.f;
  for (auto& x : c->last_launches) x = 0;
  hipEvent_t* ev = b->evs[b->cur].data();
  auto acc = [&](int k, hipEvent_t a0, hipEvent_t a1, bool count = true) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, a0, a1) == hipSuccess) {
      c->last_ms[k] += ms;
      c->last_launches[k] += count ? 1 : 0;
    }
  };
  acc(0, ev[0], ev[1]);
  for (size_t s = 0; s < b->n_seg; ++s) {
    hipEvent_t* e = ev + 2 + 13 * s;
    for (int k = 0; k < 5; ++k) acc(1 + k, e[2 * k], e[2 * k + 1]);
    if (b->seg_msm[s]) acc(7, e[10], e[11]);
  }
  hipEvent_t* ep = ev + 2 + 13 * b->n_seg;
  acc(6, ep[0], ep[1]);
  return GBV_OK;
}

int gbv_sm_batch_verify(gbv_ctx* c, gbv_sm_batch* b, uint8_t* valid) {
  int rc = gbv_sm_batch_submit(c, b);
  if (rc) return rc;
  return gbv_sm_batch_wait(c, b, valid);
}

int gbv_last_stats(gbv_ctx* c, uint32_t* fallback_chunks, uint32_t* failed_segments) {
  if (!c) return GBV_E_ARG;
  if (fallback_chunks) *fallback_chunks = c->last_fallback_chunks;
  if (failed_segments) *failed_segments = c->last_failed_segments;
  return GBV_OK;
}

int gbv_last_kernel_ms(gbv_ctx* c, float* out, int* launches, int max) {
  if (!c || !out) return 0;
  int k = std::min(max, (int)gbv_ctx::NK);
  for (int i = 0; i < k; ++i) {
    out[i] = c->last_ms[i];
    if (launches) launches[i] = c->last_launches[i];
  }
  return k;
}

int gbv_verify_same_message_multi(gbv_ctx* c, size_t n_calls, const uint32_t* call_off, const uint32_t* idx, const uint8_t* sigs96,
                                  const uint8_t* msgs32, uint8_t* valid) {
  gbv_sm_batch* b = nullptr;
  int rc = gbv_sm_batch_create(c, n_calls, call_off, idx, sigs96, msgs32, &b);
  if (rc) return rc;
  rc = gbv_sm_batch_verify(c, b, valid);
  gbv_sm_batch_destroy(c, b);
  return rc;
}

int gbv_verify_same_message(gbv_ctx* c, const uint32_t* idx, const uint8_t* sigs96, size_t n, const uint8_t* msg32, uint8_t* valid) {
  uint32_t off[2] = {0, (uint32_t)n};
  return gbv_verify_same_message_multi(c, 1, off, idx, sigs96, msg32, valid);
}

// ---- distinct-message sets -----------------------------------------------------------------
// Device buffers of one staged verifySignatureSets call after k_vs_prepare.
struct VsDev {
  uint32_t *off = nullptr, *idx = nullptr, *siglen = nullptr;
  uint8_t *raw_flag = nullptr, *raw_pk = nullptr, *msgs = nullptr, *sig = nullptr, *status = nullptr;
  Fp12* f = nullptr;
  G2J* rS = nullptr;
  void release() {
    hipFree(off); hipFree(idx); hipFree(siglen); hipFree(raw_flag); hipFree(raw_pk); hipFree(msgs); hipFree(sig);
    hipFree(status); hipFree(f); hipFree(rS);
  }
};

// Argument checks shared by the verifySignatureSets entry points: empty aggregates reject the
// whole call before any verification (aggregatePublicKeys throws, index.ts:398-412).
static int vs_check_args(gbv_ctx* c, const gbv_set* sets, size_t n, const uint32_t* arena) {
  if (n && !sets) return fail(c, GBV_E_ARG, "null sets");
  for (size_t i = 0; i < n; ++i)
    if (!sets[i].raw_pk48 && sets[i].idx_len == 0) return fail(c, GBV_E_EMPTY_AGGREGATE, "EMPTY_AGGREGATE_ARRAY");
  for (size_t i = 0; i < n; ++i) {
    if (!sets[i].msg32 || (!sets[i].sig && sets[i].sig_len)) return fail(c, GBV_E_ARG, "null msg/sig");
    if (!sets[i].raw_pk48) {
      if (!arena) return fail(c, GBV_E_ARG, "null index arena");
      for (uint32_t j = 0; j < sets[i].idx_len; ++j)
        if (arena[sets[i].idx_off + j] >= c->table_n) return fail(c, GBV_E_ARG, "validator index out of range");
    }
  }
  return GBV_OK;
}

// Stage n > 0 sets in HBM and run k_vs_prepare (per set: pubkey aggregate / decode, signature
// decode + subgroup, randomisation, hash_to_G2, Miller value) on stream s.
static int vs_stage_prepare(gbv_ctx* c, const gbv_set* sets, size_t n, const uint32_t* arena, hipStream_t s, VsDev& d) {
  uint32_t stride = 96;
  for (size_t i = 0; i < n; ++i)
    if (sets[i].sig_len == 192) stride = 192;
  std::vector<uint32_t> set_idx_off(n + 1), idx_flat, sig_len(n);
  std::vector<uint8_t> raw_flag(n), raw_pk(48 * n), msgs(32 * n), sig((size_t)stride * n, 0);
  for (size_t i = 0; i < n; ++i) {
    set_idx_off[i] = (uint32_t)idx_flat.size();
    if (sets[i].raw_pk48) {
      raw_flag[i] = 1;
      memcpy(&raw_pk[48 * i], sets[i].raw_pk48, 48);
    } else {
      for (uint32_t j = 0; j < sets[i].idx_len; ++j) idx_flat.push_back(arena[sets[i].idx_off + j]);
    }
    memcpy(&msgs[32 * i], sets[i].msg32, 32);
    uint32_t L = sets[i].sig_len;
    sig_len[i] = (L == 96 || L == 192) ? L : 0;  // other lengths: BAD_ENCODING -> false
    if (sig_len[i]) memcpy(&sig[(size_t)stride * i], sets[i].sig, L);
  }
  set_idx_off[n] = (uint32_t)idx_flat.size();
  HIP_CHECK(c, dalloc(&d.off, n + 1)); HIP_CHECK(c, dalloc(&d.idx, idx_flat.size())); HIP_CHECK(c, dalloc(&d.siglen, n));
  HIP_CHECK(c, dalloc(&d.raw_flag, n)); HIP_CHECK(c, dalloc(&d.raw_pk, 48 * n)); HIP_CHECK(c, dalloc(&d.msgs, 32 * n));
  HIP_CHECK(c, dalloc(&d.sig, (size_t)stride * n)); HIP_CHECK(c, dalloc(&d.status, n)); HIP_CHECK(c, dalloc(&d.f, n));
  HIP_CHECK(c, dalloc(&d.rS, n));
  HIP_CHECK(c, hipMemcpyAsync(d.off, set_idx_off.data(), 4 * (n + 1), hipMemcpyHostToDevice, s));
  if (!idx_flat.empty()) HIP_CHECK(c, hipMemcpyAsync(d.idx, idx_flat.data(), 4 * idx_flat.size(), hipMemcpyHostToDevice, s));
  HIP_CHECK(c, hipMemcpyAsync(d.siglen, sig_len.data(), 4 * n, hipMemcpyHostToDevice, s));
  HIP_CHECK(c, hipMemcpyAsync(d.raw_flag, raw_flag.data(), n, hipMemcpyHostToDevice, s));
  HIP_CHECK(c, hipMemcpyAsync(d.raw_pk, raw_pk.data(), 48 * n, hipMemcpyHostToDevice, s));
  HIP_CHECK(c, hipMemcpyAsync(d.msgs, msgs.data(), 32 * n, hipMemcpyHostToDevice, s));
  HIP_CHECK(c, hipMemcpyAsync(d.sig, sig.data(), (size_t)stride * n, hipMemcpyHostToDevice, s));
  Seed seed = fresh_seed();
  uint32_t nonce = c->nonce++;
  launch_vs_prepare(LaunchCfg{blocks_for(n), TPB, s}, (uint32_t)n, d.off, d.idx, d.raw_flag, d.raw_pk, d.msgs, d.sig, stride, d.siglen,
                    c->table, c->table_ok, seed, nonce, d.f, d.rS, d.status);
  HIP_CHECK(c, hipGetLastError());
  // the host vectors above are freed on return: the copies must have landed
  HIP_CHECK(c, hipStreamSynchronize(s));
  return GBV_OK;
}

int gbv_verify_sets(gbv_ctx* c, const gbv_set* sets, size_t n, const uint32_t* arena, uint8_t* all_valid, uint8_t* chunk_valid) {
  if (!c || !all_valid) return GBV_E_ARG;
  if (c->closed) return GBV_E_CLOSED;
  *all_valid = 0;
  int rc = vs_check_args(c, sets, n, arena);
  if (rc) return rc;
  if (n == 0) {  // verifySignatureSetsMaybeBatch([]) throws -> false (maybeBatch.ts:29-31,39-44)
    if (chunk_valid) chunk_valid[0] = 0;
    return GBV_OK;
  }
  HIP_CHECK(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  std::vector<uint32_t> co = chunk_offsets((uint32_t)n, MAX_SIGNATURE_SETS_PER_JOB);
  size_t C = co.size() - 1;
  VsDev d;
  uint32_t* d_chunk_off = nullptr;
  uint8_t* d_cv = nullptr;
  rc = vs_stage_prepare(c, sets, n, arena, s, d);
  if (rc == GBV_OK) {
    HIP_CHECK(c, dalloc(&d_chunk_off, C + 1));
    HIP_CHECK(c, dalloc(&d_cv, C));
    HIP_CHECK(c, hipMemcpyAsync(d_chunk_off, co.data(), 4 * (C + 1), hipMemcpyHostToDevice, s));
    launch_vs_chunk_coop(LaunchCfg{(unsigned)C, 64, s}, (uint32_t)C, d_chunk_off, d.status, d.f, d.rS, d_cv);
    HIP_CHECK(c, hipGetLastError());
    std::vector<uint8_t> cv(C);
    HIP_CHECK(c, hipMemcpyAsync(cv.data(), d_cv, C, hipMemcpyDeviceToHost, s));
    HIP_CHECK(c, hipStreamSynchronize(s));
    uint8_t all = 1;
    for (size_t k = 0; k < C; ++k) all &= cv[k];
    *all_valid = all;
    if (chunk_valid) memcpy(chunk_valid, cv.data(), C);
  }
  d.release();
  hipFree(d_chunk_off);
  hipFree(d_cv);
  return rc;
}

// One shard of a verifySignatureSets call spread over several GPUs.
int gbv_vs_partial(gbv_ctx* c, const gbv_set* sets, size_t n, const uint32_t* arena, uint8_t out576[GBV_FP12_PARTIAL_BYTES],
                   uint8_t* shard_ok) {
  if (!c || !out576 || !shard_ok) return GBV_E_ARG;
  if (c->closed) return GBV_E_CLOSED;
  int rc = vs_check_args(c, sets, n, arena);
  if (rc) return rc;
  *shard_ok = 1;
  Fp12 one = fp12_one_host();
  if (n == 0) {
    fp12_pack(out576, one);
    return GBV_OK;
  }
  HIP_CHECK(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  VsDev d;
  rc = vs_stage_prepare(c, sets, n, arena, s, d);
  Fp12 *part = nullptr, *d_out = nullptr;
  G2J* spart = nullptr;
  uint8_t *has = nullptr, *d_flag = nullptr;
  if (rc == GBV_OK) {
    size_t np = n / 64 + n / 4096 + 4;
    HIP_CHECK(c, dalloc(&part, np)); HIP_CHECK(c, dalloc(&spart, np)); HIP_CHECK(c, dalloc(&has, np));
    HIP_CHECK(c, dalloc(&d_out, 1)); HIP_CHECK(c, dalloc(&d_flag, 1));
    // status doubles as the per-"chunk" state: SET_OK == GRP_PENDING (every valid set takes part)
    launch_sm_seg_check(LaunchCfg{1, 64, s}, 0, (uint32_t)n, d.status, d.f, d.rS, part, spart, has, d_flag, d_out);
    HIP_CHECK(c, hipGetLastError());
    std::vector<uint8_t> st(n);
    HIP_CHECK(c, hipMemcpyAsync(st.data(), d.status, n, hipMemcpyDeviceToHost, s));
    Fp12 h;
    HIP_CHECK(c, hipMemcpyAsync(&h, d_out, sizeof(Fp12), hipMemcpyDeviceToHost, s));
    HIP_CHECK(c, hipStreamSynchronize(s));
    fp12_pack(out576, h);
    for (size_t i = 0; i < n; ++i)
      if (st[i] != SET_OK) *shard_ok = 0;
  }
  d.release();
  hipFree(part); hipFree(spart); hipFree(has); hipFree(d_out); hipFree(d_flag);
  return rc;
}

int gbv_fp12_check(gbv_ctx* c, const uint8_t* partials, size_t k, uint8_t* is_one) {
  if (!c || !is_one || (k && !partials)) return GBV_E_ARG;
  if (c->closed) return GBV_E_CLOSED;
  HIP_CHECK(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  Fp12* d_p = nullptr;
  uint8_t* d_o = nullptr;
  HIP_CHECK(c, dalloc(&d_p, k));
  HIP_CHECK(c, dalloc(&d_o, 1));
  std::vector<Fp12> hp(k);
  for (size_t j = 0; j < k; ++j) hp[j] = fp12_unpack(partials + GBV_FP12_PARTIAL_BYTES * j);
  if (k) HIP_CHECK(c, hipMemcpyAsync(d_p, hp.data(), sizeof(Fp12) * k, hipMemcpyHostToDevice, s));
  launch_fp12_check(LaunchCfg{1, 64, s}, (uint32_t)k, d_p, d_o);
  HIP_CHECK(c, hipGetLastError());
  HIP_CHECK(c, hipMemcpyAsync(is_one, d_o, 1, hipMemcpyDeviceToHost, s));
  HIP_CHECK(c, hipStreamSynchronize(s));
  hipFree(d_p);
  hipFree(d_o);
  return GBV_OK;
}

// ---- utilities -----------------------------------------------------------------------------
// ---- signing roots (SSZ) --------------------------------------------------------------------
static int ssz_buf(gbv_ctx* c, int k, size_t bytes, uint8_t** out) {
  if (c->ssz_cap[k] < bytes) {
    hipFree(c->ssz_buf[k]);
    c->ssz_buf[k] = nullptr;
    c->ssz_cap[k] = 0;
    size_t cap = std::max<size_t>(bytes, 1u << 20);
    HIP_CHECK(c, hipMalloc((void**)&c->ssz_buf[k], cap));
    c->ssz_cap[k] = cap;
  }
  *out = c->ssz_buf[k];
  return GBV_OK;
}

static int ssz_begin(gbv_ctx* c) {
  if (!c) return GBV_E_ARG;
  if (c->closed) return GBV_E_CLOSED;
  HIP_CHECK(c, hipSetDevice(c->device));
  for (auto& e : c->ssz_ev)
    if (!e) HIP_CHECK(c, hipEventCreate(&e));
  c->last_ssz_ms = 0.f;
  return GBV_OK;
}

// Copy n results back, wait, and record the device time between the two events.
static int ssz_finish(gbv_ctx* c, const uint8_t* d_out, size_t n, uint8_t* out32) {
  HIP_CHECK(c, hipGetLastError());
  HIP_CHECK(c, hipEventRecord(c->ssz_ev[1], c->stream));
  HIP_CHECK(c, hipMemcpyAsync(out32, d_out, 32 * n, hipMemcpyDeviceToHost, c->stream));
  HIP_CHECK(c, hipStreamSynchronize(c->stream));
  HIP_CHECK(c, hipEventElapsedTime(&c->last_ssz_ms, c->ssz_ev[0], c->ssz_ev[1]));
  return GBV_OK;
}

// Stage domains (and per-item indices) for the signing-root kernels.
static int ssz_domains(gbv_ctx* c, size_t n, const uint8_t* domains32, size_t n_domains, const uint32_t* dom_idx, uint8_t** d_dom,
                       uint32_t** d_idx) {
  if (!domains32 || n_domains == 0) return fail(c, GBV_E_ARG, "no domain");
  if (dom_idx)
    for (size_t i = 0; i < n; ++i)
      if (dom_idx[i] >= n_domains) return fail(c, GBV_E_ARG, "domain index out of range");
  int rc = ssz_buf(c, 2, 32 * n_domains, d_dom);
  if (rc) return rc;
  HIP_CHECK(c, hipMemcpyAsync(*d_dom, domains32, 32 * n_domains, hipMemcpyHostToDevice, c->stream));
  *d_idx = nullptr;
  if (dom_idx) {
    uint8_t* p = nullptr;
    if ((rc = ssz_buf(c, 3, 4 * n, &p))) return rc;
    HIP_CHECK(c, hipMemcpyAsync(p, dom_idx, 4 * n, hipMemcpyHostToDevice, c->stream));
    *d_idx = (uint32_t*)p;
  }
  return GBV_OK;
}

int gbv_sha256_digest64(gbv_ctx* c, const uint8_t* in64, size_t n, uint8_t* out32) { return gbv_merkle_roots(c, in64, n, 1, out32); }

int gbv_merkle_roots(gbv_ctx* c, const uint8_t* chunks32, size_t n, uint32_t depth, uint8_t* out32) {
  int rc = ssz_begin(c);
  if (rc) return rc;
  if (n == 0) return GBV_OK;
  if (!chunks32 || !out32) return fail(c, GBV_E_ARG, "null argument");
  if (depth > 24 || (n << depth) >> depth != n || (n << depth) > 0xFFFFFFFFull) return fail(c, GBV_E_ARG, "tree too large");
  size_t leaves = n << depth;
  uint8_t *a = nullptr, *b = nullptr;
  if ((rc = ssz_buf(c, 0, 32 * leaves, &a))) return rc;
  if ((rc = ssz_buf(c, 1, 32 * std::max<size_t>(leaves / 2, n), &b))) return rc;
  HIP_CHECK(c, hipMemcpyAsync(a, chunks32, 32 * leaves, hipMemcpyHostToDevice, c->stream));
  HIP_CHECK(c, hipEventRecord(c->ssz_ev[0], c->stream));
  // one launch per tree level: sibling chunks are adjacent, so a level is a digest64 over pairs
  for (uint32_t lvl = 0; lvl < depth; ++lvl) {
    leaves /= 2;
    launch_ssz_digest64(c->stream, a, (uint32_t)leaves, b);
    debug_sync(c->stream, "k_ssz_digest64");
    std::swap(a, b);
  }
  return ssz_finish(c, a, n, out32);
}

int gbv_signing_roots(gbv_ctx* c, const uint8_t* roots32, size_t n, const uint8_t* domains32, size_t n_domains, const uint32_t* dom_idx,
                      uint8_t* out32) {
  int rc = ssz_begin(c);
  if (rc) return rc;
  if (n == 0) return GBV_OK;
  if (!roots32 || !out32) return fail(c, GBV_E_ARG, "null argument");
  if (n > 0xFFFFFFFFull) return fail(c, GBV_E_ARG, "too many roots");
  uint8_t *d_in = nullptr, *d_out = nullptr, *d_dom = nullptr;
  uint32_t* d_idx = nullptr;
  if ((rc = ssz_domains(c, n, domains32, n_domains, dom_idx, &d_dom, &d_idx))) return rc;
  if ((rc = ssz_buf(c, 0, 32 * n, &d_in)) || (rc = ssz_buf(c, 1, 32 * n, &d_out))) return rc;
  HIP_CHECK(c, hipMemcpyAsync(d_in, roots32, 32 * n, hipMemcpyHostToDevice, c->stream));
  HIP_CHECK(c, hipEventRecord(c->ssz_ev[0], c->stream));
  launch_ssz_signing_roots(c->stream, d_in, (uint32_t)n, d_dom, d_idx, d_out);
  debug_sync(c->stream, "k_ssz_signing_roots");
  return ssz_finish(c, d_out, n, out32);
}

int gbv_attestation_signing_roots(gbv_ctx* c, const uint8_t* data128, size_t n, const uint8_t* domains32, size_t n_domains,
                                  const uint32_t* dom_idx, uint8_t* out32) {
  int rc = ssz_begin(c);
  if (rc) return rc;
  if (n == 0) return GBV_OK;
  if (!data128 || !out32) return fail(c, GBV_E_ARG, "null argument");
  if (n > 0xFFFFFFFFull) return fail(c, GBV_E_ARG, "too many objects");
  uint8_t *d_in = nullptr, *d_out = nullptr, *d_dom = nullptr;
  uint32_t* d_idx = nullptr;
  if ((rc = ssz_domains(c, n, domains32, n_domains, dom_idx, &d_dom, &d_idx))) return rc;
  if ((rc = ssz_buf(c, 0, 128 * n, &d_in)) || (rc = ssz_buf(c, 1, 32 * n, &d_out))) return rc;
  HIP_CHECK(c, hipMemcpyAsync(d_in, data128, 128 * n, hipMemcpyHostToDevice, c->stream));
  HIP_CHECK(c, hipEventRecord(c->ssz_ev[0], c->stream));
  launch_ssz_att_signing_roots(c->stream, d_in, (uint32_t)n, d_dom, d_idx, d_out);
  debug_sync(c->stream, "k_ssz_att_signing_roots");
  return ssz_finish(c, d_out, n, out32);
}

int gbv_ssz_last_kernel_ms(gbv_ctx* c, float* ms) {
  if (!c || !ms) return GBV_E_ARG;
  *ms = c->last_ssz_ms;
  return GBV_OK;
}

int gbv_util_sk_to_pk(gbv_ctx* c, const uint8_t* sk32, size_t n, uint8_t* pk48) {
  if (!c || (n && (!sk32 || !pk48))) return GBV_E_ARG;
  if (n == 0) return GBV_OK;
  HIP_CHECK(c, hipSetDevice(c->device));
  uint8_t *d_sk, *d_pk;
  HIP_CHECK(c, dalloc(&d_sk, 32 * n));
  HIP_CHECK(c, dalloc(&d_pk, 48 * n));
  HIP_CHECK(c, hipMemcpyAsync(d_sk, sk32, 32 * n, hipMemcpyHostToDevice, c->stream));
  launch_util_sk_to_pk(LaunchCfg{blocks_for(n), TPB, c->stream}, (uint32_t)n, d_sk, d_pk);
  HIP_CHECK(c, hipGetLastError());
  HIP_CHECK(c, hipMemcpyAsync(pk48, d_pk, 48 * n, hipMemcpyDeviceToHost, c->stream));
  HIP_CHECK(c, hipStreamSynchronize(c->stream));
  hipFree(d_sk);
  hipFree(d_pk);
  return GBV_OK;
}

int gbv_util_hash_to_g2(gbv_ctx* c, const uint8_t* msgs32, size_t n, uint8_t* out192) {
  if (!c || (n && (!msgs32 || !out192))) return GBV_E_ARG;
  if (n == 0) return GBV_OK;
  HIP_CHECK(c, hipSetDevice(c->device));
  uint8_t *d_m, *d_o;
  G2A* d_H;
  HIP_CHECK(c, dalloc(&d_m, 32 * n));
  HIP_CHECK(c, dalloc(&d_o, 192 * n));
  HIP_CHECK(c, dalloc(&d_H, n));
  HIP_CHECK(c, hipMemcpyAsync(d_m, msgs32, 32 * n, hipMemcpyHostToDevice, c->stream));
  launch_hash_msgs(LaunchCfg{blocks_for(n), TPB, c->stream}, d_m, (uint32_t)n, d_H);
  launch_util_g2_out(LaunchCfg{blocks_for(n), TPB, c->stream}, (uint32_t)n, d_H, d_o);
  HIP_CHECK(c, hipGetLastError());
  HIP_CHECK(c, hipMemcpyAsync(out192, d_o, 192 * n, hipMemcpyDeviceToHost, c->stream));
  HIP_CHECK(c, hipStreamSynchronize(c->stream));
  hipFree(d_m); hipFree(d_o); hipFree(d_H);
  return GBV_OK;
}

int gbv_util_sign(gbv_ctx* c, const uint8_t* sk32, size_t n, const uint32_t* grp, const uint8_t* msgs32, size_t n_msgs, uint8_t* sig96) {
  if (!c || (n && (!sk32 || !grp || !msgs32 || !sig96))) return GBV_E_ARG;
  if (n == 0) return GBV_OK;
  for (size_t i = 0; i < n; ++i)
    if (grp[i] >= n_msgs) return fail(c, GBV_E_ARG, "message index out of range");
  HIP_CHECK(c, hipSetDevice(c->device));
  uint8_t *d_sk, *d_m, *d_sig;
  uint32_t* d_grp;
  G2A* d_H;
  HIP_CHECK(c, dalloc(&d_sk, 32 * n));
  HIP_CHECK(c, dalloc(&d_m, 32 * n_msgs));
  HIP_CHECK(c, dalloc(&d_sig, 96 * n));
  HIP_CHECK(c, dalloc(&d_grp, n));
  HIP_CHECK(c, dalloc(&d_H, n_msgs));
  HIP_CHECK(c, hipMemcpyAsync(d_sk, sk32, 32 * n, hipMemcpyHostToDevice, c->stream));
  HIP_CHECK(c, hipMemcpyAsync(d_m, msgs32, 32 * n_msgs, hipMemcpyHostToDevice, c->stream));
  HIP_CHECK(c, hipMemcpyAsync(d_grp, grp, 4 * n, hipMemcpyHostToDevice, c->stream));
  launch_hash_msgs(LaunchCfg{blocks_for(n_msgs), TPB, c->stream}, d_m, (uint32_t)n_msgs, d_H);
  launch_util_sign(LaunchCfg{blocks_for(n), TPB, c->stream}, (uint32_t)n, d_sk, d_grp, d_H, d_sig);
  HIP_CHECK(c, hipGetLastError());
  HIP_CHECK(c, hipMemcpyAsync(sig96, d_sig, 96 * n, hipMemcpyDeviceToHost, c->stream));
  HIP_CHECK(c, hipStreamSynchronize(c->stream));
  hipFree(d_sk); hipFree(d_m); hipFree(d_sig); hipFree(d_grp); hipFree(d_H);
  return GBV_OK;
}

}  // extern "C"
