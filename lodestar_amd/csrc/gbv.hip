// Host side of the C ABI (include/gbv.h): the context, the HBM pubkey table, same-message
// batches (verifySignatureSetsSameMessage) with chunking exactly as the reference pool does it,
// signing roots and utilities.  verifySignatureSets lives in gbv_vs.hip.
#include "ctx.h"

using namespace gbv;

namespace {

// a failing segment with at least this many chunks checks them one thread each (throughput), below
// it one wave each (latency); see k_sm_group_check / k_sm_group_pairing
// segments of at most this many chunks skip the combined segment check (latency of small calls)
constexpr uint32_t DIRECT_CHUNK_MAX = 32;
// events per segment: [0,1] prepare, [2,3] chunk finish, [4,5] miller, [6,7] seg check,
// [8,9] group checks, [10,11] msm buckets, [12] msm reduce done
constexpr size_t EPS = 13;

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace

// The message of the last failure on the calling thread (gbv_last_error): with several host threads
// on one context, each reads its own call's error.
static thread_local std::string t_err;

int gbv_fail(gbv_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  t_err = msg;
  return code;
}

void ctx_drain(gbv_ctx* c) {
  for (hipStream_t s : {c->stream, c->stream2, c->stream4, c->stream5, c->stream6})
    if (s) (void)hipStreamSynchronize(s);
  (void)hipGetLastError();
}

int ctx_small_dev(gbv_ctx* c, size_t bytes, uint8_t** out) {
  if (c->small_dev_cap < bytes) {
    hipFree(c->small_dev);
    c->small_dev = nullptr;
    c->small_dev_cap = 0;
    size_t cap = std::max<size_t>(bytes, 1u << 16);
    HIP_CHECK(c, hipMalloc((void**)&c->small_dev, cap));
    c->small_dev_cap = cap;
  }
  *out = c->small_dev;
  return GBV_OK;
}

int ctx_small_host(gbv_ctx* c, size_t bytes, uint8_t** out) {
  if (c->small_host_cap < bytes) {
    hipHostFree(c->small_host);
    c->small_host = nullptr;
    c->small_host_cap = 0;
    size_t cap = std::max<size_t>(bytes, 1u << 16);
    HIP_CHECK(c, hipHostMalloc((void**)&c->small_host, cap, hipHostMallocDefault));
    c->small_host_cap = cap;
  }
  *out = c->small_host;
  return GBV_OK;
}

// A same-message workload staged in HBM.  The inputs are views into one device blob filled by ONE
// copy from a pinned staging blob; work buffers are sized by capacity so a batch (and the context's
// scratch batch used by the one-shot entry points) is refilled without any hipMalloc.
struct gbv_sm_batch {
  size_t n = 0, G = 0, n_calls = 0;
  size_t cap_n = 0, cap_G = 0, cap_calls = 0;
  bool has_msm = false, allocated = false;
  std::vector<uint32_t> grp_off_host;
  uint8_t *in_dev = nullptr, *in_host = nullptr;
  size_t in_cap = 0;
  uint32_t *idx = nullptr, *grp_off = nullptr, *grp_msg = nullptr, *set_grp = nullptr;
  uint8_t *sig = nullptr, *msgs = nullptr;
  uint32_t* n_fallback = nullptr;
  uint8_t *status = nullptr, *grp_state = nullptr, *valid = nullptr, *seg_ok = nullptr;
  uint8_t* seg_ok_host = nullptr;  // pinned
  uint8_t* valid_host = nullptr;   // pinned, n bytes: results of the last submitted verify
  uint32_t* nfb_host = nullptr;    // pinned: fallback chunk count of the last submitted verify
  size_t seg_cap = 64;
  std::vector<uint8_t> seg_direct = std::vector<uint8_t>(64);  // per segment: combined check skipped
  // in-flight state of the last gbv_sm_batch_submit
  bool in_flight = false;
  size_t n_seg = 0;
  // two event sets, one per tail stream (gbv_ctx::sm_submits parity): an event is only ever
  // recorded on one stream
  std::vector<hipEvent_t> evs[2];
  hipEvent_t dones[2] = {};
  int cur = 0;  // event set of the last submit
  // the input blob's host-to-device copy (stream A) of the last fill: the pinned blob is rewritten
  // only once it is done, and the streams other than A wait for it before reading the inputs
  hipEvent_t copied = nullptr;
  G2A *H = nullptr, *S = nullptr;
  G2J *rS = nullptr, *SgJ = nullptr;
  Fp12* F = nullptr;
  Fp12* Ffb = nullptr;       // 2 * FB_COOP_MAX: the two Miller values of each few-item per-set check
  G2J* Hpre = nullptr;       // per message: Q0 + Q1 before the cofactor clearing (few-message hashing)
  Fp12* Fpair = nullptr;     // 2 per chunk: the two Miller values of a chunk's own check (k_sm_group_miller2)
  uint8_t* pair_ok = nullptr;
  Fp12* Fpart = nullptr;  // per 64-chunk block partials of a segment (reused segment after segment)
  G2J* Spart = nullptr;
  uint8_t* has = nullptr;
  size_t part_stride = 0;
  G1J* rP = nullptr;
  G1J* PgJ = nullptr;
  // failure path lists: runs of failed chunks (head, end, chunk), then sets of failing runs
  uint4* fb_runs = nullptr;
  uint32_t* fb_list = nullptr;
  uint32_t* fb_cnt = nullptr;  // [runs, listed sets]
  size_t fb_cap = 0;
  // bucket MSM scratch: two sets, by segment parity
  uint32_t *msm_cnt[2] = {}, *msm_off[2] = {}, *msm_cur[2] = {};
  G2J *msm_buckets[2] = {}, *msm_part[2] = {}, *msm_head[2] = {}, *msm_tail[2] = {};
  uint32_t* msm_ent = nullptr;  // 4 per set, segment s at 4 * s0
  G2J* msm_total = nullptr;     // one per segment
  std::vector<uint8_t> seg_msm = std::vector<uint8_t>(64);
  KProf prof;  // per-kernel events of the last submit (ctx kprof_on)
};

static void sm_free_work(gbv_sm_batch* b) {
  hipFree(b->n_fallback); hipFree(b->status); hipFree(b->grp_state); hipFree(b->valid);
  hipFree(b->H); hipFree(b->S); hipFree(b->SgJ); hipFree(b->rS); hipFree(b->rP); hipFree(b->PgJ);
  hipHostFree(b->valid_host); hipHostFree(b->nfb_host);
  hipFree(b->F); hipFree(b->Fpair); hipFree(b->pair_ok); hipFree(b->Hpre); hipFree(b->Ffb); hipFree(b->seg_ok); hipHostFree(b->seg_ok_host);
  hipFree(b->Fpart); hipFree(b->Spart); hipFree(b->has);
  hipFree(b->fb_runs); hipFree(b->fb_list); hipFree(b->fb_cnt);
  for (int k = 0; k < 2; ++k) {
    hipFree(b->msm_cnt[k]); hipFree(b->msm_off[k]); hipFree(b->msm_cur[k]); hipFree(b->msm_buckets[k]); hipFree(b->msm_part[k]);
    hipFree(b->msm_head[k]); hipFree(b->msm_tail[k]);
    b->msm_cnt[k] = b->msm_off[k] = b->msm_cur[k] = nullptr;
    b->msm_buckets[k] = b->msm_part[k] = b->msm_head[k] = b->msm_tail[k] = nullptr;
  }
  hipFree(b->msm_ent); hipFree(b->msm_total);
  b->n_fallback = nullptr; b->status = b->grp_state = b->valid = b->seg_ok = b->seg_ok_host = b->valid_host = nullptr;
  b->H = b->S = nullptr; b->SgJ = b->rS = nullptr; b->rP = b->PgJ = nullptr; b->F = b->Fpart = b->Fpair = nullptr; b->pair_ok = nullptr; b->Hpre = nullptr; b->Ffb = nullptr; b->Spart = nullptr;
  b->has = nullptr; b->fb_runs = nullptr; b->fb_list = b->fb_cnt = b->nfb_host = nullptr; b->msm_ent = nullptr; b->msm_total = nullptr;
  b->allocated = false;
}

static hipError_t msm_alloc(gbv_sm_batch* b, size_t n) {
  hipError_t e = hipSuccess;
  auto chk = [&](hipError_t x) { if (x != hipSuccess && e == hipSuccess) e = x; };
  for (int k = 0; k < 2; ++k) {
    chk(dalloc(&b->msm_cnt[k], MSM_KEYS)); chk(dalloc(&b->msm_off[k], MSM_KEYS)); chk(dalloc(&b->msm_cur[k], MSM_KEYS));
    chk(dalloc(&b->msm_buckets[k], MSM_KEYS)); chk(dalloc(&b->msm_part[k], MSM_PARTS + 130));
    chk(dalloc(&b->msm_head[k], 4 * n / MSM_RUN + 64)); chk(dalloc(&b->msm_tail[k], 4 * n / MSM_RUN + 64));
  }
  chk(dalloc(&b->msm_ent, 4 * n)); chk(dalloc(&b->msm_total, b->seg_cap));
  return e;
}

// Work buffers for up to (n sets, G chunks, calls messages); grows (never shrinks) when needed.
static int sm_reserve(gbv_ctx* c, gbv_sm_batch* b, size_t n, size_t G, size_t calls, bool want_msm) {
  if (b->allocated && n <= b->cap_n && G <= b->cap_G && calls <= b->cap_calls && (!want_msm || b->has_msm)) return GBV_OK;
  if (b->allocated) {
    // grow: keep the larger of old and new so alternating call sizes do not thrash
    n = std::max(n, b->cap_n); G = std::max(G, b->cap_G); calls = std::max(calls, b->cap_calls);
    want_msm = want_msm || b->has_msm;
    sm_free_work(b);
  }
  hipError_t e = hipSuccess;
  auto chk = [&](hipError_t x) { if (x != hipSuccess && e == hipSuccess) e = x; };
  chk(dalloc(&b->n_fallback, 1));
  chk(dalloc(&b->status, n)); chk(dalloc(&b->grp_state, G)); chk(dalloc(&b->valid, n));
  chk(dalloc(&b->H, calls)); chk(dalloc(&b->Hpre, calls)); chk(dalloc(&b->S, n)); chk(dalloc(&b->rS, n)); chk(dalloc(&b->rP, n));
  chk(dalloc(&b->PgJ, G)); chk(dalloc(&b->SgJ, G)); chk(dalloc(&b->F, G));
  chk(dalloc(&b->Fpair, 2 * G)); chk(dalloc(&b->pair_ok, 2 * G)); chk(dalloc(&b->Ffb, 2 * FB_COOP_CAP));
  // block partials: one region per segment parity (two segments' reductions can be in flight)
  b->part_stride = seg_reduce_scratch(G);
  chk(dalloc(&b->Fpart, 2 * b->part_stride)); chk(dalloc(&b->Spart, 2 * b->part_stride)); chk(dalloc(&b->has, 2 * b->part_stride));
  b->fb_cap = n / 8 + G + 64;  // runs: at most one per 8-set window plus one per chunk start
  chk(dalloc(&b->fb_runs, b->fb_cap)); chk(dalloc(&b->fb_list, n)); chk(dalloc(&b->fb_cnt, 2));
  chk(dalloc(&b->seg_ok, b->seg_cap));
  chk(hipHostMalloc((void**)&b->seg_ok_host, b->seg_cap, hipHostMallocDefault));
  chk(hipHostMalloc((void**)&b->valid_host, std::max<size_t>(n, 1), hipHostMallocDefault));
  chk(hipHostMalloc((void**)&b->nfb_host, sizeof(uint32_t), hipHostMallocDefault));
  for (int k = 0; k < 2; ++k)
    if (!b->dones[k]) chk(hipEventCreateWithFlags(&b->dones[k], hipEventDisableTiming));
  if (want_msm) chk(msm_alloc(b, n));
  b->allocated = true;
  b->cap_n = n; b->cap_G = G; b->cap_calls = calls; b->has_msm = want_msm;
  if (e != hipSuccess) {
    sm_free_work(b);
    return gbv_fail(c, GBV_E_OOM, std::string("hipMalloc: ") + hipGetErrorString(e));
  }
  return GBV_OK;
}

static void sm_destroy(gbv_sm_batch* b) {
  if (!b) return;
  if (b->in_flight && b->dones[b->cur]) hipEventSynchronize(b->dones[b->cur]);  // nothing is freed under a running pass
  if (b->copied) {
    hipEventSynchronize(b->copied);
    hipEventDestroy(b->copied);
  }
  sm_free_work(b);
  b->prof.destroy();
  hipFree(b->in_dev);
  hipHostFree(b->in_host);
  for (int k = 0; k < 2; ++k) {
    for (auto& e : b->evs[k]) hipEventDestroy(e);
    if (b->dones[k]) hipEventDestroy(b->dones[k]);
  }
  delete b;
}

extern "C" {

int gbv_init(int device, gbv_ctx** out) {
  if (!out) return GBV_E_ARG;
  *out = nullptr;
  tuning_load();
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return GBV_E_DEVICE;
  if (device < 0 || device >= ndev) return GBV_E_ARG;
  gbv_ctx* c = new gbv_ctx();
  c->device = device;
  // stream A (k_sm_prepare, throughput) at the lowest priority, the latency-bound chunk tails, hash
  // and MSM streams at the highest: their few waves then dispatch ahead of k_sm_prepare's
  int prio_lo = 0, prio_hi = 0;
  bool ok = hipSetDevice(device) == hipSuccess && hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi) == hipSuccess &&
            hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, prio_lo) == hipSuccess &&
            hipStreamCreateWithPriority(&c->stream2, hipStreamNonBlocking, prio_hi) == hipSuccess &&
            hipStreamCreateWithPriority(&c->stream4, hipStreamNonBlocking, prio_hi) == hipSuccess &&
            hipStreamCreateWithPriority(&c->stream5, hipStreamNonBlocking, prio_hi) == hipSuccess &&
            hipStreamCreateWithPriority(&c->stream6, hipStreamNonBlocking, prio_hi) == hipSuccess;
  if (!ok) {
    for (hipStream_t s : {c->stream, c->stream2, c->stream4, c->stream5, c->stream6})
      if (s) hipStreamDestroy(s);
    delete c;
    return GBV_E_DEVICE;
  }
  *out = c;
  return GBV_OK;
}

void gbv_destroy(gbv_ctx* c) {
  if (!c) return;
  {
    // a call still running on another thread finishes first (one-shot calls hold a scratch mutex
    // while they wait on the device)
    std::lock_guard<std::mutex> g1(c->sm_scratch_mu), g2(c->vs_scratch_mu);
    GBV_LOCK(c);
  }
  hipSetDevice(c->device);
  c->closed = true;
  // every stream drains before anything it may still read or write is freed
  for (hipStream_t s : {c->stream, c->stream2, c->stream4, c->stream5, c->stream6})
    if (s) hipStreamSynchronize(s);
  sm_destroy(c->sm_scratch);
  vs_batch_free(c->vs_scratch);
  hipFree(c->table);
  hipFree(c->table_ok);
  hipFree(c->comb);
  hipFree(c->comb_ok);
  hipFree(c->small_dev);
  hipHostFree(c->small_host);
  for (auto* p : c->ssz_buf) hipFree(p);
  for (auto e : c->ssz_ev)
    if (e) hipEventDestroy(e);
  for (hipStream_t s : {c->stream, c->stream2, c->stream4, c->stream5, c->stream6})
    if (s) hipStreamDestroy(s);
  delete c;
}

int gbv_tune(gbv_ctx* c, const char* name, uint32_t value) {
  if (!c || !name) return GBV_E_ARG;
  GBV_LOCK(c);
  if (!strcmp(name, "msm_min")) c->msm_min = value;
  else if (!strcmp(name, "msm_cooldown")) c->msm_cooldown_len = value;
  else if (!strcmp(name, "segments")) c->segments = std::max<uint32_t>(value, 1);
  else if (!strcmp(name, "kprof")) c->kprof_on = value != 0;
  else if (!strcmp(name, "comb")) c->comb_on = value != 0 && (c->comb_on || c->table_n == 0);  // off at any time; on before ingest only
  else if (!tuning_set(name, value)) return gbv_fail(c, GBV_E_ARG, std::string("unknown setting: ") + name);
  return GBV_OK;
}

const char* gbv_last_error(gbv_ctx* c) { return c ? t_err.c_str() : "null context"; }

size_t gbv_pubkeys_count(gbv_ctx* c) {
  if (!c) return 0;
  return c->table_n.load(std::memory_order_acquire);  // no lock: the event loop never waits on a device pass
}
int gbv_comb_enabled(gbv_ctx* c) {
  if (!c) return 0;
  GBV_LOCK(c);
  return c->comb_on ? 1 : 0;
}

static int table_reserve(gbv_ctx* c, size_t need) {
  if (need <= c->table_cap) return GBV_OK;
  size_t cap = std::max(need, c->table_cap * 2);
  G1A* t = nullptr;
  uint8_t* ok = nullptr;
  HIP_CHECK(c, dalloc(&t, cap));
  if (dalloc(&ok, cap) != hipSuccess) {
    hipFree(t);
    return gbv_fail(c, GBV_E_OOM, "hipMalloc: table flags");
  }
  hipError_t e = hipMemsetAsync(ok, 0, cap, c->stream);
  if (e == hipSuccess && c->table_n) {
    e = hipMemcpyAsync(t, c->table, c->table_n * sizeof(G1A), hipMemcpyDeviceToDevice, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(ok, c->table_ok, c->table_n, hipMemcpyDeviceToDevice, c->stream);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) {
    hipFree(t);
    hipFree(ok);
    return gbv_fail(c, GBV_E_DEVICE, std::string("table grow: ") + hipGetErrorString(e));
  }
  hipFree(c->table);
  hipFree(c->table_ok);
  c->table = t;
  c->table_ok = ok;
  c->table_cap = cap;
  return GBV_OK;
}

// ---- comb tables (curve.h comb_mul): one per table slot, grown with the table -------------------
static constexpr size_t COMB_SLOT_BYTES = (size_t)COMB_ENTRIES * COMB_U4 * sizeof(uint4);

static void comb_disable(gbv_ctx* c) {
  hipFree(c->comb);
  hipFree(c->comb_ok);
  c->comb = nullptr;
  c->comb_ok = nullptr;
  c->comb_cap = 0;
  c->comb_on = false;
}

// Room for `need` slots, slots [0, keep) preserved.  The tables are an accelerator, not state: when
// HBM cannot hold them the context drops them and k_sm_prepare runs the ladder (same results).
static int comb_reserve(gbv_ctx* c, size_t need, size_t keep) {
  if (need <= c->comb_cap) return GBV_OK;
  size_t cap = std::max(need, c->comb_cap * 2);
  uint4* t = nullptr;
  uint8_t* ok = nullptr;
  if (hipMalloc(&t, cap * COMB_SLOT_BYTES) != hipSuccess || hipMalloc(&ok, cap) != hipSuccess) {
    (void)hipGetLastError();
    hipFree(t);
    comb_disable(c);
    return GBV_OK;
  }
  hipError_t e = hipMemsetAsync(ok, 0, cap, c->stream);
  keep = std::min(keep, c->comb_cap);
  if (e == hipSuccess && keep) {
    e = hipMemcpyAsync(t, c->comb, keep * COMB_SLOT_BYTES, hipMemcpyDeviceToDevice, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(ok, c->comb_ok, keep, hipMemcpyDeviceToDevice, c->stream);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) {
    hipFree(t);
    hipFree(ok);
    return gbv_fail(c, GBV_E_DEVICE, std::string("comb grow: ") + hipGetErrorString(e));
  }
  hipFree(c->comb);
  hipFree(c->comb_ok);
  c->comb = t;
  c->comb_ok = ok;
  c->comb_cap = cap;
  return GBV_OK;
}

// comb tables of slots [first, first + n) from their (final) table entries
static int comb_build(gbv_ctx* c, uint32_t first, size_t n, size_t keep) {
  if (!c->comb_on) return GBV_OK;
  int rc = comb_reserve(c, (size_t)first + n, keep);
  if (rc || !c->comb_on) return rc;
  constexpr size_t CH = 65536;  // slots per pass: 9 affine bases each in scratch (75 MB)
  G1A* bases = nullptr;
  if (dalloc(&bases, 9 * std::min(n, CH)) != hipSuccess) {
    (void)hipGetLastError();
    comb_disable(c);
    return GBV_OK;
  }
  for (size_t off = 0; off < n; off += CH)
    launch_comb_build(c->stream, first + (uint32_t)off, (uint32_t)std::min(CH, n - off), c->table, c->table_ok, bases, c->comb, c->comb_ok);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  hipFree(bases);
  if (e != hipSuccess) return gbv_fail(c, GBV_E_DEVICE, std::string("comb build: ") + hipGetErrorString(e));
  return GBV_OK;
}

int gbv_pubkeys_append(gbv_ctx* c, uint32_t first, const uint8_t* pk48, size_t n, int validate, uint8_t* status) {
  if (!c) return GBV_E_ARG;
  GBV_LOCK(c);
  if (c->closed) return GBV_E_CLOSED;
  if (n == 0) return GBV_OK;
  if (!pk48) return gbv_fail(c, GBV_E_ARG, "null pk48");
  if ((size_t)first + n > 0xFFFFFFFFull) return gbv_fail(c, GBV_E_ARG, "table index overflow");
  HIP_CHECK(c, hipSetDevice(c->device));
  int rc = table_reserve(c, (size_t)first + n);
  if (rc) return rc;
  uint8_t *d = nullptr, *h = nullptr;
  size_t st_off = align256(48 * n);
  if ((rc = ctx_small_dev(c, st_off + n, &d)) || (rc = ctx_small_host(c, std::max(48 * n, n), &h))) return rc;
  memcpy(h, pk48, 48 * n);
  HIP_CHECK(c, hipMemcpyAsync(d, h, 48 * n, hipMemcpyHostToDevice, c->stream));
  launch_pk_decompress(LaunchCfg{blocks_for(n), TPB, c->stream}, (uint32_t)n, d, validate, c->table + first, c->table_ok + first,
                       d + st_off);
  HIP_CHECK(c, hipGetLastError());
  HIP_CHECK(c, hipMemcpyAsync(h, d + st_off, n, hipMemcpyDeviceToHost, c->stream));
  HIP_CHECK(c, hipStreamSynchronize(c->stream));
  if (status) memcpy(status, h, n);
  const size_t keep = c->table_n;
  c->table_n.store(std::max(keep, (size_t)first + n), std::memory_order_release);
  return comb_build(c, first, n, keep);
}

int gbv_pubkeys_replicate(gbv_ctx* c, uint32_t src_first, uint32_t src_n, uint32_t dst_first, size_t n) {
  if (!c) return GBV_E_ARG;
  GBV_LOCK(c);
  if (src_n == 0 || (size_t)src_first + src_n > c->table_n) return gbv_fail(c, GBV_E_ARG, "bad replicate range");
  HIP_CHECK(c, hipSetDevice(c->device));
  int rc = table_reserve(c, (size_t)dst_first + n);
  if (rc) return rc;
  launch_pk_replicate(LaunchCfg{blocks_for(n, 256), 256, c->stream}, c->table, c->table_ok, src_first, src_n,
                      dst_first, (uint32_t)n);
  HIP_CHECK(c, hipGetLastError());
  HIP_CHECK(c, hipStreamSynchronize(c->stream));
  const size_t keep = c->table_n;
  c->table_n.store(std::max(keep, (size_t)dst_first + n), std::memory_order_release);
  if (c->comb_on && (rc = comb_reserve(c, (size_t)dst_first + n, keep)) != GBV_OK) return rc;
  if (c->comb_on) {  // the source slots' tables are built: copy them like the table entries
    launch_comb_replicate(c->stream, c->comb, c->comb_ok, src_first, src_n, dst_first, (uint32_t)n);
    HIP_CHECK(c, hipGetLastError());
    HIP_CHECK(c, hipStreamSynchronize(c->stream));
  }
  return GBV_OK;
}

// aggregatePublicKeys(...).toBytes() over table slots (idx) or over serialized keys (pk48 non-null:
// aggregateSerializedPublicKeys, decompressed on the device first).
static int aggregate_common(gbv_ctx* c, const uint32_t* idx, const uint8_t* pk48, size_t k, int validate, uint8_t out48[48]) {
  if (!c) return GBV_E_ARG;
  GBV_LOCK(c);
  if (c->closed) return GBV_E_CLOSED;
  if (k == 0) return gbv_fail(c, GBV_E_EMPTY_AGGREGATE, "EMPTY_AGGREGATE_ARRAY");
  if ((!idx && !pk48) || !out48) return gbv_fail(c, GBV_E_ARG, "null argument");
  if (k > 0xFFFFFFFFull) return gbv_fail(c, GBV_E_ARG, "too many keys");
  if (idx)
    for (size_t i = 0; i < k; ++i)
      if (idx[i] >= c->table_n) return gbv_fail(c, GBV_E_ARG, "validator index out of range");
  HIP_CHECK(c, hipSetDevice(c->device));
  // device scratch: [in: idx 4k or pk48 48k][bad u32][out 48][serialized path: G1A k, ok k, status k]
  size_t in_b = align256(pk48 ? 48 * k : 4 * k);
  size_t o_bad = in_b, o_out = in_b + 256, o_tab = o_out + 256;
  size_t o_ok = o_tab + align256(sizeof(G1A) * (pk48 ? k : 0)), o_st = o_ok + align256(pk48 ? k : 0);
  size_t total = o_st + align256(pk48 ? k : 0);
  uint8_t *d = nullptr, *h = nullptr;
  int rc;
  if ((rc = ctx_small_dev(c, total, &d)) || (rc = ctx_small_host(c, std::max<size_t>(in_b, 512) + k, &h))) return rc;
  memcpy(h, pk48 ? (const void*)pk48 : (const void*)idx, pk48 ? 48 * k : 4 * k);
  HIP_CHECK(c, hipMemcpyAsync(d, h, pk48 ? 48 * k : 4 * k, hipMemcpyHostToDevice, c->stream));
  HIP_CHECK(c, hipMemsetAsync(d + o_bad, 0, 4, c->stream));
  const G1A* tab = c->table;
  const uint8_t* tok = c->table_ok;
  uint32_t* d_idx = (uint32_t*)d;
  if (pk48) {  // decompress into scratch slots 0..k-1, then aggregate over the identity index list
    launch_pk_decompress(LaunchCfg{blocks_for(k), TPB, c->stream}, (uint32_t)k, d, validate, (G1A*)(d + o_tab), d + o_ok, d + o_st);
    HIP_CHECK(c, hipGetLastError());
    tab = (const G1A*)(d + o_tab);
    tok = d + o_ok;
    d_idx = nullptr;  // identity
  }
  launch_aggregate(LaunchCfg{1, 256, c->stream}, d_idx, (uint32_t)k, tab, tok, d + o_out, (uint32_t*)(d + o_bad));
  HIP_CHECK(c, hipGetLastError());
  HIP_CHECK(c, hipMemcpyAsync(h, d + o_bad, 4, hipMemcpyDeviceToHost, c->stream));
  HIP_CHECK(c, hipMemcpyAsync(h + 256, d + o_out, 48, hipMemcpyDeviceToHost, c->stream));
  if (pk48) HIP_CHECK(c, hipMemcpyAsync(h + 512, d + o_st, k, hipMemcpyDeviceToHost, c->stream));
  HIP_CHECK(c, hipStreamSynchronize(c->stream));
  uint32_t bad;
  memcpy(&bad, h, 4);
  if (pk48)
    for (size_t i = 0; i < k; ++i)
      if (h[512 + i] != GBV_PT_OK && !(h[512 + i] == GBV_PT_INFINITY && !validate))
        return gbv_fail(c, GBV_E_BAD_POINT, "pubkey " + std::to_string(i) + ": point status " + std::to_string(h[512 + i]));
  if (bad && !pk48) return gbv_fail(c, GBV_E_ARG, "aggregate over an invalid table entry");
  memcpy(out48, h + 256, 48);
  return GBV_OK;
}

int gbv_aggregate_pubkeys(gbv_ctx* c, const uint32_t* idx, size_t k, uint8_t out48[48]) {
  return aggregate_common(c, idx, nullptr, k, 0, out48);
}

int gbv_aggregate_serialized_pubkeys(gbv_ctx* c, const uint8_t* pk48, size_t k, int validate, uint8_t out48[48]) {
  if (c && k && !pk48) return gbv_fail(c, GBV_E_ARG, "null pk48");
  return aggregate_common(c, nullptr, pk48 ? pk48 : (const uint8_t*)"", k, validate, out48);
}

int gbv_signatures_validate(gbv_ctx* c, const uint8_t* sigs, size_t n, uint32_t sig_len, uint8_t* status, uint8_t* out96) {
  if (!c) return GBV_E_ARG;
  GBV_LOCK(c);
  if (c->closed) return GBV_E_CLOSED;
  if (n == 0) return GBV_OK;
  if (!sigs || !status) return gbv_fail(c, GBV_E_ARG, "null argument");
  if (sig_len != 96 && sig_len != 192) return gbv_fail(c, GBV_E_ARG, "sig_len must be 96 or 192");
  HIP_CHECK(c, hipSetDevice(c->device));
  size_t o_st = align256((size_t)sig_len * n), o_out = o_st + align256(n), total = o_out + 96 * n;
  uint8_t *d = nullptr, *h = nullptr;
  int rc;
  if ((rc = ctx_small_dev(c, total, &d)) || (rc = ctx_small_host(c, std::max<size_t>(sig_len, 97) * n, &h))) return rc;
  memcpy(h, sigs, (size_t)sig_len * n);
  HIP_CHECK(c, hipMemcpyAsync(d, h, (size_t)sig_len * n, hipMemcpyHostToDevice, c->stream));
  launch_sig_validate(LaunchCfg{blocks_for(n), TPB, c->stream}, (uint32_t)n, d, sig_len, d + o_st, d + o_out);
  HIP_CHECK(c, hipGetLastError());
  HIP_CHECK(c, hipMemcpyAsync(h, d + o_st, n, hipMemcpyDeviceToHost, c->stream));
  if (out96) HIP_CHECK(c, hipMemcpyAsync(h + n, d + o_out, 96 * n, hipMemcpyDeviceToHost, c->stream));
  HIP_CHECK(c, hipStreamSynchronize(c->stream));
  memcpy(status, h, n);
  if (out96) memcpy(out96, h + n, 96 * n);
  return GBV_OK;
}

int gbv_aggregate_signatures(gbv_ctx* c, const uint8_t* sigs, size_t n, uint32_t sig_len, int validate, uint8_t out96[96]) {
  if (!c) return GBV_E_ARG;
  GBV_LOCK(c);
  if (c->closed) return GBV_E_CLOSED;
  if (n == 0) return gbv_fail(c, GBV_E_EMPTY_AGGREGATE, "EMPTY_AGGREGATE_ARRAY");
  if (!sigs || !out96) return gbv_fail(c, GBV_E_ARG, "null argument");
  if (sig_len != 96 && sig_len != 192) return gbv_fail(c, GBV_E_ARG, "sig_len must be 96 or 192");
  if (n > 0xFFFFFFFFull) return gbv_fail(c, GBV_E_ARG, "too many signatures");
  HIP_CHECK(c, hipSetDevice(c->device));
  // device scratch: [sigs][bad u32][out 96][block partials]
  size_t nb = (n + 63) / 64;
  size_t o_bad = align256((size_t)sig_len * n), o_out = o_bad + 256, o_part = o_out + 256, total = o_part + sizeof(G2J) * nb;
  uint8_t *d = nullptr, *h = nullptr;
  int rc;
  if ((rc = ctx_small_dev(c, total, &d)) || (rc = ctx_small_host(c, std::max<size_t>((size_t)sig_len * n, 512), &h))) return rc;
  memcpy(h, sigs, (size_t)sig_len * n);
  HIP_CHECK(c, hipMemcpyAsync(d, h, (size_t)sig_len * n, hipMemcpyHostToDevice, c->stream));
  HIP_CHECK(c, hipMemsetAsync(d + o_bad, 0, 4, c->stream));
  launch_sig_aggregate(c->stream, (uint32_t)n, d, sig_len, validate, (G2J*)(d + o_part), (uint32_t*)(d + o_bad), d + o_out);
  HIP_CHECK(c, hipGetLastError());
  HIP_CHECK(c, hipMemcpyAsync(h, d + o_bad, 4, hipMemcpyDeviceToHost, c->stream));
  HIP_CHECK(c, hipMemcpyAsync(h + 256, d + o_out, 96, hipMemcpyDeviceToHost, c->stream));
  HIP_CHECK(c, hipStreamSynchronize(c->stream));
  uint32_t bad;
  memcpy(&bad, h, 4);
  if (bad) return gbv_fail(c, GBV_E_BAD_POINT, "signature failed to deserialize");
  memcpy(out96, h + 256, 96);
  return GBV_OK;
}

// ---- same-message batches ------------------------------------------------------------------
void gbv_sm_batch_destroy(gbv_ctx* c, gbv_sm_batch* b) {
  if (c) {
    GBV_LOCK(c);
    sm_destroy(b);
  } else {
    sm_destroy(b);
  }
}

// (Re)fill batch b with a workload: chunking on the host, inputs through one pinned blob and ONE
// copy, work buffers reused when they are large enough.
static int sm_fill(gbv_ctx* c, gbv_sm_batch* b, size_t n_calls, const uint32_t* call_off, const uint32_t* idx, const uint8_t* sigs96,
                   const uint8_t* msgs32) {
  if (b->in_flight) return gbv_fail(c, GBV_E_ARG, "batch in flight");
  if (n_calls && (!call_off || !msgs32)) return gbv_fail(c, GBV_E_ARG, "null argument");
  if (b->copied) HIP_CHECK(c, hipEventSynchronize(b->copied));  // the pinned blob is free again
  size_t n = n_calls ? call_off[n_calls] : 0;
  if (n && (!idx || !sigs96)) return gbv_fail(c, GBV_E_ARG, "null argument");
  if (call_off && call_off[0] != 0) return gbv_fail(c, GBV_E_ARG, "call offsets must start at 0");
  for (size_t g = 0; g < n_calls; ++g)
    if (call_off[g + 1] < call_off[g]) return gbv_fail(c, GBV_E_ARG, "call offsets not monotone");
  for (size_t i = 0; i < n; ++i)
    if (idx[i] >= c->table_n) return gbv_fail(c, GBV_E_ARG, "validator index out of range");
  // chunk every call exactly like verifySignatureSetsSameMessage (index.ts:218-219)
  std::vector<uint32_t> grp_off, grp_msg;
  grp_off.reserve(n / 64 + n_calls + 1);
  grp_msg.reserve(n / 64 + n_calls + 1);
  for (size_t g = 0; g < n_calls; ++g) {
    uint32_t len = call_off[g + 1] - call_off[g];
    if (len == 0) continue;
    std::vector<uint32_t> co = chunk_offsets(len, MAX_SIGNATURE_SETS_PER_JOB);
    for (size_t j = 0; j + 1 < co.size(); ++j) {
      grp_off.push_back(call_off[g] + co[j]);
      grp_msg.push_back((uint32_t)g);
    }
  }
  grp_off.push_back((uint32_t)n);
  size_t G = grp_msg.size();
  HIP_CHECK(c, hipSetDevice(c->device));
  bool want_msm = c->msm_min && n >= c->msm_min;
  int rc = sm_reserve(c, b, n, G, n_calls, want_msm);
  if (rc) return rc;
  // input blob: idx 4n | sig 96n | set_grp 4n | grp_off 4(G+1) | grp_msg 4G | msgs 32 calls
  size_t o_idx = 0, o_sig = align256(4 * n), o_sg = o_sig + align256(96 * n), o_go = o_sg + align256(4 * n);
  size_t o_gm = o_go + align256(4 * (G + 1)), o_m = o_gm + align256(4 * G), total = o_m + align256(32 * n_calls);
  if (b->in_cap < total) {
    hipFree(b->in_dev);
    hipHostFree(b->in_host);
    b->in_dev = b->in_host = nullptr;
    b->in_cap = 0;
    size_t cap = std::max(total, b->in_cap + b->in_cap / 2);
    HIP_CHECK(c, hipMalloc((void**)&b->in_dev, cap));
    HIP_CHECK(c, hipHostMalloc((void**)&b->in_host, cap, hipHostMallocDefault));
    b->in_cap = cap;
  }
  uint8_t* h = b->in_host;
  if (n) {
    memcpy(h + o_idx, idx, 4 * n);
    memcpy(h + o_sig, sigs96, 96 * n);
    uint32_t* sg = (uint32_t*)(h + o_sg);
    for (size_t g = 0; g < G; ++g)
      for (uint32_t i = grp_off[g]; i < grp_off[g + 1]; ++i) sg[i] = (uint32_t)g;
  }
  memcpy(h + o_go, grp_off.data(), 4 * (G + 1));
  if (G) memcpy(h + o_gm, grp_msg.data(), 4 * G);
  if (n_calls) memcpy(h + o_m, msgs32, 32 * n_calls);
  b->idx = (uint32_t*)(b->in_dev + o_idx);
  b->sig = b->in_dev + o_sig;
  b->set_grp = (uint32_t*)(b->in_dev + o_sg);
  b->grp_off = (uint32_t*)(b->in_dev + o_go);
  b->grp_msg = (uint32_t*)(b->in_dev + o_gm);
  b->msgs = b->in_dev + o_m;
  // no host wait: stream A runs the copy ahead of this batch's kernels (and behind the previous
  // batch's k_sm_prepare); the other streams wait for the event
  if (!b->copied) HIP_CHECK(c, hipEventCreateWithFlags(&b->copied, hipEventDisableTiming));
  HIP_CHECK(c, hipMemcpyAsync(b->in_dev, h, total, hipMemcpyHostToDevice, c->stream));
  HIP_CHECK(c, hipEventRecord(b->copied, c->stream));
  b->n = n;
  b->G = G;
  b->n_calls = n_calls;
  b->grp_off_host.swap(grp_off);
  return GBV_OK;
}

int gbv_sm_batch_create(gbv_ctx* c, size_t n_calls, const uint32_t* call_off, const uint32_t* idx, const uint8_t* sigs96,
                        const uint8_t* msgs32, gbv_sm_batch** out) {
  if (!c || !out) return GBV_E_ARG;
  GBV_LOCK(c);
  if (c->closed) return GBV_E_CLOSED;
  *out = nullptr;
  gbv_sm_batch* b = new gbv_sm_batch();
  int rc = sm_fill(c, b, n_calls, call_off, idx, sigs96, msgs32);
  if (rc) {
    sm_destroy(b);
    return rc;
  }
  *out = b;
  return GBV_OK;
}

int gbv_sm_batch_fill(gbv_ctx* c, gbv_sm_batch* b, size_t n_calls, const uint32_t* call_off, const uint32_t* idx, const uint8_t* sigs96,
                      const uint8_t* msgs32) {
  if (!c || !b) return GBV_E_ARG;
  GBV_LOCK(c);
  if (c->closed) return GBV_E_CLOSED;
  return sm_fill(c, b, n_calls, call_off, idx, sigs96, msgs32);
}

static int sm_submit_enqueue(gbv_ctx* c, gbv_sm_batch* b);

int gbv_sm_batch_submit(gbv_ctx* c, gbv_sm_batch* b) {
  if (!c || !b) return GBV_E_ARG;
  GBV_LOCK(c);
  if (c->closed) return GBV_E_CLOSED;
  if (b->in_flight) return gbv_fail(c, GBV_E_ARG, "batch already in flight");
  HIP_CHECK(c, hipSetDevice(c->device));
  if (b->n == 0) return GBV_OK;
  int rc = sm_submit_enqueue(c, b);
  if (rc) ctx_drain(c);  // kernels enqueued before the failure finish before anything is freed
  else b->in_flight = true;
  return rc;
}

// Pipelined over segments of ~n/S sets (cut at chunk boundaries), all enqueued without a host
// round trip so consecutive submits overlap (the chunk-level tail of batch k runs beside the
// throughput-bound k_sm_prepare of batch k+1):
//   stream H      : k_hash_msgs
//   stream A      : k_sm_prepare(segment s)  -- throughput-bound, also forms per-wave chunk sums
//   streams B0/B1 : (segment s alternates) wait(prepare s) k_sm_chunk_finish, wait(hash) k_sm_miller,
//                   k_seg_reduce_quad + k_sm_seg_check, k_sm_group_pairing (exits at once unless
//                   the segment check failed)
//   stream B0     : wait(all) k_sm_fallback (per-set retry of failed chunks only), copy-out
// Each segment ends in ONE randomised multi-pairing check over all its chunks; only a failing
// segment pays per-chunk checks and only a failing chunk pays per-set retries.
static int sm_submit_enqueue(gbv_ctx* c, gbv_sm_batch* b) {
  KProfScope kp(c->kprof_on ? &b->prof : nullptr);
  Seed seed = fresh_seed();
  uint32_t nonce = c->nonce++;
  // Same-message batches: hash on stream 4, tail on stream 2, every batch (alternating the tails of
  // consecutive batches over two streams buys nothing while the tail is shorter than k_sm_prepare).
  // Invalid-dense regime (a segment failed within the last msm_cooldown_len submits, e.g. C5's 1 %
  // invalid stream): the failure path -- latency-bound run and per-set checks, ~170 ms per 1M
  // sets at 1 % -- goes to streams 4 and 5 (alternating per batch) and the hash to stream A, so batch
  // k's failure path runs beside batch k+1's chunk tail and batch k+1's own failure path.
  ++c->sm_submits;
  const bool dense = c->msm_cooldown != 0;
  hipStream_t sa = c->stream;
  hipStream_t tail = c->stream2, sh = dense ? sa : c->stream4;
  hipStream_t sbs[2] = {tail, tail};
  // failure path + copy-out.  Dense: consecutive batches alternate stream 4 and stream 5 (free on
  // this path), so that batch k's failure path -- a chain of latency-bound pairing phases -- runs
  // beside batch k+1's instead of in front of it (C5 5.67 -> 6.07 M sets/s, 2 batches in flight)
  hipStream_t sf = dense ? ((c->sm_submits & 1) ? c->stream5 : c->stream4) : tail;
  const size_t max_seg = b->seg_cap;
  const size_t n_seg = c->segments;
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
  const size_t msm_min = c->msm_cooldown ? 0 : c->msm_min;
  if (c->msm_cooldown) --c->msm_cooldown;
  bool any_msm = false;
  for (size_t s = 0; s < S; ++s) {
    uint32_t G = gcut[s + 1] - gcut[s];
    size_t ns = b->grp_off_host[gcut[s + 1]] - b->grp_off_host[gcut[s]];
    b->seg_direct[s] = G <= DIRECT_CHUNK_MAX;
    b->seg_msm[s] = msm_min && ns >= msm_min && !b->seg_direct[s];
    any_msm |= b->seg_msm[s] != 0;
  }
  if (any_msm && !b->has_msm) {  // normally allocated when the batch is filled (no hipMalloc while work is queued)
    hipError_t e = msm_alloc(b, b->cap_n);
    if (e != hipSuccess) return gbv_fail(c, GBV_E_OOM, std::string("hipMalloc (msm): ") + hipGetErrorString(e));
    b->has_msm = true;
  }
  // events: [0,1] hash; EPS per segment; then [tail] 2 fallback
  size_t need = 2 + EPS * S + 2;
  b->cur = 0;
  std::vector<hipEvent_t>& evv = b->evs[b->cur];
  if (evv.size() < need) {
    size_t old = evv.size();
    evv.resize(need);
    for (size_t k = old; k < need; ++k) HIP_CHECK(c, hipEventCreateWithFlags(&evv[k], hipEventDefault));
  }
  hipEvent_t* ev = evv.data();
  const size_t part_stride = b->part_stride;
  if (sh != sa) HIP_CHECK(c, hipStreamWaitEvent(sh, b->copied, 0));  // the hash reads the staged messages
  HIP_CHECK(c, hipMemsetAsync(b->n_fallback, 0, 4, sh));
  HIP_CHECK(c, hipMemsetAsync(b->fb_cnt, 0, 8, sh));
  HIP_CHECK(c, hipEventRecord(ev[0], sh));
  launch_hash_msgs(LaunchCfg{blocks_for(b->n_calls), TPB, sh}, b->msgs, (uint32_t)b->n_calls, b->H, b->Hpre);
  HIP_CHECK(c, hipEventRecord(ev[1], sh));
  for (size_t s = 0; s < S; ++s) {
    hipEvent_t* e = ev + 2 + EPS * s;
    hipStream_t sb = sbs[s & 1];
    uint32_t g0 = gcut[s], G = gcut[s + 1] - gcut[s];
    uint32_t s0 = b->grp_off_host[g0], s1 = b->grp_off_host[gcut[s + 1]];
    const bool msm = b->seg_msm[s];
    G2J* Sh = msm ? nullptr : b->rS;  // MSM segment: k_sm_prepare forms the G1 terms only
    HIP_CHECK(c, hipEventRecord(e[0], sa));
    launch_sm_prepare(LaunchCfg{0, 64, sa}, s0, s1 - s0, b->idx, b->sig, b->set_grp, c->table, c->table_ok, (uint32_t)c->table_n,
                      c->comb_on ? c->comb : nullptr, c->comb_ok, seed,
                      nonce, b->S, Sh, b->rP, b->status, b->valid);  // valid: free until the tail's fallback writes it
    HIP_CHECK(c, hipEventRecord(e[1], sa));
    // A segment of a few chunks (a lone gossip call) skips the combined check (seg_direct): each
    // chunk goes straight to its own one-wave check, which is the shorter dependency chain.
    // An MSM segment runs its chunk sums and the bucket MSM on stream A right after its
    // k_sm_prepare (the MSM's bucket pass then has the whole device instead of fighting the next
    // k_sm_prepare for CUs); the tail stream waits for them.  Other segments sum their chunks on
    // the tail stream.
    hipStream_t scf = msm ? sa : sb;
    if (scf != sa) HIP_CHECK(c, hipStreamWaitEvent(scf, e[1], 0));
    HIP_CHECK(c, hipStreamWaitEvent(scf, ev[0], 0));  // n_fallback zeroed (the memsets ahead of the hash)
    HIP_CHECK(c, hipEventRecord(e[2], scf));
    launch_sm_chunk_finish(LaunchCfg{0, 64, scf}, g0, G, s0, b->grp_off, b->status, Sh, b->rP, b->PgJ, b->SgJ, b->grp_state,
                           b->n_fallback);
    HIP_CHECK(c, hipEventRecord(e[3], scf));
    hipStream_t smsm = scf;  // the bucket pass: stream A for an MSM segment
    HIP_CHECK(c, hipEventRecord(e[10], smsm));
    // segment s-2 shares this segment's bucket buffers: its reduction (tail stream) must be done
    if (msm && s >= 2 && b->seg_msm[s - 2]) HIP_CHECK(c, hipStreamWaitEvent(smsm, ev[2 + EPS * (s - 2) + 12], 0));
    if (msm)
      launch_msm_g2_buckets(smsm, s0, s1 - s0, b->set_grp, b->status, b->grp_state, b->S, seed, nonce, b->msm_cnt[s & 1], b->msm_off[s & 1],
                            b->msm_cur[s & 1], b->msm_ent + 4ull * s0, b->msm_buckets[s & 1], b->msm_head[s & 1], b->msm_tail[s & 1]);
    HIP_CHECK(c, hipEventRecord(e[11], smsm));
    if (msm) HIP_CHECK(c, hipStreamWaitEvent(sb, e[3], 0));
    // the hash: the chunk sums above read none of it (a lone call's sums run beside the hash), the
    // Miller values and checks below read H
    HIP_CHECK(c, hipStreamWaitEvent(sb, ev[1], 0));
    HIP_CHECK(c, hipEventRecord(e[4], sb));
    if (!b->seg_direct[s]) launch_sm_miller(LaunchCfg{0, 64, sb}, g0, G, b->grp_msg, b->grp_state, b->PgJ, b->H, b->F);
    HIP_CHECK(c, hipEventRecord(e[5], sb));
    if (msm) {  // the latency-bound bucket reduction overlaps the next k_sm_prepare
      HIP_CHECK(c, hipStreamWaitEvent(sb, e[11], 0));
      launch_msm_g2_reduce(sb, b->msm_buckets[s & 1], b->msm_part[s & 1], b->msm_total + s);
    }
    HIP_CHECK(c, hipEventRecord(e[12], sb));
    HIP_CHECK(c, hipEventRecord(e[6], sb));
    size_t po = (s & 1) * part_stride;
    if (b->seg_direct[s])
      HIP_CHECK(c, hipMemsetAsync(b->seg_ok + s, 0, 1, sb));
    else
      launch_sm_seg_check(LaunchCfg{1, 64, sb}, g0, G, b->grp_state, b->F, b->SgJ, b->Fpart + po, b->Spart + po, b->has + po,
                          b->seg_ok + s, nullptr, msm ? b->msm_total + s : nullptr);
    HIP_CHECK(c, hipEventRecord(e[7], sb));
    HIP_CHECK(c, hipEventRecord(e[8], sb));
    if (msm) {  // per-set / per-chunk G2 sums for the failure path (exit at once when nothing failed)
      launch_sm_redo_g2(LaunchCfg{0, 64, sb}, s0, s1 - s0, b->set_grp, b->status, b->S, seed, nonce, b->seg_ok + s, b->n_fallback, b->rS);
      launch_sm_chunk_finish_s(LaunchCfg{0, 64, sb}, g0, G, s0, b->grp_off, b->grp_state, b->rS, b->seg_ok + s, b->SgJ);
    }
    if (G >= tuning().group_thread_min)
      launch_sm_group_check(LaunchCfg{0, 64, sb}, g0, G, b->F, b->SgJ, b->seg_ok + s, b->grp_state, b->n_fallback);
    else
      launch_sm_group_pairing(LaunchCfg{G, 64, sb}, g0, G, b->grp_msg, b->PgJ, b->SgJ, b->H, b->seg_ok + s, b->grp_state, b->n_fallback,
                              b->Fpair, b->pair_ok);
    HIP_CHECK(c, hipEventRecord(e[9], sb));
  }
  hipEvent_t* ep = ev + 2 + EPS * S;
  // the tail runs on B0 after everything of this batch (B1's last segment included)
  if (S > 1) {
    size_t last_b1 = (S - 1) & 1 ? S - 1 : S - 2;  // last segment that ran on B1
    HIP_CHECK(c, hipStreamWaitEvent(sbs[0], ev[2 + EPS * last_b1 + 9], 0));
  }
  HIP_CHECK(c, hipEventRecord(ep[0], sbs[0]));
  if (sf != sbs[0]) HIP_CHECK(c, hipStreamWaitEvent(sf, ep[0], 0));
  // valid = 1 for the sets of passing chunks; the sets of failed chunks go through 8-set run
  // checks and, for failing runs only, per-set checks (compacted lists, persistent grids)
  launch_sm_fallback(LaunchCfg{blocks_for(b->n), TPB, sf}, (uint32_t)b->n, b->set_grp, b->grp_msg, b->grp_state, b->status, b->idx,
                     c->table, b->S, b->H, b->valid, 0);
  for (size_t s = 0; s < S; ++s) {
    uint32_t s0 = b->grp_off_host[gcut[s]], s1 = b->grp_off_host[gcut[s + 1]];
    launch_sm_fb_runs(LaunchCfg{0, 64, sf}, s0, s1 - s0, b->set_grp, b->grp_state, b->fb_runs, b->fb_cnt, (uint32_t)b->fb_cap);
  }
  // few items: one wave each (latency); many: one thread each (throughput) -- one of each pair exits.
  // The split (gbv_tune "fb_coop_max") is read once, so both kernels of a pair agree on it.
  const uint32_t cm = std::min(tuning().fb_coop_max.load(std::memory_order_relaxed), FB_COOP_CAP);
  launch_sm_fb_blocks_coop(LaunchCfg{0, 64, sf}, b->fb_runs, b->fb_cnt, (uint32_t)b->fb_cap, b->status, b->grp_msg, b->rS, b->rP,
                           b->H, b->valid, b->fb_list, b->fb_cnt + 1, cm);
  launch_sm_fb_blocks(LaunchCfg{FB_GRID, 64, sf}, b->fb_runs, b->fb_cnt, (uint32_t)b->fb_cap, b->status, b->grp_msg, b->rS, b->rP, b->H,
                      b->valid, b->fb_list, b->fb_cnt + 1, cm);
  launch_sm_fb_sets_coop(LaunchCfg{0, 64, sf}, b->fb_list, b->fb_cnt + 1, b->set_grp, b->grp_msg, b->idx, c->table, b->S, b->H,
                         b->valid, b->Ffb, cm);
  launch_sm_fb_sets(LaunchCfg{FB_GRID, 64, sf}, b->fb_list, b->fb_cnt + 1, b->set_grp, b->grp_msg, b->idx, c->table, b->S, b->H,
                    b->valid, cm);
  HIP_CHECK(c, hipEventRecord(ep[1], sf));
  HIP_CHECK(c, hipMemcpyAsync(b->valid_host, b->valid, b->n, hipMemcpyDeviceToHost, sf));
  HIP_CHECK(c, hipMemcpyAsync(b->nfb_host, b->n_fallback, sizeof(uint32_t), hipMemcpyDeviceToHost, sf));
  HIP_CHECK(c, hipMemcpyAsync(b->seg_ok_host, b->seg_ok, S, hipMemcpyDeviceToHost, sf));
  HIP_CHECK(c, hipEventRecord(b->dones[b->cur], sf));
  HIP_CHECK(c, hipGetLastError());
  return GBV_OK;
}

int gbv_sm_batch_wait(gbv_ctx* c, gbv_sm_batch* b, uint8_t* valid) {
  if (!c || !b) return GBV_E_ARG;
  hipEvent_t done = nullptr;
  {
    GBV_LOCK(c);
    if (b->n == 0) return GBV_OK;
    if (!b->in_flight) return gbv_fail(c, GBV_E_ARG, "batch not submitted");
    done = b->dones[b->cur];
  }
  HIP_CHECK(c, hipSetDevice(c->device));
  // block on the device without the context lock (other threads keep submitting); the batch itself
  // belongs to this caller until the wait returns
  hipError_t we = hipEventSynchronize(done);
  GBV_LOCK(c);
  b->in_flight = false;
  if (we != hipSuccess) return gbv_fail(c, GBV_E_DEVICE, std::string("hipEventSynchronize: ") + hipGetErrorString(we));
  if (valid) memcpy(valid, b->valid_host, b->n);
  if (!b->prof.recs.empty()) {
    c->last_ops[0] = kprof_format(b->prof);
    b->prof.reset();
  }
  c->last_fallback_chunks = *b->nfb_host;
  c->last_failed_segments = 0;
  for (size_t s = 0; s < b->n_seg; ++s) {
    bool failed = !(b->seg_ok_host[s] || b->seg_direct[s]);
    c->last_failed_segments += failed ? 1 : 0;
    if (failed && b->seg_msm[s])
      c->msm_cooldown = c->msm_cooldown_len;
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
    hipEvent_t* e = ev + 2 + EPS * s;
    for (int k = 0; k < 5; ++k) acc(1 + k, e[2 * k], e[2 * k + 1]);
    if (b->seg_msm[s]) acc(7, e[10], e[11]);
  }
  hipEvent_t* ep = ev + 2 + EPS * b->n_seg;
  acc(6, ep[0], ep[1]);
  return GBV_OK;
}

int gbv_sm_batch_verify(gbv_ctx* c, gbv_sm_batch* b, uint8_t* valid) {
  if (!c) return GBV_E_ARG;
  int rc = gbv_sm_batch_submit(c, b);  // the batch belongs to the caller: the wait needs no lock held
  if (rc) return rc;
  return gbv_sm_batch_wait(c, b, valid);
}

int gbv_last_ops(gbv_ctx* c, int path, char* out, size_t cap) {
  if (!c || (path != 0 && path != 1) || (cap && !out)) return GBV_E_ARG;
  GBV_LOCK(c);
  const std::string& s = c->last_ops[path];
  if (cap) {
    const size_t k = std::min(s.size(), cap - 1);
    memcpy(out, s.data(), k);
    out[k] = 0;
  }
  return (int)s.size();
}

int gbv_last_stats(gbv_ctx* c, uint32_t* fallback_chunks, uint32_t* failed_segments) {
  if (!c) return GBV_E_ARG;
  GBV_LOCK(c);
  if (fallback_chunks) *fallback_chunks = c->last_fallback_chunks;
  if (failed_segments) *failed_segments = c->last_failed_segments;
  return GBV_OK;
}

int gbv_last_kernel_ms(gbv_ctx* c, float* out, int* launches, int max) {
  if (!c || !out) return 0;
  GBV_LOCK(c);
  int k = std::min(max, (int)gbv_ctx::NK);
  for (int i = 0; i < k; ++i) {
    out[i] = c->last_ms[i];
    if (launches) launches[i] = c->last_launches[i];
  }
  return k;
}

// One-shot calls run through the context's scratch batch: refilled in place, no allocation once
// it has grown to the call size.
int gbv_verify_same_message_multi(gbv_ctx* c, size_t n_calls, const uint32_t* call_off, const uint32_t* idx, const uint8_t* sigs96,
                                  const uint8_t* msgs32, uint8_t* valid) {
  if (!c) return GBV_E_ARG;
  std::lock_guard<std::mutex> sg(c->sm_scratch_mu);  // the scratch batch: one one-shot call at a time
  gbv_sm_batch* b = nullptr;
  {
    GBV_LOCK(c);
    if (c->closed) return GBV_E_CLOSED;
    if (!c->sm_scratch) c->sm_scratch = new gbv_sm_batch();
    b = c->sm_scratch;
    int rc = sm_fill(c, b, n_calls, call_off, idx, sigs96, msgs32);
    if (rc) return rc;
    if ((rc = gbv_sm_batch_submit(c, b))) return rc;
  }
  return gbv_sm_batch_wait(c, b, valid);  // blocks without the context lock
}

int gbv_verify_same_message(gbv_ctx* c, const uint32_t* idx, const uint8_t* sigs96, size_t n, const uint8_t* msg32, uint8_t* valid) {
  uint32_t off[2] = {0, (uint32_t)n};
  return gbv_verify_same_message_multi(c, 1, off, idx, sigs96, msg32, valid);
}

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
  if (!domains32 || n_domains == 0) return gbv_fail(c, GBV_E_ARG, "no domain");
  if (dom_idx)
    for (size_t i = 0; i < n; ++i)
      if (dom_idx[i] >= n_domains) return gbv_fail(c, GBV_E_ARG, "domain index out of range");
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
  if (!c) return GBV_E_ARG;
  GBV_LOCK(c);
  int rc = ssz_begin(c);
  if (rc) return rc;
  if (n == 0) return GBV_OK;
  if (!chunks32 || !out32) return gbv_fail(c, GBV_E_ARG, "null argument");
  if (depth > 24 || (n << depth) >> depth != n || (n << depth) > 0xFFFFFFFFull) return gbv_fail(c, GBV_E_ARG, "tree too large");
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
  if (!c) return GBV_E_ARG;
  GBV_LOCK(c);
  int rc = ssz_begin(c);
  if (rc) return rc;
  if (n == 0) return GBV_OK;
  if (!roots32 || !out32) return gbv_fail(c, GBV_E_ARG, "null argument");
  if (n > 0xFFFFFFFFull) return gbv_fail(c, GBV_E_ARG, "too many roots");
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
  if (!c) return GBV_E_ARG;
  GBV_LOCK(c);
  int rc = ssz_begin(c);
  if (rc) return rc;
  if (n == 0) return GBV_OK;
  if (!data128 || !out32) return gbv_fail(c, GBV_E_ARG, "null argument");
  if (n > 0xFFFFFFFFull) return gbv_fail(c, GBV_E_ARG, "too many objects");
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
  GBV_LOCK(c);
  *ms = c->last_ssz_ms;
  return GBV_OK;
}

// ---- utilities (synthetic workloads, tests) -------------------------------------------------
int gbv_util_sk_to_pk(gbv_ctx* c, const uint8_t* sk32, size_t n, uint8_t* pk48) {
  if (!c || (n && (!sk32 || !pk48))) return GBV_E_ARG;
  GBV_LOCK(c);
  if (n == 0) return GBV_OK;
  HIP_CHECK(c, hipSetDevice(c->device));
  uint8_t* d = nullptr;
  size_t o_pk = align256(32 * n);
  int rc = ctx_small_dev(c, o_pk + 48 * n, &d);
  if (rc) return rc;
  HIP_CHECK(c, hipMemcpyAsync(d, sk32, 32 * n, hipMemcpyHostToDevice, c->stream));
  launch_util_sk_to_pk(LaunchCfg{blocks_for(n), TPB, c->stream}, (uint32_t)n, d, d + o_pk);
  HIP_CHECK(c, hipGetLastError());
  HIP_CHECK(c, hipMemcpyAsync(pk48, d + o_pk, 48 * n, hipMemcpyDeviceToHost, c->stream));
  HIP_CHECK(c, hipStreamSynchronize(c->stream));
  return GBV_OK;
}

int gbv_util_g1_mul_rand(gbv_ctx* c, const uint32_t* slots, const uint64_t* r64, size_t n, int use_comb, uint8_t* out48) {
  if (!c || (n && (!slots || !r64 || !out48))) return GBV_E_ARG;
  GBV_LOCK(c);
  if (n == 0) return GBV_OK;
  if (use_comb && !c->comb_on) return gbv_fail(c, GBV_E_ARG, "comb tables disabled");
  for (size_t i = 0; i < n; ++i)
    if (slots[i] >= c->table_n) return gbv_fail(c, GBV_E_ARG, "slot out of range");
  HIP_CHECK(c, hipSetDevice(c->device));
  uint8_t* d = nullptr;
  size_t o_r = align256(4 * n), o_o = o_r + align256(8 * n);
  int rc = ctx_small_dev(c, o_o + 48 * n, &d);
  if (rc) return rc;
  HIP_CHECK(c, hipMemcpyAsync(d, slots, 4 * n, hipMemcpyHostToDevice, c->stream));
  HIP_CHECK(c, hipMemcpyAsync(d + o_r, r64, 8 * n, hipMemcpyHostToDevice, c->stream));
  launch_util_g1_mul_rand(c->stream, (uint32_t)n, (const uint32_t*)d, (const uint64_t*)(d + o_r), c->table, c->comb, use_comb, d + o_o);
  HIP_CHECK(c, hipGetLastError());
  HIP_CHECK(c, hipMemcpyAsync(out48, d + o_o, 48 * n, hipMemcpyDeviceToHost, c->stream));
  HIP_CHECK(c, hipStreamSynchronize(c->stream));
  return GBV_OK;
}

int gbv_util_hash_to_g2(gbv_ctx* c, const uint8_t* msgs32, size_t n, uint8_t* out192) {
  if (!c || (n && (!msgs32 || !out192))) return GBV_E_ARG;
  GBV_LOCK(c);
  if (n == 0) return GBV_OK;
  HIP_CHECK(c, hipSetDevice(c->device));
  uint8_t* d = nullptr;
  size_t o_o = align256(32 * n), o_h = o_o + align256(192 * n);
  int rc = ctx_small_dev(c, o_h + sizeof(G2A) * n, &d);
  if (rc) return rc;
  HIP_CHECK(c, hipMemcpyAsync(d, msgs32, 32 * n, hipMemcpyHostToDevice, c->stream));
  launch_hash_msgs(LaunchCfg{blocks_for(n), TPB, c->stream}, d, (uint32_t)n, (G2A*)(d + o_h));
  launch_util_g2_out(LaunchCfg{blocks_for(n), TPB, c->stream}, (uint32_t)n, (G2A*)(d + o_h), d + o_o);
  HIP_CHECK(c, hipGetLastError());
  HIP_CHECK(c, hipMemcpyAsync(out192, d + o_o, 192 * n, hipMemcpyDeviceToHost, c->stream));
  HIP_CHECK(c, hipStreamSynchronize(c->stream));
  return GBV_OK;
}

int gbv_util_sign(gbv_ctx* c, const uint8_t* sk32, size_t n, const uint32_t* grp, const uint8_t* msgs32, size_t n_msgs, uint8_t* sig96) {
  if (!c || (n && (!sk32 || !grp || !msgs32 || !sig96))) return GBV_E_ARG;
  GBV_LOCK(c);
  if (n == 0) return GBV_OK;
  for (size_t i = 0; i < n; ++i)
    if (grp[i] >= n_msgs) return gbv_fail(c, GBV_E_ARG, "message index out of range");
  HIP_CHECK(c, hipSetDevice(c->device));
  size_t o_m = align256(32 * n), o_sig = o_m + align256(32 * n_msgs), o_grp = o_sig + align256(96 * n), o_h = o_grp + align256(4 * n);
  uint8_t* d = nullptr;
  int rc = ctx_small_dev(c, o_h + sizeof(G2A) * n_msgs, &d);
  if (rc) return rc;
  G2A* d_H = (G2A*)(d + o_h);
  HIP_CHECK(c, hipMemcpyAsync(d, sk32, 32 * n, hipMemcpyHostToDevice, c->stream));
  HIP_CHECK(c, hipMemcpyAsync(d + o_m, msgs32, 32 * n_msgs, hipMemcpyHostToDevice, c->stream));
  HIP_CHECK(c, hipMemcpyAsync(d + o_grp, grp, 4 * n, hipMemcpyHostToDevice, c->stream));
  launch_hash_msgs(LaunchCfg{blocks_for(n_msgs), TPB, c->stream}, d + o_m, (uint32_t)n_msgs, d_H);
  launch_util_sign(LaunchCfg{blocks_for(n), TPB, c->stream}, (uint32_t)n, d, (const uint32_t*)(d + o_grp), d_H, d + o_sig);
  HIP_CHECK(c, hipGetLastError());
  HIP_CHECK(c, hipMemcpyAsync(sig96, d + o_sig, 96 * n, hipMemcpyDeviceToHost, c->stream));
  HIP_CHECK(c, hipStreamSynchronize(c->stream));
  return GBV_OK;
}

}  // extern "C"

namespace gbv {
static Tuning g_tuning;
static std::once_flag g_tuning_once;
const Tuning& tuning() { return g_tuning; }
void tuning_load() {
  // the only setting taken from the environment: a debugging aid that changes timing, never results
  std::call_once(g_tuning_once, [] {
    if (const char* e = getenv("GBV_SYNC_DEBUG")) g_tuning.sync_debug.store((uint32_t)strtoul(e, nullptr, 10));
  });
}
bool tuning_set(const char* name, uint32_t v) {
  struct { const char* n; std::atomic<uint32_t>* p; } tab[] = {
      {"hash_pair_max", &g_tuning.hash_pair_max}, {"hash_quad_max", &g_tuning.hash_quad_max}, {"hash_coop_max", &g_tuning.hash_coop_max},
      {"prepare_split_max", &g_tuning.prepare_split_max}, {"chunk_finish_wave_max", &g_tuning.chunk_finish_wave_max},
      {"vs_pre_max", &g_tuning.vs_pre_max}, {"vs_fs_maxc", &g_tuning.vs_fs_maxc}, {"vs_quad_max", &g_tuning.vs_quad_max},
      {"vs_pair_max", &g_tuning.vs_pair_max}, {"agg_slice", &g_tuning.agg_slice}, {"fb_coop_max", &g_tuning.fb_coop_max},
      {"group_thread_min", &g_tuning.group_thread_min}, {"sm_quad_max", &g_tuning.sm_quad_max}};
  if (!strcmp(name, "fb_coop_max")) v = std::min(v, FB_COOP_CAP);  // the scratch is sized for the cap
  for (auto& t : tab)
    if (!strcmp(name, t.n)) {
      t.p->store(v, std::memory_order_relaxed);
      return true;
    }
  return false;
}

thread_local KProf* t_kprof = nullptr;

void kprof_begin(hipStream_t s, const char* name, uint32_t threads, uint32_t units) {
  KProf* p = t_kprof;
  if (!p) return;
  while (p->pool.size() < p->used + 2) {
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) {  // no timing for this pass rather than a failed submit
      (void)hipGetLastError();
      t_kprof = nullptr;
      return;
    }
    p->pool.push_back(e);
  }
  KRec r{name, threads, units, p->pool[p->used], p->pool[p->used + 1]};
  p->used += 2;
  (void)hipEventRecord(r.a, s);
  p->recs.push_back(r);
}

void kprof_end(hipStream_t s) {
  KProf* p = t_kprof;
  if (!p || p->recs.empty()) return;
  (void)hipEventRecord(p->recs.back().b, s);
}

void debug_sync(hipStream_t s, const char* kernel) {
  if (!g_tuning.sync_debug) return;
  hipError_t e = hipStreamSynchronize(s);
  if (e == hipSuccess) e = hipGetLastError();
  fprintf(stderr, "[gbv] %s: %s\n", kernel, hipGetErrorString(e));
}
}  // namespace gbv
