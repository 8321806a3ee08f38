// Host side of verifySignatureSets (IBlsVerifier.verifySignatureSets, interface.ts:47;
// BlsMultiThreadWorkerPool.verifySignatureSets, multithread/index.ts:157-207) and of its multi-GPU
// shard form.  Many calls (the pool's jobs) go through ONE device pass:
//
//   stream A : k_vs_agg        one wave per aggregate set: coalesced gather of the set's validator
//                              pubkeys from the HBM table + cross-lane tree sum (aggregatePublicKeys,
//                              bls/utils.ts:5-20; jobItem.ts:55-62)
//              k_vs_hash_sig   two block roles in one launch: hash_to_G2 of every set's signing root,
//                              and per set Signature.fromBytes(sig, true) + pubkey + the randomised
//                              terms r_i pk_i, r_i sig_i (maybeBatch.ts:17-26)
//              k_vs_miller     Miller value f(r_i pk_i, H(m_i)) per set
//   tail     : k_vs_chunk_coop one wave per <=128-set chunk (chunkifyMaximizeChunkSize,
//                              multithread/utils.ts:4-18): product of its Miller values, the
//                              (-g1, sum r_i sig_i) pair and ONE final exponentiation
//
// A call is true iff every chunk is (the AND over jobs, index.ts:185-206); a call with an empty
// aggregate is rejected (aggregatePublicKeys throws EMPTY_AGGREGATE_ARRAY, index.ts:398-412); an
// empty call is false (verifySignatureSetsMaybeBatch([]), maybeBatch.ts:29-31).
#include <cstdlib>

#include "ctx.h"

using namespace gbv;

namespace {
size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }
}  // namespace

struct gbv_vs_batch {
  size_t n = 0, n_calls = 0, C = 0, n_agg = 0, A = 0, n_big = 0, n_slices = 0;
  uint32_t sig_stride = 96;
  size_t cap_n = 0, cap_C = 0;
  bool allocated = false;
  std::vector<uint32_t> call_chunk;  // chunks of call c: [call_chunk[c], call_chunk[c+1])
  std::vector<uint8_t> call_reject;  // call holds an empty aggregate
  std::vector<uint32_t> chunk_off_host;
  uint8_t *in_dev = nullptr, *in_host = nullptr;
  size_t in_cap = 0;
  // inputs (views into in_dev)
  uint32_t *set_off = nullptr, *arena = nullptr, *agg_list = nullptr, *chunk_off = nullptr, *siglen = nullptr;
  uint4 *big = nullptr, *slices = nullptr;  // large aggregates: (set, first slice, count), slice (begin, end)
  uint8_t *raw_flag = nullptr, *raw_pk = nullptr, *msgs = nullptr, *sig = nullptr;
  // work
  G1J* pk = nullptr;  // aggregate pubkeys (Jacobian, k_vs_agg / k_vs_agg_big)
  uint8_t* pk_st = nullptr;
  G1J* agg_part = nullptr;  // slice sums of the large aggregates (grow-only)
  uint8_t* agg_part_bad = nullptr;
  size_t agg_part_cap = 0;
  G2A* H = nullptr;
  G1J* rP = nullptr;
  G2J* rS = nullptr;
  uint8_t* status = nullptr;
  uint8_t* sig_st = nullptr;  // "pre" mode: the signature verdicts alone (k_vs_sig_pre_quad), read by k_vs_chunk_s_miller
  Fp12* F = nullptr;
  G2J* Hpre = nullptr;        // per set: Q0 + Q1 before the cofactor clearing (small passes)
  G2A* Sd = nullptr;          // "pre" mode on lane quads: the decoded signatures (k_vs_sig_decode)
  uint8_t* dec_st = nullptr;  // ... and their GBV_PT_* decode codes
  Fp12* Fs = nullptr;         // per chunk: Miller value of (-g1, sum r_i sig_i) (small passes, k_vs_miller_coop)
  uint8_t* fs_flag = nullptr;
  uint8_t* chunk_valid = nullptr;
  uint8_t* chunk_valid_host = nullptr;  // pinned
  // shard mode (gbv_vs_partial): reduction scratch
  Fp12 *Fpart = nullptr, *f_out = nullptr;
  G2J* Spart = nullptr;
  uint8_t *has = nullptr, *flag = nullptr;
  size_t part_cap = 0;
  uint8_t* part_host = nullptr;  // pinned: the shard's Fp12 then its n status bytes
  size_t part_host_cap = 0;
  bool part_empty = false;
  hipEvent_t ev[7] = {};
  hipEvent_t done = nullptr;
  hipEvent_t copied = nullptr;  // the last fill's input copy (stream A); see gbv_sm_batch::copied
  hipEvent_t pre = nullptr;     // "pre" mode: k_vs_sig_pre_quad done (stream 5)
  bool in_flight = false;
  bool part_in_flight = false;  // gbv_vs_batch_partial_submit'ed, not yet waited
  // a wait is reading this batch without the context lock: a second wait is refused, a fill / submit
  // is refused (in flight), and a destroy is deferred to the end of the wait (free_pending)
  bool waiting = false;
  bool free_pending = false;
  bool fs_small = false;  // this submit forms each chunk's (-g1, sum) Miller value beside the per-set ones
  int tail = 0;
  KProf prof;  // per-kernel events of the last submit / partial (ctx kprof_on)
};

static void vs_free_work(gbv_vs_batch* b) {
  // teardown: a failing free has nothing left to report to
  (void)hipFree(b->pk); (void)hipFree(b->pk_st); (void)hipFree(b->H); (void)hipFree(b->rP); (void)hipFree(b->rS);
  (void)hipFree(b->status); (void)hipFree(b->sig_st); (void)hipFree(b->F); (void)hipFree(b->Fs); (void)hipFree(b->Hpre); (void)hipFree(b->Sd); (void)hipFree(b->dec_st); (void)hipFree(b->fs_flag); (void)hipFree(b->chunk_valid); (void)hipHostFree(b->chunk_valid_host);
  b->pk = nullptr; b->pk_st = nullptr; b->H = nullptr; b->rP = nullptr; b->rS = nullptr; b->status = nullptr; b->sig_st = nullptr; b->F = nullptr; b->Fs = nullptr; b->fs_flag = nullptr; b->Hpre = nullptr; b->Sd = nullptr; b->dec_st = nullptr;
  b->chunk_valid = nullptr; b->chunk_valid_host = nullptr;
  b->allocated = false;
}

void vs_batch_free(gbv_vs_batch* b) {
  if (!b) return;
  if ((b->in_flight || b->part_in_flight) && b->done) (void)hipEventSynchronize(b->done);
  if (b->copied) {
    (void)hipEventSynchronize(b->copied);
    (void)hipEventDestroy(b->copied);
  }
  vs_free_work(b);
  b->prof.destroy();
  hipFree(b->in_dev);
  hipHostFree(b->in_host);
  hipFree(b->Fpart); hipFree(b->Spart); hipFree(b->has); hipFree(b->f_out); hipFree(b->flag);
  hipHostFree(b->part_host);
  hipFree(b->agg_part); hipFree(b->agg_part_bad);
  for (auto e : b->ev)
    if (e) hipEventDestroy(e);
  if (b->done) hipEventDestroy(b->done);
  if (b->pre) hipEventDestroy(b->pre);
  delete b;
}

static int vs_reserve(gbv_ctx* c, gbv_vs_batch* b, size_t n, size_t C) {
  if (b->allocated && n <= b->cap_n && C <= b->cap_C) return GBV_OK;
  if (b->allocated) {
    n = std::max(n, b->cap_n);
    C = std::max(C, b->cap_C);
    vs_free_work(b);
  }
  hipError_t e = hipSuccess;
  auto chk = [&](hipError_t x) { if (x != hipSuccess && e == hipSuccess) e = x; };
  chk(dalloc(&b->pk, n)); chk(dalloc(&b->pk_st, n)); chk(dalloc(&b->H, n)); chk(dalloc(&b->rP, n)); chk(dalloc(&b->rS, n));
  chk(dalloc(&b->status, n)); chk(dalloc(&b->sig_st, n)); chk(dalloc(&b->F, n)); chk(dalloc(&b->chunk_valid, C));
  chk(dalloc(&b->Fs, C)); chk(dalloc(&b->fs_flag, C)); chk(dalloc(&b->Hpre, n));
  chk(dalloc(&b->Sd, n)); chk(dalloc(&b->dec_st, n));
  chk(hipHostMalloc((void**)&b->chunk_valid_host, std::max<size_t>(C, 1), hipHostMallocDefault));
  for (auto& ev : b->ev)
    if (!ev) chk(hipEventCreate(&ev));
  if (!b->done) chk(hipEventCreateWithFlags(&b->done, hipEventDisableTiming));
  if (!b->pre) chk(hipEventCreateWithFlags(&b->pre, hipEventDisableTiming));
  if (e != hipSuccess) {
    vs_free_work(b);
    return gbv_fail(c, GBV_E_OOM, std::string("hipMalloc: ") + hipGetErrorString(e));
  }
  b->allocated = true;
  b->cap_n = n;
  b->cap_C = C;
  return GBV_OK;
}

// Stage n_calls calls (CSR call_off over sets) in b.  Argument errors fail the whole fill;
// empty aggregates only mark their call rejected.
static int vs_fill(gbv_ctx* c, gbv_vs_batch* b, size_t n_calls, const uint32_t* call_off, const gbv_set* sets, const uint32_t* arena) {
  if (b->in_flight || b->part_in_flight) return gbv_fail(c, GBV_E_ARG, "batch in flight");
  if (n_calls && !call_off) return gbv_fail(c, GBV_E_ARG, "null call offsets");
  if (b->copied) HIP_CHECK(c, hipEventSynchronize(b->copied));  // the pinned blob is free again
  size_t n = n_calls ? call_off[n_calls] : 0;
  if (call_off && call_off[0] != 0) return gbv_fail(c, GBV_E_ARG, "call offsets must start at 0");
  const uint32_t slice = std::max<uint32_t>(tuning().agg_slice, 256);  // members per k_vs_agg_big workgroup
  for (size_t g = 0; g < n_calls; ++g)
    if (call_off[g + 1] < call_off[g]) return gbv_fail(c, GBV_E_ARG, "call offsets not monotone");
  if (n && !sets) return gbv_fail(c, GBV_E_ARG, "null sets");
  if (n > 0x7FFFFFFFull) return gbv_fail(c, GBV_E_ARG, "too many sets");
  std::vector<uint8_t> reject(n_calls, 0);
  size_t A = 0, n_agg = 0, n_big = 0, n_slices = 0;
  uint32_t stride = 96;
  for (size_t g = 0; g < n_calls; ++g)
    for (uint32_t i = call_off[g]; i < call_off[g + 1]; ++i) {
      const gbv_set& s = sets[i];
      if (!s.msg32 || (!s.sig && s.sig_len)) return gbv_fail(c, GBV_E_ARG, "null msg/sig");
      if (s.sig_len == 192) stride = 192;
      if (s.raw_pk48) continue;
      if (s.idx_len == 0) {
        reject[g] = 1;
        continue;
      }
      if (!arena) return gbv_fail(c, GBV_E_ARG, "null index arena");
      for (uint32_t j = 0; j < s.idx_len; ++j)
        if (arena[s.idx_off + j] >= c->table_n) return gbv_fail(c, GBV_E_ARG, "validator index out of range");
      A += s.idx_len;
      if (s.idx_len >= AGG_BIG_MIN) {
        ++n_big;
        n_slices += (s.idx_len + slice - 1) / slice;
      } else if (s.idx_len >= 2) {
        ++n_agg;
      }
    }
  // chunks: chunkifyMaximizeChunkSize(call, 128) per non-empty, non-rejected call
  std::vector<uint32_t> chunk_off, call_chunk(n_calls + 1, 0);
  for (size_t g = 0; g < n_calls; ++g) {
    call_chunk[g] = (uint32_t)chunk_off.size();
    uint32_t len = call_off[g + 1] - call_off[g];
    if (len == 0 || reject[g]) continue;
    std::vector<uint32_t> co = chunk_offsets(len, MAX_SIGNATURE_SETS_PER_JOB);
    for (size_t j = 0; j + 1 < co.size(); ++j) chunk_off.push_back(call_off[g] + co[j]);
  }
  call_chunk[n_calls] = (uint32_t)chunk_off.size();
  size_t C = chunk_off.size();
  // chunk ends: chunk k ends where the next chunk of the same call starts, or at its call's end
  std::vector<uint32_t> chunk_end(C);
  for (size_t g = 0; g < n_calls; ++g)
    for (uint32_t k = call_chunk[g]; k < call_chunk[g + 1]; ++k) chunk_end[k] = k + 1 < call_chunk[g + 1] ? chunk_off[k + 1] : call_off[g + 1];
  HIP_CHECK(c, hipSetDevice(c->device));
  int rc = vs_reserve(c, b, n, C);
  if (rc) return rc;
  if (b->agg_part_cap < n_slices) {
    // grow geometrically (each larger Electra aggregate would otherwise free + allocate, and a
    // hipFree synchronises the device under the passes in flight)
    const size_t cap = std::max(n_slices, 2 * b->agg_part_cap);
    hipFree(b->agg_part);
    hipFree(b->agg_part_bad);
    b->agg_part = nullptr;
    b->agg_part_bad = nullptr;
    b->agg_part_cap = 0;
    HIP_CHECK(c, dalloc(&b->agg_part, cap));
    HIP_CHECK(c, dalloc(&b->agg_part_bad, cap));
    b->agg_part_cap = cap;
  }
  // input blob: set_off 4(n+1) | arena 4A | agg_list 4 n_agg | chunk (begin,end) 8C | siglen 4n | raw_flag n |
  //             raw_pk 48n | msgs 32n | sig stride*n | big 16 n_big | slices 16 n_slices
  size_t o_so = 0, o_ar = align256(4 * (n + 1)), o_al = o_ar + align256(4 * A), o_co = o_al + align256(4 * n_agg);
  size_t o_sl = o_co + align256(8 * C), o_rf = o_sl + align256(4 * n), o_rp = o_rf + align256(n), o_m = o_rp + align256(48 * n);
  size_t o_sig = o_m + align256(32 * n), o_big = o_sig + align256((size_t)stride * n), o_slc = o_big + align256(16 * n_big);
  size_t total = o_slc + align256(16 * n_slices);
  if (b->in_cap < total) {
    hipFree(b->in_dev);
    hipHostFree(b->in_host);
    b->in_dev = b->in_host = nullptr;
    size_t cap = std::max(total, b->in_cap + b->in_cap / 2);
    b->in_cap = 0;
    HIP_CHECK(c, hipMalloc((void**)&b->in_dev, cap));
    HIP_CHECK(c, hipHostMalloc((void**)&b->in_host, cap, hipHostMallocDefault));
    b->in_cap = cap;
  }
  uint8_t* h = b->in_host;
  uint32_t* so = (uint32_t*)(h + o_so);
  uint32_t* ar = (uint32_t*)(h + o_ar);
  uint32_t* al = (uint32_t*)(h + o_al);
  uint32_t* co = (uint32_t*)(h + o_co);
  uint32_t* sl = (uint32_t*)(h + o_sl);
  uint8_t* rf = h + o_rf;
  uint4* bg = (uint4*)(h + o_big);
  uint4* slc = (uint4*)(h + o_slc);
  size_t a = 0, na = 0, nb = 0, ns = 0;
  for (size_t i = 0; i < n; ++i) {
    const gbv_set& s = sets[i];
    so[i] = (uint32_t)a;
    rf[i] = s.raw_pk48 ? 1 : 0;
    if (s.raw_pk48) {
      memcpy(h + o_rp + 48 * i, s.raw_pk48, 48);
    } else if (s.idx_len) {
      memcpy(ar + a, arena + s.idx_off, 4 * (size_t)s.idx_len);
      if (s.idx_len >= AGG_BIG_MIN) {
        const uint32_t k = (s.idx_len + slice - 1) / slice;
        bg[nb++] = make_uint4((uint32_t)i, (uint32_t)ns, k, 0);
        for (uint32_t q = 0; q < k; ++q)
          slc[ns++] = make_uint4((uint32_t)a + q * slice, (uint32_t)a + std::min(s.idx_len, (q + 1) * slice), 0, 0);
      } else if (s.idx_len >= 2) {
        al[na++] = (uint32_t)i;
      }
      a += s.idx_len;
    }
    memcpy(h + o_m + 32 * i, s.msg32, 32);
    uint32_t L = s.sig_len;
    sl[i] = (L == 96 || L == 192) ? L : 0;  // other lengths: BAD_ENCODING -> false
    uint8_t* dst = h + o_sig + (size_t)stride * i;
    if (sl[i]) memcpy(dst, s.sig, L);
    if (sl[i] < stride) memset(dst + sl[i], 0, stride - sl[i]);
  }
  so[n] = (uint32_t)a;
  // k_vs_agg runs 8 sets per wave: sets of similar size share a wave (largest first), so a 512-member
  // sync aggregate does not hold a wave of 128-member committees for 4x their time
  std::stable_sort(al, al + na, [&](uint32_t x, uint32_t y) { return sets[x].idx_len > sets[y].idx_len; });
  for (size_t k = 0; k < C; ++k) {
    co[2 * k] = chunk_off[k];
    co[2 * k + 1] = chunk_end[k];
  }
  b->set_off = (uint32_t*)(b->in_dev + o_so);
  b->arena = (uint32_t*)(b->in_dev + o_ar);
  b->agg_list = (uint32_t*)(b->in_dev + o_al);
  b->chunk_off = (uint32_t*)(b->in_dev + o_co);
  b->siglen = (uint32_t*)(b->in_dev + o_sl);
  b->raw_flag = b->in_dev + o_rf;
  b->raw_pk = b->in_dev + o_rp;
  b->msgs = b->in_dev + o_m;
  b->sig = b->in_dev + o_sig;
  b->big = (uint4*)(b->in_dev + o_big);
  b->slices = (uint4*)(b->in_dev + o_slc);
  // no host wait: stream A runs the copy ahead of the batch's kernels, other streams wait for the event
  if (!b->copied) HIP_CHECK(c, hipEventCreateWithFlags(&b->copied, hipEventDisableTiming));
  HIP_CHECK(c, hipMemcpyAsync(b->in_dev, h, total, hipMemcpyHostToDevice, c->stream));
  HIP_CHECK(c, hipEventRecord(b->copied, c->stream));
  b->n = n;
  b->n_calls = n_calls;
  b->C = C;
  b->n_agg = n_agg;
  b->n_big = n_big;
  b->n_slices = n_slices;
  b->A = A;
  b->sig_stride = stride;
  b->call_chunk.swap(call_chunk);
  b->call_reject.swap(reject);
  b->chunk_off_host.swap(chunk_off);
  return GBV_OK;
}

// "pre" mode for passes of at most tuning().vs_pre_max sets: k_vs_sig_decode + k_vs_sig_pre_quad and k_vs_pk_rand_quad in place of
// k_vs_hash_sig's signature roles
static bool vs_pre_on(const gbv_vs_batch* b) { return b->n <= tuning().vs_pre_max; }

// Small passes, and passes of few chunks (a range-sync segment of blocks: 2 chunks per block), whose
// chunk checks are latency-bound: each chunk's (-g1, sum r_i sig_i) Miller value is formed beside the
// per-set ones instead of inside the chunk check.
static bool vs_fs_small(const gbv_vs_batch* b) { return b->n <= VS_COOP_MILLER_MAX || b->C <= tuning().vs_fs_maxc.load(std::memory_order_relaxed); }

// Per-set kernels: aggregate and hash + signature + randomisation on stream A, the Miller values on
// stream m (a tail stream, so that they overlap the next batch's stream-A kernels; or stream A).
// Events: ev0 agg ev1 hash_sig ev2 | (m) ev3 miller ev4.
// with_fs: the chunk checks follow (gbv_vs_batch_submit), so a small pass also forms each chunk's
// (-g1, sum r_i sig_i) Miller value beside the per-set ones.  partial: a shard's Fp12 partial follows
// (gbv_vs_partial); it takes the same split of the signature half (pre mode) and the hash on stream m.
static int vs_enqueue_sets(gbv_ctx* c, gbv_vs_batch* b, hipStream_t m, bool with_fs, bool partial = false) {
  hipStream_t s = c->stream;
  Seed seed = fresh_seed();
  uint32_t nonce = c->nonce++;
  // passes up to GBV_VS_PRE_MAX sets: the signature half first, on stream 5, beside the aggregation below
  const bool small = with_fs && b->fs_small;  // decided once per submit (vs_submit_enqueue): the chunk checks read the same
  const bool pre = (with_fs || partial) && m != s && vs_pre_on(b);
  if (pre) {
    HIP_CHECK(c, hipStreamWaitEvent(c->stream5, b->copied, 0));
    launch_vs_sig_pre(c->stream5, (uint32_t)b->n, b->sig, b->sig_stride, b->siglen, seed, nonce, b->rS, b->status, b->sig_st, b->Sd,
                      b->dec_st);
    HIP_CHECK(c, hipEventRecord(b->pre, c->stream5));
    if (small) {
      // each chunk's sum r_i sig_i and its (-g1, sum) Miller value need no pubkey either: they follow
      // on stream 5 (a chunk with a rejected pubkey is caught by the chunk check's own status scan)
      launch_vs_chunk_s_miller(c->stream5, (uint32_t)b->C, b->sig_st, b->chunk_off, b->rS, b->Fs, b->fs_flag);
      HIP_CHECK(c, hipEventRecord(b->ev[6], c->stream5));
    }
  }
  HIP_CHECK(c, hipEventRecord(b->ev[0], s));
  if (b->n_agg) launch_vs_agg(LaunchCfg{(unsigned)b->n_agg, 64, s}, b->agg_list, b->set_off, b->arena, c->table, c->table_ok, b->pk, b->pk_st);
  launch_vs_agg_big(s, (uint32_t)b->n_slices, b->slices, (uint32_t)b->n_big, b->big, b->arena, c->table, c->table_ok, b->agg_part,
                    b->agg_part_bad, b->pk, b->pk_st);
  HIP_CHECK(c, hipEventRecord(b->ev[1], s));
  // small passes and pre mode: the hash on stream m (for few messages lane-pair maps and the
  // cooperative cofactor clearing) beside the signature work
  const bool split = (with_fs || partial) && m != s && (small || pre);
  if (split) HIP_CHECK(c, hipStreamWaitEvent(m, b->copied, 0));
  if (split) launch_hash_msgs(LaunchCfg{blocks_for(b->n), TPB, m}, b->msgs, (uint32_t)b->n, b->H, b->Hpre);
  if (pre) {
    HIP_CHECK(c, hipStreamWaitEvent(s, b->pre, 0));
    launch_vs_pk_rand(s, (uint32_t)b->n, b->set_off, b->arena, b->raw_flag, b->raw_pk, c->table, c->table_ok, b->pk, b->pk_st, seed, nonce,
                      b->rP, b->status);
  } else {
    launch_vs_hash_sig(s, (uint32_t)b->n, b->msgs, b->set_off, b->arena, b->raw_flag, b->raw_pk, b->sig, b->sig_stride, b->siglen, c->table,
                       c->table_ok, b->pk, b->pk_st, seed, nonce, b->H, b->rP, b->rS, b->status, split);
  }
  HIP_CHECK(c, hipEventRecord(b->ev[2], s));
  if (m != s) HIP_CHECK(c, hipStreamWaitEvent(m, b->ev[2], 0));
  HIP_CHECK(c, hipEventRecord(b->ev[3], m));
  if (b->n <= VS_COOP_MILLER_MAX)  // latency: one wave per set (cooperative Miller loop)
    launch_vs_miller_coop(m, (uint32_t)b->n, b->status, b->rP, b->H, b->F);
  else
    launch_vs_miller(LaunchCfg{blocks_for(b->n), TPB, m}, (uint32_t)b->n, b->status, b->rP, b->H, b->F);
  HIP_CHECK(c, hipEventRecord(b->ev[4], m));
  if (pre && small) {
    HIP_CHECK(c, hipStreamWaitEvent(m, b->ev[6], 0));
  } else if (small) {  // beside the per-set Miller values, on stream A (free after hash_sig)
    launch_vs_chunk_s_miller(s, (uint32_t)b->C, b->status, b->chunk_off, b->rS, b->Fs, b->fs_flag);
    HIP_CHECK(c, hipEventRecord(b->ev[6], s));
    if (m != s) HIP_CHECK(c, hipStreamWaitEvent(m, b->ev[6], 0));
  }
  HIP_CHECK(c, hipGetLastError());
  return GBV_OK;
}

extern "C" {

int gbv_vs_batch_create(gbv_ctx* c, size_t n_calls, const uint32_t* call_off, const gbv_set* sets, const uint32_t* arena,
                        gbv_vs_batch** out) {
  if (!c || !out) return GBV_E_ARG;
  GBV_LOCK(c);
  if (c->closed) return GBV_E_CLOSED;
  *out = nullptr;
  gbv_vs_batch* b = new gbv_vs_batch();
  int rc = vs_fill(c, b, n_calls, call_off, sets, arena);
  if (rc) {
    vs_batch_free(b);
    return rc;
  }
  *out = b;
  return GBV_OK;
}

void gbv_vs_batch_destroy(gbv_ctx* c, gbv_vs_batch* b) {
  if (c) {
    GBV_LOCK(c);
    if (b && b->waiting) {  // a wait is reading it: that wait frees it when it is done
      b->free_pending = true;
      return;
    }
    vs_batch_free(b);
  } else {
    vs_batch_free(b);
  }
}

int gbv_vs_batch_fill(gbv_ctx* c, gbv_vs_batch* b, size_t n_calls, const uint32_t* call_off, const gbv_set* sets, const uint32_t* arena) {
  if (!c || !b) return GBV_E_ARG;
  GBV_LOCK(c);
  if (c->closed) return GBV_E_CLOSED;
  return vs_fill(c, b, n_calls, call_off, sets, arena);
}

static int vs_submit_enqueue(gbv_ctx* c, gbv_vs_batch* b) {
  KProfScope kp(c->kprof_on ? &b->prof : nullptr);
  b->fs_small = vs_fs_small(b);  // one read of the setting for both the Miller stage and the chunk checks
  b->tail = (int)(c->sm_submits++ & 1);
  hipStream_t t = b->tail ? c->stream4 : c->stream2;
  int rc = vs_enqueue_sets(c, b, t, true);
  if (rc) return rc;
  const bool fs = b->fs_small;
  launch_vs_chunk_coop(LaunchCfg{(unsigned)b->C, 64, t}, (uint32_t)b->C, b->chunk_off, b->status, b->F, b->rS, b->chunk_valid,
                       fs ? b->Fs : nullptr, b->fs_flag);
  HIP_CHECK(c, hipEventRecord(b->ev[5], t));
  HIP_CHECK(c, hipMemcpyAsync(b->chunk_valid_host, b->chunk_valid, b->C, hipMemcpyDeviceToHost, t));
  HIP_CHECK(c, hipEventRecord(b->done, t));
  HIP_CHECK(c, hipGetLastError());
  return GBV_OK;
}

// Enqueue the whole verification without a host round trip: the per-set kernels on stream A, the
// Miller values and chunk checks on a tail stream, alternating per submit between stream 2 and the
// hash stream (idle in this path), so that consecutive batches' tails overlap each other and the
// next batch's per-set kernels; small passes add stream 5 for the signature half (four busy streams
// at most over the GPU_MAX_HW_QUEUES=4 hardware queues; ctx.h).
int gbv_vs_batch_submit(gbv_ctx* c, gbv_vs_batch* b) {
  if (!c || !b) return GBV_E_ARG;
  GBV_LOCK(c);
  if (c->closed) return GBV_E_CLOSED;
  if (b->in_flight || b->part_in_flight) return gbv_fail(c, GBV_E_ARG, "batch already in flight");
  HIP_CHECK(c, hipSetDevice(c->device));
  if (b->n == 0 || b->C == 0) return GBV_OK;
  int rc = vs_submit_enqueue(c, b);
  if (rc) ctx_drain(c);  // kernels enqueued before the failure finish before anything is freed
  else b->in_flight = true;
  return rc;
}

int gbv_vs_batch_wait(gbv_ctx* c, gbv_vs_batch* b, uint8_t* call_valid) {
  if (!c || !b) return GBV_E_ARG;
  HIP_CHECK(c, hipSetDevice(c->device));
  bool flying;
  {
    GBV_LOCK(c);
    if (b->waiting) return gbv_fail(c, GBV_E_ARG, "batch already being waited on");
    flying = b->in_flight;
    b->waiting = flying;
  }
  // the device wait runs without the context lock; in_flight stays set (fill / submit refuse the batch)
  // and a destroy meanwhile is deferred to the end of this call
  hipError_t we = flying ? hipEventSynchronize(b->done) : hipSuccess;
  GBV_LOCK(c);
  struct FreeIfPending {  // runs last, after the results below are read
    gbv_vs_batch* b;
    ~FreeIfPending() {
      b->waiting = false;
      if (b->free_pending) vs_batch_free(b);
    }
  } fin{b};
  if (flying) {
    b->in_flight = false;
    if (we != hipSuccess) return gbv_fail(c, GBV_E_DEVICE, std::string("hipEventSynchronize: ") + hipGetErrorString(we));
    float ms[4] = {};
    const int from[4] = {0, 1, 3, 4};  // agg, hash_sig, miller, chunk checks
    for (int k = 0; k < 4; ++k)
      if (hipEventElapsedTime(&ms[k], b->ev[from[k]], b->ev[from[k] + 1]) != hipSuccess) ms[k] = 0.f;
    memcpy(c->last_vs_ms, ms, sizeof ms);
    if (!b->prof.recs.empty()) {
      c->last_ops[1] = kprof_format(b->prof);
      b->prof.reset();
    }
  } else if (b->n && b->C) {
    return gbv_fail(c, GBV_E_ARG, "batch not submitted");
  }
  if (call_valid)
    for (size_t g = 0; g < b->n_calls; ++g) {
      uint32_t k0 = b->call_chunk[g], k1 = b->call_chunk[g + 1];
      uint8_t all = k1 > k0 ? 1 : 0;  // an empty call is false
      for (uint32_t k = k0; k < k1; ++k) all &= b->chunk_valid_host[k];
      call_valid[g] = b->call_reject[g] ? GBV_CALL_REJECTED : all;
    }
  return GBV_OK;
}

int gbv_vs_last_kernel_ms(gbv_ctx* c, float* ms4) {
  if (!c || !ms4) return GBV_E_ARG;
  GBV_LOCK(c);
  memcpy(ms4, c->last_vs_ms, sizeof c->last_vs_ms);
  return GBV_OK;
}

static gbv_vs_batch* scratch(gbv_ctx* c) {
  if (!c->vs_scratch) c->vs_scratch = new gbv_vs_batch();
  return c->vs_scratch;
}

int gbv_verify_sets_multi(gbv_ctx* c, size_t n_calls, const uint32_t* call_off, const gbv_set* sets, const uint32_t* arena,
                          uint8_t* call_valid) {
  if (!c || (n_calls && !call_valid)) return GBV_E_ARG;
  std::lock_guard<std::mutex> sg(c->vs_scratch_mu);  // the scratch batch: one one-shot call at a time
  gbv_vs_batch* b = nullptr;
  {
    GBV_LOCK(c);
    if (c->closed) return GBV_E_CLOSED;
    b = scratch(c);
    int rc = vs_fill(c, b, n_calls, call_off, sets, arena);
    if (rc) return rc;
    if ((rc = gbv_vs_batch_submit(c, b))) return rc;
  }
  return gbv_vs_batch_wait(c, b, call_valid);  // blocks without the context lock
}

int gbv_verify_sets(gbv_ctx* c, const gbv_set* sets, size_t n, const uint32_t* arena, uint8_t* all_valid, uint8_t* chunk_valid) {
  if (!c || !all_valid) return GBV_E_ARG;
  std::lock_guard<std::mutex> sg(c->vs_scratch_mu);
  *all_valid = 0;
  uint32_t off[2] = {0, (uint32_t)n};
  gbv_vs_batch* b = nullptr;
  {
    GBV_LOCK(c);
    if (c->closed) return GBV_E_CLOSED;
    b = scratch(c);
    int rc = vs_fill(c, b, 1, off, sets, arena);
    if (rc) return rc;
    // aggregatePublicKeys([]) throws before any verification: the call rejects (index.ts:398-412)
    if (b->call_reject[0]) return gbv_fail(c, GBV_E_EMPTY_AGGREGATE, "EMPTY_AGGREGATE_ARRAY");
    if ((rc = gbv_vs_batch_submit(c, b))) return rc;
  }
  uint8_t v = 0;
  int rc = gbv_vs_batch_wait(c, b, &v);
  if (rc) return rc;
  *all_valid = v;
  if (chunk_valid) {
    if (b->C)
      memcpy(chunk_valid, b->chunk_valid_host, b->C);
    else
      chunk_valid[0] = 0;  // verifySignatureSetsMaybeBatch([]) throws -> false (maybeBatch.ts:29-31,39-44)
  }
  return GBV_OK;
}

// One shard of a verifySignatureSets call spread over several GPUs: the shard's sets
// reduce to ONE Fp12 Miller product (its pairs and its own (-g1, sum r_i sig_i) pair).  Enqueued
// under the context lock, collected without it.
static int vs_partial_enqueue(gbv_ctx* c, gbv_vs_batch* b);
static int vs_partial_collect(gbv_ctx* c, gbv_vs_batch* b, uint8_t out576[GBV_FP12_PARTIAL_BYTES], uint8_t* shard_ok);

int gbv_vs_partial(gbv_ctx* c, const gbv_set* sets, size_t n, const uint32_t* arena, uint8_t out576[GBV_FP12_PARTIAL_BYTES],
                   uint8_t* shard_ok) {
  if (!c || !out576 || !shard_ok) return GBV_E_ARG;
  std::lock_guard<std::mutex> sg(c->vs_scratch_mu);
  *shard_ok = 1;
  uint32_t off[2] = {0, (uint32_t)n};
  gbv_vs_batch* b = nullptr;
  {
    GBV_LOCK(c);
    if (c->closed) return GBV_E_CLOSED;
    b = scratch(c);
    int rc = vs_fill(c, b, 1, off, sets, arena);
    if (rc) return rc;
    if (b->call_reject[0]) return gbv_fail(c, GBV_E_EMPTY_AGGREGATE, "EMPTY_AGGREGATE_ARRAY");
    if ((rc = vs_partial_enqueue(c, b))) return rc;
  }
  return vs_partial_collect(c, b, out576, shard_ok);
}

int gbv_vs_batch_partial_submit(gbv_ctx* c, gbv_vs_batch* b) {
  if (!c || !b) return GBV_E_ARG;
  GBV_LOCK(c);
  if (c->closed) return GBV_E_CLOSED;
  if (b->in_flight || b->part_in_flight) return gbv_fail(c, GBV_E_ARG, "batch in flight");
  for (uint8_t r : b->call_reject)
    if (r) return gbv_fail(c, GBV_E_EMPTY_AGGREGATE, "EMPTY_AGGREGATE_ARRAY");
  int rc = vs_partial_enqueue(c, b);
  if (rc) return rc;
  b->part_in_flight = true;
  return GBV_OK;
}

int gbv_vs_batch_partial_wait(gbv_ctx* c, gbv_vs_batch* b, uint8_t out576[GBV_FP12_PARTIAL_BYTES], uint8_t* shard_ok) {
  if (!c || !b || !out576 || !shard_ok) return GBV_E_ARG;
  {
    GBV_LOCK(c);
    if (!b->part_in_flight) return gbv_fail(c, GBV_E_ARG, "partial not submitted");
    if (b->waiting) return gbv_fail(c, GBV_E_ARG, "partial already being waited on");
    // collected below without the lock: part_in_flight stays set until then (fill / submit refuse the
    // batch, so part_host is neither regrown nor refilled) and a destroy is deferred to the end
    b->waiting = true;
  }
  *shard_ok = 1;
  const int rc = vs_partial_collect(c, b, out576, shard_ok);
  GBV_LOCK(c);
  b->part_in_flight = false;
  b->waiting = false;
  if (b->free_pending) vs_batch_free(b);
  return rc;
}

int gbv_vs_batch_partial(gbv_ctx* c, gbv_vs_batch* b, uint8_t out576[GBV_FP12_PARTIAL_BYTES], uint8_t* shard_ok) {
  if (!c || !b || !out576 || !shard_ok) return GBV_E_ARG;
  *shard_ok = 1;
  int rc = gbv_vs_batch_partial_submit(c, b);
  if (rc) return rc;
  return gbv_vs_batch_partial_wait(c, b, out576, shard_ok);
}

static int vs_partial_enqueue(gbv_ctx* c, gbv_vs_batch* b) {
  const size_t n = b->n;
  int rc;
  b->part_empty = n == 0;
  if (n == 0) return GBV_OK;
  size_t np = seg_reduce_scratch(n);
  if (b->part_cap < np) {
    hipFree(b->Fpart); hipFree(b->Spart); hipFree(b->has); hipFree(b->f_out); hipFree(b->flag);
    b->Fpart = nullptr; b->Spart = nullptr; b->has = nullptr; b->f_out = nullptr; b->flag = nullptr;
    b->part_cap = 0;
    HIP_CHECK(c, dalloc(&b->Fpart, np)); HIP_CHECK(c, dalloc(&b->Spart, np)); HIP_CHECK(c, dalloc(&b->has, np));
    HIP_CHECK(c, dalloc(&b->f_out, 1)); HIP_CHECK(c, dalloc(&b->flag, 1));
    b->part_cap = np;
  }
  if (b->part_host_cap < sizeof(Fp12) + n) {
    // grow geometrically (computed before the old capacity is dropped): a hipHostFree synchronises
    // the device under the passes in flight
    const size_t cap = std::max(sizeof(Fp12) + n, 2 * b->part_host_cap);
    hipHostFree(b->part_host);
    b->part_host = nullptr;
    b->part_host_cap = 0;
    HIP_CHECK(c, hipHostMalloc((void**)&b->part_host, cap, hipHostMallocDefault));
    b->part_host_cap = cap;
  }
  HIP_CHECK(c, hipSetDevice(c->device));
  KProfScope kp(c->kprof_on ? &b->prof : nullptr);
  // a shard of up to vs_pre_max sets (a per-GPU share of one large call at N = 8): the hash on the
  // tail stream beside the split signature / pubkey halves, the rest on the tail stream after them;
  // larger shards: the per-set kernels on stream A, the Miller values and the reduction on the tail.
  // The tail alternates per submit (stream 2 / stream 4) so that streamed shard passes overlap.
  hipStream_t s = (c->sm_submits++ & 1) ? c->stream4 : c->stream2;
  if ((rc = vs_enqueue_sets(c, b, s, false, true))) {
    ctx_drain(c);
    return rc;
  }
  // status doubles as the per-"chunk" state: SET_OK == GRP_PENDING (every valid set takes part);
  // the reduction is a tree over 64-set blocks (k_seg_reduce_quad)
  launch_sm_seg_check(LaunchCfg{1, 64, s}, 0, (uint32_t)n, b->status, b->F, b->rS, b->Fpart, b->Spart, b->has, b->flag, b->f_out);
  HIP_CHECK_DRAIN(c, hipGetLastError());
  HIP_CHECK_DRAIN(c, hipMemcpyAsync(b->part_host, b->f_out, sizeof(Fp12), hipMemcpyDeviceToHost, s));
  HIP_CHECK_DRAIN(c, hipMemcpyAsync(b->part_host + sizeof(Fp12), b->status, n, hipMemcpyDeviceToHost, s));
  HIP_CHECK_DRAIN(c, hipEventRecord(b->done, s));
  return GBV_OK;
}

static int vs_partial_collect(gbv_ctx* c, gbv_vs_batch* b, uint8_t out576[GBV_FP12_PARTIAL_BYTES], uint8_t* shard_ok) {
  if (b->part_empty) {
    fp12_pack(out576, fp12_one_host());
    return GBV_OK;
  }
  HIP_CHECK(c, hipSetDevice(c->device));
  const hipError_t we = hipEventSynchronize(b->done);  // no context lock held
  if (we != hipSuccess) {
    GBV_LOCK(c);
    return gbv_fail(c, GBV_E_DEVICE, std::string("hipEventSynchronize: ") + hipGetErrorString(we));
  }
  if (!b->prof.recs.empty()) {
    GBV_LOCK(c);
    c->last_ops[1] = kprof_format(b->prof);
    b->prof.reset();
  }
  Fp12 f;
  memcpy((void*)&f, b->part_host, sizeof(Fp12));
  fp12_pack(out576, f);
  const uint8_t* st = b->part_host + sizeof(Fp12);
  for (size_t i = 0; i < b->n; ++i)
    if (st[i] != SET_OK) *shard_ok = 0;
  return GBV_OK;
}

int gbv_fp12_check(gbv_ctx* c, const uint8_t* partials, size_t k, uint8_t* is_one) {
  if (!c || !is_one || (k && !partials)) return GBV_E_ARG;
  GBV_LOCK(c);
  if (c->closed) return GBV_E_CLOSED;
  HIP_CHECK(c, hipSetDevice(c->device));
  // a stream of its own (high priority): the check of shard pass k does not queue behind pass
  // k + 1's kernels (sharded.py verify_staged_shards keeps two in flight)
  hipStream_t s = c->stream6;
  uint8_t *d = nullptr, *h = nullptr;
  size_t o_o = align256(sizeof(Fp12) * std::max<size_t>(k, 1));
  int rc;
  if ((rc = ctx_small_dev(c, o_o + 256, &d)) || (rc = ctx_small_host(c, o_o + 256, &h))) return rc;
  for (size_t j = 0; j < k; ++j) {
    Fp12 f = fp12_unpack(partials + GBV_FP12_PARTIAL_BYTES * j);
    memcpy(h + sizeof(Fp12) * j, (const void*)&f, sizeof(Fp12));
  }
  if (k) HIP_CHECK(c, hipMemcpyAsync(d, h, sizeof(Fp12) * k, hipMemcpyHostToDevice, s));
  launch_fp12_check(LaunchCfg{1, 64, s}, (uint32_t)k, (const Fp12*)d, d + o_o);
  HIP_CHECK(c, hipGetLastError());
  HIP_CHECK(c, hipMemcpyAsync(h + o_o, d + o_o, 1, hipMemcpyDeviceToHost, s));
  HIP_CHECK(c, hipStreamSynchronize(s));
  *is_one = h[o_o];
  return GBV_OK;
}

}  // extern "C"
