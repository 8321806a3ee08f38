/*
 * gbv_stub.c -- a CPU stand-in for libgbv.so with the exact C ABI of include/gbv.h, for sanitizer
 * runs of the host code that binds it (addon/gbv_addon.c under -fsanitize=address,undefined, driven
 * by addon/test_addon_stub.js; tools/sanitize_host.sh).  Test infrastructure only: no BLS
 * arithmetic.  Its rules are those of the JavaScript stand-in of addon/test_verifier.js:
 *   - a set is valid iff its signature has 96 bytes and starts with the byte 1;
 *   - a pubkey slot is valid iff its 48-byte key does not start with the byte 0;
 *   - an aggregate set without pubkeys rejects its call (GBV_E_EMPTY_AGGREGATE / GBV_CALL_REJECTED).
 * Batches copy their inputs at fill time (like the real library's pinned staging) and complete
 * STUB_PASS_MS after submit, so waits really block on a pool thread while the JS thread goes on.
 */
#define _POSIX_C_SOURCE 200809L
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../../include/gbv.h"

#define STUB_PASS_MS 30

struct gbv_ctx {
  pthread_mutex_t mu;
  uint8_t* ok;  /* per slot: 1 usable */
  size_t n, cap;
  int live_batches;
};

struct gbv_sm_batch {
  size_t n, n_calls;
  uint8_t* valid;
  double ready;
  int in_flight;
};

struct gbv_vs_batch {
  size_t n_calls;
  uint8_t* call_valid;
  double ready;
  int in_flight;
  int part_flying;
};

static __thread char t_err[128];

static int fail(int rc, const char* msg) {
  snprintf(t_err, sizeof t_err, "%s", msg);
  return rc;
}

static double now_ms(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e3 + ts.tv_nsec / 1e6;
}

static void sleep_until(double t) {
  double d = t - now_ms();
  if (d <= 0) return;
  struct timespec ts = {(time_t)(d / 1e3), (long)((d - 1e3 * (time_t)(d / 1e3)) * 1e6)};
  nanosleep(&ts, NULL);
}

static int sig_ok(const uint8_t* sig, uint32_t len) { return len == 96 && sig && sig[0] == 1; }

int gbv_init(int device, gbv_ctx** out) {
  if (!out) return GBV_E_ARG;
  *out = NULL;
  if (device != 0) return fail(GBV_E_ARG, "stub: device 0 only");
  gbv_ctx* c = (gbv_ctx*)calloc(1, sizeof *c);
  pthread_mutex_init(&c->mu, NULL);
  *out = c;
  return GBV_OK;
}

void gbv_destroy(gbv_ctx* c) {
  if (!c) return;
  pthread_mutex_lock(&c->mu);
  if (c->live_batches) fprintf(stderr, "gbv_stub: %d batches still alive at destroy\n", c->live_batches);
  pthread_mutex_unlock(&c->mu);
  pthread_mutex_destroy(&c->mu);
  free(c->ok);
  free(c);
}

const char* gbv_last_error(gbv_ctx* c) { return c ? t_err : "null context"; }

int gbv_pubkeys_append(gbv_ctx* c, uint32_t first, const uint8_t* pk48, size_t n, int validate, uint8_t* status) {
  (void)validate;
  if (!c || (n && !pk48)) return fail(GBV_E_ARG, "null argument");
  pthread_mutex_lock(&c->mu);
  size_t need = (size_t)first + n;
  if (need > c->cap) {
    size_t cap = need > 2 * c->cap ? need : 2 * c->cap;
    uint8_t* p = (uint8_t*)realloc(c->ok, cap);
    if (!p) {
      pthread_mutex_unlock(&c->mu);
      return fail(GBV_E_OOM, "stub: oom");
    }
    memset(p + c->cap, 0, cap - c->cap);
    c->ok = p;
    c->cap = cap;
  }
  for (size_t i = 0; i < n; ++i) {
    int ok = pk48[48 * i] != 0;
    c->ok[first + i] = (uint8_t)ok;
    if (status) status[i] = ok ? GBV_PT_OK : GBV_PT_BAD_ENCODING;
  }
  if (need > c->n) c->n = need;
  pthread_mutex_unlock(&c->mu);
  return GBV_OK;
}

size_t gbv_pubkeys_count(gbv_ctx* c) {
  if (!c) return 0;
  pthread_mutex_lock(&c->mu);
  size_t n = c->n;
  pthread_mutex_unlock(&c->mu);
  return n;
}

int gbv_comb_enabled(gbv_ctx* c) { return c ? 1 : 0; }
int gbv_tune(gbv_ctx* c, const char* name, uint32_t value) {
  (void)value;
  return c && name ? GBV_OK : GBV_E_ARG;
}

/* one call: 1 / 0 / GBV_CALL_REJECTED; GBV_E_ARG for an index past the table */
static int call_result(gbv_ctx* c, const gbv_set* s, size_t n, const uint32_t* arena, uint8_t* out) {
  int all = n > 0, rejected = 0;
  for (size_t i = 0; i < n; ++i) {
    if (!s[i].msg32 || (!s[i].sig && s[i].sig_len)) return fail(GBV_E_ARG, "null msg/sig");
    int ok = sig_ok(s[i].sig, s[i].sig_len);
    if (s[i].raw_pk48) {
      ok = ok && s[i].raw_pk48[0] != 0;
    } else if (s[i].idx_len == 0) {
      rejected = 1;
    } else {
      if (!arena) return fail(GBV_E_ARG, "null index arena");
      for (uint32_t j = 0; j < s[i].idx_len; ++j) {
        uint32_t k = arena[s[i].idx_off + j];
        if (k >= c->n) return fail(GBV_E_ARG, "validator index out of range");
        ok = ok && c->ok[k];
      }
    }
    all = all && ok;
  }
  *out = rejected ? GBV_CALL_REJECTED : (uint8_t)all;
  return GBV_OK;
}

static int calls_result(gbv_ctx* c, size_t n_calls, const uint32_t* call_off, const gbv_set* sets, const uint32_t* arena,
                        uint8_t* call_valid) {
  if (n_calls && (!call_off || !call_valid)) return fail(GBV_E_ARG, "null argument");
  for (size_t g = 0; g < n_calls; ++g) {
    if (call_off[g + 1] < call_off[g]) return fail(GBV_E_ARG, "call offsets not monotone");
    int rc = call_result(c, sets + call_off[g], call_off[g + 1] - call_off[g], arena, call_valid + g);
    if (rc) return rc;
  }
  return GBV_OK;
}

int gbv_verify_sets(gbv_ctx* c, const gbv_set* sets, size_t n, const uint32_t* arena, uint8_t* all_valid, uint8_t* chunk_valid) {
  if (!c || !all_valid) return GBV_E_ARG;
  pthread_mutex_lock(&c->mu);
  uint8_t v = 0;
  int rc = call_result(c, sets, n, arena, &v);
  pthread_mutex_unlock(&c->mu);
  if (rc) return rc;
  if (v == GBV_CALL_REJECTED) return fail(GBV_E_EMPTY_AGGREGATE, "EMPTY_AGGREGATE_ARRAY");
  *all_valid = v;
  if (chunk_valid) chunk_valid[0] = v;
  return GBV_OK;
}

int gbv_verify_sets_multi(gbv_ctx* c, size_t n_calls, const uint32_t* call_off, const gbv_set* sets, const uint32_t* arena,
                          uint8_t* call_valid) {
  if (!c) return GBV_E_ARG;
  pthread_mutex_lock(&c->mu);
  int rc = calls_result(c, n_calls, call_off, sets, arena, call_valid);
  pthread_mutex_unlock(&c->mu);
  if (!rc) sleep_until(now_ms() + STUB_PASS_MS);  /* a device pass, on the caller's (pool) thread */
  return rc;
}

static int sm_result(gbv_ctx* c, size_t n_calls, const uint32_t* call_off, const uint32_t* idx, const uint8_t* sigs96,
                     const uint8_t* msgs32, uint8_t* valid) {
  if (n_calls && (!call_off || !msgs32)) return fail(GBV_E_ARG, "null argument");
  size_t n = n_calls ? call_off[n_calls] : 0;
  if (n && (!idx || !sigs96 || !valid)) return fail(GBV_E_ARG, "null argument");
  for (size_t i = 0; i < n; ++i) {
    if (idx[i] >= c->n) return fail(GBV_E_ARG, "validator index out of range");
    valid[i] = (uint8_t)(sig_ok(sigs96 + 96 * i, 96) && c->ok[idx[i]]);
  }
  return GBV_OK;
}

int gbv_verify_same_message_multi(gbv_ctx* c, size_t n_calls, const uint32_t* call_off, const uint32_t* idx, const uint8_t* sigs96,
                                  const uint8_t* msgs32, uint8_t* valid) {
  if (!c) return GBV_E_ARG;
  pthread_mutex_lock(&c->mu);
  int rc = sm_result(c, n_calls, call_off, idx, sigs96, msgs32, valid);
  pthread_mutex_unlock(&c->mu);
  if (!rc) sleep_until(now_ms() + STUB_PASS_MS);
  return rc;
}

int gbv_verify_same_message(gbv_ctx* c, const uint32_t* idx, const uint8_t* sigs96, size_t n, const uint8_t* msg32, uint8_t* valid) {
  uint32_t off[2] = {0, (uint32_t)n};
  return gbv_verify_same_message_multi(c, 1, off, idx, sigs96, msg32, valid);
}

/* aggregates: a deterministic digest of the inputs (shape only) */
int gbv_aggregate_pubkeys(gbv_ctx* c, const uint32_t* idx, size_t k, uint8_t out48[48]) {
  if (!c || !out48) return GBV_E_ARG;
  if (k == 0) return fail(GBV_E_EMPTY_AGGREGATE, "EMPTY_AGGREGATE_ARRAY");
  pthread_mutex_lock(&c->mu);
  memset(out48, 0, 48);
  out48[0] = 0x80;
  for (size_t i = 0; i < k; ++i) {
    if (idx[i] >= c->n) {
      pthread_mutex_unlock(&c->mu);
      return fail(GBV_E_ARG, "validator index out of range");
    }
    out48[1 + i % 47] ^= (uint8_t)(idx[i] * 131u + 7u);
  }
  pthread_mutex_unlock(&c->mu);
  return GBV_OK;
}

int gbv_aggregate_serialized_pubkeys(gbv_ctx* c, const uint8_t* pk48, size_t k, int validate, uint8_t out48[48]) {
  (void)validate;
  if (!c || !out48 || (k && !pk48)) return GBV_E_ARG;
  if (k == 0) return fail(GBV_E_EMPTY_AGGREGATE, "EMPTY_AGGREGATE_ARRAY");
  memset(out48, 0, 48);
  for (size_t i = 0; i < k; ++i) {
    if (pk48[48 * i] == 0) return fail(GBV_E_BAD_POINT, "BLST_BAD_ENCODING");
    for (int b = 0; b < 48; ++b) out48[b] ^= pk48[48 * i + b];
  }
  return GBV_OK;
}

int gbv_signatures_validate(gbv_ctx* c, const uint8_t* sigs, size_t n, uint32_t sig_len, uint8_t* status, uint8_t* out96) {
  if (!c || (n && (!sigs || !status))) return GBV_E_ARG;
  for (size_t i = 0; i < n; ++i) {
    int ok = sig_ok(sigs + (size_t)sig_len * i, sig_len);
    status[i] = ok ? GBV_PT_OK : GBV_PT_BAD_ENCODING;
    if (out96) {
      memset(out96 + 96 * i, 0, 96);
      if (ok) memcpy(out96 + 96 * i, sigs + (size_t)sig_len * i, 96);
      else out96[96 * i] = 0xc0;
    }
  }
  return GBV_OK;
}

int gbv_aggregate_signatures(gbv_ctx* c, const uint8_t* sigs, size_t n, uint32_t sig_len, int validate, uint8_t out96[96]) {
  (void)validate;
  if (!c || !out96 || (n && !sigs)) return GBV_E_ARG;
  if (n == 0) return fail(GBV_E_EMPTY_AGGREGATE, "EMPTY_AGGREGATE_ARRAY");
  memset(out96, 0, 96);
  for (size_t i = 0; i < n; ++i) {
    if (!sig_ok(sigs + (size_t)sig_len * i, sig_len)) return fail(GBV_E_BAD_POINT, "BLST_BAD_ENCODING");
    for (int b = 0; b < 96; ++b) out96[b] ^= sigs[(size_t)sig_len * i + b];
  }
  return GBV_OK;
}

/* ---- batches ---- */
int gbv_sm_batch_fill(gbv_ctx* c, gbv_sm_batch* b, size_t n_calls, const uint32_t* call_off, const uint32_t* idx, const uint8_t* sigs96,
                      const uint8_t* msgs32) {
  if (!c || !b) return GBV_E_ARG;
  if (b->in_flight) return fail(GBV_E_ARG, "batch in flight");
  size_t n = n_calls ? call_off[n_calls] : 0;
  uint8_t* v = (uint8_t*)realloc(b->valid, n ? n : 1);
  if (!v) return fail(GBV_E_OOM, "stub: oom");
  b->valid = v;
  pthread_mutex_lock(&c->mu);
  int rc = sm_result(c, n_calls, call_off, idx, sigs96, msgs32, b->valid);
  pthread_mutex_unlock(&c->mu);
  b->n = rc ? 0 : n;
  b->n_calls = rc ? 0 : n_calls;
  return rc;
}

int gbv_sm_batch_create(gbv_ctx* c, size_t n_calls, const uint32_t* call_off, const uint32_t* idx, const uint8_t* sigs96,
                        const uint8_t* msgs32, gbv_sm_batch** out) {
  if (!c || !out) return GBV_E_ARG;
  gbv_sm_batch* b = (gbv_sm_batch*)calloc(1, sizeof *b);
  int rc = gbv_sm_batch_fill(c, b, n_calls, call_off, idx, sigs96, msgs32);
  if (rc) {
    free(b->valid);
    free(b);
    return rc;
  }
  pthread_mutex_lock(&c->mu);
  ++c->live_batches;
  pthread_mutex_unlock(&c->mu);
  *out = b;
  return GBV_OK;
}

int gbv_sm_batch_submit(gbv_ctx* c, gbv_sm_batch* b) {
  if (!c || !b) return GBV_E_ARG;
  if (b->in_flight) return fail(GBV_E_ARG, "batch already in flight");
  b->ready = now_ms() + STUB_PASS_MS;
  b->in_flight = 1;
  return GBV_OK;
}

int gbv_sm_batch_wait(gbv_ctx* c, gbv_sm_batch* b, uint8_t* valid) {
  if (!c || !b) return GBV_E_ARG;
  if (!b->in_flight) return b->n ? fail(GBV_E_ARG, "batch not submitted") : GBV_OK;
  sleep_until(b->ready);
  b->in_flight = 0;
  if (valid && b->n) memcpy(valid, b->valid, b->n);
  return GBV_OK;
}

int gbv_sm_batch_verify(gbv_ctx* c, gbv_sm_batch* b, uint8_t* valid) {
  int rc = gbv_sm_batch_submit(c, b);
  return rc ? rc : gbv_sm_batch_wait(c, b, valid);
}

void gbv_sm_batch_destroy(gbv_ctx* c, gbv_sm_batch* b) {
  if (!b) return;
  if (b->in_flight) sleep_until(b->ready);
  if (c) {
    pthread_mutex_lock(&c->mu);
    --c->live_batches;
    pthread_mutex_unlock(&c->mu);
  }
  free(b->valid);
  free(b);
}

int gbv_vs_batch_fill(gbv_ctx* c, gbv_vs_batch* b, size_t n_calls, const uint32_t* call_off, const gbv_set* sets, const uint32_t* arena) {
  if (!c || !b) return GBV_E_ARG;
  if (b->in_flight) return fail(GBV_E_ARG, "batch in flight");
  uint8_t* v = (uint8_t*)realloc(b->call_valid, n_calls ? n_calls : 1);
  if (!v) return fail(GBV_E_OOM, "stub: oom");
  b->call_valid = v;
  pthread_mutex_lock(&c->mu);
  int rc = calls_result(c, n_calls, call_off, sets, arena, b->call_valid);
  pthread_mutex_unlock(&c->mu);
  b->n_calls = rc ? 0 : n_calls;
  return rc;
}

int gbv_vs_batch_create(gbv_ctx* c, size_t n_calls, const uint32_t* call_off, const gbv_set* sets, const uint32_t* arena,
                        gbv_vs_batch** out) {
  if (!c || !out) return GBV_E_ARG;
  gbv_vs_batch* b = (gbv_vs_batch*)calloc(1, sizeof *b);
  int rc = gbv_vs_batch_fill(c, b, n_calls, call_off, sets, arena);
  if (rc) {
    free(b->call_valid);
    free(b);
    return rc;
  }
  pthread_mutex_lock(&c->mu);
  ++c->live_batches;
  pthread_mutex_unlock(&c->mu);
  *out = b;
  return GBV_OK;
}

int gbv_vs_batch_submit(gbv_ctx* c, gbv_vs_batch* b) {
  if (!c || !b) return GBV_E_ARG;
  if (b->in_flight) return fail(GBV_E_ARG, "batch already in flight");
  if (!b->n_calls) return GBV_OK;
  b->ready = now_ms() + STUB_PASS_MS;
  b->in_flight = 1;
  return GBV_OK;
}

int gbv_vs_batch_wait(gbv_ctx* c, gbv_vs_batch* b, uint8_t* call_valid) {
  if (!c || !b) return GBV_E_ARG;
  if (b->in_flight) sleep_until(b->ready);
  b->in_flight = 0;
  if (call_valid && b->n_calls) memcpy(call_valid, b->call_valid, b->n_calls);
  return GBV_OK;
}

void gbv_vs_batch_destroy(gbv_ctx* c, gbv_vs_batch* b) {
  if (!b) return;
  if (b->in_flight) sleep_until(b->ready);
  if (c) {
    pthread_mutex_lock(&c->mu);
    --c->live_batches;
    pthread_mutex_unlock(&c->mu);
  }
  free(b->call_valid);
  free(b);
}

int gbv_vs_last_kernel_ms(gbv_ctx* c, float* ms4) {
  if (!c || !ms4) return GBV_E_ARG;
  memset(ms4, 0, 4 * sizeof(float));
  return GBV_OK;
}

/* partials: byte 0 = 1 for an all-valid shard; the check multiplies "all ones" */
int gbv_vs_partial(gbv_ctx* c, const gbv_set* sets, size_t n, const uint32_t* arena, uint8_t out576[GBV_FP12_PARTIAL_BYTES],
                   uint8_t* shard_ok) {
  if (!c || !out576 || !shard_ok) return GBV_E_ARG;
  uint8_t v = 0;
  pthread_mutex_lock(&c->mu);
  int rc = call_result(c, sets, n, arena, &v);
  pthread_mutex_unlock(&c->mu);
  if (rc) return rc;
  if (v == GBV_CALL_REJECTED) return fail(GBV_E_EMPTY_AGGREGATE, "EMPTY_AGGREGATE_ARRAY");
  memset(out576, 0, GBV_FP12_PARTIAL_BYTES);
  out576[0] = (uint8_t)(n == 0 || v);
  *shard_ok = 1;
  return GBV_OK;
}

int gbv_vs_batch_partial(gbv_ctx* c, gbv_vs_batch* b, uint8_t out576[GBV_FP12_PARTIAL_BYTES], uint8_t* shard_ok) {
  if (!c || !b || !out576 || !shard_ok) return GBV_E_ARG;
  uint8_t all = 1;
  for (size_t g = 0; g < b->n_calls; ++g) all = all && b->call_valid[g] == 1;
  memset(out576, 0, GBV_FP12_PARTIAL_BYTES);
  out576[0] = all;
  *shard_ok = 1;
  return GBV_OK;
}

int gbv_vs_batch_partial_submit(gbv_ctx* c, gbv_vs_batch* b) {
  if (!c || !b) return GBV_E_ARG;
  if (b->part_flying) return fail(GBV_E_ARG, "batch in flight");
  for (size_t g = 0; g < b->n_calls; ++g)
    if (b->call_valid[g] == GBV_CALL_REJECTED) return fail(GBV_E_EMPTY_AGGREGATE, "EMPTY_AGGREGATE_ARRAY");
  b->part_flying = 1;
  return GBV_OK;
}

int gbv_vs_batch_partial_wait(gbv_ctx* c, gbv_vs_batch* b, uint8_t out576[GBV_FP12_PARTIAL_BYTES], uint8_t* shard_ok) {
  if (!c || !b || !out576 || !shard_ok) return GBV_E_ARG;
  if (!b->part_flying) return fail(GBV_E_ARG, "partial not submitted");
  b->part_flying = 0;
  return gbv_vs_batch_partial(c, b, out576, shard_ok);
}

int gbv_fp12_check(gbv_ctx* c, const uint8_t* partials, size_t k, uint8_t* is_one) {
  if (!c || !is_one || (k && !partials)) return GBV_E_ARG;
  uint8_t one = 1;
  for (size_t j = 0; j < k; ++j) one = one && partials[GBV_FP12_PARTIAL_BYTES * j] == 1;
  *is_one = one;
  return GBV_OK;
}

int gbv_last_kernel_ms(gbv_ctx* c, float* out, int* launches, int max) {
  if (!c || !out) return 0;
  for (int i = 0; i < max && i < 8; ++i) {
    out[i] = 0.f;
    if (launches) launches[i] = 0;
  }
  return max < 8 ? max : 8;
}

int gbv_last_ops(gbv_ctx* c, int path, char* out, size_t cap) {
  if (!c || (path != 0 && path != 1) || (cap && !out)) return GBV_E_ARG;
  if (cap) out[0] = 0; /* the stub runs no kernels */
  return 0;
}

int gbv_last_stats(gbv_ctx* c, uint32_t* fb, uint32_t* seg) {
  if (!c) return GBV_E_ARG;
  if (fb) *fb = 0;
  if (seg) *seg = 0;
  return GBV_OK;
}

/* signing roots and utilities: not used by the addon; present so the symbol set matches gbv.h */
static int unsupported(void) { return fail(GBV_E_DEVICE, "stub: no device"); }
int gbv_sha256_digest64(gbv_ctx* c, const uint8_t* in64, size_t n, uint8_t* out32) { (void)c; (void)in64; (void)n; (void)out32; return unsupported(); }
int gbv_merkle_roots(gbv_ctx* c, const uint8_t* ch, size_t n, uint32_t d, uint8_t* out32) { (void)c; (void)ch; (void)n; (void)d; (void)out32; return unsupported(); }
int gbv_signing_roots(gbv_ctx* c, const uint8_t* r, size_t n, const uint8_t* d, size_t nd, const uint32_t* di, uint8_t* o) {
  (void)c; (void)r; (void)n; (void)d; (void)nd; (void)di; (void)o;
  return unsupported();
}
int gbv_attestation_signing_roots(gbv_ctx* c, const uint8_t* a, size_t n, const uint8_t* d, size_t nd, const uint32_t* di, uint8_t* o) {
  (void)c; (void)a; (void)n; (void)d; (void)nd; (void)di; (void)o;
  return unsupported();
}
int gbv_ssz_last_kernel_ms(gbv_ctx* c, float* ms) { (void)c; if (ms) *ms = 0.f; return GBV_OK; }
int gbv_util_sk_to_pk(gbv_ctx* c, const uint8_t* sk, size_t n, uint8_t* pk) { (void)c; (void)sk; (void)n; (void)pk; return unsupported(); }
int gbv_util_sign(gbv_ctx* c, const uint8_t* sk, size_t n, const uint32_t* g, const uint8_t* m, size_t nm, uint8_t* s) {
  (void)c; (void)sk; (void)n; (void)g; (void)m; (void)nm; (void)s;
  return unsupported();
}
int gbv_util_hash_to_g2(gbv_ctx* c, const uint8_t* m, size_t n, uint8_t* o) { (void)c; (void)m; (void)n; (void)o; return unsupported(); }
int gbv_util_g1_mul_rand(gbv_ctx* c, const uint32_t* s, const uint64_t* r, size_t n, int u, uint8_t* o) {
  (void)c; (void)s; (void)r; (void)n; (void)u; (void)o;
  return unsupported();
}
int gbv_pubkeys_replicate(gbv_ctx* c, uint32_t a, uint32_t b, uint32_t d, size_t n) { (void)c; (void)a; (void)b; (void)d; (void)n; return unsupported(); }
