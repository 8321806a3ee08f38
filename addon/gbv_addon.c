/*
 * gbv_addon.c -- Node-API addon (C) over the C ABI of include/gbv.h: the binding a Lodestar
 * GpuBlsVerifier (TypeScript, beside BlsMultiThreadWorkerPool; selected at
 * beacon-node/src/chain/chain.ts:223-225) calls.  It mirrors IBlsVerifier
 * (beacon-node/src/chain/bls/interface.ts:25-68) with index-form signature sets:
 *
 *   open(device)                                  -> ctx             (gbv_init)
 *   addPubkeys(ctx, firstIndex, pk48s, validate)  -> Uint8Array      (gbv_pubkeys_append; syncPubkeys /
 *                                                                      addFinalizedPubkey, pubkeyCache.ts:50-69)
 *   verifySets(ctx, sets)                         -> Promise<boolean> (gbv_verify_sets; verifySignatureSets)
 *   verifySetsMulti(ctx, calls)                   -> Promise<Array<boolean | Error>> (gbv_verify_sets_multi:
 *                                                                      several calls in one device pass)
 *   verifySameMessageMulti(ctx, calls)            -> Promise<(Uint8Array | boolean[])[]>
 *                                                     (gbv_verify_same_message_multi; verifySignatureSetsSameMessage:
 *                                                      a packed call answers with 0 / 1 bytes, an object call with booleans)
 *   aggregatePubkeys(ctx, indices)                -> Uint8Array(48)  (gbv_aggregate_pubkeys)
 *   aggregateSerializedPubkeys(ctx, pk48s, validate) -> Uint8Array(48) (syncCommittee.ts:37)
 *   close(ctx)                                    -> Promise<void>   (waits for in-flight work, gbv_destroy)
 *
 * The streamed pair (what a GpuBlsVerifier's job queue drives; MAX_PASSES passes on the device at once,
 * each on its own refillable batches -- gbv_sm_batch_fill / gbv_vs_batch_fill + submit):
 *   submitPass(ctx, sameMessageCalls | null, defaultCalls | null) -> pass  (synchronous: inputs copied
 *                                                  to pinned memory, kernels enqueued; no device wait)
 *   waitPass(pass)                                -> Promise<{sameMessage: Uint8Array (flat form: one
 *                                                             0 / 1 byte per set of the pass) |
 *                                                             (boolean[] | Uint8Array)[] (per call) | Error,
 *                                                             default: (boolean | Error)[] | Error}>
 *   freePasses(ctx)                               -> number of pass slots not in flight
 * and the rest of IBlsVerifier's needs: verifySetsSync(ctx, sets) -> boolean (verifyOnMainThread,
 * index.ts:168-181), pubkeyCount(ctx), vsPartial(ctx, sets) -> Promise<{partial, ok}> and
 * fp12Check(ctx, partials) -> boolean (multi-GPU shards, gbv_vs_partial / gbv_fp12_check), and the
 * device hashing of the signature-set builders: merkleRoots(ctx, chunks, depth) (gbv_merkle_roots) and
 * signingRoots(ctx, objectRoots, domains, domIdx) (gbv_signing_roots).
 *
 * A set is {index: number} or {indices: Uint32Array | number[]} or {pubkey: Uint8Array(48)}, plus
 * {signingRoot: Uint8Array(32), signature: Uint8Array}.  JS buffers are only borrowed during the
 * synchronous part of a call: everything is copied into C-owned memory before the work is queued
 * on the libuv pool (napi_async_work), and results are delivered on the JS thread.  One context is
 * used by one device call at a time (include/gbv.h): a per-context mutex serialises the pool threads.
 *
 * Error mapping: per-set false results are values, never errors; an aggregate set
 * without pubkeys rejects with code "EMPTY_AGGREGATE_ARRAY" (bls/utils.ts:12 -> index.ts:398-412),
 * a closed context with "QUEUE_ABORTED" (index.ts:303-305), device failures with "GBV_E_DEVICE",
 * malformed arguments with "GBV_E_ARG" (or a TypeError for a wrong JS type).
 */
#define NAPI_VERSION 6
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <node_api.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/gbv.h"

#define MAX_PASSES 3
struct pass_s;
typedef struct {
  gbv_sm_batch* sm;
  gbv_vs_batch* vs;
  int busy;              /* JS thread only: a submitted pass not yet waited */
  struct pass_s* pass;   /* JS thread only: that pass (reclaim_orphans frees one its caller dropped unwaited) */
  pthread_mutex_t mu;    /* held by the pool thread waiting on the pass, and by close() */
} pass_slot;

typedef struct {
  gbv_ctx* ctx;
  pthread_mutex_t mu;
  int closed;
  int inflight;
  pass_slot slots[MAX_PASSES];
} addon_ctx;

/* ---- helpers ------------------------------------------------------------------------------ */
#define NAPI_OK(env, call)                                                   \
  do {                                                                       \
    if ((call) != napi_ok) {                                                 \
      napi_throw_error((env), "GBV_E_NAPI", "Node-API call failed: " #call); \
      return NULL;                                                           \
    }                                                                        \
  } while (0)

static const char* code_of(int rc) {
  switch (rc) {
    case GBV_E_EMPTY_AGGREGATE: return "EMPTY_AGGREGATE_ARRAY";
    case GBV_E_CLOSED: return "QUEUE_ABORTED";
    case GBV_E_DEVICE: return "GBV_E_DEVICE";
    case GBV_E_OOM: return "GBV_E_OOM";
    case GBV_E_BAD_POINT: return "GBV_E_BAD_POINT";
    default: return "GBV_E_ARG";
  }
}

static napi_value make_error(napi_env env, int rc, const char* msg) {
  napi_value code, text, err;
  napi_create_string_utf8(env, code_of(rc), NAPI_AUTO_LENGTH, &code);
  napi_create_string_utf8(env, msg && *msg ? msg : code_of(rc), NAPI_AUTO_LENGTH, &text);
  napi_create_error(env, code, text, &err);
  return err;
}

static void throw_rc(napi_env env, int rc, const char* msg) { napi_throw(env, make_error(env, rc, msg)); }

static addon_ctx* get_ctx(napi_env env, napi_value v) {
  napi_valuetype t;
  if (napi_typeof(env, v, &t) != napi_ok || t != napi_external) {
    napi_throw_type_error(env, "GBV_E_ARG", "expected a context from open()");
    return NULL;
  }
  void* p = NULL;
  napi_get_value_external(env, v, &p);
  return (addon_ctx*)p;
}

/* Borrow the bytes of a Uint8Array / Buffer (only valid during the synchronous part). */
static int get_bytes(napi_env env, napi_value v, const uint8_t** data, size_t* len) {
  bool is_ta = false;
  napi_is_typedarray(env, v, &is_ta);
  if (is_ta) {
    napi_typedarray_type type;
    size_t n, off;
    void* d;
    napi_value ab;
    if (napi_get_typedarray_info(env, v, &type, &n, &d, &ab, &off) != napi_ok || type != napi_uint8_array) return 0;
    *data = (const uint8_t*)d;
    *len = n;
    return 1;
  }
  bool is_buf = false;
  napi_is_buffer(env, v, &is_buf);
  if (is_buf) {
    void* d;
    if (napi_get_buffer_info(env, v, &d, len) != napi_ok) return 0;
    *data = (const uint8_t*)d;
    return 1;
  }
  return 0;
}


/* Property keys created once per marshalled argument, not once per object: napi_get_named_property
 * builds the key string on every call (~0.5-1 us each on this Node), a per-set cost in the object
 * forms and a per-call cost in the packed form. */
enum { K_SIGNING_ROOT, K_SIGNATURE, K_PUBKEY, K_INDICES, K_INDEX, K_MESSAGE, K_SETS, K_SIGNATURES, K_COUNTS, K_MESSAGES, K_N };
static const char* const KEY_NAMES[K_N] = {"signingRoot", "signature", "pubkey", "indices", "index", "message", "sets", "signatures",
                                           "counts", "messages"};
typedef struct { napi_value k[K_N]; } keyset;
static void keys_init(napi_env env, keyset* ks) {
  for (int i = 0; i < K_N; ++i) napi_create_string_utf8(env, KEY_NAMES[i], NAPI_AUTO_LENGTH, &ks->k[i]);
}
/* obj[key] when present and neither undefined nor null */
static int get_key(napi_env env, napi_value obj, napi_value key, napi_value* out) {
  if (napi_get_property(env, obj, key, out) != napi_ok) {
    const napi_extended_error_info* info;
    napi_get_last_error_info(env, &info);
    return 0;
  }
  napi_valuetype t;
  napi_typeof(env, *out, &t);
  return t != napi_undefined && t != napi_null;
}

static int get_u32(napi_env env, napi_value v, uint32_t* out) {
  napi_valuetype t;
  if (napi_typeof(env, v, &t) != napi_ok || t != napi_number) return 0;
  return napi_get_value_uint32(env, v, out) == napi_ok;
}

/* growable byte / u32 vectors (C-owned copies of JS inputs) */
typedef struct { uint8_t* p; size_t n, cap; } bvec;
typedef struct { uint32_t* p; size_t n, cap; } uvec;
static void bv_push(bvec* v, const void* d, size_t n) {
  if (v->n + n > v->cap) {
    v->cap = (v->n + n) * 2 + 64;
    v->p = (uint8_t*)realloc(v->p, v->cap);
  }
  memcpy(v->p + v->n, d, n);
  v->n += n;
}
static void uv_push(uvec* v, uint32_t x) {
  if (v->n == v->cap) {
    v->cap = v->cap * 2 + 64;
    v->p = (uint32_t*)realloc(v->p, v->cap * sizeof(uint32_t));
  }
  v->p[v->n++] = x;
}
static void uv_push_n(uvec* v, const uint32_t* x, size_t n) {
  if (v->n + n > v->cap) {
    v->cap = (v->n + n) * 2 + 64;
    v->p = (uint32_t*)realloc(v->p, v->cap * sizeof(uint32_t));
  }
  memcpy(v->p + v->n, x, n * sizeof(uint32_t));
  v->n += n;
}

/* Borrow a Uint32Array's elements (only valid during the synchronous part). */
static int get_u32_array(napi_env env, napi_value v, const uint32_t** data, size_t* n) {
  bool is_ta = false;
  napi_is_typedarray(env, v, &is_ta);
  if (!is_ta) return 0;
  napi_typedarray_type type;
  size_t off;
  void* d;
  napi_value ab;
  if (napi_get_typedarray_info(env, v, &type, n, &d, &ab, &off) != napi_ok || type != napi_uint32_array) return 0;
  *data = (const uint32_t*)d;
  return 1;
}

/* ---- signature-set marshalling ---------------------------------------------------------- */
/* Copied sets: per set (arena offset/len, raw-pk offset or -1, msg offset, sig offset/len). */
typedef struct {
  uvec call_off;
  uvec idx_off, idx_len, arena;
  uvec raw_off; /* 0xFFFFFFFF: none */
  uvec sig_off, sig_len;
  bvec bytes; /* roots, signatures, raw pubkeys */
  uvec msg_off;
} sets_buf;

static void sets_free(sets_buf* s) {
  free(s->call_off.p); free(s->idx_off.p); free(s->idx_len.p); free(s->arena.p); free(s->raw_off.p);
  free(s->sig_off.p); free(s->sig_len.p); free(s->bytes.p); free(s->msg_off.p);
  memset(s, 0, sizeof *s);
}

/* Append the sets of one JS array; returns 0 (and throws) on a malformed argument. */
static int marshal_sets(napi_env env, napi_value arr, sets_buf* s) {
  keyset ks;
  keys_init(env, &ks);
  bool is_arr = false;
  napi_is_array(env, arr, &is_arr);
  if (!is_arr) {
    napi_throw_type_error(env, "GBV_E_ARG", "sets must be an array");
    return 0;
  }
  uint32_t n = 0;
  napi_get_array_length(env, arr, &n);
  for (uint32_t i = 0; i < n; ++i) {
    napi_value e, v;
    napi_get_element(env, arr, i, &e);
    napi_valuetype t;
    napi_typeof(env, e, &t);
    if (t != napi_object) {
      napi_throw_type_error(env, "GBV_E_ARG", "a signature set must be an object");
      return 0;
    }
    const uint8_t* d;
    size_t len;
    if (!get_key(env, e, ks.k[K_SIGNING_ROOT], &v) || !get_bytes(env, v, &d, &len) || len != 32) {
      napi_throw_type_error(env, "GBV_E_ARG", "signingRoot must be a 32-byte Uint8Array");
      return 0;
    }
    uv_push(&s->msg_off, (uint32_t)s->bytes.n);
    bv_push(&s->bytes, d, 32);
    if (!get_key(env, e, ks.k[K_SIGNATURE], &v) || !get_bytes(env, v, &d, &len)) {
      napi_throw_type_error(env, "GBV_E_ARG", "signature must be a Uint8Array");
      return 0;
    }
    uv_push(&s->sig_off, (uint32_t)s->bytes.n);
    uv_push(&s->sig_len, (uint32_t)len);
    bv_push(&s->bytes, d, len);
    uv_push(&s->idx_off, (uint32_t)s->arena.n);
    if (get_key(env, e, ks.k[K_PUBKEY], &v)) {
      if (!get_bytes(env, v, &d, &len) || len != 48) {
        napi_throw_type_error(env, "GBV_E_ARG", "pubkey must be a 48-byte Uint8Array");
        return 0;
      }
      uv_push(&s->raw_off, (uint32_t)s->bytes.n);
      bv_push(&s->bytes, d, 48);
      uv_push(&s->idx_len, 0);
    } else if (get_key(env, e, ks.k[K_INDICES], &v)) {
      uv_push(&s->raw_off, 0xFFFFFFFFu);
      bool ta = false, ja = false;
      napi_is_typedarray(env, v, &ta);
      napi_is_array(env, v, &ja);
      uint32_t k = 0;
      if (ta) {
        napi_typedarray_type type;
        size_t cnt, off;
        void* p;
        napi_value ab;
        napi_get_typedarray_info(env, v, &type, &cnt, &p, &ab, &off);
        if (type != napi_uint32_array) {
          napi_throw_type_error(env, "GBV_E_ARG", "indices must be a Uint32Array or an array of numbers");
          return 0;
        }
        for (size_t j = 0; j < cnt; ++j) uv_push(&s->arena, ((const uint32_t*)p)[j]);
        k = (uint32_t)cnt;
      } else if (ja) {
        napi_get_array_length(env, v, &k);
        for (uint32_t j = 0; j < k; ++j) {
          napi_value x;
          uint32_t u;
          napi_get_element(env, v, j, &x);
          if (!get_u32(env, x, &u)) {
            napi_throw_type_error(env, "GBV_E_ARG", "indices must be numbers");
            return 0;
          }
          uv_push(&s->arena, u);
        }
      } else {
        napi_throw_type_error(env, "GBV_E_ARG", "indices must be a Uint32Array or an array of numbers");
        return 0;
      }
      uv_push(&s->idx_len, k);
    } else if (get_key(env, e, ks.k[K_INDEX], &v)) {
      uint32_t u;
      if (!get_u32(env, v, &u)) {
        napi_throw_type_error(env, "GBV_E_ARG", "index must be a number");
        return 0;
      }
      uv_push(&s->raw_off, 0xFFFFFFFFu);
      uv_push(&s->arena, u);
      uv_push(&s->idx_len, 1);
    } else {
      napi_throw_type_error(env, "GBV_E_ARG", "a set needs index, indices or pubkey");
      return 0;
    }
  }
  return 1;
}

/* gbv_set records pointing into the copied bytes (built on the pool thread, after all pushes). */
static gbv_set* sets_records(sets_buf* s) {
  size_t n = s->msg_off.n;
  gbv_set* r = (gbv_set*)calloc(n ? n : 1, sizeof(gbv_set));
  for (size_t i = 0; i < n; ++i) {
    r[i].idx_off = s->idx_off.p[i];
    r[i].idx_len = s->idx_len.p[i];
    r[i].raw_pk48 = s->raw_off.p[i] == 0xFFFFFFFFu ? NULL : s->bytes.p + s->raw_off.p[i];
    r[i].msg32 = s->bytes.p + s->msg_off.p[i];
    r[i].sig = s->sig_len.p[i] ? s->bytes.p + s->sig_off.p[i] : NULL;
    r[i].sig_len = s->sig_len.p[i];
  }
  return r;
}

/* ---- async work ------------------------------------------------------------------------------ */
enum { OP_VERIFY_SETS, OP_VERIFY_SETS_MULTI, OP_SAME_MESSAGE_MULTI, OP_CLOSE };

typedef struct {
  int op;
  addon_ctx* ac;
  napi_deferred deferred;
  napi_async_work work;
  sets_buf sets;
  /* same-message: per set index + 96-byte signature, per call a message */
  uvec sm_idx;
  bvec sm_sigs, sm_msgs;
  bvec sm_packed;    /* per same-message call: 1 = packed sets (answered with a Uint8Array) */
  uint8_t* out;
  size_t n_out;
  int rc;
  char err[256];
  napi_ref ctx_ref;  /* keeps the context external (and so ac) alive until complete() */
} job;

static void lock_begin(addon_ctx* ac) {
  pthread_mutex_lock(&ac->mu);
}
static void lock_end(addon_ctx* ac) { pthread_mutex_unlock(&ac->mu); }

static void execute(napi_env env, void* data) {
  (void)env;
  job* j = (job*)data;
  addon_ctx* ac = j->ac;
  lock_begin(ac);
  if (!ac->ctx) {
    j->rc = GBV_E_CLOSED;
    lock_end(ac);
    return;
  }
  switch (j->op) {
    case OP_VERIFY_SETS: {
      gbv_set* r = sets_records(&j->sets);
      j->out = (uint8_t*)calloc(1, 1);
      j->rc = gbv_verify_sets(ac->ctx, r, j->sets.msg_off.n, j->sets.arena.p, j->out, NULL);
      free(r);
      break;
    }
    case OP_VERIFY_SETS_MULTI: {
      gbv_set* r = sets_records(&j->sets);
      size_t nc = j->sets.call_off.n ? j->sets.call_off.n - 1 : 0;
      j->out = (uint8_t*)calloc(nc ? nc : 1, 1);
      j->n_out = nc;
      j->rc = gbv_verify_sets_multi(ac->ctx, nc, j->sets.call_off.p, r, j->sets.arena.p, j->out);
      free(r);
      break;
    }
    case OP_SAME_MESSAGE_MULTI: {
      size_t nc = j->sets.call_off.n ? j->sets.call_off.n - 1 : 0;
      j->n_out = j->sm_idx.n;
      j->out = (uint8_t*)calloc(j->n_out ? j->n_out : 1, 1);
      j->rc = gbv_verify_same_message_multi(ac->ctx, nc, j->sets.call_off.p, j->sm_idx.p, j->sm_sigs.p, j->sm_msgs.p, j->out);
      break;
    }
    case OP_CLOSE:
      for (int k = 0; k < MAX_PASSES; ++k) {  /* after any pool thread still waiting on a pass */
        pthread_mutex_lock(&ac->slots[k].mu);
        if (ac->slots[k].sm) gbv_sm_batch_destroy(ac->ctx, ac->slots[k].sm);
        if (ac->slots[k].vs) gbv_vs_batch_destroy(ac->ctx, ac->slots[k].vs);
        ac->slots[k].sm = NULL;
        ac->slots[k].vs = NULL;
        pthread_mutex_unlock(&ac->slots[k].mu);
      }
      gbv_destroy(ac->ctx);
      ac->ctx = NULL;
      j->rc = GBV_OK;
      break;
  }
  if (j->rc && ac->ctx) snprintf(j->err, sizeof j->err, "%s", gbv_last_error(ac->ctx));
  lock_end(ac);
}

static void complete(napi_env env, napi_status status, void* data) {
  job* j = (job*)data;
  napi_value result = NULL;
  j->ac->inflight--;
  if (status != napi_ok) {
    napi_reject_deferred(env, j->deferred, make_error(env, GBV_E_DEVICE, "async work cancelled"));
  } else if (j->rc != GBV_OK) {
    napi_reject_deferred(env, j->deferred, make_error(env, j->rc, j->err));
  } else {
    switch (j->op) {
      case OP_VERIFY_SETS:
        napi_get_boolean(env, j->out[0] == 1, &result);
        break;
      case OP_VERIFY_SETS_MULTI:
        napi_create_array_with_length(env, j->n_out, &result);
        for (size_t c = 0; c < j->n_out; ++c) {
          napi_value x;
          if (j->out[c] == GBV_CALL_REJECTED)
            x = make_error(env, GBV_E_EMPTY_AGGREGATE, "EMPTY_AGGREGATE_ARRAY");
          else
            napi_get_boolean(env, j->out[c] == 1, &x);
          napi_set_element(env, result, (uint32_t)c, x);
        }
        break;
      case OP_SAME_MESSAGE_MULTI: {
        size_t nc = j->sets.call_off.n ? j->sets.call_off.n - 1 : 0;
        napi_create_array_with_length(env, nc, &result);
        for (size_t c = 0; c < nc; ++c) {
          uint32_t a = j->sets.call_off.p[c], b = j->sets.call_off.p[c + 1];
          napi_value arr;
          if (c < j->sm_packed.n && j->sm_packed.p[c]) {  /* packed call: a Uint8Array, as waitPass answers it */
            void* dst = NULL;
            napi_value ab;
            napi_create_arraybuffer(env, b > a ? b - a : 1, &dst, &ab);
            if (b > a) memcpy(dst, j->out + a, b - a);
            napi_create_typedarray(env, napi_uint8_array, b - a, ab, 0, &arr);
          } else {
            napi_create_array_with_length(env, b - a, &arr);
            for (uint32_t i = a; i < b; ++i) {
              napi_value x;
              napi_get_boolean(env, j->out[i] == 1, &x);
              napi_set_element(env, arr, i - a, x);
            }
          }
          napi_set_element(env, result, (uint32_t)c, arr);
        }
        break;
      }
      case OP_CLOSE:
        napi_get_undefined(env, &result);
        break;
    }
    napi_resolve_deferred(env, j->deferred, result);
  }
  napi_delete_async_work(env, j->work);
  napi_delete_reference(env, j->ctx_ref);
  sets_free(&j->sets);
  free(j->sm_idx.p); free(j->sm_sigs.p); free(j->sm_msgs.p); free(j->sm_packed.p);
  free(j->out);
  free(j);
}

/* ctxv: the context external the job works on, referenced until the job completes so that a
 * context dropped by JS while work is queued is not finalized under it. */
static napi_value queue(napi_env env, job* j, const char* name, napi_value ctxv) {
  napi_value promise, res_name;
  napi_create_reference(env, ctxv, 1, &j->ctx_ref);
  napi_create_promise(env, &j->deferred, &promise);
  napi_create_string_utf8(env, name, NAPI_AUTO_LENGTH, &res_name);
  napi_create_async_work(env, NULL, res_name, execute, complete, j, &j->work);
  j->ac->inflight++;
  napi_queue_async_work(env, j->work);
  return promise;
}

/* A promise already rejected with QUEUE_ABORTED: work submitted after close() (the pool's
 * verifySignatureSets is async, so its QueueError surfaces as a rejection, index.ts:303-305). */
static napi_value rejected_closed(napi_env env) {
  napi_value p;
  napi_deferred d;
  napi_create_promise(env, &d, &p);
  napi_reject_deferred(env, d, make_error(env, GBV_E_CLOSED, "QUEUE_ABORTED"));
  return p;
}

static job* new_job(napi_env env, addon_ctx* ac, int op) {
  (void)env;
  job* j = (job*)calloc(1, sizeof(job));
  j->op = op;
  j->ac = ac;
  return j;
}

static void drop_job(job* j) {
  sets_free(&j->sets);
  free(j->sm_idx.p); free(j->sm_sigs.p); free(j->sm_msgs.p); free(j->sm_packed.p);
  free(j);
}

/* ---- exported functions ------------------------------------------------------------------- */
static void pass_release(struct pass_s* p);
static void ctx_finalize(napi_env env, void* data, void* hint) {
  (void)env; (void)hint;
  addon_ctx* ac = (addon_ctx*)data;
  /* passes still referenced by a slot: one whose JS object is gone is freed here; one whose object
   * lives on loses its context (its own finalizer frees it) -- in either order of the two finalizers
   * (Node-API orders none of them at environment teardown) no pass reaches freed memory */
  for (int k = 0; k < MAX_PASSES; ++k)
    if (ac->slots[k].pass) pass_release(ac->slots[k].pass);
  if (ac->ctx) {
    for (int k = 0; k < MAX_PASSES; ++k) {
      if (ac->slots[k].sm) gbv_sm_batch_destroy(ac->ctx, ac->slots[k].sm);
      if (ac->slots[k].vs) gbv_vs_batch_destroy(ac->ctx, ac->slots[k].vs);
    }
    gbv_destroy(ac->ctx);
  }
  for (int k = 0; k < MAX_PASSES; ++k) pthread_mutex_destroy(&ac->slots[k].mu);
  pthread_mutex_destroy(&ac->mu);
  free(ac);
}

static napi_value js_open(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  uint32_t dev = 0;
  if (argc >= 1 && !get_u32(env, argv[0], &dev)) {
    napi_throw_type_error(env, "GBV_E_ARG", "device must be a number");
    return NULL;
  }
  gbv_ctx* c = NULL;
  int rc = gbv_init((int)dev, &c);
  if (rc != GBV_OK) {
    throw_rc(env, rc, "gbv_init failed: no usable HIP device");
    return NULL;
  }
  addon_ctx* ac = (addon_ctx*)calloc(1, sizeof(addon_ctx));
  ac->ctx = c;
  pthread_mutex_init(&ac->mu, NULL);
  for (int k = 0; k < MAX_PASSES; ++k) pthread_mutex_init(&ac->slots[k].mu, NULL);
  napi_value ext;
  NAPI_OK(env, napi_create_external(env, ac, ctx_finalize, NULL, &ext));
  return ext;
}

static napi_value js_add_pubkeys(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  addon_ctx* ac = argc >= 1 ? get_ctx(env, argv[0]) : NULL;
  if (!ac) return NULL;
  uint32_t first;
  const uint8_t* d;
  size_t len;
  if (argc < 3 || !get_u32(env, argv[1], &first) || !get_bytes(env, argv[2], &d, &len) || len % 48) {
    napi_throw_type_error(env, "GBV_E_ARG", "addPubkeys(ctx, firstIndex, pk48s: Uint8Array of n*48 bytes, validate)");
    return NULL;
  }
  bool validate = false;
  if (argc >= 4) napi_get_value_bool(env, argv[3], &validate);
  if (ac->closed || !ac->ctx) {
    throw_rc(env, GBV_E_CLOSED, "QUEUE_ABORTED");
    return NULL;
  }
  size_t n = len / 48;
  void* st_data = NULL;
  napi_value ab, st;
  NAPI_OK(env, napi_create_arraybuffer(env, n ? n : 1, &st_data, &ab));
  NAPI_OK(env, napi_create_typedarray(env, napi_uint8_array, n, ab, 0, &st));
  lock_begin(ac);
  int rc = gbv_pubkeys_append(ac->ctx, first, d, n, validate ? 1 : 0, (uint8_t*)st_data);
  const char* msg = rc ? gbv_last_error(ac->ctx) : "";
  if (rc) throw_rc(env, rc, msg);
  lock_end(ac);
  return rc ? NULL : st;
}

static napi_value aggregate_impl(napi_env env, napi_callback_info info, int serialized) {
  size_t argc = 3;
  napi_value argv[3];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  addon_ctx* ac = argc >= 1 ? get_ctx(env, argv[0]) : NULL;
  if (!ac) return NULL;
  if (ac->closed || !ac->ctx) {
    throw_rc(env, GBV_E_CLOSED, "QUEUE_ABORTED");
    return NULL;
  }
  uint8_t out[48];
  int rc;
  if (serialized) {
    const uint8_t* d;
    size_t len;
    if (argc < 2 || !get_bytes(env, argv[1], &d, &len) || len % 48) {
      napi_throw_type_error(env, "GBV_E_ARG", "aggregateSerializedPubkeys(ctx, pk48s: Uint8Array of n*48 bytes, validate)");
      return NULL;
    }
    bool validate = false;
    if (argc >= 3) napi_get_value_bool(env, argv[2], &validate);
    lock_begin(ac);
    rc = gbv_aggregate_serialized_pubkeys(ac->ctx, d, len / 48, validate ? 1 : 0, out);
  } else {
    sets_buf tmp;
    memset(&tmp, 0, sizeof tmp);
    bool ja = false;
    if (argc >= 2) napi_is_array(env, argv[1], &ja);
    if (!ja) {
      napi_throw_type_error(env, "GBV_E_ARG", "aggregatePubkeys(ctx, indices: number[])");
      return NULL;
    }
    uint32_t k = 0;
    napi_get_array_length(env, argv[1], &k);
    for (uint32_t i = 0; i < k; ++i) {
      napi_value x;
      uint32_t u;
      napi_get_element(env, argv[1], i, &x);
      if (!get_u32(env, x, &u)) {
        sets_free(&tmp);
        napi_throw_type_error(env, "GBV_E_ARG", "indices must be numbers");
        return NULL;
      }
      uv_push(&tmp.arena, u);
    }
    lock_begin(ac);
    rc = gbv_aggregate_pubkeys(ac->ctx, tmp.arena.p, k, out);
    sets_free(&tmp);
  }
  if (rc) {
    throw_rc(env, rc, gbv_last_error(ac->ctx));
    lock_end(ac);
    return NULL;
  }
  lock_end(ac);
  void* p;
  napi_value ab, res;
  NAPI_OK(env, napi_create_arraybuffer(env, 48, &p, &ab));
  memcpy(p, out, 48);
  NAPI_OK(env, napi_create_typedarray(env, napi_uint8_array, 48, ab, 0, &res));
  return res;
}

static napi_value js_aggregate_pubkeys(napi_env env, napi_callback_info info) { return aggregate_impl(env, info, 0); }
static napi_value js_aggregate_serialized(napi_env env, napi_callback_info info) { return aggregate_impl(env, info, 1); }

/* aggregateSignatures(ctx, sigs: Uint8Array of n*96 bytes, validate) -> Uint8Array(96), synchronous
 * like blst's aggregateSignatures (singleThread.ts:55); gbv_aggregate_signatures. */
static napi_value js_aggregate_signatures(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  addon_ctx* ac = argc >= 1 ? get_ctx(env, argv[0]) : NULL;
  if (!ac) return NULL;
  const uint8_t* d;
  size_t len;
  if (argc < 2 || !get_bytes(env, argv[1], &d, &len) || len % 96) {
    napi_throw_type_error(env, "GBV_E_ARG", "aggregateSignatures(ctx, sig96s: Uint8Array of n*96 bytes, validate)");
    return NULL;
  }
  bool validate = true;
  if (argc >= 3) napi_get_value_bool(env, argv[2], &validate);
  if (ac->closed || !ac->ctx) {
    throw_rc(env, GBV_E_CLOSED, "QUEUE_ABORTED");
    return NULL;
  }
  uint8_t out[96];
  lock_begin(ac);
  int rc = gbv_aggregate_signatures(ac->ctx, len ? d : (const uint8_t*)"", len / 96, 96, validate ? 1 : 0, out);
  if (rc) {
    throw_rc(env, rc, gbv_last_error(ac->ctx));
    lock_end(ac);
    return NULL;
  }
  lock_end(ac);
  void* p;
  napi_value ab, res;
  NAPI_OK(env, napi_create_arraybuffer(env, 96, &p, &ab));
  memcpy(p, out, 96);
  NAPI_OK(env, napi_create_typedarray(env, napi_uint8_array, 96, ab, 0, &res));
  return res;
}

/* validateSignatures(ctx, sigs: Uint8Array of n*96 bytes) -> Uint8Array(n) of GBV_PT_* codes:
 * Signature.fromBytes(sig, true) per signature (singleThread.ts:44-52); gbv_signatures_validate. */
static napi_value js_validate_signatures(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  addon_ctx* ac = argc >= 1 ? get_ctx(env, argv[0]) : NULL;
  if (!ac) return NULL;
  const uint8_t* d;
  size_t len;
  if (argc < 2 || !get_bytes(env, argv[1], &d, &len) || len % 96) {
    napi_throw_type_error(env, "GBV_E_ARG", "validateSignatures(ctx, sig96s: Uint8Array of n*96 bytes)");
    return NULL;
  }
  if (ac->closed || !ac->ctx) {
    throw_rc(env, GBV_E_CLOSED, "QUEUE_ABORTED");
    return NULL;
  }
  size_t n = len / 96;
  void* st_data = NULL;
  napi_value ab, st;
  NAPI_OK(env, napi_create_arraybuffer(env, n ? n : 1, &st_data, &ab));
  NAPI_OK(env, napi_create_typedarray(env, napi_uint8_array, n, ab, 0, &st));
  lock_begin(ac);
  int rc = gbv_signatures_validate(ac->ctx, n ? d : (const uint8_t*)"", n, 96, (uint8_t*)st_data, NULL);
  if (rc) throw_rc(env, rc, gbv_last_error(ac->ctx));
  lock_end(ac);
  return rc ? NULL : st;
}

static napi_value js_verify_sets(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  addon_ctx* ac = argc >= 1 ? get_ctx(env, argv[0]) : NULL;
  if (!ac) return NULL;
  if (argc < 2) {
    napi_throw_type_error(env, "GBV_E_ARG", "verifySets(ctx, sets)");
    return NULL;
  }
  if (ac->closed) return rejected_closed(env);
  job* j = new_job(env, ac, OP_VERIFY_SETS);
  if (!j) return NULL;
  if (!marshal_sets(env, argv[1], &j->sets)) {
    drop_job(j);
    return NULL;
  }
  return queue(env, j, "gbvVerifySets", argv[0]);
}

static napi_value js_verify_sets_multi(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  addon_ctx* ac = argc >= 1 ? get_ctx(env, argv[0]) : NULL;
  if (!ac) return NULL;
  bool ja = false;
  if (argc >= 2) napi_is_array(env, argv[1], &ja);
  if (!ja) {
    napi_throw_type_error(env, "GBV_E_ARG", "verifySetsMulti(ctx, calls: sets[][])");
    return NULL;
  }
  if (ac->closed) return rejected_closed(env);
  job* j = new_job(env, ac, OP_VERIFY_SETS_MULTI);
  if (!j) return NULL;
  uint32_t nc = 0;
  napi_get_array_length(env, argv[1], &nc);
  uv_push(&j->sets.call_off, 0);
  for (uint32_t c = 0; c < nc; ++c) {
    napi_value call;
    napi_get_element(env, argv[1], c, &call);
    if (!marshal_sets(env, call, &j->sets)) {
      drop_job(j);
      return NULL;
    }
    uv_push(&j->sets.call_off, (uint32_t)j->sets.msg_off.n);
  }
  return queue(env, j, "gbvVerifySetsMulti", argv[0]);
}

static int marshal_same_message(napi_env env, napi_value arr, uvec* off, uvec* idx, bvec* sigs, bvec* msgs, bvec* packed);

static napi_value js_verify_same_message_multi(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  addon_ctx* ac = argc >= 1 ? get_ctx(env, argv[0]) : NULL;
  if (!ac) return NULL;
  bool ja = false;
  if (argc >= 2) napi_is_array(env, argv[1], &ja);
  if (!ja) {
    napi_throw_type_error(env, "GBV_E_ARG", "verifySameMessageMulti(ctx, calls: {sets: {index, signature}[], message}[])");
    return NULL;
  }
  if (ac->closed) return rejected_closed(env);
  job* j = new_job(env, ac, OP_SAME_MESSAGE_MULTI);
  if (!j) return NULL;
  if (!marshal_same_message(env, argv[1], &j->sets.call_off, &j->sm_idx, &j->sm_sigs, &j->sm_msgs, &j->sm_packed)) {
    drop_job(j);
    return NULL;
  }
  return queue(env, j, "gbvVerifySameMessageMulti", argv[0]);
}

/* ---- streamed passes ------------------------------------------------------------------------ */
typedef struct pass_s {
  addon_ctx* ac;
  int slot;
  int has_sm, has_df;
  int rc_sm, rc_df;
  char err_sm[256], err_df[256];
  uvec sm_off;             /* same-message calls: set offsets */
  size_t n_df;             /* default calls */
  uint8_t *sm_valid, *df_valid;
  bvec sm_packed;          /* per same-message call: 1 = packed sets (result as a Uint8Array) */
  int sm_flat;             /* the pass-wide flat form: one Uint8Array of every set's result */
  napi_deferred deferred;
  napi_async_work work;
  napi_ref ctx_ref;        /* the context external, alive while the pass is */
  int queued;              /* waitPass called */
  int done;                /* waitPass settled */
  int external_gone;       /* the JS pass object was finalized */
} pass;

/* The flat form of a pass's same-message calls, built by the JS queue (addon/gpu_bls_verifier.js
 * _runPass): {counts: Uint32Array(calls), messages: Uint8Array(32 calls), indices: Uint32Array(n),
 * signatures: Uint8Array(96 n)} -- four buffers per PASS, where the per-call forms cost ~10 Node-API
 * calls per call (~4 us each call on this Node) and the object form ~4 per set.  Returns 1, 0 (and
 * throws) on a malformed argument, -1 when obj is not the flat form. */
static int marshal_same_message_flat(napi_env env, napi_value obj, uvec* off, uvec* idx, bvec* sigs, bvec* msgs) {
  keyset ks;
  keys_init(env, &ks);
  napi_value cv, mv, iv, sv;
  if (!get_key(env, obj, ks.k[K_COUNTS], &cv)) return -1;
  const uint32_t *cnt, *ix;
  const uint8_t *m, *sg;
  size_t nc = 0, n = 0, ml = 0, sl = 0;
  if (!get_u32_array(env, cv, &cnt, &nc) || !get_key(env, obj, ks.k[K_MESSAGES], &mv) || !get_bytes(env, mv, &m, &ml) || ml != 32 * nc ||
      !get_key(env, obj, ks.k[K_INDICES], &iv) || !get_u32_array(env, iv, &ix, &n) || !get_key(env, obj, ks.k[K_SIGNATURES], &sv) ||
      !get_bytes(env, sv, &sg, &sl) || sl != 96 * n) {
    napi_throw_type_error(env, "GBV_E_ARG", "flat calls: {counts: Uint32Array(c), messages: Uint8Array(32 c), indices: Uint32Array(n), signatures: Uint8Array(96 n)}");
    return 0;
  }
  uint64_t total = 0;
  uv_push(off, 0);
  for (size_t c = 0; c < nc; ++c) {
    total += cnt[c];
    if (total > n) {
      napi_throw_range_error(env, "GBV_E_ARG", "flat calls: counts exceed the indices");
      return 0;
    }
    uv_push(off, (uint32_t)total);
  }
  if (total != n) {
    napi_throw_range_error(env, "GBV_E_ARG", "flat calls: counts do not sum to the indices");
    return 0;
  }
  uv_push_n(idx, ix, n);
  bv_push(sigs, sg, 96 * n);
  bv_push(msgs, m, 32 * nc);
  return 1;
}

/* Marshal a same-message call list ({sets, message}[]) into idx / sigs / msgs.  A call's sets are either
 * {index, signature}[] or the packed form {indices: Uint32Array(n), signatures: Uint8Array(96 n)}
 * (copied in two memcpys; packed[c] = 1 then, so waitPass answers that call with a Uint8Array). */
static int marshal_same_message(napi_env env, napi_value arr, uvec* off, uvec* idx, bvec* sigs, bvec* msgs, bvec* packed) {
  keyset ks;
  keys_init(env, &ks);
  bool ja = false;
  napi_is_array(env, arr, &ja);
  if (!ja) {
    napi_throw_type_error(env, "GBV_E_ARG", "sameMessageCalls must be an array of {sets, message}");
    return 0;
  }
  uint32_t nc = 0;
  napi_get_array_length(env, arr, &nc);
  uv_push(off, 0);
  static const uint8_t zero96[96] = {0};
  for (uint32_t c = 0; c < nc; ++c) {
    napi_value call, sets, msg;
    napi_get_element(env, arr, c, &call);
    const uint8_t* d;
    size_t len;
    bool sa = false;
    if (!get_key(env, call, ks.k[K_MESSAGE], &msg) || !get_bytes(env, msg, &d, &len) || len != 32 || !get_key(env, call, ks.k[K_SETS], &sets) ||
        napi_is_array(env, sets, &sa) != napi_ok) {
      napi_throw_type_error(env, "GBV_E_ARG", "each call needs sets and message: 32-byte Uint8Array");
      return 0;
    }
    bv_push(msgs, d, 32);
    if (!sa) {  /* packed: signatures as one Uint8Array(96 n), or as an array of n Uint8Arrays */
      napi_value iv, sv;
      const uint32_t* ix = NULL;
      size_t n = 0;
      bool list = false;
      bool ixl = false;
      if (!get_key(env, sets, ks.k[K_INDICES], &iv) || napi_is_array(env, iv, &ixl) != napi_ok || (!ixl && !get_u32_array(env, iv, &ix, &n)) ||
          !get_key(env, sets, ks.k[K_SIGNATURES], &sv) || napi_is_array(env, sv, &list) != napi_ok) {
        napi_throw_type_error(env, "GBV_E_ARG", "sets: {index, signature}[] or {indices: Uint32Array(n), signatures: Uint8Array(96 n) | Uint8Array[]}");
        return 0;
      }
      if (ixl) {  /* indices as a plain array of numbers (no typed array allocated per call by the caller) */
        uint32_t m = 0;
        napi_get_array_length(env, iv, &m);
        n = m;
        for (uint32_t i = 0; i < m; ++i) {
          napi_value x;
          uint32_t u;
          napi_get_element(env, iv, i, &x);
          if (!get_u32(env, x, &u)) {
            napi_throw_type_error(env, "GBV_E_ARG", "indices must be numbers");
            return 0;
          }
          uv_push(idx, u);
        }
      }
      if (list) {  /* the caller's own signature objects (chain/bls/gpu/index.ts): copied here, one memcpy each */
        uint32_t m = 0;
        napi_get_array_length(env, sv, &m);
        if (m != n) {
          napi_throw_type_error(env, "GBV_E_ARG", "signatures: one Uint8Array per index");
          return 0;
        }
        if (!ixl) uv_push_n(idx, ix, n);
        if (sigs->n + 96 * n > sigs->cap) {
          sigs->cap = (sigs->n + 96 * n) * 2 + 64;
          sigs->p = (uint8_t*)realloc(sigs->p, sigs->cap);
        }
        for (uint32_t i = 0; i < m; ++i) {
          napi_value e;
          napi_get_element(env, sv, i, &e);
          if (!get_bytes(env, e, &d, &len)) {
            napi_throw_type_error(env, "GBV_E_ARG", "signatures: one Uint8Array per index");
            return 0;
          }
          /* another length throws in Signature.fromBytes -> false for that set (zero bytes: BAD_ENCODING) */
          memcpy(sigs->p + sigs->n, len == 96 ? d : zero96, 96);
          sigs->n += 96;
        }
      } else {
        if (!get_bytes(env, sv, &d, &len) || len != 96 * n) {
          napi_throw_type_error(env, "GBV_E_ARG", "sets: {index, signature}[] or {indices: Uint32Array(n), signatures: Uint8Array(96 n) | Uint8Array[]}");
          return 0;
        }
        if (!ixl) uv_push_n(idx, ix, n);
        bv_push(sigs, d, 96 * n);
      }
      uv_push(off, (uint32_t)idx->n);
      const uint8_t one = 1;
      if (packed) bv_push(packed, &one, 1);
      continue;
    }
    const uint8_t zero = 0;
    if (packed) bv_push(packed, &zero, 1);
    uint32_t n = 0;
    napi_get_array_length(env, sets, &n);
    for (uint32_t i = 0; i < n; ++i) {
      napi_value e, v;
      uint32_t ix;
      napi_get_element(env, sets, i, &e);
      if (!get_key(env, e, ks.k[K_INDEX], &v) || !get_u32(env, v, &ix) || !get_key(env, e, ks.k[K_SIGNATURE], &v) || !get_bytes(env, v, &d, &len)) {
        napi_throw_type_error(env, "GBV_E_ARG", "a same-message set is {index: number, signature: Uint8Array}");
        return 0;
      }
      uv_push(idx, ix);
      bv_push(sigs, len == 96 ? d : zero96, 96); /* another length throws in fromBytes -> false */
    }
    uv_push(off, (uint32_t)idx->n);
  }
  return 1;
}

static void pass_free(napi_env env, pass* p) {
  if (p->ctx_ref) napi_delete_reference(env, p->ctx_ref);
  free(p->sm_off.p);
  free(p->sm_packed.p);
  free(p->sm_valid);
  free(p->df_valid);
  free(p);
}

/* The context's finalizer lets go of a pass its slot still holds (see ctx_finalize). */
static void pass_release(struct pass_s* p) {
  if (p->queued) return;  /* its waitPass work owns it (torn down with the environment) */
  if (p->external_gone) {
    /* the reference to the context external is being torn down with it: only the memory is freed */
    free(p->sm_off.p);
    free(p->sm_packed.p);
    free(p->sm_valid);
    free(p->df_valid);
    free(p);
  } else {
    p->ac = NULL;
  }
}

/* The JS pass object is gone.  A finalizer touches neither the context nor the device (Node-API does
 * not order finalizers at environment teardown, so the context may be freed already): a pass whose
 * waitPass is still running is freed by pass_complete; a pass never waited (a broken caller: every
 * submitted pass must be waited once) stays in its slot, marked, and the next submitPass or close()
 * waits for it and frees it (reclaim_orphans); a pass whose context is gone is freed here. */
static void pass_finalize(napi_env env, void* data, void* hint) {
  (void)hint;
  pass* p = (pass*)data;
  if (!p->ac) {
    pass_free(env, p);
    return;
  }
  if (!p->done) {
    p->external_gone = 1;
    return;
  }
  pass_free(env, p);
}

/* Free the slots of passes whose JS objects were dropped without waitPass (JS thread). */
static void reclaim_orphans(napi_env env, addon_ctx* ac) {
  for (int k = 0; k < MAX_PASSES; ++k) {
    pass_slot* sl = &ac->slots[k];
    pass* p = sl->pass;
    if (!p || p->queued || !p->external_gone) continue;
    pthread_mutex_lock(&sl->mu);
    if (ac->ctx && p->has_sm && !p->rc_sm && sl->sm) gbv_sm_batch_wait(ac->ctx, sl->sm, NULL);
    if (ac->ctx && p->has_df && !p->rc_df && sl->vs) gbv_vs_batch_wait(ac->ctx, sl->vs, NULL);
    pthread_mutex_unlock(&sl->mu);
    sl->busy = 0;
    sl->pass = NULL;
    ac->inflight--;
    pass_free(env, p);
  }
}

/* submitPass(ctx, sameMessageCalls | null, defaultCalls | null): fill and submit both device batches of
 * one pass on a free slot, synchronously (no device wait); a group that fails to stage is reported by
 * waitPass as that group's Error.  Throws GBV_E_BUSY when MAX_PASSES passes are already in flight. */
static napi_value js_submit_pass(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  addon_ctx* ac = argc >= 1 ? get_ctx(env, argv[0]) : NULL;
  if (!ac) return NULL;
  if (ac->closed || !ac->ctx) {
    throw_rc(env, GBV_E_CLOSED, "QUEUE_ABORTED");
    return NULL;
  }
  reclaim_orphans(env, ac);
  int k = 0;
  while (k < MAX_PASSES && ac->slots[k].busy) ++k;
  if (k == MAX_PASSES) {
    napi_throw_error(env, "GBV_E_BUSY", "every pass slot is in flight");
    return NULL;
  }
  pass_slot* sl = &ac->slots[k];
  napi_valuetype t0 = napi_null, t1 = napi_null;
  if (argc >= 2) napi_typeof(env, argv[1], &t0);
  if (argc >= 3) napi_typeof(env, argv[2], &t1);
  pass* p = (pass*)calloc(1, sizeof(pass));
  p->ac = ac;
  p->slot = k;
  uvec sm_idx = {0};
  bvec sm_sigs = {0}, sm_msgs = {0};
  sets_buf df;
  memset(&df, 0, sizeof df);
  int ok = 1;
  if (t0 != napi_null && t0 != napi_undefined) {
    p->has_sm = 1;
    bool sm_arr = false;
    napi_is_array(env, argv[1], &sm_arr);
    const int flat = sm_arr ? -1 : marshal_same_message_flat(env, argv[1], &p->sm_off, &sm_idx, &sm_sigs, &sm_msgs);
    if (flat < 0)
      ok = marshal_same_message(env, argv[1], &p->sm_off, &sm_idx, &sm_sigs, &sm_msgs, &p->sm_packed);
    else
      ok = flat, p->sm_flat = 1;
  }
  if (ok && t1 != napi_null && t1 != napi_undefined) {
    bool ja = false;
    napi_is_array(env, argv[2], &ja);
    if (!ja) {
      napi_throw_type_error(env, "GBV_E_ARG", "defaultCalls must be an array of set arrays");
      ok = 0;
    } else {
      p->has_df = 1;
      uint32_t nc = 0;
      napi_get_array_length(env, argv[2], &nc);
      uv_push(&df.call_off, 0);
      for (uint32_t c = 0; ok && c < nc; ++c) {
        napi_value call;
        napi_get_element(env, argv[2], c, &call);
        ok = marshal_sets(env, call, &df);
        uv_push(&df.call_off, (uint32_t)df.msg_off.n);
      }
      p->n_df = nc;
    }
  }
  if (!ok) {
    free(sm_idx.p); free(sm_sigs.p); free(sm_msgs.p);
    sets_free(&df);
    pass_free(env, p);
    return NULL;
  }
  /* stage + enqueue (the context lock inside libgbv orders this against pool threads) */
  pthread_mutex_lock(&sl->mu);
  static const uint32_t zero_off[1] = {0};
  if (!sl->sm && gbv_sm_batch_create(ac->ctx, 0, zero_off, NULL, NULL, NULL, &sl->sm) != GBV_OK) sl->sm = NULL;
  if (!sl->vs && gbv_vs_batch_create(ac->ctx, 0, zero_off, NULL, NULL, &sl->vs) != GBV_OK) sl->vs = NULL;
  if (p->has_sm) {
    size_t nc = p->sm_off.n ? p->sm_off.n - 1 : 0;
    p->sm_valid = (uint8_t*)calloc(sm_idx.n ? sm_idx.n : 1, 1);
    p->rc_sm = !sl->sm ? GBV_E_OOM
                       : gbv_sm_batch_fill(ac->ctx, sl->sm, nc, p->sm_off.p, sm_idx.p, sm_sigs.p ? sm_sigs.p : (const uint8_t*)"",
                                           sm_msgs.p ? sm_msgs.p : (const uint8_t*)"");
    if (!p->rc_sm) p->rc_sm = gbv_sm_batch_submit(ac->ctx, sl->sm);
    if (p->rc_sm) snprintf(p->err_sm, sizeof p->err_sm, "%s", gbv_last_error(ac->ctx));
  }
  if (p->has_df) {
    gbv_set* r = sets_records(&df);
    p->df_valid = (uint8_t*)calloc(p->n_df ? p->n_df : 1, 1);
    p->rc_df = !sl->vs ? GBV_E_OOM : gbv_vs_batch_fill(ac->ctx, sl->vs, p->n_df, df.call_off.p, r, df.arena.p);
    if (!p->rc_df) p->rc_df = gbv_vs_batch_submit(ac->ctx, sl->vs);
    if (p->rc_df) snprintf(p->err_df, sizeof p->err_df, "%s", gbv_last_error(ac->ctx));
    free(r);
  }
  pthread_mutex_unlock(&sl->mu);
  free(sm_idx.p); free(sm_sigs.p); free(sm_msgs.p);
  sets_free(&df);
  sl->busy = 1;
  sl->pass = p;
  ac->inflight++;
  napi_create_reference(env, argv[0], 1, &p->ctx_ref);
  napi_value ext;
  NAPI_OK(env, napi_create_external(env, p, pass_finalize, NULL, &ext));
  return ext;
}

static void pass_execute(napi_env env, void* data) {
  (void)env;
  pass* p = (pass*)data;
  addon_ctx* ac = p->ac;
  pass_slot* sl = &ac->slots[p->slot];
  pthread_mutex_lock(&sl->mu);  /* the device wait; close() destroys the slot only after it */
  if (p->has_sm && !p->rc_sm) {
    p->rc_sm = sl->sm && ac->ctx ? gbv_sm_batch_wait(ac->ctx, sl->sm, p->sm_valid) : GBV_E_CLOSED;
    if (p->rc_sm) snprintf(p->err_sm, sizeof p->err_sm, "%s", ac->ctx ? gbv_last_error(ac->ctx) : "QUEUE_ABORTED");
  }
  if (p->has_df && !p->rc_df) {
    p->rc_df = sl->vs && ac->ctx ? gbv_vs_batch_wait(ac->ctx, sl->vs, p->df_valid) : GBV_E_CLOSED;
    if (p->rc_df) snprintf(p->err_df, sizeof p->err_df, "%s", ac->ctx ? gbv_last_error(ac->ctx) : "QUEUE_ABORTED");
  }
  pthread_mutex_unlock(&sl->mu);
}

static void pass_complete(napi_env env, napi_status status, void* data) {
  pass* p = (pass*)data;
  p->ac->slots[p->slot].busy = 0;
  p->ac->slots[p->slot].pass = NULL;
  p->ac->inflight--;
  napi_value result, x;
  napi_create_object(env, &result);
  if (status != napi_ok) {
    napi_reject_deferred(env, p->deferred, make_error(env, GBV_E_DEVICE, "async work cancelled"));
  } else {
    if (!p->has_sm) {
      napi_get_null(env, &x);
    } else if (p->rc_sm) {
      x = make_error(env, p->rc_sm, p->err_sm);
    } else if (p->sm_flat) {  /* one Uint8Array of 0 / 1 over every set of the pass, in call order */
      const size_t n = p->sm_off.n ? p->sm_off.p[p->sm_off.n - 1] : 0;
      void* dst = NULL;
      napi_value ab;
      napi_create_arraybuffer(env, n ? n : 1, &dst, &ab);
      if (n) memcpy(dst, p->sm_valid, n);
      napi_create_typedarray(env, napi_uint8_array, n, ab, 0, &x);
    } else {
      size_t nc = p->sm_off.n ? p->sm_off.n - 1 : 0;
      napi_create_array_with_length(env, nc, &x);
      for (size_t c = 0; c < nc; ++c) {
        uint32_t a = p->sm_off.p[c], b = p->sm_off.p[c + 1];
        napi_value arr;
        if (c < p->sm_packed.n && p->sm_packed.p[c]) {  /* packed call: one Uint8Array of 0 / 1 */
          void* dst = NULL;
          napi_value ab;
          napi_create_arraybuffer(env, b > a ? b - a : 1, &dst, &ab);
          if (b > a) memcpy(dst, p->sm_valid + a, b - a);
          napi_create_typedarray(env, napi_uint8_array, b - a, ab, 0, &arr);
        } else {
          napi_create_array_with_length(env, b - a, &arr);
          for (uint32_t i = a; i < b; ++i) {
            napi_value v;
            napi_get_boolean(env, p->sm_valid[i] == 1, &v);
            napi_set_element(env, arr, i - a, v);
          }
        }
        napi_set_element(env, x, (uint32_t)c, arr);
      }
    }
    napi_set_named_property(env, result, "sameMessage", x);
    if (!p->has_df) {
      napi_get_null(env, &x);
    } else if (p->rc_df) {
      x = make_error(env, p->rc_df, p->err_df);
    } else {
      napi_create_array_with_length(env, p->n_df, &x);
      for (size_t c = 0; c < p->n_df; ++c) {
        napi_value v;
        if (p->df_valid[c] == GBV_CALL_REJECTED)
          v = make_error(env, GBV_E_EMPTY_AGGREGATE, "EMPTY_AGGREGATE_ARRAY");
        else
          napi_get_boolean(env, p->df_valid[c] == 1, &v);
        napi_set_element(env, x, (uint32_t)c, v);
      }
    }
    napi_set_named_property(env, result, "default", x);
    napi_resolve_deferred(env, p->deferred, result);
  }
  napi_delete_async_work(env, p->work);
  p->done = 1;
  free(p->sm_valid);
  free(p->df_valid);
  p->sm_valid = p->df_valid = NULL;
  if (p->external_gone) pass_free(env, p);  /* else the external's finalizer frees it */
}

/* waitPass(pass) -> Promise: the device wait runs on the libuv pool; every submitted pass must be
 * waited exactly once (its slot is released when the promise settles). */
static napi_value js_wait_pass(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  napi_valuetype t;
  if (argc < 1 || napi_typeof(env, argv[0], &t) != napi_ok || t != napi_external) {
    napi_throw_type_error(env, "GBV_E_ARG", "expected a pass from submitPass()");
    return NULL;
  }
  pass* p = NULL;
  napi_get_value_external(env, argv[0], (void**)&p);
  if (!p || p->queued) {
    napi_throw_error(env, "GBV_E_ARG", "pass already waited");
    return NULL;
  }
  p->queued = 1;
  napi_value promise, name;
  napi_create_promise(env, &p->deferred, &promise);
  napi_create_string_utf8(env, "gbvWaitPass", NAPI_AUTO_LENGTH, &name);
  napi_create_async_work(env, NULL, name, pass_execute, pass_complete, p, &p->work);
  napi_queue_async_work(env, p->work);
  return promise;
}

static napi_value js_free_passes(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1], r;
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  addon_ctx* ac = argc >= 1 ? get_ctx(env, argv[0]) : NULL;
  if (!ac) return NULL;
  uint32_t f = 0;
  for (int k = 0; k < MAX_PASSES; ++k) f += ac->slots[k].busy ? 0 : 1;
  napi_create_uint32(env, (ac->closed || !ac->ctx) ? 0 : f, &r);
  return r;
}

static napi_value js_pubkey_count(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1], r;
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  addon_ctx* ac = argc >= 1 ? get_ctx(env, argv[0]) : NULL;
  if (!ac) return NULL;
  napi_create_double(env, ac->ctx ? (double)gbv_pubkeys_count(ac->ctx) : 0.0, &r);
  return r;
}

/* verifySetsSync(ctx, sets) -> boolean: verifyOnMainThread (index.ts:168-181) -- blocks the JS thread
 * like the reference's main-thread verifySignatureSetsMaybeBatch. */
static napi_value js_verify_sets_sync(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  addon_ctx* ac = argc >= 1 ? get_ctx(env, argv[0]) : NULL;
  if (!ac) return NULL;
  if (argc < 2) {
    napi_throw_type_error(env, "GBV_E_ARG", "verifySetsSync(ctx, sets)");
    return NULL;
  }
  if (ac->closed || !ac->ctx) {
    throw_rc(env, GBV_E_CLOSED, "QUEUE_ABORTED");
    return NULL;
  }
  sets_buf sb;
  memset(&sb, 0, sizeof sb);
  if (!marshal_sets(env, argv[1], &sb)) {
    sets_free(&sb);
    return NULL;
  }
  gbv_set* r = sets_records(&sb);
  uint8_t all = 0;
  int rc = gbv_verify_sets(ac->ctx, r, sb.msg_off.n, sb.arena.p, &all, NULL);
  free(r);
  sets_free(&sb);
  if (rc) {
    throw_rc(env, rc, gbv_last_error(ac->ctx));
    return NULL;
  }
  napi_value res;
  napi_get_boolean(env, all == 1, &res);
  return res;
}

/* vsPartial(ctx, sets) -> {partial: Uint8Array(576), ok: boolean} (gbv_vs_partial, synchronous):
 * this GPU's Fp12 Miller product over its shard of one large verifySignatureSets call. */
static napi_value js_vs_partial(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  addon_ctx* ac = argc >= 1 ? get_ctx(env, argv[0]) : NULL;
  if (!ac) return NULL;
  if (ac->closed || !ac->ctx) {
    throw_rc(env, GBV_E_CLOSED, "QUEUE_ABORTED");
    return NULL;
  }
  sets_buf sb;
  memset(&sb, 0, sizeof sb);
  if (argc < 2 || !marshal_sets(env, argv[1], &sb)) {
    sets_free(&sb);
    if (argc < 2) napi_throw_type_error(env, "GBV_E_ARG", "vsPartial(ctx, sets)");
    return NULL;
  }
  gbv_set* r = sets_records(&sb);
  void* part;
  napi_value ab, ta, res, okv;
  NAPI_OK(env, napi_create_arraybuffer(env, GBV_FP12_PARTIAL_BYTES, &part, &ab));
  uint8_t ok = 0;
  int rc = gbv_vs_partial(ac->ctx, r, sb.msg_off.n, sb.arena.p, (uint8_t*)part, &ok);
  free(r);
  sets_free(&sb);
  if (rc) {
    throw_rc(env, rc, gbv_last_error(ac->ctx));
    return NULL;
  }
  NAPI_OK(env, napi_create_typedarray(env, napi_uint8_array, GBV_FP12_PARTIAL_BYTES, ab, 0, &ta));
  napi_create_object(env, &res);
  napi_get_boolean(env, ok == 1, &okv);
  napi_set_named_property(env, res, "partial", ta);
  napi_set_named_property(env, res, "ok", okv);
  return res;
}

/* fp12Check(ctx, partials: Uint8Array of k*576 bytes) -> boolean (gbv_fp12_check). */
static napi_value js_fp12_check(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  addon_ctx* ac = argc >= 1 ? get_ctx(env, argv[0]) : NULL;
  if (!ac) return NULL;
  const uint8_t* d;
  size_t len;
  if (argc < 2 || !get_bytes(env, argv[1], &d, &len) || len % GBV_FP12_PARTIAL_BYTES) {
    napi_throw_type_error(env, "GBV_E_ARG", "fp12Check(ctx, partials: Uint8Array of k*576 bytes)");
    return NULL;
  }
  if (ac->closed || !ac->ctx) {
    throw_rc(env, GBV_E_CLOSED, "QUEUE_ABORTED");
    return NULL;
  }
  uint8_t one = 0;
  int rc = gbv_fp12_check(ac->ctx, len ? d : NULL, len / GBV_FP12_PARTIAL_BYTES, &one);
  if (rc) {
    throw_rc(env, rc, gbv_last_error(ac->ctx));
    return NULL;
  }
  napi_value res;
  napi_get_boolean(env, one == 1, &res);
  return res;
}

/* merkleRoots(ctx, chunks: Uint8Array of n * 2^depth * 32 bytes, depth) -> Uint8Array(32 n)
 * (gbv_merkle_roots: ContainerType.hashTreeRoot over field roots on the device). */
static napi_value js_merkle_roots(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  addon_ctx* ac = argc >= 1 ? get_ctx(env, argv[0]) : NULL;
  if (!ac) return NULL;
  const uint8_t* d;
  size_t len;
  uint32_t depth = 0;
  if (argc < 3 || !get_bytes(env, argv[1], &d, &len) || !get_u32(env, argv[2], &depth) || depth > 24 ||
      len % ((size_t)32 << depth)) {
    napi_throw_type_error(env, "GBV_E_ARG", "merkleRoots(ctx, chunks: Uint8Array of n*2^depth*32 bytes, depth <= 24)");
    return NULL;
  }
  if (ac->closed || !ac->ctx) {
    throw_rc(env, GBV_E_CLOSED, "QUEUE_ABORTED");
    return NULL;
  }
  size_t n = len / ((size_t)32 << depth);
  void* out = NULL;
  napi_value ab, ta;
  NAPI_OK(env, napi_create_arraybuffer(env, n ? 32 * n : 1, &out, &ab));
  NAPI_OK(env, napi_create_typedarray(env, napi_uint8_array, 32 * n, ab, 0, &ta));
  lock_begin(ac);
  int rc = gbv_merkle_roots(ac->ctx, n ? d : (const uint8_t*)"", n, depth, (uint8_t*)out);
  if (rc) throw_rc(env, rc, gbv_last_error(ac->ctx));
  lock_end(ac);
  return rc ? NULL : ta;
}

/* signingRoots(ctx, objectRoots: Uint8Array(32 n), domains: Uint8Array(32 k), domIdx: Uint32Array(n) | null)
 * -> Uint8Array(32 n) (gbv_signing_roots: computeSigningRoot, signingRoot.ts:7-13). */
static napi_value js_signing_roots(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  addon_ctx* ac = argc >= 1 ? get_ctx(env, argv[0]) : NULL;
  if (!ac) return NULL;
  const uint8_t *r, *dm;
  size_t rlen, dlen;
  if (argc < 3 || !get_bytes(env, argv[1], &r, &rlen) || rlen % 32 || !get_bytes(env, argv[2], &dm, &dlen) || dlen % 32 || dlen == 0) {
    napi_throw_type_error(env, "GBV_E_ARG", "signingRoots(ctx, objectRoots: Uint8Array(32 n), domains: Uint8Array(32 k), domIdx)");
    return NULL;
  }
  size_t n = rlen / 32;
  const uint32_t* idx = NULL;
  napi_valuetype t = napi_undefined;
  if (argc >= 4) napi_typeof(env, argv[3], &t);
  if (t != napi_undefined && t != napi_null) {
    bool is_ta = false;
    napi_is_typedarray(env, argv[3], &is_ta);
    napi_typedarray_type type;
    size_t m = 0, off;
    void* p = NULL;
    napi_value ab;
    if (!is_ta || napi_get_typedarray_info(env, argv[3], &type, &m, &p, &ab, &off) != napi_ok || type != napi_uint32_array || m != n) {
      napi_throw_type_error(env, "GBV_E_ARG", "domIdx must be a Uint32Array of one index per root");
      return NULL;
    }
    idx = (const uint32_t*)p;
  }
  if (ac->closed || !ac->ctx) {
    throw_rc(env, GBV_E_CLOSED, "QUEUE_ABORTED");
    return NULL;
  }
  void* out = NULL;
  napi_value ab, ta;
  NAPI_OK(env, napi_create_arraybuffer(env, n ? 32 * n : 1, &out, &ab));
  NAPI_OK(env, napi_create_typedarray(env, napi_uint8_array, 32 * n, ab, 0, &ta));
  lock_begin(ac);
  int rc = gbv_signing_roots(ac->ctx, n ? r : (const uint8_t*)"", n, dm, dlen / 32, idx, (uint8_t*)out);
  if (rc) throw_rc(env, rc, gbv_last_error(ac->ctx));
  lock_end(ac);
  return rc ? NULL : ta;
}

/* replicatePubkeys(ctx, srcFirst, srcN, dstFirst, n): slot[dstFirst + i] = slot[srcFirst + i % srcN]
 * (gbv_pubkeys_replicate: synthetic tables for benches and tests). */
static napi_value js_replicate_pubkeys(napi_env env, napi_callback_info info) {
  size_t argc = 5;
  napi_value argv[5];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  addon_ctx* ac = argc >= 1 ? get_ctx(env, argv[0]) : NULL;
  if (!ac) return NULL;
  uint32_t a = 0, b = 0, d = 0, n = 0;
  if (argc < 5 || !get_u32(env, argv[1], &a) || !get_u32(env, argv[2], &b) || !get_u32(env, argv[3], &d) || !get_u32(env, argv[4], &n)) {
    napi_throw_type_error(env, "GBV_E_ARG", "replicatePubkeys(ctx, srcFirst, srcN, dstFirst, n)");
    return NULL;
  }
  if (ac->closed || !ac->ctx) {
    throw_rc(env, GBV_E_CLOSED, "QUEUE_ABORTED");
    return NULL;
  }
  lock_begin(ac);
  int rc = gbv_pubkeys_replicate(ac->ctx, a, b, d, n);
  if (rc) throw_rc(env, rc, gbv_last_error(ac->ctx));
  lock_end(ac);
  return NULL;
}

static napi_value js_close(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  addon_ctx* ac = argc >= 1 ? get_ctx(env, argv[0]) : NULL;
  if (!ac) return NULL;
  if (ac->closed) {  // idempotent, like the pool's close()
    napi_value p;
    napi_deferred d;
    napi_create_promise(env, &d, &p);
    napi_value u;
    napi_get_undefined(env, &u);
    napi_resolve_deferred(env, d, u);
    return p;
  }
  reclaim_orphans(env, ac);
  job* j = (job*)calloc(1, sizeof(job));
  j->op = OP_CLOSE;
  j->ac = ac;
  ac->closed = 1;  // new calls reject with QUEUE_ABORTED; queued ones run before the destroy (mutex order)
  return queue(env, j, "gbvClose", argv[0]);
}

/* GBV_SEGV_TRACE=1 (diagnosis only): on SIGSEGV / SIGBUS, print the faulting address, the thread and
 * a backtrace of that thread to stderr, then die by the same signal.  It replaces the process's own
 * handler for these signals (V8's WebAssembly trap handler among them), so it stays off by default. */
static void segv_trace(int sig, siginfo_t* si, void* uc) {
  (void)uc;
  void* frames[64];
  char msg[160];
  int n = backtrace(frames, 64);
  int l = snprintf(msg, sizeof msg, "[gbv addon] signal %d at address %p in thread %ld\n", sig, si ? si->si_addr : NULL,
                   (long)syscall(SYS_gettid));
  if (l > 0 && write(2, msg, (size_t)l) < 0) {}
  backtrace_symbols_fd(frames, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

static napi_value init(napi_env env, napi_value exports) {
  if (getenv("GBV_SEGV_TRACE")) {
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = segv_trace;
    sa.sa_flags = SA_SIGINFO;
    sigaction(SIGSEGV, &sa, NULL);
    sigaction(SIGBUS, &sa, NULL);
  }
  napi_property_descriptor props[] = {
      {"open", NULL, js_open, NULL, NULL, NULL, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), NULL},
      {"addPubkeys", NULL, js_add_pubkeys, NULL, NULL, NULL, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), NULL},
      {"verifySets", NULL, js_verify_sets, NULL, NULL, NULL, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), NULL},
      {"verifySetsMulti", NULL, js_verify_sets_multi, NULL, NULL, NULL, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), NULL},
      {"verifySameMessageMulti", NULL, js_verify_same_message_multi, NULL, NULL, NULL, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), NULL},
      {"aggregatePubkeys", NULL, js_aggregate_pubkeys, NULL, NULL, NULL, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), NULL},
      {"aggregateSerializedPubkeys", NULL, js_aggregate_serialized, NULL, NULL, NULL, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), NULL},
      {"aggregateSignatures", NULL, js_aggregate_signatures, NULL, NULL, NULL, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), NULL},
      {"validateSignatures", NULL, js_validate_signatures, NULL, NULL, NULL, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), NULL},
      {"close", NULL, js_close, NULL, NULL, NULL, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), NULL},
      {"submitPass", NULL, js_submit_pass, NULL, NULL, NULL, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), NULL},
      {"waitPass", NULL, js_wait_pass, NULL, NULL, NULL, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), NULL},
      {"freePasses", NULL, js_free_passes, NULL, NULL, NULL, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), NULL},
      {"pubkeyCount", NULL, js_pubkey_count, NULL, NULL, NULL, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), NULL},
      {"verifySetsSync", NULL, js_verify_sets_sync, NULL, NULL, NULL, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), NULL},
      {"vsPartial", NULL, js_vs_partial, NULL, NULL, NULL, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), NULL},
      {"fp12Check", NULL, js_fp12_check, NULL, NULL, NULL, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), NULL},
      {"merkleRoots", NULL, js_merkle_roots, NULL, NULL, NULL, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), NULL},
      {"signingRoots", NULL, js_signing_roots, NULL, NULL, NULL, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), NULL},
      {"replicatePubkeys", NULL, js_replicate_pubkeys, NULL, NULL, NULL, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), NULL},
  };
  napi_define_properties(env, exports, sizeof props / sizeof props[0], props);
  napi_value mp;
  napi_create_uint32(env, MAX_PASSES, &mp);
  napi_set_named_property(env, exports, "MAX_PASSES", mp);
  return exports;
}

NAPI_MODULE(gbv_addon, init)
