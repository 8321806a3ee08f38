/*
 * gbv.h -- C ABI of the MI355X BLS12-381 signature-set verifier ("GPU BLS verifier").
 *
 * This is the drop-in boundary for Lodestar's IBlsVerifier hot path
 * (/root/reference/packages/beacon-node/src/chain/bls/interface.ts:25-68).  A Node-API addon
 *  or the Python host mirror (lodestar_amd/verifier.py) binds these symbols; no
 * torch or HIP types appear in the signatures.  Each context owns one GPU, three HIP streams
 * (per-set throughput kernels, chunk-level tail, hashing) and the HBM-resident pubkey table.
 * Entry points may be called from several host threads: each holds the context's lock while it
 * touches the context (the one-shot calls share one scratch batch and run one at a time); the
 * batch waits release it while they block on the device.  A batch object (gbv_sm_batch,
 * gbv_vs_batch) belongs to one caller from fill/submit to wait.  gbv_last_error reports the last
 * failure of the calling thread.
 *
 * Error convention: return 0 on success; per-set "false" results are carried
 * in the output byte arrays, never as errors.  Negative codes map to promise rejections:
 *   GBV_E_EMPTY_AGGREGATE  -- an aggregate set has no pubkeys (blst EMPTY_AGGREGATE_ARRAY,
 *                             bls/utils.ts:12 throws -> job.reject, multithread/index.ts:398-412)
 *   GBV_E_DEVICE           -- HIP error (rejects in-flight work like a worker comms failure,
 *                             multithread/index.ts:498-507)
 *   GBV_E_CLOSED           -- context destroyed / closed (QueueError QUEUE_ABORTED, index.ts:303-305)
 *   GBV_E_ARG              -- invalid argument (null pointer, index out of table range)
 *   GBV_E_BAD_POINT        -- a serialized point failed to deserialize where the reference throws
 *                             (aggregateSerializedPublicKeys over a malformed key)
 */
#ifndef GBV_H
#define GBV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GBV_OK 0
#define GBV_E_ARG (-1)
#define GBV_E_DEVICE (-2)
#define GBV_E_EMPTY_AGGREGATE (-3)
#define GBV_E_CLOSED (-4)
#define GBV_E_OOM (-5)
#define GBV_E_BAD_POINT (-6)

/* Per-call result byte of the multi-call entry points: 0 false, 1 true, GBV_CALL_REJECTED when the
 * call's promise rejects (an aggregate set without pubkeys: EMPTY_AGGREGATE_ARRAY). */
#define GBV_CALL_REJECTED 2

/* Point status codes written by gbv_pubkeys_append (blst BLST_ERROR equivalents). */
#define GBV_PT_OK 0
#define GBV_PT_BAD_ENCODING 1
#define GBV_PT_NOT_ON_CURVE 2
#define GBV_PT_NOT_IN_GROUP 3
#define GBV_PT_INFINITY 4

typedef struct gbv_ctx gbv_ctx;

/* One signature set of IBlsVerifier.verifySignatureSets (ISignatureSet,
 * state-transition/src/util/signatureSets.ts:4-23), in index form: the pubkeys are validator
 * indices into the HBM-resident index2pubkey table (epochCache.ts:126-133) -- idx_len == 1 for a
 * SingleSignatureSet, k for an AggregatedSignatureSet -- unless raw_pk48 is non-null (sets whose
 * pubkey comes from the message itself, e.g. blsToExecutionChange.ts:19-44; validated like
 * PublicKey.fromBytes(pk, true)). */
typedef struct gbv_set {
  uint32_t idx_off;          /* offset into index_arena */
  uint32_t idx_len;          /* number of pubkeys (0 => GBV_E_EMPTY_AGGREGATE) */
  const uint8_t* raw_pk48;   /* optional compressed pubkey, overrides the indices */
  const uint8_t* msg32;      /* signing root */
  const uint8_t* sig;        /* signature bytes as received (untrusted) */
  uint32_t sig_len;          /* 96 (compressed) or 192 (uncompressed); other lengths are invalid */
} gbv_set;

/* Create a context on HIP device `device` (one process per GPU; device is usually 0 or LOCAL_RANK). */
int gbv_init(int device, gbv_ctx** out);
/* Release the device table, stream and buffers.  Replaces close() of the worker pool
 * (multithread/index.ts:238-259). */
void gbv_destroy(gbv_ctx* ctx);
/* Human-readable description of the last error on this context. */
const char* gbv_last_error(gbv_ctx* ctx);

/* index2pubkey ingest (pubkeyCache.ts:50-69 syncPubkeys, epochCache.ts:1064-1083 addFinalizedPubkey):
 * decompress n 48-byte pubkeys on the device into table slots [first_index, first_index + n).
 * validate != 0 additionally runs the G1 subgroup + infinity check (PublicKey.fromBytes(pk, true)).
 * status (optional, n bytes) receives GBV_PT_* per key; invalid keys make their slot unusable. */
int gbv_pubkeys_append(gbv_ctx* ctx, uint32_t first_index, const uint8_t* pk48, size_t n, int validate,
                       uint8_t* status);
/* Number of table slots currently allocated (max index + 1). */
size_t gbv_pubkeys_count(gbv_ctx* ctx);
/* 1 when the per-slot comb tables for r*pk are built and used by the same-message path (default;
 * gbv_tune(ctx, "comb", 0) before the first gbv_pubkeys_append, or a failed allocation, selects the
 * ladder; results are identical either way).  No reference counterpart: an accelerator of index2pubkey. */
int gbv_comb_enabled(gbv_ctx* ctx);
/* Change a pipeline setting (no reference counterpart; results are identical for every value -- tests
 * and experiments use it to reach each pipeline form; nothing is read from the environment except
 * GBV_SYNC_DEBUG, a per-launch synchronisation for debugging).  Per context: "msm_min" (segments of at
 * least this many sets form their G2 sum with the bucket MSM; 0 = never), "msm_cooldown" (submits
 * without the MSM after a failing MSM segment), "segments" (pipeline segments per same-message
 * batch), "kprof" (1: record per-kernel timings, gbv_last_ops), "comb" (0: r*pk by the ladder; 1 only
 * before any key is appended).  Process-wide launch shapes: "hash_pair_max",
 * "hash_quad_max", "hash_coop_max", "prepare_split_max", "chunk_finish_wave_max", "vs_pre_max",
 * "vs_fs_maxc", "vs_quad_max", "vs_pair_max", "agg_slice", and the same-message failure path's split between
 * one wave per check (latency) and one thread per check (throughput): "fb_coop_max" (run / per-set checks,
 * at most 16384) and "group_thread_min" (chunk checks); "sm_quad_max" (chunk Miller values on lane quads
 * up to this many chunks of a segment).  GBV_E_ARG for an unknown name. */
int gbv_tune(gbv_ctx* ctx, const char* name, uint32_t value);

/* IBlsVerifier.verifySignatureSets (interface.ts:47; multithread/index.ts:157-207).
 * The sets are split with chunkifyMaximizeChunkSize(sets, 128) (multithread/utils.ts:4-18) and
 * each chunk is verified as one randomised batch (maybeBatch.ts:15-45).  *all_valid = AND over
 * chunks (0 for an empty list).  chunk_valid (optional) receives one byte per chunk.
 * Returns GBV_E_EMPTY_AGGREGATE if any set has idx_len == 0 and raw_pk48 == NULL. */
int gbv_verify_sets(gbv_ctx* ctx, const gbv_set* sets, size_t n, const uint32_t* index_arena,
                    uint8_t* all_valid, uint8_t* chunk_valid);

/* Many independent verifySignatureSets calls in ONE device pass -- the pool's dispatch of several
 * jobs (multithread/index.ts:357-514) and the worker's grouping of batchable requests
 * (worker.ts:29-107): call c covers sets [call_off[c], call_off[c+1]), call_off[0] == 0.  Every
 * call is chunked with chunkifyMaximizeChunkSize(128) and each chunk verified as one randomised
 * batch (verifyMultipleAggregateSignatures semantics, maybeBatch.ts:15-45); call_valid[c] is the
 * AND over the call's chunks (0 for an empty call) or GBV_CALL_REJECTED.  A failing call does not
 * affect the others (multithread.test.ts:109-129: an invalid set fails only its own request). */
int gbv_verify_sets_multi(gbv_ctx* ctx, size_t n_calls, const uint32_t* call_off, const gbv_set* sets,
                          const uint32_t* index_arena, uint8_t* call_valid);

/* Device-resident form of gbv_verify_sets_multi (inputs staged in HBM once, verified many times:
 * range sync / replay benches).  submit enqueues the whole verification and returns; wait blocks and
 * writes call_valid.  Per-set kernels run on the context's throughput stream and the chunk checks on
 * a tail stream, so consecutive batches overlap. */
typedef struct gbv_vs_batch gbv_vs_batch;
int gbv_vs_batch_create(gbv_ctx* ctx, size_t n_calls, const uint32_t* call_off, const gbv_set* sets,
                        const uint32_t* index_arena, gbv_vs_batch** out);
/* Refill an existing batch with a new workload (same rules as create), reusing its HBM and pinned
 * buffers: the streamed verifier keeps a few batches and cycles them.  The batch must not be in
 * flight.  The input copy is queued on the device, not waited for. */
int gbv_vs_batch_fill(gbv_ctx* ctx, gbv_vs_batch* b, size_t n_calls, const uint32_t* call_off, const gbv_set* sets,
                      const uint32_t* index_arena);
int gbv_vs_batch_submit(gbv_ctx* ctx, gbv_vs_batch* b);
int gbv_vs_batch_wait(gbv_ctx* ctx, gbv_vs_batch* b, uint8_t* call_valid);
void gbv_vs_batch_destroy(gbv_ctx* ctx, gbv_vs_batch* b);
/* Device ms of the last waited verifySignatureSets pass: [aggregate, hash+signature, miller, chunk checks]. */
int gbv_vs_last_kernel_ms(gbv_ctx* ctx, float* ms4);

/* IBlsVerifier.verifySignatureSetsSameMessage (interface.ts:55-59; multithread/index.ts:212-236):
 * n sets {validator index, 96-byte signature} over one 32-byte message.  valid[i] receives the
 * per-set boolean in input order (all-true on a passing randomised aggregate check, otherwise
 * per-set verification, jobItem.ts:93-125). */
int gbv_verify_same_message(gbv_ctx* ctx, const uint32_t* idx, const uint8_t* sigs96, size_t n,
                            const uint8_t* msg32, uint8_t* valid);

/* Many independent verifySignatureSetsSameMessage calls in one device pass (the GPU analogue of
 * the pool's job grouping, multithread/index.ts:519-534): call g covers sets
 * [call_off[g], call_off[g+1]) with message msgs32[32*g].  Each call is chunked exactly like
 * gbv_verify_same_message.  valid has call_off[n_calls] bytes. */
int gbv_verify_same_message_multi(gbv_ctx* ctx, size_t n_calls, const uint32_t* call_off, const uint32_t* idx,
                                  const uint8_t* sigs96, const uint8_t* msgs32, uint8_t* valid);

/* aggregatePublicKeys(index2pubkey[idx[0..k)]).toBytes() (bls/utils.ts:5-20), byte-identical.
 * k == 0 returns GBV_E_EMPTY_AGGREGATE. */
int gbv_aggregate_pubkeys(gbv_ctx* ctx, const uint32_t* idx, size_t k, uint8_t out48[48]);

/* aggregateSerializedPublicKeys(pk48[0..k)).toBytes() (state-transition/src/util/syncCommittee.ts:37,
 * epoch/processSyncCommitteeUpdates.ts:35): the 512-key sync-committee aggregate, byte-identical.
 * The keys are decompressed on the device (validate != 0 adds the subgroup/infinity check); a key
 * that fails to deserialize returns GBV_E_BAD_POINT, k == 0 GBV_E_EMPTY_AGGREGATE. */
int gbv_aggregate_serialized_pubkeys(gbv_ctx* ctx, const uint8_t* pk48, size_t k, int validate, uint8_t out48[48]);

/* Signature.fromBytes(sig, true) over n signatures of sig_len (96 or 192) bytes: status[i] = GBV_PT_*
 * (decode, on-curve, subgroup, infinity), out96 (optional) the recompressed accepted points (the
 * compressed infinity encoding for rejected inputs).  The "BLS deserializing signatures" perf id
 * (beacon-node/test/perf/bls/bls.test.ts:89-100). */
int gbv_signatures_validate(gbv_ctx* ctx, const uint8_t* sigs, size_t n, uint32_t sig_len, uint8_t* status, uint8_t* out96);

/* aggregateSignatures(sigs.map(s => Signature.fromBytes(s, validate))).toBytes() -- the aggregate of
 * BlsSingleThreadVerifier.verifySignatureSetsSameMessage (beacon-node/src/chain/bls/singleThread.ts:44-57),
 * byte-identical.  validate != 0 applies Signature.fromBytes(sig, true) (infinity and subgroup
 * rejected); validate == 0 lets an infinity signature contribute nothing.  A signature that fails
 * to deserialize returns GBV_E_BAD_POINT (the reference's fromBytes throw), n == 0
 * GBV_E_EMPTY_AGGREGATE. */
int gbv_aggregate_signatures(gbv_ctx* ctx, const uint8_t* sigs, size_t n, uint32_t sig_len, int validate, uint8_t out96[96]);

/* ---- device-resident batches (inputs staged in HBM once, verified many times) ------------- */
typedef struct gbv_sm_batch gbv_sm_batch;
/* Stage a same-message workload (as gbv_verify_same_message_multi) in HBM. */
int gbv_sm_batch_create(gbv_ctx* ctx, size_t n_calls, const uint32_t* call_off, const uint32_t* idx,
                        const uint8_t* sigs96, const uint8_t* msgs32, gbv_sm_batch** out);
/* Verify a staged batch; valid (host, optional) receives the per-set booleans. */
int gbv_sm_batch_verify(gbv_ctx* ctx, gbv_sm_batch* b, uint8_t* valid);
/* Streaming form of gbv_sm_batch_verify: submit enqueues the whole verification and returns;
 * wait blocks until it is done and copies the per-set booleans.  Submitting batch k+1 before
 * waiting on batch k overlaps k's chunk-level tail with k+1's per-set kernel (gossip stream).
 * A batch can have one verification in flight at a time. */
/* Refill an existing batch (as gbv_vs_batch_fill). */
int gbv_sm_batch_fill(gbv_ctx* ctx, gbv_sm_batch* b, size_t n_calls, const uint32_t* call_off, const uint32_t* idx,
                      const uint8_t* sigs96, const uint8_t* msgs32);
int gbv_sm_batch_submit(gbv_ctx* ctx, gbv_sm_batch* b);
int gbv_sm_batch_wait(gbv_ctx* ctx, gbv_sm_batch* b, uint8_t* valid);
void gbv_sm_batch_destroy(gbv_ctx* ctx, gbv_sm_batch* b);
/* ---- multi-GPU verifySignatureSets (one process per GPU) ----------------------------------
 * Sets shard across GPUs; each GPU reduces its shard to ONE Fp12 Miller product (its sets' pairs
 * and its own (-g1, sum r_i sig_i) pair, no final exponentiation) -- an opaque 576-byte blob in
 * the device's internal layout.  The blobs are all-gathered (RCCL over xGMI, 576 B per GPU) and
 * every rank runs gbv_fp12_check on all of them: prod == 1 after ONE final exponentiation iff every
 * set of every shard is valid (randomised batch verification, blst
 * verifyMultipleAggregateSignatures semantics, replaces BlsMultiThreadWorkerPool.verifySignatureSets
 * at multithread/index.ts:157-207 for calls too large for one device).  shard_ok = 0 when a set of
 * the shard is malformed / not in the subgroup / has an infinity aggregate pubkey (the call is then
 * false).  Empty aggregates reject like gbv_verify_sets. */
#define GBV_FP12_PARTIAL_BYTES 576
int gbv_vs_partial(gbv_ctx* ctx, const gbv_set* sets, size_t n, const uint32_t* index_arena,
                   uint8_t out576[GBV_FP12_PARTIAL_BYTES], uint8_t* shard_ok);
/* The same partial over every set of a staged batch (gbv_vs_batch_create / fill: all its calls as
 * one shard), device-resident inputs: the multi-GPU range-sync / replay form. */
int gbv_vs_batch_partial(gbv_ctx* ctx, gbv_vs_batch* b, uint8_t out576[GBV_FP12_PARTIAL_BYTES], uint8_t* shard_ok);
/* gbv_vs_batch_partial in two halves, so that a rank keeps several shard passes in flight (the
 * exchange and final exponentiation of pass k overlap the kernels of pass k + 1, lodestar_amd/sharded.py
 * verify_staged_shards): submit enqueues without a host wait (EMPTY_AGGREGATE rejects here); wait
 * blocks on the pass, without the context lock, and writes the partial and shard_ok. */
int gbv_vs_batch_partial_submit(gbv_ctx* ctx, gbv_vs_batch* b);
int gbv_vs_batch_partial_wait(gbv_ctx* ctx, gbv_vs_batch* b, uint8_t out576[GBV_FP12_PARTIAL_BYTES], uint8_t* shard_ok);
int gbv_fp12_check(gbv_ctx* ctx, const uint8_t* partials576, size_t k, uint8_t* is_one);

/* Device time (ms, summed over launches) and launch count of each kernel of the last
 * gbv_sm_batch_verify, measured with HIP events on the stream each kernel runs on:
 * [hash, prepare, chunk_finish, miller, seg_check, group_pairing, fallback, msm] (msm: the bucket
 * pass of segments whose G2 sum comes from the bucket MSM); returns the number of entries written
 * (at most 8). */
int gbv_last_kernel_ms(gbv_ctx* ctx, float* ms_out, int* launches_out, int max);
/* Per-kernel device time of the last waited pass, one line per launch: "<kernel> <grid work-items>
 * <units> <ms>\n" (units: the sets / messages / chunks the launch covers; ms from two HIP events on
 * the kernel's own stream).  path 0: same-message batches, 1: verifySignatureSets passes and shard
 * partials.  Recorded only while gbv_tune(ctx, "kprof", 1) is set (off by default: it adds two
 * events per kernel).  Writes at most cap - 1 bytes and a NUL; returns the full length (bench.py
 * rooflines; no reference counterpart). */
int gbv_last_ops(gbv_ctx* ctx, int path, char* out, size_t cap);
/* Fast-path health of the last waited same-message verification: chunks that went to the per-set
 * retry (malformed sets or failing chunk checks) and segments whose combined check failed.  Both
 * are 0 for an all-valid batch (up to the 2^-64 batch-verification error). */
int gbv_last_stats(gbv_ctx* ctx, uint32_t* fallback_chunks, uint32_t* failed_segments);

/* ---- signing roots: batched SHA-256 over SSZ nodes ------------------
 * The builders hash a signing root for every set they hand the verifier (the signatureSets builders via
 * computeSigningRoot, state-transition/src/util/signingRoot.ts:7-13).  Inputs and outputs are host
 * buffers; n = 0 is a no-op.  Each call records its kernel time (HIP events, gbv_ssz_last_kernel_ms). */
/* out32[i] = sha256(in64[i]): persistent-merkle-tree hasher.digest64(a, b) = sha256(a || b)
 * (@chainsafe/as-sha256 0.5.0; light-client/src/utils/verifyMerkleBranch.ts:23). */
int gbv_sha256_digest64(gbv_ctx* ctx, const uint8_t* in64, size_t n, uint8_t* out32);
/* Merkle roots of n objects of 2^depth 32-byte chunks each (object-major, zero padding already in
 * place): ContainerType.hashTreeRoot over the field roots of a container (@chainsafe/ssz 0.11.1).
 * depth <= 24; depth 0 copies the single chunk. */
int gbv_merkle_roots(gbv_ctx* ctx, const uint8_t* chunks32, size_t n, uint32_t depth, uint8_t* out32);
/* computeSigningRoot from object roots: out32[i] = sha256(object_roots32[i] || domains32[d]) with
 * d = dom_idx ? dom_idx[i] : 0 (signingRoot.ts:7-13).  dom_idx[i] >= n_domains is GBV_E_ARG. */
int gbv_signing_roots(gbv_ctx* ctx, const uint8_t* object_roots32, size_t n, const uint8_t* domains32, size_t n_domains,
                      const uint32_t* dom_idx, uint8_t* out32);
/* getAttestationDataSigningRoot (beacon-node/src/chain/validation/attestation.ts:657-665):
 * computeSigningRoot(ssz.phase0.AttestationData, data, domain) from the 128-byte SSZ serialisation of
 * each AttestationData (types/src/phase0/sszTypes.ts:247-256); domains as in gbv_signing_roots. */
int gbv_attestation_signing_roots(gbv_ctx* ctx, const uint8_t* data128, size_t n, const uint8_t* domains32, size_t n_domains,
                                  const uint32_t* dom_idx, uint8_t* out32);
/* Device time (ms) of the kernels of the last signing-root call above. */
int gbv_ssz_last_kernel_ms(gbv_ctx* ctx, float* ms_out);

/* ---- utilities for tests and synthetic workloads (not on the verification path) ----------- */
/* sk32 (big-endian scalars) -> compressed pubkeys, on the device. */
int gbv_util_sk_to_pk(gbv_ctx* ctx, const uint8_t* sk32, size_t n, uint8_t* pk48);
/* sig[i] = sk[i] * H(msgs32[grp[i]]) compressed, on the device. */
int gbv_util_sign(gbv_ctx* ctx, const uint8_t* sk32, size_t n, const uint32_t* grp, const uint8_t* msgs32,
                  size_t n_msgs, uint8_t* sig96);
/* hash_to_G2 of n 32-byte messages, uncompressed 192-byte affine output. */
int gbv_util_hash_to_g2(gbv_ctx* ctx, const uint8_t* msgs32, size_t n, uint8_t* out192);
/* [r] index2pubkey[slot] (compressed) for the batch scalar r = a - b*x^2 of each 64-bit digit word,
 * through the slot's comb table (use_comb = 1) or the endomorphism ladder (0): test hook for the
 * tables k_sm_prepare reads. */
int gbv_util_g1_mul_rand(gbv_ctx* ctx, const uint32_t* slots, const uint64_t* r64, size_t n, int use_comb, uint8_t* out48);
/* Duplicate table slots: slot[dst_first + i] = slot[src_first + (i % src_n)], i < n (synthetic tables). */
int gbv_pubkeys_replicate(gbv_ctx* ctx, uint32_t src_first, uint32_t src_n, uint32_t dst_first, size_t n);

#ifdef __cplusplus
}
#endif
#endif /* GBV_H */
