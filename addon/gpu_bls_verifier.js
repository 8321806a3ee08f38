// GpuBlsVerifier -- Lodestar's IBlsVerifier (beacon-node/src/chain/bls/interface.ts:25-68) over the
// Node-API addon (addon/gbv_addon.c -> include/gbv.h), in plain JavaScript for the Node in this image
// (v12; the TypeScript class in INTEGRATION.md is this file with types).  It replaces
// BlsMultiThreadWorkerPool (multithread/index.ts:113) and keeps its scheduling contract:
//   * verifySignatureSets: chunkifyMaximizeChunkSize(sets, 128) jobs, AND of their results; [] -> false;
//     an aggregate set without pubkeys rejects its own call (EMPTY_AGGREGATE_ARRAY, index.ts:398-412)
//   * verifySignatureSetsSameMessage: per-set booleans, per-set retry of failing chunks on the device
//     (jobItem.ts:93-125)
//   * opts.batchable: buffered up to MAX_BUFFER_WAIT_MS or until more than MAX_BUFFERED_SIGS sigs
//     (index.ts:320-339); opts.priority: front of the queue (index.ts:343-349); opts.verifyOnMainThread:
//     synchronous on the JS thread (index.ts:168-181)
//   * canAcceptWork(): passes in flight < MAX_PASSES and jobs < 512 (index.ts:149-155)
//   * close(): queued and buffered jobs reject with QUEUE_ABORTED, passes already on the device finish
//   * per-request failure isolation: a bad set fails only its own call (multithread.test.ts:109-129)
// The worker pool becomes the device: every job queued when a pass starts goes into it (same-message
// jobs as one device batch, default jobs as another), and up to MAX_PASSES passes are on the device at
// once (submitPass / waitPass), so consecutive gossip dispatches overlap.
// Metrics: the reference's lodestar_bls_thread_pool_* families (metrics/lodestar.ts:401-504) plus
// *_gpu_* ones, rendered in the Prometheus text format by metricsText(), and -- when the node passes
// its own families (o.metrics = metrics.blsThreadPool plus the two gpu families registered on
// metrics.register, chain/bls/gpu/index.ts) -- fed into the node's registry as well, where /metrics
// and the dashboards read them.
"use strict";

const MAX_SIGNATURE_SETS_PER_JOB = 128; // multithread/index.ts:56
const MAX_BUFFERED_SIGS = 32; // multithread/index.ts:65
const MAX_BUFFER_WAIT_MS = 100; // multithread/index.ts:74
const MAX_JOBS_CAN_ACCEPT_WORK = 512; // multithread/index.ts:79
// A device pass takes queued jobs up to this many sets (the Python verifier's MAX_PASS_SETS): a burst
// of gossip calls then becomes several passes, so the addon's marshalling of pass k + 1 and the
// resolution of pass k - 1 run while pass k is on the device.
const MAX_PASS_SETS = 1 << 18;
// index2pubkey position of a registered key object, kept on the object itself (a symbol-keyed property,
// invisible to other code): one monomorphic property load per set instead of a WeakMap lookup
const KEY_INDEX = Symbol("gbv.validatorIndex");

/** chunkifyMaximizeChunkSize (multithread/utils.ts:4-18) */
function chunkifyMaximizeChunkSize(arr, minPerChunk) {
  const chunkCount = Math.floor(arr.length / minPerChunk);
  if (chunkCount <= 1) return [arr];
  const perChunk = Math.ceil(arr.length / chunkCount);
  const out = [];
  for (let i = 0; i < arr.length; i += perChunk) out.push(arr.slice(i, i + perChunk));
  return out;
}

/** chunkifyMaximizeChunkSize over [0, n) as [begin, end) ranges */
function chunkRanges(n, minPerChunk) {
  const chunkCount = Math.floor(n / minPerChunk);
  if (chunkCount <= 1) return [[0, n]];
  const perChunk = Math.ceil(n / chunkCount);
  const out = [];
  for (let i = 0; i < n; i += perChunk) out.push([i, Math.min(i + perChunk, n)]);
  return out;
}

class QueueError extends Error {
  constructor(code) {
    super(code);
    this.code = code;
    this.type = {code};
  }
}

// ---- metrics -----------------------------------------------------------------------------------
class Family {
  constructor(kind, name, help, labelNames, buckets) {
    this.kind = kind;
    this.name = name;
    this.help = help;
    this.labelNames = labelNames || [];
    this.buckets = buckets ? buckets.slice().sort((a, b) => a - b) : null;
    this.series = new Map();
  }
  _get(labels) {
    const key = this.labelNames.map((l) => String((labels || {})[l])).join("\u0000");
    let s = this.series.get(key);
    if (!s) {
      s = {labels: labels || {}, value: 0, sum: 0, count: 0, counts: this.buckets ? this.buckets.map(() => 0) : null};
      this.series.set(key, s);
    }
    return s;
  }
  inc(labels, v) {
    if (typeof labels === "number" || labels === undefined) [labels, v] = [{}, labels];
    this._get(labels).value += v === undefined ? 1 : v;
  }
  set(v, labels) {
    this._get(labels).value = v;
  }
  observe(v, labels) {
    const s = this._get(labels);
    s.sum += v;
    s.count += 1;
    this.buckets.forEach((b, i) => {
      if (v <= b) s.counts[i] += 1;
    });
  }
  value(labels) {
    const s = this.series.get(this.labelNames.map((l) => String((labels || {})[l])).join("\u0000"));
    return s ? (this.kind === "histogram" ? s.count : s.value) : 0;
  }
  text() {
    const lbl = (o, extra) => {
      const kv = Object.entries(Object.assign({}, o, extra || {})).map(([k, v]) => `${k}="${v}"`);
      return kv.length ? `{${kv.join(",")}}` : "";
    };
    const out = [`# HELP ${this.name} ${this.help}`, `# TYPE ${this.name} ${this.kind}`];
    for (const s of this.series.values()) {
      if (this.kind === "histogram") {
        this.buckets.forEach((b, i) => out.push(`${this.name}_bucket${lbl(s.labels, {le: b})} ${s.counts[i]}`));
        out.push(`${this.name}_bucket${lbl(s.labels, {le: "+Inf"})} ${s.count}`);
        out.push(`${this.name}_sum${lbl(s.labels)} ${s.sum}`, `${this.name}_count${lbl(s.labels)} ${s.count}`);
      } else {
        out.push(`${this.name}${lbl(s.labels)} ${s.value}`);
      }
    }
    return out.join("\n");
  }
}

// One family fed to the local registry and to the node's (prom-client style: inc(labels?, v?),
// set(labels?, v) / set(v), observe(labels?, v) / observe(v)).
class TeeFamily {
  constructor(local, ext) {
    this.local = local;
    this.ext = ext;
    this.name = local.name;
  }
  inc(labels, v) {
    this.local.inc(labels, v);
    if (typeof labels === "number" || labels === undefined) this.ext.inc(labels === undefined ? 1 : labels);
    else this.ext.inc(labels, v === undefined ? 1 : v);
  }
  set(v, labels) {
    this.local.set(v, labels);
    if (labels) this.ext.set(labels, v);
    else this.ext.set(v);
  }
  observe(v, labels) {
    this.local.observe(v, labels);
    if (labels) this.ext.observe(labels, v);
    else this.ext.observe(v);
  }
  value(labels) {
    return this.local.value(labels);
  }
  text() {
    return this.local.text();
  }
}

class BlsPoolMetrics {
  /** @param {object} [external] the node's families by the reference's property names
   * (metrics.blsThreadPool: totalSigSets, jobWaitTime, ...; plus gpuDevicePasses, gpuPassTime) */
  constructor(external) {
    const p = "lodestar_bls_thread_pool_";
    const g = (n, h, l) => new Family("gauge", n, h, l);
    const hi = (n, h, b) => new Family("histogram", n, h, null, b);
    this.families = {
      jobsWorkerTime: g(p + "time_seconds_sum", "Total time spent verifying signature sets measured on the worker", ["workerId"]),
      successJobsSignatureSetsCount: g(p + "success_jobs_signature_sets_count", "Count of total verified signature sets"),
      errorAggregateSignatureSetsCount: g(p + "error_aggregate_signature_sets_count", "Count of error when aggregating pubkeys or signatures", ["type"]),
      errorJobsSignatureSetsCount: g(p + "error_jobs_signature_sets_count", "Count of total error-ed signature sets"),
      jobWaitTime: hi(p + "queue_job_wait_time_seconds", "Time from job added to the queue to starting the job in seconds", [0.01, 0.02, 0.5, 0.1, 0.3, 1]),
      queueLength: g(p + "queue_length", "Count of total block processor queue length"),
      workersBusy: g(p + "workers_busy", "Count of current busy workers"),
      totalJobsGroupsStarted: g(p + "job_groups_started_total", "Count of total jobs groups started in bls thread pool, job groups include +1 jobs"),
      totalJobsStarted: g(p + "jobs_started_total", "Count of total jobs started in bls thread pool, jobs include +1 signature sets", ["type"]),
      totalSigSetsStarted: g(p + "sig_sets_started_total", "Count of total signature sets started in bls thread pool, sig sets include 1 pk, msg, sig", ["type"]),
      batchRetries: g(p + "batch_retries_total", "Count of total batches that failed and had to be verified again."),
      batchSigsSuccess: g(p + "batch_sigs_success_total", "Count of total batches that failed and had to be verified again."),
      sameMessageRetryJobs: g(p + "same_message_jobs_retries_total", "Count of total same message jobs that failed and had to be verified again."),
      sameMessageRetrySets: g(p + "same_message_sets_retries_total", "Count of total same message sets that failed and had to be verified again."),
      mainThreadDurationInThreadPool: hi(p + "main_thread_time_seconds", "Time to verify signatures in main thread with thread pool mode", [0]),
      timePerSigSet: hi("lodestar_bls_worker_thread_time_per_sigset_seconds", "Time to verify each sigset with worker thread mode", [0.5e-3, 0.75e-3, 1e-3, 1.5e-3, 2e-3, 5e-3]),
      totalSigSets: g(p + "sig_sets_total", "Count of total signature sets"),
      prioritizedSigSets: g(p + "prioritized_sig_sets_total", "Count of total prioritized signature sets"),
      batchableSigSets: g(p + "batchable_sig_sets_total", "Count of total batchable signature sets"),
      gpuDevicePasses: new Family("counter", p + "gpu_device_passes_total", "Device passes (one or more jobs verified together)"),
      gpuPassTime: hi(p + "gpu_pass_time_seconds", "Device pass wall time, submit to results", [0.005, 0.01, 0.02, 0.05, 0.1, 0.3, 1]),
    };
    if (external) {
      for (const [k, f] of Object.entries(this.families)) if (external[k]) this.families[k] = new TeeFamily(f, external[k]);
    }
    Object.assign(this, this.families);
  }
  text() {
    return Object.values(this.families).map((f) => f.text()).join("\n") + "\n";
  }
}

/** The families a Lodestar node hands GpuBlsVerifier (chain/bls/gpu/index.ts): its blsThreadPool
 * families (metrics/lodestar.ts:401-504) and the two *_gpu_* ones registered on metrics.register, the
 * node's RegistryMetricCreator.  Null without metrics (the node runs without --metrics). */
function nodeMetricFamilies(metrics) {
  if (!metrics) return null;
  const p = "lodestar_bls_thread_pool_";
  return Object.assign({}, metrics.blsThreadPool, {
    gpuDevicePasses: metrics.register.gauge({name: p + "gpu_device_passes_total", help: "Device passes (one or more jobs verified together)"}),
    gpuPassTime: metrics.register.histogram({name: p + "gpu_pass_time_seconds", help: "Device pass wall time, submit to results",
      buckets: [0.005, 0.01, 0.02, 0.05, 0.1, 0.3, 1]}),
  });
}

// ---- the verifier --------------------------------------------------------------------------------
class GpuBlsVerifier {
  /**
   * @param {object} o  {addon: the gbv addon (or a stand-in with the same functions), device?: number,
   *                    ctx?: an already open context, metrics?: the node's metric families (BlsPoolMetrics)}
   */
  constructor(o) {
    this.addon = o.addon;
    this.device = o.device || 0;
    this.ctx = o.ctx || this.addon.open(this.device);
    this.maxPasses = this.addon.MAX_PASSES || 3;
    this.jobs = [];
    this.bufferedJobs = null;
    this.passesBusy = 0;
    this.closed = false;
    this.idleWaiters = [];
    this.runScheduled = false;
    this.metrics = new BlsPoolMetrics(o.metrics || null);
    if (o.metrics && o.metrics.queueLength && o.metrics.queueLength.addCollect) {
      // read at scrape time, as the pool does (multithread/index.ts:141-146)
      o.metrics.queueLength.addCollect(() => {
        this.metrics.queueLength.set(this.jobs.length);
        this.metrics.workersBusy.set(this.passesBusy);
      });
    }
    this.devicePasses = 0;
    // index2pubkey by object identity: the PublicKey objects of the node's table (registered by
    // loadIndex2pubkey and the index2pubkey listener) -> their validator index.  The reference's
    // same-message call hands {publicKey, signature} (interface.ts:55-59, attestation.ts:134-137); the
    // key object it passes is index2pubkey[validatorIndex], so its index selects the HBM copy.
    this.keyIndex = new WeakMap();
  }

  addPubkeys(firstIndex, pk48s, validate) {
    return this.addon.addPubkeys(this.ctx, firstIndex, pk48s, !!validate);
  }

  /** Record keys[k] (the node's PublicKey object for validator firstIndex + k) in the identity map.
   * The device copy of those keys is added separately (addPubkeys). */
  registerPubkeyObjects(firstIndex, keys) {
    for (let k = 0; k < keys.length; ++k) {
      const o = keys[k];
      if (o === null || typeof o !== "object") continue;
      if (Object.isExtensible(o)) o[KEY_INDEX] = firstIndex + k;
      else this.keyIndex.set(o, firstIndex + k); // a frozen / sealed key object: by identity in the map
    }
  }

  /** validator index of a key object of index2pubkey, or undefined for a key outside the table */
  indexOf(publicKey) {
    if (publicKey === null || typeof publicKey !== "object") return undefined;
    const k = publicKey[KEY_INDEX];
    return k !== undefined ? k : this.keyIndex.get(publicKey);
  }

  /** a same-message set's validator index: its `index`, else its key object's */
  _setIndex(s) {
    if (s.index !== undefined) return s.index;
    const pk = s.publicKey;
    if (pk === null || typeof pk !== "object") return undefined;
    const k = pk[KEY_INDEX];
    return k !== undefined ? k : this.keyIndex.get(pk);
  }

  /** the indices of a list of key objects, or undefined when any is outside the table */
  indicesOf(publicKeys) {
    const out = new Array(publicKeys.length);
    for (let k = 0; k < publicKeys.length; ++k) {
      const i = this.indexOf(publicKeys[k]);
      if (i === undefined) return undefined;
      out[k] = i;
    }
    return out;
  }

  /** Device hashing for the signature-set builders (addon/gossip_sets.js): Merkle roots of objects of
   * 2^depth chunks (gbv_merkle_roots) and computeSigningRoot over object roots (gbv_signing_roots). */
  merkleRoots(chunks, depth) {
    return this.addon.merkleRoots(this.ctx, chunks, depth);
  }

  signingRoots(objectRoots, domains, domIdx) {
    return this.addon.signingRoots(this.ctx, objectRoots, domains, domIdx || null);
  }

  canAcceptWork() {
    return this.passesBusy < this.maxPasses && this.jobs.length < MAX_JOBS_CAN_ACCEPT_WORK;
  }

  /** Checks of one call before it is queued, so a bad call rejects alone (getAggregatedPubkey throws
   * while the reference builds that job, jobItem.ts:55-62). */
  _validate(sets) {
    let nKeys = -1;
    for (const s of sets) {
      if (!s.signingRoot || s.signingRoot.length !== 32) throw Object.assign(new TypeError("signingRoot must be 32 bytes"), {code: "GBV_E_ARG"});
      if (s.pubkey) {
        if (s.pubkey.length !== 48) throw Object.assign(new TypeError("pubkey must be 48 bytes"), {code: "GBV_E_ARG"});
        continue;
      }
      const idx = s.indices !== undefined ? s.indices : [s.index];
      for (const i of idx) {
        if (nKeys < 0) nKeys = this.addon.pubkeyCount(this.ctx);
        if (!(i >= 0 && i < nKeys)) throw Object.assign(new RangeError("validator index out of range"), {code: "GBV_E_ARG"});
      }
    }
  }

  async verifySignatureSets(sets, opts = {}) {
    const m = this.metrics;
    m.totalSigSets.inc(sets.length);
    if (opts.priority) m.prioritizedSigSets.inc(sets.length);
    if (opts.batchable) m.batchableSigSets.inc(sets.length);
    if (this.closed) throw new QueueError("QUEUE_ABORTED");
    this._validate(sets);
    if (opts.verifyOnMainThread) {
      const t = process.hrtime();
      try {
        return this.addon.verifySetsSync(this.ctx, sets);
      } finally {
        const d = process.hrtime(t);
        m.mainThreadDurationInThreadPool.observe(d[0] + d[1] / 1e9);
      }
    }
    const results = await Promise.all(
      chunkifyMaximizeChunkSize(sets, MAX_SIGNATURE_SETS_PER_JOB).map(
        (chunk) => new Promise((resolve, reject) => this._queue({type: "default", resolve, reject, addedTimeMs: Date.now(), opts, sets: chunk}))
      )
    );
    return results.every((r) => r === true);
  }

  /** sets: the reference's {publicKey, signature}[] (interface.ts:55-59) -> boolean[].  A set's key is
   * found by `index` when the caller gives one, else by the identity of its publicKey object in
   * index2pubkey (registerPubkeyObjects); a key outside the table is verified from its bytes
   * (publicKey.toBytes()) as a one-set verifySignatureSets job, whose boolean is that set's answer
   * (the reference's per-set retry verifies each set alone, jobItem.ts:93-125).  Or the packed form
   * {indices: Uint32Array(n), signatures: Uint8Array(96 n)} -> Uint8Array(n) of 0 / 1 (the same answer
   * without a JS object per set: two memcpys in the addon instead of 2n property reads) */
  async verifySignatureSetsSameMessage(sets, message, opts = {}) {
    if (this.closed) throw new QueueError("QUEUE_ABORTED");
    if (!message || message.length !== 32) throw Object.assign(new TypeError("message must be 32 bytes"), {code: "GBV_E_ARG"});
    const packed = !Array.isArray(sets);
    const sigList = packed && Array.isArray(sets.signatures);
    if (packed && !(sets.indices instanceof Uint32Array && sets.signatures &&
        sets.signatures.length === (sigList ? 1 : 96) * sets.indices.length))
      throw Object.assign(new TypeError("packed sets: {indices: Uint32Array(n), signatures: Uint8Array(96 n) | Uint8Array[n]}"), {code: "GBV_E_ARG"});
    const n = packed ? sets.indices.length : sets.length;
    const nKeys = n ? this.addon.pubkeyCount(this.ctx) : 0;
    const badIndex = () => Object.assign(new RangeError("validator index out of range"), {code: "GBV_E_ARG"});
    let outside = null; // object form: the positions of sets whose key is not in index2pubkey
    let resolved = null; // object form: the sets' indices, resolved once here (a key object is read once)
    if (packed) {
      const pi = sets.indices;
      for (let i = 0; i < n; ++i) if (pi[i] >= nKeys) throw badIndex();
    } else {
      resolved = new Uint32Array(n);
      for (let i = 0; i < n; ++i) {
        const k = this._setIndex(sets[i]);
        if (k === undefined) (outside || (outside = [])).push(i);
        else if (!(k >= 0 && k < nKeys)) throw badIndex();
        else resolved[i] = k;
      }
      if (outside) return this._sameMessageOutsideKeys(sets, outside, message, opts);
    }
    if (n < 2 * MAX_SIGNATURE_SETS_PER_JOB) {
      // one chunk (every gossip call): its job's promise is the call's (no Promise.all, no concat)
      const chunk = packed ? {indices: sets.indices, signatures: sets.signatures, length: n} : sets;
      return new Promise((resolve, reject) =>
        this._queue({type: "sameMessage", resolve, reject, addedTimeMs: Date.now(), opts, sets: chunk, message, indices: resolved}));
    }
    const chunks = packed
      ? chunkRanges(n, MAX_SIGNATURE_SETS_PER_JOB).map(([a, b]) => ({indices: sets.indices.subarray(a, b),
        signatures: sigList ? sets.signatures.slice(a, b) : sets.signatures.subarray(96 * a, 96 * b), length: b - a}))
      : chunkifyMaximizeChunkSize(sets, MAX_SIGNATURE_SETS_PER_JOB);
    const results = await Promise.all(
      chunks.map(
        (chunk) =>
          new Promise((resolve, reject) => this._queue({type: "sameMessage", resolve, reject, addedTimeMs: Date.now(), opts, sets: chunk, message}))
      )
    );
    if (!packed) return [].concat(...results);
    if (results.length === 1) return results[0];
    const out = new Uint8Array(n);
    let o = 0;
    for (const r of results) {
      out.set(r, o);
      o += r.length;
    }
    return out;
  }

  /** A same-message call holding keys outside index2pubkey: the sets with table keys go to the device as
   * one same-message job, every other set as a one-set verifySignatureSets job over its key bytes; the
   * booleans come back in call order. */
  async _sameMessageOutsideKeys(sets, outside, message, opts) {
    const n = sets.length;
    const isOut = new Uint8Array(n);
    for (const i of outside) isOut[i] = 1;
    const inside = [];
    for (let i = 0; i < n; ++i) if (!isOut[i]) inside.push(i);
    const loose = outside.map((i) => {
      const pk = sets[i].publicKey;
      const bytes = pk instanceof Uint8Array ? pk : pk && typeof pk.toBytes === "function" ? pk.toBytes() : null;
      if (!bytes || bytes.length !== 48)
        throw Object.assign(new TypeError("set without index: publicKey must be an index2pubkey key, a PublicKey or 48 bytes"), {code: "GBV_E_ARG"});
      return {pubkey: bytes, signingRoot: message, signature: sets[i].signature};
    });
    const pIn = inside.length
      ? this.verifySignatureSetsSameMessage(inside.map((i) => ({index: this._setIndex(sets[i]), signature: sets[i].signature})), message, opts)
      : Promise.resolve([]);
    const pOut = loose.map((s) => new Promise((resolve, reject) => this._queue({type: "default", resolve, reject, addedTimeMs: Date.now(), opts, sets: [s]})));
    const [rIn, rOut] = await Promise.all([pIn, Promise.all(pOut)]);
    const out = new Array(n);
    inside.forEach((i, k) => (out[i] = rIn[k]));
    outside.forEach((i, k) => (out[i] = rOut[k] === true));
    return out;
  }

  /** The IBlsVerifier call shape (chain/bls/gpu/index.ts, validation/attestation.ts:134-137): one
   * {publicKey, signature} per set -> boolean[], keys resolved by identity.  The objects ride in the job
   * as they are with their resolved indices beside them; _runPass copies every job of a pass into four
   * pass-wide buffers (_packSameMessage) -- a per-call typed array of signatures, or Node-API property
   * reads per set, cost more. */
  verifySameMessageSets(sets, message, opts = {}) {
    return this.verifySignatureSetsSameMessage(sets, message, opts);
  }

  async close() {
    if (this.closed) return;
    this.closed = true;
    if (this.bufferedJobs) {
      clearTimeout(this.bufferedJobs.timeout);
      for (const j of this.bufferedJobs.jobs.concat(this.bufferedJobs.prioritizedJobs)) j.reject(new QueueError("QUEUE_ABORTED"));
      this.bufferedJobs = null;
    }
    for (const j of this.jobs) j.reject(new QueueError("QUEUE_ABORTED"));
    this.jobs = [];
    while (this.passesBusy > 0) await new Promise((r) => this.idleWaiters.push(r));
    await this.addon.close(this.ctx);
  }

  metricsText() {
    this.metrics.queueLength.set(this.jobs.length);
    this.metrics.workersBusy.set(this.passesBusy);
    return this.metrics.text();
  }

  // ---- queue (index.ts:302-352, 357-534, 539-550) --------------------------------------------
  _queue(job) {
    if (this.closed) throw new QueueError("QUEUE_ABORTED");
    const sigs = job.type === "sameMessage" ? 1 : job.sets.length; // jobItemSigSets (jobItem.ts:38-45)
    if (job.opts.batchable) {
      if (!this.bufferedJobs) {
        this.bufferedJobs = {jobs: [], prioritizedJobs: [], sigCount: 0, firstPush: Date.now(), timeout: setTimeout(() => this._runBufferedJobs(), MAX_BUFFER_WAIT_MS)};
      }
      (job.opts.priority ? this.bufferedJobs.prioritizedJobs : this.bufferedJobs.jobs).push(job);
      this.bufferedJobs.sigCount += sigs;
      if (this.bufferedJobs.sigCount > MAX_BUFFERED_SIGS) {
        clearTimeout(this.bufferedJobs.timeout);
        this._runBufferedJobs();
      }
    } else {
      if (job.opts.priority) this.jobs.unshift(job);
      else this.jobs.push(job);
      this._schedule();
    }
  }

  _runBufferedJobs() {
    const b = this.bufferedJobs;
    if (!b) return;
    this.bufferedJobs = null;
    for (const j of b.jobs) this.jobs.push(j);
    for (const j of b.prioritizedJobs) this.jobs.unshift(j);
    this._schedule();
  }

  _schedule() {
    if (this.runScheduled) return;
    this.runScheduled = true;
    setImmediate(() => {
      this.runScheduled = false;
      this._runJobs();
    });
  }

  _runJobs() {
    while (!this.closed && this.jobs.length > 0 && this.passesBusy < this.maxPasses) {
      let k = 0;
      for (let sets = 0; k < this.jobs.length && (k === 0 || sets < MAX_PASS_SETS); ++k) sets += this.jobs[k].sets.length;
      const jobs = k === this.jobs.length ? this.jobs : this.jobs.slice(0, k);
      this.jobs = k === this.jobs.length ? [] : this.jobs.slice(k);
      this._runPass(jobs);
    }
  }

  /** The pass's same-message jobs as the addon's flat form: counts / messages per call, indices and
   * 96-byte signatures per set, in job order (job.off: the job's first set).  A signature of another
   * length stays zero bytes: a bad encoding, false for that set alone -- as Signature.fromBytes throwing
   * inside the pool's aggregate sends the chunk to the per-set retry, where that set fails
   * (jobItem.ts:93-125). */
  _packSameMessage(sm) {
    let total = 0;
    for (const j of sm) total += j.sets.length;
    const counts = new Uint32Array(sm.length);
    const messages = new Uint8Array(32 * sm.length);
    const indices = new Uint32Array(total);
    const signatures = new Uint8Array(96 * total);
    let o = 0;
    for (let c = 0; c < sm.length; ++c) {
      const j = sm[c], s = j.sets, n = s.length;
      counts[c] = n;
      messages.set(j.message, 32 * c);
      j.off = o;
      if (Array.isArray(s)) {
        if (j.indices) indices.set(j.indices, o); // resolved and checked when the call was validated
        for (let i = 0; i < n; ++i) {
          const e = s[i], g = e.signature;
          if (!j.indices) indices[o + i] = this._setIndex(e); // a chunk of a long call: in the table, checked
          if (g.length === 96) signatures.set(g, 96 * (o + i));
        }
      } else {
        indices.set(s.indices, o);
        if (Array.isArray(s.signatures)) {
          for (let i = 0; i < n; ++i) if (s.signatures[i].length === 96) signatures.set(s.signatures[i], 96 * (o + i));
        } else {
          signatures.set(s.signatures, 96 * o);
        }
      }
      o += n;
    }
    return {counts, messages, indices, signatures};
  }

  _runPass(jobs) {
    const m = this.metrics;
    const now = Date.now();
    const sm = jobs.filter((j) => j.type === "sameMessage");
    const df = jobs.filter((j) => j.type === "default");
    m.totalJobsGroupsStarted.inc();
    m.totalJobsStarted.inc({type: "default"}, df.length);
    m.totalJobsStarted.inc({type: "sameMessage"}, sm.length);
    m.totalSigSetsStarted.inc({type: "default"}, df.reduce((a, j) => a + j.sets.length, 0));
    m.totalSigSetsStarted.inc({type: "sameMessage"}, sm.reduce((a, j) => a + j.sets.length, 0));
    for (const j of jobs) m.jobWaitTime.observe((now - j.addedTimeMs) / 1000);
    let pass;
    const t0 = process.hrtime();
    try {
      pass = this.addon.submitPass(this.ctx, sm.length ? this._packSameMessage(sm) : null, df.length ? df.map((j) => j.sets) : null);
    } catch (e) {
      for (const j of jobs) j.reject(e);
      return;
    }
    this.passesBusy++;
    this.addon
      .waitPass(pass)
      .then(
        (res) => {
          this._resolveSameMessage(sm, res.sameMessage);
          this._resolveDefault(df, res.default);
        },
        (e) => {
          for (const j of jobs) j.reject(e); // device failure rejects the pass (index.ts:498-507)
        }
      )
      .then(() => {
        const d = process.hrtime(t0);
        const sec = d[0] + d[1] / 1e9;
        const nSets = jobs.reduce((a, j) => a + j.sets.length, 0);
        m.gpuDevicePasses.inc();
        m.gpuPassTime.observe(sec);
        m.jobsWorkerTime.inc({workerId: this.device}, sec);
        if (nSets) m.timePerSigSet.observe(sec / nSets);
        this.devicePasses++;
        this.passesBusy--;
        if (this.passesBusy === 0) this.idleWaiters.splice(0).forEach((r) => r());
        if (this.jobs.length) this._schedule();
      });
  }

  _resolveSameMessage(sm, res) {
    const m = this.metrics;
    if (!sm.length) return;
    if (res instanceof Error) {
      m.errorJobsSignatureSetsCount.inc(sm.length);
      for (const j of sm) j.reject(res);
      return;
    }
    // res: one 0 / 1 byte per set of the pass (the flat form); a job's sets start at job.off
    sm.forEach((j) => {
      const n = j.sets.length;
      let r, all = true;
      if (Array.isArray(j.sets)) {
        r = new Array(n);
        for (let i = 0; i < n; ++i) all = (r[i] = res[j.off + i] === 1) && all;
      } else {
        r = res.subarray(j.off, j.off + n);
        all = r.indexOf(0) < 0;
      }
      m.successJobsSignatureSetsCount.inc(1);
      if (all) {
        m.batchSigsSuccess.inc(n);
      } else {
        // the chunk's aggregate check failed: its sets were verified one by one on the device
        m.sameMessageRetryJobs.inc(1);
        m.sameMessageRetrySets.inc(n);
      }
      j.resolve(r);
    });
  }

  _resolveDefault(df, res) {
    const m = this.metrics;
    if (!df.length) return;
    df.forEach((j, k) => {
      const r = res instanceof Error ? res : res[k];
      if (r instanceof Error) {
        if (r.code === "EMPTY_AGGREGATE_ARRAY") m.errorAggregateSignatureSetsCount.inc({type: "default"}, 1);
        m.errorJobsSignatureSetsCount.inc(j.sets.length);
        j.reject(r);
      } else {
        m.successJobsSignatureSetsCount.inc(j.sets.length);
        if (r) m.batchSigsSuccess.inc(j.sets.length);
        j.resolve(r);
      }
    });
  }
}

module.exports = {
  GpuBlsVerifier,
  BlsPoolMetrics,
  nodeMetricFamilies,
  QueueError,
  chunkifyMaximizeChunkSize,
  MAX_SIGNATURE_SETS_PER_JOB,
  MAX_BUFFERED_SIGS,
  MAX_BUFFER_WAIT_MS,
  MAX_JOBS_CAN_ACCEPT_WORK,
  MAX_PASS_SETS,
};
