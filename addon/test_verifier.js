// Tests of the JavaScript GpuBlsVerifier (addon/gpu_bls_verifier.js).  Used by tests/test_addon.py.
//   node addon/test_verifier.js cpu               queueing, buffering, priority, canAcceptWork, close,
//                                                 failure isolation and metrics, with a stand-in device
//   node addon/test_verifier.js gpu <fixtures>    the golden cases and overlapping passes on device 0
// The cases mirror the reference's own: test/unit/chain/bls/bls.test.ts:34-83 (verify all / one
// invalid / one malformed, for both methods) and test/e2e/chain/bls/multithread.test.ts:85-129 (many
// calls submitted synchronously and asynchronously, batched, with and without priority; a batched
// invalid request does not fail the others).
"use strict";
const path = require("path");
const fs = require("fs");
const V = require(path.join(__dirname, "gpu_bls_verifier.js"));

const report = {};
const sleep = (ms) => new Promise((r) => setTimeout(r, ms));
const hex = (h) => Uint8Array.from(Buffer.from(h, "hex"));

// ---- a stand-in device with the addon's functions: a set is valid iff its signature starts with 1
class FakeAddon {
  constructor() {
    this.MAX_PASSES = 3;
    this.passes = [];
    this.gate = null; // when set, waitPass waits for it
    this.closed = false;
    this.destroyedAfter = null;
  }
  open() {
    return {};
  }
  pubkeyCount() {
    return 1 << 20;
  }
  valid(s) {
    return s.signature.length > 0 && s.signature[0] === 1;
  }
  verifySetsSync(ctx, sets) {
    this.passes.push(["sync", sets.length]);
    return sets.length > 0 && sets.every((s) => this.valid(s));
  }
  submitPass(ctx, sm, df) {
    if (this.closed) throw Object.assign(new Error("QUEUE_ABORTED"), {code: "QUEUE_ABORTED"});
    const rec = {sm: null, df: df ? df.map((c) => c.length) : null};
    this.passes.push(rec);
    // the flat pass form {counts, messages, indices, signatures}: one 0 / 1 byte per set, like the addon
    if (sm) rec.sm = Array.from(sm.counts);
    if (sm) rec.smIdx = Array.from(sm.indices);
    if (df) rec.dfPk = df.map((c) => c.map((s) => (s.pubkey ? s.pubkey[0] : null)));
    const res = {
      sameMessage: sm ? Uint8Array.from({length: sm.indices.length}, (_, i) => (sm.signatures[96 * i] === 1 ? 1 : 0)) : null,
      default: df
        ? df.map((c) =>
          c.some((s) => s.indices !== undefined && s.indices.length === 0)
            ? Object.assign(new Error("EMPTY_AGGREGATE_ARRAY"), {code: "EMPTY_AGGREGATE_ARRAY"})
            : c.length > 0 && c.every((s) => this.valid(s))
        )
        : null,
    };
    return {res};
  }
  async waitPass(p) {
    if (this.gate) await this.gate;
    await sleep(1);
    return p.res;
  }
  async close() {
    this.closed = true;
    this.destroyedAfter = this.passes.length;
  }
}

const set = (ok, index = 0) => ({index, signingRoot: new Uint8Array(32), signature: Uint8Array.from([ok ? 1 : 0].concat(new Array(95).fill(0)))});
const smSet = (ok, index = 0) => ({index, signature: Uint8Array.from([ok ? 1 : 0].concat(new Array(95).fill(0)))});
const msg = new Uint8Array(32);

async function expectReject(p, code) {
  try {
    await p;
    return "resolved";
  } catch (e) {
    return e.code === code ? "ok" : "wrong code " + e.code;
  }
}

async function cpu() {
  const shapes = [0, 255, 256, 300].map((n) => V.chunkifyMaximizeChunkSize(new Array(n).fill(0), 128).map((c) => c.length));
  report.chunkify = JSON.stringify(shapes) === JSON.stringify([[0], [255], [128, 128], [150, 150]]);

  // bls.test.ts: verify all / one invalid / empty
  let a = new FakeAddon();
  let v = new V.GpuBlsVerifier({addon: a});
  report.basic = [await v.verifySignatureSets([set(1), set(1), set(1)]), await v.verifySignatureSets([set(1), set(0), set(1)]),
    await v.verifySignatureSets([])];
  report.sameMessage = await v.verifySignatureSetsSameMessage([smSet(1), smSet(0), smSet(1)], msg);
  report.largeChunked = (await v.verifySignatureSets(new Array(300).fill(0).map(() => set(1)))) === true &&
    JSON.stringify(a.passes[a.passes.length - 1].df) === "[150,150]";

  // multithread.test.ts:109-129: a batched invalid request does not fail the others (one pass)
  a = new FakeAddon();
  v = new V.GpuBlsVerifier({addon: a});
  const bad = v.verifySignatureSets([set(0)], {batchable: true, priority: true});
  const good = new Array(8).fill(0).map(() => v.verifySignatureSets([set(1), set(1), set(1)], {batchable: true}));
  report.batchedInvalidIsolated = (await bad) === false && (await Promise.all(good)).every((x) => x === true);
  report.batchedOnePass = a.passes.length === 1 && JSON.stringify(a.passes[0].df) === JSON.stringify([1, 3, 3, 3, 3, 3, 3, 3, 3]);

  // buffering: batchable jobs wait for the 100 ms timer unless more than 32 sigs are buffered
  a = new FakeAddon();
  v = new V.GpuBlsVerifier({addon: a});
  let t0 = Date.now();
  const buffered = [0, 1, 2].map(() => v.verifySignatureSets([set(1)], {batchable: true}));
  await sleep(20);
  const stillBuffered = a.passes.length === 0;
  await Promise.all(buffered);
  report.bufferTimer = stillBuffered && Date.now() - t0 >= 95 && a.passes.length === 1;
  t0 = Date.now();
  await v.verifySignatureSets(new Array(V.MAX_BUFFERED_SIGS + 1).fill(0).map(() => set(1)), {batchable: true});
  report.bufferFlush = Date.now() - t0 < 90;

  // priority: front of the queue
  a = new FakeAddon();
  v = new V.GpuBlsVerifier({addon: a});
  v.passesBusy = v.maxPasses; // hold the queue
  const f1 = v.verifySignatureSets([set(1), set(1)]);
  const f2 = v.verifySignatureSets(new Array(5).fill(0).map(() => set(1)), {priority: true});
  await sleep(0);
  report.priority = JSON.stringify(v.jobs.map((j) => j.sets.length)) === "[5,2]" && v.canAcceptWork() === false;
  v.passesBusy = 0;
  v._schedule();
  await Promise.all([f1, f2]);

  // passes overlap: MAX_PASSES in flight, later calls wait and then go out as ONE pass
  a = new FakeAddon();
  let release;
  a.gate = new Promise((r) => (release = r));
  v = new V.GpuBlsVerifier({addon: a});
  const first = [];
  for (let k = 0; k < 3; k++) {
    first.push(v.verifySignatureSets(new Array(k + 1).fill(0).map(() => set(1))));
    await new Promise((r) => setImmediate(r));
  }
  const later = [0, 1, 2, 3].map((k) => v.verifySignatureSets([set(k !== 1)]));
  await sleep(5);
  report.overlap = v.passesBusy === 3 && v.jobs.length === 4 && !v.canAcceptWork();
  release();
  const r1 = await Promise.all(first);
  const r2 = await Promise.all(later);
  report.overlapResults = r1.every((x) => x === true) && JSON.stringify(r2) === "[true,false,true,true]" &&
    JSON.stringify(a.passes[3].df) === "[1,1,1,1]" && v.devicePasses === 4;

  // close: queued jobs reject with QUEUE_ABORTED, passes on the device finish first, then the context
  a = new FakeAddon();
  a.gate = new Promise((r) => (release = r));
  v = new V.GpuBlsVerifier({addon: a});
  const running = [];
  for (let k = 0; k < 3; k++) {
    running.push(v.verifySignatureSets([set(1)]));
    await new Promise((r) => setImmediate(r));
  }
  const queued = v.verifySignatureSets([set(1)]);
  const buffered2 = v.verifySignatureSets([set(1)], {batchable: true});
  queued.catch(() => {}); // rejections are awaited below; keep Node from warning meanwhile
  buffered2.catch(() => {});
  await sleep(2);
  const closing = v.close();
  await sleep(5);
  const notYet = a.destroyedAfter === null;
  release();
  await closing;
  report.close = notYet && a.destroyedAfter === 3 && (await Promise.all(running)).every((x) => x === true) &&
    (await expectReject(queued, "QUEUE_ABORTED")) === "ok" && (await expectReject(buffered2, "QUEUE_ABORTED")) === "ok" &&
    (await expectReject(v.verifySignatureSets([set(1)]), "QUEUE_ABORTED")) === "ok";

  // errors: an empty aggregate rejects its own call only; a bad index rejects before queueing
  a = new FakeAddon();
  v = new V.GpuBlsVerifier({addon: a});
  const e1 = v.verifySignatureSets([{indices: [], signingRoot: new Uint8Array(32), signature: new Uint8Array(96)}], {batchable: true});
  e1.catch(() => {});
  const ok1 = v.verifySignatureSets([set(1)], {batchable: true});
  report.emptyAggregate = (await expectReject(e1, "EMPTY_AGGREGATE_ARRAY")) === "ok" && (await ok1) === true;
  report.badIndex = (await expectReject(v.verifySignatureSets([set(1, 1 << 20)]), "GBV_E_ARG")) === "ok" &&
    (await expectReject(v.verifySignatureSetsSameMessage([smSet(1, 1 << 21)], msg), "GBV_E_ARG")) === "ok";

  // the reference's same-message call shape (interface.ts:55-59, attestation.ts:134-137):
  // {publicKey, signature} with no index, the key objects those of index2pubkey (registered by
  // identity); a key outside the table is verified from its bytes as a one-set job
  // verifyOnMainThread: synchronous device call, no queue
  report.mainThread = (await v.verifySignatureSets([set(1)], {verifyOnMainThread: true})) === true &&
    JSON.stringify(a.passes[a.passes.length - 1]) === '["sync",1]';

  const ka = new FakeAddon();
  const kv = new V.GpuBlsVerifier({addon: ka});
  const keyObjs = [0, 1, 2, 3].map((i) => ({toBytes: () => new Uint8Array(48).fill(i + 1)}));
  kv.registerPubkeyObjects(10, keyObjs);
  const pkSet = (ok, pk) => ({publicKey: pk, signature: smSet(ok).signature});
  const stranger = {toBytes: () => new Uint8Array(48).fill(9)};
  const rId = await kv.verifySignatureSetsSameMessage([pkSet(1, keyObjs[0]), pkSet(0, keyObjs[3]), pkSet(1, keyObjs[2])], msg);
  const idPass = ka.passes[ka.passes.length - 1];
  report.sameMessageByKeyIdentity = JSON.stringify(rId) === "[true,false,true]" && JSON.stringify(idPass.smIdx) === "[10,13,12]" &&
    kv.indexOf(keyObjs[1]) === 11 && kv.indexOf(stranger) === undefined &&
    JSON.stringify(kv.indicesOf([keyObjs[3], keyObjs[0]])) === "[13,10]" && kv.indicesOf([keyObjs[0], stranger]) === undefined;
  const nPass = ka.passes.length;
  const rOut = await kv.verifySignatureSetsSameMessage([pkSet(1, keyObjs[1]), pkSet(1, stranger), pkSet(0, stranger),
    pkSet(0, new Uint8Array(48).fill(7))], msg);
  const outPasses = ka.passes.slice(nPass);
  const smIdx = [].concat(...outPasses.filter((p) => p.smIdx).map((p) => p.smIdx));
  const dfPk = [].concat(...outPasses.filter((p) => p.dfPk).map((p) => [].concat(...p.dfPk)));
  report.sameMessageOutsideKeys = JSON.stringify(rOut) === "[true,true,false,false]" && JSON.stringify(smIdx) === "[11]" &&
    JSON.stringify(dfPk.sort()) === "[7,9,9]";
  report.sameMessageKeyless = (await expectReject(kv.verifySignatureSetsSameMessage([{signature: smSet(1).signature}], msg), "GBV_E_ARG")) === "ok";

  // metrics: the reference's families
  const text = v.metricsText();
  report.metrics = ["lodestar_bls_thread_pool_sig_sets_total", "lodestar_bls_thread_pool_jobs_started_total",
    "lodestar_bls_thread_pool_queue_job_wait_time_seconds_bucket", "lodestar_bls_thread_pool_workers_busy",
    "lodestar_bls_thread_pool_error_aggregate_signature_sets_count", "lodestar_bls_worker_thread_time_per_sigset_seconds",
    "lodestar_bls_thread_pool_gpu_device_passes_total"].every((n) => text.includes(n));
  report.metricValues = v.metrics.totalSigSets.value() === 4 && v.metrics.errorAggregateSignatureSetsCount.value({type: "default"}) === 1;
}

// ---- a stand-in of the node's metrics: prom-client-shaped families on a registry, the blsThreadPool
// object built with the reference's names (metrics/metrics/lodestar.ts:401-504)
class PromFamily {
  constructor(kind, cfg) {
    this.kind = kind;
    this.name = cfg.name;
    this.series = new Map();
    this.collects = [];
  }
  _s(labels) {
    const k = JSON.stringify(labels || {});
    if (!this.series.has(k)) this.series.set(k, {value: 0, count: 0});
    return this.series.get(k);
  }
  inc(a, b) {
    if (typeof a === "object") this._s(a).value += b === undefined ? 1 : b;
    else this._s(null).value += a === undefined ? 1 : a;
  }
  set(a, b) {
    if (typeof a === "object") this._s(a).value = b;
    else this._s(null).value = a;
  }
  observe(a, b) {
    const s = typeof a === "object" ? this._s(a) : this._s(null);
    s.value += typeof a === "object" ? b : a;
    s.count += 1;
  }
  addCollect(fn) {
    this.collects.push(fn);
  }
  total() {
    let t = 0;
    for (const s of this.series.values()) t += this.kind === "histogram" ? s.count : s.value;
    return t;
  }
}
function fakeNodeMetrics() {
  const families = new Map();
  const mk = (kind) => (cfg) => {
    const f = new PromFamily(kind, cfg);
    families.set(cfg.name, f);
    return f;
  };
  const register = {gauge: mk("gauge"), histogram: mk("histogram"), families};
  const p = "lodestar_bls_thread_pool_";
  const g = (name) => register.gauge({name});
  const h = (name) => register.histogram({name});
  const blsThreadPool = {
    jobsWorkerTime: g(p + "time_seconds_sum"), successJobsSignatureSetsCount: g(p + "success_jobs_signature_sets_count"),
    errorAggregateSignatureSetsCount: g(p + "error_aggregate_signature_sets_count"), errorJobsSignatureSetsCount: g(p + "error_jobs_signature_sets_count"),
    jobWaitTime: h(p + "queue_job_wait_time_seconds"), queueLength: g(p + "queue_length"), workersBusy: g(p + "workers_busy"),
    totalJobsGroupsStarted: g(p + "job_groups_started_total"), totalJobsStarted: g(p + "jobs_started_total"),
    totalSigSetsStarted: g(p + "sig_sets_started_total"), batchRetries: g(p + "batch_retries_total"), batchSigsSuccess: g(p + "batch_sigs_success_total"),
    sameMessageRetryJobs: g(p + "same_message_jobs_retries_total"), sameMessageRetrySets: g(p + "same_message_sets_retries_total"),
    latencyToWorker: h(p + "latency_to_worker"), latencyFromWorker: h(p + "latency_from_worker"),
    mainThreadDurationInThreadPool: h(p + "main_thread_time_seconds"), timePerSigSet: h("lodestar_bls_worker_thread_time_per_sigset_seconds"),
    totalSigSets: g(p + "sig_sets_total"), prioritizedSigSets: g(p + "prioritized_sig_sets_total"), batchableSigSets: g(p + "batchable_sig_sets_total"),
  };
  return {blsThreadPool, register};
}

async function cpuNodeMetrics() {
  // the binding's wiring (chain/bls/gpu/index.ts): the node's families in, fed by every call
  const node = fakeNodeMetrics();
  const a = new FakeAddon();
  const v = new V.GpuBlsVerifier({addon: a, metrics: V.nodeMetricFamilies(node)});
  await v.verifySignatureSets([set(1), set(1)], {priority: true});
  await v.verifySignatureSets([set(1), set(0)], {batchable: true});
  const sm = await v.verifySameMessageSets([smSet(1, 3), smSet(0, 4), smSet(1, 5)], msg);
  const short = await v.verifySameMessageSets([{index: 1, signature: new Uint8Array(32)}], msg);
  for (const f of node.blsThreadPool.queueLength.collects) f();  // a scrape
  const fam = node.register.families;
  const got = (n) => (fam.has(n) ? fam.get(n).total() : -1);
  const p = "lodestar_bls_thread_pool_";
  report.nodeMetricsFed = got(p + "sig_sets_total") === 4 && got(p + "prioritized_sig_sets_total") === 2 &&
    got(p + "batchable_sig_sets_total") === 2 && got(p + "jobs_started_total") === 4 && got(p + "sig_sets_started_total") === 8 &&
    got(p + "job_groups_started_total") >= 2 && got(p + "queue_job_wait_time_seconds") === 4 && got(p + "gpu_device_passes_total") >= 2 &&
    got(p + "gpu_pass_time_seconds") >= 2 && got(p + "same_message_jobs_retries_total") === 2 && got(p + "time_seconds_sum") > 0;
  report.nodeMetricsScrape = fam.get(p + "queue_length").series.size === 1 && fam.get(p + "workers_busy").series.size === 1;
  // the IBlsVerifier-shaped same-message call: objects in, the packed device form, boolean[] out
  report.sameMessageObjectsPacked = JSON.stringify(sm) === "[true,false,true]" && JSON.stringify(short) === "[false]";
}

// ---- GPU: the real addon --------------------------------------------------------------------
const toSets = (c) =>
  c.sets.map((s) => {
    const o = {signingRoot: hex(s.msg), signature: hex(s.sig)};
    if (s.raw_pk) o.pubkey = hex(s.raw_pk);
    else if (s.indices.length === 1) o.index = s.indices[0];
    else o.indices = s.indices;
    return o;
  });

async function gpu(fixPath) {
  const addon = require(path.join(__dirname, "gbv_addon.node"));
  const fix = JSON.parse(fs.readFileSync(fixPath, "utf8"));
  const v = new V.GpuBlsVerifier({addon, device: 0});
  v.addPubkeys(0, Uint8Array.from(Buffer.concat(fix.keys.pks.map((p) => Buffer.from(p, "hex")))), true);
  // every verifySignatureSets case as its own concurrent call: they share device passes
  const vs = await Promise.all(fix.verify_sets.map((c) => v.verifySignatureSets(toSets(c)).then((r) => r === c.expected,
    (e) => c.expected === "reject" && e.code === "EMPTY_AGGREGATE_ARRAY")));
  report.verifySets = vs;
  const sm = await Promise.all(fix.same_message.map((c) =>
    v.verifySignatureSetsSameMessage(c.indices.map((idx, k) => ({index: idx, signature: hex(c.sigs[k])})), hex(c.msg))
      .then((r) => JSON.stringify(r) === JSON.stringify(c.expected))));
  report.sameMessage = sm;
  // the reference's call shape on the device: {publicKey, signature} with no index, stand-in PublicKey
  // objects registered as index2pubkey's (loadIndex2pubkey); then every second set's key replaced by an
  // unregistered object with the same bytes (a key outside the table): the same booleans
  const keyObjs = fix.keys.pks.map((p) => ({toBytes: () => hex(p)}));
  v.registerPubkeyObjects(0, keyObjs);
  report.sameMessageByKey = await Promise.all(fix.same_message.map((c) =>
    v.verifySignatureSetsSameMessage(c.indices.map((idx, k) => ({publicKey: keyObjs[idx], signature: hex(c.sigs[k])})), hex(c.msg))
      .then((r) => JSON.stringify(r) === JSON.stringify(c.expected))));
  report.sameMessageOutsideKeys = await Promise.all(fix.same_message.map((c) =>
    v.verifySignatureSetsSameMessage(c.indices.map((idx, k) => ({publicKey: k % 2 ? {toBytes: () => hex(fix.keys.pks[idx])} : keyObjs[idx],
      signature: hex(c.sigs[k])})), hex(c.msg))
      .then((r) => JSON.stringify(r) === JSON.stringify(c.expected))));
  // multithread.test.ts:85-106: 8 x (verifySignatureSets + verifySignatureSetsSameMessage), synchronously
  // and with a tick between submissions, batched or not, with and without priority
  const valid = toSets(fix.verify_sets.find((c) => c.name === "distinct_valid"));
  const smc = fix.same_message.find((c) => c.name === "all_valid");
  const smSets = smc.indices.map((idx, k) => ({index: idx, signature: hex(smc.sigs[k])}));
  const many = [];
  for (const sleepTick of [false, true]) {
    for (const opts of [{}, {priority: true}, {batchable: true}, {batchable: true, priority: true}]) {
      const ps = [];
      for (let i = 0; i < 8; i++) {
        ps.push(v.verifySignatureSets(valid, opts));
        ps.push(v.verifySignatureSetsSameMessage(smSets, hex(smc.msg), opts));
        if (sleepTick) await sleep(5);
      }
      const rs = await Promise.all(ps);
      many.push(rs.every((r, i) => (i % 2 === 0 ? r === true : JSON.stringify(r) === "[true,true,true]")));
    }
  }
  report.manyCalls = many;
  // multithread.test.ts:109-129: a batched request with a 32-byte signature fails alone
  const invalid = Object.assign({}, valid[0], {signature: new Uint8Array(32)});
  const inv = v.verifySignatureSets([invalid], {batchable: true, priority: true});
  const rest = new Array(8).fill(0).map(() => v.verifySignatureSets(valid, {batchable: true}));
  report.batchedInvalid = (await inv) === false && (await Promise.all(rest)).every((r) => r === true);
  report.mainThread = (await v.verifySignatureSets(valid, {verifyOnMainThread: true})) === true;
  report.devicePasses = v.devicePasses;
  report.metrics = v.metricsText().includes("lodestar_bls_thread_pool_gpu_device_passes_total");
  const pending = v.verifySignatureSets(valid);
  await v.close();
  report.inflightBeforeClose = await pending.then((r) => r === true, (e) => e.code === "QUEUE_ABORTED");
  report.afterClose = await v.verifySignatureSets(valid).then(() => "resolved", (e) => e.code);
}

(async () => {
  const mode = process.argv[2];
  if (mode === "cpu") {
    await cpu();
    await cpuNodeMetrics();
  }
  else await gpu(process.argv[3]);
  process.stdout.write(JSON.stringify(report) + "\n");
  process.exit(0);  // Node 12's teardown finalizer crash: see bench_api.js
})().catch((e) => {
  process.stdout.write(JSON.stringify({fatal: String((e && e.stack) || e), code: e && e.code}) + "\n");
  process.exit(1);
});
