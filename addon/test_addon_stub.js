// The real Node-API addon (addon/gbv_addon.c) over the CPU stand-in library tests/native/gbv_stub.c,
// for sanitizer runs of the host C (tools/sanitize_host.sh builds both with
// -fsanitize=address,undefined).  Every entry point, the streamed pass slots, concurrent async work on
// the libuv pool, close() while passes are in flight (multithread/index.ts:238-259: queued work
// rejects with QUEUE_ABORTED, running work finishes first), context finalisation by the GC, and the
// JavaScript GpuBlsVerifier (addon/gpu_bls_verifier.js) driving the addon.  Stand-in rules (as
// addon/test_verifier.js): a set is valid iff its signature starts with 1; a key starting with 0 is
// invalid.  Prints one JSON line; tests/test_addon.py checks it.
//   node --expose-gc addon/test_addon_stub.js <path to the addon .node>
"use strict";
const path = require("path");
const A = require(path.resolve(process.argv[2] || path.join(__dirname, "gbv_addon.node")));
const V = require(path.join(__dirname, "gpu_bls_verifier.js"));

const report = {};
const sig = (ok) => Uint8Array.from([ok ? 1 : 0].concat(new Array(95).fill(0)));
const root = new Uint8Array(32);
const set = (ok, index = 0) => ({index, signingRoot: root, signature: sig(ok)});
const codeOf = async (p) => {
  try {
    await p;
    return "resolved";
  } catch (e) {
    return e.code;
  }
};
const codeOfSync = (f) => {
  try {
    f();
    return "returned";
  } catch (e) {
    return e.code;
  }
};

async function direct() {
  const ctx = A.open(0);
  const keys = new Uint8Array(48 * 8).fill(1);
  keys[48 * 5] = 0; // slot 5 unusable
  const st = A.addPubkeys(ctx, 0, keys, true);
  report.ingest = Array.from(st).join(",") === "0,0,0,0,0,1,0,0" && A.pubkeyCount(ctx) === 8;

  report.verifySets = [
    await A.verifySets(ctx, [set(1, 0), set(1, 1)]),
    await A.verifySets(ctx, [set(1, 0), set(0, 1)]),
    await A.verifySets(ctx, []),
    await A.verifySets(ctx, [set(1, 5)]),
    await A.verifySets(ctx, [{indices: [0, 1, 2], signingRoot: root, signature: sig(1)}]),
    await A.verifySets(ctx, [{pubkey: new Uint8Array(48).fill(1), signingRoot: root, signature: sig(1)}]),
  ].join(",") === "true,false,false,false,true,true";
  report.emptyAggregate = await codeOf(A.verifySets(ctx, [{indices: [], signingRoot: root, signature: sig(1)}]));
  report.badIndex = await codeOf(A.verifySets(ctx, [set(1, 1 << 20)]));
  const multi = await A.verifySetsMulti(ctx, [[set(1)], [set(0)], [{indices: [], signingRoot: root, signature: sig(1)}], []]);
  report.verifySetsMulti = multi[0] === true && multi[1] === false && multi[2].code === "EMPTY_AGGREGATE_ARRAY" && multi[3] === false;
  const sm = await A.verifySameMessageMulti(ctx, [{sets: [{index: 0, signature: sig(1)}, {index: 1, signature: sig(0)}], message: root},
    {sets: [{index: 2, signature: new Uint8Array(10)}], message: root}]);
  report.sameMessage = JSON.stringify(sm) === "[[true,false],[false]]";
  report.aggregate = A.aggregatePubkeys(ctx, [0, 1, 2]).length === 48 &&
    codeOfSync(() => A.aggregatePubkeys(ctx, [])) === "EMPTY_AGGREGATE_ARRAY";
  report.aggregateSerialized = A.aggregateSerializedPubkeys(ctx, keys.subarray(0, 96), true).length === 48 &&
    codeOfSync(() => A.aggregateSerializedPubkeys(ctx, keys, true)) === "GBV_E_BAD_POINT";
  const two = new Uint8Array(192);
  two[0] = 1;
  two[96] = 1;
  report.aggregateSignatures = A.aggregateSignatures(ctx, two, true).length === 96 &&
    codeOfSync(() => A.aggregateSignatures(ctx, new Uint8Array(96), true)) === "GBV_E_BAD_POINT";
  report.validateSignatures = Array.from(A.validateSignatures(ctx, Uint8Array.from([...two, ...new Uint8Array(96)]))).join(",") === "0,0,1";
  report.argErrors = [codeOfSync(() => A.verifySets({}, [])), codeOfSync(() => A.addPubkeys(ctx, 0, new Uint8Array(47), true)),
    codeOfSync(() => A.submitPass(ctx, 7, null))].join(",");

  // many calls in flight on the libuv pool at once, the synchronous form between them
  const many = [];
  for (let i = 0; i < 24; ++i) many.push(A.verifySets(ctx, [set(i % 5 !== 4, i % 8 === 5 ? 0 : i % 8)]));
  const syncOk = A.verifySetsSync(ctx, [set(1, 3)]);
  const manyRes = await Promise.all(many);
  report.concurrent = syncOk === true && manyRes.every((r, i) => r === (i % 5 !== 4));

  // the streamed pair: every slot in flight, a fourth submit throws, results right
  const passes = [];
  for (let k = 0; k < A.MAX_PASSES; ++k)
    passes.push(A.submitPass(ctx, [{sets: [{index: 0, signature: sig(1)}, {index: 1, signature: sig(k !== 1)}], message: root}],
      [[set(1)], [set(k !== 2)]]));
  report.freeWhileBusy = A.freePasses(ctx);
  report.busyThrows = codeOfSync(() => A.submitPass(ctx, null, [[set(1)]]));
  const res = await Promise.all(passes.map((p) => A.waitPass(p)));
  report.streamed = res.map((r, k) => JSON.stringify(r.sameMessage) === JSON.stringify([[true, k !== 1]]) &&
    JSON.stringify(r.default) === JSON.stringify([true, k !== 2]));
  report.freeAfter = A.freePasses(ctx);
  report.waitTwice = codeOfSync(() => A.waitPass(passes[0]));

  // shards
  const p1 = A.vsPartial(ctx, [set(1, 0), set(1, 1)]);
  const p2 = A.vsPartial(ctx, [set(1, 2)]);
  const pb = A.vsPartial(ctx, [set(0, 2)]);
  const cat = (xs) => {
    const o = new Uint8Array(576 * xs.length);
    xs.forEach((x, i) => o.set(x.partial, 576 * i));
    return o;
  };
  report.shards = A.fp12Check(ctx, cat([p1, p2])) === true && A.fp12Check(ctx, cat([p1, pb])) === false;

  // close() while two passes are on the device: their waits finish first, later calls reject
  const q1 = A.submitPass(ctx, null, [[set(1)]]);
  const q2 = A.submitPass(ctx, [{sets: [{index: 0, signature: sig(1)}], message: root}], null);
  const w1 = A.waitPass(q1), w2 = A.waitPass(q2);
  const pending = A.verifySets(ctx, [set(1)]);
  const closing = A.close(ctx);
  report.afterClose = [await codeOf(A.verifySets(ctx, [set(1)])), codeOfSync(() => A.submitPass(ctx, null, [[set(1)]])),
    codeOfSync(() => A.verifySetsSync(ctx, [set(1)]))].join(",");
  const r1 = await w1, r2 = await w2;
  report.inflightBeforeClose = r1.default[0] === true && r2.sameMessage[0][0] === true;
  report.pendingAtClose = await codeOf(pending);
  await closing;
  await A.close(ctx); // idempotent
  report.pubkeyCountClosed = A.pubkeyCount(ctx) === 0;
}

async function verifier() {
  // the JavaScript GpuBlsVerifier over the real addon (stand-in device)
  const v = new V.GpuBlsVerifier({addon: A});
  const keys = new Uint8Array(48 * 4).fill(1);
  v.addPubkeys(0, keys, true);
  const bad = v.verifySignatureSets([set(0)], {batchable: true});
  const good = [0, 1, 2, 3].map(() => v.verifySignatureSets([set(1), set(1, 1)], {batchable: true}));
  const smp = v.verifySignatureSetsSameMessage([{index: 0, signature: sig(1)}, {index: 1, signature: sig(0)}], root);
  report.jsBatched = (await bad) === false && (await Promise.all(good)).every((x) => x === true) &&
    JSON.stringify(await smp) === "[true,false]";
  // packed same-message calls: one chunk, and 300 sets in two chunks (chunkifyMaximizeChunkSize)
  const packed = (oks) => ({indices: Uint32Array.from(oks.map((_, i) => i % 4)), signatures: Uint8Array.from(Buffer.concat(oks.map((ok) => Buffer.from(sig(ok)))))});
  const p1 = await v.verifySignatureSetsSameMessage(packed([1, 0, 1]), root);
  const big = new Array(300).fill(1).map((_, i) => (i % 97 === 5 ? 0 : 1));
  const p2 = await v.verifySignatureSetsSameMessage(packed(big), root);
  report.jsPacked = p1 instanceof Uint8Array && Array.from(p1).join(",") === "1,0,1" && p2.length === 300 &&
    Array.from(p2).every((x, i) => x === big[i]);
  report.jsPackedBadLength = await codeOf(v.verifySignatureSetsSameMessage({indices: Uint32Array.from([0]), signatures: new Uint8Array(95)}, root));
  // close() with work on the device and queued behind it: device passes resolve, queued jobs reject
  // with QUEUE_ABORTED (multithread/index.ts:238-259), later calls too
  const calls = [v.verifySignatureSets(new Array(300).fill(0).map((_, i) => set(1, i % 4)))].concat(
    [0, 1, 2, 3, 4, 5].map((i) => v.verifySignatureSetsSameMessage([{index: i % 4, signature: sig(1)}], root)));
  await new Promise((r) => setImmediate(r));
  const closing = v.close();
  const after = await codeOf(v.verifySignatureSets([set(1)]));
  const settled = await Promise.allSettled(calls);
  report.jsClose = after === "QUEUE_ABORTED" && settled.every((x) => (x.status === "fulfilled" && (x.value === true || x.value[0] === true)) ||
    (x.status === "rejected" && x.reason.code === "QUEUE_ABORTED")) && settled.some((x) => x.status === "fulfilled");
  await closing;
}

async function finalizers() {
  // contexts dropped without close(): ctx_finalize frees them when the GC runs
  for (let i = 0; i < 8; ++i) {
    const c = A.open(0);
    A.addPubkeys(c, 0, new Uint8Array(48).fill(1), false);
    await A.verifySets(c, [set(1)]);
  }
  if (global.gc) {
    global.gc();
    await new Promise((r) => setTimeout(r, 10));
    global.gc();
  }
  report.finalized = true;
}

(async () => {
  try {
    await direct();
    await verifier();
    await finalizers();
  } catch (e) {
    report.fatal = String(e && e.stack ? e.stack : e);
  }
  console.log(JSON.stringify(report));
})();
