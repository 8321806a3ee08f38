// Exercises the Node-API addon (addon/gbv_addon.node) from JavaScript, as a Lodestar GpuBlsVerifier
// would call it.  Used by tests/test_addon.py.
//   node addon/test_addon.js cpu               exports, argument and error mapping (no GPU needed)
//   node addon/test_addon.js gpu <fixtures>    every golden case through the addon on device 0
"use strict";
const path = require("path");
const fs = require("fs");
const addon = require(path.join(__dirname, "gbv_addon.node"));

const EXPORTS = ["open", "addPubkeys", "verifySets", "verifySetsMulti", "verifySameMessageMulti", "aggregatePubkeys",
  "aggregateSerializedPubkeys", "aggregateSignatures", "validateSignatures", "close", "submitPass", "waitPass", "freePasses",
  "pubkeyCount", "verifySetsSync", "vsPartial", "fp12Check", "merkleRoots", "signingRoots", "replicatePubkeys"];
const hex = (h) => Uint8Array.from(Buffer.from(h, "hex"));
const report = {};

function expectThrow(fn, code) {
  try {
    fn();
  } catch (e) {
    return e.code === code ? "ok" : "wrong code " + e.code;
  }
  return "no throw";
}

function toSets(c) {
  return c.sets.map((s) => {
    const o = {signingRoot: hex(s.msg), signature: hex(s.sig)};
    if (s.raw_pk) o.pubkey = hex(s.raw_pk);
    else if (s.indices.length === 1) o.index = s.indices[0];
    else o.indices = Uint32Array.from(s.indices);
    return o;
  });
}

// BlsSingleThreadVerifier.verifySignatureSetsSameMessage (singleThread.ts:36-80) written over the
// addon, as the TypeScript side of a drop-in would: device aggregate pubkey, device signature
// validation, device aggregateSignatures, one unrandomized verify, per-set retry in one pass.
async function singleThreadSameMessage(ctx, sets, message) {
  const pk = addon.aggregatePubkeys(ctx, sets.map((s) => s.index)); // throws EMPTY_AGGREGATE_ARRAY on []
  const sigs = Buffer.concat(sets.map((s) => Buffer.from(s.signature.length === 96 ? s.signature : new Uint8Array(96))));
  const st = addon.validateSignatures(ctx, Uint8Array.from(sigs));
  let isAllValid = Array.from(st).every((x) => x === 0);
  if (isAllValid) {
    const agg = addon.aggregateSignatures(ctx, Uint8Array.from(sigs), true);
    isAllValid = await addon.verifySets(ctx, [{pubkey: pk, signingRoot: message, signature: agg}]);
  }
  if (isAllValid) return sets.map(() => true);
  const todo = sets.map((_, i) => i).filter((i) => st[i] === 0);
  const res = await addon.verifySetsMulti(ctx, todo.map((i) => [{index: sets[i].index, signingRoot: message, signature: sets[i].signature}]));
  const out = sets.map(() => false);
  todo.forEach((i, k) => (out[i] = res[k] === true));
  return out;
}

async function cpu() {
  report.exports = EXPORTS.filter((k) => typeof addon[k] === "function");
  report.maxPasses = addon.MAX_PASSES;
  report.open = expectThrow(() => addon.open(0), "GBV_E_DEVICE");
  report.badCtx = expectThrow(() => addon.verifySets({}, []), "GBV_E_ARG");
  report.badArg = expectThrow(() => addon.open("x"), "GBV_E_ARG");
}

async function gpu(fixPath) {
  const fix = JSON.parse(fs.readFileSync(fixPath, "utf8"));
  const ctx = addon.open(0);
  const pks = Buffer.concat(fix.keys.pks.map((p) => Buffer.from(p, "hex")));
  const st = addon.addPubkeys(ctx, 0, Uint8Array.from(pks), true);
  report.ingest = Array.from(st).every((x) => x === 0);
  // verifySets, one call per fixture case (rejections carry EMPTY_AGGREGATE_ARRAY)
  const vs = [];
  for (const c of fix.verify_sets) {
    try {
      const r = await addon.verifySets(ctx, toSets(c));
      vs.push(r === c.expected);
    } catch (e) {
      vs.push(c.expected === "reject" && e.code === "EMPTY_AGGREGATE_ARRAY");
    }
  }
  report.verifySets = vs;
  // all cases in one device pass
  const multi = await addon.verifySetsMulti(ctx, fix.verify_sets.map(toSets));
  report.verifySetsMulti = multi.map((r, i) => {
    const want = fix.verify_sets[i].expected;
    return want === "reject" ? r instanceof Error && r.code === "EMPTY_AGGREGATE_ARRAY" : r === want;
  });
  const calls = fix.same_message.map((c) => ({
    message: hex(c.msg),
    sets: c.indices.map((idx, k) => ({index: idx, signature: hex(c.sigs[k])})),
  }));
  const sm = await addon.verifySameMessageMulti(ctx, calls);
  report.sameMessage = sm.map((r, i) => JSON.stringify(r) === JSON.stringify(fix.same_message[i].expected));
  report.aggregate = fix.aggregate_pubkeys.map((c) => Buffer.from(addon.aggregatePubkeys(ctx, c.indices)).toString("hex") === c.expected);
  report.aggregateSerialized = fix.aggregate_pubkeys.map((c) => {
    const ser = Buffer.concat(c.indices.map((i) => Buffer.from(fix.keys.pks[i], "hex")));
    return Buffer.from(addon.aggregateSerializedPubkeys(ctx, Uint8Array.from(ser), false)).toString("hex") === c.expected;
  });
  report.emptyAggregate = expectThrow(() => addon.aggregatePubkeys(ctx, []), "EMPTY_AGGREGATE_ARRAY");
  // single-thread semantics (tests/golden/single_thread.json) over the addon primitives
  const stf = JSON.parse(fs.readFileSync(path.join(path.dirname(fixPath), "single_thread.json"), "utf8"));
  addon.addPubkeys(ctx, stf.extra_index, hex(stf.extra_pk), true);
  const single = [];
  for (const c of stf.same_message) {
    const sets = c.indices.map((idx, k) => ({index: idx, signature: hex(c.sigs[k])}));
    try {
      single.push(JSON.stringify(await singleThreadSameMessage(ctx, sets, hex(c.msg))) === JSON.stringify(c.expected));
    } catch (e) {
      single.push(c.expected === "reject" && e.code === "EMPTY_AGGREGATE_ARRAY");
    }
  }
  report.singleThread = single;
  report.aggregateSignatures = stf.aggregate_signatures.map((c) => {
    const sigs = Uint8Array.from(Buffer.concat(c.sigs.map((x) => Buffer.from(x, "hex"))));
    try {
      return Buffer.from(addon.aggregateSignatures(ctx, sigs, c.validate)).toString("hex") === c.expected;
    } catch (e) {
      return (c.expected === "bad_point" && e.code === "GBV_E_BAD_POINT") || (c.expected === "empty" && e.code === "EMPTY_AGGREGATE_ARRAY");
    }
  });
  // the streamed pair: MAX_PASSES passes submitted before any is waited, a bad set in each
  const passes = [];
  for (let k = 0; k < addon.MAX_PASSES; k++) {
    passes.push(addon.submitPass(ctx, calls, fix.verify_sets.map(toSets)));
  }
  report.freeWhileBusy = addon.freePasses(ctx);
  let busyThrows = "no throw";
  try {
    addon.submitPass(ctx, calls, null);
  } catch (e) {
    busyThrows = e.code;
  }
  report.busyThrows = busyThrows;
  const results = await Promise.all(passes.map((p) => addon.waitPass(p)));
  report.streamed = results.map((r) =>
    r.sameMessage.every((x, i) => JSON.stringify(x) === JSON.stringify(fix.same_message[i].expected)) &&
    r.default.every((x, i) => (fix.verify_sets[i].expected === "reject" ? x instanceof Error && x.code === "EMPTY_AGGREGATE_ARRAY" : x === fix.verify_sets[i].expected)));
  report.freeAfter = addon.freePasses(ctx);
  report.verifySetsSync = addon.verifySetsSync(ctx, toSets(fix.verify_sets[0])) === fix.verify_sets[0].expected;
  report.pubkeyCount = addon.pubkeyCount(ctx);
  // one verifySignatureSets call as two shards on this device: partials, then one final exponentiation
  const all = toSets(fix.verify_sets[0]);
  const p1 = addon.vsPartial(ctx, all.slice(0, 1)), p2 = addon.vsPartial(ctx, all.slice(1));
  report.shards = p1.ok && p2.ok && addon.fp12Check(ctx, Uint8Array.from(Buffer.concat([Buffer.from(p1.partial), Buffer.from(p2.partial)]))) === true;
  const wrong = toSets(fix.verify_sets[1]);
  const w1 = addon.vsPartial(ctx, wrong.slice(0, 2)), w2 = addon.vsPartial(ctx, wrong.slice(2));
  report.shardsWrong = addon.fp12Check(ctx, Uint8Array.from(Buffer.concat([Buffer.from(w1.partial), Buffer.from(w2.partial)]))) === false;
  // concurrent submissions are serialised per context and all resolve
  const conc = await Promise.all([0, 1, 2, 3].map(() => addon.verifySets(ctx, toSets(fix.verify_sets[0]))));
  report.concurrent = conc.every((r) => r === fix.verify_sets[0].expected);
  const pending = addon.verifySets(ctx, toSets(fix.verify_sets[0]));
  await addon.close(ctx);
  report.inflightBeforeClose = await pending.then((r) => r === fix.verify_sets[0].expected, (e) => e.code === "QUEUE_ABORTED");
  report.afterClose = await addon.verifySets(ctx, toSets(fix.verify_sets[0])).then(() => "resolved", (e) => e.code);
}

(async () => {
  const mode = process.argv[2];
  if (mode === "cpu") await cpu();
  else await gpu(process.argv[3]);
  process.stdout.write(JSON.stringify(report) + "\n");
  process.exit(0);  // Node 12's teardown finalizer crash: see bench_api.js
})().catch((e) => {
  process.stdout.write(JSON.stringify({fatal: String(e && e.stack || e), code: e && e.code}) + "\n");
  process.exit(1);
});
