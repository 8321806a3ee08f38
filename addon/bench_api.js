// The C2 gossip stream through the JavaScript GpuBlsVerifier over the Node-API addon -- the path a
// Lodestar node would use (verifySignatureSetsSameMessage per gossip call, multithread/index.ts:212-236
// call shape) -- timed end to end on the GPU box: every call issued, every promise awaited, every
// boolean checked.  Run by bench.py (api_path_js) with a workload directory it writes:
//   meta.json {n_sets, n_calls, n_keys, table}, call_off.u32, idx.u32, sigs.bin (96 n), msgs.bin (32 calls),
//   keys.bin (48 n_keys: the table is keys[i mod n_keys], built with addPubkeys + replicatePubkeys)
//   node addon/bench_api.js <dir> [reps]
// Prints one JSON line: packed-form, IBlsVerifier-shaped ("ibls": {publicKey, signature} objects, keys
// found by identity and packed per pass inside the clock, as the Lodestar binding does) and index-form
// object sets/s (best of reps), passes, validity.
"use strict";
const path = require("path");
const fs = require("fs");
const V = require(path.join(__dirname, "gpu_bls_verifier.js"));
const addon = require(path.join(__dirname, "gbv_addon.node"));

const dir = process.argv[2];
const reps = parseInt(process.argv[3] || "3", 10);
const meta = JSON.parse(fs.readFileSync(path.join(dir, "meta.json")));
const u32 = (f) => {
  const b = fs.readFileSync(path.join(dir, f));
  return new Uint32Array(b.buffer, b.byteOffset, b.length / 4);
};
const bytes = (f) => {
  const b = fs.readFileSync(path.join(dir, f));
  return new Uint8Array(b.buffer, b.byteOffset, b.length);
};

async function main() {
  const callOff = u32("call_off.u32");
  const idx = u32("idx.u32");
  const sigs = bytes("sigs.bin");
  const msgs = bytes("msgs.bin");
  const keys = bytes("keys.bin");
  const v = new V.GpuBlsVerifier({addon});
  const st = v.addPubkeys(0, keys, true);
  if (!st.every((x) => x === 0)) throw new Error("key ingest failed");
  addon.replicatePubkeys(v.ctx, 0, meta.n_keys, meta.n_keys, meta.table - meta.n_keys);
  const nCalls = meta.n_calls;
  const message = (g) => msgs.subarray(32 * g, 32 * g + 32);
  // index2pubkey's PublicKey objects (stand-ins: identity is all the verifier reads of them), registered
  // the way the binding's loadIndex2pubkey does
  const keyObjs = new Array(meta.table);
  for (let i = 0; i < meta.table; ++i) keyObjs[i] = {validator: i};
  v.registerPubkeyObjects(0, keyObjs);
  // the caller's deserialized gossip data, built before the clock: packed views; one {publicKey,
  // signature} object per set, the reference's call shape (interface.ts:55-59, attestation.ts:134-137);
  // and one {index, signature} object per set (the index form)
  const packed = [];
  const ibls = [];
  const objects = [];
  for (let g = 0; g < nCalls; ++g) {
    const a = callOff[g], b = callOff[g + 1];
    packed.push({indices: idx.subarray(a, b), signatures: sigs.subarray(96 * a, 96 * b)});
    const sets = new Array(b - a), isets = new Array(b - a);
    for (let i = a; i < b; ++i) {
      sets[i - a] = {index: idx[i], signature: sigs.subarray(96 * i, 96 * i + 96)};
      isets[i - a] = {publicKey: keyObjs[idx[i]], signature: sigs.subarray(96 * i, 96 * i + 96)};
    }
    objects.push(sets);
    ibls.push(isets);
  }
  const nSets = callOff[nCalls];
  async function stream(form) {
    const calls = form === "packed" ? packed : form === "ibls" ? ibls : objects;
    const p0 = v.devicePasses;
    const t0 = process.hrtime.bigint();
    // "ibls": the IBlsVerifier call shape the Lodestar binding uses (chain/bls/gpu/index.ts over
    // verifySameMessageSets): one {publicKey, signature} object per set in (index by key identity),
    // boolean[] out; the packing into the device form happens here, inside the clock
    const res = form === "ibls"
      ? await Promise.all(calls.map((s, g) => v.verifySameMessageSets(s, message(g))))
      : await Promise.all(calls.map((s, g) => v.verifySignatureSetsSameMessage(s, message(g))));
    let ok = 0;
    for (const r of res) for (let i = 0; i < r.length; ++i) ok += r[i] ? 1 : 0;
    const sec = Number(process.hrtime.bigint() - t0) / 1e9;
    if (ok !== nSets) throw new Error(form + ": " + ok + " of " + nSets + " sets valid");
    return {rate: nSets / sec, sec, passes: v.devicePasses - p0};
  }
  await stream("packed"); // warm the pass slots (first-use allocation stays out of the clock)
  const out = {sets: nSets, calls: nCalls, reps};
  for (const form of ["packed", "ibls", "objects"]) {
    let best = null;
    for (let r = 0; r < reps; ++r) {
      const x = await stream(form);
      if (!best || x.rate > best.rate) best = x;
    }
    out[form] = {sets_per_s: Math.round(best.rate), seconds: Number(best.sec.toFixed(4)), device_passes: best.passes};
  }
  // one lone 64-set call through the same path (submit -> promise resolves), median of 20
  const lat = [];
  for (let r = 0; r < 20; ++r) {
    const t0 = process.hrtime.bigint();
    const res = await v.verifySignatureSetsSameMessage({indices: idx.subarray(0, 64), signatures: sigs.subarray(0, 96 * 64)}, message(0));
    lat.push(Number(process.hrtime.bigint() - t0) / 1e6);
    if (res.length !== 64 || !res.every((x) => x === 1)) throw new Error("lone call failed");
  }
  lat.sort((a, b) => a - b);
  out.lone_call_p50_ms = Number(lat[10].toFixed(3));
  out.all_valid = true;
  await v.close();
  out.closed = true;
  console.log(JSON.stringify(out));
  // exit here: Node 12 runs Node-API finalizers deferred at environment teardown on a disposed isolate
  // (segfault in node_napi_env__::CallFinalizer -> v8::HandleScope::Initialize, profiles/r06/jsexit);
  // everything this process measured or checked is printed and every context closed by now
  process.exit(0);
}

main().catch((e) => {
  console.log(JSON.stringify({fatal: String(e && e.stack ? e.stack : e)}));
  process.exitCode = 1;
});
