// The gossip-side builders (addon/gossip_sets.js) against the oracle's fixture tests/golden/gossip_sets.json
// (tests/golden/make_gossip_fixture.py).  Used by tests/test_addon.py.
//   node addon/test_gossip.js cpu <fixture>   the builders' sets with a host SHA-256 stand-in for the device
//   node addon/test_gossip.js gpu <fixture>   device hashing through the addon, then every call -- and each
//                                             one-set corruption of it -- through GpuBlsVerifier
//                                             .verifySignatureSets(sets, {batchable: true, priority: true})
//                                             (aggregateAndProof.ts:229's call shape)
"use strict";
const path = require("path");
const fs = require("fs");
const crypto = require("crypto");
const G = require(path.join(__dirname, "gossip_sets.js"));
const V = require(path.join(__dirname, "gpu_bls_verifier.js"));

const hex = (h) => Uint8Array.from(Buffer.from(h, "hex"));
const toHex = (b) => Buffer.from(b).toString("hex");
const report = {};

class HostHasher {
  constructor() {
    this.calls = [];
  }
  static sha(b) {
    return new Uint8Array(crypto.createHash("sha256").update(b).digest());
  }
  merkleRoots(chunks, depth) {
    this.calls.push(["merkle", depth]);
    const w = 32 << depth;
    const out = new Uint8Array(chunks.length / w * 32);
    for (let o = 0; o < chunks.length / w; ++o) {
      let layer = [];
      for (let k = 0; k < 1 << depth; ++k) layer.push(chunks.subarray(o * w + 32 * k, o * w + 32 * k + 32));
      while (layer.length > 1) {
        const next = [];
        for (let i = 0; i < layer.length; i += 2) next.push(HostHasher.sha(Buffer.concat([Buffer.from(layer[i]), Buffer.from(layer[i + 1])])));
        layer = next;
      }
      out.set(layer[0], 32 * o);
    }
    return out;
  }
  signingRoots(roots, domains, idx) {
    this.calls.push(["signing", roots.length / 32]);
    const out = new Uint8Array(roots.length);
    for (let i = 0; i < roots.length / 32; ++i) {
      const d = idx ? idx[i] : 0;
      out.set(HostHasher.sha(Buffer.concat([Buffer.from(roots.subarray(32 * i, 32 * i + 32)), Buffer.from(domains.subarray(32 * d, 32 * d + 32))])), 32 * i);
    }
    return out;
  }
}

function world(fix) {
  const cfg = fix.config;
  const config = new G.BeaconConfig(cfg.forks.map(([name, epoch, v]) => ({name, epoch, version: hex(v)})), hex(cfg.gvr));
  const state = {config, slot: fix.state_slot, currentSyncCommittee: fix.sync_committee, nextSyncCommittee: fix.next_sync_committee};
  return {config, state};
}

const dataOf = (d) => ({slot: d.slot, index: d.index, beaconBlockRoot: hex(d.beacon_block_root), source: {epoch: d.source_epoch, root: hex(d.source_root)},
  target: {epoch: d.target_epoch, root: hex(d.target_root)}});

function build(fix, call, hasher) {
  const {config, state} = world(fix);
  if (call.kind === "aggregate_and_proof") {
    const m = call.signed.message;
    const a = m.aggregate;
    const signed = {message: {aggregatorIndex: m.aggregator_index, selectionProof: hex(m.selection_proof),
      aggregate: {aggregationBits: a.bits, data: dataOf(a.data), signature: hex(a.signature), committeeBits: a.committee_bits}}, signature: hex(call.signed.signature)};
    return G.aggregateAndProofSignatureSets(config, signed, call.attesting_indices, hasher);
  }
  if (call.kind === "contribution_and_proof") {
    const m = call.signed.message;
    const c = m.contribution;
    const signed = {message: {aggregatorIndex: m.aggregator_index, selectionProof: hex(m.selection_proof),
      contribution: {slot: c.slot, beaconBlockRoot: hex(c.beacon_block_root), subcommitteeIndex: c.subcommittee_index, aggregationBits: c.bits,
        signature: hex(c.signature)}}, signature: hex(call.signed.signature)};
    return G.contributionAndProofSignatureSets(state, signed, hasher);
  }
  const m = call.message;
  return G.syncCommitteeSignatureSets(state, [{slot: m.slot, beaconBlockRoot: hex(m.beacon_block_root), validatorIndex: m.validator_index,
    signature: hex(m.signature)}], hasher);
}

function matches(sets, call) {
  return sets.length === call.expected_sets.length && sets.every((s, i) => {
    const e = call.expected_sets[i];
    const key = s.indices ? Array.from(s.indices) : s.index;
    return toHex(s.signingRoot) === e.root && JSON.stringify(key) === JSON.stringify(e.key) && (e.kind === "aggregate") === !!s.indices;
  });
}

async function main() {
  const mode = process.argv[2];
  const fix = JSON.parse(fs.readFileSync(process.argv[3]));
  if (mode === "cpu") {
    report.builders = fix.calls.map((call) => {
      const h = new HostHasher();
      const sets = build(fix, call, h);
      return matches(sets, call) && h.calls.filter((c) => c[0] === "signing").length === 1;
    });
    return;
  }
  const addon = require(path.join(__dirname, "gbv_addon.node"));
  const v = new V.GpuBlsVerifier({addon});
  const pks = fix.pubkeys.map(hex);
  const n = fix.world.n_validators;
  const all = new Uint8Array(48 * n);
  for (let i = 0; i < n; ++i) all.set(pks[i % pks.length], 48 * i);
  const st = v.addPubkeys(0, all, true);
  report.ingest = st.every((x) => x === 0);
  report.deviceBuilders = [];
  report.calls = [];
  const pending = [];
  for (const call of fix.calls) {
    const sets = build(fix, call, v);
    report.deviceBuilders.push(matches(sets, call));
    const want = [call.expected_valid].concat(call.corruptions.map((c) => c.expected_valid));
    const variants = [sets].concat(call.corruptions.map((c) => sets.map((s, i) => (i === c.set ? Object.assign({}, s, {signature: hex(c.signature)}) : s))));
    // every variant at once: the queue buffers them (batchable) and they share device passes
    pending.push(Promise.all(variants.map((ss) => v.verifySignatureSets(ss, {batchable: true, priority: true}))).then(
      (got) => JSON.stringify(got) === JSON.stringify(want)));
  }
  report.calls = await Promise.all(pending);
  report.devicePasses = v.devicePasses;
  await v.close();
}

main()
  .catch((e) => {
    report.fatal = String(e && e.stack ? e.stack : e);
  })
  .then(() => {
    console.log(JSON.stringify(report));
    process.exit(0);  // Node 12's teardown finalizer crash: see bench_api.js
  });
