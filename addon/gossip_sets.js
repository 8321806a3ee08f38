// Gossip-side signature-set builders in index form, for the JavaScript GpuBlsVerifier
// (addon/gpu_bls_verifier.js) -- the same rules as lodestar_amd/gossip_sets.py, in the shape a Lodestar
// maintainer would put beside packages/beacon-node/src/chain/validation/signatureSets/:
//   aggregateAndProofSignatureSets   validateAggregateAndProof's three sets (aggregateAndProof.ts:211-229):
//                                    getSelectionProofSignatureSet (selectionProof.ts:7-27),
//                                    getAggregateAndProofSignatureSet (aggregateAndProof.ts:13-40; phase0 or
//                                    electra AggregateAndProof by the fork of the epoch start slot), and the
//                                    aggregate over its attesting indices (getAttestationDataSigningRoot,
//                                    attestation.ts:657-665)
//   contributionAndProofSignatureSets  syncCommitteeContributionAndProof.ts:73-92 (+ getContributionIndices :109-119)
//   syncCommitteeSignatureSets       syncCommittee.ts:10-23
// Sets come out as {index} / {indices} + signingRoot + signature.  Every container root is a tree of
// 32-byte nodes hashed on the device level by level (hasher.merkleRoots: gbv_merkle_roots, one launch
// per distinct subtree depth per level), the signing roots in one hasher.signingRoots call
// (gbv_signing_roots).  Domains (config constants) are computed once per fork with node's SHA-256, as
// the reference's config cache does (config/src/genesisConfig/index.ts:27-87,125-139).
"use strict";
const crypto = require("crypto");

const SLOTS_PER_EPOCH = 32;
const EPOCHS_PER_SYNC_COMMITTEE_PERIOD = 256;
const MAX_VALIDATORS_PER_COMMITTEE = 2048;
const MAX_COMMITTEES_PER_SLOT = 64;
const SYNC_COMMITTEE_SUBNET_SIZE = 128;
const FORK_ORDER = ["phase0", "altair", "bellatrix", "capella", "deneb", "electra"];
const DOMAIN = {
  BEACON_ATTESTER: [1, 0, 0, 0],
  SELECTION_PROOF: [5, 0, 0, 0],
  AGGREGATE_AND_PROOF: [6, 0, 0, 0],
  SYNC_COMMITTEE: [7, 0, 0, 0],
  SYNC_COMMITTEE_SELECTION_PROOF: [8, 0, 0, 0],
  CONTRIBUTION_AND_PROOF: [9, 0, 0, 0],
};

const sha256 = (b) => new Uint8Array(crypto.createHash("sha256").update(b).digest());
const cat = (...xs) => Uint8Array.from(Buffer.concat(xs.map((x) => Buffer.from(x))));

// ---- config: fork schedule and domains ------------------------------------------------------------
class BeaconConfig {
  /** forks: [{name, epoch, version: Uint8Array(4)}], gvr: Uint8Array(32) */
  constructor(forks, gvr) {
    this.forks = forks.slice().sort((a, b) => a.epoch - b.epoch);
    this.gvr = gvr;
    this.cache = new Map();
  }
  forkIndex(slot) {
    const epoch = Math.floor(slot / SLOTS_PER_EPOCH);
    let k = 0;
    this.forks.forEach((f, i) => {
      if (f.epoch <= epoch) k = i;
    });
    return k;
  }
  forkSeq(slot) {
    return FORK_ORDER.indexOf(this.forks[this.forkIndex(slot)].name);
  }
  domainOf(k, type) {
    const key = k + ":" + type.join(",");
    let d = this.cache.get(key);
    if (!d) {
      // computeDomain: type || hash_tree_root(ForkData{version, gvr})[0..28)
      const forkDataRoot = sha256(cat(this.forks[k].version, new Uint8Array(28), this.gvr));
      d = cat(Uint8Array.from(type), forkDataRoot.subarray(0, 28));
      this.cache.set(key, d);
    }
    return d;
  }
  /** getDomain(stateSlot, type, messageSlot) */
  getDomain(stateSlot, type, messageSlot) {
    const k = this.forkIndex(stateSlot);
    const epoch = Math.floor((messageSlot === undefined ? stateSlot : messageSlot) / SLOTS_PER_EPOCH);
    return this.domainOf(epoch < this.forks[k].epoch ? Math.max(k - 1, 0) : k, type);
  }
  /** getDomainAtFork(getForkName(slot), type) */
  getDomainAtForkOfSlot(slot, type) {
    return this.domainOf(this.forkIndex(slot), type);
  }
}

// ---- SSZ trees ---------------------------------------------------------------------------------------
class Node {
  constructor(children, depth) {
    this.children = children;
    let d = 0;
    while (1 << d < children.length) ++d;
    this.depth = depth === undefined ? d : depth;
  }
}
const u64 = (v) => {
  const b = new Uint8Array(32);
  let x = BigInt(v);
  for (let i = 0; i < 8; ++i, x >>= 8n) b[i] = Number(x & 0xffn);
  return b;
};
const chunks = (b) => {
  const out = [];
  for (let i = 0; i < b.length; i += 32) {
    const c = new Uint8Array(32);
    c.set(b.subarray(i, Math.min(i + 32, b.length)));
    out.push(c);
  }
  return out.length ? out : [new Uint8Array(32)];
};
const packBits = (bits) => {
  const out = new Uint8Array((bits.length + 7) >> 3);
  bits.forEach((bit, i) => {
    if (bit) out[i >> 3] |= 1 << (i & 7);
  });
  return out;
};
const bytesNode = (b) => new Node(chunks(b));
const bitvectorNode = (bits) => {
  const c = chunks(packBits(bits));
  return c.length === 1 ? c[0] : new Node(c);
};
const bitlistNode = (bits, limit) => {
  const chunkLimit = Math.ceil(limit / 256);
  let depth = 0;
  while (1 << depth < chunkLimit) ++depth;
  return new Node([new Node(bits.length ? chunks(packBits(bits)) : [], depth), u64(bits.length)]);
};
const checkpointNode = (c) => new Node([u64(c.epoch), c.root]);
const attestationDataNode = (d) => new Node([u64(d.slot), u64(d.index), d.beaconBlockRoot, checkpointNode(d.source), checkpointNode(d.target)]);
const attestationNode = (a, electra) =>
  electra
    ? new Node([bitlistNode(a.aggregationBits, MAX_VALIDATORS_PER_COMMITTEE * MAX_COMMITTEES_PER_SLOT), attestationDataNode(a.data),
      bytesNode(a.signature), bitvectorNode(a.committeeBits || new Array(MAX_COMMITTEES_PER_SLOT).fill(false))])
    : new Node([bitlistNode(a.aggregationBits, MAX_VALIDATORS_PER_COMMITTEE), attestationDataNode(a.data), bytesNode(a.signature)]);
const aggregateAndProofNode = (m, electra) => new Node([u64(m.aggregatorIndex), attestationNode(m.aggregate, electra), bytesNode(m.selectionProof)]);
const contributionNode = (c) =>
  new Node([u64(c.slot), c.beaconBlockRoot, u64(c.subcommitteeIndex), bitvectorNode(c.aggregationBits), bytesNode(c.signature)]);
const contributionAndProofNode = (m) => new Node([u64(m.aggregatorIndex), contributionNode(m.contribution), bytesNode(m.selectionProof)]);

/** Roots of many trees on the device, level by level (one merkleRoots launch per depth per level). */
function deviceRoots(hasher, trees) {
  const height = new Map();
  const order = [];
  const visit = (n) => {
    if (!(n instanceof Node)) return 0;
    if (height.has(n)) return height.get(n);
    let h = 0;
    for (const c of n.children) h = Math.max(h, visit(c) + 1);
    height.set(n, h);
    order.push(n);
    return h;
  };
  trees.forEach(visit);
  const memo = new Map();
  const levels = new Map();
  for (const n of order) {
    const h = height.get(n);
    if (!levels.has(h)) levels.set(h, []);
    levels.get(h).push(n);
  }
  for (const h of Array.from(levels.keys()).sort((a, b) => a - b)) {
    const byDepth = new Map();
    for (const n of levels.get(h)) {
      if (!byDepth.has(n.depth)) byDepth.set(n.depth, []);
      byDepth.get(n.depth).push(n);
    }
    for (const depth of Array.from(byDepth.keys()).sort((a, b) => a - b)) {
      const nodes = byDepth.get(depth);
      const blob = new Uint8Array(nodes.length * (32 << depth));
      nodes.forEach((n, i) => n.children.forEach((c, j) => blob.set(c instanceof Node ? memo.get(c) : c, i * (32 << depth) + 32 * j)));
      const roots = hasher.merkleRoots(blob, depth);
      nodes.forEach((n, i) => memo.set(n, roots.subarray(32 * i, 32 * i + 32)));
    }
  }
  return trees.map((t) => (t instanceof Node ? memo.get(t) : t));
}

/** pending: [{index | indices, signature, obj (tree or 32-byte root), domain}] -> index-form sets */
function resolve(pending, hasher) {
  const objs = deviceRoots(hasher, pending.map((p) => p.obj));
  const domains = [];
  const domOf = new Map();
  const idx = new Uint32Array(pending.length);
  pending.forEach((p, i) => {
    const key = Buffer.from(p.domain).toString("hex");
    if (!domOf.has(key)) {
      domOf.set(key, domains.length);
      domains.push(p.domain);
    }
    idx[i] = domOf.get(key);
  });
  const roots = pending.length ? hasher.signingRoots(cat(...objs), cat(...domains), idx) : new Uint8Array(0);
  return pending.map((p, i) => {
    const s = {signingRoot: roots.slice(32 * i, 32 * i + 32), signature: p.signature};
    if (p.indices) s.indices = Uint32Array.from(p.indices);
    else s.index = p.index;
    return s;
  });
}

const isElectra = (config, slot) => config.forkSeq(slot) >= FORK_ORDER.indexOf("electra");

/** signedAgg: {message: {aggregatorIndex, aggregate: {aggregationBits, data, signature, committeeBits?},
 * selectionProof}, signature}; attestingIndices from getIndexedAttestation */
function aggregateAndProofSignatureSets(config, signedAgg, attestingIndices, hasher) {
  const m = signedAgg.message;
  const slot = m.aggregate.data.slot;
  const epochStart = Math.floor(slot / SLOTS_PER_EPOCH) * SLOTS_PER_EPOCH;
  const targetStart = m.aggregate.data.target.epoch * SLOTS_PER_EPOCH;
  return resolve(
    [
      {index: m.aggregatorIndex, signature: m.selectionProof, obj: u64(slot), domain: config.getDomainAtForkOfSlot(slot, DOMAIN.SELECTION_PROOF)},
      {index: m.aggregatorIndex, signature: signedAgg.signature, obj: aggregateAndProofNode(m, isElectra(config, epochStart)),
        domain: config.getDomainAtForkOfSlot(epochStart, DOMAIN.AGGREGATE_AND_PROOF)},
      {indices: attestingIndices, signature: m.aggregate.signature, obj: attestationDataNode(m.aggregate.data),
        domain: config.getDomainAtForkOfSlot(targetStart, DOMAIN.BEACON_ATTESTER)},
    ],
    hasher
  );
}

/** getIndexedSyncCommittee(slot) over {slot, currentSyncCommittee, nextSyncCommittee?} */
function indexedSyncCommittee(state, slot) {
  const period = Math.floor(Math.floor((slot + 1) / SLOTS_PER_EPOCH) / EPOCHS_PER_SYNC_COMMITTEE_PERIOD);
  const own = Math.floor(Math.floor(state.slot / SLOTS_PER_EPOCH) / EPOCHS_PER_SYNC_COMMITTEE_PERIOD);
  if (period === own) return state.currentSyncCommittee;
  if (period === own + 1 && state.nextSyncCommittee) return state.nextSyncCommittee;
  throw Object.assign(new Error("NO_SYNC_COMMITTEE"), {code: "NO_SYNC_COMMITTEE"});
}

function contributionIndices(state, c) {
  const start = c.subcommitteeIndex * SYNC_COMMITTEE_SUBNET_SIZE;
  const sub = indexedSyncCommittee(state, c.slot).slice(start, start + SYNC_COMMITTEE_SUBNET_SIZE);
  if (sub.length !== c.aggregationBits.length) throw new Error("aggregation bits length mismatch");
  return sub.filter((v, i) => c.aggregationBits[i]);
}

/** state: {config, slot, currentSyncCommittee, nextSyncCommittee?} */
function contributionAndProofSignatureSets(state, signed, hasher) {
  const m = signed.message;
  const c = m.contribution;
  const participants = contributionIndices(state, c);
  if (participants.length === 0) throw Object.assign(new Error("NO_PARTICIPANT"), {code: "NO_PARTICIPANT"});
  const cfg = state.config;
  return resolve(
    [
      {index: m.aggregatorIndex, signature: m.selectionProof, obj: new Node([u64(c.slot), u64(c.subcommitteeIndex)]),
        domain: cfg.getDomain(state.slot, DOMAIN.SYNC_COMMITTEE_SELECTION_PROOF, c.slot)},
      {index: m.aggregatorIndex, signature: signed.signature, obj: contributionAndProofNode(m),
        domain: cfg.getDomain(state.slot, DOMAIN.CONTRIBUTION_AND_PROOF, c.slot)},
      {indices: participants, signature: c.signature, obj: c.beaconBlockRoot, domain: cfg.getDomain(state.slot, DOMAIN.SYNC_COMMITTEE, c.slot)},
    ],
    hasher
  );
}

function syncCommitteeSignatureSets(state, msgs, hasher) {
  return resolve(
    msgs.map((m) => ({index: m.validatorIndex, signature: m.signature, obj: m.beaconBlockRoot,
      domain: state.config.getDomain(state.slot, DOMAIN.SYNC_COMMITTEE, m.slot)})),
    hasher
  );
}

module.exports = {
  BeaconConfig,
  aggregateAndProofSignatureSets,
  contributionAndProofSignatureSets,
  syncCommitteeSignatureSets,
  contributionIndices,
  deviceRoots,
};
