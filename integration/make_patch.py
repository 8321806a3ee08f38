#!/usr/bin/env python3
"""Write integration/lodestar-gpu-bls.patch: the exact edit a Lodestar maintainer applies to
cjustinobi/lodestar (packages/, reference @ 2025-01-31) to run IBlsVerifier on the MI355X through this
repo's Node-API addon.  Run in a container that holds the reference checkout:

    python3 integration/make_patch.py [/root/reference]

It copies the touched reference files into a scratch tree, applies the edits below as exact string
replacements (each must match once, so a drifted reference fails loudly), adds the new files, and
writes `diff -ruN` of the two trees.  The patch applies with `patch -p1` from the reference root
(tests/test_integration_patch.py checks that, and that every hunk lands).  It does not compile here:
tsc / Node >= 20 are absent.

What it changes:
  * state-transition: ISignatureSet carries the validator indices beside the PublicKey objects
    (SingleSignatureSet.index, AggregatedSignatureSet.indices); every builder that reads index2pubkey
    fills them (randao, proposer, proposer / attester slashings, attestations, exits, sync aggregate);
    index2pubkey growth is announced to listeners (syncPubkeys, addFinalizedPubkey);
  * beacon-node: the sync-committee gossip builders that read index2pubkey (sync committee message,
    contribution, sync selection proof) fill the index; a new chain option selects GpuBlsVerifier
    (chain/bls/gpu/index.ts, over addon/gpu_bls_verifier.js + gbv_addon.node, copied beside it), which
    mirrors index2pubkey in HBM and finds any other key object's index by its identity.
  * callers of IBlsVerifier are not edited (no file of chain/validation/ outside signatureSets/, and
    not chain/bls/interface.ts): the same-message call keeps the interface's {publicKey, signature}.
"""
import os
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "lodestar-gpu-bls.patch")
ST = "packages/state-transition/src/"
BN = "packages/beacon-node/src/"

EDITS = {
    ST + "util/signatureSets.ts": [
        ('import {Root} from "@lodestar/types";', 'import {Root, ValidatorIndex} from "@lodestar/types";'),
        ("""export type SingleSignatureSet = {
  type: SignatureSetType.single;
  pubkey: PublicKey;
  signingRoot: Root;
  signature: Uint8Array;
};""", """export type SingleSignatureSet = {
  type: SignatureSetType.single;
  pubkey: PublicKey;
  /** Index of `pubkey` in index2pubkey, when it comes from there: GpuBlsVerifier reads the key from its
   * HBM copy of the table instead of the object */
  index?: ValidatorIndex;
  signingRoot: Root;
  signature: Uint8Array;
};"""),
        ("""export type AggregatedSignatureSet = {
  type: SignatureSetType.aggregate;
  pubkeys: PublicKey[];
  signingRoot: Root;
  signature: Uint8Array;
};""", """export type AggregatedSignatureSet = {
  type: SignatureSetType.aggregate;
  pubkeys: PublicKey[];
  /** Indices of `pubkeys` in index2pubkey (same order), when they come from there */
  indices?: ValidatorIndex[];
  signingRoot: Root;
  signature: Uint8Array;
};"""),
        ("""export function createSingleSignatureSetFromComponents(
  pubkey: PublicKey,
  signingRoot: Root,
  signature: Uint8Array
): SingleSignatureSet {
  return {
    type: SignatureSetType.single,
    pubkey,
    signingRoot,
    signature,
  };
}""", """export function createSingleSignatureSetFromComponents(
  pubkey: PublicKey,
  signingRoot: Root,
  signature: Uint8Array,
  index?: ValidatorIndex
): SingleSignatureSet {
  return {
    type: SignatureSetType.single,
    pubkey,
    index,
    signingRoot,
    signature,
  };
}"""),
        ("""export function createAggregateSignatureSetFromComponents(
  pubkeys: PublicKey[],
  signingRoot: Root,
  signature: Uint8Array
): AggregatedSignatureSet {
  return {
    type: SignatureSetType.aggregate,
    pubkeys,
    signingRoot,
    signature,
  };
}""", """export function createAggregateSignatureSetFromComponents(
  pubkeys: PublicKey[],
  signingRoot: Root,
  signature: Uint8Array,
  indices?: ValidatorIndex[]
): AggregatedSignatureSet {
  return {
    type: SignatureSetType.aggregate,
    pubkeys,
    indices,
    signingRoot,
    signature,
  };
}

/** An aggregate set over validators of index2pubkey, in both forms (objects for blst, indices for the GPU) */
export function createAggregateSignatureSetFromIndices(
  index2pubkey: PublicKey[],
  indices: ValidatorIndex[],
  signingRoot: Root,
  signature: Uint8Array
): AggregatedSignatureSet {
  return createAggregateSignatureSetFromComponents(
    indices.map((i) => index2pubkey[i]),
    signingRoot,
    signature,
    indices
  );
}"""),
    ],
    ST + "signatureSets/randao.ts": [
        ("""    pubkey: epochCtx.index2pubkey[block.proposerIndex],
""", """    pubkey: epochCtx.index2pubkey[block.proposerIndex],
    index: block.proposerIndex,
"""),
    ],
    ST + "signatureSets/proposer.ts": [
        ("""    pubkey: epochCtx.index2pubkey[signedBlock.message.proposerIndex],
""", """    pubkey: epochCtx.index2pubkey[signedBlock.message.proposerIndex],
    index: signedBlock.message.proposerIndex,
"""),
        ("""    pubkey: epochCtx.index2pubkey[signedBlockHeader.message.proposerIndex],
""", """    pubkey: epochCtx.index2pubkey[signedBlockHeader.message.proposerIndex],
    index: signedBlockHeader.message.proposerIndex,
"""),
    ],
    ST + "signatureSets/proposerSlashings.ts": [
        ("""  const pubkey = epochCtx.index2pubkey[proposerSlashing.signedHeader1.message.proposerIndex];
""", """  const index = proposerSlashing.signedHeader1.message.proposerIndex;
  const pubkey = epochCtx.index2pubkey[index];
"""),
        ("""      type: SignatureSetType.single,
      pubkey,
""", """      type: SignatureSetType.single,
      pubkey,
      index,
"""),
    ],
    ST + "signatureSets/attesterSlashings.ts": [
        ("""    pubkeys: indexedAttestation.attestingIndices.map((i) => state.epochCtx.index2pubkey[i]),
""", """    pubkeys: indexedAttestation.attestingIndices.map((i) => state.epochCtx.index2pubkey[i]),
    indices: indexedAttestation.attestingIndices,
"""),
    ],
    ST + "signatureSets/indexedAttestation.ts": [
        ("""  createAggregateSignatureSetFromComponents,
} from "../util/index.js";""", """  createAggregateSignatureSetFromIndices,
} from "../util/index.js";"""),
        ("""  return createAggregateSignatureSetFromComponents(
    attestingIndices.map((i) => state.epochCtx.index2pubkey[i]),
    getAttestationDataSigningRoot(state, attestation.data),""", """  return createAggregateSignatureSetFromIndices(
    state.epochCtx.index2pubkey,
    attestingIndices,
    getAttestationDataSigningRoot(state, attestation.data),"""),
    ],
    ST + "signatureSets/voluntaryExits.ts": [
        ("""    pubkey: epochCtx.index2pubkey[signedVoluntaryExit.message.validatorIndex],
""", """    pubkey: epochCtx.index2pubkey[signedVoluntaryExit.message.validatorIndex],
    index: signedVoluntaryExit.message.validatorIndex,
"""),
    ],
    ST + "block/processSyncCommittee.ts": [
        ("""    pubkeys: participantIndices.map((i) => epochCtx.index2pubkey[i]),
""", """    pubkeys: participantIndices.map((i) => epochCtx.index2pubkey[i]),
    indices: participantIndices,
"""),
    ],
    ST + "cache/pubkeyCache.ts": [
        ("""export type Index2PubkeyCache = PublicKey[];""", """export type Index2PubkeyCache = PublicKey[];

/**
 * Called with (first index, compressed keys, the new PublicKey objects) whenever index2pubkey gains
 * entries (syncPubkeys, EpochCache.addFinalizedPubkey): GpuBlsVerifier keeps a copy of the table in GPU
 * memory and finds a key object's index by its identity.
 */
export type Index2PubkeyListener = (firstIndex: ValidatorIndex, pubkeys: Uint8Array[], keys: PublicKey[]) => void;
export const index2pubkeyListeners = new Set<Index2PubkeyListener>();"""),
        ("""  const newCount = validators.length;
  index2pubkey.length = newCount;
  for (let i = pubkey2index.size; i < newCount; i++) {
    const pubkey = validators[i].pubkey;""", """  const newCount = validators.length;
  const firstNew = pubkey2index.size;
  const added: Uint8Array[] | null = index2pubkeyListeners.size > 0 ? [] : null;
  index2pubkey.length = newCount;
  for (let i = pubkey2index.size; i < newCount; i++) {
    const pubkey = validators[i].pubkey;
    added?.push(pubkey);"""),
        ("""    index2pubkey[i] = PublicKey.fromBytes(pubkey); // Optimize for aggregation
  }
}""", """    index2pubkey[i] = PublicKey.fromBytes(pubkey); // Optimize for aggregation
  }
  if (added && added.length > 0) {
    const keys = index2pubkey.slice(firstNew, newCount);
    for (const listener of index2pubkeyListeners) listener(firstNew, added, keys);
  }
}"""),
    ],
    ST + "cache/epochCache.ts": [
        ("""  UnfinalizedPubkeyIndexMap,
  newUnfinalizedPubkeyIndexMap,
  syncPubkeys,
  toMemoryEfficientHexStr,
} from "./pubkeyCache.js";""", """  UnfinalizedPubkeyIndexMap,
  index2pubkeyListeners,
  newUnfinalizedPubkeyIndexMap,
  syncPubkeys,
  toMemoryEfficientHexStr,
} from "./pubkeyCache.js";"""),
        ("""    this.index2pubkey[index] = PublicKey.fromBytes(pubkeyBytes); // Optimize for aggregation
  }""", """    this.index2pubkey[index] = PublicKey.fromBytes(pubkeyBytes); // Optimize for aggregation
    for (const listener of index2pubkeyListeners) listener(index, [pubkeyBytes], [this.index2pubkey[index]]);
  }"""),
    ],
    ST + "index.ts": [
        ("""export {
  type Index2PubkeyCache,
  type UnfinalizedPubkeyIndexMap,
  newUnfinalizedPubkeyIndexMap,
} from "./cache/pubkeyCache.js";""", """export {
  type Index2PubkeyCache,
  type Index2PubkeyListener,
  type UnfinalizedPubkeyIndexMap,
  index2pubkeyListeners,
  newUnfinalizedPubkeyIndexMap,
} from "./cache/pubkeyCache.js";"""),
    ],
    BN + "chain/bls/index.ts": [
        ("""export {BlsSingleThreadVerifier} from "./singleThread.js";""", """export {BlsSingleThreadVerifier} from "./singleThread.js";
export {GpuBlsVerifier} from "./gpu/index.js";"""),
    ],
    BN + "chain/options.ts": [
        ("""    blsVerifyAllMainThread?: boolean;
""", """    blsVerifyAllMainThread?: boolean;
    /** Verify every BLS signature set on an MI355X GPU (chain/bls/gpu, include/gbv.h) */
    blsVerifyOnGpu?: boolean;
    /** HIP device of this beacon node (one process per GPU) */
    blsGpuDevice?: number;
"""),
        ("""  blsVerifyAllMainThread: false,
  blsVerifyAllMultiThread: false,""", """  blsVerifyAllMainThread: false,
  blsVerifyOnGpu: false,
  blsGpuDevice: 0,
  blsVerifyAllMultiThread: false,"""),
    ],
    BN + "chain/chain.ts": [
        ("""import {BlsMultiThreadWorkerPool, BlsSingleThreadVerifier, IBlsVerifier} from "./bls/index.js";""",
         """import {BlsMultiThreadWorkerPool, BlsSingleThreadVerifier, GpuBlsVerifier, IBlsVerifier} from "./bls/index.js";"""),
        ("""    const bls = opts.blsVerifyAllMainThread
      ? new BlsSingleThreadVerifier({metrics})
      : new BlsMultiThreadWorkerPool(opts, {logger, metrics});""", """    const bls = opts.blsVerifyOnGpu
      ? new GpuBlsVerifier(opts, {logger, metrics})
      : opts.blsVerifyAllMainThread
        ? new BlsSingleThreadVerifier({metrics})
        : new BlsMultiThreadWorkerPool(opts, {logger, metrics});"""),
        ("""    this.index2pubkey = cachedState.epochCtx.index2pubkey;
""", """    this.index2pubkey = cachedState.epochCtx.index2pubkey;
    // the GPU verifier's HBM copy of index2pubkey: the keys known now, then every later addition
    // (index2pubkeyListeners)
    if (bls instanceof GpuBlsVerifier) bls.loadIndex2pubkey(this.index2pubkey);
"""),
    ],
    BN + "chain/validation/signatureSets/syncCommittee.ts": [
        ("""    pubkey: state.epochCtx.index2pubkey[syncCommittee.validatorIndex],
""", """    pubkey: state.epochCtx.index2pubkey[syncCommittee.validatorIndex],
    index: syncCommittee.validatorIndex,
"""),
    ],
    BN + "chain/validation/signatureSets/contributionAndProof.ts": [
        ("""    pubkey: epochCtx.index2pubkey[signedContributionAndProof.message.aggregatorIndex],
""", """    pubkey: epochCtx.index2pubkey[signedContributionAndProof.message.aggregatorIndex],
    index: signedContributionAndProof.message.aggregatorIndex,
"""),
    ],
    BN + "chain/validation/signatureSets/syncCommitteeSelectionProof.ts": [
        ("""    pubkey: epochCtx.index2pubkey[contributionAndProof.aggregatorIndex],
""", """    pubkey: epochCtx.index2pubkey[contributionAndProof.aggregatorIndex],
    index: contributionAndProof.aggregatorIndex,
"""),
    ],
}

GPU_INDEX_TS = '''/**
 * GpuBlsVerifier: IBlsVerifier on an MI355X GPU (HIP kernels for gfx950 behind the C ABI include/gbv.h of
 * the lodestar_amd build).  Ships with two files copied from that build into this directory:
 *   gbv_addon.node        the Node-API addon (addon/gbv_addon.c), linked to libgbv.so
 *   gpu_bls_verifier.js   the job queue over the addon (addon/gpu_bls_verifier.js): the same chunking,
 *                         batchable buffering, priority, canAcceptWork and close() semantics as
 *                         BlsMultiThreadWorkerPool (multithread/index.ts), with up to 3 passes on the device.
 * Signature sets are handed over in index form: the validator indices the builders put in
 * ISignatureSet.index / .indices, or else the index of the set's PublicKey object in index2pubkey (the
 * queue keeps index2pubkey's objects in an identity map, filled here and by index2pubkeyListeners),
 * select keys from the GPU's copy of index2pubkey; a key outside the table (e.g. a BLS-to-execution
 * change's) passes its compressed bytes.  Callers are not edited: verifySignatureSetsSameMessage takes
 * the interface's {publicKey, signature} sets as validation/attestation.ts hands them.
 */
import {createRequire} from "node:module";
import {PublicKey, aggregatePublicKeys} from "@chainsafe/blst";
import {ISignatureSet, Index2PubkeyCache, SignatureSetType, index2pubkeyListeners} from "@lodestar/state-transition";
import {Logger} from "@lodestar/utils";
import {Metrics} from "../../../metrics/index.js";
import {IBlsVerifier, VerifySignatureOpts} from "../interface.js";

type IndexFormSet =
  | {index: number; signingRoot: Uint8Array; signature: Uint8Array}
  | {indices: number[]; signingRoot: Uint8Array; signature: Uint8Array}
  | {pubkey: Uint8Array; signingRoot: Uint8Array; signature: Uint8Array};

/** keys per addPubkeys call when the whole table is loaded */
const LOAD_BATCH = 1 << 16;

/** the job queue of gpu_bls_verifier.js (its GpuBlsVerifier class) as this binding uses it */
interface GpuQueue {
  addPubkeys(firstIndex: number, pk48s: Uint8Array, validate: boolean): Uint8Array;
  registerPubkeyObjects(firstIndex: number, keys: PublicKey[]): void;
  indexOf(publicKey: PublicKey): number | undefined;
  indicesOf(publicKeys: PublicKey[]): number[] | undefined;
  canAcceptWork(): boolean;
  verifySignatureSets(sets: IndexFormSet[], opts: VerifySignatureOpts): Promise<boolean>;
  verifySameMessageSets(
    sets: {publicKey: PublicKey; signature: Uint8Array}[],
    message: Uint8Array,
    opts: Omit<VerifySignatureOpts, "verifyOnMainThread">
  ): Promise<boolean[]>;
  close(): Promise<void>;
}

export class GpuBlsVerifier implements IBlsVerifier {
  private readonly queue: GpuQueue;
  private readonly logger: Logger;
  private readonly onNewPubkeys = (firstIndex: number, pubkeys: Uint8Array[], keys: PublicKey[]): void => {
    this.queue.addPubkeys(firstIndex, Buffer.concat(pubkeys), false);
    this.queue.registerPubkeyObjects(firstIndex, keys);
  };

  constructor(opts: {blsGpuDevice?: number}, modules: {logger: Logger; metrics: Metrics | null}) {
    this.logger = modules.logger;
    // The native addon and its queue load here, when a node is started with --chain.blsVerifyOnGpu,
    // never at import time: chain/bls re-exports this class, and this package is an ES module.
    const require = createRequire(import.meta.url);
    const addon = require("./gbv_addon.node");
    const {GpuBlsVerifier: QueueOverAddon, nodeMetricFamilies} = require("./gpu_bls_verifier.js");
    // the queue feeds the node's lodestar_bls_thread_pool_* families (metrics/lodestar.ts:401-504) and
    // two *_gpu_* ones registered on metrics.register; queue length / busy passes are read at scrape time
    this.queue = new QueueOverAddon({addon, device: opts.blsGpuDevice ?? 0, metrics: nodeMetricFamilies(modules.metrics)});
    index2pubkeyListeners.add(this.onNewPubkeys);
  }

  /** Copy the keys index2pubkey holds now into GPU memory (later additions arrive through
   * index2pubkeyListeners).  The keys were validated on deposit (processDeposit.ts:163-166). */
  loadIndex2pubkey(index2pubkey: Index2PubkeyCache): void {
    for (let first = 0; first < index2pubkey.length; first += LOAD_BATCH) {
      const objs = index2pubkey.slice(first, first + LOAD_BATCH);
      this.queue.addPubkeys(first, Buffer.concat(objs.map((pk) => pk.toBytes())), false);
      this.queue.registerPubkeyObjects(first, objs);
    }
    this.logger.info("GPU BLS verifier: index2pubkey loaded", {validators: index2pubkey.length});
  }

  canAcceptWork(): boolean {
    return this.queue.canAcceptWork();
  }

  async verifySignatureSets(sets: ISignatureSet[], opts: VerifySignatureOpts = {}): Promise<boolean> {
    return this.queue.verifySignatureSets(
      sets.map((set) => toIndexForm(set, this.queue)),
      opts
    );
  }

  /** validation/attestation.ts:134-137 hands one {publicKey, signature} per set, publicKey being
   * index2pubkey[validatorIndex]: the queue finds each index by the object's identity and packs the call
   * into the pass-wide index / signature buffers of the addon; a key outside the table is verified from
   * its bytes */
  async verifySignatureSetsSameMessage(
    sets: {publicKey: PublicKey; signature: Uint8Array}[],
    message: Uint8Array,
    opts: Omit<VerifySignatureOpts, "verifyOnMainThread"> = {}
  ): Promise<boolean[]> {
    return this.queue.verifySameMessageSets(sets, message, opts);
  }

  async close(): Promise<void> {
    index2pubkeyListeners.delete(this.onNewPubkeys);
    await this.queue.close();
  }
}

function toIndexForm(set: ISignatureSet, queue: GpuQueue): IndexFormSet {
  const {signingRoot, signature} = set;
  if (set.type === SignatureSetType.single) {
    const index = set.index ?? queue.indexOf(set.pubkey);
    return index !== undefined ? {index, signingRoot, signature} : {pubkey: set.pubkey.toBytes(), signingRoot, signature};
  }
  const indices = set.indices ?? queue.indicesOf(set.pubkeys);
  if (indices !== undefined) return {indices, signingRoot, signature};
  // an aggregate built from keys outside index2pubkey: hand the aggregate key over (validated on the device)
  return {pubkey: aggregatePublicKeys(set.pubkeys).toBytes(), signingRoot, signature};
}
'''

NEW_FILES = {BN + "chain/bls/gpu/index.ts": GPU_INDEX_TS}


def main(ref):
    work = tempfile.mkdtemp(prefix="lodestar-patch-")
    a, b = os.path.join(work, "a"), os.path.join(work, "b")
    try:
        for rel, edits in EDITS.items():
            src = os.path.join(ref, rel)
            for root in (a, b):
                os.makedirs(os.path.dirname(os.path.join(root, rel)), exist_ok=True)
                shutil.copyfile(src, os.path.join(root, rel))
            text = open(src).read()
            for old, new in edits:
                if text.count(old) != 1:
                    raise SystemExit("%s: edit anchor found %d times:\n%s" % (rel, text.count(old), old))
                text = text.replace(old, new)
            open(os.path.join(b, rel), "w").write(text)
        for rel, text in NEW_FILES.items():
            os.makedirs(os.path.dirname(os.path.join(b, rel)), exist_ok=True)
            open(os.path.join(b, rel), "w").write(text)
        p = subprocess.run(["diff", "-ruN", "a", "b"], cwd=work, capture_output=True, text=True)
        if p.returncode not in (0, 1):
            raise SystemExit(p.stderr)
        header = ("# Lodestar (cjustinobi/lodestar @ 2025-01-31): run IBlsVerifier on an MI355X GPU.\n"
                  "# Generated by integration/make_patch.py; apply from the repository root with `patch -p1`.\n"
                  "# Copy addon/gbv_addon.node and addon/gpu_bls_verifier.js of the lodestar_amd build into\n"
                  "# packages/beacon-node/src/chain/bls/gpu/ and start the node with --chain.blsVerifyOnGpu.\n")
        # drop the file timestamps so the patch is the same on every run
        body = "\n".join(l.split("\t")[0] if l.startswith(("--- ", "+++ ")) else l for l in p.stdout.split("\n"))
        open(OUT, "w").write(header + body)
        print("wrote", OUT, len(p.stdout.splitlines()), "lines,", len(EDITS), "files edited,", len(NEW_FILES), "added")
    finally:
        shutil.rmtree(work)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
