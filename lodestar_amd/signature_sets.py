"""Index-form signature-set builders: getBlockSignatureSets and its sub-builders.

Reference: packages/state-transition/src/signatureSets/index.ts:26-73 (getBlockSignatureSets) with
  randao.ts:19-31, proposer.ts:15-32, proposerSlashings.ts:9-41, attesterSlashings.ts:7-39,
  indexedAttestation.ts:21-51, voluntaryExits.ts:21-44, blsToExecutionChange.ts:19-44 and
  block/processSyncCommittee.ts:59-111 (getSyncCommitteeSignatureSet); domains from
  config/src/genesisConfig/index.ts:27-87 (getDomain, getDomainAtFork, getDomainForVoluntaryExit)
  and computeSigningRoot, state-transition/src/util/signingRoot.ts:7-13.

The builders emit the same sets in the same order as the reference, with one change SURVEY.md
8(a) a11/a12 asks for: pubkeys are validator indices into the HBM-resident index2pubkey table
(SingleSignatureSet.index / AggregatedSignatureSet.indices), except BLS-to-execution changes whose key
comes from the message itself (raw 48 bytes, validated like PublicKey.fromBytes(pk, true)).

Hashing: the small object roots (an epoch, a block header, an exit, a BLS change) are hashed here
with hashlib, as the reference hashes them on its host; every AttestationData root and every
signing root (SigningData{object_root, domain}) is computed on the device in two batched calls
(gbv_attestation_signing_roots, gbv_signing_roots) through the ``hasher`` -- a GpuBlsVerifier.

Attesting indices (epochCache.ts:938-973): before electra the committee of (data.slot, data.index)
intersected with the aggregation bits; from electra on the committees named by ``committee_bits``
(getBeaconCommittees, epochCache.ts:813-849), concatenated in committee order and intersected with
the aggregation bits that span all of them -- up to MAX_COMMITTEES_PER_SLOT = 64 committees, i.e.
aggregates of tens of thousands of pubkeys, which k_vs_agg_big sums on the device.
``BeaconBlock.body_root`` is the hash_tree_root of the block body, which the block-import pipeline
computes anyway; the execution payload and the rest of the body are not re-hashed here.
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

from .verifier import AggregatedSignatureSet, ISignatureSet, SingleSignatureSet

SLOTS_PER_EPOCH = 32                      # params/src/presets/mainnet.ts:38
MAX_COMMITTEES_PER_SLOT = 64              # presets/mainnet.ts:10
FORK_ORDER = ("phase0", "altair", "bellatrix", "capella", "deneb", "electra")  # ForkSeq (params/src/forkName.ts)
SYNC_COMMITTEE_SIZE = 512                 # presets/mainnet.ts:90
DOMAIN_BEACON_PROPOSER = bytes([0, 0, 0, 0])      # params/src/index.ts:139-149
DOMAIN_BEACON_ATTESTER = bytes([1, 0, 0, 0])
DOMAIN_RANDAO = bytes([2, 0, 0, 0])
DOMAIN_DEPOSIT = bytes([3, 0, 0, 0])
DOMAIN_VOLUNTARY_EXIT = bytes([4, 0, 0, 0])
DOMAIN_SELECTION_PROOF = bytes([5, 0, 0, 0])
DOMAIN_AGGREGATE_AND_PROOF = bytes([6, 0, 0, 0])
DOMAIN_SYNC_COMMITTEE = bytes([7, 0, 0, 0])
DOMAIN_BLS_TO_EXECUTION_CHANGE = bytes([10, 0, 0, 0])
G2_POINT_AT_INFINITY = bytes([0xC0]) + bytes(95)  # state-transition/src/constants/constants.ts:5


# ---- SSZ hash_tree_root of the small containers the builders sign -------------------------------
def _sha(b: bytes) -> bytes:
    return hashlib.sha256(b).digest()


def _merkleize(chunks: Sequence[bytes]) -> bytes:
    """Binary Merkle root, zero-padded to the next power of two (consensus-spec merkleize)."""
    layer = list(chunks) or [bytes(32)]
    n = 1
    while n < len(layer):
        n *= 2
    layer += [bytes(32)] * (n - len(layer))
    while len(layer) > 1:
        layer = [_sha(layer[i] + layer[i + 1]) for i in range(0, len(layer), 2)]
    return layer[0]


def _u64(v: int) -> bytes:
    return int(v).to_bytes(8, "little") + bytes(24)


def _bytes_root(b: bytes) -> bytes:
    """hash_tree_root of a ByteVector: packed into 32-byte chunks, zero padded."""
    b = bytes(b)
    chunks = [b[i:i + 32].ljust(32, b"\0") for i in range(0, len(b), 32)] or [bytes(32)]
    return _merkleize(chunks)


def compute_fork_data_root(current_version: bytes, genesis_validators_root: bytes) -> bytes:
    """computeForkDataRoot (config/src/genesisConfig/index.ts:133-139)."""
    return _merkleize([bytes(current_version).ljust(32, b"\0"), bytes(genesis_validators_root)])


def compute_domain(domain_type: bytes, fork_version: bytes, genesis_validators_root: bytes) -> bytes:
    """computeDomain (config/src/genesisConfig/index.ts:125-131)."""
    return bytes(domain_type) + compute_fork_data_root(fork_version, genesis_validators_root)[:28]


def compute_start_slot_at_epoch(epoch: int) -> int:
    return epoch * SLOTS_PER_EPOCH


def compute_epoch_at_slot(slot: int) -> int:
    return slot // SLOTS_PER_EPOCH


# ---- containers (the fields the signature sets read) -------------------------------------------
@dataclass
class Checkpoint:
    epoch: int
    root: bytes


@dataclass
class AttestationData:
    """phase0 AttestationData (types/src/phase0/sszTypes.ts:247-256)."""
    slot: int
    index: int
    beacon_block_root: bytes
    source: Checkpoint
    target: Checkpoint

    def serialize(self) -> bytes:
        """128-byte SSZ serialisation (the device hashes this into the object root)."""
        return (int(self.slot).to_bytes(8, "little") + int(self.index).to_bytes(8, "little") + bytes(self.beacon_block_root)
                + int(self.source.epoch).to_bytes(8, "little") + bytes(self.source.root)
                + int(self.target.epoch).to_bytes(8, "little") + bytes(self.target.root))


@dataclass
class Attestation:
    """phase0 Attestation, or electra's (types/src/electra/sszTypes.ts) when committee_bits is set:
    aggregation_bits then span the committees named by committee_bits, data.index is 0."""
    aggregation_bits: Sequence[bool]
    data: AttestationData
    signature: bytes
    committee_bits: Optional[Sequence[bool]] = None


@dataclass
class IndexedAttestation:
    attesting_indices: Sequence[int]
    data: AttestationData
    signature: bytes


@dataclass
class BeaconBlockHeader:
    slot: int
    proposer_index: int
    parent_root: bytes
    state_root: bytes
    body_root: bytes

    def hash_tree_root(self) -> bytes:
        return _merkleize([_u64(self.slot), _u64(self.proposer_index), bytes(self.parent_root), bytes(self.state_root),
                           bytes(self.body_root)])


@dataclass
class SignedBeaconBlockHeader:
    message: BeaconBlockHeader
    signature: bytes


@dataclass
class ProposerSlashing:
    signed_header_1: SignedBeaconBlockHeader
    signed_header_2: SignedBeaconBlockHeader


@dataclass
class AttesterSlashing:
    attestation_1: IndexedAttestation
    attestation_2: IndexedAttestation


@dataclass
class VoluntaryExit:
    epoch: int
    validator_index: int

    def hash_tree_root(self) -> bytes:
        return _merkleize([_u64(self.epoch), _u64(self.validator_index)])


@dataclass
class SignedVoluntaryExit:
    message: VoluntaryExit
    signature: bytes


@dataclass
class BLSToExecutionChange:
    validator_index: int
    from_bls_pubkey: bytes
    to_execution_address: bytes

    def hash_tree_root(self) -> bytes:
        return _merkleize([_u64(self.validator_index), _bytes_root(self.from_bls_pubkey), _bytes_root(self.to_execution_address)])


@dataclass
class SignedBLSToExecutionChange:
    message: BLSToExecutionChange
    signature: bytes


@dataclass
class SyncAggregate:
    sync_committee_bits: Sequence[bool]
    sync_committee_signature: bytes


@dataclass
class BeaconBlockBody:
    randao_reveal: bytes
    body_root: bytes  # hash_tree_root(BeaconBlockBody), from the import pipeline
    proposer_slashings: List[ProposerSlashing] = field(default_factory=list)
    attester_slashings: List[AttesterSlashing] = field(default_factory=list)
    attestations: List[Attestation] = field(default_factory=list)
    voluntary_exits: List[SignedVoluntaryExit] = field(default_factory=list)
    sync_aggregate: Optional[SyncAggregate] = None
    bls_to_execution_changes: List[SignedBLSToExecutionChange] = field(default_factory=list)


@dataclass
class BeaconBlock:
    slot: int
    proposer_index: int
    parent_root: bytes
    state_root: bytes
    body: BeaconBlockBody

    def hash_tree_root(self) -> bytes:
        """hash_tree_root(BeaconBlock) == hash_tree_root of its header (same field roots)."""
        return BeaconBlockHeader(self.slot, self.proposer_index, self.parent_root, self.state_root,
                                 self.body.body_root).hash_tree_root()


@dataclass
class SignedBeaconBlock:
    message: BeaconBlock
    signature: bytes


# ---- config (fork schedule, domains) and the index-form epoch context ---------------------------
@dataclass
class Fork:
    name: str
    epoch: int
    version: bytes


class BeaconConfig:
    """The fork schedule and the domain rules of config/src/genesisConfig/index.ts:27-87."""

    def __init__(self, forks: Sequence[Fork], genesis_validators_root: bytes, deneb_fork_epoch: Optional[int] = None):
        self.forks = sorted(forks, key=lambda f: f.epoch)
        self.by_name = {f.name: f for f in self.forks}
        self.genesis_validators_root = bytes(genesis_validators_root)
        self.deneb_fork_epoch = deneb_fork_epoch if deneb_fork_epoch is not None else (
            self.by_name["deneb"].epoch if "deneb" in self.by_name else 2 ** 64 - 1)
        self._cache: Dict[Tuple[str, bytes], bytes] = {}

    def fork_seq(self, slot: int) -> int:
        """getForkSeq(slot): the position of the active fork in FORK_ORDER."""
        return FORK_ORDER.index(self.fork_info(slot)[0].name)

    def fork_info(self, slot: int) -> Tuple[Fork, Fork]:
        """(fork at slot, the fork before it) -- chainForkConfig.getForkInfo + prevForkName."""
        epoch = compute_epoch_at_slot(slot)
        k = 0
        for i, f in enumerate(self.forks):
            if f.epoch <= epoch:
                k = i
        return self.forks[k], self.forks[max(k - 1, 0)]

    def _domain(self, fork: Fork, domain_type: bytes) -> bytes:
        key = (fork.name, bytes(domain_type))
        d = self._cache.get(key)
        if d is None:
            d = self._cache[key] = compute_domain(domain_type, fork.version, self.genesis_validators_root)
        return d

    def get_domain(self, state_slot: int, domain_type: bytes, message_slot: Optional[int] = None) -> bytes:
        epoch = compute_epoch_at_slot(state_slot if message_slot is None else message_slot)
        cur, prev = self.fork_info(state_slot)
        return self._domain(prev if epoch < cur.epoch else cur, domain_type)

    def get_domain_at_fork(self, fork_name: str, domain_type: bytes) -> bytes:
        return self._domain(self.by_name[fork_name], domain_type)

    def get_domain_for_voluntary_exit(self, state_slot: int, message_slot: Optional[int] = None) -> bytes:
        if state_slot < self.deneb_fork_epoch * SLOTS_PER_EPOCH:
            return self.get_domain(state_slot, DOMAIN_VOLUNTARY_EXIT, message_slot)
        return self.get_domain_at_fork("capella", DOMAIN_VOLUNTARY_EXIT)


class EpochState:
    """The slice of CachedBeaconState the builders read: state slot, config, beacon committees
    (EpochCache.getBeaconCommittee) and the current sync committee's validator indices
    (currentSyncCommitteeIndexed.validatorIndices).  index2pubkey itself lives in HBM."""

    def __init__(self, config: BeaconConfig, slot: int, get_beacon_committee: Callable[[int, int], Sequence[int]],
                 current_sync_committee: Sequence[int]):
        self.config = config
        self.slot = slot
        self.get_beacon_committee = get_beacon_committee
        self.current_sync_committee = list(current_sync_committee)

    def attesting_indices(self, att: Attestation, fork_seq: Optional[int] = None) -> List[int]:
        """getIndexedAttestation / getAttestingIndices (epochCache.ts:938-973), sorted.  Before electra
        the committee of (slot, index); from electra on the committees of committee_bits concatenated
        (getBeaconCommittees, :813-849).  Either way intersected with the aggregation bits, whose
        length must match (BitArray.intersectValues)."""
        if fork_seq is None or fork_seq < FORK_ORDER.index("electra"):
            committee = self.get_beacon_committee(att.data.slot, att.data.index)
        else:
            if att.committee_bits is None:
                raise ValueError("electra attestation without committee_bits")
            indices = [i for i, bit in enumerate(att.committee_bits) if bit]
            if not indices:
                raise ValueError("Attempt to get committees without providing CommitteeIndex")
            committee = []
            for ci in indices:
                if ci >= MAX_COMMITTEES_PER_SLOT:
                    raise ValueError("COMMITTEE_INDEX_OUT_OF_RANGE %d" % ci)
                committee.extend(self.get_beacon_committee(att.data.slot, ci))
        if len(att.aggregation_bits) != len(committee):
            raise ValueError("aggregation bits length %d != committee size %d" % (len(att.aggregation_bits), len(committee)))
        return sorted(v for v, bit in zip(committee, att.aggregation_bits) if bit)


# ---- builders ------------------------------------------------------------------------------------
# A pending set: (kind, index-form pubkey, signature, object root or AttestationData bytes, domain)
_ATT = "att"


class _Pending:
    __slots__ = ("kind", "key", "signature", "obj", "domain")

    def __init__(self, kind, key, signature, obj, domain):
        self.kind, self.key, self.signature, self.obj, self.domain = kind, key, signature, obj, domain


def _randao(state: EpochState, block: BeaconBlock) -> _Pending:
    epoch = compute_epoch_at_slot(block.slot)
    domain = state.config.get_domain(state.slot, DOMAIN_RANDAO, block.slot)
    return _Pending("single", block.proposer_index, block.body.randao_reveal, _u64(epoch), domain)


def _proposer(state: EpochState, signed: SignedBeaconBlock) -> _Pending:
    b = signed.message
    domain = state.config.get_domain(state.slot, DOMAIN_BEACON_PROPOSER, b.slot)
    return _Pending("single", b.proposer_index, signed.signature, b.hash_tree_root(), domain)


def _proposer_slashing(state: EpochState, ps: ProposerSlashing) -> List[_Pending]:
    idx = ps.signed_header_1.message.proposer_index
    out = []
    for sh in (ps.signed_header_1, ps.signed_header_2):
        domain = state.config.get_domain(state.slot, DOMAIN_BEACON_PROPOSER, sh.message.slot)
        out.append(_Pending("single", idx, sh.signature, sh.message.hash_tree_root(), domain))
    return out


def _indexed_attestation(state: EpochState, ia: IndexedAttestation) -> _Pending:
    domain = state.config.get_domain(state.slot, DOMAIN_BEACON_ATTESTER, compute_start_slot_at_epoch(ia.data.target.epoch))
    return _Pending(_ATT, list(ia.attesting_indices), ia.signature, ia.data.serialize(), domain)


def _sync_aggregate(state: EpochState, block: BeaconBlock) -> Optional[_Pending]:
    agg = block.body.sync_aggregate
    if agg is None:
        return None
    committee = state.current_sync_committee
    participants = [v for v, bit in zip(committee, agg.sync_committee_bits) if bit]
    if not participants:
        # processSyncCommittee.ts:93-101: no participation -> the signature must be the infinity point
        if bytes(agg.sync_committee_signature) == G2_POINT_AT_INFINITY:
            return None
        raise ValueError("Empty sync committee signature is not infinity")
    previous_slot = max(block.slot, 1) - 1
    domain = state.config.get_domain(state.slot, DOMAIN_SYNC_COMMITTEE, previous_slot)
    return _Pending("agg", participants, agg.sync_committee_signature, bytes(block.parent_root), domain)


def _voluntary_exit(state: EpochState, se: SignedVoluntaryExit) -> _Pending:
    domain = state.config.get_domain_for_voluntary_exit(state.slot, compute_start_slot_at_epoch(se.message.epoch))
    return _Pending("single", se.message.validator_index, se.signature, se.message.hash_tree_root(), domain)


def _bls_change(state: EpochState, sc: SignedBLSToExecutionChange) -> _Pending:
    domain = state.config.get_domain_at_fork("phase0", DOMAIN_BLS_TO_EXECUTION_CHANGE)
    return _Pending("raw", bytes(sc.message.from_bls_pubkey), sc.signature, sc.message.hash_tree_root(), domain)


def _block_pending(state: EpochState, signed: SignedBeaconBlock, skip_proposer_signature: bool) -> List[_Pending]:
    """The reference order (signatureSets/index.ts:37-70)."""
    b = signed.message
    body = b.body
    out = [_randao(state, b)]
    for ps in body.proposer_slashings:
        out += _proposer_slashing(state, ps)
    for a_s in body.attester_slashings:
        out += [_indexed_attestation(state, a_s.attestation_1), _indexed_attestation(state, a_s.attestation_2)]
    fork = state.config.fork_seq(b.slot)  # getForkSeq(signedBlock.message.slot), index.ts:35
    for att in body.attestations:
        out.append(_indexed_attestation(state, IndexedAttestation(state.attesting_indices(att, fork), att.data, att.signature)))
    for se in body.voluntary_exits:
        out.append(_voluntary_exit(state, se))
    if not skip_proposer_signature:
        out.append(_proposer(state, signed))
    sync = _sync_aggregate(state, b)  # altair+: absent (None) body field before altair
    if sync is not None:
        out.append(sync)
    for sc in body.bls_to_execution_changes:
        out.append(_bls_change(state, sc))
    return out


def _resolve(pending: List[_Pending], hasher) -> List[ISignatureSet]:
    """Signing roots of every pending set in two device calls, then the index-form sets."""
    domains: List[bytes] = []
    dom_of: Dict[bytes, int] = {}

    def dom_idx(d):
        if d not in dom_of:
            dom_of[d] = len(domains)
            domains.append(d)
        return dom_of[d]

    att = [p for p in pending if p.kind == _ATT]
    rest = [p for p in pending if p.kind != _ATT]
    roots: Dict[int, bytes] = {}
    if att:
        local_domains: List[bytes] = []
        local_of: Dict[bytes, int] = {}
        idx = []
        for p in att:
            if p.domain not in local_of:
                local_of[p.domain] = len(local_domains)
                local_domains.append(p.domain)
            idx.append(local_of[p.domain])
        r = hasher.attestation_data_signing_roots(b"".join(p.obj for p in att), local_domains, idx)
        for p, root in zip(att, r):
            roots[id(p)] = root
    if rest:
        idx = [dom_idx(p.domain) for p in rest]
        r = hasher.compute_signing_roots(b"".join(p.obj for p in rest), domains, idx)
        for p, root in zip(rest, r):
            roots[id(p)] = root
    out: List[ISignatureSet] = []
    for p in pending:
        root = roots[id(p)]
        if p.kind in (_ATT, "agg"):
            out.append(AggregatedSignatureSet(p.key, root, bytes(p.signature)))
        elif p.kind == "raw":
            out.append(SingleSignatureSet(0, root, bytes(p.signature), pubkey=p.key))
        else:
            out.append(SingleSignatureSet(int(p.key), root, bytes(p.signature)))
    return out


def get_block_signature_sets(state: EpochState, signed_block: SignedBeaconBlock, hasher,
                             skip_proposer_signature: bool = False) -> List[ISignatureSet]:
    """getBlockSignatureSets (signatureSets/index.ts:26-73) in index form."""
    return _resolve(_block_pending(state, signed_block, skip_proposer_signature), hasher)


def get_blocks_signature_sets(state: EpochState, signed_blocks: Sequence[SignedBeaconBlock], hasher,
                              skip_proposer_signature: bool = False) -> List[List[ISignatureSet]]:
    """The sets of every block of a range-sync segment (verifyBlocksSignatures.ts:32-51: one
    verifySignatureSets call per block), with the signing roots of all blocks in the same two
    device calls."""
    pend = [_block_pending(state, b, skip_proposer_signature) for b in signed_blocks]
    flat = _resolve([p for ps in pend for p in ps], hasher)
    out, k = [], 0
    for ps in pend:
        out.append(flat[k:k + len(ps)])
        k += len(ps)
    return out


def get_attestations_signature_sets(state: EpochState, signed_block: SignedBeaconBlock, hasher) -> List[ISignatureSet]:
    """getAttestationsSignatureSets (indexedAttestation.ts:39-51)."""
    fork = state.config.fork_seq(signed_block.message.slot)
    return _resolve([_indexed_attestation(state, IndexedAttestation(state.attesting_indices(a, fork), a.data, a.signature))
                     for a in signed_block.message.body.attestations], hasher)
