"""Index-form signature-set builders of gossip validation (the callers of IBlsVerifier besides block
import), with every container signing root hashed on the device.

Reference (packages/beacon-node/src/chain/validation/):
  * signatureSets/selectionProof.ts:7-27            getSelectionProofSigningRoot / ...SignatureSet
  * signatureSets/aggregateAndProof.ts:13-40        getAggregateAndProofSigningRoot / ...SignatureSet
    (phase0 or electra AggregateAndProof by the fork of the attestation epoch's start slot)
  * aggregateAndProof.ts:211-229                    the three sets of a gossip aggregate: selection
    proof, aggregator signature, and the aggregate itself over its attesting indices
    (createAggregateSignatureSetFromComponents, getAttestationDataSigningRoot attestation.ts:657-665)
  * signatureSets/syncCommittee.ts:10-23            getSyncCommitteeSignatureSet
  * signatureSets/contributionAndProof.ts:10-27     getContributionAndProofSignatureSet
  * signatureSets/syncCommitteeSelectionProof.ts:10-27
  * signatureSets/syncCommitteeContribution.ts:6-18
  * syncCommitteeContributionAndProof.ts:73-92, :109-119  the three sets of a contribution, participants
    from getIndexedSyncCommittee(contribution.slot) intersected with the aggregation bits
SSZ types: types/src/phase0/sszTypes.ts:113,310-317,451-466 (CommitteeBits, Attestation,
AggregateAndProof), types/src/electra/sszTypes.ts:49-68,97-112, types/src/altair/sszTypes.ts:47-91.
Domains: params/src/index.ts:139-149.

As in lodestar_amd/signature_sets.py (the block builders), pubkeys are validator indices into the
HBM-resident index2pubkey table.  Hashing: every container root of these messages is a tree of
32-byte nodes over leaves taken from the message (uint64 chunks, roots, packed bitfields, 96-byte
signatures split into chunks); the trees of all the messages of a call are hashed on the device level
by level (gbv_merkle_roots, one launch per distinct subtree depth per level) and the signing roots
(SigningData{object root, domain}) in one gbv_signing_roots call -- nothing is hashed on the host.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Sequence, Tuple, Union

from .signature_sets import (DOMAIN_AGGREGATE_AND_PROOF, DOMAIN_BEACON_ATTESTER, DOMAIN_SELECTION_PROOF, DOMAIN_SYNC_COMMITTEE,
                             FORK_ORDER, MAX_COMMITTEES_PER_SLOT, AttestationData, BeaconConfig, compute_epoch_at_slot,
                             compute_start_slot_at_epoch)
from .verifier import AggregatedSignatureSet, ISignatureSet, SingleSignatureSet

DOMAIN_SYNC_COMMITTEE_SELECTION_PROOF = bytes([8, 0, 0, 0])  # params/src/index.ts:147
DOMAIN_CONTRIBUTION_AND_PROOF = bytes([9, 0, 0, 0])          # params/src/index.ts:148
MAX_VALIDATORS_PER_COMMITTEE = 2048                          # presets/mainnet.ts:14
SYNC_COMMITTEE_SIZE = 512
SYNC_COMMITTEE_SUBNET_COUNT = 4                              # params/src/index.ts:196
SYNC_COMMITTEE_SUBNET_SIZE = SYNC_COMMITTEE_SIZE // SYNC_COMMITTEE_SUBNET_COUNT
EPOCHS_PER_SYNC_COMMITTEE_PERIOD = 256                       # presets/mainnet.ts:91


# ---- SSZ trees (hashed on the device) ------------------------------------------------------------
class Node:
    """hash_tree_root of a container / vector: merkleize(children), zero-padded to 2**depth leaves.
    A child is a 32-byte leaf or another Node.  mix_len: mix_in_length (a list's root)."""
    __slots__ = ("children", "depth", "mix_len")

    def __init__(self, children: Sequence[Union[bytes, "Node"]], depth: Optional[int] = None, mix_len: Optional[int] = None):
        self.children = list(children)
        d = 0
        while (1 << d) < len(self.children):
            d += 1
        self.depth = d if depth is None else depth
        assert len(self.children) <= (1 << self.depth)
        self.mix_len = mix_len


def _u64(v: int) -> bytes:
    return int(v).to_bytes(8, "little") + bytes(24)


def _chunks(b: bytes) -> List[bytes]:
    b = bytes(b)
    return [b[i:i + 32].ljust(32, b"\0") for i in range(0, len(b), 32)] or [bytes(32)]


def _bytes_node(b: bytes) -> Node:
    """A fixed-length byte vector (Bytes96 signature: three chunks, padded to four)."""
    return Node(_chunks(b))


def _pack_bits(bits: Sequence[bool]) -> bytes:
    out = bytearray((len(bits) + 7) // 8)
    for i, bit in enumerate(bits):
        if bit:
            out[i >> 3] |= 1 << (i & 7)
    return bytes(out)


def _bitvector_node(bits: Sequence[bool]) -> Union[bytes, Node]:
    ch = _chunks(_pack_bits(bits))
    return ch[0] if len(ch) == 1 else Node(ch)


def _bitlist_node(bits: Sequence[bool], limit: int) -> Node:
    """BitList[limit]: the packed bits (no delimiter) merkleized to the limit's chunk count, then the
    bit length mixed in."""
    chunk_limit = (limit + 255) // 256
    depth = 0
    while (1 << depth) < chunk_limit:
        depth += 1
    body = Node(_chunks(_pack_bits(bits)) if bits else [], depth=depth)
    return Node([body, _u64(len(bits))], mix_len=len(bits))


def _checkpoint_node(epoch: int, root: bytes) -> Node:
    return Node([_u64(epoch), bytes(root)])


def attestation_data_node(d: AttestationData) -> Node:
    return Node([_u64(d.slot), _u64(d.index), bytes(d.beacon_block_root), _checkpoint_node(d.source.epoch, d.source.root),
                 _checkpoint_node(d.target.epoch, d.target.root)])


def device_roots(hasher, trees: Sequence[Union[bytes, Node]]) -> List[bytes]:
    """Roots of many trees on the device: level by level from the leaves, every pending subtree of a
    level hashed by one gbv_merkle_roots launch per distinct depth."""
    memo: Dict[int, bytes] = {}
    # post-order list of every Node, each with its height (longest path to a leaf)
    order: List[Node] = []
    height: Dict[int, int] = {}

    def visit(n):
        if isinstance(n, (bytes, bytearray)) or id(n) in height:
            return 0 if isinstance(n, (bytes, bytearray)) else height[id(n)]
        h = 0
        for c in n.children:
            h = max(h, visit(c) + 1)
        height[id(n)] = h
        order.append(n)
        return h

    for t in trees:
        visit(t)
    levels: Dict[int, List[Node]] = {}
    for n in order:
        levels.setdefault(height[id(n)], []).append(n)
    for h in sorted(levels):
        by_depth: Dict[int, List[Node]] = {}
        for n in levels[h]:
            by_depth.setdefault(n.depth, []).append(n)
        for depth, nodes in sorted(by_depth.items()):
            blob = []
            for n in nodes:
                leaves = [c if isinstance(c, (bytes, bytearray)) else memo[id(c)] for c in n.children]
                leaves += [bytes(32)] * ((1 << depth) - len(leaves))
                blob.extend(leaves)
            roots = hasher.merkle_roots(b"".join(blob), depth)
            for n, r in zip(nodes, roots):
                memo[id(n)] = r
    return [bytes(t) if isinstance(t, (bytes, bytearray)) else memo[id(t)] for t in trees]


# ---- containers ------------------------------------------------------------------------------------
@dataclass
class Attestation:
    """phase0 Attestation, or electra's when committee_bits is set (aggregation bits spanning the
    committees named by committee_bits)."""
    aggregation_bits: Sequence[bool]
    data: AttestationData
    signature: bytes
    committee_bits: Optional[Sequence[bool]] = None

    def node(self, electra: bool) -> Node:
        if electra:
            cb = self.committee_bits if self.committee_bits is not None else [False] * MAX_COMMITTEES_PER_SLOT
            return Node([_bitlist_node(self.aggregation_bits, MAX_VALIDATORS_PER_COMMITTEE * MAX_COMMITTEES_PER_SLOT),
                         attestation_data_node(self.data), _bytes_node(self.signature), _bitvector_node(cb)])
        return Node([_bitlist_node(self.aggregation_bits, MAX_VALIDATORS_PER_COMMITTEE), attestation_data_node(self.data),
                     _bytes_node(self.signature)])


@dataclass
class AggregateAndProof:
    aggregator_index: int
    aggregate: Attestation
    selection_proof: bytes

    def node(self, electra: bool) -> Node:
        return Node([_u64(self.aggregator_index), self.aggregate.node(electra), _bytes_node(self.selection_proof)])


@dataclass
class SignedAggregateAndProof:
    message: AggregateAndProof
    signature: bytes


@dataclass
class SyncCommitteeMessage:
    slot: int
    beacon_block_root: bytes
    validator_index: int
    signature: bytes


@dataclass
class SyncCommitteeContribution:
    slot: int
    beacon_block_root: bytes
    subcommittee_index: int
    aggregation_bits: Sequence[bool]  # SYNC_COMMITTEE_SUBNET_SIZE bits
    signature: bytes

    def node(self) -> Node:
        return Node([_u64(self.slot), bytes(self.beacon_block_root), _u64(self.subcommittee_index),
                     _bitvector_node(self.aggregation_bits), _bytes_node(self.signature)])


@dataclass
class ContributionAndProof:
    aggregator_index: int
    contribution: SyncCommitteeContribution
    selection_proof: bytes

    def node(self) -> Node:
        return Node([_u64(self.aggregator_index), self.contribution.node(), _bytes_node(self.selection_proof)])


@dataclass
class SignedContributionAndProof:
    message: ContributionAndProof
    signature: bytes


class GossipState:
    """The slice of the head state gossip validation reads: config, state slot, and the sync
    committees by period (EpochCache.getIndexedSyncCommittee: current / next)."""

    def __init__(self, config: BeaconConfig, slot: int, current_sync_committee: Sequence[int],
                 next_sync_committee: Optional[Sequence[int]] = None):
        self.config = config
        self.slot = slot
        self.current_sync_committee = list(current_sync_committee)
        self.next_sync_committee = list(next_sync_committee) if next_sync_committee is not None else None

    def indexed_sync_committee(self, slot: int) -> List[int]:
        """getIndexedSyncCommittee(slot) (epochCache.ts:1161-1180): the period of epoch(slot + 1)."""
        period = compute_epoch_at_slot(slot + 1) // EPOCHS_PER_SYNC_COMMITTEE_PERIOD
        own = compute_epoch_at_slot(self.slot) // EPOCHS_PER_SYNC_COMMITTEE_PERIOD
        if period == own:
            return self.current_sync_committee
        if period == own + 1 and self.next_sync_committee is not None:
            return self.next_sync_committee
        raise ValueError("NO_SYNC_COMMITTEE for slot %d" % slot)


# ---- pending sets: (kind, key, signature, object tree, domain) ------------------------------------
@dataclass
class _Pending:
    kind: str  # "single" / "agg"
    key: Union[int, List[int]]
    signature: bytes
    obj: Union[bytes, Node]
    domain: bytes


def _resolve(pending: Sequence[_Pending], hasher) -> List[ISignatureSet]:
    objs = device_roots(hasher, [p.obj for p in pending])
    domains: List[bytes] = []
    dom_of: Dict[bytes, int] = {}
    idx = []
    for p in pending:
        if p.domain not in dom_of:
            dom_of[p.domain] = len(domains)
            domains.append(p.domain)
        idx.append(dom_of[p.domain])
    roots = hasher.compute_signing_roots(b"".join(objs), domains, idx) if pending else []
    out: List[ISignatureSet] = []
    for p, r in zip(pending, roots):
        if p.kind == "agg":
            out.append(AggregatedSignatureSet(list(p.key), r, bytes(p.signature)))
        else:
            out.append(SingleSignatureSet(int(p.key), r, bytes(p.signature)))
    return out


def _electra(config: BeaconConfig, slot: int) -> bool:
    return config.fork_seq(slot) >= FORK_ORDER.index("electra")


def selection_proof_pending(config: BeaconConfig, slot: int, aggregator_index: int, agg: SignedAggregateAndProof) -> _Pending:
    """getSelectionProofSignatureSet (selectionProof.ts:16-27): ssz.Slot under DOMAIN_SELECTION_PROOF
    at the fork of the slot."""
    domain = config.get_domain_at_fork(config.fork_info(slot)[0].name, DOMAIN_SELECTION_PROOF)
    return _Pending("single", aggregator_index, agg.message.selection_proof, _u64(slot), domain)


def aggregate_and_proof_pending(config: BeaconConfig, epoch: int, aggregator_index: int, agg: SignedAggregateAndProof) -> _Pending:
    """getAggregateAndProofSignatureSet (aggregateAndProof.ts:13-40): the phase0 or electra
    AggregateAndProof by the fork of the epoch's start slot."""
    slot = compute_start_slot_at_epoch(epoch)
    fork = config.fork_info(slot)[0].name
    domain = config.get_domain_at_fork(fork, DOMAIN_AGGREGATE_AND_PROOF)
    return _Pending("single", aggregator_index, agg.signature, agg.message.node(_electra(config, slot)), domain)


def attestation_data_pending(config: BeaconConfig, attesting_indices: Sequence[int], data: AttestationData, signature: bytes) -> _Pending:
    """createAggregateSignatureSetFromComponents(attesting pubkeys, getAttestationDataSigningRoot)
    (aggregateAndProof.ts:216-221, attestation.ts:657-665: DOMAIN_BEACON_ATTESTER at the fork of the
    target epoch's start slot)."""
    slot = compute_start_slot_at_epoch(data.target.epoch)
    domain = config.get_domain_at_fork(config.fork_info(slot)[0].name, DOMAIN_BEACON_ATTESTER)
    return _Pending("agg", list(attesting_indices), signature, attestation_data_node(data), domain)


def aggregate_and_proof_signature_sets(config: BeaconConfig, agg: SignedAggregateAndProof, attesting_indices: Sequence[int],
                                       hasher) -> List[ISignatureSet]:
    """The three sets validateAggregateAndProof hands to verifySignatureSets (aggregateAndProof.ts:
    211-229, {batchable: true, priority}): selection proof, aggregator signature, the aggregate over
    its attesting indices (getIndexedAttestation, computed by the caller from the committee)."""
    m = agg.message
    att_slot = m.aggregate.data.slot
    return _resolve([selection_proof_pending(config, att_slot, m.aggregator_index, agg),
                     aggregate_and_proof_pending(config, compute_epoch_at_slot(att_slot), m.aggregator_index, agg),
                     attestation_data_pending(config, attesting_indices, m.aggregate.data, m.aggregate.signature)], hasher)


def sync_committee_pending(state: GossipState, msg: SyncCommitteeMessage) -> _Pending:
    """getSyncCommitteeSignatureSet (syncCommittee.ts:10-23)."""
    domain = state.config.get_domain(state.slot, DOMAIN_SYNC_COMMITTEE, msg.slot)
    return _Pending("single", msg.validator_index, msg.signature, bytes(msg.beacon_block_root), domain)


def sync_committee_signature_sets(state: GossipState, msgs: Sequence[SyncCommitteeMessage], hasher) -> List[ISignatureSet]:
    return _resolve([sync_committee_pending(state, m) for m in msgs], hasher)


def contribution_indices(state: GossipState, contribution: SyncCommitteeContribution) -> List[int]:
    """getContributionIndices (syncCommitteeContributionAndProof.ts:109-119)."""
    start = contribution.subcommittee_index * SYNC_COMMITTEE_SUBNET_SIZE
    sub = state.indexed_sync_committee(contribution.slot)[start:start + SYNC_COMMITTEE_SUBNET_SIZE]
    if len(contribution.aggregation_bits) != len(sub):
        raise ValueError("aggregation bits length %d != subcommittee size %d" % (len(contribution.aggregation_bits), len(sub)))
    return [v for v, bit in zip(sub, contribution.aggregation_bits) if bit]


def sync_selection_proof_pending(state: GossipState, cap: ContributionAndProof) -> _Pending:
    """getSyncCommitteeSelectionProofSignatureSet (syncCommitteeSelectionProof.ts:10-27):
    SyncAggregatorSelectionData{slot, subcommitteeIndex}."""
    slot = cap.contribution.slot
    domain = state.config.get_domain(state.slot, DOMAIN_SYNC_COMMITTEE_SELECTION_PROOF, slot)
    return _Pending("single", cap.aggregator_index, cap.selection_proof, Node([_u64(slot), _u64(cap.contribution.subcommittee_index)]),
                    domain)


def contribution_and_proof_pending(state: GossipState, signed: SignedContributionAndProof) -> _Pending:
    """getContributionAndProofSignatureSet (contributionAndProof.ts:10-27)."""
    domain = state.config.get_domain(state.slot, DOMAIN_CONTRIBUTION_AND_PROOF, signed.message.contribution.slot)
    return _Pending("single", signed.message.aggregator_index, signed.signature, signed.message.node(), domain)


def sync_contribution_pending(state: GossipState, contribution: SyncCommitteeContribution, participants: Sequence[int]) -> _Pending:
    """getSyncCommitteeContributionSignatureSet (syncCommitteeContribution.ts:6-18)."""
    domain = state.config.get_domain(state.slot, DOMAIN_SYNC_COMMITTEE, contribution.slot)
    return _Pending("agg", list(participants), contribution.signature, bytes(contribution.beacon_block_root), domain)


def contribution_and_proof_signature_sets(state: GossipState, signed: SignedContributionAndProof, hasher) -> List[ISignatureSet]:
    """The three sets validateSyncCommitteeGossipContributionAndProof hands to verifySignatureSets
    (syncCommitteeContributionAndProof.ts:73-92, {batchable: true})."""
    cap = signed.message
    participants = contribution_indices(state, cap.contribution)
    if not participants:
        raise ValueError("NO_PARTICIPANT")
    return _resolve([sync_selection_proof_pending(state, cap), contribution_and_proof_pending(state, signed),
                     sync_contribution_pending(state, cap.contribution, participants)], hasher)
