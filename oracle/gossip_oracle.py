"""CPU oracle for the gossip-side signature-set builders (VERDICT r03 "missing" 1; SURVEY.md 8(a)
a11/a12, north_star "beacon-node gossip validation ... can swap it in").  TEST INFRASTRUCTURE ONLY:
only tests/ and tests/golden/ generators import it; the product path (lodestar_amd) never does.

Restates over plain JSON-shaped dicts (the fixture format of tests/golden/gossip_sets.json), with
oracle/ssz_oracle.py's merkleization (pinned by K1):
  * validateAggregateAndProof's three sets, beacon-node/src/chain/validation/aggregateAndProof.ts:
    211-229 -- getSelectionProofSignatureSet (signatureSets/selectionProof.ts:7-27: ssz.Slot,
    DOMAIN_SELECTION_PROOF at the fork of the slot), getAggregateAndProofSignatureSet
    (signatureSets/aggregateAndProof.ts:13-40: phase0 / electra AggregateAndProof by the fork of the
    epoch's start slot, DOMAIN_AGGREGATE_AND_PROOF at that fork), and the aggregate over its attesting
    indices under getAttestationDataSigningRoot (attestation.ts:657-665);
  * validateSyncCommitteeGossipContributionAndProof's three sets, syncCommitteeContributionAndProof.ts:
    73-92 -- getSyncCommitteeSelectionProofSignatureSet (SyncAggregatorSelectionData),
    getContributionAndProofSignatureSet (ContributionAndProof), getSyncCommitteeContributionSignatureSet
    over getContributionIndices (:109-119);
  * getSyncCommitteeSignatureSet (signatureSets/syncCommittee.ts:10-23).
SSZ shapes: phase0 Attestation {BitList[2048], AttestationData, Bytes96}, electra Attestation
{BitList[131072], AttestationData, Bytes96, BitVector[64]}, AggregateAndProof {uint64, Attestation,
Bytes96}, SyncCommitteeContribution {uint64, Root, uint64, BitVector[128], Bytes96},
ContributionAndProof {uint64, SyncCommitteeContribution, Bytes96}, SyncAggregatorSelectionData
{uint64, uint64} (types/src/{phase0,altair,electra}/sszTypes.ts).  BitList roots: the packed bits
merkleized to ceil(limit / 256) chunks, then the length mixed in; BitVector roots: the packed bits.
Domains through oracle/block_oracle.py's getDomain / getDomainAtFork restatement.

PARITY UNPINNED for the container roots: the phase0 / electra AggregateAndProof roots and the
SyncCommitteeContribution / ContributionAndProof roots are restated here the same way as in
lodestar_amd/gossip_sets.py and addon/gossip_sets.js, and no vector held by the reference fixes them
(its validation tests build these containers at run time and sign them with its own BLS; nothing in
/root/reference records a root).  tests/golden/gossip_sets.json is therefore self-consistent under
this restatement, not pinned; K1 pins the merkleization primitives (uint64, Bytes48, container
padding) and the domains / fork selection match selectionProof.ts, aggregateAndProof.ts and
attestation.ts:657-665.
"""
from oracle import block_oracle as BO
from oracle import ssz_oracle as S

SLOTS_PER_EPOCH = 32
EPOCHS_PER_SYNC_COMMITTEE_PERIOD = 256
SUBNET_SIZE = 128
DOMAIN_HEX = {"selection": "05000000", "aggregate_and_proof": "06000000", "sync": "07000000", "sync_selection": "08000000",
              "contribution_and_proof": "09000000", "attester": "01000000"}


def _domain(cfg, fork_index, kind):
    return S.compute_domain(bytes.fromhex(DOMAIN_HEX[kind]), bytes.fromhex(cfg["forks"][fork_index][2]), bytes.fromhex(cfg["gvr"]))


def domain_at_fork_of_slot(cfg, kind, slot):
    """getDomainAtFork(getForkName(slot), kind)"""
    return _domain(cfg, BO._fork_at(cfg, slot), kind)


def get_domain(cfg, state_slot, kind, message_slot):
    """getDomain(stateSlot, kind, messageSlot): the state's fork, or the one before it for a message
    of an earlier epoch than the state's fork epoch (config/src/genesisConfig/index.ts:27-87)."""
    k = BO._fork_at(cfg, state_slot)
    use = k if message_slot // SLOTS_PER_EPOCH >= cfg["forks"][k][1] else max(k - 1, 0)
    return _domain(cfg, use, kind)


def _is_electra(cfg, slot):
    return "electra" in [f[0] for f in cfg["forks"][:BO._fork_at(cfg, slot) + 1]]


def _bits_bytes(bits):
    out = bytearray((len(bits) + 7) // 8)
    for i, b in enumerate(bits):
        if b:
            out[i // 8] |= 1 << (i % 8)
    return bytes(out)


def bitlist_root(bits, limit):
    packed = _bits_bytes(bits)
    chunks = [packed[i:i + 32].ljust(32, b"\0") for i in range(0, len(packed), 32)]
    n_limit = (limit + 255) // 256
    chunks += [bytes(32)] * (n_limit - len(chunks))
    return S.merkleize([S.merkleize(chunks), S.uint64_chunk(len(bits))])


def bitvector_root(bits):
    return S.bytes_root(_bits_bytes(bits))


def attestation_data_root(d):
    return S.attestation_data_root(BO.att_data_bytes(d))


def attestation_root(att, electra):
    parts = [bitlist_root(att["bits"], 2048 * 64 if electra else 2048), attestation_data_root(att["data"]),
             S.bytes_root(bytes.fromhex(att["signature"]))]
    if electra:
        parts.append(bitvector_root(att.get("committee_bits") or [False] * 64))
    return S.merkleize(parts)


def aggregate_and_proof_root(m, electra):
    return S.merkleize([S.uint64_chunk(m["aggregator_index"]), attestation_root(m["aggregate"], electra),
                        S.bytes_root(bytes.fromhex(m["selection_proof"]))])


def contribution_root(c):
    return S.merkleize([S.uint64_chunk(c["slot"]), bytes.fromhex(c["beacon_block_root"]), S.uint64_chunk(c["subcommittee_index"]),
                        bitvector_root(c["bits"]), S.bytes_root(bytes.fromhex(c["signature"]))])


def contribution_and_proof_root(m):
    return S.merkleize([S.uint64_chunk(m["aggregator_index"]), contribution_root(m["contribution"]),
                        S.bytes_root(bytes.fromhex(m["selection_proof"]))])


def aggregate_and_proof_sets(cfg, signed, attesting_indices):
    """[(kind, key, signing_root, signature)] in the reference order."""
    m = signed["message"]
    att = m["aggregate"]
    slot = att["data"]["slot"]
    epoch_start = (slot // SLOTS_PER_EPOCH) * SLOTS_PER_EPOCH
    sel = S.compute_signing_root(S.uint64_chunk(slot), domain_at_fork_of_slot(cfg, "selection", slot))
    aap = S.compute_signing_root(aggregate_and_proof_root(m, _is_electra(cfg, epoch_start)),
                                 domain_at_fork_of_slot(cfg, "aggregate_and_proof", epoch_start))
    target_start = att["data"]["target_epoch"] * SLOTS_PER_EPOCH
    agg = S.compute_signing_root(attestation_data_root(att["data"]), domain_at_fork_of_slot(cfg, "attester", target_start))
    return [("single", m["aggregator_index"], sel, bytes.fromhex(m["selection_proof"])),
            ("single", m["aggregator_index"], aap, bytes.fromhex(signed["signature"])),
            ("aggregate", sorted(attesting_indices), agg, bytes.fromhex(att["signature"]))]


def indexed_sync_committee(fix, slot):
    period = ((slot + 1) // SLOTS_PER_EPOCH) // EPOCHS_PER_SYNC_COMMITTEE_PERIOD
    own = (fix["state_slot"] // SLOTS_PER_EPOCH) // EPOCHS_PER_SYNC_COMMITTEE_PERIOD
    if period == own:
        return fix["sync_committee"]
    if period == own + 1 and fix.get("next_sync_committee"):
        return fix["next_sync_committee"]
    raise ValueError("NO_SYNC_COMMITTEE")


def contribution_participants(fix, c):
    start = c["subcommittee_index"] * SUBNET_SIZE
    sub = indexed_sync_committee(fix, c["slot"])[start:start + SUBNET_SIZE]
    assert len(sub) == len(c["bits"])
    return [v for v, b in zip(sub, c["bits"]) if b]


def contribution_and_proof_sets(fix, signed):
    cfg, st = fix["config"], fix["state_slot"]
    m = signed["message"]
    c = m["contribution"]
    sel_root = S.merkleize([S.uint64_chunk(c["slot"]), S.uint64_chunk(c["subcommittee_index"])])
    sel = S.compute_signing_root(sel_root, get_domain(cfg, st, "sync_selection", c["slot"]))
    cap = S.compute_signing_root(contribution_and_proof_root(m), get_domain(cfg, st, "contribution_and_proof", c["slot"]))
    agg = S.compute_signing_root(bytes.fromhex(c["beacon_block_root"]), get_domain(cfg, st, "sync", c["slot"]))
    return [("single", m["aggregator_index"], sel, bytes.fromhex(m["selection_proof"])),
            ("single", m["aggregator_index"], cap, bytes.fromhex(signed["signature"])),
            ("aggregate", contribution_participants(fix, c), agg, bytes.fromhex(c["signature"]))]


def sync_committee_message_set(fix, msg):
    root = S.compute_signing_root(bytes.fromhex(msg["beacon_block_root"]), get_domain(fix["config"], fix["state_slot"], "sync", msg["slot"]))
    return ("single", msg["validator_index"], root, bytes.fromhex(msg["signature"]))
