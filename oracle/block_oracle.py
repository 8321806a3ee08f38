"""CPU oracle for getBlockSignatureSets.  TEST INFRASTRUCTURE ONLY.

Only tests/, tests/golden/ generators and bench.py's cpu_baseline leg may import this module; the
product path (lodestar_amd) never does.

Restates, over plain JSON-shaped dicts (the fixture format of tests/golden/c4_block.json):
  * getBlockSignatureSets, state-transition/src/signatureSets/index.ts:26-73 -- set order: randao,
    proposer slashings, attester slashings, attestations, voluntary exits, proposer, sync aggregate,
    BLS-to-execution changes;
  * the sub-builders randao.ts:19-31, proposer.ts:15-32, proposerSlashings.ts:9-41,
    attesterSlashings.ts:7-39, indexedAttestation.ts:21-51, voluntaryExits.ts:21-44,
    blsToExecutionChange.ts:19-44, block/processSyncCommittee.ts:59-111;
  * getDomain / getDomainAtFork / getDomainForVoluntaryExit, config/src/genesisConfig/index.ts:27-87,
    and computeDomain / computeForkDataRoot (:125-139);
  * getAttestingIndices, state-transition/src/cache/epochCache.ts:953-973: pre-electra the committee of
    (slot, index); electra the committees of committeeBits concatenated (getBeaconCommittees,
    :813-849); either intersected with the aggregation bits (BitArray.intersectValues).
Hashing through oracle/ssz_oracle.py (pinned by K1).  The builders under test are
lodestar_amd/signature_sets.py; this file shares no code with them.
"""
from oracle import ssz_oracle as S

SLOTS_PER_EPOCH = 32
DOMAINS = {"proposer": "00000000", "attester": "01000000", "randao": "02000000", "exit": "04000000",
           "sync": "07000000", "bls_change": "0a000000"}


def _root_u64(v):
    return S.uint64_chunk(v)


def _merkle(chunks):
    return S.merkleize(list(chunks))


def header_root(h):
    return _merkle([_root_u64(h["slot"]), _root_u64(h["proposer_index"]), bytes.fromhex(h["parent_root"]),
                    bytes.fromhex(h["state_root"]), bytes.fromhex(h["body_root"])])


def exit_root(e):
    return _merkle([_root_u64(e["epoch"]), _root_u64(e["validator_index"])])


def bls_change_root(c):
    pk = bytes.fromhex(c["from_bls_pubkey"])
    return _merkle([_root_u64(c["validator_index"]), S.bytes_root(pk), bytes.fromhex(c["to_execution_address"]).ljust(32, b"\0")])


def att_data_bytes(d):
    return S.attestation_data_serialize(d["slot"], d["index"], bytes.fromhex(d["beacon_block_root"]),
                                        (d["source_epoch"], bytes.fromhex(d["source_root"])),
                                        (d["target_epoch"], bytes.fromhex(d["target_root"])))


def _fork_at(cfg, slot):
    """index of the fork active at slot in the (epoch-sorted) schedule"""
    epoch = slot // SLOTS_PER_EPOCH
    k = 0
    for i, (_, e, _) in enumerate(cfg["forks"]):
        if e <= epoch:
            k = i
    return k


def _domain_of(cfg, fork_index, kind):
    version = bytes.fromhex(cfg["forks"][fork_index][2])
    return S.compute_domain(bytes.fromhex(DOMAINS[kind]), version, bytes.fromhex(cfg["gvr"]))


def get_domain(cfg, state_slot, kind, message_slot):
    k = _fork_at(cfg, state_slot)
    fork_epoch = cfg["forks"][k][1]
    use = k if message_slot // SLOTS_PER_EPOCH >= fork_epoch else max(k - 1, 0)
    return _domain_of(cfg, use, kind)


def get_domain_at_fork(cfg, name, kind):
    k = [f[0] for f in cfg["forks"]].index(name)
    return _domain_of(cfg, k, kind)


def exit_domain(cfg, state_slot, message_slot):
    if state_slot < cfg["deneb_epoch"] * SLOTS_PER_EPOCH:
        return get_domain(cfg, state_slot, "exit", message_slot)
    return get_domain_at_fork(cfg, "capella", "exit")


def block_signature_sets(fix, block=None, committees=None):
    """[(kind, key, signing_root, signature)] with kind in single / aggregate / raw and key the
    validator index, the attesting indices or the raw 48-byte pubkey."""
    cfg = fix["config"]
    st = fix["state_slot"]
    b = block or fix["block"]
    com = committees or fix["committees"]
    out = []
    sig = lambda h: bytes.fromhex(h)
    # randao
    out.append(("single", b["proposer_index"], S.compute_signing_root(_root_u64(b["slot"] // SLOTS_PER_EPOCH),
                                                                       get_domain(cfg, st, "randao", b["slot"])), sig(b["randao_reveal"])))
    for ps in b["proposer_slashings"]:
        idx = ps[0]["message"]["proposer_index"]
        for sh in ps:
            out.append(("single", idx, S.compute_signing_root(header_root(sh["message"]),
                                                               get_domain(cfg, st, "proposer", sh["message"]["slot"])), sig(sh["signature"])))
    for a_s in b["attester_slashings"]:
        for ia in a_s:
            dom = get_domain(cfg, st, "attester", ia["data"]["target_epoch"] * SLOTS_PER_EPOCH)
            out.append(("aggregate", list(ia["attesting_indices"]),
                        S.compute_signing_root(S.attestation_data_root(att_data_bytes(ia["data"])), dom), sig(ia["signature"])))
    electra = "electra" in [f[0] for f in cfg["forks"][:_fork_at(cfg, b["slot"]) + 1]]
    for att in b["attestations"]:
        d = att["data"]
        if electra:
            committee = [v for ci, bit in enumerate(att["committee_bits"]) if bit for v in com["%d,%d" % (d["slot"], ci)]]
        else:
            committee = com["%d,%d" % (d["slot"], d["index"])]
        assert len(committee) == len(att["bits"]), "intersectValues: length mismatch"
        indices = sorted(v for v, bit in zip(committee, att["bits"]) if bit)
        dom = get_domain(cfg, st, "attester", d["target_epoch"] * SLOTS_PER_EPOCH)
        out.append(("aggregate", indices, S.compute_signing_root(S.attestation_data_root(att_data_bytes(d)), dom), sig(att["signature"])))
    for se in b["voluntary_exits"]:
        m = se["message"]
        out.append(("single", m["validator_index"], S.compute_signing_root(exit_root(m), exit_domain(cfg, st, m["epoch"] * SLOTS_PER_EPOCH)),
                    sig(se["signature"])))
    out.append(("single", b["proposer_index"], S.compute_signing_root(header_root(b), get_domain(cfg, st, "proposer", b["slot"])),
                sig(b["signature"])))
    sa = b["sync_aggregate"]
    parts = [v for v, bit in zip(fix["sync_committee"], sa["bits"]) if bit]
    if parts:
        prev = max(b["slot"], 1) - 1
        out.append(("aggregate", parts, S.compute_signing_root(bytes.fromhex(b["parent_root"]), get_domain(cfg, st, "sync", prev)),
                    sig(sa["signature"])))
    for sc in b["bls_changes"]:
        m = sc["message"]
        out.append(("raw", bytes.fromhex(m["from_bls_pubkey"]),
                    S.compute_signing_root(bls_change_root(m), get_domain_at_fork(cfg, "phase0", "bls_change")), sig(sc["signature"])))
    return out
