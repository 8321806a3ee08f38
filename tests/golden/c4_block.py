"""C4 full-block fixture helpers (test infrastructure): the synthetic world, JSON -> the
lodestar_amd.signature_sets objects, and the corruption variants ("one invalid member in turn for
each set kind").

World convention (shared with bench.py): validator v has the interop key interopSecretKey(v mod
1024) (state-transition/src/util/interop.ts:18-22) over a 2^20-entry index2pubkey table.
"""
import copy
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
FIX_PATH = os.path.join(HERE, "c4_block.json")
# electra-era block: 8 attestations whose aggregation bits span up to 64 committees (committee_bits)
FIX_PATH_ELECTRA = os.path.join(HERE, "c4_block_electra.json")
N_VALIDATORS = 1 << 20
N_KEYS = 1024


def load(electra=False):
    with open(FIX_PATH_ELECTRA if electra else FIX_PATH) as f:
        return json.load(f)


def _b(h):
    return bytes.fromhex(h)


def to_objects(fix, block=None, committees=None):
    """(EpochState, SignedBeaconBlock) of the product builders from the fixture dicts."""
    from lodestar_amd import signature_sets as B
    cfg = fix["config"]
    config = B.BeaconConfig([B.Fork(n, e, _b(v)) for n, e, v in cfg["forks"]], _b(cfg["gvr"]), cfg["deneb_epoch"])
    com = committees or fix["committees"]
    state = B.EpochState(config, fix["state_slot"], lambda s, i: com["%d,%d" % (s, i)], fix["sync_committee"])
    b = block or fix["block"]

    def data(d):
        return B.AttestationData(d["slot"], d["index"], _b(d["beacon_block_root"]), B.Checkpoint(d["source_epoch"], _b(d["source_root"])),
                                 B.Checkpoint(d["target_epoch"], _b(d["target_root"])))

    def header(h):
        return B.BeaconBlockHeader(h["slot"], h["proposer_index"], _b(h["parent_root"]), _b(h["state_root"]), _b(h["body_root"]))

    body = B.BeaconBlockBody(
        randao_reveal=_b(b["randao_reveal"]), body_root=_b(b["body_root"]),
        proposer_slashings=[B.ProposerSlashing(*[B.SignedBeaconBlockHeader(header(sh["message"]), _b(sh["signature"])) for sh in ps])
                            for ps in b["proposer_slashings"]],
        attester_slashings=[B.AttesterSlashing(*[B.IndexedAttestation(ia["attesting_indices"], data(ia["data"]), _b(ia["signature"]))
                                                 for ia in a_s]) for a_s in b["attester_slashings"]],
        attestations=[B.Attestation(a["bits"], data(a["data"]), _b(a["signature"]), a.get("committee_bits")) for a in b["attestations"]],
        voluntary_exits=[B.SignedVoluntaryExit(B.VoluntaryExit(e["message"]["epoch"], e["message"]["validator_index"]), _b(e["signature"]))
                         for e in b["voluntary_exits"]],
        sync_aggregate=B.SyncAggregate(b["sync_aggregate"]["bits"], _b(b["sync_aggregate"]["signature"])),
        bls_to_execution_changes=[B.SignedBLSToExecutionChange(
            B.BLSToExecutionChange(c["message"]["validator_index"], _b(c["message"]["from_bls_pubkey"]), _b(c["message"]["to_execution_address"])),
            _b(c["signature"])) for c in b["bls_changes"]])
    blk = B.BeaconBlock(b["slot"], b["proposer_index"], _b(b["parent_root"]), _b(b["state_root"]), body)
    return state, B.SignedBeaconBlock(blk, _b(b["signature"]))


def _set_offsets(b):
    """Index of the first set of each kind in getBlockSignatureSets order."""
    k = {"randao": 0}
    k["proposer_slashing"] = 1
    k["attester_slashing"] = k["proposer_slashing"] + 2 * len(b["proposer_slashings"])
    k["attestation"] = k["attester_slashing"] + 2 * len(b["attester_slashings"])
    k["exit"] = k["attestation"] + len(b["attestations"])
    k["proposer"] = k["exit"] + len(b["voluntary_exits"])
    k["sync"] = k["proposer"] + 1
    k["bls_change"] = k["sync"] + 1
    return k


def corrupt(fix, kind):
    """(block dict, committees dict, index of the set that becomes invalid) for one corruption kind."""
    b = copy.deepcopy(fix["block"])
    com = fix["committees"]
    off = _set_offsets(b)
    if kind == "attestation_member":
        # one committee member replaced by a validator outside the committee: the aggregate pubkey
        # no longer matches the signature
        att = b["attestations"][7]
        a = att["data"]
        ci = att["committee_bits"].index(True) if "committee_bits" in att else a["index"]
        key = "%d,%d" % (a["slot"], ci)
        com = dict(com)
        members = list(com[key])
        v = (members[5] + 1) % N_VALIDATORS
        while v in members:
            v = (v + 1) % N_VALIDATORS
        members[5] = v
        com[key] = members
        return b, com, off["attestation"] + 7
    if kind == "sync_bit":
        bits = b["sync_aggregate"]["bits"]
        i = bits.index(True)
        bits[i] = False  # one participant dropped from the aggregate
        return b, com, off["sync"]
    if kind == "randao":
        b["randao_reveal"] = b["signature"]  # a valid point, signing another root
        return b, com, off["randao"]
    if kind == "proposer":
        r = bytearray(_b(b["body_root"]))
        r[0] ^= 1
        b["body_root"] = r.hex()
        return b, com, off["proposer"]
    if kind == "exit":
        b["voluntary_exits"][0]["message"]["validator_index"] += 1
        return b, com, off["exit"]
    if kind == "bls_change":
        b["bls_changes"][0]["message"]["from_bls_pubkey"] = fix["other_pubkey"]
        return b, com, off["bls_change"]
    if kind == "proposer_slashing":
        ps = b["proposer_slashings"][0]
        ps[1]["signature"] = ps[0]["signature"]
        return b, com, off["proposer_slashing"] + 1
    if kind == "attester_slashing":
        ia = b["attester_slashings"][0][0]
        ia["attesting_indices"] = ia["attesting_indices"][:-1]
        return b, com, off["attester_slashing"]
    if kind == "attestation_agg_bit":
        # electra: one participant of a multi-committee aggregate dropped (its signature still counts it)
        bits = b["attestations"][3]["bits"]
        bits[bits.index(True)] = False
        return b, com, off["attestation"] + 3
    if kind == "attestation_committee_swap":
        # electra: committee_bits name another committee of the same size than the one that signed
        cb = b["attestations"][6]["committee_bits"]
        i, j = cb.index(True), cb.index(False)
        cb[i], cb[j] = False, True
        return b, com, off["attestation"] + 6
    raise KeyError(kind)


CORRUPTIONS = ["attestation_member", "sync_bit", "randao", "proposer", "exit", "bls_change", "proposer_slashing", "attester_slashing"]
CORRUPTIONS_ELECTRA = CORRUPTIONS + ["attestation_agg_bit", "attestation_committee_swap"]
