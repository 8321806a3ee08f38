"""Shared by the gossip-builder tests: tests/golden/gossip_sets.json (tests/golden/make_gossip_fixture.py)
turned into the product builders' inputs, and a hashlib stand-in for the device hasher (CPU tests)."""
import json
import os

from lodestar_amd import gossip_sets as G
from lodestar_amd.signature_sets import AttestationData, BeaconConfig, Checkpoint, Fork

HERE = os.path.dirname(os.path.abspath(__file__))
PATH = os.path.join(HERE, "golden", "gossip_sets.json")


def load():
    return json.load(open(PATH))


def config(fix):
    cfg = fix["config"]
    return BeaconConfig([Fork(n, e, bytes.fromhex(v)) for n, e, v in cfg["forks"]], bytes.fromhex(cfg["gvr"]), cfg["deneb_epoch"])


def gossip_state(fix):
    return G.GossipState(config(fix), fix["state_slot"], fix["sync_committee"], fix.get("next_sync_committee"))


def _data(d):
    return AttestationData(d["slot"], d["index"], bytes.fromhex(d["beacon_block_root"]), Checkpoint(d["source_epoch"], bytes.fromhex(d["source_root"])),
                           Checkpoint(d["target_epoch"], bytes.fromhex(d["target_root"])))


def signed_aggregate(call):
    s = call["signed"]
    m = s["message"]
    a = m["aggregate"]
    att = G.Attestation(a["bits"], _data(a["data"]), bytes.fromhex(a["signature"]), a.get("committee_bits"))
    return G.SignedAggregateAndProof(G.AggregateAndProof(m["aggregator_index"], att, bytes.fromhex(m["selection_proof"])),
                                     bytes.fromhex(s["signature"]))


def signed_contribution(call):
    s = call["signed"]
    m = s["message"]
    c = m["contribution"]
    con = G.SyncCommitteeContribution(c["slot"], bytes.fromhex(c["beacon_block_root"]), c["subcommittee_index"], c["bits"],
                                      bytes.fromhex(c["signature"]))
    return G.SignedContributionAndProof(G.ContributionAndProof(m["aggregator_index"], con, bytes.fromhex(m["selection_proof"])),
                                        bytes.fromhex(s["signature"]))


def sync_message(call):
    m = call["message"]
    return G.SyncCommitteeMessage(m["slot"], bytes.fromhex(m["beacon_block_root"]), m["validator_index"], bytes.fromhex(m["signature"]))


def build(fix, call, hasher):
    """The product builders' sets of one fixture call."""
    if call["kind"] == "aggregate_and_proof":
        return G.aggregate_and_proof_signature_sets(config(fix), signed_aggregate(call), call["attesting_indices"], hasher)
    if call["kind"] == "contribution_and_proof":
        return G.contribution_and_proof_signature_sets(gossip_state(fix), signed_contribution(call), hasher)
    return G.sync_committee_signature_sets(gossip_state(fix), [sync_message(call)], hasher)


class HostHasher:
    """hashlib stand-in for the device hasher's merkle_roots / compute_signing_roots (CPU tests only)."""

    def __init__(self):
        self.calls = []

    def merkle_roots(self, chunks, depth):
        from oracle import ssz_oracle as S
        self.calls.append(("merkle", depth))
        b = bytes(chunks)
        w = 32 << depth
        return [S.merkle_root_fixed([b[i + 32 * k:i + 32 * k + 32] for k in range(1 << depth)], depth) for i in range(0, len(b), w)]

    def compute_signing_roots(self, object_roots, domains, dom_idx=None):
        from oracle import ssz_oracle as S
        self.calls.append(("signing", len(object_roots) // 32))
        b = bytes(object_roots)
        doms = [domains] if isinstance(domains, (bytes, bytearray)) else list(domains)
        return [S.compute_signing_root(b[32 * i:32 * i + 32], doms[dom_idx[i] if dom_idx else 0]) for i in range(len(b) // 32)]


def expected(call):
    return [(e["kind"], e["key"], bytes.fromhex(e["root"])) for e in call["expected_sets"]]


def as_tuples(sets):
    out = []
    for s in sets:
        if hasattr(s, "indices"):
            out.append(("aggregate", list(s.indices), bytes(s.signing_root)))
        else:
            out.append(("single", int(s.index), bytes(s.signing_root)))
    return out
