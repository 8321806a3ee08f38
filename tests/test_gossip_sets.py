"""Gossip-side signature-set builders in index form (lodestar_amd/gossip_sets.py; JS:
addon/gossip_sets.js) against the oracle's restatement (oracle/gossip_oracle.py) and its fixture
tests/golden/gossip_sets.json: validateAggregateAndProof's three sets (aggregateAndProof.ts:211-229,
phase0 and electra AggregateAndProof), validateSyncCommitteeGossipContributionAndProof's three sets
(syncCommitteeContributionAndProof.ts:73-92) and getSyncCommitteeSignatureSet (syncCommittee.ts:10-23).

CPU: the fixture is self-consistent under the oracle; the product builders reproduce every set (kind,
validator indices, signing root) with a hashlib stand-in for the device hasher.  GPU: the same with
the device computing every container root and signing root, and each call -- and each one-set
corruption of it -- verified through GpuBlsVerifier with exactly the oracle's answer.
Parity note -- PARITY UNPINNED for the container roots (phase0 / electra AggregateAndProof,
SyncCommitteeContribution, ContributionAndProof): no reference-held vector records one, so the fixture
is self-consistent under oracle/gossip_oracle.py's restatement, not pinned.  K1 pins the merkleization
rules (uint64 / Bytes48 / container padding); the BitList length mix-in and BitVector packing are
restated from the SSZ spec @chainsafe/ssz 0.11.1 implements."""
import asyncio

import pytest

import gossip_fixture as GF
from oracle import gossip_oracle as GO


@pytest.fixture(scope="module")
def fix():
    return GF.load()


def test_fixture_self_consistent_under_oracle(fix):
    cfg = fix["config"]
    kinds = []
    for call in fix["calls"]:
        if call["kind"] == "aggregate_and_proof":
            ss = GO.aggregate_and_proof_sets(cfg, call["signed"], call["attesting_indices"])
        elif call["kind"] == "contribution_and_proof":
            ss = GO.contribution_and_proof_sets(fix, call["signed"])
        else:
            ss = [GO.sync_committee_message_set(fix, call["message"])]
        assert [(k, key, root) for k, key, root, _ in ss] == GF.expected(call)
        assert call["expected_valid"] is True and all(c["expected_valid"] is False for c in call["corruptions"])
        kinds.append(call["kind"])
    assert kinds.count("aggregate_and_proof") == 2 and "contribution_and_proof" in kinds and "sync_committee_message" in kinds
    assert any(c.get("electra") for c in fix["calls"])


def test_builders_match_oracle_host_hasher(fix):
    for call in fix["calls"]:
        h = GF.HostHasher()
        sets = GF.build(fix, call, h)
        assert GF.as_tuples(sets) == GF.expected(call), call["kind"]
        assert h.calls[-1][0] == "signing" and sum(1 for c in h.calls if c[0] == "signing") == 1  # one signing-root launch per call
    # the signatures are carried through unchanged (set order = the reference's)
    call = fix["calls"][0]
    sets = GF.build(fix, call, GF.HostHasher())
    m = call["signed"]["message"]
    assert [s.signature.hex() for s in sets] == [m["selection_proof"], call["signed"]["signature"], m["aggregate"]["signature"]]


def test_contribution_participants_and_errors(fix):
    from lodestar_amd import gossip_sets as G
    call = [c for c in fix["calls"] if c["kind"] == "contribution_and_proof"][0]
    st = GF.gossip_state(fix)
    sc = GF.signed_contribution(call)
    assert G.contribution_indices(st, sc.message.contribution) == GO.contribution_participants(fix, call["signed"]["message"]["contribution"])
    sc.message.contribution.aggregation_bits = [False] * 128
    with pytest.raises(ValueError, match="NO_PARTICIPANT"):
        G.contribution_and_proof_signature_sets(st, sc, GF.HostHasher())
    far = G.GossipState(st.config, st.slot + 2 * 256 * 32, st.current_sync_committee)
    with pytest.raises(ValueError, match="NO_SYNC_COMMITTEE"):
        far.indexed_sync_committee(st.slot)


@pytest.mark.gpu
def test_gossip_sets_on_gpu(fix):
    """Device hashing of every root, then each call and its corruptions verified on the GPU."""
    from lodestar_amd import GpuBlsVerifier
    v = GpuBlsVerifier(0)
    try:
        pks = [bytes.fromhex(p) for p in fix["pubkeys"]]
        n = fix["world"]["n_validators"]
        assert v.add_pubkeys(0, pks, validate=True) == bytes(len(pks))
        v.replicate_pubkeys(0, len(pks), len(pks), n - len(pks))
        results = []
        for call in fix["calls"]:
            sets = GF.build(fix, call, v)
            assert GF.as_tuples(sets) == GF.expected(call), call["kind"]
            calls = [sets]
            for c in call["corruptions"]:
                bad = list(sets)
                s = bad[c["set"]]
                bad[c["set"]] = type(s)(**dict(s.__dict__, signature=bytes.fromhex(c["signature"])))
                calls.append(bad)
            got = v.verify_signature_sets_multi_sync(calls)
            assert got == [call["expected_valid"]] + [c["expected_valid"] for c in call["corruptions"]], call["kind"]
            results.append(got)

        async def through_queue():  # the reference's call shape: {batchable: true, priority}
            from lodestar_amd.verifier import VerifySignatureOpts
            opts = VerifySignatureOpts(batchable=True, priority=True)
            sets = GF.build(fix, fix["calls"][0], v)
            return await v.verify_signature_sets(sets, opts)
        assert asyncio.run(through_queue()) is True
    finally:
        v.close_sync()
