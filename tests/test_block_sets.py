"""C4: getBlockSignatureSets in index form (lodestar_amd/signature_sets.py) and the
full block through verifySignatureSets.

CPU: the product builders against the oracle's independent restatement (oracle/block_oracle.py),
set by set -- kind, validator indices / raw pubkey, signing root -- with the signing roots hashed by a
host stand-in for the device hasher (oracle SSZ, test infrastructure only).
GPU: the same builders with the device hasher (gbv_attestation_signing_roots / gbv_signing_roots),
then the block verified on the device: true for the fixture block, false for every corruption kind
("one invalid member in turn for each set kind"), each corruption checked false by the oracle when
the fixture was generated (tests/golden/make_c4_fixture.py).
"""
import hashlib
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import c4_block as C  # noqa: E402

FIX = C.load()
FIXE = C.load(electra=True)  # electra: 8 attestations over up to 64 committees each (committee_bits)
R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


class HostHasher:
    """The two hasher calls the builders make, on the CPU with the oracle's SSZ (tests only)."""

    def __init__(self):
        from oracle import ssz_oracle
        self.S = ssz_oracle
        self.calls = []

    def attestation_data_signing_roots(self, datas, domains, dom_idx):
        self.calls.append(("att", len(datas) // 128))
        return [self.S.attestation_signing_root(datas[128 * i:128 * i + 128], domains[dom_idx[i]]) for i in range(len(datas) // 128)]

    def compute_signing_roots(self, roots, domains, dom_idx):
        self.calls.append(("roots", len(roots) // 32))
        return [self.S.compute_signing_root(roots[32 * i:32 * i + 32], domains[dom_idx[i]]) for i in range(len(roots) // 32)]


def _as_expected(sets):
    from lodestar_amd import AggregatedSignatureSet
    out = []
    for s in sets:
        if isinstance(s, AggregatedSignatureSet):
            out.append({"kind": "aggregate", "key": list(s.indices), "root": s.signing_root.hex()})
        elif s.pubkey is not None:
            out.append({"kind": "raw", "key": s.pubkey.hex(), "root": s.signing_root.hex()})
        else:
            out.append({"kind": "single", "key": s.index, "root": s.signing_root.hex()})
    return out


def test_builders_match_oracle_restatement():
    from lodestar_amd.signature_sets import get_block_signature_sets
    state, block = C.to_objects(FIX)
    h = HostHasher()
    sets = get_block_signature_sets(state, block, h)
    assert _as_expected(sets) == FIX["expected_sets"]
    # two batched hasher calls for the whole block: attestation data, everything else
    assert sorted(c[0] for c in h.calls) == ["att", "roots"]
    assert dict(h.calls)["att"] == 128 + 2  # 128 attestations + the attester slashing's two
    # signatures travel unchanged, in reference order
    assert bytes(sets[0].signature).hex() == FIX["block"]["randao_reveal"]
    assert bytes(sets[-3].signature).hex() == FIX["block"]["signature"]


def test_electra_builders_match_oracle_restatement():
    """getAttestingIndices from electra on (epochCache.ts:953-973): the committees of committee_bits
    concatenated and intersected with the aggregation bits -- aggregates of ~1-4 k validators."""
    from lodestar_amd.signature_sets import get_block_signature_sets
    state, block = C.to_objects(FIXE)
    h = HostHasher()
    sets = get_block_signature_sets(state, block, h)
    assert _as_expected(sets) == FIXE["expected_sets"]
    assert dict(h.calls)["att"] == 8 + 2
    sizes = [len(s.indices) for s in sets[5:13]]
    assert min(sizes) >= 1000 and max(sizes) == 64 * 64, sizes
    # the same block read with the pre-electra rule fails (aggregation bits span many committees)
    from lodestar_amd import signature_sets as B
    with pytest.raises(ValueError):
        state.attesting_indices(block.message.body.attestations[0], B.FORK_ORDER.index("deneb"))


def test_electra_attestation_without_committee_bits_is_rejected():
    from lodestar_amd import signature_sets as B
    state, block = C.to_objects(FIXE)
    att = block.message.body.attestations[0]
    electra = B.FORK_ORDER.index("electra")
    with pytest.raises(ValueError):
        state.attesting_indices(B.Attestation(att.aggregation_bits, att.data, att.signature, None), electra)
    with pytest.raises(ValueError):  # getBeaconCommittees([]) throws
        state.attesting_indices(B.Attestation([], att.data, att.signature, [False] * 64), electra)


@pytest.mark.parametrize("kind", C.CORRUPTIONS_ELECTRA)
def test_electra_builders_track_corruptions(kind):
    from lodestar_amd.signature_sets import get_block_signature_sets
    from oracle import block_oracle as BO
    b2, com2, k = C.corrupt(FIXE, kind)
    state, block = C.to_objects(FIXE, b2, com2)
    got = _as_expected(get_block_signature_sets(state, block, HostHasher()))
    want = [{"kind": kd, "key": key.hex() if kd == "raw" else key, "root": root.hex()} for kd, key, root, _ in BO.block_signature_sets(FIXE, b2, com2)]
    assert got == want
    assert FIXE["corruptions"][kind] == {"set": k, "valid": False}


@pytest.mark.parametrize("kind", C.CORRUPTIONS)
def test_builders_track_corruptions(kind):
    """Each corruption changes exactly the set the oracle says becomes invalid."""
    from lodestar_amd.signature_sets import get_block_signature_sets
    from oracle import block_oracle as BO
    b2, com2, k = C.corrupt(FIX, kind)
    state, block = C.to_objects(FIX, b2, com2)
    got = _as_expected(get_block_signature_sets(state, block, HostHasher()))
    want = [{"kind": kd, "key": key.hex() if kd == "raw" else key, "root": root.hex()} for kd, key, root, _ in BO.block_signature_sets(FIX, b2, com2)]
    assert got == want
    assert FIX["corruptions"][kind] == {"set": k, "valid": False}


def test_skip_proposer_and_no_sync_participation():
    from lodestar_amd.signature_sets import G2_POINT_AT_INFINITY, get_block_signature_sets
    import copy
    state, block = C.to_objects(FIX)
    sets = get_block_signature_sets(state, block, HostHasher(), skip_proposer_signature=True)
    assert len(sets) == len(FIX["expected_sets"]) - 1
    b2 = copy.deepcopy(FIX["block"])
    b2["sync_aggregate"]["bits"] = [False] * 512
    b2["sync_aggregate"]["signature"] = G2_POINT_AT_INFINITY.hex()
    state, block = C.to_objects(FIX, b2)
    assert len(get_block_signature_sets(state, block, HostHasher())) == len(FIX["expected_sets"]) - 1
    b2["sync_aggregate"]["signature"] = FIX["block"]["signature"]
    state, block = C.to_objects(FIX, b2)
    with pytest.raises(ValueError):  # processSyncCommittee.ts:100: "Empty sync committee signature is not infinity"
        get_block_signature_sets(state, block, HostHasher())


# ---- GPU ------------------------------------------------------------------------------------------
def _sk(i):
    d = hashlib.sha256(i.to_bytes(32, "little")).digest()
    return (int.from_bytes(d, "little") % R_ORDER).to_bytes(32, "big")


@pytest.fixture(scope="module")
def gpu():
    from lodestar_amd import GpuBlsVerifier
    v = GpuBlsVerifier(0)
    pks = v.util_sk_to_pk([_sk(i) for i in range(C.N_KEYS)])
    # the device KeyGen of all 1024 interop keys equals the oracle's (fixture), byte for byte
    assert [p.hex() for p in pks] == FIX["pubkeys"]
    assert v.add_pubkeys(0, pks, validate=True) == bytes(C.N_KEYS)
    v.replicate_pubkeys(0, C.N_KEYS, C.N_KEYS, C.N_VALIDATORS - C.N_KEYS)
    assert v.pubkey_count == C.N_VALIDATORS
    yield v
    v.close_sync()


@pytest.mark.gpu
def test_gpu_block_signing_roots_match_oracle(gpu):
    from lodestar_amd.signature_sets import get_block_signature_sets
    state, block = C.to_objects(FIX)
    assert _as_expected(get_block_signature_sets(state, block, gpu)) == FIX["expected_sets"]


@pytest.mark.gpu
def test_gpu_block_verifies(gpu):
    from lodestar_amd.signature_sets import get_block_signature_sets
    state, block = C.to_objects(FIX)
    sets = get_block_signature_sets(state, block, gpu)
    assert gpu.verify_signature_sets_sync(sets) is FIX["expected_valid"] is True


@pytest.mark.gpu
def test_gpu_block_corruptions_one_pass(gpu):
    """The clean block and every corruption as separate verifySignatureSets calls of ONE device pass
    (range sync: one call per block, verifyBlocksSignatures.ts:32-51): only the clean one is true."""
    from lodestar_amd.signature_sets import get_block_signature_sets
    calls = []
    for kind in [None] + C.CORRUPTIONS:
        if kind is None:
            state, block = C.to_objects(FIX)
        else:
            b2, com2, _ = C.corrupt(FIX, kind)
            state, block = C.to_objects(FIX, b2, com2)
        calls.append(get_block_signature_sets(state, block, gpu))
    res = gpu.verify_signature_sets_multi_sync(calls)
    assert res == [True] + [FIX["corruptions"][k]["valid"] for k in C.CORRUPTIONS]
    assert res == [True] + [False] * len(C.CORRUPTIONS)


@pytest.mark.gpu
def test_gpu_range_sync_segment_staged(gpu):
    """A range-sync segment: 16 copies of the block (8 clean, 8 with the sync-bit corruption) staged
    as one gbv_vs_batch and verified twice; get_blocks_signature_sets hashes every block's roots in
    two device calls."""
    from lodestar_amd.signature_sets import get_blocks_signature_sets
    state, block = C.to_objects(FIX)
    b2, com2, _ = C.corrupt(FIX, "sync_bit")
    _, bad_block = C.to_objects(FIX, b2, com2)
    blocks = [block if i % 2 == 0 else bad_block for i in range(16)]
    calls = get_blocks_signature_sets(state, blocks, gpu)
    assert [len(c) for c in calls] == [138] * 16
    st = gpu.stage_signature_sets(calls)
    try:
        for _ in range(2):
            assert st.verify() == [1 if i % 2 == 0 else 0 for i in range(16)]
    finally:
        st.close()


@pytest.mark.gpu
def test_gpu_electra_block_and_corruptions_one_pass(gpu):
    """The electra block (aggregates of ~1-4 k validators: k_vs_agg_big slices) and each of its
    corruptions as calls of one device pass: only the clean block is true (oracle-made fixture)."""
    from lodestar_amd.signature_sets import get_block_signature_sets
    calls = []
    for kind in [None] + C.CORRUPTIONS_ELECTRA:
        b2, com2 = (None, None) if kind is None else C.corrupt(FIXE, kind)[:2]
        state, block = C.to_objects(FIXE, b2, com2)
        calls.append(get_block_signature_sets(state, block, gpu))
    assert _as_expected(calls[0]) == FIXE["expected_sets"]
    res = gpu.verify_signature_sets_multi_sync(calls)
    assert res == [FIXE["expected_valid"]] + [FIXE["corruptions"][k]["valid"] for k in C.CORRUPTIONS_ELECTRA]
    assert res == [True] + [False] * len(C.CORRUPTIONS_ELECTRA)
    # the electra block alone (latency form: one call) and its aggregate pubkeys byte-exact
    assert gpu.verify_signature_sets_sync(calls[0]) is True
    agg = calls[0][5]
    from oracle import bls_oracle as O
    want = O.g1_compress(O.aggregate_pubkeys([O.g1_decompress(bytes.fromhex(FIXE["pubkeys"][v % C.N_KEYS])) for v in agg.indices]))
    assert gpu.aggregate_pubkeys(agg.indices) == want


@pytest.mark.gpu
def test_gpu_mixed_aggregate_sizes(gpu):
    """Sets of 1, 2, 127, 512, 1023 (small kernel) and 1024, 2048, 2049, 5000, 8192, 8193, 20000
    (sliced kernel: one slice up to agg_slice = 8192 members, then several) members in one pass,
    each signed by the sum of its members' keys; then one member swapped."""
    from lodestar_amd import AggregatedSignatureSet, SingleSignatureSet
    import numpy as np
    rng = np.random.Generator(np.random.PCG64(0xA66))
    sizes = [1, 2, 127, 512, 1023, 1024, 2048, 2049, 5000, 8192, 8193, 20000]
    sks = [int.from_bytes(_sk(i), "big") for i in range(C.N_KEYS)]
    msgs = [hashlib.sha256(b"agg-size" + bytes([k])).digest() for k in range(len(sizes))]
    members = [rng.choice(C.N_VALIDATORS, size=n, replace=False).tolist() for n in sizes]
    agg_sk = [(sum(sks[v % C.N_KEYS] for v in m) % R_ORDER).to_bytes(32, "big") for m in members]
    sigs = gpu.util_sign(agg_sk, list(range(len(sizes))), msgs)
    sets = [SingleSignatureSet(m[0], msgs[k], sigs[k]) if len(m) == 1 else AggregatedSignatureSet(m, msgs[k], sigs[k])
            for k, m in enumerate(members)]
    calls = [[s] for s in sets] + [sets]
    bad = []
    for k in range(1, len(sizes)):
        m = list(members[k])
        m[-1] = (m[-1] + 1) % C.N_VALIDATORS  # another validator (another key: 1024 keys, consecutive indices)
        bad.append([AggregatedSignatureSet(m, msgs[k], sigs[k])])
    res = gpu.verify_signature_sets_multi_sync(calls + bad)
    assert res == [True] * (len(sizes) + 1) + [False] * (len(sizes) - 1)


@pytest.mark.gpu
def test_gpu_sync_committee_aggregate_512(gpu):
    """f2: the 512-member sync-committee aggregate pubkey, byte-exact against the oracle -- from the
    HBM table (aggregatePublicKeys over indices) and from serialized keys
    (aggregateSerializedPublicKeys, processSyncCommitteeUpdates.ts:35)."""
    members = FIX["sync_committee"]
    assert gpu.aggregate_pubkeys(members).hex() == FIX["sync_committee_aggregate"]
    ser = [bytes.fromhex(FIX["pubkeys"][m % C.N_KEYS]) for m in members]
    assert gpu.aggregate_serialized_pubkeys(ser).hex() == FIX["sync_committee_aggregate"]
    assert gpu.aggregate_serialized_pubkeys(ser, validate=True).hex() == FIX["sync_committee_aggregate"]
