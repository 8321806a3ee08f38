"""C3: 128-member committee aggregates gathered from the HBM-resident
index2pubkey table of 2^20 validators, >= 10k sets, through verifySignatureSets.

Expected booleans hold by construction (each aggregate signature is the device signature of the
summed interop secret keys -- util_sign is pinned bit-exactly by K1 -- except the injected ones);
three sets are re-checked by the CPU oracle from the device pubkeys, which
tests/test_block_sets.py pins against the oracle's KeyGen for all 1024 keys.
"""
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
N_KEYS = 1024
N_TABLE = 1 << 20
N_SETS = 10240
PER_CALL = 128


def _sk_int(i):
    d = hashlib.sha256(i.to_bytes(32, "little")).digest()
    return int.from_bytes(d, "little") % R_ORDER


@pytest.fixture(scope="module")
def c3():
    from lodestar_amd import AggregatedSignatureSet, GpuBlsVerifier
    v = GpuBlsVerifier(0)
    sks = [_sk_int(i) for i in range(N_KEYS)]
    pks = v.util_sk_to_pk([s.to_bytes(32, "big") for s in sks])
    assert v.add_pubkeys(0, pks) == bytes(N_KEYS)
    v.replicate_pubkeys(0, N_KEYS, N_KEYS, N_TABLE - N_KEYS)
    rng = np.random.Generator(np.random.PCG64(0x1D5))
    committees = [rng.choice(N_TABLE, size=128, replace=False) for _ in range(N_SETS)]
    msgs = [hashlib.sha256(b"gbv-c3" + i.to_bytes(4, "little")).digest() for i in range(N_SETS)]
    agg_sk = [(sum(sks[int(x) % N_KEYS] for x in c) % R_ORDER).to_bytes(32, "big") for c in committees]
    sigs = v.util_sign(agg_sk, list(range(N_SETS)), msgs)
    sets = [AggregatedSignatureSet(c.tolist(), msgs[i], sigs[i]) for i, c in enumerate(committees)]
    yield v, sets, pks
    v.close_sync()


def test_c3_all_valid_and_injected(c3):
    from lodestar_amd import AggregatedSignatureSet
    v, sets, _ = c3
    calls = [list(sets[i:i + PER_CALL]) for i in range(0, N_SETS, PER_CALL)]
    assert len(calls) == 80
    assert v.verify_signature_sets_multi_sync(calls) == [True] * 80
    ms = v.vs_last_kernel_ms()
    assert ms[0] > 0  # the wave-per-set gather kernel ran
    bad = [list(c) for c in calls]
    s = bad[3][17]  # one committee member replaced by a validator outside the committee
    idx = list(s.indices)
    idx[40] = (idx[40] + 1) % N_TABLE if (idx[40] + 1) % N_TABLE not in idx else (idx[40] + 7) % N_TABLE
    bad[3][17] = AggregatedSignatureSet(idx, s.signing_root, s.signature)
    s = bad[11][0]  # a valid aggregate signature over another message
    bad[11][0] = AggregatedSignatureSet(s.indices, bad[11][1].signing_root, s.signature)
    s = bad[42][127]  # malformed signature (bls.test.ts:79 pattern)
    bad[42][127] = AggregatedSignatureSet(s.indices, s.signing_root, bytes([10]) * 96)
    s = bad[60][64]  # infinity signature
    bad[60][64] = AggregatedSignatureSet(s.indices, s.signing_root, bytes([0xC0]) + bytes(95))
    s = bad[79][5]  # signature of the right message by a committee one member short
    bad[79][5] = AggregatedSignatureSet(list(s.indices)[:-1], s.signing_root, s.signature)
    want = [c not in (3, 11, 42, 60, 79) for c in range(80)]
    assert v.verify_signature_sets_multi_sync(bad) == want


def test_c3_staged_reverify(c3):
    v, sets, _ = c3
    calls = [list(sets[i:i + PER_CALL]) for i in range(0, N_SETS, PER_CALL)]
    st = v.stage_signature_sets(calls)
    try:
        for _ in range(2):
            assert st.verify() == [1] * 80
    finally:
        st.close()


def test_c3_oracle_spot_check(c3):
    from oracle import bls_oracle as O
    v, sets, pks = c3
    for i in (0, 4321, N_SETS - 1):
        s = sets[i]
        agg = O.aggregate_pubkeys([O.g1_decompress(pks[x % N_KEYS]) for x in s.indices])
        assert O.set_is_valid(agg, s.signing_root, s.signature)
        # and the device's aggregatePublicKeys of the same committee is byte-identical
        assert v.aggregate_pubkeys(list(s.indices)) == O.g1_compress(agg)


def test_c3_large_pass_thread_forms(c3):
    """A pass of 40 960 sets (the fixture's 80 calls four times over): above the 16 384-set bound of
    the split signature/pubkey form and the 32 768-set bound of the lane-pair Miller values, so the
    throughput kernels run -- k_vs_hash_sig with both roles, k_vs_miller one thread per set, the chunk
    checks without precomputed (-g1, sum) values -- with a bad pubkey and a bad signature placed in
    the last copy."""
    from lodestar_amd import AggregatedSignatureSet
    v, sets, _ = c3
    calls = [list(sets[i:i + PER_CALL]) for i in range(0, N_SETS, PER_CALL)] * 4
    assert sum(len(c) for c in calls) == 4 * N_SETS
    assert v.verify_signature_sets_multi_sync(calls) == [True] * 320
    bad = [list(c) for c in calls]
    s = bad[250][9]  # committee one member short
    bad[250][9] = AggregatedSignatureSet(list(s.indices)[:-1], s.signing_root, s.signature)
    s = bad[319][127]  # malformed signature bytes
    bad[319][127] = AggregatedSignatureSet(s.indices, s.signing_root, bytes([10]) * 96)
    assert v.verify_signature_sets_multi_sync(bad) == [c not in (250, 319) for c in range(320)]

