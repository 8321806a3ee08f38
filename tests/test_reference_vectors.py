"""Vectors the reference's own tests hold (tests/golden/reference_vectors.json, extracted by
tests/golden/extract_reference_vectors.py):
  * the 100 interop pubkeys (state-transition/test-cache/interop-pubkeys.json) -- KeyGen + compression;
  * K2 (cli/test/utils/cachedKeys.ts:15-26) and K6 (beacon-node/test/utils/validator.ts:18);
  * the 53 BLS signatures of 4 mainnet blocks (beacon-node/test/unit/sync/backfill/blocks.json) --
    accepted by blst on mainnet, so Signature.fromBytes(sig, true) must accept each and the point must
    recompress to the same bytes;
  * pubkey ingest (f1: syncPubkeys / addFinalizedPubkey / the deposit check
    PublicKey.fromBytes(pk, true), block/processDeposit.ts:163-166) with every reject status.
"""
import json
import os

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
VEC = json.load(open(os.path.join(HERE, "golden", "reference_vectors.json")))


def test_oracle_interop_pubkeys():
    from oracle import bls_oracle as O
    for i in range(16):  # all 100 on the GPU below; the pure-Python KeyGen is ~0.15 s per key
        assert O.g1_compress(O.sk_to_pk(O.interop_secret_key(i))).hex() == VEC["interop_pubkeys"][i]


def test_oracle_k2_keygen():
    from oracle import bls_oracle as O
    for i, (sk, pk) in enumerate(zip(VEC["cached_keys"]["sks"], VEC["cached_keys"]["pks"])):
        k = O.keygen(bytes([0xAA + i]) * 32)
        assert k == int(sk, 16)
        assert O.g1_compress(O.sk_to_pk(k)).hex() == pk


def test_oracle_mainnet_signatures_roundtrip():
    from oracle import bls_oracle as O
    for s in VEC["mainnet_signatures"]:
        b = bytes.fromhex(s["sig"])
        pt = O.signature_from_bytes(b, True)
        assert O.g2_compress(pt) == b, s["where"]


def test_oracle_reject_cases_and_k6():
    from oracle import bls_oracle as O
    assert O.pubkey_from_bytes(bytes.fromhex(VEC["validator_pubkey"]), validate=True) is not None
    names = {c["name"]: c for c in VEC["g1_reject_cases"]}
    assert names["not_in_group"]["status_validate"] == 3 and names["not_in_group"]["status_no_validate"] == 0
    assert names["infinity"]["status_validate"] == 4


# ---- GPU ------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def v():
    from lodestar_amd import GpuBlsVerifier
    v = GpuBlsVerifier(0)
    yield v
    v.close_sync()


@pytest.mark.gpu
def test_gpu_interop_and_k2_keygen(v):
    from oracle import bls_oracle as O
    sks = [O.interop_secret_key(i).to_bytes(32, "big") for i in range(100)]
    assert [p.hex() for p in v.util_sk_to_pk(sks)] == VEC["interop_pubkeys"]
    k2 = [bytes.fromhex(s) for s in VEC["cached_keys"]["sks"]]
    assert [p.hex() for p in v.util_sk_to_pk(k2)] == VEC["cached_keys"]["pks"]


@pytest.mark.gpu
def test_gpu_pubkey_ingest_statuses(v):
    """gbv_pubkeys_append with and without validation: every reference / K2 / K6 key accepted,
    every reject case with the blst error class the oracle assigns.  One documented difference: an
    infinity key without validation -- accepted by blst's PublicKey.fromBytes(pk) -- is reported as
    GBV_PT_INFINITY and its slot marked unusable (index2pubkey holds deposit-validated keys only,
    processDeposit.ts:163-166, so it never occurs there)."""
    good = [bytes.fromhex(p) for p in VEC["interop_pubkeys"] + VEC["cached_keys"]["pks"] + [VEC["validator_pubkey"]]]
    assert v.add_pubkeys(0, good, validate=True) == bytes(len(good))
    base = len(good)
    cases = VEC["g1_reject_cases"]
    pks = [bytes.fromhex(c["pk"]) for c in cases]
    st_v = v.add_pubkeys(base, pks, validate=True)
    st_n = v.add_pubkeys(base + len(pks), pks, validate=False)
    for c, a, b in zip(cases, st_v, st_n):
        assert a == c["status_validate"], c["name"]
        want_n = 4 if c["name"] == "infinity" else c["status_no_validate"]
        assert b == want_n, c["name"]
    # a rejected slot is unusable: aggregating over it is an argument error, a valid one works
    from lodestar_amd import GbvError
    with pytest.raises(GbvError):
        v.aggregate_pubkeys([0, base])
    assert v.aggregate_pubkeys([0]).hex() == VEC["interop_pubkeys"][0]


@pytest.mark.gpu
def test_gpu_mainnet_signatures_validate_and_recompress(v):
    sigs = [bytes.fromhex(s["sig"]) for s in VEC["mainnet_signatures"]]
    assert len(sigs) == 53
    st, out = v.signatures_validate(sigs)
    assert st == bytes(len(sigs))
    assert out == sigs
