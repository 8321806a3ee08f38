"""GPU parity: the gfx950 path (through the C ABI) against the golden fixtures made by the oracle.

Run on an MI355X: python -m pytest tests -m gpu
"""
import hashlib
import json
import os

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = json.load(open(os.path.join(HERE, "golden", "fixtures.json")))


@pytest.fixture(scope="module")
def v():
    from lodestar_amd import GpuBlsVerifier
    ver = GpuBlsVerifier(0)
    st = ver.add_pubkeys(0, [bytes.fromhex(p) for p in FIX["keys"]["pks"]], validate=True)
    assert st == bytes(len(FIX["keys"]["pks"]))
    yield ver
    ver.close_sync()


def _sets(case):
    from lodestar_amd import AggregatedSignatureSet, SingleSignatureSet
    out = []
    for s in case["sets"]:
        root, sig = bytes.fromhex(s["msg"]), bytes.fromhex(s["sig"])
        if "raw_pk" in s:
            out.append(SingleSignatureSet(0, root, sig, pubkey=bytes.fromhex(s["raw_pk"])))
        elif len(s["indices"]) == 1:
            out.append(SingleSignatureSet(s["indices"][0], root, sig))
        else:
            out.append(AggregatedSignatureSet(s["indices"], root, sig))
    return out


@pytest.mark.parametrize("case", FIX["verify_sets"], ids=[c["name"] for c in FIX["verify_sets"]])
def test_verify_sets_fixture(v, case):
    from lodestar_amd import EmptyAggregateError
    sets = _sets(case)
    if case["expected"] == "reject":
        with pytest.raises(EmptyAggregateError):
            v.verify_signature_sets_sync(sets)
    else:
        assert v.verify_signature_sets_sync(sets) == case["expected"]


@pytest.mark.parametrize("case", FIX["same_message"], ids=[c["name"] for c in FIX["same_message"]])
def test_same_message_fixture(v, case):
    sets = [(i, bytes.fromhex(s)) for i, s in zip(case["indices"], case["sigs"])]
    assert v.verify_signature_sets_same_message_sync(sets, bytes.fromhex(case["msg"])) == case["expected"]


def test_same_message_multi_one_pass(v):
    calls = [([(i, bytes.fromhex(s)) for i, s in zip(c["indices"], c["sigs"])], bytes.fromhex(c["msg"]))
             for c in FIX["same_message"]]
    res = v.verify_same_message_multi_sync(calls)
    assert res == [c["expected"] for c in FIX["same_message"]]


@pytest.mark.parametrize("case", FIX["aggregate_pubkeys"], ids=lambda c: str(c["indices"]))
def test_aggregate_pubkeys_fixture(v, case):
    assert v.aggregate_pubkeys(case["indices"]).hex() == case["expected"]


def test_aggregate_pubkeys_empty_rejects(v):
    from lodestar_amd import EmptyAggregateError
    with pytest.raises(EmptyAggregateError):
        v.aggregate_pubkeys([])


def test_hash_to_g2_fixture(v):
    outs = v.util_hash_to_g2([bytes.fromhex(c["msg"]) for c in FIX["hash_to_g2"]])
    assert [o.hex() for o in outs] == [c["expected"] for c in FIX["hash_to_g2"]]


def test_keygen_and_sign_k1(v):
    """K1: interop key 0 deposit signature (genesisState.test.ts:50-54) produced on the GPU."""
    sk = int(FIX["keys"]["sks"][0], 16).to_bytes(32, "big")
    assert v.util_sk_to_pk([sk])[0].hex() == FIX["keys"]["pks"][0]
    pk = bytes.fromhex(FIX["keys"]["pks"][0])
    H = lambda b: hashlib.sha256(b).digest()
    wc = bytearray(H(pk)); wc[0] = 0
    obj = H(H(H(pk[:32] + pk[32:] + bytes(16)) + bytes(wc)) + H((32000000000).to_bytes(8, "little") + bytes(56)))
    root = H(obj + bytes([3, 0, 0, 0]) + H(bytes([0, 0, 0, 1]) + bytes(60))[:28])
    sig = v.util_sign([sk], [0], [root])[0]
    assert sig.hex() == ("a95af8ff0f8c06af4d29aef05ce865f85f82df42b606008ec5b1bcb42b17ae47f4b78cdce1db31ce32d18f42a6b296b4"
                         "014a2164981780e56b5a40d7723c27b8423173e58fa36f075078b177634f66351412b867c103f532aedd50bcd9b98446")


def test_async_interface(v):
    import asyncio
    from lodestar_amd import VerifySignatureOpts
    case = FIX["verify_sets"][0]
    sm = FIX["same_message"][1]

    async def go():
        a = v.verify_signature_sets(_sets(case), VerifySignatureOpts(batchable=True))
        b = v.verify_signature_sets_same_message([(i, bytes.fromhex(s)) for i, s in zip(sm["indices"], sm["sigs"])],
                                                 bytes.fromhex(sm["msg"]), VerifySignatureOpts(priority=True))
        return await asyncio.gather(a, b)
    ra, rb = asyncio.run(go())
    assert ra == case["expected"] and rb == sm["expected"]


def test_verify_sets_multi_one_pass(v):
    """Every verify_sets fixture as one call of ONE device pass (gbv_verify_sets_multi): each call
    keeps its own answer, and the call with an empty aggregate rejects alone."""
    from lodestar_amd import EmptyAggregateError
    cases = FIX["verify_sets"]
    res = v.verify_signature_sets_multi_sync([_sets(c) for c in cases])
    for c, r in zip(cases, res):
        if c["expected"] == "reject":
            assert isinstance(r, EmptyAggregateError), c["name"]
        else:
            assert r == c["expected"], c["name"]


def test_staged_signature_sets_reverify(v):
    """gbv_vs_batch: the same staged calls verified three times (fresh random scalars each time)."""
    cases = [c for c in FIX["verify_sets"] if c["expected"] != "reject"]
    st = v.stage_signature_sets([_sets(c) for c in cases])
    try:
        want = [1 if c["expected"] else 0 for c in cases]
        for _ in range(3):
            assert st.verify() == want
        ms = v.vs_last_kernel_ms()
        assert len(ms) == 4 and ms[1] > 0
    finally:
        st.close()


@pytest.mark.parametrize("case", FIX["aggregate_pubkeys"], ids=lambda c: str(c["indices"]))
def test_aggregate_serialized_pubkeys_fixture(v, case):
    """aggregateSerializedPublicKeys (syncCommittee.ts:37) over the same keys as bytes."""
    pks = [bytes.fromhex(FIX["keys"]["pks"][i]) for i in case["indices"]]
    assert v.aggregate_serialized_pubkeys(pks).hex() == case["expected"]
    assert v.aggregate_serialized_pubkeys(pks, validate=True).hex() == case["expected"]


def test_aggregate_serialized_pubkeys_errors(v):
    from lodestar_amd import EmptyAggregateError
    from lodestar_amd._native import BadPointError
    pk0 = bytes.fromhex(FIX["keys"]["pks"][0])
    with pytest.raises(EmptyAggregateError):
        v.aggregate_serialized_pubkeys([])
    with pytest.raises(BadPointError):
        v.aggregate_serialized_pubkeys([pk0, bytes(48)])  # no compression flag
    inf = bytes([0xC0]) + bytes(47)
    # infinity deserializes without validation and contributes nothing; validation rejects it
    assert v.aggregate_serialized_pubkeys([pk0, inf]) == pk0
    with pytest.raises(BadPointError):
        v.aggregate_serialized_pubkeys([pk0, inf], validate=True)


def test_signatures_validate_recompresses(v):
    """Signature.fromBytes(sig, true): accepted signatures recompress byte-identically; the
    malformed / infinity encodings of the fixtures are rejected with their blst error class."""
    sigs = [bytes.fromhex(s["sig"]) for c in FIX["verify_sets"] for s in c["sets"] if len(s["sig"]) == 192]
    st, out = v.signatures_validate(sigs)
    good = [i for i in range(len(sigs)) if st[i] == 0]
    assert len(good) >= len(sigs) // 2
    for i in good:
        assert out[i] == sigs[i]
    st, _ = v.signatures_validate([bytes([10]) * 96, bytes([0xC0]) + bytes(95), bytes(96)])
    assert list(st) == [1, 4, 1]  # GBV_PT_BAD_ENCODING, GBV_PT_INFINITY, GBV_PT_BAD_ENCODING
