"""Pin the CPU oracle (oracle/bls_oracle.py) against the reference's in-repo known answers.

K1..K6 are listed in SURVEY.md section 8(c).  Nothing here touches the GPU or the product package.
"""
import hashlib

import pytest

from oracle import bls_oracle as o

K1_PK = "a99a76ed7796f7be22d5b7e85deeb7c5677e88e511e0b337618f8c4eb61349b4bf2d153f649f7b53359fe8b94a38e44c"
K1_WC = "00fad2a6bfb0e7f1f0f45460944fbd8dfa7f37da06a4d13b3983cc90bb46963b"
K1_SIG = ("a95af8ff0f8c06af4d29aef05ce865f85f82df42b606008ec5b1bcb42b17ae47f4b78cdce1db31ce32d18f42a6b296b4"
          "014a2164981780e56b5a40d7723c27b8423173e58fa36f075078b177634f66351412b867c103f532aedd50bcd9b98446")
# cli/test/utils/cachedKeys.ts:15-26
K2_PKS = [
    "8be678633e927aa0435addad5dcd5283fef6110d91362519cd6d43e61f6c017d724fa579cc4b2972134e050b6ba120c0",
    "8e602f8ec17777c22f465f9b4707c2840647790f15f5c33bd8850f274d5c320850105639960ae4effe57aa5dd279bb98",
    "832a777fe5d89724583bcce5b4794d0b38be419a2daed09d7ee6af2c7c09465e0e2cd07a305c38e59e83e211e8ded246",
    "8076b9d469d71902e06cce3af0528c190850d3dabfb8314eba1ef4eb789131de0dd75d2fe4b7964f347bfe61597cde54",
]
K2_SKS = [
    "0e5bd52621b6a8956086dcf0ecc89f0cdca56cebb2a8516c2d4252a9867fc551",
    "19773a731561958a4f257b85af81769bcb1146476936c4d9add796d4d3fda020",
    "6c9e69a6781538c945ead231aecbec9cf6ca3500df59bc85f711fc97a768694e",
    "2948f046357e74993187a6ef40acb961911c52ac7a4257babe6af197f447e892",
]
# beacon-node/test/unit/chain/opPools/attestationPool.test.ts:10-13
K4_SIG = ("b2afb700f6c561ce5e1b4fedaec9d7c06b822d38c720cf588adfda748860a940adf51634b6788f298c552de40183b5a2"
          "03b2bbe8b7dd147f0bb5bc97080a12efbb631c8888cb31a99cc4706eb3711865b8ea818c10126e4d818b542e9dbf9ae8")
# beacon-node/test/utils/validator.ts:18
K6_PK = "84105a985058fc8740a48bf1ede9d223ef09e8c6b1735ba0a55cf4a9ff2ff92376b778798365e488dab07a652eb04576"


def deposit_signing_root(pk_bytes, fork_version=b"\x00\x00\x00\x01"):
    """SSZ hash_tree_root(DepositMessage) + computeDomain(DOMAIN_DEPOSIT, GENESIS_FORK_VERSION, ZERO_HASH).

    The reference's unit/e2e tests run with LODESTAR_PRESET=minimal (beacon-node/test/globalSetup.ts:7-9),
    so GENESIS_FORK_VERSION = 0x00000001 (config/src/chainConfig/configs/minimal.ts:26)."""
    H = lambda b: hashlib.sha256(b).digest()
    wc = bytearray(H(pk_bytes))
    wc[0] = 0
    pk_root = H(pk_bytes[:32] + pk_bytes[32:] + bytes(16))
    amount = (32000000000).to_bytes(8, "little") + bytes(24)
    obj_root = H(H(pk_root + bytes(wc)) + H(amount + bytes(32)))
    fork_data_root = H(fork_version + bytes(28) + bytes(32))
    domain = bytes([3, 0, 0, 0]) + fork_data_root[:28]
    return bytes(wc), H(obj_root + domain)


def test_generators():
    assert o.g1_on_curve(o.G1_GEN) and o.g2_on_curve(o.G2_GEN)
    assert o.g1_in_subgroup_naive(o.G1_GEN) and o.g2_in_subgroup_naive(o.G2_GEN)


def test_k1_interop_deposit():
    sk = o.interop_secret_key(0)
    assert hex(sk) == "0x25295f0d1d592a90b333e26e85149708208e9f8e8bc18f6c77bd62f8ad7a6866"
    pk = o.g1_compress(o.sk_to_pk(sk))
    assert pk.hex() == K1_PK
    wc, root = deposit_signing_root(pk)
    assert wc.hex() == K1_WC
    sig = o.g2_compress(o.sign(sk, root))
    assert sig.hex() == K1_SIG  # pins hash_to_G2 + scalar mult + G2 compression bit-exactly
    assert o.set_is_valid(o.g1_decompress(pk), root, sig)
    assert not o.set_is_valid(o.g1_decompress(pk), root[:-1] + b"\x00", sig)


@pytest.mark.parametrize("i", range(4))
def test_k2_keygen(i):
    sk = o.keygen(bytes([0xAA + i]) * 32)
    assert sk == int(K2_SKS[i], 16)
    assert o.g1_compress(o.sk_to_pk(sk)).hex() == K2_PKS[i]


def test_k3_infinity_encodings():
    assert o.g1_decompress(bytes([0xC0]) + bytes(47)) is None
    assert o.g2_decompress(bytes([0xC0]) + bytes(95)) is None
    assert o.g1_compress(None) == bytes([0xC0]) + bytes(47)
    # infinity is not a valid signature (Signature.fromBytes(sig, true) infinity check)
    with pytest.raises(o.DecodeError):
        o.signature_from_bytes(bytes([0xC0]) + bytes(95), True)
    # infinity flag with stray bits -> BAD_ENCODING
    with pytest.raises(o.DecodeError):
        o.g2_decompress(bytes([0xE0]) + bytes(95))
    with pytest.raises(o.DecodeError):
        o.g2_decompress(bytes([0xC0]) + bytes(94) + b"\x01")


def test_k4_valid_signature_random_data():
    pt = o.signature_from_bytes(bytes.fromhex(K4_SIG), True)
    assert o.g2_in_subgroup_naive(pt)
    assert o.g2_compress(pt).hex() == K4_SIG


def test_k6_pubkey_decompress():
    pt = o.pubkey_from_bytes(bytes.fromhex(K6_PK), True)
    assert o.g1_in_subgroup_naive(pt)
    assert o.g1_compress(pt).hex() == K6_PK


def test_malformed_signatures():
    # bls.test.ts:44-50 pattern: Buffer.alloc(96, 10) throws in fromBytes
    with pytest.raises(o.DecodeError):
        o.signature_from_bytes(bytes([10]) * 96, True)
    with pytest.raises(o.DecodeError):
        o.signature_from_bytes(bytes(32), True)  # multithread.test.ts:109-129 32-byte sig
    # non-canonical x >= p
    b = bytearray(bytes.fromhex(K4_SIG))
    x1 = int.from_bytes(bytes([b[0] & 0x1F]) + bytes(b[1:48]), "big") + o.P
    if x1 < (1 << 381):
        nb = bytearray(x1.to_bytes(48, "big"))
        nb[0] |= b[0] & 0xE0
        with pytest.raises(o.DecodeError):
            o.signature_from_bytes(bytes(nb) + bytes(b[48:]), True)


def test_subgroup_checks_match_naive():
    q = o.iso_map_g2(o.map_to_curve_sswu_g2((5, 7)))
    assert o.g2_on_curve(q)
    assert o.g2_in_subgroup(q) == o.g2_in_subgroup_naive(q) == False
    hq = o.clear_cofactor_g2(q)
    assert o.g2_in_subgroup(hq) and o.g2_in_subgroup_naive(hq)
    x = 1
    while o.fp_sqrt(x ** 3 + 4) is None:
        x += 1
    pt = (x, o.fp_sqrt(x ** 3 + 4))
    assert o.g1_in_subgroup(pt) == o.g1_in_subgroup_naive(pt) == False


def test_pairing_bilinear():
    e1 = o.pairing(o.g1_mul(o.G1_GEN, 5), o.G2_GEN)
    e2 = o.pairing(o.G1_GEN, o.g2_mul(o.G2_GEN, 5))
    assert e1 == e2 and e1 != o.F12_ONE
    assert o.f12_pow(e1, o.R) == o.F12_ONE


def test_chunkify():
    # beacon-node/test/unit/chain/bls/utils.test.ts (minPerChunk 3)
    c = o.chunkify_maximize_chunk_size
    assert c([], 3) == [[]]
    assert c([0], 3) == [[0]]
    assert c(list(range(5)), 3) == [[0, 1, 2, 3, 4]]
    assert c(list(range(6)), 3) == [[0, 1, 2], [3, 4, 5]]
    assert c(list(range(7)), 3) == [[0, 1, 2, 3], [4, 5, 6]]
    assert c(list(range(9)), 3) == [[0, 1, 2], [3, 4, 5], [6, 7, 8]]


def test_single_thread_same_message_semantics():
    """singleThread.ts:36-80 vs the pool (index.ts:212-236): the unrandomized aggregate accepts
    signatures whose errors cancel (swapped_keys), so the single-thread verifier answers all true
    where the pool's randomized check falls back to per-set results.  Pins the golden vectors of
    tests/golden/single_thread.json against the live oracle on the cases that decide it."""
    import json
    import os
    st = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "single_thread.json")))
    fix = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "fixtures.json")))
    pks = [o.g1_decompress(bytes.fromhex(p)) for p in fix["keys"]["pks"]]
    by_name = {c["name"]: c for c in st["same_message"]}
    sm = by_name["swapped_keys"]
    sets = [(pks[i], bytes.fromhex(s)) for i, s in zip(sm["indices"], sm["sigs"])]
    assert o.single_thread_verify_same_message(sets, bytes.fromhex(sm["msg"])) == [True, True, True] == sm["expected"]
    assert sm["pool_expected"] == [True, False, False]
    for name in ("all_valid", "one_wrong_message", "one_malformed", "six_two_bad"):  # bls.test.ts:68-82: both agree
        assert by_name[name]["expected"] == by_name[name]["pool_expected"]
    with pytest.raises(ValueError):
        o.single_thread_verify_same_message([], bytes(32))
    assert by_name["empty"]["expected"] == "reject"
    # aggregateSignatures vectors: a two-signature sum matches the live oracle
    a = [c for c in st["aggregate_signatures"] if c["name"] == "two"][0]
    pts = [o.signature_from_bytes(bytes.fromhex(s), True) for s in a["sigs"]]
    assert o.g2_compress(o.g2_add(pts[0], pts[1])).hex() == a["expected"]
