#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ with the CPU oracle (oracle/bls_oracle.py).

Run from the repo root: python tests/golden/make_fixtures.py
Cases mirror the reference's own behavioural tests:
  beacon-node/test/unit/chain/bls/bls.test.ts:34-83 (valid / wrong signing root / malformed sig),
  beacon-node/test/e2e/chain/bls/multithread.test.ts:109-129 (32-byte signature),
  beacon-node/test/unit/chain/validation/attestation/validateGossipAttestationsSameAttData.test.ts,
plus the blst edge classes of SURVEY.md Appendix A (infinity, non-subgroup, uncompressed, raw
pubkeys, empty aggregate -> rejection).
"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import bls_oracle as o  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
NKEYS = 16
SKS = [o.interop_secret_key(i) for i in range(NKEYS)]
PKS = [o.sk_to_pk(sk) for sk in SKS]
PKB = [o.g1_compress(p) for p in PKS]


def msg(tag):
    return hashlib.sha256(b"gbv-fixture" + tag.encode()).digest()


_h_cache = {}


def sign(sk, m):
    if m not in _h_cache:
        _h_cache[m] = o.hash_to_g2(m)
    return o.g2_compress(o.g2_mul(_h_cache[m], sk % o.R))


def non_subgroup_sig():
    u = 1
    while True:
        q = o.iso_map_g2(o.map_to_curve_sswu_g2((u, 3)))
        if q is not None and not o.g2_in_subgroup(q):
            return o.g2_compress(q)
        u += 1


def set_single(i, m, sig):
    return {"indices": [i], "msg": m.hex(), "sig": sig.hex()}


def set_agg(idx, m, sig):
    return {"indices": list(idx), "msg": m.hex(), "sig": sig.hex()}


def expected_sets(sets):
    conv = []
    for s in sets:
        d = {"msg": bytes.fromhex(s["msg"]), "sig": bytes.fromhex(s["sig"])}
        if "raw_pk" in s:
            try:
                d["pubkey"] = o.pubkey_from_bytes(bytes.fromhex(s["raw_pk"]), True)
            except o.DecodeError:
                return False  # builder-side PublicKey.fromBytes(pk, true) failure -> set invalid
        elif len(s["indices"]) == 1:
            d["pubkey"] = PKS[s["indices"][0]]
        else:
            d["pubkeys"] = [PKS[i] for i in s["indices"]]
        conv.append(d)
    try:
        return o.pool_verify_signature_sets(conv)
    except ValueError:
        return "reject"


def main():
    m = [msg("m%d" % i) for i in range(8)]
    bad = bytes([10]) * 96
    inf = bytes([0xC0]) + bytes(95)
    vs_cases = []

    def add(name, sets):
        vs_cases.append({"name": name, "sets": sets, "expected": expected_sets(sets)})
        print("verify_sets", name, vs_cases[-1]["expected"], flush=True)

    three = [set_single(i, m[i], sign(SKS[i], m[i])) for i in range(3)]
    add("distinct_valid", three)
    wrong = [dict(s) for s in three]
    wrong[1] = set_single(1, m[1], sign(SKS[1], m[7]))
    add("wrong_signing_root", wrong)
    mal = [dict(s) for s in three]
    mal[2] = set_single(2, m[2], bad)
    add("malformed_sig", mal)
    add("empty", [])
    add("single_valid", [three[0]])
    add("single_invalid", [wrong[1]])
    agg_idx = list(range(8))
    agg_sig = sign(sum(SKS[i] for i in agg_idx), m[3])
    add("aggregate_valid", [set_agg(agg_idx, m[3], agg_sig), three[0]])
    add("aggregate_wrong_member", [set_agg([0, 1, 2, 3, 4, 5, 6, 9], m[3], agg_sig), three[0]])
    add("aggregate_empty_rejects", [set_agg([], m[3], agg_sig), three[0]])
    add("infinity_sig", [three[0], set_single(5, m[5], inf)])
    add("short_sig_32B", [three[0], {"indices": [4], "msg": m[4].hex(), "sig": bytes(32).hex()}])
    add("non_subgroup_sig", [three[0], set_single(6, m[6], non_subgroup_sig())])
    unc = o.g2_serialize(o.g2_mul(o.hash_to_g2(m[6]), SKS[6]))
    add("uncompressed_192B_valid", [three[0], set_single(6, m[6], unc)])
    # raw pubkey sets (blsToExecutionChange.ts:19-44): K1 interop deposit as a raw-pk set
    add("raw_pk_valid", [{"raw_pk": PKB[7].hex(), "msg": m[7].hex(), "sig": sign(SKS[7], m[7]).hex()}, three[1]])
    add("raw_pk_bad_encoding", [{"raw_pk": (bytes([0x00]) + PKB[7][1:]).hex(), "msg": m[7].hex(),
                                 "sig": sign(SKS[7], m[7]).hex()}])
    dup = [set_single(i % 4, m[i % 8], sign(SKS[i % 4], m[i % 8])) for i in range(12)]
    add("twelve_valid_duplicates", dup)

    sm_cases = []

    def add_sm(name, message, items):
        sets = [(PKS[i], bytes.fromhex(s)) for i, s in items]
        exp = o.pool_verify_same_message(sets, message)
        sm_cases.append({"name": name, "msg": message.hex(), "indices": [i for i, _ in items],
                         "sigs": [s for _, s in items], "expected": exp})
        print("same_message", name, exp, flush=True)

    mm = msg("same")
    good = [(i, sign(SKS[i], mm).hex()) for i in range(6)]
    add_sm("all_valid", mm, good[:3])
    add_sm("one_wrong_message", mm, [good[0], (1, sign(SKS[1], m[0]).hex()), good[2]])
    add_sm("one_malformed", mm, [good[0], (1, bad.hex()), good[2]])
    add_sm("one_infinity", mm, [good[0], (1, inf.hex()), good[2]])
    add_sm("swapped_keys", mm, [good[0], (2, good[1][1]), (1, good[2][1])])
    add_sm("single_valid", mm, good[:1])
    add_sm("empty", mm, [])
    add_sm("six_two_bad", mm, [good[0], good[1], (2, sign(SKS[2], m[1]).hex()), good[3], (4, non_subgroup_sig().hex()), good[5]])

    agg_cases = []
    for idx in ([0], [0, 1], list(range(16)), [3, 3], [5, 2, 9]):
        agg_cases.append({"indices": idx, "expected": o.g1_compress(o.aggregate_pubkeys([PKS[i] for i in idx])).hex()})

    h2g2 = []
    for i in range(4):
        mm2 = msg("h%d" % i)
        h2g2.append({"msg": mm2.hex(), "expected": o.g2_serialize(o.hash_to_g2(mm2)).hex()})

    keys = {"sks": ["%064x" % sk for sk in SKS], "pks": [p.hex() for p in PKB]}
    with open(os.path.join(OUT, "fixtures.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_fixtures.py", "keys": keys, "verify_sets": vs_cases,
                   "same_message": sm_cases, "aggregate_pubkeys": agg_cases, "hash_to_g2": h2g2}, f, indent=1)
    print("wrote fixtures.json")


if __name__ == "__main__":
    main()
