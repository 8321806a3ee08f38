#!/usr/bin/env python3
"""Golden vectors for the BlsSingleThreadVerifier semantics (singleThread.ts:36-80), from the CPU
oracle (oracle/bls_oracle.py single_thread_verify_same_message).

Run from the repo root after make_fixtures.py: python tests/golden/make_single_thread_fixtures.py
Writes tests/golden/single_thread.json:
  * every same_message case of fixtures.json with its single-thread booleans ("reject" for the
    empty list, where aggregatePublicKeys throws) -- swapped_keys is the case where the two
    verifiers disagree: the unrandomized aggregate holds, so every set is true;
  * extra cases over one appended key, -pk0 (index NKEYS): its aggregate with pk0 is the point at
    infinity, which blst's verify rejects (PK_IS_INFINITY), so the per-set retry decides;
  * aggregate_signatures: aggregateSignatures(...).toBytes() byte vectors.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import bls_oracle as o  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def main():
    fix = json.load(open(os.path.join(OUT, "fixtures.json")))
    pks = [o.g1_decompress(bytes.fromhex(p)) for p in fix["keys"]["pks"]]
    sks = [int(s, 16) for s in fix["keys"]["sks"]]
    neg_index = len(pks)
    pks.append(o.g1_neg(pks[0]))
    extra_pk = o.g1_compress(pks[neg_index]).hex()

    cases = []
    for c in fix["same_message"]:
        sets = [(pks[i], bytes.fromhex(s)) for i, s in zip(c["indices"], c["sigs"])]
        try:
            exp = o.single_thread_verify_same_message(sets, bytes.fromhex(c["msg"]))
        except ValueError:
            exp = "reject"
        cases.append({"name": c["name"], "msg": c["msg"], "indices": c["indices"], "sigs": c["sigs"], "expected": exp,
                      "pool_expected": c["expected"]})
        print(c["name"], exp, flush=True)

    mm = bytes.fromhex(fix["same_message"][0]["msg"])
    other = bytes(32)
    s0 = bytes.fromhex(fix["same_message"][0]["sigs"][0])  # sk0 over mm
    h_mm, h_other = o.hash_to_g2(mm), o.hash_to_g2(other)
    neg_s0 = o.g2_compress(o.g2_neg(o.g2_decompress(s0)))  # -sk0 over mm: valid for -pk0
    neg_other = o.g2_compress(o.g2_mul(h_other, (-sks[0]) % o.R))  # -sk0 over another message
    s1 = o.g2_compress(o.g2_mul(h_mm, sks[1] % o.R))
    for name, items in (("cancelling_keys", [(0, s0), (neg_index, neg_s0)]),
                        ("cancelling_keys_other_message", [(0, s0), (neg_index, neg_other)]),
                        ("cancelling_plus_valid", [(0, s0), (1, s1), (neg_index, neg_s0)])):
        sets = [(pks[i], s) for i, s in items]
        exp = o.single_thread_verify_same_message(sets, mm)
        pool = o.pool_verify_same_message(sets, mm)
        cases.append({"name": name, "msg": mm.hex(), "indices": [i for i, _ in items], "sigs": [s.hex() for _, s in items],
                      "expected": exp, "pool_expected": pool})
        print(name, exp, pool, flush=True)

    aggs = []
    sig_pool = [bytes.fromhex(s) for s in fix["same_message"][-1]["sigs"]]  # six_two_bad: holds a non-subgroup point
    for name, sigs, validate in (("one", sig_pool[:1], True), ("two", sig_pool[:2], True), ("five_valid", [sig_pool[i] for i in (0, 1, 2, 3, 5)], True),
                                 ("with_non_subgroup", sig_pool, True), ("with_non_subgroup_unvalidated", sig_pool, False),
                                 ("cancel_to_infinity", [s0, neg_s0], True), ("empty", [], True)):
        try:
            pts = [o.signature_from_bytes(s, validate) for s in sigs]
            if not pts:
                raise ValueError("EMPTY_AGGREGATE_ARRAY")
            acc = None
            for p in pts:
                acc = o.g2_add(acc, p)
            exp = o.g2_compress(acc).hex()
        except o.DecodeError:
            exp = "bad_point"
        except ValueError:
            exp = "empty"
        aggs.append({"name": name, "sigs": [s.hex() for s in sigs], "validate": validate, "expected": exp})
        print("aggregate", name, exp[:16], flush=True)

    with open(os.path.join(OUT, "single_thread.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_single_thread_fixtures.py", "extra_pk": extra_pk, "extra_index": neg_index,
                   "same_message": cases, "aggregate_signatures": aggs}, f, indent=1)
    print("wrote single_thread.json")


if __name__ == "__main__":
    main()
