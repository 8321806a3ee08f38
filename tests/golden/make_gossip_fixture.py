#!/usr/bin/env python3
"""Generate tests/golden/gossip_sets.json: gossip messages whose signature sets the gossip builders
(lodestar_amd/gossip_sets.py, addon/gossip_sets.js) must reproduce, signed and checked by the CPU
oracle (oracle/gossip_oracle.py, oracle/bls_oracle.py; test infrastructure).

Contents:
  * a deneb-era SignedAggregateAndProof (phase0 AggregateAndProof type) and an electra-era one
    (electra type: aggregation bits over the committees named by committee_bits), each with its
    attesting indices -- validateAggregateAndProof's three sets (aggregateAndProof.ts:211-229);
  * a SignedContributionAndProof -- validateSyncCommitteeGossipContributionAndProof's three sets
    (syncCommitteeContributionAndProof.ts:73-92), participants from the sync committee's
    subcommittee and the aggregation bits;
  * four SyncCommitteeMessages (syncCommittee.ts:10-23);
  * for every message, the oracle's sets (kind, key, signing root) and the pool's answer for the
    message's verifySignatureSets call (oracle pool_verify_signature_sets) -> true;
  * corruptions, one per set kind of each call: the signature of that one set replaced by a valid
    signature over another root (the bls.test.ts:73 pattern) -> the call is false.
Runtime: about a minute on 8 cores (pure-Python pairings).  Run: python tests/golden/make_gossip_fixture.py
"""
import json
import os
import sys
from multiprocessing import Pool

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import bls_oracle as O  # noqa: E402
from oracle import gossip_oracle as GO  # noqa: E402

N_KEYS = 64  # validator v has interopSecretKey(v mod 64)
N_VALIDATORS = 4096
SLOTS = 32


def _pk(k):
    return O.g1_compress(O.sk_to_pk(O.interop_secret_key(k))).hex()


def _sign(args):
    sk, root = args
    return O.g2_compress(O.sign(sk, root)).hex()


def _sk_of(key, sks):
    if isinstance(key, list):
        return sum(sks[v % N_KEYS] for v in key) % O.R
    return sks[key % N_KEYS]


def main():
    rng = np.random.Generator(np.random.PCG64(0x6055))
    rb = lambda n=32: rng.integers(0, 256, size=n, dtype=np.uint8).tobytes().hex()
    with Pool(8) as pool:
        pks = pool.map(_pk, range(N_KEYS))
    sks = [O.interop_secret_key(k) for k in range(N_KEYS)]
    forks = [["phase0", 0, "00000000"], ["altair", 10, "01000000"], ["bellatrix", 20, "02000000"],
             ["capella", 30, "03000000"], ["deneb", 40, "04000000"], ["electra", 60, "05000000"]]
    cfg = {"forks": forks, "gvr": rb(), "deneb_epoch": 40}
    state_slot = 59 * SLOTS + 3  # deneb; the electra messages come from an electra-era state below
    sync_committee = rng.choice(N_VALIDATORS, size=512, replace=False).astype(int).tolist()
    fix = {"generator": "tests/golden/make_gossip_fixture.py (oracle/gossip_oracle.py + oracle/bls_oracle.py)",
           "world": {"n_validators": N_VALIDATORS, "n_keys": N_KEYS, "key_of_validator": "interopSecretKey(v mod %d)" % N_KEYS},
           "pubkeys": pks, "config": cfg, "state_slot": state_slot, "sync_committee": sync_committee, "calls": []}

    def att_msg(slot, electra):
        ep = slot // SLOTS
        data = {"slot": slot, "index": 0 if electra else 5, "beacon_block_root": rb(), "source_epoch": ep - 1, "source_root": rb(),
                "target_epoch": ep, "target_root": rb()}
        if electra:
            cbits = [ci in (3, 17, 40) for ci in range(64)]
            n_bits = 3 * 64
        else:
            cbits, n_bits = None, 128
        committee = rng.choice(N_VALIDATORS, size=n_bits, replace=False).astype(int).tolist()
        bits = [bool(x) for x in (rng.random(n_bits) < 0.8)]
        att = {"bits": bits, "data": data, "signature": ""}
        if electra:
            att["committee_bits"] = cbits
        attesting = sorted(v for v, b in zip(committee, bits) if b)
        aggregator = committee[7]
        m = {"aggregator_index": aggregator, "aggregate": att, "selection_proof": ""}
        return {"message": m, "signature": ""}, attesting

    calls = []
    for electra, slot in ((False, state_slot - 2), (True, 61 * SLOTS + 9)):
        signed, attesting = att_msg(slot, electra)
        calls.append({"kind": "aggregate_and_proof", "electra": electra, "signed": signed, "attesting_indices": attesting})
    # contribution and proof (deneb state; subcommittee 2)
    c_slot = state_slot - 1
    bits = [bool(x) for x in (rng.random(128) < 0.7)]
    sub = sync_committee[256:384]
    contribution = {"slot": c_slot, "beacon_block_root": rb(), "subcommittee_index": 2, "bits": bits, "signature": ""}
    calls.append({"kind": "contribution_and_proof",
                  "signed": {"message": {"aggregator_index": sub[5], "contribution": contribution, "selection_proof": ""}, "signature": ""}})
    for q in range(4):
        calls.append({"kind": "sync_committee_message", "message": {"slot": state_slot - q % 2, "beacon_block_root": rb(),
                                                                    "validator_index": sync_committee[q * 37], "signature": ""}})

    def sets_of(call):
        if call["kind"] == "aggregate_and_proof":
            return GO.aggregate_and_proof_sets(cfg, call["signed"], call["attesting_indices"])
        if call["kind"] == "contribution_and_proof":
            return GO.contribution_and_proof_sets(fix, call["signed"])
        return [GO.sync_committee_message_set(fix, call["message"])]

    # sign: inner signatures first (the aggregate's / the contribution's signature and the selection
    # proofs are fields of the containers the outer signature covers), then the outer signature
    def put(call, k, sig):
        if call["kind"] == "aggregate_and_proof":
            m = call["signed"]["message"]
            if k == 0:
                m["selection_proof"] = sig
            elif k == 1:
                call["signed"]["signature"] = sig
            else:
                m["aggregate"]["signature"] = sig
        elif call["kind"] == "contribution_and_proof":
            m = call["signed"]["message"]
            if k == 0:
                m["selection_proof"] = sig
            elif k == 1:
                call["signed"]["signature"] = sig
            else:
                m["contribution"]["signature"] = sig
        else:
            call["message"]["signature"] = sig

    for order in ((0, 2), (1,)):  # selection proofs + aggregates, then the aggregator signatures
        jobs, where = [], []
        for ci, call in enumerate(calls):
            ss = sets_of(call)
            for k in order:
                if k < len(ss):
                    kind, key, root, _ = ss[k]
                    jobs.append((_sk_of(key, sks), root))
                    where.append((ci, k))
        with Pool(8) as pool:
            sigs = pool.map(_sign, jobs)
        for (ci, k), sig in zip(where, sigs):
            put(calls[ci], k, sig)

    def pool_dicts(ss):
        out = []
        for kind, key, root, sig in ss:
            if kind == "single":
                out.append({"pubkey": O.g1_decompress(bytes.fromhex(pks[key % N_KEYS])), "msg": root, "sig": sig})
            else:
                out.append({"pubkeys": [O.g1_decompress(bytes.fromhex(pks[v % N_KEYS])) for v in key], "msg": root, "sig": sig})
        return out

    other_root = bytes(range(32))
    for ci, call in enumerate(calls):
        ss = sets_of(call)
        call["expected_sets"] = [{"kind": kind, "key": key, "root": root.hex()} for kind, key, root, _ in ss]
        call["expected_valid"] = O.pool_verify_signature_sets(pool_dicts(ss))
        assert call["expected_valid"] is True, (ci, call["kind"])
        # one corruption per set kind: that set's signature over another root
        call["corruptions"] = []
        for k, (kind, key, root, sig) in enumerate(ss):
            bad = O.g2_compress(O.sign(_sk_of(key, sks), other_root)).hex()
            ss2 = list(ss)
            ss2[k] = (kind, key, root, bytes.fromhex(bad))
            want = O.pool_verify_signature_sets(pool_dicts(ss2))
            assert want is False
            call["corruptions"].append({"set": k, "signature": bad, "expected_valid": want})
    fix["calls"] = calls
    out = os.path.join(HERE, "gossip_sets.json")
    with open(out, "w") as f:
        json.dump(fix, f, separators=(",", ":"))
    print("wrote", out, os.path.getsize(out), "bytes;", len(calls), "calls")


if __name__ == "__main__":
    main()
