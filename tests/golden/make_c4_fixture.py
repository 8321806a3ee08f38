#!/usr/bin/env python3
"""Generate tests/golden/c4_block.json: one full deneb-era block (config C4) with
128 attestations of 128-member committees, a sync aggregate over a 512-member committee, randao,
proposer, two voluntary exits, a BLS-to-execution change, a proposer slashing and an attester
slashing, signed and checked by the CPU oracle (test infrastructure).

Expected values, all from the oracle (oracle/block_oracle.py, oracle/bls_oracle.py):
  * every set's kind, key and signing root (getBlockSignatureSets restated independently of the
    product builders in lodestar_amd/signature_sets.py);
  * the whole block verified by the oracle's restatement of BlsMultiThreadWorkerPool
    (pool_verify_signature_sets: chunks of <=128, randomised batch, AND) -> true;
  * for every corruption kind of tests/golden/c4_block.py, the corrupted set alone -> false.
With --electra: tests/golden/c4_block_electra.json, an electra-era block (fork schedule up to electra)
whose 8 attestations (MAX_ATTESTATIONS_ELECTRA) each span committees named by committee_bits --
six over all 64 committees of their slot, one over 32, one over 17 -- so the attestation aggregates
hold ~4 k validators each (getAttestingIndices, epochCache.ts:953-973).
Runtime: a few minutes on 8 cores (pure-Python pairings).  Run: python tests/golden/make_c4_fixture.py [--electra]
"""
import json
import os
import sys
from multiprocessing import Pool

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

from oracle import bls_oracle as O  # noqa: E402
from oracle import block_oracle as BO  # noqa: E402
import c4_block as C  # noqa: E402

N = C.N_VALIDATORS
K = C.N_KEYS
SLOTS = 32


def _pk(k):
    return O.g1_compress(O.sk_to_pk(O.interop_secret_key(k))).hex()


def _sign(args):
    sk, root = args
    return O.g2_compress(O.sign(sk, root)).hex()


_PK_CACHE = {}


def _dec(pkb):
    p = _PK_CACHE.get(pkb)
    if p is None:
        p = _PK_CACHE[pkb] = O.g1_decompress(pkb)
    return p


def _valid_one(args):
    pkb_list, raw, root, sig = args
    if raw is not None:
        try:
            pk = O.pubkey_from_bytes(raw, validate=True)
        except O.DecodeError:
            return False
    else:
        pk = O.aggregate_pubkeys([_dec(p) for p in pkb_list])
    return O.set_is_valid(pk, root, sig)


def main(electra=False):
    rng = np.random.Generator(np.random.PCG64(0xC4E if electra else 0xC4))
    rb = lambda n=32: rng.integers(0, 256, size=n, dtype=np.uint8).tobytes().hex()
    with Pool(8) as pool:
        pks = pool.map(_pk, range(K))
    sks = [O.interop_secret_key(k) for k in range(K)]
    epoch = 50
    slot = epoch * SLOTS + 5
    forks = [["phase0", 0, "00000000"], ["altair", 10, "01000000"], ["bellatrix", 20, "02000000"],
             ["capella", 30, "03000000"], ["deneb", 40, "04000000"]]
    if electra:
        forks.append(["electra", 45, "05000000"])
    cfg = {"forks": forks, "gvr": rb(), "deneb_epoch": 40}
    committees = {}
    atts = []
    if not electra:
        for j in range(128):
            a_slot = slot - 1 - (j % 8)
            a_idx = j // 8
            members = rng.choice(N, size=128, replace=False).astype(int).tolist()
            committees["%d,%d" % (a_slot, a_idx)] = members
            bits = [True] * 128
            if j % 10 == 3:
                for q in (1, 50, 99):
                    bits[q] = False
            ep = a_slot // SLOTS
            atts.append({"bits": bits, "data": {"slot": a_slot, "index": a_idx, "beacon_block_root": rb(), "source_epoch": ep - 1,
                                                "source_root": rb(), "target_epoch": ep, "target_root": rb()}, "signature": ""})
    else:
        # one aggregate per slot over that slot's committees (64 committees of 64 members each)
        for j in range(8):
            a_slot = slot - 1 - j
            for ci in range(64):
                committees["%d,%d" % (a_slot, ci)] = rng.choice(N, size=64, replace=False).astype(int).tolist()
            if j < 6:
                cbits = [True] * 64
            elif j == 6:
                cbits = [ci % 2 == 0 for ci in range(64)]
            else:
                pick = set(rng.choice(64, size=17, replace=False).tolist())
                cbits = [ci in pick for ci in range(64)]
            n_bits = 64 * sum(cbits)
            bits = [True] * n_bits
            if j % 3 == 1:
                for q in rng.choice(n_bits, size=5, replace=False).tolist():
                    bits[q] = False
            ep = a_slot // SLOTS
            atts.append({"bits": bits, "committee_bits": cbits,
                         "data": {"slot": a_slot, "index": 0, "beacon_block_root": rb(), "source_epoch": ep - 1,
                                  "source_root": rb(), "target_epoch": ep, "target_root": rb()}, "signature": ""})
    sync_committee = rng.choice(N, size=512, replace=False).astype(int).tolist()
    sbits = [True] * 512
    for q in rng.choice(512, size=17, replace=False).tolist():
        sbits[q] = False
    proposer = int(rng.integers(0, N))
    slasher = int(rng.integers(0, N))
    hdr = lambda sr: {"slot": slot - 40, "proposer_index": slasher, "parent_root": "11" * 32, "state_root": sr, "body_root": "22" * 32}
    ia_members = rng.choice(N, size=64, replace=False).astype(int).tolist()
    ia_data = lambda bbr: {"slot": slot - 60, "index": 3, "beacon_block_root": bbr, "source_epoch": epoch - 3, "source_root": "33" * 32,
                           "target_epoch": epoch - 2, "target_root": "44" * 32}
    bls_key = 1000
    block = {
        "slot": slot, "proposer_index": proposer, "parent_root": rb(), "state_root": rb(), "body_root": rb(),
        "randao_reveal": "", "signature": "",
        "proposer_slashings": [[{"message": hdr("55" * 32), "signature": ""}, {"message": hdr("66" * 32), "signature": ""}]],
        "attester_slashings": [[{"attesting_indices": sorted(ia_members), "data": ia_data("77" * 32), "signature": ""},
                                {"attesting_indices": sorted(ia_members), "data": ia_data("88" * 32), "signature": ""}]],
        "attestations": atts,
        "voluntary_exits": [{"message": {"epoch": epoch - 5 + q, "validator_index": int(rng.integers(0, N))}, "signature": ""} for q in range(2)],
        "sync_aggregate": {"bits": sbits, "signature": ""},
        "bls_changes": [{"message": {"validator_index": int(rng.integers(0, N)), "from_bls_pubkey": pks[bls_key],
                                     "to_execution_address": rb(20)}, "signature": ""}],
    }
    fix = {"generator": "tests/golden/make_c4_fixture.py (oracle/block_oracle.py + oracle/bls_oracle.py)",
           "world": {"n_validators": N, "n_keys": K, "key_of_validator": "interopSecretKey(v mod 1024)"},
           "config": cfg, "state_slot": slot, "committees": committees, "sync_committee": sync_committee, "block": block,
           "other_pubkey": pks[bls_key + 1]}
    # signature slots in getBlockSignatureSets order
    slots = [("randao_reveal",)]
    slots += [("proposer_slashings", 0, i, "signature") for i in range(2)]
    slots += [("attester_slashings", 0, i, "signature") for i in range(2)]
    slots += [("attestations", j, "signature") for j in range(len(atts))]
    slots += [("voluntary_exits", q, "signature") for q in range(2)]
    slots += [("signature",), ("sync_aggregate", "signature"), ("bls_changes", 0, "signature")]
    sets = BO.block_signature_sets(fix)
    assert len(sets) == len(slots) == (18 if electra else 138)
    jobs = []
    for kind, key, root, _ in sets:
        if kind == "raw":
            sk = sks[bls_key]
        elif kind == "single":
            sk = sks[key % K]
        else:
            sk = sum(sks[v % K] for v in key) % O.R
        jobs.append((sk, root))
    with Pool(8) as pool:
        sigs = pool.map(_sign, jobs)
    for path, sig in zip(slots, sigs):
        obj = block
        for p in path[:-1]:
            obj = obj[p]
        obj[path[-1]] = sig
    sets = BO.block_signature_sets(fix)
    fix["expected_sets"] = [{"kind": kind, "key": key.hex() if kind == "raw" else key, "root": root.hex()} for kind, key, root, _ in sets]

    def pool_dicts(ss):
        out = []
        for kind, key, root, sig in ss:
            if kind == "raw":
                pk = {"pubkey": O.pubkey_from_bytes(key, validate=True)}
            elif kind == "single":
                pk = {"pubkey": _dec(bytes.fromhex(pks[key % K]))}
            else:
                pk = {"pubkeys": [_dec(bytes.fromhex(pks[v % K])) for v in key]}
            out.append(dict(pk, msg=root, sig=sig))
        return out
    fix["expected_valid"] = O.pool_verify_signature_sets(pool_dicts(sets))
    assert fix["expected_valid"] is True
    corr = {}
    args = []
    kinds = C.CORRUPTIONS_ELECTRA if electra else C.CORRUPTIONS
    for kind in kinds:
        b2, com2, k = C.corrupt(fix, kind)
        s2 = BO.block_signature_sets(fix, b2, com2)
        kind_k, key, root, sig = s2[k]
        raw = key if kind_k == "raw" else None
        members = [] if raw is not None else ([key] if kind_k == "single" else key)
        args.append(([bytes.fromhex(pks[v % K]) for v in members], raw, root, sig))
        corr[kind] = {"set": k}
    with Pool(8) as pool:
        res = pool.map(_valid_one, args)
    for kind, r in zip(kinds, res):
        assert r is False, kind
        corr[kind]["valid"] = r
    fix["corruptions"] = corr
    # f2: aggregateSerializedPublicKeys over the whole 512-member sync committee
    # (processSyncCommitteeUpdates.ts:35), byte-exact, and the 1024 interop pubkeys of the world
    agg = O.aggregate_pubkeys([O.g1_decompress(bytes.fromhex(pks[v % K])) for v in sync_committee])
    fix["sync_committee_aggregate"] = O.g1_compress(agg).hex()
    fix["pubkeys"] = pks
    path = C.FIX_PATH_ELECTRA if electra else C.FIX_PATH
    with open(path, "w") as f:
        json.dump(fix, f, separators=(",", ":"))
    print("wrote %s: %d sets, %d bytes" % (path, len(sets), os.path.getsize(path)))


if __name__ == "__main__":
    main(electra="--electra" in sys.argv)
