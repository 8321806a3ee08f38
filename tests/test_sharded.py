"""Multi-GPU host logic (lodestar_amd/sharded.py) on CPU: world_size-2 gloo process groups over
127.0.0.1, with an oracle-backed stand-in for the device (test infrastructure only) so the
sharding, the 577-byte all-gather of Fp12 Miller partials, the combined final exponentiation and
the per-set boolean gather are exercised without a GPU.  Expected answers come from the oracle's
restatement of the reference pool (oracle.bls_oracle.pool_verify_*).
"""
import os
import random
import socket

import pytest
import torch.multiprocessing as mp

from lodestar_amd.sharded import PARTIAL_BYTES, balanced_ranges, set_weight
from lodestar_amd.verifier import AggregatedSignatureSet, SingleSignatureSet
from oracle import bls_oracle as O

N_KEYS = 6


def _keys():
    sks = [O.interop_secret_key(i) for i in range(N_KEYS)]
    return sks, [O.sk_to_pk(sk) for sk in sks]


def _f12_to_bytes(f):
    out = b""
    for six in f:
        for two in six:
            out += two[0].to_bytes(48, "big") + two[1].to_bytes(48, "big")
    return out


def _f12_from_bytes(b):
    v = [int.from_bytes(b[48 * i:48 * i + 48], "big") for i in range(12)]
    f2 = [(v[2 * k], v[2 * k + 1]) for k in range(6)]
    return ((f2[0], f2[1], f2[2]), (f2[3], f2[4], f2[5]))


class OracleDevice:
    """CPU stand-in with the GpuBlsVerifier methods ShardedVerifier uses (oracle arithmetic)."""

    def __init__(self, pks):
        self.pks = pks
        self.rng = random.Random(os.getpid())
        self.in_flight = 0
        self.max_in_flight = 0

    def _pk(self, s):
        if isinstance(s, AggregatedSignatureSet):
            return O.aggregate_pubkeys([self.pks[i] for i in s.indices])
        return self.pks[s.index]

    def vs_partial(self, sets):
        f, sig_acc, ok = O.F12_ONE, None, True
        for s in sets:
            try:
                sig = O.signature_from_bytes(bytes(s.signature), True)
            except O.DecodeError:
                ok = False
                continue
            pk = self._pk(s)
            if pk is None or sig is None:
                ok = False
                continue
            r = self.rng.getrandbits(64) | 1
            f = O.f12_mul(f, O.miller_loop(O.g1_mul(pk, r), O.hash_to_g2(bytes(s.signing_root))))
            sig_acc = O.g2_add(sig_acc, O.g2_mul(sig, r))
        if sig_acc is not None:
            f = O.f12_mul(f, O.miller_loop(O.g1_neg(O.G1_GEN), sig_acc))
        blob = _f12_to_bytes(f)
        assert len(blob) == PARTIAL_BYTES
        return blob, ok

    def fp12_check(self, partials):
        f = O.F12_ONE
        for b in partials:
            f = O.f12_mul(f, _f12_from_bytes(b))
        return O.final_exponentiation(f) == O.F12_ONE

    def verify_same_message_multi_sync(self, calls):
        return [O.pool_verify_same_message([(self.pks[i], sig) for i, sig in sets], msg) for sets, msg in calls]


def _sets(sks, bad=None):
    msgs = [bytes([i + 1]) * 32 for i in range(5)]
    sets = [SingleSignatureSet(i, msgs[i], O.g2_compress(O.sign(sks[i], msgs[i]))) for i in range(3)]
    agg_sk = (sks[3] + sks[4]) % O.R
    sets.append(AggregatedSignatureSet([3, 4], msgs[3], O.g2_compress(O.sign(agg_sk, msgs[3]))))
    sets.append(SingleSignatureSet(5, msgs[4], O.g2_compress(O.sign(sks[5], msgs[4]))))
    if bad == "wrong_msg":
        sets[4] = SingleSignatureSet(5, msgs[4], O.g2_compress(O.sign(sks[5], msgs[0])))
    elif bad == "malformed":
        sets[1] = SingleSignatureSet(1, msgs[1], bytes([10]) * 96)
    elif bad == "malformed_last":  # in the last rank's shard
        sets[4] = SingleSignatureSet(5, msgs[4], bytes([10]) * 96)
    return sets


class OracleStaged:
    """Stand-in for a StagedSignatureSets holding this rank's shard (ShardedVerifier.verify_staged_shard,
    verify_staged_shards): partial(), or partial_submit() / partial_wait() with the passes in flight
    counted on the device stand-in."""

    def __init__(self, device, sets):
        self.device, self.sets = device, sets
        self.flying = None

    def partial(self):
        return self.device.vs_partial(self.sets)

    def partial_submit(self):
        assert self.flying is None, "submitted twice"
        self.flying = self.device.vs_partial(self.sets)
        self.device.in_flight += 1
        self.device.max_in_flight = max(self.device.max_in_flight, self.device.in_flight)

    def partial_wait(self):
        assert self.flying is not None, "not submitted"
        r, self.flying = self.flying, None
        self.device.in_flight -= 1
        return r


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from lodestar_amd import EmptyAggregateError
        from lodestar_amd.sharded import ShardedVerifier
        sks, pks = _keys()
        sv = ShardedVerifier(OracleDevice(pks))
        res = {"shard": sv.shard_of(_sets(sks))}
        res["valid"] = sv.verify_signature_sets(_sets(sks))
        res["wrong_msg"] = sv.verify_signature_sets(_sets(sks, "wrong_msg"))
        res["malformed"] = sv.verify_signature_sets(_sets(sks, "malformed"))
        res["malformed_last"] = sv.verify_signature_sets(_sets(sks, "malformed_last"))
        # the staged form: each rank stages its own shard, then partial -> all-gather -> one check
        for name, bad in (("staged", None), ("staged_wrong", "wrong_msg"), ("staged_malformed", "malformed_last")):
            call = _sets(sks, bad)
            lo, hi = sv.shard_of(call)
            res[name] = sv.verify_staged_shard(OracleStaged(sv.device, call[lo:hi]))
        # streamed: four staged calls (two valid, one wrong message, one malformed in the last shard)
        # with two shard passes in flight on each rank; one answer per call
        stream = []
        for bad in (None, "wrong_msg", None, "malformed_last"):
            call = _sets(sks, bad)
            lo, hi = sv.shard_of(call)
            stream.append(OracleStaged(sv.device, call[lo:hi]))
        res["streamed"] = sv.verify_staged_shards(stream, depth=2)
        res["streamed_max_in_flight"] = sv.device.max_in_flight
        res["streamed_left"] = sv.device.in_flight
        res["ranges"] = sv.call_ranges([128, 128] + [32] * 8)
        res["empty"] = sv.verify_signature_sets([])
        try:
            sv.verify_signature_sets(_sets(sks) + [AggregatedSignatureSet([], bytes(32), bytes(96))])
            res["empty_agg"] = "no error"
        except EmptyAggregateError:
            res["empty_agg"] = "rejected"
        msg = bytes([7]) * 32
        good = [(i, O.g2_compress(O.sign(sks[i], msg))) for i in range(4)]
        calls = [(good[:2], msg), ([good[2], (3, bytes([10]) * 96)], msg), ([(0, good[1][1])], msg)]
        res["sm"] = sv.verify_same_message_multi(calls)
        # a device error on ONE rank (e.g. an index out of range there) must raise on every rank,
        # not leave the other rank blocked in the all-gather
        from lodestar_amd import GbvError

        class RaisingOnRank1(OracleDevice):
            def verify_same_message_multi_sync(self, calls):
                if rank == 1:
                    raise GbvError(-1, "validator index out of range")
                return super().verify_same_message_multi_sync(calls)
        try:
            ShardedVerifier(RaisingOnRank1(pks)).verify_same_message_multi(calls)
            res["sm_err"] = "no error"
        except GbvError:
            res["sm_err"] = "raised"
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_balanced_ranges_cover_and_balance():
    w = [set_weight(AggregatedSignatureSet(list(range(k)), bytes(32), bytes(96))) for k in (1, 128, 1, 1, 512, 1, 128)]
    for parts in (1, 2, 3, 8):
        r = balanced_ranges(w, parts)
        assert len(r) == parts and r[0][0] == 0 and r[-1][1] == len(w)
        assert all(r[i][1] == r[i + 1][0] for i in range(parts - 1))
    # one call larger than a rank's share starts on the first rank, not piled onto the last one
    assert balanced_ranges([200, 50, 50], 2) == [(0, 1), (1, 3)]
    assert balanced_ranges([50, 50, 200], 2) == [(0, 2), (2, 3)]
    assert sum(b - a for a, b in balanced_ranges([128] * 3, 8)) == 3  # fewer calls than ranks: some ranges empty


def test_sharded_world2_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=600) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sks, pks = _keys()
    table_sets = lambda sets: [{"pubkeys": [pks[i] for i in s.indices]} if isinstance(s, AggregatedSignatureSet)
                               else {"pubkey": pks[s.index]} for s in sets]
    for rank in (0, 1):
        r = out[rank]
        assert r["valid"] is True and r["wrong_msg"] is False and r["malformed"] is False
        assert r["malformed_last"] is False
        assert r["staged"] is True and r["staged_wrong"] is False and r["staged_malformed"] is False
        assert r["streamed"] == [True, False, True, False]
        assert r["streamed_max_in_flight"] == 2 and r["streamed_left"] == 0
        assert r["ranges"] == [(0, 2), (2, 10)]  # 256 sets each (by call count: 352 and 160)
        assert r["empty"] is False and r["empty_agg"] == "rejected"
        assert r["sm"] == [[True, True], [True, False], [False]]
        assert r["sm_err"] == "raised"
    # the two shards partition the call
    assert out[0]["shard"][0] == 0 and out[0]["shard"][1] == out[1]["shard"][0] and out[1]["shard"][1] == 5
    # and the answers match the oracle's restatement of the reference pool
    for bad, want in ((None, True), ("wrong_msg", False), ("malformed", False)):
        sets = _sets(sks, bad)
        d = [dict(t, msg=bytes(s.signing_root), sig=bytes(s.signature)) for t, s in zip(table_sets(sets), sets)]
        assert O.pool_verify_signature_sets(d) is want


# ---- world sizes 4 and 8 (the driver's 8-GPU node has one rank per GPU) ---------------------------
def _presigned():
    """Signatures made once in the parent (oracle signing is slow): the _sets() call, its wrong-message
    variant, and four same-message signatures."""
    sks, pks = _keys()
    msgs = [bytes([i + 1]) * 32 for i in range(5)]
    sig = {i: O.g2_compress(O.sign(sks[i], msgs[i])) for i in range(3)}
    sig["agg"] = O.g2_compress(O.sign((sks[3] + sks[4]) % O.R, msgs[3]))
    sig[5] = O.g2_compress(O.sign(sks[5], msgs[4]))
    sig["wrong"] = O.g2_compress(O.sign(sks[5], msgs[0]))
    msg = bytes([7]) * 32
    sm = [O.g2_compress(O.sign(sks[i], msg)) for i in range(4)]
    return {"pks": pks, "msgs": msgs, "sig": sig, "sm_msg": msg, "sm": sm}


def _call(d, bad=None):
    m, sig = d["msgs"], d["sig"]
    sets = [SingleSignatureSet(i, m[i], sig[i]) for i in range(3)]
    sets.append(AggregatedSignatureSet([3, 4], m[3], sig["agg"]))
    sets.append(SingleSignatureSet(5, m[4], sig["wrong"] if bad == "wrong_last" else sig[5]))
    if bad == "malformed_last":
        sets[4] = SingleSignatureSet(5, m[4], bytes([10]) * 96)
    return sets


def _world_n_worker(rank, world, port, q, d):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from lodestar_amd import GbvError
        from lodestar_amd.sharded import ShardedVerifier
        sv = ShardedVerifier(OracleDevice(d["pks"]))
        res = {"shard": sv.shard_of(_call(d))}
        # streamed staged shards, two in flight: 5 sets over `world` ranks leave some shards empty; the
        # bad set of the second and third calls sits in the last non-empty shard
        stream = []
        for bad in (None, "wrong_last", "malformed_last"):
            call = _call(d, bad)
            lo, hi = sv.shard_of(call)
            stream.append(OracleStaged(sv.device, call[lo:hi]))
        res["streamed"] = sv.verify_staged_shards(stream, depth=2)
        res["left"] = sv.device.in_flight
        # fewer same-message calls than ranks: ranks without calls still join the gather
        msg, sm = d["sm_msg"], d["sm"]
        calls = [([(0, sm[0]), (1, sm[1])], msg), ([(2, sm[2]), (3, bytes([10]) * 96)], msg), ([(0, sm[1])], msg)]
        res["sm_ranges"] = sv.call_ranges([len(c[0]) for c in calls])
        res["sm"] = sv.verify_same_message_multi(calls)

        # a device error on the LAST rank during a streamed pass: every rank raises (none blocks in the
        # all-gather), the failing rank with its own error
        class FailingStaged(OracleStaged):
            def partial_wait(self):
                super().partial_wait()
                raise GbvError(-5, "device fault on rank %d" % rank)
        err_stream = []
        for k in range(3):
            call = _call(d)
            lo, hi = sv.shard_of(call)
            cls = FailingStaged if (rank == world - 1 and k == 1) else OracleStaged
            err_stream.append(cls(sv.device, call[lo:hi]))
        try:
            sv.verify_staged_shards(err_stream, depth=2)
            res["err"] = "no error"
        except GbvError as e:
            res["err"] = str(e)
        res["err_left"] = sv.device.in_flight
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [4, 8])
def test_sharded_world_n_gloo(world):
    """verify_staged_shards and verify_same_message_multi at 4 and 8 ranks (gloo): uneven and empty
    shards, fewer calls than ranks, a bad set in the last shard, a device error on one rank."""
    d = _presigned()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_world_n_worker, args=(r, world, port, q, d)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=900) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    shards = [out[r]["shard"] for r in range(world)]
    assert shards[0][0] == 0 and shards[-1][1] == 5 and all(shards[r][1] == shards[r + 1][0] for r in range(world - 1))
    if world == 8:
        assert any(lo == hi for lo, hi in shards)  # empty shards take part with the Fp12 one
    sm_ranges = out[0]["sm_ranges"]
    assert sum(1 for a, b in sm_ranges if b > a) <= 3 and sm_ranges[-1][1] == 3
    for r in range(world):
        x = out[r]
        assert x["streamed"] == [True, False, False] and x["left"] == 0
        assert x["sm"] == [[True, True], [True, False], [False]]
        assert x["sm_ranges"] == sm_ranges
        assert x["err_left"] == 0
        if r == world - 1:
            assert x["err"].endswith("device fault on rank %d" % r), x["err"]
        else:
            assert x["err"].endswith("device error on a peer rank"), x["err"]
