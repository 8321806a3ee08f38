"""8(e) on the GPU with two processes: ShardedVerifier over a world-size-2 process group whose
ranks both drive the box's one MI355X (each with its own gbv context and HBM table; gloo carries
the 577-byte partial all-gather and the boolean gathers here, RCCL on a multi-GPU node).

Each rank verifies its cost-balanced shard of one verifySignatureSets call on the device
(gbv_vs_partial), the partials are all-gathered and every rank runs the one final exponentiation
(gbv_fp12_check); same-message calls shard by call with the booleans all-gathered.  Expected
answers hold by construction (GPU-signed sets, util_sign pinned by K1 in test_gpu_parity.py) with
one wrong-message set or one malformed signature injected into each shard in turn.
"""
import hashlib
import socket

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
N_KEYS = 64


def _sk(i):
    d = hashlib.sha256(b"sharded" + i.to_bytes(4, "little")).digest()
    return (int.from_bytes(d, "little") % R_ORDER).to_bytes(32, "big")


def _worker(rank, world, port, q):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    v = None
    try:
        from lodestar_amd import AggregatedSignatureSet, GpuBlsVerifier, SingleSignatureSet
        from lodestar_amd.sharded import ShardedVerifier
        v = GpuBlsVerifier(0)
        sks = [_sk(i) for i in range(N_KEYS)]
        pks = v.util_sk_to_pk(sks)
        assert v.add_pubkeys(0, pks, validate=True) == bytes(N_KEYS)
        sv = ShardedVerifier(v)

        def sets(n, tag):
            out = []
            for i in range(n):
                m = hashlib.sha256(tag + i.to_bytes(4, "little")).digest()
                if i % 7 == 0:  # an aggregate set (committee of 16)
                    idx = [(5 * i + 3 * j) % N_KEYS for j in range(16)]
                    agg = sum(int.from_bytes(sks[k], "big") for k in idx) % R_ORDER
                    out.append(AggregatedSignatureSet(idx, m, v.util_sign([agg.to_bytes(32, "big")], [0], [m])[0]))
                else:
                    k = (11 * i) % N_KEYS
                    out.append(SingleSignatureSet(k, m, v.util_sign([sks[k]], [0], [m])[0]))
            return out

        base = sets(200, b"call")
        res = {"shard": sv.shard_of(base), "valid": sv.verify_signature_sets(base)}
        for pos in (10, 190):  # one bad set in rank 0's shard, then in rank 1's
            wrong = list(base)
            s = wrong[pos]
            wrong[pos] = SingleSignatureSet(s.index, hashlib.sha256(b"other").digest(), s.signature)
            res["wrong_%d" % pos] = sv.verify_signature_sets(wrong)
            bad = list(base)
            bad[pos] = SingleSignatureSet(s.index, s.signing_root, bytes([10]) * 96)
            res["malformed_%d" % pos] = sv.verify_signature_sets(bad)
        msg = hashlib.sha256(b"same message").digest()
        sigs = v.util_sign([sks[k] for k in range(12)], [0] * 12, [msg])
        calls = [([(k, sigs[k]) for k in range(6)], msg),
                 ([(6, sigs[6]), (7, sigs[0]), (8, bytes([10]) * 96)], msg),
                 ([(k, sigs[k]) for k in range(9, 12)], msg)]
        res["sm"] = sv.verify_same_message_multi(calls)
        q.put((rank, res))
    finally:
        if v is not None:
            v.close_sync()
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_sharded_world2_on_gpu():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    s0, s1 = out[0]["shard"], out[1]["shard"]
    assert s0[0] == 0 and s0[1] == s1[0] and s1[1] == 200 and 0 < s0[1] < 200
    for rank in (0, 1):
        r = out[rank]
        assert r["valid"] is True
        assert r["wrong_10"] is False and r["wrong_190"] is False
        assert r["malformed_10"] is False and r["malformed_190"] is False
        assert r["sm"] == [[True] * 6, [True, False, False], [True] * 3]
