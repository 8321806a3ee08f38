"""The streamed IBlsVerifier path on the GPU: several device passes in flight at once (each on its
own refillable batches, gbv_sm_batch_fill / gbv_vs_batch_fill), with a bad set injected into every
pass, and one-shot calls on the same context while passes run (the context lock, include/gbv.h).

Reference behaviour: every queued job resolves with its own result (multithread/index.ts:357-534),
an invalid set fails only its own request (multithread.test.ts:109-129), same-message chunks fall
back to per-set verification (jobItem.ts:93-125).  Expected booleans hold by construction: every
set is signed on the GPU with its own interop key except the injected ones.

Run on an MI355X: python -m pytest tests -m gpu
"""
import asyncio
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
N_KEYS = 256
N_TABLE = 4096


def _sk(i):
    d = hashlib.sha256(i.to_bytes(32, "little")).digest()
    return (int.from_bytes(d, "little") % R_ORDER).to_bytes(32, "big")


@pytest.fixture(scope="module")
def world():
    from lodestar_amd import GpuBlsVerifier
    v = GpuBlsVerifier(0)
    sks = [_sk(i) for i in range(N_KEYS)]
    pks = v.util_sk_to_pk(sks)
    assert v.add_pubkeys(0, pks, validate=True) == bytes(N_KEYS)
    v.replicate_pubkeys(0, N_KEYS, N_KEYS, N_TABLE - N_KEYS)
    yield v, sks
    v.close_sync()


def _round(v, sks, seed, n_calls):
    """n_calls same-message gossip calls (32-128 sets) and 8 distinct-message verifySignatureSets
    calls of 16 sets; one same-message set and one default call get a signature over another
    message (bls.test.ts:73), one same-message set the malformed bytes([10]*96) (bls.test.ts:79)."""
    from lodestar_amd import SingleSignatureSet
    rng = np.random.Generator(np.random.PCG64(seed))
    sizes = [int(x) for x in rng.integers(32, 129, size=n_calls)]
    msgs = [hashlib.sha256(b"gbv-stream" + seed.to_bytes(4, "little") + g.to_bytes(8, "little")).digest() for g in range(n_calls)]
    idx = rng.integers(0, N_TABLE, size=sum(sizes))
    grp = np.repeat(np.arange(n_calls), sizes)
    sigs = v.util_sign([sks[int(i) % N_KEYS] for i in idx], grp.tolist(), msgs)
    want = [True] * len(idx)
    bad_wrong, bad_malformed = int(rng.integers(0, len(idx))), int(rng.integers(0, len(idx)))
    other = v.util_sign([sks[int(idx[bad_wrong]) % N_KEYS]], [0], [hashlib.sha256(b"other").digest()])[0]
    sigs[bad_wrong], want[bad_wrong] = other, False
    sigs[bad_malformed], want[bad_malformed] = bytes([10]) * 96, False
    calls, pos = [], 0
    for g, n in enumerate(sizes):
        calls.append(([(int(idx[pos + k]), sigs[pos + k]) for k in range(n)], msgs[g], want[pos:pos + n]))
        pos += n
    # default jobs: 8 calls x 16 distinct-message single sets, call 3 holds a wrong-message signature
    d_msgs = [hashlib.sha256(b"gbv-stream-d" + seed.to_bytes(4, "little") + k.to_bytes(4, "little")).digest() for k in range(128)]
    d_idx = rng.integers(0, N_TABLE, size=128)
    d_sigs = v.util_sign([sks[int(i) % N_KEYS] for i in d_idx], list(range(128)), d_msgs)
    d_sigs[3 * 16 + 5] = v.util_sign([sks[int(d_idx[3 * 16 + 5]) % N_KEYS]], [0], [d_msgs[0]])[0]
    dcalls = [[SingleSignatureSet(int(d_idx[16 * c + k]), d_msgs[16 * c + k], d_sigs[16 * c + k]) for k in range(16)] for c in range(8)]
    return calls, dcalls, [c != 3 for c in range(8)]


def test_overlapping_passes_with_a_bad_set_in_each(world):
    v, sks = world
    from lodestar_amd.verifier import MAX_PASSES_IN_FLIGHT
    rounds = [_round(v, sks, 100 + r, 40) for r in range(MAX_PASSES_IN_FLIGHT + 1)]

    async def go():
        futs, busy_seen = [], 0
        for calls, dcalls, _ in rounds:
            fs = [asyncio.ensure_future(v.verify_signature_sets_same_message(s, m)) for s, m, _ in calls]
            fd = [asyncio.ensure_future(v.verify_signature_sets(c)) for c in dcalls]
            futs.append((fs, fd))
            for _ in range(200):  # let this round's jobs go out as their own pass
                await asyncio.sleep(0)
                if not v._jobs:
                    break
            busy_seen = max(busy_seen, v._busy)
        res = [(await asyncio.gather(*fs), await asyncio.gather(*fd)) for fs, fd in futs]
        return res, busy_seen

    passes0 = v.device_passes
    res, busy_seen = asyncio.run(go())
    for (calls, dcalls, dwant), (rs, rd) in zip(rounds, res):
        assert [r for r in rs] == [w for _, _, w in calls]
        assert rd == dwant
    assert busy_seen >= 2, busy_seen  # passes overlapped on the device
    assert v.device_passes - passes0 >= 2
    assert v.pool_metrics.value("lodestar_bls_thread_pool_same_message_jobs_retries_total") >= 2


def test_one_shot_call_while_passes_run(world):
    """verifyOnMainThread (a one-shot call on the context's scratch batch) while a streamed pass is on
    the device: the context lock keeps them apart and both are right."""
    v, sks = world
    from lodestar_amd import SingleSignatureSet, VerifySignatureOpts
    calls, dcalls, dwant = _round(v, sks, 7, 120)

    async def go():
        fs = [asyncio.ensure_future(v.verify_signature_sets_same_message(s, m)) for s, m, _ in calls]
        while v._jobs or not v._busy:
            await asyncio.sleep(0)
        main = [await v.verify_signature_sets(c, VerifySignatureOpts(verify_on_main_thread=True)) for c in dcalls]
        single = v.verify_signature_set(dcalls[0][0])
        return await asyncio.gather(*fs), main, single

    rs, main, single = asyncio.run(go())
    assert rs == [w for _, _, w in calls]
    assert main == dwant and single is True
    assert isinstance(dcalls[0][0], SingleSignatureSet)


def test_packed_same_message_sets_match_the_list_form(world):
    v, sks = world
    from lodestar_amd import PackedSameMessageSets
    calls, _, _ = _round(v, sks, 11, 6)

    async def go():
        out = []
        for s, m, _ in calls:
            packed = PackedSameMessageSets(np.array([i for i, _ in s]), b"".join(sig for _, sig in s))
            out.append(await v.verify_signature_sets_same_message(packed, m))
        return out

    got = asyncio.run(go())
    for (s, m, want), g in zip(calls, got):
        assert isinstance(g, np.ndarray) and g.tolist() == want
