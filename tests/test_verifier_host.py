"""Host logic of the IBlsVerifier mirror (lodestar_amd/verifier.py) on CPU: queueing, batchable
buffering, priority, chunking, close() -> QUEUE_ABORTED, canAcceptWork -- the scheduling rules of
BlsMultiThreadWorkerPool (packages/beacon-node/src/chain/bls/multithread/index.ts:149-155,
157-236, 302-352, 519-550).  The device calls are replaced by a recorder (no GPU, no oracle
needed: these tests are about which device passes happen and what the promises resolve to).
"""
import asyncio

import pytest

import numpy as np

from lodestar_amd import QueueAbortedError, SingleSignatureSet, VerifySignatureOpts
from lodestar_amd._native import EmptyAggregateError, GbvError
from lodestar_amd.verifier import (AggregatedSignatureSet, GpuBlsVerifier, MAX_BUFFERED_SIGS, MAX_PASSES_IN_FLIGHT,
                                   PackedSameMessageSets, StagedSameMessage, chunkify_maximize_chunk_size)


class Recorder(GpuBlsVerifier):
    """GpuBlsVerifier with the device passes replaced: a set is "valid" iff its signature starts
    with 0x01; every device pass is logged."""

    pubkey_count = 1 << 20  # table slots (no device to ask)

    def __init__(self):  # no gbv_init: nothing touches a GPU
        self._device = 0
        self._init_host_state()
        self.destroyed_after = None
        self.passes = []

        rec = self

        class _Lib:
            def gbv_destroy(self, ctx):
                rec.destroyed_after = list(rec.passes)
        self._lib = _Lib()
        self._ctx = None

    # one device pass = fill + submit (recorded here) and wait (returns what submit computed)
    def _pass_submit(self, slot, sm, df):
        r_sm = r_df = None
        if sm:
            calls = [(list(zip(j.sets[0].tolist(), [j.sets[1][96 * i:96 * i + 96] for i in range(len(j.sets[0]))])), j.message)
                     for j in sm]
            r_sm = bytes(int(b) for r in self.verify_same_message_multi_sync(calls) for b in r)
        if df:
            r_df = self.verify_signature_sets_multi_sync([j.sets for j in df])
        return object(), r_sm, r_df

    def _pass_wait(self, slot, sm, df, st_sm, st_df):
        return st_sm, st_df

    def verify_signature_sets_sync(self, sets):
        self.passes.append(("sets", len(sets)))
        return len(sets) > 0 and all(bytes(s.signature)[:1] == b"\x01" for s in sets)

    def verify_signature_sets_multi_sync(self, calls):
        self.passes.append(("multi", [len(c) for c in calls]))
        out = []
        for c in calls:
            if any(isinstance(s, AggregatedSignatureSet) and not s.indices for s in c):
                out.append(EmptyAggregateError(-3, "EMPTY_AGGREGATE_ARRAY"))
            else:
                out.append(len(c) > 0 and all(bytes(s.signature)[:1] == b"\x01" for s in c))
        return out

    def verify_same_message_multi_sync(self, calls):
        self.passes.append(("sm", [len(c[0]) for c in calls]))
        return [[bytes(sig)[:1] == b"\x01" for _, sig in sets] for sets, _ in calls]


def _set(ok=True):
    return SingleSignatureSet(0, bytes(32), (b"\x01" if ok else b"\x00") + bytes(95))


def run(coro):
    return asyncio.run(coro)


def test_chunkify_matches_reference():
    # multithread/utils.ts:4-18 and its unit test shapes
    assert chunkify_maximize_chunk_size([], 128) == [[]]
    assert [len(c) for c in chunkify_maximize_chunk_size(list(range(255)), 128)] == [255]
    assert [len(c) for c in chunkify_maximize_chunk_size(list(range(256)), 128)] == [128, 128]
    assert [len(c) for c in chunkify_maximize_chunk_size(list(range(300)), 128)] == [150, 150]
    assert [len(c) for c in chunkify_maximize_chunk_size(list(range(10)), 3)] == [4, 4, 2]


def test_verify_sets_and_empty():
    async def go():
        v = Recorder()
        a = await v.verify_signature_sets([_set(), _set()])
        b = await v.verify_signature_sets([_set(), _set(False)])
        c = await v.verify_signature_sets([])
        return a, b, c
    assert run(go()) == (True, False, False)


def test_large_call_is_chunked_into_jobs_and_anded():
    async def go():
        v = Recorder()
        ok = await v.verify_signature_sets([_set()] * 300)
        bad = await v.verify_signature_sets([_set()] * 299 + [_set(False)])
        return v, ok, bad
    v, ok, bad = run(go())
    assert ok is True and bad is False
    # the call's two 150-set jobs (chunkifyMaximizeChunkSize) go to the device in one pass
    assert ("multi", [150, 150]) in v.passes


def test_batchable_requests_are_buffered_then_flushed_together():
    async def go():
        v = Recorder()
        opts = VerifySignatureOpts(batchable=True)
        futs = [asyncio.ensure_future(v.verify_signature_sets([_set()], opts)) for _ in range(3)]
        await asyncio.sleep(0.01)
        assert v.passes == []  # still inside the 100 ms buffer window (index.ts:65)
        res = await asyncio.gather(*futs)
        return v, res
    v, res = run(go())
    # the three buffered requests are one device pass (the worker's batchable grouping, worker.ts:51-86)
    assert res == [True, True, True] and v.passes == [("multi", [1, 1, 1])]


def test_batchable_buffer_flushes_past_max_buffered_sigs():
    async def go():
        v = Recorder()
        opts = VerifySignatureOpts(batchable=True)
        t0 = asyncio.get_running_loop().time()
        fut = asyncio.ensure_future(v.verify_signature_sets([_set()] * (MAX_BUFFERED_SIGS + 1), opts))
        r = await fut
        return r, asyncio.get_running_loop().time() - t0
    r, dt = run(go())
    assert r is True and dt < 0.09  # flushed at once, not after the 100 ms timer


def test_bad_set_fails_only_its_own_request():
    # multithread.test.ts:109-129: one bad request in a batch does not fail the others
    async def go():
        v = Recorder()
        opts = VerifySignatureOpts(batchable=True)
        return await asyncio.gather(v.verify_signature_sets([_set()], opts), v.verify_signature_sets([_set(False)], opts),
                                    v.verify_signature_sets([_set()], opts))
    assert run(go()) == [True, False, True]


def test_same_message_jobs_share_one_device_pass():
    async def go():
        v = Recorder()
        r = await asyncio.gather(
            v.verify_signature_sets_same_message([(0, b"\x01" + bytes(95)), (1, b"\x00" + bytes(95))], bytes(32)),
            v.verify_signature_sets_same_message([(2, b"\x01" + bytes(95))], bytes([1]) * 32))
        return v, r
    v, r = run(go())
    assert r == [[True, False], [True]]
    assert [p for p in v.passes if p[0] == "sm"] == [("sm", [2, 1])]


def test_priority_jobs_go_first():
    async def go():
        v = Recorder()
        v._busy = MAX_PASSES_IN_FLIGHT  # hold the queue as if every pass slot were on the device
        f1 = asyncio.ensure_future(v.verify_signature_sets([_set()] * 2))
        f2 = asyncio.ensure_future(v.verify_signature_sets([_set()] * 5, VerifySignatureOpts(priority=True)))
        await asyncio.sleep(0)
        order = [len(j.sets) for j in v._jobs]
        assert v.can_accept_work() is False
        v._busy = 0
        v._schedule()
        await asyncio.gather(f1, f2)
        return order
    assert run(go()) == [5, 2]


def test_close_rejects_queued_jobs_with_queue_aborted():
    async def go():
        v = Recorder()
        fut = asyncio.ensure_future(v.verify_signature_sets([_set()], VerifySignatureOpts(batchable=True)))
        await asyncio.sleep(0)
        await v.close()
        with pytest.raises(QueueAbortedError):
            await fut
        with pytest.raises(QueueAbortedError):
            await v.verify_signature_sets([_set()])
        return v.can_accept_work()
    run(go())


def test_verify_on_main_thread_is_synchronous():
    async def go():
        v = Recorder()
        r = await v.verify_signature_sets([_set()], VerifySignatureOpts(verify_on_main_thread=True))
        return v, r
    v, r = run(go())
    assert r is True and v.passes == [("sets", 1)] and v._jobs == []


class Slow(Recorder):
    """Device passes block until released (they run on worker threads, several at once)."""

    def __init__(self):
        super().__init__()
        import threading
        self.started = threading.Semaphore(0)
        self.release = threading.Event()

    def verify_signature_sets_multi_sync(self, calls):
        self.started.release()
        assert self.release.wait(5)
        return super().verify_signature_sets_multi_sync(calls)


async def _wait_started(v, k):
    for _ in range(k):
        while not v.started.acquire(blocking=False):
            await asyncio.sleep(0.001)


def test_close_waits_for_the_running_device_passes():
    """close() while device passes run on worker threads: they finish (their jobs resolve) before
    gbv_destroy frees the context; jobs still queued reject with QUEUE_ABORTED."""
    async def go():
        v = Slow()
        running = []
        for k in range(MAX_PASSES_IN_FLIGHT):  # every pass slot busy
            running.append(asyncio.ensure_future(v.verify_signature_sets([_set()])))
            while v._busy < k + 1:
                await asyncio.sleep(0)
        await _wait_started(v, MAX_PASSES_IN_FLIGHT)
        assert v._busy == MAX_PASSES_IN_FLIGHT and not v.can_accept_work()
        queued = asyncio.ensure_future(v.verify_signature_sets([_set()]))
        await asyncio.sleep(0)
        assert len(v._jobs) == 1  # waits for a free pass slot
        closing = asyncio.ensure_future(v.close())
        await asyncio.sleep(0.02)
        assert v.destroyed_after is None  # still waiting for the passes in flight
        v.release.set()
        await closing
        assert v.destroyed_after == [("multi", [1])] * MAX_PASSES_IN_FLIGHT
        assert [await r for r in running] == [True] * MAX_PASSES_IN_FLIGHT
        with pytest.raises(QueueAbortedError):
            await queued
    run(go())


def test_passes_overlap_and_the_next_takes_every_queued_job():
    """Up to MAX_PASSES_IN_FLIGHT passes run at once (index.ts:357-534 keeps every worker busy);
    jobs queued meanwhile go into ONE pass when a slot frees up."""
    async def go():
        v = Slow()
        first = []
        for k in range(MAX_PASSES_IN_FLIGHT):  # one pass each: the next call arrives once a pass started
            first.append(asyncio.ensure_future(v.verify_signature_sets([_set()] * (k + 1))))
            while v._busy < k + 1:
                await asyncio.sleep(0)
        await _wait_started(v, MAX_PASSES_IN_FLIGHT)
        later = [asyncio.ensure_future(v.verify_signature_sets([_set(k != 1)])) for k in range(4)]
        await asyncio.sleep(0.01)
        assert len(v._jobs) == 4 and not v.can_accept_work()
        v.release.set()
        res = await asyncio.gather(*first, *later)
        return v, res
    v, res = run(go())
    assert res == [True] * MAX_PASSES_IN_FLIGHT + [True, False, True, True]
    # passes are recorded as their device waits finish, so the queued jobs' pass may land among the
    # first ones: compare as a multiset
    assert sorted(v.passes) == sorted([("multi", [k + 1]) for k in range(MAX_PASSES_IN_FLIGHT)] + [("multi", [1, 1, 1, 1])])
    assert v.device_passes == MAX_PASSES_IN_FLIGHT + 1


def test_invalid_call_rejects_alone_before_queueing():
    """an out-of-range index or a malformed root rejects its own call, not the others
    that would share its device pass."""
    async def go():
        v = Recorder()
        opts = VerifySignatureOpts(batchable=True)
        good = asyncio.ensure_future(v.verify_signature_sets([_set()], opts))
        with pytest.raises(GbvError):
            await v.verify_signature_sets([SingleSignatureSet(1 << 20, bytes(32), b"\x01" + bytes(95))], opts)
        with pytest.raises(ValueError):
            await v.verify_signature_sets([SingleSignatureSet(0, bytes(31), b"\x01" + bytes(95))], opts)
        with pytest.raises(GbvError):
            await v.verify_signature_sets_same_message([(1 << 20, b"\x01" + bytes(95))], bytes(32))
        empty = asyncio.ensure_future(v.verify_signature_sets([AggregatedSignatureSet([], bytes(32), b"\x01" + bytes(95))], opts))
        r = await good
        with pytest.raises(EmptyAggregateError):
            await empty
        return v, r
    v, r = run(go())
    assert r is True and v.passes == [("multi", [1, 1])]


def test_packed_same_message_sets():
    async def go():
        v = Recorder()
        sigs = b"".join((b"\x01" if i % 3 else b"\x00") + bytes(95) for i in range(200))
        r = await v.verify_signature_sets_same_message(PackedSameMessageSets(np.arange(200), sigs), bytes(32))
        return v, r
    v, r = run(go())
    assert isinstance(r, np.ndarray) and r.tolist() == [i % 3 != 0 for i in range(200)]
    assert v.passes == [("sm", [200])]  # 200 < 256: one chunk (chunkifyMaximizeChunkSize)


def test_close_sync_rejects_buffered_jobs():
    async def go():
        v = Recorder()
        fut = asyncio.ensure_future(v.verify_signature_sets([_set()], VerifySignatureOpts(batchable=True)))
        await asyncio.sleep(0)
        v.close_sync()
        with pytest.raises(QueueAbortedError):
            await fut
        return v
    v = run(go())
    assert v.passes == [] and v.destroyed_after == []


def test_staged_batches_are_released_before_the_context():
    """staged handles still alive at close are destroyed before gbv_destroy; closing
    them afterwards is a no-op."""
    v = Recorder()
    log = []

    class _Lib:
        def gbv_sm_batch_destroy(self, ctx, h):
            log.append(("sm", ctx))

        def gbv_destroy(self, ctx):
            log.append(("ctx", ctx))
    v._lib = _Lib()
    v._ctx = "ctx"
    st = StagedSameMessage(v, "h", 1)
    v._staged.add(st)
    v.close_sync()
    assert log == [("sm", "ctx"), ("ctx", "ctx")]
    st.close()
    del st
    assert log == [("sm", "ctx"), ("ctx", "ctx")]


def test_metric_families_match_the_reference_names():
    async def go():
        v = Recorder()
        await v.verify_signature_sets([_set(), _set(False)], VerifySignatureOpts(batchable=True, priority=True))
        await v.verify_signature_sets_same_message([(0, b"\x01" + bytes(95)), (1, b"\x00" + bytes(95))], bytes(32))
        return v
    v = run(go())
    m = v.pool_metrics
    text = m.exposition().decode()
    for name in ("lodestar_bls_thread_pool_sig_sets_total", "lodestar_bls_thread_pool_jobs_started_total",
                 "lodestar_bls_thread_pool_queue_job_wait_time_seconds", "lodestar_bls_thread_pool_workers_busy",
                 "lodestar_bls_thread_pool_same_message_sets_retries_total", "lodestar_bls_worker_thread_time_per_sigset_seconds",
                 "lodestar_bls_thread_pool_gpu_device_passes_total"):
        assert name in text, name
    assert m.value("lodestar_bls_thread_pool_sig_sets_total") == 4
    assert m.value("lodestar_bls_thread_pool_batchable_sig_sets_total") == 2
    assert m.value("lodestar_bls_thread_pool_prioritized_sig_sets_total") == 2
    assert m.value("lodestar_bls_thread_pool_jobs_started_total", {"type": "sameMessage"}) == 1
    assert m.value("lodestar_bls_thread_pool_same_message_sets_retries_total") == 2
    assert m.value("lodestar_bls_thread_pool_gpu_device_passes_total") == 2


def test_deep_queue_is_cut_into_overlapping_passes(monkeypatch):
    # a burst of gossip calls deeper than MAX_PASS_SETS becomes several passes (each <= the cap plus
    # its last job), so they overlap on the device; every call still resolves with its own booleans
    import lodestar_amd.verifier as V
    monkeypatch.setattr(V, "MAX_PASS_SETS", 100)

    async def go():
        v = Recorder()
        sig = lambda ok: (b"\x01" if ok else b"\x00") + bytes(95)  # noqa: E731
        calls = [[(i, sig((i + g) % 7 != 0)) for i in range(40)] for g in range(10)]
        res = await asyncio.gather(*[v.verify_signature_sets_same_message(c, bytes([g]) * 32) for g, c in enumerate(calls)])
        return v, calls, res
    v, calls, res = run(go())
    sm_passes = [p[1] for p in v.passes if p[0] == "sm"]
    assert sum(len(p) for p in sm_passes) == 10 and len(sm_passes) >= 3
    assert all(sum(p) - p[-1] < 100 for p in sm_passes)
    assert res == [[(i + g) % 7 != 0 for i in range(40)] for g in range(10)]


def test_out_of_range_index_rejects_its_call_inside_a_shared_pass():
    # the index range check runs over the whole pass; only the call naming a missing slot rejects
    async def go():
        v = Recorder()
        ok = b"\x01" + bytes(95)
        good1 = v.submit_signature_sets_same_message(PackedSameMessageSets(np.array([1, 2], dtype=np.uint32), ok * 2), bytes(32))
        bad = v.submit_signature_sets_same_message(PackedSameMessageSets(np.array([3, 1 << 20], dtype=np.uint32), ok * 2), bytes(32))
        good2 = v.submit_signature_sets_same_message([(5, ok)], bytes(32))
        r1 = await good1
        with pytest.raises(GbvError):
            await bad
        r2 = await good2
        return v, r1, r2
    v, r1, r2 = run(go())
    assert r1.tolist() == [True, True] and r2 == [True]
    assert [p for p in v.passes if p[0] == "sm"] == [("sm", [2, 1])]


def test_same_message_public_method_is_a_coroutine():
    """The IBlsVerifier method is async (like the reference's): it composes with gather, wait_for and
    create_task, and an argument error rejects when awaited, not at the call."""
    async def go():
        v = Recorder()
        ok = b"\x01" + bytes(95)
        coro = v.verify_signature_sets_same_message([(0, ok)], bytes(5))  # bad message length: no raise yet
        assert asyncio.iscoroutine(coro)
        with pytest.raises(ValueError):
            await coro
        t = asyncio.create_task(v.verify_signature_sets_same_message([(1, ok)], bytes(32)))
        a, b = await asyncio.gather(v.verify_signature_sets_same_message([(2, ok), (3, ok)], bytes(32)),
                                    asyncio.wait_for(v.verify_signature_sets_same_message([(4, ok)], bytes(32)), 10))
        return await t, a, b
    r, a, b = run(go())
    assert r == [True] and a == [True, True] and b == [True]
