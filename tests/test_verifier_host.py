"""Host logic of the IBlsVerifier mirror (lodestar_amd/verifier.py) on CPU: queueing, batchable
buffering, priority, chunking, close() -> QUEUE_ABORTED, canAcceptWork -- the scheduling rules of
BlsMultiThreadWorkerPool (packages/beacon-node/src/chain/bls/multithread/index.ts:149-155,
157-236, 302-352, 519-550).  The device calls are replaced by a recorder (no GPU, no oracle
needed: these tests are about which device passes happen and what the promises resolve to).
"""
import asyncio

import pytest

from lodestar_amd import QueueAbortedError, SingleSignatureSet, VerifySignatureOpts
from lodestar_amd.verifier import GpuBlsVerifier, MAX_BUFFERED_SIGS, chunkify_maximize_chunk_size


class Recorder(GpuBlsVerifier):
    """GpuBlsVerifier with the device passes replaced: a set is "valid" iff its signature starts
    with 0x01; every device pass is logged."""

    def __init__(self):  # no gbv_init: nothing touches a GPU
        self._closed = False
        self._jobs = []
        self._buffered = None
        self._busy = 0
        self._idle = None
        self._run_scheduled = False
        self.destroyed_after = None
        self.metrics = {"total_sig_sets": 0, "batchable_sig_sets": 0, "same_message_sets": 0,
                        "device_passes": 0, "same_message_retry_sets": 0}
        self.passes = []

        rec = self

        class _Lib:
            def gbv_destroy(self, ctx):
                rec.destroyed_after = list(rec.passes)
        self._lib = _Lib()
        self._ctx = None

    def verify_signature_sets_sync(self, sets):
        self.passes.append(("sets", len(sets)))
        return len(sets) > 0 and all(bytes(s.signature)[:1] == b"\x01" for s in sets)

    def verify_signature_sets_multi_sync(self, calls):
        self.passes.append(("multi", [len(c) for c in calls]))
        return [len(c) > 0 and all(bytes(s.signature)[:1] == b"\x01" for s in c) for c in calls]

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
        v._busy = 1  # hold the queue as if a device pass were in flight
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


def test_close_waits_for_the_running_device_pass():
    """close() while a device pass runs on the worker thread: the pass finishes (its job resolves)
    before gbv_destroy frees the context; queued jobs reject with QUEUE_ABORTED."""
    import threading

    class Slow(Recorder):
        def __init__(self):
            super().__init__()
            self.started = threading.Event()
            self.release = threading.Event()

        def verify_signature_sets_multi_sync(self, calls):
            self.started.set()
            assert self.release.wait(5)
            return super().verify_signature_sets_multi_sync(calls)

    async def go():
        v = Slow()
        running = asyncio.ensure_future(v.verify_signature_sets([_set()]))
        while not v.started.is_set():
            await asyncio.sleep(0.001)
        queued = asyncio.ensure_future(v.verify_signature_sets([_set()]))
        await asyncio.sleep(0)
        closing = asyncio.ensure_future(v.close())
        await asyncio.sleep(0.02)
        assert v.destroyed_after is None  # still waiting for the pass in flight
        v.release.set()
        await closing
        assert v.destroyed_after == [("multi", [1])]
        assert await running is True
        with pytest.raises(QueueAbortedError):
            await queued
    run(go())
