"""Host-only cost of the IBlsVerifier same-message path (no GPU): bench.py's api_stream_rate workload
(13k gossip calls of 32-128 packed sets, ~1M sets) issued through GpuBlsVerifier with the device
library replaced by a stub whose batch wait sleeps for one device pass's measured time (12.8 ms per
2^18 sets, C2's staged rate).  Prints the wall time, the time to create the 13k call futures and to
build the caller's asyncio.gather, so the Python share of bench.py's api_path_sets_per_s can be
read off without a GPU.  Usage: python tools/api_host_overhead.py [--profile]"""
import asyncio
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lodestar_amd import PackedSameMessageSets  # noqa: E402
from lodestar_amd import verifier as V  # noqa: E402

PASS_S = (1 << 18) / 20.4e6


class StubLib:
    def __getattr__(self, name):
        def f(*a):
            if name == "gbv_sm_batch_wait":
                time.sleep(PASS_S)
            return 0
        return f


def make_verifier():
    v = object.__new__(V.GpuBlsVerifier)
    v._init_host_state()
    v._lib, v._ctx, v._device = StubLib(), ctypes.c_void_p(1), 0
    V.GpuBlsVerifier.pubkey_count = property(lambda self: 1 << 21)
    V._native.check = lambda lib, ctx, rc: None
    return v


def main():
    v = make_verifier()
    rng = np.random.default_rng(1)
    sizes = rng.integers(32, 129, size=13000)
    off = np.concatenate([[0], np.cumsum(sizes)])
    n = int(off[-1])
    idx = rng.integers(0, 1 << 20, size=n).astype(np.uint32)
    mv = memoryview(bytes(96 * n))
    reqs = [(PackedSameMessageSets(idx[off[g]:off[g + 1]], mv[96 * off[g]:96 * off[g + 1]]), bytes(32)) for g in range(len(sizes))]
    call = v.submit_signature_sets_same_message

    async def go():
        t = time.perf_counter()
        fs = [call(s, m) for s, m in reqs]
        t1 = time.perf_counter()
        g = asyncio.gather(*fs)
        t2 = time.perf_counter()
        res = await g
        assert sum(len(r) for r in res) == n
        return t1 - t, t2 - t1

    asyncio.run(go())
    for _ in range(3):
        t = time.perf_counter()
        tc, tg = asyncio.run(go())
        dt = time.perf_counter() - t
        print("%d sets in %d calls: %.1f ms (%.2fM sets/s); creating the calls %.1f ms (%.2f us/call), gather %.1f ms" % (
            n, len(reqs), dt * 1e3, n / dt / 1e6, tc * 1e3, tc / len(reqs) * 1e6, tg * 1e3))
    if "--profile" in sys.argv:
        import cProfile
        import pstats
        cProfile.runctx("asyncio.run(go())", globals(), locals(), "/tmp/api_host.prof")
        pstats.Stats("/tmp/api_host.prof").sort_stats("tottime").print_stats(15)


if __name__ == "__main__":
    main()
