"""Probe of a small verifySignatureSets pass (range-sync segment, C4 shape): builds --blocks blocks with
bench.make_blocks, then times lone passes (one at a time, no overlap) and prints the median.  Run it
under `rocprofv3 --kernel-trace` to get the per-kernel timeline of those passes (tools/vs_timeline.py
prints the last pass).  Usage: python tools/vs_probe.py [--blocks 64] [--reps 5] [--electra]"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=64)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--electra", action="store_true")
    ap.add_argument("--inflight", type=str, default="", help="comma list of pass depths for a throughput sweep, e.g. 1,2,3")
    a = ap.parse_args()
    from lodestar_amd import GpuBlsVerifier
    v = GpuBlsVerifier(0)
    log = lambda m: print("[probe] " + m, file=sys.stderr, flush=True)
    bench.build_table(v, log)
    sk_ints = [bench.interop_sk_int(i) for i in range(bench.N_KEYS)]
    rng = np.random.Generator(np.random.PCG64(0xC4E if a.electra else 0xC4))
    calls = bench.make_blocks(v, sk_ints, a.blocks, rng, electra=a.electra)
    n = sum(len(c) for c in calls)
    st = v.stage_signature_sets(calls)
    assert st.verify() == [1] * a.blocks
    lat = []
    for _ in range(a.reps):
        t = time.perf_counter()
        assert st.verify() == [1] * a.blocks
        lat.append((time.perf_counter() - t) * 1e3)
    ms = v.vs_last_kernel_ms()
    print("pass of %d blocks, %d sets: median %.3f ms (%s); last pass stage ms %s; %.0f sets/s one pass at a time" % (
        a.blocks, n, float(np.median(lat)), " ".join("%.2f" % x for x in lat), [round(x, 3) for x in ms], n / (np.median(lat) * 1e-3)))
    st.close()
    if a.inflight:
        lone = []
        for _ in range(2 + a.reps):
            t = time.perf_counter()
            assert v.verify_signature_sets_sync(calls[0]) is True
            lone.append((time.perf_counter() - t) * 1e3)
        print("lone block (%d sets): median %.3f ms" % (len(calls[0]), float(np.median(lone[2:]))))
        for d in [int(x) for x in a.inflight.split(",")]:
            stages = [v.stage_signature_sets(calls) for _ in range(d)]
            for b in stages:
                assert b.verify() == [1] * a.blocks
            dt = bench._timed_staged(stages, max(6, 3 * d), [1] * a.blocks)
            for b in stages:
                b.close()
            print("%d passes in flight: %.3f ms per pass, %.0f sets/s" % (d, dt * 1e3, n / dt))
    v.close_sync()


if __name__ == "__main__":
    main()
