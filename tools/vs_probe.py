"""verifySignatureSets probe: the C3 pass (512 calls of 128-member aggregates) and the C1 throughput
pass (512 calls of 128 single sets) under each Miller form for passes above vs_pair_max
(vs_miller_k = 1: a thread per set, 2 / 4: k_vs_miller_group), every boolean checked, with the
per-kernel times of the last pass.  Usage: python tools/vs_probe.py [--ks 1,2,4] [--steps 6]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def run(v, calls, steps, label, k):
    v.tune("vs_miller_k", k)
    stages = [v.stage_signature_sets(calls) for _ in range(2)]
    try:
        for st in stages:
            assert st.verify() == [1] * len(calls)
        dt, ops = bench._timed_ops(v, stages, steps, [1] * len(calls))
    finally:
        for st in stages:
            st.close()
        v.tune("vs_miller_k", 1)
    n = sum(len(c) for c in calls)
    print("%s k=%d: %.3f M sets/s, %.2f ms per pass" % (label, k, n / dt / 1e6, dt * 1e3), flush=True)
    for name, g, u, ms in ops:
        print("  %-28s grid %8d units %8d %9.3f ms" % (name, g, u, ms), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ks", default="1,2,4")
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--calls", type=int, default=512)
    a = ap.parse_args()
    from lodestar_amd import GpuBlsVerifier
    v = GpuBlsVerifier(0)
    log = lambda m: print("[vs] " + m, file=sys.stderr, flush=True)
    sks, _ = bench.build_table(v, log)
    sk_ints = [bench.interop_sk_int(i) for i in range(bench.N_KEYS)]
    rng = np.random.Generator(np.random.PCG64(0xC3))
    c3 = bench._agg_sets(v, sk_ints, a.calls * 128, b"gbv-c3", rng)
    c3 = [c3[i:i + 128] for i in range(0, len(c3), 128)]
    c1 = bench._single_sets(v, sks, a.calls * 128, b"gbv-c1-many", rng)
    c1 = [c1[i:i + 128] for i in range(0, len(c1), 128)]
    ks = [int(x) for x in a.ks.split(",")]
    for k in ks:
        run(v, c3, a.steps, "C3", k)
    for k in ks:
        run(v, c1, a.steps, "C1", k)
    v.close_sync()


if __name__ == "__main__":
    main()
