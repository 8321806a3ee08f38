"""verifySignatureSets probe: the C3 pass (512 calls of 128-member aggregates) and the C1 throughput
pass (512 calls of 128 single sets), 2 (or --depths) passes in flight, every boolean checked, with the per-kernel
times of the last pass; optional launch-shape settings (gbv_tune) per run.
Usage: python tools/vs_probe.py [--tune name=value ...] [--steps 6]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def run(v, calls, steps, label, depth):
    stages = [v.stage_signature_sets(calls) for _ in range(depth)]
    try:
        for st in stages:
            assert st.verify() == [1] * len(calls)
        dt, ops = bench._timed_ops(v, stages, steps, [1] * len(calls))
    finally:
        for st in stages:
            st.close()
    n = sum(len(c) for c in calls)
    print("%s (%d in flight): %.3f M sets/s, %.2f ms per pass" % (label, depth, n / dt / 1e6, dt * 1e3), flush=True)
    for name, g, u, ms in ops:
        print("  %-28s grid %8d units %8d %9.3f ms" % (name, g, u, ms), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tune", action="append", default=[], metavar="NAME=VALUE")
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--calls", type=int, default=512)
    ap.add_argument("--depths", default="2", help="passes in flight, comma-separated")
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
    for t in a.tune:
        name, value = t.split("=")
        v.tune(name, int(value))
    for d in [int(x) for x in a.depths.split(",")]:
        run(v, c3, a.steps, "C3", d)
        run(v, c1, a.steps, "C1", d)
    v.close_sync()


if __name__ == "__main__":
    main()
