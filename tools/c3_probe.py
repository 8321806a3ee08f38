"""C3 probe: bench.c3_bench's verifySignatureSets pass (512 calls x 128 aggregate sets of 128 members
over the 1M table), 2 passes in flight, more steps than the bench line; prints sets/s and the last
pass's stage times.  Usage: python tools/c3_probe.py [--calls 512] [--steps 8]"""
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
    ap.add_argument("--calls", type=int, default=512)
    ap.add_argument("--steps", type=int, default=8)
    a = ap.parse_args()
    from lodestar_amd import GpuBlsVerifier
    v = GpuBlsVerifier(0)
    log = lambda m: print("[c3] " + m, file=sys.stderr, flush=True)
    bench.build_table(v, log)
    sk_ints = [bench.interop_sk_int(i) for i in range(bench.N_KEYS)]
    rng = np.random.Generator(np.random.PCG64(0xC3))
    sets = bench._agg_sets(v, sk_ints, a.calls * 128, b"gbv-c3", rng)
    calls = [sets[i:i + 128] for i in range(0, len(sets), 128)]
    stages = [v.stage_signature_sets(calls) for _ in range(2)]
    for st in stages:
        assert st.verify() == [1] * a.calls
    dt = bench._timed_staged(stages, a.steps, [1] * a.calls)
    print("C3 %.3f M sets/s, %.2f ms per pass (2 in flight); last pass stage ms %s" % (
        len(sets) / dt / 1e6, dt * 1e3, [round(x, 3) for x in v.vs_last_kernel_ms()]))
    for st in stages:
        st.close()
    v.close_sync()


if __name__ == "__main__":
    main()
