"""C5 probe: the 1M-set same-message stream with 1 % invalid sets (bench.c5_bench, every boolean
checked), more steps than the bench line, plus the per-stage kernel times of the last batch.
Usage: python tools/c5_probe.py [--sets 1048576] [--steps 8] [--depth 2] [--tune name=value]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--depth", type=int, default=2)
    ap.add_argument("--tune", action="append", default=[], metavar="NAME=VALUE", help="gbv_tune settings for the run")
    a = ap.parse_args()
    from lodestar_amd import GpuBlsVerifier
    v = GpuBlsVerifier(0)
    log = lambda m: print("[c5] " + m, file=sys.stderr, flush=True)
    sks, _ = bench.build_table(v, log)
    call_off, idx, sigs, msgs = bench.build_workload(v, sks, a.sets, 0, log)
    for t in a.tune:
        name, value = t.split("=")
        v.tune(name, int(value))
    r = bench.c5_bench(v, call_off, idx, sigs, msgs, steps=a.steps, depth=a.depth)
    print("C5 %.3f M sets/s, %.1f ms per step, fallback chunks %s, failed segments %s" % (
        r["value"] / 1e6, r["ms_per_step"], r["last_fallback_chunks"], r["last_failed_segments"]), flush=True)
    for k in r["last_step_kernels"]:
        print("  %-28s grid %8d units %8d %9.3f ms" % (k["kernel"], k["grid"], k["units"], k["ms"]), flush=True)
    v.close_sync()


if __name__ == "__main__":
    main()
