"""C4 / C4e probe: the block-shaped verifySignatureSets passes (bench.c4_bench: 64 phase0 blocks or 16
Electra blocks per pass, 2 in flight, every boolean checked) under optional gbv_tune settings, with
the last pass's per-kernel times.  Usage: python tools/c4_probe.py [--electra] [--depth 2] [--tune name=value ...]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--electra", action="store_true")
    ap.add_argument("--tune", action="append", default=[], metavar="NAME=VALUE")
    ap.add_argument("--depth", type=int, default=2, help="passes in flight")
    a = ap.parse_args()
    from lodestar_amd import GpuBlsVerifier
    v = GpuBlsVerifier(0)
    log = lambda m: print("[c4] " + m, file=sys.stderr, flush=True)
    sks, pks = bench.build_table(v, log)
    sk_ints = [bench.interop_sk_int(i) for i in range(bench.N_KEYS)]
    for t in a.tune:
        name, value = t.split("=")
        v.tune(name, int(value))
    r = bench.c4_bench(v, sk_ints, None, False, n_blocks=16 if a.electra else 64, electra=a.electra, depth=a.depth)
    print("%s %s depth %d: %.1f k sets/s, lone block %.2f ms" % ("C4e" if a.electra else "C4", " ".join(a.tune), a.depth, r["value"] / 1e3,
                                                         r["lone_block_latency_ms_p50"]), flush=True)
    for k in r["roofline"].get("kernels", []):
        print("  %-28s grid %8d units %8d %9.3f ms" % (k["kernel"], k["grid"], k["units"], k["ms"]), flush=True)
    v.close_sync()


if __name__ == "__main__":
    main()
