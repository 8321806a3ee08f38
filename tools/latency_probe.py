"""Where the time of one lone 64-set same-message call goes (bench.py's p50 path), on the GPU.

    python tools/latency_probe.py            # per-call wall time and per-kernel event times
    rocprofv3 --kernel-trace -d gpurun_out/lat -- python3 tools/latency_probe.py   # timeline
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from lodestar_amd import GpuBlsVerifier  # noqa: E402

v = GpuBlsVerifier(0)
sks, _ = bench.build_table(v, lambda m: None)
call_off, idx, sigs, msgs = bench.build_workload(v, sks, 4096, 0, lambda m: None)
n = 64
calls = [([(int(idx[i]), sigs[96 * i:96 * i + 96]) for i in range(n)], msgs[:32])]
for rep in range(12):
    t0 = time.perf_counter()
    res = v.verify_same_message_multi_sync(calls)
    t1 = time.perf_counter()
    kms, cnt = v.last_kernel_ms()
    print("call %.2f ms  kernels %s  valid %d" % ((t1 - t0) * 1e3, dict(zip(bench.KERNELS, [round(float(x), 2) for x in kms])),
                                                  sum(sum(r) for r in res)), flush=True)
# the same lone call with one invalid set (set 5 carries set 6's signature): chunk check fails, then
# the run checks and the per-set checks (the few-item cooperative failure path)
bad = [(calls[0][0][i][0], calls[0][0][6][1] if i == 5 else calls[0][0][i][1]) for i in range(n)]
for rep in range(6):
    t0 = time.perf_counter()
    res = v.verify_same_message_multi_sync([(bad, calls[0][1])])
    t1 = time.perf_counter()
    kms, cnt = v.last_kernel_ms()
    assert list(res[0]) == [i != 5 for i in range(n)], res
    print("bad call %.2f ms  kernels %s  valid %d" % ((t1 - t0) * 1e3, dict(zip(bench.KERNELS, [round(float(x), 2) for x in kms])),
                                                      sum(sum(r) for r in res)), flush=True)
# C1: one verifySignatureSets call of 128 distinct-message single-pubkey sets
rng = np.random.Generator(np.random.PCG64(0xC1))
sets = bench._single_sets(v, sks, 128, b"gbv-c1", rng)
for rep in range(8):
    t0 = time.perf_counter()
    ok = v.verify_signature_sets_sync(sets)
    t1 = time.perf_counter()
    print("c1 call %.2f ms  kernels %s  ok %s" % ((t1 - t0) * 1e3, dict(zip(bench.VS_KERNELS, [round(float(x), 2) for x in v.vs_last_kernel_ms()])), ok),
          flush=True)
# C4: one deneb block and one electra block (8 aggregates of 32 768 validators) as lone calls
sk_ints = [bench.interop_sk_int(i) for i in range(bench.N_KEYS)]
for name, electra in (("c4 block", False), ("c4e block", True)):
    calls = bench.make_blocks(v, sk_ints, 1, np.random.Generator(np.random.PCG64(0xB10C)), electra=electra)
    for rep in range(6):
        t0 = time.perf_counter()
        ok = v.verify_signature_sets_sync(calls[0])
        t1 = time.perf_counter()
        print("%s %.2f ms  kernels %s  ok %s" % (name, (t1 - t0) * 1e3, dict(zip(bench.VS_KERNELS, [round(float(x), 2) for x in v.vs_last_kernel_ms()])),
                                              ok), flush=True)
v.close_sync()
