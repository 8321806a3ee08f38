"""Where the time of one small same-message call goes (create / submit+wait / destroy), on the GPU."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import bench  # noqa: E402
from lodestar_amd import GpuBlsVerifier  # noqa: E402

v = GpuBlsVerifier(0)
call_off, idx, sigs, msgs, _ = bench.build_workload(v, 4096, 0, lambda m: None)
n = 64
off = np.array([0, n], dtype=np.uint32)
for rep in range(8):
    t0 = time.perf_counter()
    st = v.stage_same_message(off, idx[:n], sigs[:96 * n], msgs[:32])
    t1 = time.perf_counter()
    res = st.verify(True)
    t2 = time.perf_counter()
    st.close()
    t3 = time.perf_counter()
    kms, cnt = v.last_kernel_ms()
    print("create %.2f ms  verify %.2f ms  destroy %.2f ms  kernels %s  valid %d" % (
        (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, [round(x, 2) for x in kms], res.count(1)), flush=True)
