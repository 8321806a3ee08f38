"""CPU baseline leg of bench.py -- TEST/BENCH INFRASTRUCTURE ONLY (see oracle/bls_oracle.py header).

Times oracle/c/blsport.c (a C port of the same-message verification path; "CPU stand-in, not
blst") through the reference pool's shape: availableParallelism()-1 worker
threads (multithread/index.ts:46, poolSize.ts:7) pulling <=128-set chunks, on a bounded sample of
the bench workload.  Never imported by the product package.
"""
import ctypes
import os
import subprocess
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "c", "libblsport.so")


def load():
    src = os.path.join(HERE, "c", "blsport.c")
    if os.environ.get("GBV_BLSPORT_LIB"):  # a sanitizer build (tools/sanitize_host.sh)
        lib = ctypes.CDLL(os.environ["GBV_BLSPORT_LIB"])
    else:
        if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
            subprocess.check_call([os.path.join(HERE, "c", "build.sh")])
        lib = ctypes.CDLL(LIB)
    lib.port_verify_same_message_batch.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_char_p,
                                                   ctypes.c_char_p, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_uint64]
    lib.port_g1_decompress.argtypes = [ctypes.c_char_p, ctypes.c_void_p]
    return lib


def pool_threads():
    """availableParallelism() - 1, bounded by the CPU share the job may use."""
    n = len(os.sched_getaffinity(0))
    cap = os.environ.get("OMP_NUM_THREADS")
    if cap and cap.isdigit():
        n = min(n, int(cap))
    return max(1, n - 1)


def measure_same_message(call_off, idx, sigs96, msgs32, table_pk48, n_keys, target_sets=32768, threads=None):
    """Verify the first calls of the workload (about `target_sets` sets) on the CPU pool shape.
    table_pk48: compressed pubkeys of the key set (validator i uses key i mod n_keys).
    Returns the `cpu_baseline` dict of the bench line."""
    lib = load()
    threads = threads or pool_threads()
    call_off = np.asarray(call_off, dtype=np.uint32)
    k = int(np.searchsorted(call_off, min(target_sets, int(call_off[-1])), side="left"))
    k = max(1, min(k, len(call_off) - 1))
    n = int(call_off[k])
    # index2pubkey is already deserialized in the reference (PublicKey objects): not timed
    aff = []
    for pk in table_pk48:
        out = ctypes.create_string_buffer(96)
        assert lib.port_g1_decompress(pk, out) == 0
        aff.append(out.raw)
    aff = np.frombuffer(b"".join(aff), dtype=np.uint8).reshape(len(table_pk48), 96)
    pk_aff = np.ascontiguousarray(aff[np.asarray(idx[:n]) % n_keys]).tobytes()
    valid = (ctypes.c_uint8 * n)()
    off = np.ascontiguousarray(call_off[:k + 1])
    t = time.perf_counter()
    lib.port_verify_same_message_batch(threads, k, off.ctypes.data, pk_aff, bytes(sigs96[:96 * n]), bytes(msgs32[:32 * k]),
                                       valid, int.from_bytes(os.urandom(8), "little"))
    dt = time.perf_counter() - t
    ok = sum(valid)
    return {"value": round(n / dt, 1), "unit": "sets/s", "cores": threads, "kind": "port",
            "sample": "%d sets in %d same-message calls (first calls of the bench workload), %.2fs wall, "
                      "%d/%d valid; oracle/c/blsport.c, C port not blst, %d worker threads" % (n, k, dt, ok, n, threads),
            "all_valid": ok == n}


def _declare_vs(lib):
    lib.port_verify_sets_batch.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_uint64]


def affine_rows(lib, pks48):
    """96-byte affine rows (x||y) of compressed pubkeys -- the deserialized index2pubkey the
    reference already holds (not timed)."""
    rows = []
    for pk in pks48:
        out = ctypes.create_string_buffer(96)
        assert lib.port_g1_decompress(bytes(pk), out) == 0
        rows.append(out.raw)
    return b"".join(rows)


def run_verify_sets(lib, calls, pk_rows, threads=1, seed=None):
    """verifySignatureSets calls on the port.  calls: list of lists of (pk row indices, msg32, sig96);
    pk_rows: concatenated 96-byte affine rows.  Returns (per-call booleans, seconds)."""
    _declare_vs(lib)
    call_off, pk_off, pk_idx, msgs, sigs = [0], [0], [], [], []
    for c in calls:
        for rows, m, s in c:
            pk_idx.extend(rows)
            pk_off.append(len(pk_idx))
            msgs.append(bytes(m))
            sigs.append(bytes(s) if len(s) == 96 else bytes(96))
        call_off.append(len(pk_off) - 1)
    co = np.array(call_off, dtype=np.uint32)
    po = np.array(pk_off, dtype=np.uint32)
    pi = np.array(pk_idx or [0], dtype=np.uint32)
    out = (ctypes.c_uint8 * max(len(calls), 1))()
    seed = seed if seed is not None else int.from_bytes(os.urandom(8), "little")
    t = time.perf_counter()
    lib.port_verify_sets_batch(threads, len(calls), co.ctypes.data, po.ctypes.data, pi.ctypes.data, pk_rows, b"".join(msgs) or b"\0",
                               b"".join(sigs) or b"\0", out, seed)
    dt = time.perf_counter() - t
    return [bool(out[i]) for i in range(len(calls))], dt


def measure_verify_sets(calls, pk_rows, threads=None, label=""):
    """`cpu_baseline` dict of a verifySignatureSets config: the port through the pool shape
    (threads workers pulling <=128-set jobs) on the given bounded sample of calls."""
    lib = load()
    threads = threads or pool_threads()
    res, dt = run_verify_sets(lib, calls, pk_rows, threads)
    n = sum(len(c) for c in calls)
    return {"value": round(n / dt, 1), "unit": "sets/s", "cores": threads, "kind": "port",
            "sample": "%d sets in %d verifySignatureSets calls%s, %.2fs wall, %d/%d calls true; oracle/c/blsport.c "
                      "(C port, not blst), %d worker threads" % (n, len(calls), label, dt, sum(res), len(calls), threads),
            "all_valid": all(res)}


def measure_lone_call_latency(idx, sigs96, msg32, table_pk48, n_keys, n=64, reps=5):
    """Latency of ONE verifySignatureSetsSameMessage call of n sets on the CPU port, the way the
    reference pool runs a lone gossip call: one job, aggregateWithRandomness + one verify, no other
    work to share the cores with -- i.e. single-threaded (multithread/index.ts:212-236, jobItem.ts:
    69-88).  Beside bench.py's p50_batch_latency_ms (the same call on the GPU through the API).
    Returns {"p50_ms", "reps", "threads", "kind", "sample"}."""
    lib = load()
    aff = {}
    rows = []
    for i in range(n):
        k = int(idx[i]) % n_keys
        if k not in aff:
            out = ctypes.create_string_buffer(96)
            assert lib.port_g1_decompress(bytes(table_pk48[k]), out) == 0
            aff[k] = out.raw
        rows.append(aff[k])
    off = np.array([0, n], dtype=np.uint32)
    lat, ok = [], True
    for _ in range(reps):
        valid = (ctypes.c_uint8 * n)()
        t = time.perf_counter()
        lib.port_verify_same_message_batch(1, 1, off.ctypes.data, b"".join(rows), bytes(sigs96[:96 * n]), bytes(msg32[:32]), valid,
                                           int.from_bytes(os.urandom(8), "little"))
        lat.append((time.perf_counter() - t) * 1e3)
        ok = ok and sum(valid) == n
    return {"p50_ms": round(float(np.median(lat)), 3), "reps": reps, "threads": 1, "kind": "port", "all_valid": ok,
            "sample": "one %d-set same-message call (the first call's message), oracle/c/blsport.c (C port, not blst), "
                      "one thread as the pool runs a lone job" % n}
