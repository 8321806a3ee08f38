#!/usr/bin/env python3
"""Headline benchmark: signature sets verified per second on MI355X (BASELINE.json `metric`).

Workload (BASELINE.json configs[1]): the gossip attestation stream -- 1,048,576
single-pubkey signature sets in verifySignatureSetsSameMessage calls of 32-128 sets (uniform
sizes, numpy PCG64(seed=2)), validators drawn without replacement from a 1,048,576-entry
HBM-resident index2pubkey table whose keys are interop keys sk_i = interopSecretKey(i mod 1024)
(state-transition/src/util/interop.ts:18-22), messages m_g = sha256("gbv-bench" || u64le(g)),
signatures sk*H(m) produced on the GPU before timing.  A "step" = one verification pass over the
whole staged workload (inputs resident in HBM, per-set booleans copied back to the host).

Multi-GPU: one process per GPU (torch.distributed.run), each rank verifies its own 1M-set stream
(weak scaling, no data-path collective); barrier + max-over-ranks time around the timed steps.

Prints ONE JSON line on rank 0 (contract in the task statement) with `roofline` for the dominant
kernel (k_sm_prepare, integer-VALU bound) and `cpu_baseline` (the C port in oracle/, timed on the
host cores of this box on a bounded sample).
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
N_VALIDATORS = 1 << 20
N_KEYS = 1024
# Algorithmic work per unit, in Fp-multiplication equivalents (FME; 1 FME = 300 u32 MACs,
# 12-limb Montgomery), counted from the k_sm_prepare code path:
#   G2 decompress 952 (two 379-bit sliding-window exponentiations, 378 sqr + 86 mul each)
#   + G2 subgroup check 1170 (63 dbl x 16 + 5 madd x 29 + psi)
#   + randomisation 2088 (4 table madds, affine tables ~40, G1 ladder 31 x 18, G2 ladder 31 x 45;
#     the shared inversion is a binary GCD: no multiplications, so it counts 1)
#   + per-group chunk scan 177 (3 levels x (43 + 16))  = 4387 per set.
W_PREPARE_FME = 4387
# With the G2 sum of a segment formed by the bucket MSM (k_msm.hip; segments >= 131072 sets, the
# bench's 1M-set batch), k_sm_prepare keeps decompress 952 + subgroup 1170 + the G1 half of the
# randomisation 593 (2 table madds x 11 + affine tables 13 + ladder 31 x 18) + G1 scan 48 (3 x 16).
W_PREPARE_FME_MSM = 2763
MAC_PER_FME = 300
# Integer VALU peak: v_mad_u64_u32 measured at 37.0 T lane-ops/s on MI355X
# (tools/ubench_int.hip, profiles/r01_ubench_int.txt); theoretical 256 CU x 4 SIMD x 16 lanes x 2.4 GHz = 39.3 T.
PEAK_MAC_PER_S = 37.0e12
# VALU issue peak: 1024 SIMDs, one wave64 instruction per SIMD every 4 cycles at 2.4 GHz
PEAK_VALU_WAVE_INSTR_PER_S = 1024 * 2.4e9 / 4
PMC_SUMMARY = os.path.join(ROOT, "profiles", "pmc_latest.json")  # tools/pmc.sh + tools/pmc_parse.py
# k_sm_prepare algorithmic bytes per set: reads idx 4 + signature 96 + set_grp 4 + table entry 128
# (G1 affine, two 64-byte Fp slots) + table_ok 1; writes status 1 + affine signature 256 + chunk
# group sums ((1/8 + 1/80) x (384 + 192)).  The measured traffic above this is scratch spilling.
ALG_BYTES_PER_SET = 4 + 96 + 4 + 128 + 1 + 1 + 256 + round((1 / 8 + 1 / 80) * (384 + 192))


def pmc_evidence(units_per_launch, kernel="k_sm_prepare<false>"):
    """HBM traffic per launch and VALU issue utilisation of k_sm_prepare from the committed
    rocprofv3 --pmc summary (separate passes; FETCH_SIZE doubled per the gfx950 calibration in the
    MI355X guide: it counts 64 B per 128-B request; rocprofv3 reports kilobytes)."""
    try:
        summary = json.load(open(PMC_SUMMARY))
        d = summary.get(kernel) or summary["k_sm_prepare"]
    except (OSError, KeyError, ValueError):
        return None, None
    per_set = (2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024.0 / d["grid_size"]
    valu = d["SQ_INSTS_VALU"] / (d["duration_ms"] * 1e-3 * PEAK_VALU_WAVE_INSTR_PER_S)
    ev = {"source": os.path.relpath(PMC_SUMMARY, ROOT), "kernel": kernel if kernel in summary else "k_sm_prepare",
          "pmc_grid_sets": int(d["grid_size"]),
          "hbm_bytes_per_set": round(per_set, 1), "algorithmic_bytes_per_set": ALG_BYTES_PER_SET, "valu_wave_instr_per_set": round(d["SQ_INSTS_VALU"] / d["SQ_WAVES"]),
          "valu_issue_utilisation": round(valu, 4),
          "valu_lane_utilisation": round(d["SQ_THREAD_CYCLES_VALU"] / (64.0 * d["SQ_ACTIVE_INST_VALU"]), 4)}
    return per_set * units_per_launch, ev


# device kernels of one same-message verify, in gbv_last_kernel_ms order
KERNELS = ["hash", "prepare", "chunk_finish", "miller", "seg_check", "group_pairing", "fallback", "msm"]


def interop_sk_bytes(i):
    d = hashlib.sha256(i.to_bytes(32, "little")).digest()
    return (int.from_bytes(d, "little") % R_ORDER).to_bytes(32, "big")


def build_workload(v, n_sets, rank, log):
    t0 = time.time()
    sks = [interop_sk_bytes(i) for i in range(N_KEYS)]
    pks = v.util_sk_to_pk(sks)
    st = v.add_pubkeys(0, pks)
    assert st == bytes(N_KEYS), "pubkey ingest failed"
    v.replicate_pubkeys(0, N_KEYS, N_KEYS, N_VALIDATORS - N_KEYS)
    rng = np.random.Generator(np.random.PCG64(2))
    sizes = []
    total = 0
    while total < n_sets:
        s = int(rng.integers(32, 129))
        s = min(s, n_sets - total)
        sizes.append(s)
        total += s
    call_off = np.zeros(len(sizes) + 1, dtype=np.uint32)
    call_off[1:] = np.cumsum(sizes)
    perm = np.random.Generator(np.random.PCG64(0x1D5 + rank)).permutation(N_VALIDATORS)
    idx = perm[np.arange(n_sets) % N_VALIDATORS].astype(np.uint32)
    grp = np.repeat(np.arange(len(sizes), dtype=np.uint32), sizes)
    msgs = [hashlib.sha256(b"gbv-bench" + (g + rank * 10_000_000).to_bytes(8, "little")).digest()
            for g in range(len(sizes))]
    sk_arr = np.frombuffer(b"".join(sks), dtype=np.uint8).reshape(N_KEYS, 32)
    set_sks = sk_arr[idx % N_KEYS]
    log("workload: %d sets in %d calls, keys/table ready in %.1fs" % (n_sets, len(sizes), time.time() - t0))
    t1 = time.time()
    sigs = []
    CH = 1 << 18
    for a in range(0, n_sets, CH):
        b = min(n_sets, a + CH)
        sigs.extend(v.util_sign([bytes(r) for r in set_sks[a:b]], grp[a:b].tolist(), msgs))
        log("  signed %d/%d (%.1fs)" % (b, n_sets, time.time() - t1))
    log("signed %d sets on the GPU in %.1fs" % (n_sets, time.time() - t1))
    return call_off, idx, b"".join(sigs), b"".join(msgs), pks


# Signing-root row: getAttestationDataSigningRoot = 9 SHA-256 digests of 64 bytes
# (8 AttestationData nodes + the SigningData node), 2 compressions each.  Algorithmic VALU ops per
# digest with gfx950's 3-input ops (v_alignbit rotates, v_bitop3 xor3/maj/ch, v_add3): 64 rounds x 14
# per compression x 2 + 48 schedule words x 10 + 16 state adds = 2288 (the second block's schedule is
# constant).  Peak: 256 CU x 64 lanes x 2.4 GHz = 39.3 T lane-ops/s (full-rate 32-bit VALU).
SSZ_DIGESTS_PER_ROOT = 9
SSZ_OPS_PER_DIGEST = 2288
SSZ_PEAK_OPS = 256 * 64 * 2.4e9
SSZ_BYTES_PER_ROOT = 128 + 32 + 4  # AttestationData in, root out, domain index


def signing_roots_bench(v, n=1 << 20, reps=5, cpu_sample=20000):
    """Secondary line for the signing-root row: AttestationData signing roots per second with the
    inputs resident in HBM (kernel time from HIP events on the launch stream), the PCIe-inclusive rate
    of the host-buffer call, and the hashlib oracle on one host core over a bounded sample."""
    rng = np.random.default_rng(11)
    datas = rng.integers(0, 256, size=(n, 128), dtype=np.uint8).tobytes()
    doms = rng.integers(0, 256, size=(4, 32), dtype=np.uint8).tobytes()
    dom_idx = rng.integers(0, 4, size=n).tolist()
    v.attestation_data_signing_roots(datas[:128 * 1024], doms, dom_idx[:1024])
    kms, walls = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        roots = v.attestation_data_signing_roots(datas, doms, dom_idx)
        walls.append(time.perf_counter() - t0)
        kms.append(v.ssz_last_kernel_ms())
    assert len(roots) == n
    k_ms = float(np.mean(kms))
    achieved = n * SSZ_DIGESTS_PER_ROOT * SSZ_OPS_PER_DIGEST / (k_ms * 1e-3)
    out = {"metric": "AttestationData signing roots/sec", "value": round(n / (k_ms * 1e-3), 1), "unit": "roots/s",
           "roots_per_launch": n, "kernel": "k_ssz_att_signing_roots", "avg_launch_ms": round(k_ms, 4),
           "pcie_inclusive_roots_per_s": round(n / float(np.median(walls)), 1),
           "roofline": {"bound": "valu-int", "achieved": round(achieved / 1e12, 4), "peak": round(SSZ_PEAK_OPS / 1e12, 2),
                        "unit": "T lane-ops/s", "frac": round(achieved / SSZ_PEAK_OPS, 4),
                        "work_per_unit": "%d digest64 x %d ops" % (SSZ_DIGESTS_PER_ROOT, SSZ_OPS_PER_DIGEST),
                        "hbm_GBps": round(n * SSZ_BYTES_PER_ROOT / (k_ms * 1e-3) / 1e9, 1)}}
    if cpu_sample:
        from oracle import ssz_oracle
        d0 = doms[:32]
        t0 = time.perf_counter()
        for i in range(cpu_sample):
            ssz_oracle.attestation_signing_root(datas[128 * i:128 * i + 128], d0)
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(cpu_sample / dt, 1), "unit": "roots/s", "cores": 1, "kind": "port",
                               "sample": "%d roots, oracle/ssz_oracle.py (hashlib SHA-256), %.2fs" % (cpu_sample, dt)}
    return out


def inject_invalid(sigs, call_off, n_sets, frac):
    """SURVEY 8(d) C5 recipe: `frac` of the sets chosen by PCG64(0xC0FFEE); 90 % of them get a valid
    point signed over another message (the signature of a set in a later call, bls.test.ts:73 pattern),
    10 % the malformed bytes([10]*96) (bls.test.ts:79).  Returns (sigs, expected valid count)."""
    rng = np.random.Generator(np.random.PCG64(0xC0FFEE))
    bad = np.sort(rng.choice(n_sets, size=int(round(frac * n_sets)), replace=False))
    buf = bytearray(sigs)
    shift = int(call_off[-1] - call_off[-2]) + 256  # lands in another call, so another message
    for k, i in enumerate(bad.tolist()):
        if k % 10 == 9:
            buf[96 * i:96 * i + 96] = bytes([10]) * 96
        else:
            j = (i + shift) % n_sets
            buf[96 * i:96 * i + 96] = sigs[96 * j:96 * j + 96]
    return bytes(buf), n_sets - len(bad)


def p50_batch_latency(v, call_off, idx, sigs, msgs, reps=20):
    """Latency of one gossip batch (one verifySignatureSetsSameMessage call of 64 sets) alone."""
    n = 64
    lat = []
    for r in range(reps):
        t = time.perf_counter()
        v.verify_same_message_multi_sync([([(int(idx[i]), sigs[96 * i:96 * i + 96]) for i in range(n)], msgs[:32])])
        lat.append((time.perf_counter() - t) * 1e3)
    return float(np.median(lat))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--sets", type=int, default=1 << 20)
    ap.add_argument("--cpu-sample", type=int, default=None, help="sets in the CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--invalid-frac", type=float, default=0.0,
                    help="C5: fraction of invalid sets (90%% wrong-message signatures, 10%% malformed bytes)")
    ap.add_argument("--no-signing-roots", action="store_true", help="skip the signing-root secondary line")
    ap.add_argument("--no-stream", dest="stream", action="store_false",
                    help="one batch at a time (no overlap of consecutive verifications)")
    ap.add_argument("--inflight", type=int, default=3, help="staged batches queued on the device at once")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo")

    def log(msg):
        if rank == 0:
            print("[bench] " + msg, file=sys.stderr, flush=True)

    from lodestar_amd import GpuBlsVerifier
    from lodestar_amd.build import build
    build()
    v = GpuBlsVerifier(local_rank)
    call_off, idx, sigs, msgs, key_pks = build_workload(v, args.sets, rank, log)
    expect_valid = args.sets
    if args.invalid_frac > 0:
        sigs, expect_valid = inject_invalid(sigs, call_off, args.sets, args.invalid_frac)
        log("injected %d invalid sets (C5 recipe)" % (args.sets - expect_valid))
    staged = v.stage_same_message(call_off, idx, sigs, msgs)
    # streaming submission: staged copies of the workload so that one batch's chunk-level tail
    # overlaps the next batch's per-set kernel (each verification still runs start to finish)
    depth = max(1, args.inflight) if args.stream else 1
    stages = [staged] + [v.stage_same_message(call_off, idx, sigs, msgs) for _ in range(depth - 1)]

    for _ in range(args.warmup):
        for st in stages:  # every staged copy once: first-use costs stay out of the timed region
            res = st.verify(True)
    if args.warmup:
        ok = res.count(1)
        assert ok == expect_valid, "warmup: %d of %d sets verified" % (ok, expect_valid)
        log("warmup ok: %d of %d sets valid" % (ok, args.sets))

    kms = np.zeros(len(KERNELS))
    kcnt = np.zeros(len(KERNELS))

    def barrier():
        if dist is not None:
            dist.barrier()

    slow_path = [0, 0]

    def collect(b):
        r = b.wait(True)
        log("  step done at %.1f ms" % ((time.perf_counter() - t0) * 1e3))
        fb, seg = v.last_stats()
        slow_path[0] += fb
        slow_path[1] += seg
        ms, cnt = v.last_kernel_ms()
        kms[:] += np.array(ms)
        kcnt[:] += np.array(cnt)
        return r.count(1)

    n_valid = []
    barrier()
    t0 = time.perf_counter()
    # batch k is submitted once batch k - depth (the same staged copy) has been collected, so up to
    # `depth` verifications are queued on the device at any time
    for k in range(args.steps):
        b = stages[k % depth]
        if k >= depth:
            n_valid.append(collect(b))
        b.submit()
    for k in range(max(0, args.steps - depth), args.steps):
        n_valid.append(collect(stages[k % depth]))
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    assert n_valid == [expect_valid] * args.steps, n_valid
    if slow_path != [0, 0] and not args.invalid_frac:
        log("WARNING: fast path fell back (chunks, segments) = %s on an all-valid workload" % slow_path)
    avg_launch_ms = kms / np.maximum(kcnt, 1)
    kms /= max(args.steps, 1)
    prep_launches_per_step = kcnt[1] / max(args.steps, 1)
    total_sets = args.sets * world * args.steps
    value = total_sets / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    lat = p50_batch_latency(v, call_off, idx, sigs, msgs)

    n_chunks = len(call_off) - 1  # calls of 32-128 sets are single chunks
    # per launch: algorithmic MACs of the sets one k_sm_prepare launch processes / its average duration
    units_per_launch = args.sets / max(prep_launches_per_step, 1)
    t_launch = avg_launch_ms[1] * 1e-3
    w_fme = W_PREPARE_FME_MSM if kcnt[7] > 0 else W_PREPARE_FME
    achieved = units_per_launch * w_fme * MAC_PER_FME / t_launch / 1e12 if t_launch > 0 else 0.0
    peak = PEAK_MAC_PER_S / 1e12
    traffic, pmc = pmc_evidence(units_per_launch, "k_sm_prepare<false>" if kcnt[7] > 0 else "k_sm_prepare<true>")
    roofline = {"bound": "valu-int", "kernel": "k_sm_prepare", "achieved": round(achieved, 4), "peak": peak,
                "unit": "T u32-MAC/s", "frac": round(achieved / peak, 5),
                "traffic": round(traffic) if traffic is not None else None, "pmc": pmc,
                "work_per_unit_fme": w_fme, "units_per_launch": round(units_per_launch, 1),
                "avg_launch_ms": round(float(avg_launch_ms[1]), 3),
                "kernel_ms_per_step": {k: round(float(x), 3) for k, x in zip(KERNELS, kms)},
                "slow_path_chunks_segments": slow_path}

    ssz = None
    if rank == 0 and not args.no_signing_roots:
        ssz = signing_roots_bench(v, cpu_sample=0 if args.no_cpu_baseline else 20000)
        log("signing roots: %s" % ssz)

    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        from oracle import cpu_baseline
        cpu = cpu_baseline.measure_same_message(call_off, idx, sigs, msgs, key_pks, N_KEYS,
                                                target_sets=args.cpu_sample or 32768)
        log("cpu baseline: %s" % cpu)

    line = {
        "metric": "signature sets verified/sec (batch verify, same-message gossip stream)",
        "value": round(value, 1),
        "unit": "sets/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "p50_batch_latency_ms": round(lat, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32 (381-bit Montgomery, integer VALU)",
        "data": "synthetic (interop keys, sha256 messages, GPU-signed)",
        "config": {"workload": "C2 gossip attestation stream: 1M single-pubkey sets, same-message calls of 32-128",
                   "sets_per_gpu": args.sets, "calls_per_gpu": n_chunks, "table": N_VALIDATORS,
                   "parallelism": "replicas/dp%d" % world,
                   "submission": "streamed: %d batches in flight" % depth if depth > 1 else "one batch at a time",
                   "invalid_frac": args.invalid_frac},
        "roofline": roofline,
        "cpu_baseline": cpu,
        "signing_roots": ssz,
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    staged.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
