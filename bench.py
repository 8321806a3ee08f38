#!/usr/bin/env python3
"""Headline benchmark: signature sets verified per second on MI355X (BASELINE.json `metric`).

Headline workload (BASELINE.json configs[1]): the gossip attestation stream --
1,048,576 single-pubkey signature sets in verifySignatureSetsSameMessage calls of 32-128 sets
(uniform sizes, numpy PCG64(seed=2)), validators drawn without replacement from a 1,048,576-entry
HBM-resident index2pubkey table whose keys are interop keys sk_i = interopSecretKey(i mod 1024)
(state-transition/src/util/interop.ts:18-22), messages m_g = sha256("gbv-bench" || u64le(g)),
signatures sk*H(m) produced on the GPU before timing.  A "step" = one verification pass over the
whole staged workload (inputs resident in HBM, per-set booleans copied back to the host).

Secondary lines in the same JSON object (single GPU, rank 0): the verifySignatureSets configs
  c1  one verifySignatureSets call of 128 distinct-message single-pubkey sets (the perf id
      "BLS verifyMultipleSignatures 128 - blst", test/perf/bls/bls.test.ts:70-85): lone-call latency,
      plus the throughput of 512 such calls per device pass;
  c3  65,536 128-member committee aggregates gathered from the 2^20-entry HBM table, 512 calls of 128;
  c4  range sync: 64 full blocks (128 attestations x 128 members + 512-member sync aggregate + randao
      + proposer = 131 sets each), one verifySignatureSets call per block (verifyBlocksSignatures.ts:32-51);
each with `roofline` (dominant kernel k_vs_hash_sig, integer VALU) and `cpu_baseline` (the C port in
oracle/, pool shape, bounded sample).

Multi-GPU: `--gpus N` (N > 1) without a torch.distributed environment starts
`python -m torch.distributed.run --nproc-per-node N bench.py ...` as a child BEFORE anything touches a
GPU and exits with its code.  Each rank drives one GPU (LOCAL_RANK), ranks join an RCCL ("nccl")
process group; barrier + max-over-ranks time around the timed steps.
  --mode gossip (default): every rank verifies its own 1M-set stream (replicas, weak scaling; no
      collective on the data path).
  --mode replay (C5): ONE stream of --sets sets (default 1M) with --invalid-frac invalid sets (default
      1 %) sharded by call across the ranks; each step every rank verifies its share and the per-set
      booleans are all-gathered over RCCL (strong scaling).
"""
import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
N_VALIDATORS = 1 << 20
N_KEYS = 1024
MAC_PER_FME = 300  # u32 x u32 -> u64 MACs per Fp product (12-limb Montgomery: 144 + 144 + 12)
# Algorithmic work per unit in Fp-multiplication equivalents (FME), COUNTED on the device code path by
# the host build of the same arithmetic (tests/native/hosttest.cpp ht_count_*; pinned by
# tests/test_host_arith.py::test_roofline_work_constants_are_counted):
FME_SIG_VALIDATE = 2108     # Signature.fromBytes(sig, true): G2 decompress + subgroup check
FME_RANDOMIZE_G1 = 593      # r_i pk_i (endomorphism-split 32-step ladder + affine tables)
FME_COMB_G1 = 126           # r_i pk_i from the validator's comb table (7 doublings + 7 mixed additions)
FME_RANDOMIZE_PAIR = 2086   # r_i pk_i and r_i sig_i with one shared inversion
FME_RANDOMIZE_PAIR_JAC = 2096  # the same with P Jacobian (aggregate pubkeys straight from k_vs_agg)
FME_HASH_TO_G2 = 4802       # RFC 9380 hash_to_G2 (SSWU with one norm exponentiation per map + 3-isogeny + h_eff + to affine)
FME_MILLER_1J = 6803        # Miller value of one pair, Jacobian P
# k_vs_miller_group: k pairs on one accumulator (one f^2 per bit): the first pair 6815 (P with Z != 1,
# as r_i pk_i is on the device), each further pair 4571 (its lines without another squaring)
FME_MILLER_GROUP_FIRST = 6815
FME_MILLER_GROUP_MORE = 4571


def fme_miller_group(k):
    return FME_MILLER_GROUP_FIRST + (k - 1) * FME_MILLER_GROUP_MORE

FME_G1_SCAN = 48            # 3-level 8-lane chunk scan of r_i pk_i (3 Jacobian G1 additions)
FME_G2_DECODE = 938         # G2 decompression alone (k_sig_decode, k_vs_sig_decode)
FME_G2_SUBGROUP = FME_SIG_VALIDATE - FME_G2_DECODE  # the psi-based G2 subgroup check (1170)
FME_RANDOMIZE_G2 = 1491     # r_i sig_i alone (randomize_g2: endomorphism-split ladder + affine tables)
FME_HASH_MAPS = 2091        # hash_to_G2's two SSWU maps + isogenies + Q0 + Q1 (k_hash_msgs_pre)
FME_HASH_CLEAR = 2711       # hash_to_G2's cofactor clearing + affine form (k_hash_clear_quad / _coop)
# k_sm_prepare<false> (bench: G2 sum by bucket MSM) and <true> (per-set G2 ladders)
W_PREPARE_FME_MSM = FME_SIG_VALIDATE + FME_RANDOMIZE_G1 + FME_G1_SCAN
W_PREPARE_FME_MSM_COMB = FME_SIG_VALIDATE + FME_COMB_G1 + FME_G1_SCAN
W_PREPARE_FME = FME_SIG_VALIDATE + FME_RANDOMIZE_PAIR + 177
# k_vs_hash_sig: both block roles per set
W_VS_HASH_SIG = FME_HASH_TO_G2 + FME_SIG_VALIDATE + FME_RANDOMIZE_PAIR_JAC
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
# with comb tables the 128-byte table record is replaced by 8 comb entries (96 B) + the 1-byte flag
ALG_BYTES_PER_SET_COMB = ALG_BYTES_PER_SET - 128 + 8 * 96 + 1
# k_vs_agg gather: per member a 4-byte index + the 128-byte affine table record + its 1-byte flag
AGG_BYTES_PER_MEMBER = 4 + 128 + 1
# host-counted (tests/native/hosttest.cpp ht_count_op): mixed G1 addition, Fp12 product, Jacobian G2
# addition, final exponentiation
FME_G1_MADD = 11
FME_FP12_MUL = 54
FME_G2_ADD = 59
FME_FINAL_EXP = 7709
# verifySignatureSets kernels: algorithmic bytes per set (Fp in 64-byte slots: G1J 192, G2A 256,
# G2J 384, Fp12 768).  hash_sig reads msg 32 + sig 96 + set_off 8 + index 4 + table record 128 + flag 1
# and writes H 256 + rP 192 + rS 384 + status 1; miller reads rP 192 + H 256 + status 1, writes F 768.
VS_ALG_BYTES = {"hash_sig": 32 + 96 + 8 + 4 + 128 + 1 + 256 + 192 + 384 + 1, "miller": 192 + 256 + 1 + 768}


def _pmc_summary():
    try:
        return json.load(open(PMC_SUMMARY))
    except (OSError, ValueError):
        return None


def pmc_at(kernel, grid):
    """Counters of `kernel` at launches of exactly `grid` work-items from the committed PMC summary
    (tools/pmc.sh -> tools/pmc_parse.py: per kernel, per grid size), or None -- counters are only
    attached to a roofline whose launch has the same grid as the profiled one."""
    summary = _pmc_summary()
    if not summary:
        return None
    d = (summary.get("kernels") or {}).get(kernel, {}).get(str(int(grid)))
    return d if d and "FETCH_SIZE" in d and "WRITE_SIZE" in d else None


def pmc_evidence(kernels, units, alg_bytes_per_unit):
    """HBM traffic and VALU issue of one launch of each of `kernels` [(name, grid work-items)] that
    together process `units` (sets, messages, chunks), from separate rocprofv3 --pmc passes (FETCH_SIZE
    doubled per the gfx950 calibration of the MI355X guide: it counts 64 B per 128-B request;
    rocprofv3 reports kilobytes).  Returns (bytes per launch, evidence) or (None, reason)."""
    ds = [(k, g, pmc_at(k, g)) for k, g in kernels]
    missing = ["%s@%d" % (k, g) for k, g, d in ds if d is None]
    if missing:
        return None, {"source": os.path.relpath(PMC_SUMMARY, ROOT), "missing_at_grid": missing}
    total = sum((2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024.0 for _, _, d in ds)
    have_sq = all("SQ_INSTS_VALU" in d and "SQ_WAVES" in d for _, _, d in ds)
    dur = sum(d["duration_ms"] for _, _, d in ds)
    summary = _pmc_summary() or {}
    ev = {"source": os.path.relpath(PMC_SUMMARY, ROOT), "collected": summary.get("collected"),
          "kernel": " + ".join(k for k, _, _ in ds), "pmc_grid": [int(g) for _, g, _ in ds], "pmc_grid_units": int(units),
          "hbm_bytes_per_unit": round(total / max(units, 1), 1), "algorithmic_bytes_per_unit": alg_bytes_per_unit,
          "write_bytes_per_unit": round(sum(d["WRITE_SIZE"] for _, _, d in ds) * 1024.0 / max(units, 1), 1),
          "valu_wave_instr_per_unit": round(sum(d["SQ_INSTS_VALU"] for _, _, d in ds) / max(units, 1), 1) if have_sq else None,
          "valu_issue_utilisation": round(sum(d["SQ_INSTS_VALU"] for _, _, d in ds) / (dur * 1e-3 * PEAK_VALU_WAVE_INSTR_PER_S), 4) if have_sq else None,
          "ms_at_pmc": {k: round(d["duration_ms"], 3) for k, _, d in ds}}
    if len(ds) == 1 and "SQ_ACTIVE_INST_VALU" in ds[0][2] and "SQ_THREAD_CYCLES_VALU" in ds[0][2]:
        d = ds[0][2]
        ev["valu_lane_utilisation"] = round(d["SQ_THREAD_CYCLES_VALU"] / (64.0 * d["SQ_ACTIVE_INST_VALU"]), 4)
    return total, ev


# device kernels of one same-message verify, in gbv_last_kernel_ms order
KERNELS = ["hash", "prepare", "chunk_finish", "miller", "seg_check", "group_pairing", "fallback", "msm"]
VS_KERNELS = ["agg", "hash_sig", "miller", "chunk_check"]


def interop_sk_int(i):
    d = hashlib.sha256(i.to_bytes(32, "little")).digest()
    return int.from_bytes(d, "little") % R_ORDER


def interop_sk_bytes(i):
    return interop_sk_int(i).to_bytes(32, "big")


def build_table(v, log):
    sks = [interop_sk_bytes(i) for i in range(N_KEYS)]
    pks = v.util_sk_to_pk(sks)
    st = v.add_pubkeys(0, pks)
    assert st == bytes(N_KEYS), "pubkey ingest failed"
    v.replicate_pubkeys(0, N_KEYS, N_KEYS, N_VALIDATORS - N_KEYS)
    return sks, pks


def build_workload(v, sks, n_sets, seed_rank, log, first_call=0):
    """C2 stream: call sizes 32..128 (PCG64(2)), validators without replacement, GPU-signed."""
    t0 = time.time()
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
    perm = np.random.Generator(np.random.PCG64(0x1D5 + seed_rank)).permutation(N_VALIDATORS)
    idx = perm[np.arange(n_sets) % N_VALIDATORS].astype(np.uint32)
    grp = np.repeat(np.arange(len(sizes), dtype=np.uint32), sizes)
    msgs = [hashlib.sha256(b"gbv-bench" + (g + first_call + seed_rank * 10_000_000).to_bytes(8, "little")).digest()
            for g in range(len(sizes))]
    sk_arr = np.frombuffer(b"".join(sks), dtype=np.uint8).reshape(N_KEYS, 32)
    set_sks = sk_arr[idx % N_KEYS]
    t1 = time.time()
    sigs = []
    CH = 1 << 18
    for a in range(0, n_sets, CH):
        b = min(n_sets, a + CH)
        sigs.extend(v.util_sign([bytes(r) for r in set_sks[a:b]], grp[a:b].tolist(), msgs))
    log("workload: %d sets in %d calls, signed on the GPU in %.1fs (%.1fs total)" % (n_sets, len(sizes), time.time() - t1, time.time() - t0))
    return call_off, idx, b"".join(sigs), b"".join(msgs)


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
    10 % the malformed bytes([10]*96) (bls.test.ts:79).  Returns (sigs, expected per-set validity)."""
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
    valid = np.ones(n_sets, dtype=np.uint8)
    valid[bad] = 0
    return bytes(buf), valid


def p50_batch_latency(v, idx, sigs, msgs, reps=20):
    """Latency of one gossip batch (one verifySignatureSetsSameMessage call of 64 sets) alone, through
    the API path (host buffers in, booleans out: marshalling, upload and download included)."""
    n = 64
    lat = []
    calls = [([(int(idx[i]), sigs[96 * i:96 * i + 96]) for i in range(n)], msgs[:32])]
    for r in range(reps):
        t = time.perf_counter()
        v.verify_same_message_multi_sync(calls)
        lat.append((time.perf_counter() - t) * 1e3)
    return float(np.median(lat))


def api_path_rate(v, call_off, idx, sigs, msgs, n_sets=1 << 18):
    """PCIe- and marshalling-inclusive sets/s of the one-shot API (gbv_verify_same_message_multi from
    host buffers), on the first n_sets sets of the workload."""
    k = int(np.searchsorted(call_off, n_sets))
    n = int(call_off[k])
    v.verify_same_message_raw(call_off[:k + 1], idx[:n], sigs[:96 * n], msgs[:32 * k])  # warm the scratch batch
    t = time.perf_counter()
    res = v.verify_same_message_raw(call_off[:k + 1], idx[:n], sigs[:96 * n], msgs[:32 * k])
    dt = time.perf_counter() - t
    assert res.count(1) == n
    return round(n / dt, 1), n


def api_path_js(call_off, idx, sigs, msgs, key_pks, log, reps=3):
    """The C2 stream through the JavaScript GpuBlsVerifier over the Node-API addon (addon/bench_api.js, a
    Node child process with its own device context): every gossip call issued as
    verifySignatureSetsSameMessage, packed and object-form inputs, every boolean checked.  None when Node
    or the addon is missing."""
    import shutil
    import tempfile
    node = shutil.which("node") or shutil.which("nodejs")
    addon = os.path.join(ROOT, "addon", "gbv_addon.node")
    if node is None or not os.path.exists(addon):
        return None
    keep = os.environ.get("GBV_JS_INPUTS")  # diagnosis: keep the child's inputs in this directory
    d = keep or tempfile.mkdtemp(prefix="gbv-api-js-")
    os.makedirs(d, exist_ok=True)
    try:
        n_calls = len(call_off) - 1
        with open(os.path.join(d, "meta.json"), "w") as f:
            json.dump({"n_sets": int(call_off[-1]), "n_calls": n_calls, "n_keys": len(key_pks), "table": N_VALIDATORS}, f)
        np.asarray(call_off, dtype=np.uint32).tofile(os.path.join(d, "call_off.u32"))
        np.asarray(idx, dtype=np.uint32).tofile(os.path.join(d, "idx.u32"))
        for name, blob in (("sigs.bin", sigs), ("msgs.bin", msgs), ("keys.bin", b"".join(key_pks))):
            with open(os.path.join(d, name), "wb") as f:
                f.write(blob)
        p = subprocess.run([node, os.path.join(ROOT, "addon", "bench_api.js"), d, str(reps)], capture_output=True, text=True, timeout=400)
        lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
        r = json.loads(lines[-1]) if lines else {}
        if p.returncode != 0:
            log("api path (js): child exit %d %s %s" % (p.returncode, p.stdout[-500:], p.stderr[-1500:]))
        # a child that printed its checked results and then died at process teardown (after close():
        # no device work left) still measured them; its exit status goes into the record
        if not (r.get("all_valid") and (p.returncode == 0 or (p.returncode < 0 and r.get("closed")))):
            return None
        if p.returncode != 0:
            r["child_exit"] = p.returncode
        r["how"] = ("node addon/bench_api.js: every gossip call of the C2 workload through GpuBlsVerifier.verifySignatureSetsSameMessage "
                    "(addon/gpu_bls_verifier.js) over the Node-API addon, all promises awaited, every boolean checked; "
                    "'packed' = {indices: Uint32Array, signatures: Uint8Array} per call, 'objects' = one {index, signature} per set "
                    "(built before the clock); 'ibls' = the IBlsVerifier shape the Lodestar binding uses (chain/bls/gpu/index.ts): one "
                    "{publicKey, signature} object per set (the key found by the identity of its index2pubkey object), packed per call into the device form INSIDE the clock, boolean[] out "
                    "(verifySameMessageSets); best of %d; its own device context beside the bench's" % reps)
        return r
    finally:
        if not keep:
            shutil.rmtree(d, ignore_errors=True)


# ---- verifySignatureSets configs (C1, C3, C4) ------------------------------------------------------
# Algorithmic work (FME) and bytes of one launch of each kernel a verifySignatureSets pass can run,
# as a function of the launch's units (gbv_last_ops: sets, messages or chunks) and the pass (n sets,
# gathered members of aggregates below / above AGG_BIG_MIN).  Counted on the device code path by the
# host build (tests/test_host_arith.py pins every constant).
AGG_BIG_MIN = 1024


def vs_op_work(name, units, ps):
    n, C = ps["n_sets"], ps["n_chunks"]
    hash_sig_chunk = n * FME_G2_ADD + C * FME_MILLER_1J  # k_vs_chunk_s_miller: sum r_i sig_i + (-g1, sum) Miller value
    table = {
        "k_vs_agg": (ps["members_small"] * FME_G1_MADD, ps["members_small"] * AGG_BYTES_PER_MEMBER),
        "k_vs_agg_big": (ps["members_big"] * FME_G1_MADD, ps["members_big"] * AGG_BYTES_PER_MEMBER),
        "k_vs_hash_sig": (units * W_VS_HASH_SIG, units * VS_ALG_BYTES["hash_sig"]),
        "k_hash_msgs": (units * FME_HASH_TO_G2, units * (32 + 256)),
        "k_hash_msgs_pair": (units * FME_HASH_TO_G2, units * (32 + 256)),
        "k_hash_msgs_quad": (units * FME_HASH_TO_G2, units * (32 + 256)),
        "k_hash_msgs_pre": (units * FME_HASH_MAPS, units * (32 + 384)),
        "k_hash_clear_quad": (units * FME_HASH_CLEAR, units * (384 + 256)),
        "k_hash_clear_coop": (units * FME_HASH_CLEAR, units * (384 + 256)),
        "k_vs_sig_decode": (units * FME_G2_DECODE, units * (96 + 4 + 256 + 1)),
        "k_vs_sig_pre_quad": (units * (FME_G2_SUBGROUP + FME_RANDOMIZE_G2), units * (256 + 1 + 384 + 2)),
        "k_vs_pk_rand_quad": (units * FME_RANDOMIZE_G1, units * (8 + 4 + 129 + 1 + 192)),
        "k_vs_miller": (units * FME_MILLER_1J, units * VS_ALG_BYTES["miller"]),
        "k_vs_miller_pair": (units * FME_MILLER_1J, units * VS_ALG_BYTES["miller"]),
        "k_vs_miller_quad": (units * FME_MILLER_1J, units * VS_ALG_BYTES["miller"]),
        "k_vs_miller_coop": (units * FME_MILLER_1J, units * VS_ALG_BYTES["miller"]),
        "k_vs_chunk_s_miller": (hash_sig_chunk, n * (384 + 1) + C * 768),
        "k_vs_chunk_coop<false>": (n * (FME_FP12_MUL + FME_G2_ADD) + C * (FME_FINAL_EXP + FME_MILLER_1J), n * (768 + 384 + 1) + C),
        "k_vs_chunk_coop<true>": (n * FME_FP12_MUL + C * (FME_FINAL_EXP + FME_FP12_MUL), n * (768 + 1) + C * 769),
    }
    return table.get(name, (None, None))


def _vs_roofline(v, n_sets, ops, members_small=0, members_big=0, n_chunks=0):
    """Roofline of a verifySignatureSets pass from its per-kernel HIP-event timings (gbv_last_ops:
    every launched kernel, its grid and units, its device ms on its own stream).  The roofline object
    describes the kernel that took longest among those whose algorithmic work is known (summed over
    its launches in the pass); `kernels` lists every launch with its fraction of the VALU peak.  PMC
    counters are attached only from a profiled launch of that kernel at the same grid."""
    ps = {"n_sets": n_sets, "n_chunks": n_chunks or max(1, -(-n_sets // 128)), "members_small": members_small, "members_big": members_big}
    agg = {}
    for name, threads, units, ms in ops:
        e = agg.setdefault(name, {"ms": 0.0, "launches": 0, "grid": threads, "units": units, "grids": []})
        e["ms"] += max(ms, 0.0)
        e["launches"] += 1
        e["grids"].append(threads)
    kernels = []
    for name, e in agg.items():
        w, b = vs_op_work(name, e["units"], ps)
        frac = round(w * MAC_PER_FME / (e["ms"] * 1e-3) / PEAK_MAC_PER_S, 4) if w and e["ms"] > 0 else None
        kernels.append({"kernel": name, "grid": e["grid"], "units": e["units"], "launches": e["launches"], "ms": round(e["ms"], 3),
                        "work_fme": w, "frac": frac})
    timed = [k for k in kernels if k["work_fme"] and k["ms"] > 0]
    if not timed:
        return {"bound": "valu-int", "kernel": None, "kernels": kernels, "note": "no per-kernel timings recorded"}
    dom = max(timed, key=lambda k: k["ms"])
    t = dom["ms"] / dom["launches"]
    achieved = dom["work_fme"] / dom["launches"] * MAC_PER_FME / (t * 1e-3) / 1e12
    w, alg_b = vs_op_work(dom["kernel"], dom["units"], ps)
    traffic, ev = (None, None)
    if dom["launches"] == 1:
        traffic, ev = pmc_evidence([(dom["kernel"], dom["grid"])], dom["units"], round(alg_b / max(dom["units"], 1), 1))
    out = {"bound": "valu-int", "kernel": dom["kernel"], "achieved": round(achieved, 4), "peak": PEAK_MAC_PER_S / 1e12,
           "unit": "T u32-MAC/s", "frac": round(achieved * 1e12 / PEAK_MAC_PER_S, 5),
           "traffic": None if traffic is None else round(traffic), "pmc": ev,
           "work_per_launch_fme": int(w), "algorithmic_bytes_per_launch": alg_b, "units_per_launch": dom["units"], "grid": dom["grid"],
           "avg_launch_ms": round(t, 3), "timing": "HIP events around each launch on its own stream (gbv_last_ops)",
           "kernels": sorted(kernels, key=lambda k: -k["ms"]), "miller_fme_per_set": FME_MILLER_1J}
    if members_small + members_big:
        for name in ("k_vs_agg", "k_vs_agg_big"):
            if name in agg and agg[name]["ms"] > 0:
                m = members_small if name == "k_vs_agg" else members_big
                out.setdefault("agg_gather_GBps_formula", {})[name] = round(m * AGG_BYTES_PER_MEMBER / (agg[name]["ms"] * 1e-3) / 1e9, 1)
    return out


def _members(calls):
    small = big = 0
    for c in calls:
        for s in c:
            k = len(getattr(s, "indices", []))
            if k >= AGG_BIG_MIN:
                big += k
            elif k >= 2:
                small += k
    return small, big


def _timed_ops(v, stages, steps, want):
    """_timed_staged with per-kernel timing on; returns (seconds per step, the last pass's ops)."""
    v.tune("kprof", 1)
    try:
        dt = _timed_staged(stages, steps, want)
    finally:
        v.tune("kprof", 0)
    return dt, v.last_ops(1)


def _timed_staged(stages, steps, want):
    """Verify staged vs batches `steps` times with len(stages) in flight; returns seconds per step."""
    depth = len(stages)
    t0 = time.perf_counter()
    for k in range(steps):
        b = stages[k % depth]
        if k >= depth:
            assert b.wait() == want
        b.submit()
    for k in range(max(0, steps - depth), steps):
        assert stages[k % depth].wait() == want
    return (time.perf_counter() - t0) / steps


def _single_sets(v, sks, n, tag, rng):
    from lodestar_amd import SingleSignatureSet
    idx = rng.choice(N_VALIDATORS, size=n, replace=False)
    msgs = [hashlib.sha256(tag + i.to_bytes(8, "little")).digest() for i in range(n)]
    sigs = v.util_sign([sks[int(k) % N_KEYS] for k in idx], list(range(n)), msgs)
    return [SingleSignatureSet(int(idx[i]), msgs[i], sigs[i]) for i in range(n)]


def _agg_sets(v, sk_ints, n, tag, rng, k=128):
    from lodestar_amd import AggregatedSignatureSet
    coms = [rng.choice(N_VALIDATORS, size=k, replace=False) for _ in range(n)]
    msgs = [hashlib.sha256(tag + i.to_bytes(8, "little")).digest() for i in range(n)]
    agg = [(sum(sk_ints[int(x) % N_KEYS] for x in c) % R_ORDER).to_bytes(32, "big") for c in coms]
    sigs = []
    for a in range(0, n, 1 << 16):
        sigs.extend(v.util_sign(agg[a:a + (1 << 16)], list(range(a, min(n, a + (1 << 16)))), msgs))
    return [AggregatedSignatureSet(coms[i].tolist(), msgs[i], sigs[i]) for i in range(n)]


def _port_calls(calls):
    """verifySignatureSets calls -> the port's (pk rows, msg, sig) form over the 1024-key table."""
    from lodestar_amd import AggregatedSignatureSet
    out = []
    for c in calls:
        out.append([([x % N_KEYS for x in s.indices] if isinstance(s, AggregatedSignatureSet) else [s.index % N_KEYS],
                     s.signing_root, s.signature) for s in c])
    return out


def c1_bench(v, sks, pk_rows, cpu):
    rng = np.random.Generator(np.random.PCG64(0xC1))
    sets = _single_sets(v, sks, 128, b"gbv-c1", rng)
    for _ in range(3):
        assert v.verify_signature_sets_sync(sets) is True
    lat = []
    for _ in range(15):
        t = time.perf_counter()
        ok = v.verify_signature_sets_sync(sets)
        lat.append((time.perf_counter() - t) * 1e3)
        assert ok
    p50 = float(np.median(lat))
    v.tune("kprof", 1)  # one more lone call, timed kernel by kernel (outside the latency samples)
    assert v.verify_signature_sets_sync(sets) is True
    v.tune("kprof", 0)
    ops_lone = v.last_ops(1)
    # throughput: 512 such calls staged, 2 passes in flight
    many = _single_sets(v, sks, 512 * 128, b"gbv-c1-many", rng)
    calls = [many[i:i + 128] for i in range(0, len(many), 128)]
    stages = [v.stage_signature_sets(calls) for _ in range(2)]
    for st in stages:
        assert st.verify() == [1] * len(calls)
    dt, ops = _timed_ops(v, stages, 6, [1] * len(calls))
    for st in stages:
        st.close()
    out = {"metric": "verifySignatureSets: 128 distinct-message single-pubkey sets per call (verifyMultipleSignatures 128)",
           "unit": "sets/s", "value": round(128 / (p50 * 1e-3), 1), "latency_ms_p50": round(p50, 3),
           "lone_call_kernels": [{"kernel": k, "grid": g, "units": u, "ms": round(m, 3)} for k, g, u, m in ops_lone],
           "throughput_value": round(len(many) / dt, 1), "throughput_config": "512 calls x 128 sets per pass, 2 passes in flight",
           "roofline": _vs_roofline(v, len(many), ops)}
    if cpu:
        from oracle import cpu_baseline
        out["cpu_baseline"] = cpu_baseline.measure_verify_sets(_port_calls([sets]), pk_rows, threads=1,
                                                               label=" (one call of 128, single thread: the perf id's shape)")
    return out


def c3_bench(v, sk_ints, pk_rows, cpu, n_calls=512):
    rng = np.random.Generator(np.random.PCG64(0xC3))
    t0 = time.time()
    sets = _agg_sets(v, sk_ints, n_calls * 128, b"gbv-c3", rng)
    calls = [sets[i:i + 128] for i in range(0, len(sets), 128)]
    build_s = time.time() - t0
    stages = [v.stage_signature_sets(calls) for _ in range(2)]
    for st in stages:
        assert st.verify() == [1] * n_calls
    dt, ops = _timed_ops(v, stages, 6, [1] * n_calls)
    for st in stages:
        st.close()
    small, big = _members(calls)
    out = {"metric": "verifySignatureSets: 128-member committee aggregates from the HBM table (1M validators)",
           "unit": "sets/s", "value": round(len(sets) / dt, 1), "ms_per_pass": round(dt * 1e3, 3),
           "config": "%d aggregate sets of 128 members in %d calls of 128, 2 passes in flight (workload built in %.1fs)" % (len(sets), n_calls, build_s),
           "roofline": _vs_roofline(v, len(sets), ops, members_small=small, members_big=big)}
    if cpu:
        from oracle import cpu_baseline
        out["cpu_baseline"] = cpu_baseline.measure_verify_sets(_port_calls(calls[:32]), pk_rows, label=" (the first 32 calls)")
    return out


ELECTRA_COMMITTEE = 512  # ~1M validators / 32 slots / 64 committees (mainnet)


def make_blocks(v, sk_ints, n_blocks, rng, electra=False):
    """A range-sync segment of synthetic blocks through the product builders
    (lodestar_amd/signature_sets.py), every signature made on the GPU.  deneb: 128 attestations of
    128-member committees; electra: 8 attestations (MAX_ATTESTATIONS_ELECTRA) each over the 64
    committees of its slot (committee_bits), 512 members each -- aggregates of 32 768 validators;
    both with a 512-member sync aggregate, randao and proposer."""
    from lodestar_amd import AggregatedSignatureSet, SingleSignatureSet
    from lodestar_amd import signature_sets as B
    forks = [B.Fork("phase0", 0, bytes(4)), B.Fork("altair", 10, bytes([1, 0, 0, 0])),
             B.Fork("bellatrix", 20, bytes([2, 0, 0, 0])), B.Fork("capella", 30, bytes([3, 0, 0, 0])),
             B.Fork("deneb", 40, bytes([4, 0, 0, 0]))]
    if electra:
        forks.append(B.Fork("electra", 45, bytes([5, 0, 0, 0])))
    config = B.BeaconConfig(forks, hashlib.sha256(b"gbv-c4").digest())
    slot0 = 50 * 32
    committees = {}
    perm = rng.permutation(N_VALIDATORS) if electra else None  # a slot's committees are disjoint

    def committee(s, i):
        key = (s, i)
        if key not in committees:
            if electra:
                o = (s * 64 * ELECTRA_COMMITTEE + i * ELECTRA_COMMITTEE) % N_VALIDATORS
                committees[key] = perm[o:o + ELECTRA_COMMITTEE].tolist()
            else:
                committees[key] = rng.choice(N_VALIDATORS, size=128, replace=False).tolist()
        return committees[key]
    sync = rng.choice(N_VALIDATORS, size=512, replace=False).tolist()
    rb = lambda: rng.integers(0, 256, size=32, dtype=np.uint8).tobytes()
    blocks = []
    for b in range(n_blocks):
        slot = slot0 + 1 + b
        atts = []
        for j in range(8 if electra else 128):
            a_slot, a_idx = slot - 1 - (j % 8), (0 if electra else j // 8)
            ep = a_slot // 32
            data = B.AttestationData(a_slot, a_idx, rb(), B.Checkpoint(ep - 1, rb()), B.Checkpoint(ep, rb()))
            if electra:
                atts.append(B.Attestation([True] * (64 * ELECTRA_COMMITTEE), data, bytes(96), [True] * 64))
            else:
                committee(a_slot, a_idx)
                atts.append(B.Attestation([True] * 128, data, bytes(96)))
        body = B.BeaconBlockBody(randao_reveal=bytes(96), body_root=rb(), attestations=atts,
                                 sync_aggregate=B.SyncAggregate([True] * 512, bytes(96)))
        blocks.append(B.SignedBeaconBlock(B.BeaconBlock(slot, int(rng.integers(0, N_VALIDATORS)), rb(), rb(), body), bytes(96)))
    state = B.EpochState(config, slot0 + 1, committee, sync)
    unsigned = B.get_blocks_signature_sets(state, blocks, v)
    flat = [s for c in unsigned for s in c]
    sks = []
    for s in flat:
        members = np.asarray(s.indices if isinstance(s, AggregatedSignatureSet) else [s.index], dtype=np.int64)
        cnt = np.bincount(members % N_KEYS, minlength=N_KEYS)  # sum of the members' keys, by key multiplicity
        sks.append((sum(int(c) * sk_ints[k] for k, c in enumerate(cnt) if c) % R_ORDER).to_bytes(32, "big"))
    sigs = v.util_sign(sks, list(range(len(flat))), [s.signing_root for s in flat])
    calls, k = [], 0
    for c in unsigned:
        out = []
        for s in c:
            if isinstance(s, AggregatedSignatureSet):
                out.append(AggregatedSignatureSet(s.indices, s.signing_root, sigs[k]))
            else:
                out.append(SingleSignatureSet(s.index, s.signing_root, sigs[k]))
            k += 1
        calls.append(out)
    return calls


def _pmc_gather(ops, kernel, members):
    """HBM read rate of the pubkey gather kernel from the committed PMC summary at the grid this pass
    launched it with (FETCH_SIZE doubled per the gfx950 calibration, over that launch's own duration):
    measured, not by formula, and the bytes fetched per gathered member."""
    grids = [g for k, g, _, _ in ops if k == kernel]
    d = pmc_at(kernel, grids[0]) if grids else None
    if not d:
        return None
    fetched = 2 * d["FETCH_SIZE"] * 1024.0
    return {"source": os.path.relpath(PMC_SUMMARY, ROOT), "kernel": kernel, "pmc_grid": grids[0],
            "hbm_read_GBps": round(fetched / (d["duration_ms"] * 1e-3) / 1e9, 1),
            "fetched_bytes_per_member": round(fetched / max(members, 1), 1), "algorithmic_bytes_per_member": AGG_BYTES_PER_MEMBER,
            "launch_ms_at_pmc": round(d["duration_ms"], 3), "hbm_peak_GBps": 8000.0}


def c4_bench(v, sk_ints, pk_rows, cpu, n_blocks=64, electra=False, depth=2):
    rng = np.random.Generator(np.random.PCG64(0xC4E if electra else 0xC4))
    t0 = time.time()
    calls = make_blocks(v, sk_ints, n_blocks, rng, electra=electra)
    build_s = time.time() - t0
    n_sets = sum(len(c) for c in calls)
    members = sum(len(getattr(s, "indices", [])) for c in calls for s in c)
    # lone block (one verifySignatureSets call, the gossip-block / unknown-block path)
    for _ in range(2):
        assert v.verify_signature_sets_sync(calls[0]) is True
    lat = []
    for _ in range(10):
        t = time.perf_counter()
        assert v.verify_signature_sets_sync(calls[0]) is True
        lat.append((time.perf_counter() - t) * 1e3)
    stages = [v.stage_signature_sets(calls) for _ in range(depth)]
    for st in stages:
        assert st.verify() == [1] * n_blocks
    dt, ops = _timed_ops(v, stages, 6, [1] * n_blocks)
    for st in stages:
        st.close()
    small, big = _members(calls)
    n_chunks = sum(max(1, len(c) // 128) for c in calls)  # chunkifyMaximizeChunkSize(call, 128)
    out = {"metric": "verifySignatureSets: full %sblocks (getBlockSignatureSets, index form), one call per block" % (
               "electra " if electra else ""),
           "unit": "sets/s", "value": round(n_sets / dt, 1), "blocks_per_s": round(n_blocks / dt, 2),
           "lone_block_latency_ms_p50": round(float(np.median(lat)), 3), "sets_per_block": len(calls[0]),
           "config": "range-sync segment of %d blocks (%d sets, %d pubkeys gathered), %d passes in flight (built in %.1fs)" % (
               n_blocks, n_sets, members, depth, build_s),
           "roofline": _vs_roofline(v, n_sets, ops, members_small=small, members_big=big, n_chunks=n_chunks)}
    g = _pmc_gather(ops, "k_vs_agg_big" if electra else "k_vs_agg", big if electra else small)
    if g:
        out["roofline"]["agg_gather_pmc"] = g
    if cpu:
        from oracle import cpu_baseline
        k = 1 if electra else 4
        out["cpu_baseline"] = cpu_baseline.measure_verify_sets(_port_calls(calls[:k]), pk_rows, label=" (the first %d blocks)" % k)
    return out


def c5_bench(v, call_off, idx, sigs, msgs, steps=6, depth=3, frac=0.01):
    """C5 at N = 1: the headline stream with 1 % invalid sets (SURVEY 8(d) recipe: 90 % wrong-message
    signatures, 10 % malformed bytes([10]*96)), every per-set boolean checked against the injection
    map -- the per-set fallback path (jobItem.ts:93-125) under load.  Multi-GPU: --mode replay."""
    n = int(call_off[-1])
    bad_sigs, expect = inject_invalid(sigs, call_off, n, frac)
    want = expect.tobytes()
    stages = [v.stage_same_message(call_off, idx, bad_sigs, msgs) for _ in range(depth)]
    for st in stages:
        assert st.verify(True) == want
    t0 = time.perf_counter()
    for k in range(steps):
        b = stages[k % depth]
        if k >= depth:
            assert b.wait(True) == want
        if k == steps - 1:
            v.tune("kprof", 1)  # the last batch also timed kernel by kernel
        b.submit()
    v.tune("kprof", 0)
    for k in range(max(0, steps - depth), steps):
        assert stages[k % depth].wait(True) == want
    dt = (time.perf_counter() - t0) / steps
    fb, seg = v.last_stats()
    ops = v.last_ops(0)
    for st in stages:
        st.close()
    return {"metric": "signature sets verified/sec (same-message stream, 1% invalid: per-set fallback), 1 GPU",
            "unit": "sets/s", "value": round(n / dt, 1), "ms_per_step": round(dt * 1e3, 3), "steps": steps,
            "config": "C5 recipe on the C2 stream: %d sets, %d invalid (90%% wrong message, 10%% malformed), %d batches in flight" % (
                n, int((expect == 0).sum()), depth),
            "all_booleans_checked": True, "last_fallback_chunks": fb, "last_failed_segments": seg,
            "last_step_kernels": [{"kernel": k, "grid": g, "units": u, "ms": round(m, 3)} for k, g, u, m in ops]}


def api_stream_rate(v, call_off, idx, sigs, msgs, n_sets=1 << 20):
    """The IBlsVerifier path itself: every gossip call of the workload (n_sets sets, 13k calls of
    32-128) issued as an async verifySignatureSetsSameMessage (packed inputs) through the verifier's
    job queue, which cuts it into passes of <= MAX_PASS_SETS sets with up to MAX_PASSES_IN_FLIGHT on
    the device at once; every boolean checked.  Host buffers in, booleans out: the Python calls,
    futures, marshalling, PCIe and result splitting are inside the timed region.  The request
    objects (the caller's deserialized gossip data) are built before it."""
    import asyncio
    from lodestar_amd import PackedSameMessageSets
    k = min(int(np.searchsorted(call_off, n_sets)), len(call_off) - 1)
    n = int(call_off[k])
    sig_mv = memoryview(sigs)
    reqs = [(PackedSameMessageSets(idx[call_off[g]:call_off[g + 1]], sig_mv[96 * int(call_off[g]):96 * int(call_off[g + 1])]),
             msgs[32 * g:32 * g + 32]) for g in range(k)]
    call = v.submit_signature_sets_same_message  # the IBlsVerifier method minus its coroutine frame

    async def go():
        res = await asyncio.gather(*[call(s, m) for s, m in reqs])
        return int(np.count_nonzero(np.concatenate(res)))

    asyncio.run(go())  # warm the pass slots
    p0 = v.device_passes
    t = time.perf_counter()
    ok = asyncio.run(go())
    dt = time.perf_counter() - t
    assert ok == n
    return round(n / dt, 1), n, v.device_passes - p0


_JSON_OUT = None


def claim_stdout():
    """The bench line must be alone on stdout, but native libraries print there too (RCCL's version
    banner at process-group init): fd 1 is pointed at stderr for the rest of the process and the
    line goes out through a private copy of the original stdout."""
    global _JSON_OUT
    sys.stdout.flush()
    _JSON_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)


def emit_json(line):
    print(json.dumps(line), file=_JSON_OUT or sys.stdout, flush=True)


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--sets", type=int, default=1 << 20)
    ap.add_argument("--mode", choices=["gossip", "replay", "vs-shard"], default="gossip")
    ap.add_argument("--cpu-sample", type=int, default=None, help="sets in the C2 CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--invalid-frac", type=float, default=None,
                    help="fraction of invalid sets (90%% wrong-message signatures, 10%% malformed bytes); "
                         "default 0 for gossip, 0.01 for replay (C5)")
    ap.add_argument("--no-signing-roots", action="store_true", help="skip the signing-root secondary line")
    ap.add_argument("--no-extras", action="store_true", help="skip the c1/c3/c4 secondary lines")
    ap.add_argument("--no-api", action="store_true",
                    help="skip the API-path rates (their 2^18-set passes would mix launch sizes into a rocprof summary)")
    ap.add_argument("--no-stream", dest="stream", action="store_false",
                    help="one batch at a time (no overlap of consecutive verifications)")
    ap.add_argument("--inflight", type=int, default=3, help="staged batches queued on the device at once")
    ap.add_argument("--c3-calls", type=int, default=512, help="128-set calls per C3 device pass")
    ap.add_argument("--c4-blocks", type=int, default=64, help="blocks per C4 device pass (range-sync segment)")
    ap.add_argument("--c4-depth", type=int, default=3, help="C4 passes in flight (the verifier queue allows 3)")
    ap.add_argument("--c4e-blocks", type=int, default=16, help="electra blocks per C4e device pass")
    ap.add_argument("--tune", action="append", default=[], metavar="NAME=VALUE",
                    help="gbv_tune setting applied before anything runs (experiments; include/gbv.h lists the names)")
    ap.add_argument("--no-vs-shard", action="store_true", help="skip the sharded verifySignatureSets object of the gossip line")
    ap.add_argument("--shard-depth", type=int, default=3, help="vs-shard: shard passes in flight per rank (staged copies; 3 measured best for 8 192 - 16 384-set shards, profiles/r06/shards)")
    ap.add_argument("--shard-calls", type=int, default=512,
                    help="vs-shard: 128-member aggregate sets / 128 in the ONE sharded verifySignatureSets call")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU: relaunch under torch.distributed.run as a child, before any GPU call
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
               "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))

    claim_stdout()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and args.gpus != world:
        sys.exit("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    invalid_frac = args.invalid_frac if args.invalid_frac is not None else (0.01 if args.mode == "replay" else 0.0)
    dist = None
    torch = None
    # the sharded verifySignatureSets line (`vs_shard`) rides on the default gossip line at every N
    want_vs_shard = args.mode == "gossip" and not args.no_extras and not args.no_vs_shard
    if world > 1 or args.mode == "vs-shard" or want_vs_shard:
        # torch (and RCCL) initialise the GPU before libgbv does; --mode vs-shard (and the vs_shard object
        # of the default line) joins a real RCCL process group even at one rank, so the same collective
        # runs at every N
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(free_port()))
            dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))  # RCCL over xGMI

    def log(msg):
        if rank == 0:
            print("[bench] " + msg, file=sys.stderr, flush=True)

    def barrier():
        if dist is not None and world > 1:
            dist.barrier(device_ids=[local_rank])

    from lodestar_amd import GpuBlsVerifier
    from lodestar_amd.build import build
    build()
    v = GpuBlsVerifier(local_rank)
    for kv in args.tune:
        name, val = kv.split("=", 1)
        v.tune(name, int(val))
        log("tune %s = %s" % (name, val))
    sks, key_pks = build_table(v, log)
    sk_ints = [interop_sk_int(i) for i in range(N_KEYS)]
    if args.mode == "vs-shard":
        return vs_shard_main(args, v, sk_ints, world, rank, local_rank, dist, log)

    if args.mode == "gossip":
        # every rank its own stream (replicas, weak scaling)
        call_off, idx, sigs, msgs = build_workload(v, sks, args.sets, rank, log)
        n_mine = args.sets
        gather = None
        expect = np.ones(n_mine, dtype=np.uint8)
        if invalid_frac > 0:
            sigs, expect = inject_invalid(sigs, call_off, n_mine, invalid_frac)
    else:
        # C5: ONE stream (invalid sets injected over the whole of it), calls sharded across ranks;
        # per-set booleans all-gathered over RCCL
        call_off_all, idx_all, sigs_all, msgs_all = build_workload(v, sks, args.sets, 0, log)
        expect_all = np.ones(args.sets, dtype=np.uint8)
        if invalid_frac > 0:
            sigs_all, expect_all = inject_invalid(sigs_all, call_off_all, args.sets, invalid_frac)
        n_calls = len(call_off_all) - 1
        # the product's split (ShardedVerifier.call_ranges): contiguous call ranges of near-equal SET count
        sizes = np.diff(call_off_all.astype(np.int64)).tolist()
        if dist is not None:
            from lodestar_amd.sharded import ShardedVerifier
            ranges = ShardedVerifier(v).call_ranges(sizes)
        else:
            ranges = [(0, n_calls)]
        c0, c1 = ranges[rank]
        s0, s1 = int(call_off_all[c0]), int(call_off_all[c1])
        call_off = (call_off_all[c0:c1 + 1] - s0).astype(np.uint32)
        idx = idx_all[s0:s1]
        sigs = sigs_all[96 * s0:96 * s1]
        msgs = msgs_all[32 * c0:32 * c1]
        expect = expect_all[s0:s1]
        n_mine = s1 - s0
        widths = [int(call_off_all[b] - call_off_all[a]) for a, b in ranges]
        gather = (max(widths), widths, int(expect_all.sum())) if world > 1 else None
    if invalid_frac > 0:
        log("injected %d invalid sets on rank 0 (C5 recipe)" % int((expect == 0).sum()))
    staged = v.stage_same_message(call_off, idx, sigs, msgs)
    depth = max(1, args.inflight) if args.stream else 1
    stages = [staged] + [v.stage_same_message(call_off, idx, sigs, msgs) for _ in range(depth - 1)]
    expect_b = expect.tobytes()

    for _ in range(args.warmup):
        for st in stages:  # every staged copy once: first-use costs stay out of the timed region
            res = st.verify(True)
            assert res == expect_b, "warmup: %d of %d sets verified (expected %d)" % (res.count(1), n_mine, int(expect.sum()))
    log("warmup ok")

    kms = np.zeros(len(KERNELS))
    kcnt = np.zeros(len(KERNELS))
    slow_path = [0, 0]
    gathered = []
    if gather is not None:
        width = gather[0]
        out_bufs = [torch.empty(width, dtype=torch.uint8, device="cuda") for _ in range(world)]

    def collect(b):
        r = b.wait(True)
        assert r == expect_b
        fb, seg = v.last_stats()
        slow_path[0] += fb
        slow_path[1] += seg
        ms, cnt = v.last_kernel_ms()
        kms[:] += np.array(ms)
        kcnt[:] += np.array(cnt)
        if gather is not None:  # RCCL all-gather of the per-set booleans (every rank ends with all of them)
            t = torch.zeros(width, dtype=torch.uint8, device="cuda")
            t[:n_mine] = torch.frombuffer(bytearray(r), dtype=torch.uint8).to("cuda")
            dist.all_gather(out_bufs, t)
            gathered.append(sum(int(o[:w].sum().item()) for o, w in zip(out_bufs, gather[1])))

    barrier()
    t0 = time.perf_counter()
    # batch k is submitted once batch k - depth (the same staged copy) has been collected, so up to
    # `depth` verifications are queued on the device at any time
    for k in range(args.steps):
        b = stages[k % depth]
        if k >= depth:
            collect(b)
        if k == args.steps - 1:
            v.tune("kprof", 1)  # the last batch is also timed kernel by kernel (two events per kernel)
        b.submit()
    v.tune("kprof", 0)
    for k in range(max(0, args.steps - depth), args.steps):
        collect(stages[k % depth])
    barrier()
    elapsed = time.perf_counter() - t0
    step_ops = v.last_ops(0)  # the last collected batch = the last submitted one
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if slow_path != [0, 0] and not invalid_frac:
        log("WARNING: fast path fell back (chunks, segments) = %s on an all-valid workload" % slow_path)
    avg_launch_ms = kms / np.maximum(kcnt, 1)
    kms /= max(args.steps, 1)
    prep_launches_per_step = kcnt[1] / max(args.steps, 1)
    total_sets = (args.sets * world if args.mode == "gossip" else args.sets) * args.steps
    value = total_sets / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    if gathered:  # every rank holds every per-set boolean of the stream after each step
        assert all(g == gather[2] for g in gathered), (gathered[:3], gather[2])

    lat = p50_batch_latency(v, idx, sigs, msgs)
    do_api = rank == 0 and not invalid_frac and not args.no_api
    api_rate, api_n = api_path_rate(v, call_off, idx, sigs, msgs) if do_api else (None, 0)
    api_stream, api_stream_n, api_stream_passes = api_stream_rate(v, call_off, idx, sigs, msgs) if do_api else (None, 0, 0)
    if api_stream:
        log("api stream: %s sets/s over %d sets in %d device passes" % (api_stream, api_stream_n, api_stream_passes))

    # per launch: algorithmic MACs of the sets one k_sm_prepare launch processes / its average duration
    units_per_launch = n_mine / max(prep_launches_per_step, 1)
    t_launch = avg_launch_ms[1] * 1e-3
    comb = v.comb_enabled()
    w_fme = (W_PREPARE_FME_MSM_COMB if comb else W_PREPARE_FME_MSM) if kcnt[7] > 0 else W_PREPARE_FME
    achieved = units_per_launch * w_fme * MAC_PER_FME / t_launch / 1e12 if t_launch > 0 else 0.0
    peak = PEAK_MAC_PER_S / 1e12
    prep_kernel = "k_sm_prepare<false>" if kcnt[7] > 0 else "k_sm_prepare<true>"
    # the stage's two kernels as this run launched them (grid from gbv_last_ops) -> PMC at that grid
    stage_ops = [(k, g, u, m) for k, g, u, m in step_ops if k in ("k_sig_decode", prep_kernel)]
    traffic, pmc = pmc_evidence([(k, g) for k, g, _, _ in stage_ops], units_per_launch,
                                ALG_BYTES_PER_SET_COMB if comb else ALG_BYTES_PER_SET) if stage_ops else (None, None)
    per_unit = {"k_sig_decode": FME_G2_DECODE, prep_kernel: w_fme - FME_G2_DECODE}
    roofline = {"bound": "valu-int", "kernel": "k_sm_prepare stage (k_sig_decode + %s, one stream)" % prep_kernel,
                "achieved": round(achieved, 4), "peak": peak,
                "unit": "T u32-MAC/s", "frac": round(achieved / peak, 5),
                "traffic": round(traffic) if traffic is not None else None, "pmc": pmc,
                "work_per_unit_fme": w_fme, "comb_tables": comb,
                "units_per_launch": round(units_per_launch, 1),
                "avg_launch_ms": round(float(avg_launch_ms[1]), 3),
                "timing": "HIP events on stream A around the stage, every step; per-kernel events on the last step (gbv_last_ops)",
                "stage_kernels": [{"kernel": k, "grid": g, "units": u, "ms": round(m, 3), "work_per_unit_fme": per_unit.get(k),
                                   "frac": round(u * per_unit[k] * MAC_PER_FME / (m * 1e-3) / PEAK_MAC_PER_S, 4) if m > 0 and k in per_unit else None}
                                  for k, g, u, m in stage_ops],
                "last_step_kernels": [{"kernel": k, "grid": g, "units": u, "ms": round(m, 3)} for k, g, u, m in step_ops],
                "kernel_ms_per_step": {k: round(float(x), 3) for k, x in zip(KERNELS, kms)},
                "slow_path_chunks_segments": slow_path}

    extras = {}
    cpu_ok = rank == 0 and not args.no_cpu_baseline
    pk_rows = None
    if rank == 0 and world == 1 and not args.no_extras and args.mode == "gossip":
        if cpu_ok:
            from oracle import cpu_baseline
            pk_rows = cpu_baseline.affine_rows(cpu_baseline.load(), key_pks)
        for name, fn, a, kw in (("c1", c1_bench, sks, {}), ("c3", c3_bench, sk_ints, {"n_calls": args.c3_calls}),
                                # C4 at the verifier queue's MAX_PASSES_IN_FLIGHT (3): 64-block segments are
                                # latency-bound, a third pass fills the device (1.27 -> 1.33 M, profiles/r05x);
                                # C4e and the 65 536-set C1 / C3 passes gain nothing from it (r05x, r05y)
                                ("c4", c4_bench, sk_ints, {"n_blocks": args.c4_blocks, "depth": args.c4_depth}),
                                ("c4e", c4_bench, sk_ints, {"n_blocks": args.c4e_blocks, "electra": True})):
            t = time.time()
            extras[name] = fn(v, a, pk_rows, cpu_ok, **kw)
            log("%s: %s sets/s (%.1fs)" % (name, extras[name]["value"], time.time() - t))
        t = time.time()
        extras["c5"] = c5_bench(v, call_off, idx, sigs, msgs)
        log("c5: %s sets/s (%.1fs)" % (extras["c5"]["value"], time.time() - t))

    vs_shard = None
    if want_vs_shard:
        # the north_star multi-GPU path beside the gossip replicas: ONE verifySignatureSets call sharded
        # over every rank, Fp12 Miller partials all-gathered over RCCL, one final exponentiation each;
        # at N = 1 the same exchange over an RCCL group of one, the anchor of the strong-scaling curve
        vs_shard = vs_shard_measure(args, v, sk_ints, world, rank, log)
        if rank == 0:
            log("vs-shard: %s sets/s over %d ranks" % (vs_shard["value"], world))

    ssz = None
    if rank == 0 and world == 1 and not args.no_signing_roots:
        ssz = signing_roots_bench(v, cpu_sample=0 if args.no_cpu_baseline else 20000)
        log("signing roots: %s roots/s" % ssz["value"])

    # the Node child last: every other device measurement of this process is done before it runs
    api_js = api_path_js(call_off, idx, sigs, msgs, key_pks, log) if do_api and world == 1 else None
    if api_js:
        log("api stream (js): packed %s, IBlsVerifier-shaped %s, objects %s sets/s, lone call %s ms" % (
            api_js["packed"]["sets_per_s"], api_js["ibls"]["sets_per_s"], api_js["objects"]["sets_per_s"], api_js["lone_call_p50_ms"]))

    cpu = None
    cpu_lat = None
    if cpu_ok:
        from oracle import cpu_baseline
        cpu = cpu_baseline.measure_same_message(call_off, idx, sigs, msgs, key_pks, N_KEYS,
                                                target_sets=args.cpu_sample or 32768)
        log("cpu baseline: %s" % cpu)
        if not invalid_frac:
            cpu_lat = cpu_baseline.measure_lone_call_latency(idx, sigs, msgs, key_pks, N_KEYS)
            log("cpu lone-call latency: %s ms" % cpu_lat["p50_ms"])

    if args.mode == "gossip":
        metric = "signature sets verified/sec (batch verify, same-message gossip stream)"
        workload = "C2 gossip attestation stream: 1M single-pubkey sets per GPU, same-message calls of 32-128"
        scaling, parallelism = "weak", "replicas/dp%d" % world
    else:
        metric = "signature sets verified/sec (batch verify, sharded epoch replay with per-set fallback)"
        workload = "C5 epoch replay: %d single-pubkey sets sharded by call over %d GPUs, %.1f%% invalid" % (args.sets, world, 100 * invalid_frac)
        scaling, parallelism = "strong", "shards%d + RCCL all-gather of per-set booleans" % world
    line = {
        "metric": metric,
        "value": round(value, 1),
        "unit": "sets/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "p50_batch_latency_ms": round(lat, 3),
        "cpu_lone_call_latency": cpu_lat,
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "u32 (381-bit Montgomery, integer VALU)",
        "data": "synthetic (interop keys, sha256 messages, GPU-signed)",
        "config": {"workload": workload, "sets_per_gpu": n_mine, "calls_per_gpu": len(call_off) - 1, "table": N_VALIDATORS,
                   "parallelism": parallelism,
                   "submission": "streamed: %d batches in flight" % depth if depth > 1 else "one batch at a time",
                   "timed_region": "device passes over staged batches: the inputs were copied to HBM once before the "
                                   "clock (host-to-device copies outside the timed region); per-set booleans copied back "
                                   "inside it. The host-inclusive rates are api_path_sets_per_s, api_path.oneshot_sets_per_s "
                                   "(PCIe included) and the api_path_js lines",
                   "invalid_frac": invalid_frac},
        "api_path_sets_per_s": api_stream,
        "api_path": {"how": "asyncio: every gossip call of the workload issued through GpuBlsVerifier.verify_signature_sets_same_message "
                            "(packed inputs, prebuilt requests); the job queue cuts passes of <= 2^18 sets, up to 3 on the device "
                            "at once; every boolean checked",
                     "sample_sets": api_stream_n, "device_passes": api_stream_passes,
                     "oneshot_sets_per_s": api_rate, "oneshot_how": "one gbv_verify_same_message_multi call from host buffers"},
        "api_path_js_sets_per_s": api_js["packed"]["sets_per_s"] if api_js else None,
        "api_path_js_iblsverifier_shaped_sets_per_s": api_js["ibls"]["sets_per_s"] if api_js and "ibls" in api_js else None,
        "api_path_js": api_js,
        "roofline": roofline,
        "cpu_baseline": cpu,
        "c1": extras.get("c1"),
        "c3": extras.get("c3"),
        "c4": extras.get("c4"),
        "c4e": extras.get("c4e"),
        "c5": extras.get("c5"),
        "signing_roots": ssz,
        "vs_shard": vs_shard,
    }
    if rank == 0:
        emit_json(line)
    for st in stages:
        st.close()
    if dist is not None:
        barrier()
        dist.destroy_process_group()


def vs_shard_main(args, v, sk_ints, world, rank, local_rank, dist, log):
    line = vs_shard_measure(args, v, sk_ints, world, rank, log)
    if rank == 0:
        emit_json(line)
    import torch.distributed as tdist
    tdist.barrier()
    tdist.destroy_process_group()


def vs_shard_measure(args, v, sk_ints, world, rank, log):
    """--mode vs-shard (and the `vs_shard` object of a multi-GPU gossip line): ONE verifySignatureSets
    call (args.shard_calls x 128 sets of 128-member aggregates, a C3-sized range-sync / replay call) sharded over the ranks by cost-balanced
    contiguous ranges (lodestar_amd/sharded.py).  Each rank stages its shard in HBM (twice); a step is
    gbv_vs_batch_partial (the shard's Fp12 Miller product) -> 577-byte RCCL all-gather -> one final
    exponentiation over all partials (gbv_fp12_check) on every rank, streamed with two shard passes
    in flight per rank (verify_staged_shards).  Before timing: the sharded
    answer equals the single-GPU gbv_verify_sets answer, and a call with one wrong signature in
    another shard is false."""
    import torch
    import torch.distributed as tdist
    from lodestar_amd.sharded import ShardedVerifier
    from lodestar_amd import AggregatedSignatureSet
    backend = tdist.get_backend()
    sv = ShardedVerifier(v)
    rng = np.random.Generator(np.random.PCG64(0x5A))
    sets = _agg_sets(v, sk_ints, 128 * args.shard_calls, b"gbv-shard", rng)
    lo, hi = sv.shard_of(sets)
    # `depth` staged copies of this rank's shard: the step loop keeps that many shard passes in flight
    # (ShardedVerifier.verify_staged_shards), the exchange of pass k beside pass k + 1's kernels
    depth = max(1, args.shard_depth)
    stages = [v.stage_signature_sets([sets[lo:hi]]) for _ in range(depth)]
    staged = stages[0]
    log("vs-shard: %d sets, rank 0 shard [%d, %d), backend %s" % (len(sets), lo, hi, backend))
    assert sv.verify_staged_shard(staged) is True
    single = v.verify_signature_sets_sync(sets) if rank == 0 else None  # the same call on one GPU
    bad = list(sets)
    j = len(sets) - 1 - 7  # the last shard
    bad[j] = AggregatedSignatureSet(sets[j].indices, sets[j].signing_root, sets[0].signature)
    bad_small = bad[-256:]  # one-shot marshalling kept small: the wrong set sits in the last rank's share
    wrong = sv.verify_signature_sets(bad_small)
    ok_small = sv.verify_signature_sets(sets[-256:])
    seq = [stages[k % depth] for k in range(args.steps)]
    if args.warmup:
        warm = [stages[k % depth] for k in range(max(depth, args.warmup))]
        assert sv.verify_staged_shards(warm, depth=depth) == [True] * len(warm)
    tdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    assert sv.verify_staged_shards(seq, depth=depth) == [True] * args.steps
    torch.cuda.synchronize()
    tdist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
    elapsed = float(t.item())
    # one pass alone (no overlap), for the per-pass latency the multi-GPU projection uses
    t1 = time.perf_counter()
    assert sv.verify_staged_shard(staged) is True
    lone_ms = (time.perf_counter() - t1) * 1e3
    for st in stages:
        st.close()
    line = None
    if rank == 0:
        line = {"metric": "signature sets verified/sec (one verifySignatureSets call sharded over GPUs: Fp12 partials + RCCL all-gather)",
                "value": round(len(sets) * args.steps / elapsed, 1), "unit": "sets/s", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
                "scaling": "strong", "vs_baseline": None, "dtype": "u32 (381-bit Montgomery, integer VALU)",
                "data": "synthetic (interop keys, 128-member committee aggregates, GPU-signed)",
                "config": {"workload": "C3-shaped call of %d aggregate sets as ONE verifySignatureSets call" % len(sets),
                           "parallelism": "cost-balanced shards%d + RCCL all-gather of 577-byte Fp12 partials" % world},
                "world_size": world, "backend": backend, "gathered_from_ranks": list(range(world)),
                "partial_bytes_per_gpu": 577, "rank0_shard": [lo, hi], "passes_in_flight": depth,
                "lone_pass_ms": round(lone_ms, 3),
                "parity": {"sharded_equals_single_gpu": single is True, "wrong_signature_call_false": wrong is False,
                           "clean_small_call_true": ok_small is True}}
    return line


if __name__ == "__main__":
    main()
