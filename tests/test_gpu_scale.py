"""GPU parity at bench scale: many same-message calls across several pipeline segments, with invalid
sets injected the way the reference tests build them (bls.test.ts:73 valid-point signature over
another message, bls.test.ts:79 malformed bytes([10]*96)), plus the infinity signature.

Expected booleans hold by construction: every set is signed on the GPU with its own interop key
(util_sign, pinned bit-exactly by the K1 deposit signature in test_gpu_parity.py) except the
injected ones.  A spot sample is re-checked against the CPU oracle.

Run on an MI355X: python -m pytest tests -m gpu
"""
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
N_KEYS = 256
N_TABLE = 4096


def _sk(i):
    d = hashlib.sha256(i.to_bytes(32, "little")).digest()
    return (int.from_bytes(d, "little") % R_ORDER).to_bytes(32, "big")


@pytest.fixture(scope="module")
def world():
    from lodestar_amd import GpuBlsVerifier
    v = GpuBlsVerifier(0)
    sks = [_sk(i) for i in range(N_KEYS)]
    pks = v.util_sk_to_pk(sks)
    assert v.add_pubkeys(0, pks, validate=True) == bytes(N_KEYS)
    v.replicate_pubkeys(0, N_KEYS, N_KEYS, N_TABLE - N_KEYS)
    yield v, sks, pks
    v.close_sync()


@pytest.mark.gpu
def test_comb_tables_match_ladder(world):
    """The per-slot comb tables k_sm_prepare reads (built on append, copied on replicate) give the
    same [a - b x^2] pk as the endomorphism ladder, for appended and replicated slots; a few are
    checked against the oracle."""
    v, sks, pks = world
    if not v.comb_enabled():
        pytest.skip("comb tables disabled (gbv_tune comb 0)")
    rng = np.random.Generator(np.random.PCG64(77))
    slots = [0, 1, N_KEYS - 1, N_KEYS, N_KEYS + 1, N_TABLE - 1] + [int(x) for x in rng.integers(0, N_TABLE, size=250)]
    r64 = [0, 2**64 - 1, 0x0123456789ABCDEF, 1 << 63, 0xFFFFFFFF, 1 << 32] + [int(x) for x in rng.integers(0, 2**63, size=250)]
    from oracle import bls_oracle as O
    # raw entries of slot 0: T[e] = sum_b (bit b of e ? +1 : -1) B_b (b < 7) + B_7
    pk0 = O.pubkey_from_bytes(pks[0], validate=False)
    base = [O.g1_mul(pk0, 1 << (8 * j)) for j in range(4)]
    lam = (-(O.X * O.X)) % O.R
    base += [O.g1_mul(b, lam) for b in base]
    ents = list(range(0, 128, 9)) + [127]
    got = _util_raw(v, [0] * len(ents), ents)
    for e, g in zip(ents, got):
        acc = base[7]
        for b in range(7):
            acc = O.g1_add(acc, base[b] if (e >> b) & 1 else O.g1_neg(base[b]))
        assert g == O.g1_compress(acc), e
    comb = v.util_g1_mul_rand(slots, r64, True)
    ladder = v.util_g1_mul_rand(slots, r64, False)
    bad = [i for i in range(len(slots)) if comb[i] != ladder[i]]
    assert not bad, (len(bad), bad[:8])
    for i in range(4):
        s, r = slots[i], r64[i]
        a = sum(((1 if (r >> j) & 1 else -1) << j) for j in range(32))
        b = sum(((1 if (r >> (32 + j)) & 1 else -1) << j) for j in range(32))
        pk = O.pubkey_from_bytes(pks[s % N_KEYS], validate=False)
        assert comb[i] == O.g1_compress(O.g1_mul(pk, (a - b * O.X * O.X) % O.R))


def _util_raw(v, slots, ents):
    import ctypes
    from lodestar_amd import _native
    s = np.ascontiguousarray(slots, dtype=np.uint32)
    r = np.ascontiguousarray(ents, dtype=np.uint64)
    out = ctypes.create_string_buffer(48 * len(slots))
    _native.check(v._lib, v._ctx, v._lib.gbv_util_g1_mul_rand(v._ctx, s.ctypes.data, r.ctypes.data, len(slots), 2, out))
    return [out.raw[48 * i:48 * i + 48] for i in range(len(slots))]


def _workload(v, sks, n_sets, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    sizes = []
    while sum(sizes) < n_sets:
        sizes.append(int(min(rng.integers(32, 129), n_sets - sum(sizes))))
    off = np.zeros(len(sizes) + 1, dtype=np.uint32)
    off[1:] = np.cumsum(sizes)
    idx = rng.integers(0, N_TABLE, size=n_sets).astype(np.uint32)
    grp = np.repeat(np.arange(len(sizes)), sizes)
    msgs = [hashlib.sha256(b"gbv-scale" + seed.to_bytes(4, "little") + g.to_bytes(8, "little")).digest()
            for g in range(len(sizes))]
    sigs = v.util_sign([sks[int(i) % N_KEYS] for i in idx], grp.tolist(), msgs)
    return off, idx, grp, sigs, msgs


def _run_staged(v, off, idx, sigs, msgs):
    st = v.stage_same_message(off, idx, b"".join(sigs), b"".join(msgs))
    try:
        return [b == 1 for b in st.verify(True)]
    finally:
        st.close()


def _tune(v, segments, msm_min, cooldown):
    v.tune("segments", segments)
    v.tune("msm_min", msm_min)
    v.tune("msm_cooldown", cooldown)


@pytest.fixture(autouse=True)
def _default_settings(request):
    """Every test starts from, and leaves, the context's default pipeline settings."""
    yield
    if "world" in request.fixturenames:
        v = request.getfixturevalue("world")[0]
        _tune(v, 1, 131072, 16)
        for name, value in FORM_DEFAULTS.items():
            v.tune(name, value)


# process-wide launch-form defaults (kernel_common.h Tuning) that tests below move
FORM_DEFAULTS = {"fb_coop_max": 16384, "group_thread_min": 512, "sm_quad_max": 8192}
# "thread": one thread per chunk / run / set check and per chunk Miller value (throughput forms);
# "wave": one wave per check and lane quads per chunk Miller value (latency forms)
FORMS = {"thread": {"fb_coop_max": 0, "group_thread_min": 0, "sm_quad_max": 0},
         "wave": {"fb_coop_max": 16384, "group_thread_min": 1 << 30, "sm_quad_max": 1 << 30}}


@pytest.fixture(params=["ladder", "msm"])
def segments(world, request):
    v = world[0]
    # four pipeline segments; G2 terms per set (32-step ladders) or per segment (bucket MSM,
    # k_msm.hip): both must give the same booleans, and an all-valid stream must pass the segment
    # checks either way; cooldown 0 keeps the MSM on after a failing segment
    _tune(v, 4, 0 if request.param == "ladder" else 1000, 0)
    return request.param


def test_same_message_all_valid_multi_segment(world, segments):
    v, sks, _ = world
    off, idx, grp, sigs, msgs = _workload(v, sks, 80000, 11)
    res = _run_staged(v, off, idx, sigs, msgs)
    assert all(res)
    ms, cnt = v.last_kernel_ms()
    assert cnt[4] >= 2, "expected several pipeline segments"
    # the fast path alone must carry an all-valid stream: no failed segment, no retried chunk
    assert v.last_stats() == (0, 0)


def test_same_message_injected_invalid(world, segments):
    v, sks, _ = world
    off, idx, grp, sigs, msgs = _workload(v, sks, 80000, 12)
    n = len(sigs)
    bad = {}
    # wrong message: a valid G2 point that signs another call's message
    for i in (5, 40001, 79990):
        j = int(np.searchsorted(off, i, side="right"))  # a set in the next call
        j = int(off[j]) if j < len(off) - 1 else 0
        bad[i] = sigs[j] if grp[j] != grp[i] else sigs[(i + 200) % n]
    bad[33333] = bytes([10]) * 96                  # malformed (no compression flag)
    bad[50000] = bytes([0xC0]) + bytes(95)         # infinity signature
    bad[60000] = sigs[60000][:95] + bytes([sigs[60000][95] ^ 1])  # flipped bit: off-curve or wrong point
    sigs = list(sigs)
    for i, s in bad.items():
        sigs[i] = s
    res = _run_staged(v, off, idx, sigs, msgs)
    fb, seg = v.last_stats()
    # the wrong-message sets' chunks fail their checks (malformed and infinity signatures are excluded
    # from their chunk's sums by status, so their chunks pass), and at least one segment fails
    assert fb >= 3 and seg >= 1
    expected = [True] * n
    for i in bad:
        expected[i] = False
    assert res == expected


@pytest.mark.parametrize("form", ["thread", "wave"])
@pytest.mark.parametrize("mode", ["ladder", "msm"])
def test_same_message_one_percent_invalid(world, mode, form):
    """C5-style density: 1 % of 60 000 sets invalid, so hundreds of chunks fail.  The
    failure path (group checks, 8-set run checks, per-set checks) must return exactly the per-set
    booleans in both launch forms: one thread per check (k_sm_group_check, k_sm_fb_blocks,
    k_sm_fb_sets, k_sm_miller) and one wave per check (k_sm_group_pairing, k_sm_fb_blocks_coop,
    k_sm_fb_sets_*, k_sm_miller_quad).  In MSM mode the failing segment first recomputes its per-set
    G2 terms (k_sm_redo_g2)."""
    v, sks, _ = world
    _tune(v, 1, 1000 if mode == "msm" else 0, 0)
    for name, value in FORMS[form].items():
        v.tune(name, value)
    _one_percent(v, sks)


def _one_percent(v, sks):
    off, idx, grp, sigs, msgs = _workload(v, sks, 60000, 14)
    n = len(sigs)
    rng = np.random.Generator(np.random.PCG64(0xC0FFEE))
    bad = sorted(rng.choice(n, size=n // 100, replace=False).tolist())
    sigs = list(sigs)
    for k, i in enumerate(bad):
        if k % 10 == 9:
            sigs[i] = bytes([10]) * 96
        else:
            j = (i + 300) % n
            assert grp[j] != grp[i]
            sigs[i] = sigs[j]
    res = _run_staged(v, off, idx, sigs, msgs)
    fb, seg = v.last_stats()
    assert fb > 256 and seg >= 1
    expected = [True] * n
    for i in bad:
        expected[i] = False
    assert res == expected


@pytest.mark.parametrize("n_sets", [300, 700])
def test_same_message_small_pass_roles(world, n_sets):
    """One small pass (one segment) through the latency prepare (k_sm_prep_roles_quad: subgroup
    checks and r sig / r pk on lane quads) -- or per segment by the MSM while an earlier test's
    failure keeps its cooldown on.  All-valid must pass the segment check outright (the G1 and G2
    scalars agree), and injected invalid sets come back exactly."""
    v, sks, _ = world
    off, idx, grp, sigs, msgs = _workload(v, sks, n_sets, 15 + n_sets)
    assert all(_run_staged(v, off, idx, sigs, msgs))
    assert v.last_stats() == (0, 0)
    n = len(sigs)
    bad = {3: sigs[(3 + 200) % n], n - 2: bytes([0xC0]) + bytes(95)}  # another call's signature; infinity
    assert grp[3] != grp[(3 + 200) % n]
    sigs = list(sigs)
    for i, s in bad.items():
        sigs[i] = s
    assert _run_staged(v, off, idx, sigs, msgs) == [i not in bad for i in range(n)]


def test_same_message_spot_check_oracle(world):
    """A few GPU-signed sets re-verified by the CPU oracle (pins util_sign beyond K1)."""
    from oracle import bls_oracle as O
    v, sks, pks = world
    off, idx, grp, sigs, msgs = _workload(v, sks, 64, 13)
    for i in (0, 17, 63):
        k = int(idx[i]) % N_KEYS
        assert O.set_is_valid(O.pubkey_from_bytes(pks[k]), msgs[int(grp[i])], sigs[i])


def test_verify_sets_large_chunks(world):
    """verifySignatureSets over 300 distinct-message sets (chunks of <=128) with one bad set."""
    from lodestar_amd import SingleSignatureSet
    v, sks, _ = world
    msgs = [hashlib.sha256(b"vs" + i.to_bytes(4, "little")).digest() for i in range(300)]
    idx = [(7 * i) % N_TABLE for i in range(300)]
    sigs = v.util_sign([sks[i % N_KEYS] for i in idx], list(range(300)), msgs)
    sets = [SingleSignatureSet(idx[i], msgs[i], sigs[i]) for i in range(300)]
    assert v.verify_signature_sets_sync(sets) is True
    sets[150] = SingleSignatureSet(idx[150], msgs[151], sigs[150])
    assert v.verify_signature_sets_sync(sets) is False


def _vs_sets(v, sks, n, tag):
    from lodestar_amd import AggregatedSignatureSet, SingleSignatureSet
    msgs = [hashlib.sha256(tag + i.to_bytes(4, "little")).digest() for i in range(n)]
    out = []
    for i in range(n):
        if i % 5 == 0:  # a 128-member committee aggregate (C3 shape) from the HBM table
            idx = [(13 * i + 7 * j) % N_TABLE for j in range(128)]
            agg = sum(int.from_bytes(sks[k % N_KEYS], "big") for k in idx) % R_ORDER
            sig = v.util_sign([agg.to_bytes(32, "big")], [0], [msgs[i]])[0]
            out.append(AggregatedSignatureSet(idx, msgs[i], sig))
        else:
            k = (11 * i) % N_TABLE
            out.append(SingleSignatureSet(k, msgs[i], v.util_sign([sks[k % N_KEYS]], [0], [msgs[i]])[0]))
    return out


def test_vs_shard_partials_combine(world):
    """8(e): per-shard Fp12 Miller partials (gbv_vs_partial) + one final exponentiation over all
    of them (gbv_fp12_check) agree with the single-device verifySignatureSets."""
    from lodestar_amd import SingleSignatureSet
    v, sks, _ = world
    sets = _vs_sets(v, sks, 150, b"shard")
    assert v.verify_signature_sets_sync(sets) is True
    cuts = [0, 37, 101, 150]
    parts = [v.vs_partial(sets[a:b]) for a, b in zip(cuts, cuts[1:])]
    assert all(ok for _, ok in parts) and all(len(p) == 576 for p, _ in parts)
    assert v.fp12_check([p for p, _ in parts]) is True
    # a valid point over the wrong message in the middle shard: every shard decodes, product fails
    bad = list(sets)
    bad[61] = SingleSignatureSet(bad[61].index, bad[62].signing_root, bad[61].signature)
    parts = [v.vs_partial(bad[a:b]) for a, b in zip(cuts, cuts[1:])]
    assert all(ok for _, ok in parts)
    assert v.fp12_check([p for p, _ in parts]) is False
    assert v.verify_signature_sets_sync(bad) is False
    # malformed signature: that shard reports shard_ok = False
    bad = list(sets)
    bad[121] = SingleSignatureSet(bad[121].index, bad[121].signing_root, bytes([10]) * 96)
    assert v.vs_partial(bad[101:150])[1] is False


def test_sharded_verifier_single_rank(world):
    """ShardedVerifier over a 1-rank gloo group on the GPU box (the N>1 collective path itself is
    covered by tests/test_sharded.py with 2 gloo ranks)."""
    import socket
    import torch.distributed as dist
    from lodestar_amd.sharded import ShardedVerifier
    v, sks, _ = world
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1)
    try:
        sv = ShardedVerifier(v)
        sets = _vs_sets(v, sks, 40, b"rank1")
        assert sv.verify_signature_sets(sets) is True
        msg = hashlib.sha256(b"sm").digest()
        sigs = v.util_sign([sks[k] for k in range(8)], [0] * 8, [msg])
        calls = [([(k, sigs[k]) for k in range(5)], msg), ([(5, sigs[5]), (6, sigs[0])], msg)]
        assert sv.verify_same_message_multi(calls) == [[True] * 5, [True, False]]
        # streamed staged shards: two passes in flight (gbv_vs_batch_partial_submit / _wait), a
        # wrong-message call between valid ones, each handle re-verified
        from lodestar_amd import SingleSignatureSet
        bad = list(sets)
        bad[17] = SingleSignatureSet(bad[17].index, bad[18].signing_root, bad[17].signature)
        stages = [v.stage_signature_sets([sets]), v.stage_signature_sets([bad]), v.stage_signature_sets([sets])]
        try:
            seq = [stages[k % 3] for k in range(7)]
            assert sv.verify_staged_shards(seq, depth=2) == [k % 3 != 1 for k in range(7)]
            assert sv.verify_staged_shards(seq, depth=3) == [k % 3 != 1 for k in range(7)]
            with pytest.raises(Exception):
                stages[0].partial_wait()  # not submitted
        finally:
            for st in stages:
                st.close()
    finally:
        dist.destroy_process_group()


def test_same_message_msm_single_segment(world):
    """One 100 000-set segment through the bucket MSM at its default size threshold (the bench's
    shape at 1/10 scale): the segment check must pass on the MSM's sum alone, and the MSM kernels
    must have run (their time is reported in slot 7 of last_kernel_ms)."""
    v, sks, _ = world
    _tune(v, 1, 65536, 0)
    off, idx, grp, sigs, msgs = _workload(v, sks, 100000, 15)
    res = _run_staged(v, off, idx, sigs, msgs)
    assert all(res)
    assert v.last_stats() == (0, 0)
    ms, cnt = v.last_kernel_ms()
    assert len(cnt) == 8 and cnt[7] == 1
    # one wrong-message signature: the MSM segment fails, the redo + per-chunk path finds the set
    sigs = list(sigs)
    sigs[77777] = sigs[(77777 + 300) % len(sigs)]
    res = _run_staged(v, off, idx, sigs, msgs)
    assert res == [i != 77777 for i in range(len(sigs))]
    fb, seg = v.last_stats()
    assert fb == 1 and seg == 1


def test_msm_duplicate_signatures(world):
    """One key signing one message 20 000 times in one MSM segment: every (half, window) of the bucket
    MSM then holds thousands of repeated digits of the same point, so the bucket sums (k_msm_runs) meet
    acc = +-q -- the doubling and infinity cases of the complete mixed addition. The segment check must
    pass on the MSM's sum, and a wrong-message signature among the copies must be the one set
    rejected."""
    v, sks, _ = world
    _tune(v, 1, 1000, 0)
    n = 20000
    off = np.array([0, n], dtype=np.uint32)
    idx = np.full(n, 7, dtype=np.uint32)
    msg = hashlib.sha256(b"gbv-dup").digest()
    sig = v.util_sign([sks[7]], [0], [msg])[0]
    sigs = [sig] * n
    assert all(_run_staged(v, off, idx, sigs, [msg]))
    assert v.last_stats() == (0, 0)
    ms, cnt = v.last_kernel_ms()
    assert cnt[7] == 1
    sigs[12345] = v.util_sign([sks[7]], [0], [hashlib.sha256(b"gbv-dup-other").digest()])[0]
    assert _run_staged(v, off, idx, sigs, [msg]) == [i != 12345 for i in range(n)]


def test_msm_cooldown_after_failing_segment(world):
    """After an MSM segment fails, the next submits use the per-set ladders (an invalid-dense stream
    would otherwise pay the MSM and the G2 recomputation); booleans are the same either way."""
    v, sks, _ = world
    _tune(v, 1, 1000, 2)
    off, idx, grp, sigs, msgs = _workload(v, sks, 5000, 16)
    bad = list(sigs)
    bad[123] = bytes([10]) * 96
    want = [i != 123 for i in range(len(sigs))]
    st = v.stage_same_message(off, idx, b"".join(bad), b"".join(msgs))
    try:
        # a chunk holding a malformed set is excluded from the segment check, so this one passes;
        # a wrong-message signature makes the segment fail
        bad[4000] = sigs[(4000 + 300) % len(sigs)]
        want[4000] = False
        st.close()
        st = v.stage_same_message(off, idx, b"".join(bad), b"".join(msgs))
        msm_runs = []
        for _ in range(4):
            assert [b == 1 for b in st.verify(True)] == want
            msm_runs.append(v.last_kernel_ms()[1][7])
        assert msm_runs == [1, 0, 0, 1]  # MSM, cooldown x2, MSM again
    finally:
        st.close()
