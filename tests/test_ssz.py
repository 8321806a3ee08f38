"""Signing-root row: SSZ hashing on the device against the oracle.

CPU tests pin the oracle (oracle/ssz_oracle.py) with K1 and check the device SHA-256/SSZ code built
for the host; `gpu` tests run the gfx950 kernels through the C ABI (gbv_sha256_digest64,
gbv_merkle_roots, gbv_signing_roots, gbv_attestation_signing_roots) against the oracle on seeded
inputs.  Bit-exact throughout (byte work).
"""
import ctypes
import hashlib
import os
import random
import struct
import subprocess

import pytest

from oracle import ssz_oracle as S

HERE = os.path.dirname(os.path.abspath(__file__))
HOSTLIB = os.path.join(HERE, "native", "libhosttest.so")

# beacon-node/test/e2e/interop/genesisState.test.ts:50-54 (K1)
K1_PK = bytes.fromhex("a99a76ed7796f7be22d5b7e85deeb7c5677e88e511e0b337618f8c4eb61349b4bf2d153f649f7b53359fe8b94a38e44c")
K1_SIG = bytes.fromhex("a95af8ff0f8c06af4d29aef05ce865f85f82df42b606008ec5b1bcb42b17ae47f4b78cdce1db31ce32d18f42a6b296b4"
                       "014a2164981780e56b5a40d7723c27b8423173e58fa36f075078b177634f66351412b867c103f532aedd50bcd9b98446")
DOMAIN_DEPOSIT = bytes([3, 0, 0, 0])            # params/src/index.ts:142
MINIMAL_GENESIS_FORK_VERSION = bytes([0, 0, 0, 1])  # config/src/chainConfig/configs/minimal.ts:26
DOMAIN_BEACON_ATTESTER = bytes([1, 0, 0, 0])    # params/src/index.ts:140


def k1_deposit_parts():
    wc = bytearray(hashlib.sha256(K1_PK).digest())
    wc[0] = 0
    return bytes(wc), 32_000_000_000


def random_att_data(rng, extreme=False):
    m = (1 << 64) - 1
    u = (lambda: m) if extreme else (lambda: rng.getrandbits(64))
    r = lambda: bytes(rng.getrandbits(8) for _ in range(32))
    return S.attestation_data_serialize(u(), u(), r(), (u(), r()), (u(), r()))


# ---- CPU: oracle pinned by K1 ------------------------------------------------------------------
def test_k1_deposit_root_pins_merkleization():
    """The K1 signature is over computeSigningRoot(DepositMessage, DOMAIN_DEPOSIT domain): the
    oracle's container merkleization, Bytes48 root, uint64 chunk and computeDomain must reproduce the
    signing root that the interop key signs to K1_SIG."""
    from oracle import bls_oracle as o
    wc, amount = k1_deposit_parts()
    obj = S.deposit_message_root(K1_PK, wc, amount)
    domain = S.compute_domain(DOMAIN_DEPOSIT, MINIMAL_GENESIS_FORK_VERSION, bytes(32))
    root = S.compute_signing_root(obj, domain)
    sk = o.interop_secret_key(0)
    assert o.g2_compress(o.sign(sk, root)) == K1_SIG


def test_zero_hashes_and_padding():
    z = bytes(32)
    zh1 = hashlib.sha256(z + z).digest()
    assert zh1.hex() == "f5a5fd42d16a20302798ef6ed309979b43003d2320d9f0e8ea9831a92759fb4b"
    assert S.merkleize([z] * 4) == hashlib.sha256(zh1 + zh1).digest()
    a = bytes(range(32))
    assert S.merkleize([a, a, a]) == S.merkleize([a, a, a, z])
    assert S.merkleize([a]) == a


def test_attestation_root_layout():
    """AttestationData root = 8-leaf tree of slot, index, beaconBlockRoot, source, target."""
    rng = random.Random(5)
    d = random_att_data(rng)
    slot, index = struct.unpack_from("<QQ", d)
    leaves = [S.uint64_chunk(slot), S.uint64_chunk(index), d[16:48],
              S.checkpoint_root(struct.unpack_from("<Q", d, 48)[0], d[56:88]),
              S.checkpoint_root(struct.unpack_from("<Q", d, 88)[0], d[96:128])] + [bytes(32)] * 3
    H = lambda a, b: hashlib.sha256(a + b).digest()
    lv = [H(leaves[i], leaves[i + 1]) for i in range(0, 8, 2)]
    assert S.attestation_data_root(d) == H(H(lv[0], lv[1]), H(lv[2], lv[3]))


# ---- CPU: device SHA-256 / SSZ code built for the host ------------------------------------------
@pytest.fixture(scope="module")
def hostlib():
    csrc = os.path.join(HERE, "..", "lodestar_amd", "csrc")
    srcs = [os.path.join(HERE, "native", "hosttest.cpp")] + [os.path.join(csrc, f) for f in os.listdir(csrc) if f.endswith(".h")]
    if not os.path.exists(HOSTLIB) or os.path.getmtime(HOSTLIB) < max(os.path.getmtime(s) for s in srcs):
        subprocess.check_call([os.path.join(HERE, "native", "build_hosttest.sh")])
    return ctypes.CDLL(HOSTLIB)


def test_host_digest64(hostlib):
    rng = random.Random(1)
    for t in range(200):
        m = bytes(64) if t == 0 else bytes([0xFF]) * 64 if t == 1 else bytes(rng.getrandbits(8) for _ in range(64))
        out = ctypes.create_string_buffer(32)
        hostlib.ht_digest64(out, m)
        assert out.raw == hashlib.sha256(m).digest()


def test_host_attestation_signing_root(hostlib):
    rng = random.Random(2)
    for t in range(50):
        d = random_att_data(rng, extreme=(t == 0))
        dom = bytes(rng.getrandbits(8) for _ in range(32))
        out = ctypes.create_string_buffer(32)
        hostlib.ht_att_signing_root(out, d, dom)
        assert out.raw == S.attestation_signing_root(d, dom)


# ---- GPU: the gfx950 kernels through the C ABI -------------------------------------------------
@pytest.fixture(scope="module")
def v():
    from lodestar_amd import GpuBlsVerifier
    v = GpuBlsVerifier(0)
    yield v
    v.close_sync()


@pytest.mark.gpu
def test_gpu_digest64(v):
    rng = random.Random(3)
    ins = [bytes(64), bytes([0xFF]) * 64] + [bytes(rng.getrandbits(8) for _ in range(64)) for _ in range(3000)]
    assert v.sha256_digest64(ins) == [hashlib.sha256(m).digest() for m in ins]
    assert v.sha256_digest64(b"") == []
    assert v.sha256_digest64([ins[2]]) == [hashlib.sha256(ins[2]).digest()]


@pytest.mark.gpu
@pytest.mark.parametrize("depth", [0, 1, 2, 3, 5])
def test_gpu_merkle_roots(v, depth):
    rng = random.Random(10 + depth)
    n = 257
    objs = [[bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(1 << depth)] for _ in range(n)]
    got = v.merkle_roots([c for o in objs for c in o], depth)
    assert got == [S.merkle_root_fixed(o, depth) for o in objs]


@pytest.mark.gpu
def test_gpu_signing_roots_domains(v):
    rng = random.Random(4)
    roots = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(1000)]
    doms = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(5)]
    idx = [rng.randrange(5) for _ in roots]
    assert v.compute_signing_roots(roots, doms, idx) == [S.compute_signing_root(r, doms[i]) for r, i in zip(roots, idx)]
    assert v.compute_signing_roots(roots, doms[3]) == [S.compute_signing_root(r, doms[3]) for r in roots]
    from lodestar_amd import GbvError
    with pytest.raises(GbvError):
        v.compute_signing_roots(roots[:2], doms, [0, 5])


@pytest.mark.gpu
def test_gpu_attestation_signing_roots(v):
    rng = random.Random(6)
    datas = [random_att_data(rng, extreme=True), bytes(128)] + [random_att_data(rng) for _ in range(2046)]
    doms = [S.compute_domain(DOMAIN_BEACON_ATTESTER, bytes([0, 0, 0, f]), bytes(rng.getrandbits(8) for _ in range(32)))
            for f in range(4)]
    idx = [rng.randrange(4) for _ in datas]
    got = v.attestation_data_signing_roots(datas, doms, idx)
    assert got == [S.attestation_signing_root(d, doms[i]) for d, i in zip(datas, idx)]
    assert v.attestation_data_signing_roots([], doms) == []


@pytest.mark.gpu
def test_gpu_k1_signing_root_feeds_verification(v):
    """DepositMessage signing root built entirely from device hashes (Bytes48 root, container root,
    ForkData root, SigningData root), then verified against K1 on the device."""
    from lodestar_amd import SingleSignatureSet
    wc, amount = k1_deposit_parts()
    pk_root = v.merkle_roots(K1_PK + bytes(16), 1)[0]
    obj = v.merkle_roots(pk_root + wc + S.uint64_chunk(amount) + bytes(32), 2)[0]
    fork_data_root = v.merkle_roots(MINIMAL_GENESIS_FORK_VERSION + bytes(28) + bytes(32), 1)[0]
    domain = DOMAIN_DEPOSIT + fork_data_root[:28]
    root = v.compute_signing_roots([obj], domain)[0]
    assert root == S.compute_signing_root(S.deposit_message_root(K1_PK, wc, amount),
                                          S.compute_domain(DOMAIN_DEPOSIT, MINIMAL_GENESIS_FORK_VERSION, bytes(32)))
    assert v.verify_signature_set(SingleSignatureSet(0, root, K1_SIG, pubkey=K1_PK))
    assert not v.verify_signature_set(SingleSignatureSet(0, root[:-1] + b"\x01", K1_SIG, pubkey=K1_PK))


@pytest.mark.gpu
def test_gpu_attestation_roots_at_scale(v):
    """1M AttestationData values (a bench-sized launch): a seeded sample against the oracle, and
    duplicated inputs must give duplicated roots (size-independent consistency)."""
    import numpy as np
    n = 1 << 20
    rng = np.random.default_rng(7)
    base = rng.integers(0, 256, size=(n // 2, 128), dtype=np.uint8)
    datas = np.concatenate([base, base[::-1]])
    dom = bytes(range(32))
    roots = v.attestation_data_signing_roots(datas.tobytes(), dom)
    assert len(roots) == n
    for i in random.Random(8).sample(range(n), 500):
        assert roots[i] == S.attestation_signing_root(datas[i].tobytes(), dom)
    assert all(roots[i] == roots[n - 1 - i] for i in range(0, n // 2, 997))
    assert v.ssz_last_kernel_ms() > 0
