"""CPU restatement of the BLS12-381 signature-set verification path -- TEST INFRASTRUCTURE ONLY.

This module is the parity ORACLE.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it, and only as the checker.  The product path
(``lodestar_amd``) never imports anything under ``oracle/``.

What it restates (the reference's arithmetic lives in the third-party ``@chainsafe/blst`` 2.1.0,
pinned at ``/root/reference/yarn.lock:446-457`` and NOT vendored, so its published algorithms are
restated here from their specifications):

* BLS12-381 field tower Fp / Fp2 / Fp6 / Fp12, G1 (y^2 = x^3 + 4) and G2 (y^2 = x^3 + 4(1+i)).
* ZCash point (de)serialisation as blst implements it (``Signature.fromBytes(sig, true)``,
  ``PublicKey.fromBytes`` / ``toBytes``) -- flag bits c/i/s, canonical x < p, infinity rules.
* RFC 9380 ``BLS12381G2_XMD:SHA-256_SSWU_RO_`` hash_to_G2 with the POP DST
  ``BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_`` (IETF BLS draft-04, minimal-pubkey-size).
* Optimal-ate pairing (Miller loop over |x| with x = -0xd201000000010000, final exponentiation).
* KeyGen (IETF BLS draft-04 HKDF, salted with H("BLS-SIG-KEYGEN-SALT-")), Sign, Verify,
  aggregatePublicKeys, blst-style randomised batch verification.
* Lodestar's orchestration semantics that decide the booleans callers see:
  ``verifySignatureSetsMaybeBatch`` (packages/beacon-node/src/chain/bls/maybeBatch.ts:15-45),
  ``chunkifyMaximizeChunkSize`` (multithread/utils.ts:4-18),
  ``BlsMultiThreadWorkerPool.verifySignatureSets`` / ``verifySignatureSetsSameMessage``
  (multithread/index.ts:157-236), same-message retry (jobItem.ts:93-125, index.ts:552-563).

Parity is pinned by the in-repo known-answer vectors of SURVEY.md section 8(c): K1 interop-key-0
deposit signature (beacon-node/test/e2e/interop/genesisState.test.ts:50-54), K2 cached KeyGen
keys (cli/test/utils/cachedKeys.ts:15-26), K3 infinity encodings, K4 the "valid signature of random
data" (beacon-node/test/unit/chain/opPools/attestationPool.test.ts:10-13) and K6 the generated
validator pubkey (beacon-node/test/utils/validator.ts:18).  See tests/test_oracle_kat.py.
"""
from __future__ import annotations

import hashlib
import hmac
import os
import random as _random

# --------------------------------------------------------------------------------------------
# Parameters
# --------------------------------------------------------------------------------------------
P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
X = -0xD201000000010000  # curve parameter (negative)
X_ABS = 0xD201000000010000
DST_POP = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"

# Counter of Fp multiplications (mul + sqr) used to fix the algorithmic-work constants.
FP_MUL_COUNT = [0]


def fp_inv(a):
    return pow(a, P - 2, P)


def fp_sqrt(a):
    """Return a square root of a in Fp or None (p = 3 mod 4)."""
    a %= P
    s = pow(a, (P + 1) // 4, P)
    return s if s * s % P == a else None


def fp_is_square(a):
    a %= P
    return a == 0 or pow(a, (P - 1) // 2, P) == 1


# --------------------------------------------------------------------------------------------
# Fp2 = Fp[i]/(i^2+1); elements are tuples (c0, c1)
# --------------------------------------------------------------------------------------------
F2_ZERO = (0, 0)
F2_ONE = (1, 0)


def f2(a, b=0):
    return (a % P, b % P)


def f2_add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def f2_sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def f2_neg(a):
    return ((-a[0]) % P, (-a[1]) % P)


def f2_mul(a, b):
    FP_MUL_COUNT[0] += 3
    t0 = a[0] * b[0]
    t1 = a[1] * b[1]
    return ((t0 - t1) % P, ((a[0] + a[1]) * (b[0] + b[1]) - t0 - t1) % P)


def f2_sqr(a):
    FP_MUL_COUNT[0] += 2
    return ((a[0] + a[1]) * (a[0] - a[1]) % P, 2 * a[0] * a[1] % P)


def f2_muls(a, s):
    return (a[0] * s % P, a[1] * s % P)


def f2_conj(a):
    return (a[0], (-a[1]) % P)


def f2_inv(a):
    n = fp_inv((a[0] * a[0] + a[1] * a[1]) % P)
    return (a[0] * n % P, (-a[1]) * n % P)


def f2_mul_xi(a):  # multiply by xi = 1 + i
    return ((a[0] - a[1]) % P, (a[0] + a[1]) % P)


def f2_pow(a, e):
    r = F2_ONE
    while e:
        if e & 1:
            r = f2_mul(r, a)
        a = f2_sqr(a)
        e >>= 1
    return r


def f2_is_zero(a):
    return a[0] == 0 and a[1] == 0


def f2_sgn0(a):
    """RFC 9380 sgn0 for Fp2."""
    sign_0 = a[0] & 1
    zero_0 = a[0] == 0
    sign_1 = a[1] & 1
    return sign_0 | (zero_0 and sign_1)


def f2_is_square(a):
    # a is a square in Fp2 iff its norm is a square in Fp
    return fp_is_square((a[0] * a[0] + a[1] * a[1]) % P)


def f2_sqrt(a):
    """A square root of a in Fp2 (any of the two), or None."""
    if f2_is_zero(a):
        return F2_ZERO
    a0, a1 = a
    if a1 == 0:
        s = fp_sqrt(a0)
        if s is not None:
            return (s, 0)
        s = fp_sqrt(-a0 % P)  # sqrt(a0) = i * sqrt(-a0)
        return (0, s) if s is not None else None
    alpha = fp_sqrt((a0 * a0 + a1 * a1) % P)
    if alpha is None:
        return None
    inv2 = fp_inv(2)
    delta = (a0 + alpha) * inv2 % P
    x0 = fp_sqrt(delta)
    if x0 is None:
        delta = (a0 - alpha) * inv2 % P
        x0 = fp_sqrt(delta)
        if x0 is None:
            return None
    x1 = a1 * fp_inv(2 * x0 % P) % P
    r = (x0, x1)
    assert f2_sqr(r) == (a0 % P, a1 % P)
    return r


def f2_lexi_larger(y):
    """ZCash 'lexicographically largest' for Fp2: compare c1 first, then c0."""
    half = (P - 1) // 2
    if y[1] != 0:
        return y[1] > half
    return y[0] > half


# --------------------------------------------------------------------------------------------
# Fp6 = Fp2[v]/(v^3 - xi), Fp12 = Fp6[w]/(w^2 - v)
# --------------------------------------------------------------------------------------------
F6_ZERO = (F2_ZERO, F2_ZERO, F2_ZERO)
F6_ONE = (F2_ONE, F2_ZERO, F2_ZERO)
F12_ONE = (F6_ONE, F6_ZERO)


def f6_add(a, b):
    return (f2_add(a[0], b[0]), f2_add(a[1], b[1]), f2_add(a[2], b[2]))


def f6_sub(a, b):
    return (f2_sub(a[0], b[0]), f2_sub(a[1], b[1]), f2_sub(a[2], b[2]))


def f6_neg(a):
    return (f2_neg(a[0]), f2_neg(a[1]), f2_neg(a[2]))


def f6_mul(a, b):
    t0 = f2_mul(a[0], b[0])
    t1 = f2_mul(a[1], b[1])
    t2 = f2_mul(a[2], b[2])
    c0 = f2_add(t0, f2_mul_xi(f2_add(f2_mul(a[1], b[2]), f2_mul(a[2], b[1]))))
    c1 = f2_add(f2_add(f2_mul(a[0], b[1]), f2_mul(a[1], b[0])), f2_mul_xi(t2))
    c2 = f2_add(f2_add(f2_mul(a[0], b[2]), t1), f2_mul(a[2], b[0]))
    return (c0, c1, c2)


def f6_mul_v(a):
    return (f2_mul_xi(a[2]), a[0], a[1])


def f6_inv(a):
    c0, c1, c2 = a
    t0 = f2_sub(f2_sqr(c0), f2_mul_xi(f2_mul(c1, c2)))
    t1 = f2_sub(f2_mul_xi(f2_sqr(c2)), f2_mul(c0, c1))
    t2 = f2_sub(f2_sqr(c1), f2_mul(c0, c2))
    d = f2_add(f2_mul(c0, t0), f2_mul_xi(f2_add(f2_mul(c2, t1), f2_mul(c1, t2))))
    di = f2_inv(d)
    return (f2_mul(t0, di), f2_mul(t1, di), f2_mul(t2, di))


def f12_mul(a, b):
    t0 = f6_mul(a[0], b[0])
    t1 = f6_mul(a[1], b[1])
    c1 = f6_sub(f6_sub(f6_mul(f6_add(a[0], a[1]), f6_add(b[0], b[1])), t0), t1)
    return (f6_add(t0, f6_mul_v(t1)), c1)


def f12_sqr(a):
    return f12_mul(a, a)


def f12_conj(a):
    return (a[0], f6_neg(a[1]))


def f12_inv(a):
    d = f6_sub(f6_mul(a[0], a[0]), f6_mul_v(f6_mul(a[1], a[1])))
    di = f6_inv(d)
    return (f6_mul(a[0], di), f6_neg(f6_mul(a[1], di)))


def f12_pow(a, e):
    r = F12_ONE
    while e:
        if e & 1:
            r = f12_mul(r, a)
        a = f12_sqr(a)
        e >>= 1
    return r


XI = (1, 1)
# Frobenius constants: v^p = v * xi^((p-1)/3), w^p = w * xi^((p-1)/6)
FROB_V1 = f2_pow(XI, (P - 1) // 3)
FROB_V2 = f2_pow(XI, 2 * (P - 1) // 3)
FROB_W = f2_pow(XI, (P - 1) // 6)


def f6_frob(a):
    return (f2_conj(a[0]), f2_mul(f2_conj(a[1]), FROB_V1), f2_mul(f2_conj(a[2]), FROB_V2))


def f12_frob(a):
    c0 = f6_frob(a[0])
    c1 = f6_frob(a[1])
    c1 = (f2_mul(c1[0], FROB_W), f2_mul(c1[1], FROB_W), f2_mul(c1[2], FROB_W))
    return (c0, c1)


def f12_frob_n(a, n):
    for _ in range(n):
        a = f12_frob(a)
    return a


def f12_from_f2_at(c, pos):
    """Fp12 element whose only non-zero coefficient is c at w^pos (pos in 0..5)."""
    # w^pos = v^(pos//2) * w^(pos%2)
    six = [F2_ZERO, F2_ZERO, F2_ZERO]
    six[pos // 2] = c
    if pos % 2 == 0:
        return (tuple(six), F6_ZERO)
    return (F6_ZERO, tuple(six))


# --------------------------------------------------------------------------------------------
# Generic short-Weierstrass affine arithmetic (a = 0).  Points: None (infinity) or (x, y).
# --------------------------------------------------------------------------------------------
class _Fp:
    zero = 0
    one = 1
    add = staticmethod(lambda a, b: (a + b) % P)
    sub = staticmethod(lambda a, b: (a - b) % P)
    neg = staticmethod(lambda a: (-a) % P)
    mul = staticmethod(lambda a, b: a * b % P)
    sqr = staticmethod(lambda a: a * a % P)
    inv = staticmethod(fp_inv)
    muls = staticmethod(lambda a, s: a * s % P)


class _Fp2:
    zero = F2_ZERO
    one = F2_ONE
    add = staticmethod(f2_add)
    sub = staticmethod(f2_sub)
    neg = staticmethod(f2_neg)
    mul = staticmethod(f2_mul)
    sqr = staticmethod(f2_sqr)
    inv = staticmethod(f2_inv)
    muls = staticmethod(f2_muls)


B1 = 4
B2 = (4, 4)


def _on_curve(F, b, pt):
    if pt is None:
        return True
    x, y = pt
    return F.sqr(y) == F.add(F.mul(F.sqr(x), x), b)


def _pt_neg(F, pt):
    return None if pt is None else (pt[0], F.neg(pt[1]))


def _pt_add(F, p1, p2):
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    x1, y1 = p1
    x2, y2 = p2
    if x1 == x2:
        if y1 == y2 and y1 != F.zero:
            lam = F.mul(F.muls(F.sqr(x1), 3), F.inv(F.muls(y1, 2)))
        else:
            return None
    else:
        lam = F.mul(F.sub(y2, y1), F.inv(F.sub(x2, x1)))
    x3 = F.sub(F.sub(F.sqr(lam), x1), x2)
    y3 = F.sub(F.mul(lam, F.sub(x1, x3)), y1)
    return (x3, y3)


def _pt_mul(F, pt, k):
    if k < 0:
        return _pt_mul(F, _pt_neg(F, pt), -k)
    res = None
    add = pt
    while k:
        if k & 1:
            res = _pt_add(F, res, add)
        add = _pt_add(F, add, add)
        k >>= 1
    return res


def g1_on_curve(pt):
    return _on_curve(_Fp, B1, pt)


def g2_on_curve(pt):
    return _on_curve(_Fp2, B2, pt)


def g1_add(a, b):
    return _pt_add(_Fp, a, b)


def g2_add(a, b):
    return _pt_add(_Fp2, a, b)


def g1_neg(a):
    return _pt_neg(_Fp, a)


def g2_neg(a):
    return _pt_neg(_Fp2, a)


def g1_mul(a, k):
    return _pt_mul(_Fp, a, k)


def g2_mul(a, k):
    return _pt_mul(_Fp2, a, k)


G1_GEN = (
    0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB,
    0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1,
)
G2_GEN = (
    (
        0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
        0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E,
    ),
    (
        0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
        0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE,
    ),
)

# psi endomorphism on E2 (untwist-Frobenius-twist): psi(x, y) = (conj(x) * PSI_X, conj(y) * PSI_Y)
PSI_X = f2_inv(f2_pow(XI, (P - 1) // 3))
PSI_Y = f2_inv(f2_pow(XI, (P - 1) // 2))


def g2_psi(pt):
    if pt is None:
        return None
    return (f2_mul(f2_conj(pt[0]), PSI_X), f2_mul(f2_conj(pt[1]), PSI_Y))


# GLV endomorphism on E1: phi(x, y) = (beta * x, y), beta a primitive cube root of unity.
# beta is chosen so that phi(P) = [-x^2] P on G1 (Scott, "A note on group membership tests").
def _find_beta():
    for cand in (pow(2, (P - 1) // 3, P), pow(3, (P - 1) // 3, P), pow(5, (P - 1) // 3, P)):
        if cand == 1:
            continue
        for b in (cand, cand * cand % P):
            gp = (b * G1_GEN[0] % P, G1_GEN[1])
            if gp == g1_mul(G1_GEN, (-X * X) % R):
                return b
    raise AssertionError("beta not found")


BETA = _find_beta()


def g1_in_subgroup(pt):
    """G1 membership (Scott 2021): phi(P) == [-x^2] P.  Cross-checked against [r]P == O in tests."""
    if pt is None:
        return True
    return (BETA * pt[0] % P, pt[1]) == g1_mul(pt, -X * X)


def g2_in_subgroup(pt):
    """G2 membership (Scott 2021): psi(P) == [x] P.  Cross-checked against [r]P == O in tests."""
    if pt is None:
        return True
    return g2_psi(pt) == g2_mul(pt, X)


def g1_in_subgroup_naive(pt):
    return g1_mul(pt, R) is None


def g2_in_subgroup_naive(pt):
    return g2_mul(pt, R) is None


# --------------------------------------------------------------------------------------------
# ZCash serialisation (blst semantics)
# --------------------------------------------------------------------------------------------
class DecodeError(Exception):
    """Mirrors blst's BLST_BAD_ENCODING / POINT_NOT_ON_CURVE / POINT_NOT_IN_GROUP / PK_IS_INFINITY."""


def g1_compress(pt):
    if pt is None:
        return bytes([0xC0]) + bytes(47)
    x, y = pt
    b = bytearray(x.to_bytes(48, "big"))
    b[0] |= 0x80
    if y > (P - 1) // 2:
        b[0] |= 0x20
    return bytes(b)


def g1_decompress(b):
    """blst POINTonE1_Uncompress_Z: returns point (None = infinity) or raises DecodeError."""
    if len(b) != 48:
        raise DecodeError("BAD_ENCODING")
    in0 = b[0]
    if not in0 & 0x80:
        raise DecodeError("BAD_ENCODING")
    if in0 & 0x40:
        if (in0 & 0x3F) == 0 and not any(b[1:]):
            return None
        raise DecodeError("BAD_ENCODING")
    x = int.from_bytes(bytes([in0 & 0x1F]) + b[1:], "big")
    if x >= P:
        raise DecodeError("BAD_ENCODING")
    y = fp_sqrt((x * x * x + B1) % P)
    if y is None:
        raise DecodeError("POINT_NOT_ON_CURVE")
    if (y > (P - 1) // 2) != bool(in0 & 0x20):
        y = (-y) % P
    if x == 0:
        raise DecodeError("POINT_NOT_IN_GROUP")
    return (x, y)


def g2_compress(pt):
    if pt is None:
        return bytes([0xC0]) + bytes(95)
    x, y = pt
    b = bytearray(x[1].to_bytes(48, "big") + x[0].to_bytes(48, "big"))
    b[0] |= 0x80
    if f2_lexi_larger(y):
        b[0] |= 0x20
    return bytes(b)


def g2_serialize(pt):
    """Uncompressed 192-byte encoding."""
    if pt is None:
        return bytes([0x40]) + bytes(191)
    x, y = pt
    return x[1].to_bytes(48, "big") + x[0].to_bytes(48, "big") + y[1].to_bytes(48, "big") + y[0].to_bytes(48, "big")


def g2_decompress(b):
    """blst POINTonE2_Uncompress_Z (96 bytes)."""
    if len(b) != 96:
        raise DecodeError("BAD_ENCODING")
    in0 = b[0]
    if not in0 & 0x80:
        raise DecodeError("BAD_ENCODING")
    if in0 & 0x40:
        if (in0 & 0x3F) == 0 and not any(b[1:]):
            return None
        raise DecodeError("BAD_ENCODING")
    x1 = int.from_bytes(bytes([in0 & 0x1F]) + b[1:48], "big")
    x0 = int.from_bytes(b[48:96], "big")
    if x1 >= P or x0 >= P:
        raise DecodeError("BAD_ENCODING")
    x = (x0, x1)
    y = f2_sqrt(f2_add(f2_mul(f2_sqr(x), x), B2))
    if y is None:
        raise DecodeError("POINT_NOT_ON_CURVE")
    if f2_lexi_larger(y) != bool(in0 & 0x20):
        y = f2_neg(y)
    if f2_is_zero(x):
        raise DecodeError("POINT_NOT_IN_GROUP")
    return (x, y)


def g2_deserialize_uncompressed(b):
    """blst POINTonE2_Deserialize_Z for a 192-byte input (parity unpinned: SURVEY 8(c) (ii))."""
    if len(b) != 192:
        raise DecodeError("BAD_ENCODING")
    in0 = b[0]
    if in0 & 0x80:
        raise DecodeError("BAD_ENCODING")
    if in0 & 0xE0:
        if (in0 & 0x40) and (in0 & 0x3F) == 0 and not any(b[1:]):
            return None
        raise DecodeError("BAD_ENCODING")
    vals = [int.from_bytes(b[i * 48:(i + 1) * 48], "big") for i in range(4)]
    if any(v >= P for v in vals):
        raise DecodeError("BAD_ENCODING")
    pt = ((vals[1], vals[0]), (vals[3], vals[2]))
    if not g2_on_curve(pt):
        raise DecodeError("POINT_NOT_ON_CURVE")
    if f2_is_zero(pt[0]):
        raise DecodeError("POINT_NOT_IN_GROUP")
    return pt


def signature_from_bytes(b, validate=True):
    """@chainsafe/blst ``Signature.fromBytes(bytes, true)``: decode + (infinity, subgroup) checks."""
    b = bytes(b)
    if len(b) == 96:
        pt = g2_decompress(b)
    elif len(b) == 192:
        pt = g2_deserialize_uncompressed(b)
    else:
        raise DecodeError("BAD_ENCODING")
    if validate:
        if pt is None:
            raise DecodeError("PK_IS_INFINITY")
        if not g2_in_subgroup(pt):
            raise DecodeError("POINT_NOT_IN_GROUP")
    return pt


def pubkey_from_bytes(b, validate=False):
    """@chainsafe/blst ``PublicKey.fromBytes(bytes, validate)``."""
    pt = g1_decompress(bytes(b))
    if validate:
        if pt is None:
            raise DecodeError("PK_IS_INFINITY")
        if not g1_in_subgroup(pt):
            raise DecodeError("POINT_NOT_IN_GROUP")
    return pt


# --------------------------------------------------------------------------------------------
# RFC 9380 hash_to_curve for G2 (BLS12381G2_XMD:SHA-256_SSWU_RO_)
# --------------------------------------------------------------------------------------------
def expand_message_xmd(msg: bytes, dst: bytes, len_in_bytes: int) -> bytes:
    b_in_bytes, r_in_bytes = 32, 64
    ell = (len_in_bytes + b_in_bytes - 1) // b_in_bytes
    assert ell <= 255 and len(dst) <= 255
    dst_prime = dst + bytes([len(dst)])
    z_pad = bytes(r_in_bytes)
    l_i_b = len_in_bytes.to_bytes(2, "big")
    b0 = hashlib.sha256(z_pad + msg + l_i_b + b"\x00" + dst_prime).digest()
    b1 = hashlib.sha256(b0 + b"\x01" + dst_prime).digest()
    out = [b1]
    for i in range(2, ell + 1):
        prev = out[-1]
        out.append(hashlib.sha256(bytes(x ^ y for x, y in zip(b0, prev)) + bytes([i]) + dst_prime).digest())
    return b"".join(out)[:len_in_bytes]


def hash_to_field_fp2(msg: bytes, count: int, dst: bytes = DST_POP):
    L = 64
    data = expand_message_xmd(msg, dst, count * 2 * L)
    res = []
    for i in range(count):
        e = []
        for j in range(2):
            off = L * (j + i * 2)
            e.append(int.from_bytes(data[off:off + L], "big") % P)
        res.append((e[0], e[1]))
    return res


SSWU_A = (0, 240)
SSWU_B = (1012, 1012)
SSWU_Z = ((-2) % P, (-1) % P)


def map_to_curve_sswu_g2(u):
    """RFC 9380 6.6.2 simplified SWU onto E2': y^2 = x^3 + A'x + B'."""
    A, B, Z = SSWU_A, SSWU_B, SSWU_Z
    u2 = f2_sqr(u)
    zu2 = f2_mul(Z, u2)
    tv1 = f2_add(f2_sqr(zu2), zu2)  # Z^2 u^4 + Z u^2
    if f2_is_zero(tv1):
        x1 = f2_mul(B, f2_inv(f2_mul(Z, A)))
    else:
        x1 = f2_mul(f2_mul(f2_neg(B), f2_inv(A)), f2_add(F2_ONE, f2_inv(tv1)))
    gx1 = f2_add(f2_add(f2_mul(f2_sqr(x1), x1), f2_mul(A, x1)), B)
    x2 = f2_mul(zu2, x1)
    gx2 = f2_add(f2_add(f2_mul(f2_sqr(x2), x2), f2_mul(A, x2)), B)
    if f2_is_square(gx1):
        x, y = x1, f2_sqrt(gx1)
    else:
        x, y = x2, f2_sqrt(gx2)
    if f2_sgn0(u) != f2_sgn0(y):
        y = f2_neg(y)
    return (x, y)


def _hx(s):
    return int(s, 16)


# RFC 9380 Appendix E.3: 3-isogeny E2' -> E2 (each constant is c0 + c1*I)
_K = P  # shorthand
ISO_XNUM = [
    (_hx("5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97d6"),
     _hx("5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97d6")),
    (0, _hx("11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71a")),
    (_hx("11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71e"),
     _hx("8ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38d")),
    (_hx("171d6541fa38ccfaed6dea691f5fb614cb14b4e7f4e810aa22d6108f142b85757098e38d0f671c7188e2aaaaaaaa5ed1"), 0),
]
ISO_XDEN = [
    (0, (-72) % P),
    (12, (-12) % P),
    (1, 0),
]
ISO_YNUM = [
    (_hx("1530477c7ab4113b59a4c18b076d11930f7da5d4a07f649bf54439d87d27e500fc8c25ebf8c92f6812cfc71c71c6d706"),
     _hx("1530477c7ab4113b59a4c18b076d11930f7da5d4a07f649bf54439d87d27e500fc8c25ebf8c92f6812cfc71c71c6d706")),
    (0, _hx("5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97be")),
    (_hx("11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71c"),
     _hx("8ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38f")),
    (_hx("124c9ad43b6cf79bfbf7043de3811ad0761b0f37a1e26286b0e977c69aa274524e79097a56dc4bd9e1b371c71c718b10"), 0),
]
ISO_YDEN = [
    ((-432) % P, (-432) % P),
    (0, (-216) % P),
    (18, (-18) % P),
    (1, 0),
]


def _poly_eval(coeffs, x):
    acc = F2_ZERO
    for c in reversed(coeffs):
        acc = f2_add(f2_mul(acc, x), c)
    return acc


def iso_map_g2(pt):
    x, y = pt
    xn = _poly_eval(ISO_XNUM, x)
    xd = _poly_eval(ISO_XDEN, x)
    yn = _poly_eval(ISO_YNUM, x)
    yd = _poly_eval(ISO_YDEN, x)
    if f2_is_zero(xd) or f2_is_zero(yd):
        return None
    return (f2_mul(xn, f2_inv(xd)), f2_mul(y, f2_mul(yn, f2_inv(yd))))


def clear_cofactor_g2(pt):
    """RFC 9380 G.3: h_eff * P via psi (Budroni-Pintore)."""
    t1 = g2_mul(pt, X)
    t2 = g2_psi(pt)
    t3 = g2_psi(g2_psi(g2_add(pt, pt)))
    t3 = g2_add(t3, g2_neg(t2))
    t2 = g2_add(t1, t2)
    t2 = g2_mul(t2, X)
    t3 = g2_add(t3, t2)
    t3 = g2_add(t3, g2_neg(t1))
    return g2_add(t3, g2_neg(pt))


def hash_to_g2(msg: bytes, dst: bytes = DST_POP):
    u0, u1 = hash_to_field_fp2(msg, 2, dst)
    q0 = iso_map_g2(map_to_curve_sswu_g2(u0))
    q1 = iso_map_g2(map_to_curve_sswu_g2(u1))
    return clear_cofactor_g2(g2_add(q0, q1))


# --------------------------------------------------------------------------------------------
# Pairing: optimal ate over |x|, lines from the twist E2'(Fp2) mapped into Fp12.
# untwist(x', y') = (x' w^-2, y' w^-3) since w^6 = xi.
# --------------------------------------------------------------------------------------------
def _line_value(lam, xT, yT, Pg1):
    """Line through T (on the twist) with twist-slope lam, evaluated at P in E(Fp):
       l = yP - lam' (xP - xT w^-2) - yT w^-3,  with lam' = lam * w^-1.
    Multiplying by w^3 (in Fp4 subfield, killed by the final exponentiation) gives
       l * w^3 = yP w^3 - lam xP w^2 + (lam xT - yT).
    """
    xP, yP = Pg1
    c0 = f2_sub(f2_mul(lam, xT), yT)  # w^0
    c2 = f2_muls(lam, (-xP) % P)     # w^2
    c3 = (yP % P, 0)                 # w^3
    l = f12_from_f2_at(c0, 0)
    l = _f12_add(l, f12_from_f2_at(c2, 2))
    l = _f12_add(l, f12_from_f2_at(c3, 3))
    return l


def _f12_add(a, b):
    return (f6_add(a[0], b[0]), f6_add(a[1], b[1]))


def miller_loop(Pg1, Qg2):
    """f_{|x|,Q}(P), conjugated because x < 0.  Returns F12_ONE if either input is infinity."""
    if Pg1 is None or Qg2 is None:
        return F12_ONE
    f = F12_ONE
    T = Qg2
    for bit in bin(X_ABS)[3:]:
        # doubling
        xT, yT = T
        lam = f2_mul(f2_muls(f2_sqr(xT), 3), f2_inv(f2_muls(yT, 2)))
        f = f12_mul(f12_sqr(f), _line_value(lam, xT, yT, Pg1))
        T = g2_add(T, T)
        if bit == "1":
            xT, yT = T
            xQ, yQ = Qg2
            lam = f2_mul(f2_sub(yQ, yT), f2_inv(f2_sub(xQ, xT)))
            f = f12_mul(f, _line_value(lam, xT, yT, Pg1))
            T = g2_add(T, Qg2)
    return f12_conj(f)


FE_HARD = (P ** 4 - P ** 2 + 1) // R


def final_exponentiation(f):
    """f^((p^12-1)/r): easy part by Frobenius, hard part by plain exponentiation (slow, exact)."""
    t = f12_mul(f12_conj(f), f12_inv(f))  # f^(p^6-1)
    t = f12_mul(f12_frob_n(t, 2), t)      # ^(p^2+1)
    return f12_pow(t, FE_HARD)


def pairing(Pg1, Qg2):
    return final_exponentiation(miller_loop(Pg1, Qg2))


def pairing_product_is_one(pairs):
    f = F12_ONE
    for Pg1, Qg2 in pairs:
        f = f12_mul(f, miller_loop(Pg1, Qg2))
    return final_exponentiation(f) == F12_ONE


# --------------------------------------------------------------------------------------------
# BLS signature scheme (IETF draft-04 POP ciphersuite, min-pubkey-size)
# --------------------------------------------------------------------------------------------
def _hkdf_extract(salt, ikm):
    return hmac.new(salt, ikm, hashlib.sha256).digest()


def _hkdf_expand(prk, info, length):
    out, t, i = b"", b"", 1
    while len(out) < length:
        t = hmac.new(prk, t + info + bytes([i]), hashlib.sha256).digest()
        out += t
        i += 1
    return out[:length]


def keygen(ikm: bytes, key_info: bytes = b"") -> int:
    """IETF BLS draft-04 KeyGen as implemented by blst_keygen (SecretKey.fromKeygen)."""
    assert len(ikm) >= 32
    salt = b"BLS-SIG-KEYGEN-SALT-"
    sk = 0
    while sk == 0:
        salt = hashlib.sha256(salt).digest()
        prk = _hkdf_extract(salt, ikm + b"\x00")
        okm = _hkdf_expand(prk, key_info + (48).to_bytes(2, "big"), 48)
        sk = int.from_bytes(okm, "big") % R
    return sk


def interop_secret_key(index: int) -> int:
    """state-transition/src/util/interop.ts:18-22 (bytesToBigInt / intToBytes are little-endian)."""
    d = hashlib.sha256(index.to_bytes(32, "little")).digest()
    return int.from_bytes(d, "little") % R


def sk_to_pk(sk: int):
    return g1_mul(G1_GEN, sk)


def sign(sk: int, msg: bytes):
    return g2_mul(hash_to_g2(msg), sk)


def core_verify(pk, msg: bytes, sig) -> bool:
    """blst verify(msg, pk, sig) after Signature.fromBytes(sig, true) succeeded."""
    if pk is None or sig is None:
        return False
    return pairing_product_is_one([(pk, hash_to_g2(msg)), (g1_neg(G1_GEN), sig)])


def aggregate_pubkeys(pks):
    """blst aggregatePublicKeys: throws on an empty list (EMPTY_AGGREGATE_ARRAY)."""
    if len(pks) == 0:
        raise ValueError("EMPTY_AGGREGATE_ARRAY")
    acc = None
    for pk in pks:
        acc = g1_add(acc, pk)
    return acc


def set_is_valid(pk, msg, sig_bytes) -> bool:
    """Truth for one (aggregate-pubkey, message, signature-bytes) set, per SURVEY Appendix A."""
    try:
        sig = signature_from_bytes(sig_bytes, True)
    except DecodeError:
        return False
    return core_verify(pk, msg, sig)


def verify_multiple_aggregate_signatures(sets, rng=None) -> bool:
    """blst randomised batch verification: prod e(r_i pk_i, H(m_i)) * e(-g1, sum r_i sig_i) == 1.
    sets: list of (pk_point, msg, sig_point).  64-bit non-zero random scalars."""
    rng = rng or _random.SystemRandom()
    pairs = []
    sig_acc = None
    for pk, msg, sig in sets:
        if pk is None:
            return False
        r = 0
        while r == 0:
            r = rng.getrandbits(64)
        pairs.append((g1_mul(pk, r), hash_to_g2(msg)))
        sig_acc = g2_add(sig_acc, g2_mul(sig, r))
    pairs.append((g1_neg(G1_GEN), sig_acc))
    return pairing_product_is_one(pairs)


def verify_signature_sets_maybe_batch(sets, rng=None) -> bool:
    """maybeBatch.ts:15-45.  sets: list of (pk_point, msg, sig_bytes).  Any throw -> False."""
    try:
        if len(sets) >= 2:
            return verify_multiple_aggregate_signatures(
                [(pk, m, signature_from_bytes(s, True)) for pk, m, s in sets], rng)
        if len(sets) == 0:
            raise ValueError("Empty signature set")
        return all(core_verify(pk, m, signature_from_bytes(s, True)) for pk, m, s in sets)
    except (DecodeError, ValueError):
        return False


def chunkify_maximize_chunk_size(arr, min_per_chunk):
    """multithread/utils.ts:4-18."""
    chunk_count = len(arr) // min_per_chunk
    if chunk_count <= 1:
        return [list(arr)]
    per_chunk = -(-len(arr) // chunk_count)
    return [list(arr[i:i + per_chunk]) for i in range(0, len(arr), per_chunk)]


MAX_SIGNATURE_SETS_PER_JOB = 128


def pool_verify_signature_sets(sets, table=None) -> bool:
    """BlsMultiThreadWorkerPool.verifySignatureSets (index.ts:157-207) booleans.

    sets: list of dicts {"pubkeys": [point,...] | "pubkey": point, "msg": bytes, "sig": bytes}.
    Raises ValueError (promise rejection) when an aggregate set has no pubkeys."""
    results = []
    for chunk in chunkify_maximize_chunk_size(sets, MAX_SIGNATURE_SETS_PER_JOB):
        ser = []
        for s in chunk:
            if "pubkeys" in s:
                pk = aggregate_pubkeys(s["pubkeys"])  # raises -> job rejects
            else:
                pk = s["pubkey"]
            # toBytes -> fromBytes round trip (worker.ts:111), no validation
            pk = g1_decompress(g1_compress(pk))
            ser.append((pk, s["msg"], s["sig"]))
        results.append(verify_signature_sets_maybe_batch(ser))
    return all(results)


def pool_verify_same_message(sets, msg) -> list:
    """verifySignatureSetsSameMessage (index.ts:212-236) + retry (jobItem.ts:93-125).

    sets: list of (pk_point, sig_bytes).  Returns list of booleans in input order."""
    out = []
    for chunk in chunkify_maximize_chunk_size(sets, MAX_SIGNATURE_SETS_PER_JOB):
        ok = False
        try:
            if len(chunk) == 0:
                raise ValueError("empty")
            rng = _random.SystemRandom()
            pk_acc, sig_acc = None, None
            for pk, sb in chunk:
                sig = signature_from_bytes(sb, True)
                r = 0
                while r == 0:
                    r = rng.getrandbits(64)
                pk_acc = g1_add(pk_acc, g1_mul(pk, r))
                sig_acc = g2_add(sig_acc, g2_mul(sig, r))
            ok = verify_signature_sets_maybe_batch(
                [(g1_decompress(g1_compress(pk_acc)), msg, g2_compress(sig_acc))])
        except (DecodeError, ValueError):
            ok = False
        if ok:
            out.extend([True] * len(chunk))
        else:
            out.extend(verify_signature_sets_maybe_batch([(pk, msg, sb)]) for pk, sb in chunk)
    return out


def single_thread_verify_same_message(sets, msg) -> list:
    """BlsSingleThreadVerifier.verifySignatureSetsSameMessage (singleThread.ts:36-80): the
    UNRANDOMIZED aggregate verify(msg, aggregatePublicKeys(pks), aggregateSignatures(sigs)); all
    true when it holds, else verify per set.  sets: list of (pk_point, sig_bytes).  Raises
    ValueError on an empty list (aggregatePublicKeys throws, :41)."""
    pk = aggregate_pubkeys([p for p, _ in sets])
    sigs, all_valid = [], True
    for _, sb in sets:                                   # :44-52, Signature.fromBytes(sig, true)
        try:
            sigs.append(signature_from_bytes(sb, True))
        except DecodeError:
            sigs.append(None)
            all_valid = False
    if all_valid:                                        # :54-57
        agg = None
        for sg in sigs:
            agg = g2_add(agg, sg)
        # blst verify: an infinite pubkey is rejected (PK_IS_INFINITY); an infinite aggregate
        # signature leaves e(pk, H(m)) != 1.  core_verify answers False for both.
        all_valid = core_verify(pk, msg, agg)
    if all_valid:
        return [True] * len(sets)
    return [sg is not None and core_verify(p, msg, sg) for (p, _), sg in zip(sets, sigs)]   # :62-71


def random_scalar(rng=None):
    rng = rng or _random.Random(0)
    return rng.randrange(1, R)
