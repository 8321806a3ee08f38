"""The wave-cooperative programs (tools/gen_coop.py -> lodestar_amd/csrc/coop_tables.h), executed
in Python exactly as coop.h executes them (same rounds, same term lists, integers mod p), against
the oracle's Fp12 / G2 / pairing arithmetic.  CPU only.

The drivers below (miller_loop / final_exp) are the specification of the device drivers in
lodestar_amd/csrc/coop.h: same program sequence, same operand layout.
"""
import os
import random
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)

import gen_coop  # noqa: E402
from oracle import bls_oracle as O  # noqa: E402

P = O.P
PROGS, CONSTS = gen_coop.build_all()
BY_NAME = {p["name"]: p for p in PROGS}


def run(name, *operands):
    """Run program `name`; operands are lists of ints (inputs) or None (outputs). Returns outputs."""
    p = BY_NAME[name]
    ops = [list(o) if o is not None else [0] * p["signature"][i][1] for i, o in enumerate(operands)]
    Z = [0] * p["nz"]
    terms = p["terms"]

    def lin(t0, tn):
        acc = 0
        for src, idx, c in terms[t0:t0 + tn]:
            v = Z[idx] if src == gen_coop.SRC_Z else CONSTS[idx] if src == gen_coop.SRC_C else ops[src][idx]
            acc += c * v
        return acc % P

    for k, (a0, an, b0, bn) in enumerate(p["prods"]):
        Z[k] = lin(a0, an) * lin(b0, bn) % P
    for t0, tn, z in p["parts"]:
        Z[z] = lin(t0, tn)
    vals = [(op, i, lin(t0, tn)) for (t0, tn, op, i) in p["outs"]]
    for op, i, v in vals:  # outputs land after every output was computed (in-place safe)
        ops[op][i] = v
    return ops


def flat12(a):
    return [c for six in a for two in six for c in two]


def unflat12(v):
    f2 = [(v[2 * k], v[2 * k + 1]) for k in range(6)]
    return ((f2[0], f2[1], f2[2]), (f2[3], f2[4], f2[5]))


def rnd12(rng):
    return unflat12([rng.randrange(P) for _ in range(12)])


def cyclotomic(rng):
    f = rnd12(rng)
    t = O.f12_mul(O.f12_conj(f), O.f12_inv(f))
    return O.f12_mul(O.f12_frob_n(t, 2), t)


@pytest.fixture
def rng():
    return random.Random(1234)


def test_fp12_mul(rng):
    for _ in range(3):
        a, b = rnd12(rng), rnd12(rng)
        assert unflat12(run("FP12_MUL", flat12(a), flat12(b), None)[2]) == O.f12_mul(a, b)


def test_fp12_mul_in_place(rng):
    a, b = rnd12(rng), rnd12(rng)
    p = BY_NAME["FP12_MUL"]
    ops = [flat12(a), flat12(b)]
    Z = [0] * len(p["prods"])
    # aliasing out == a is what the drivers do; run() already writes outputs last
    out = run("FP12_MUL", ops[0], ops[1], None)[2]
    assert unflat12(out) == O.f12_mul(a, b) and len(Z) == 54


def test_fp12_sqr(rng):
    a = rnd12(rng)
    assert unflat12(run("FP12_SQR", flat12(a), None)[1]) == O.f12_sqr(a)


def test_cyclotomic_sqr(rng):
    for _ in range(2):
        g = cyclotomic(rng)
        assert unflat12(run("FP12_CYC_SQR", flat12(g), None)[1]) == O.f12_sqr(g)


def line_fp12(l):
    c0, c2, c3 = (l[0], l[1]), (l[2], l[3]), (l[4], l[5])
    x = O.f12_from_f2_at(c0, 0)
    x = O._f12_add(x, O.f12_from_f2_at(c2, 2))
    return O._f12_add(x, O.f12_from_f2_at(c3, 3))


def test_mul_line(rng):
    f = rnd12(rng)
    l = [rng.randrange(P) for _ in range(6)]
    assert unflat12(run("FP12_MUL_LINE", flat12(f), l, None)[2]) == O.f12_mul(f, line_fp12(l))


@pytest.mark.parametrize("n", [1, 2])
def test_frobenius(rng, n):
    a = rnd12(rng)
    assert unflat12(run("FP12_FROB%d" % n, flat12(a), None)[1]) == O.f12_frob_n(a, n)


def proj_to_aff(t):
    x, y, z = (t[0], t[1]), (t[2], t[3]), (t[4], t[5])
    zi = O.f2_inv(z)
    return (O.f2_mul(x, zi), O.f2_mul(y, zi))


def test_dbl_and_add_steps():
    Q = O.g2_mul(O.G2_GEN, 12345)
    T = [Q[0][0], Q[0][1], Q[1][0], Q[1][1], 1, 0]
    Pp = [(-O.G1_GEN[0]) % P, O.G1_GEN[1]]
    ops = run("G2_DBL_STEP", T, Pp, None, None)
    assert proj_to_aff(ops[2]) == O.g2_add(Q, Q)
    T2 = ops[2]
    # the line-free doubling (cofactor clearing's [|x|] chains) gives the same projective point
    assert run("G2_DBL_PT", T, None)[1] == T2
    # the fused Miller-bit program: the Fp12 square and the same doubling step and line
    f = flat12(O.f12_mul(O.F12_ONE, unflat12([(7 * k + 3) % P for k in range(12)])))
    fused = run("MILLER_SQR_DBL", f, T, Pp, None, None, None)
    assert fused[3] == flat12(O.f12_mul(unflat12(f), unflat12(f)))
    assert fused[4] == T2 and fused[5] == run("G2_DBL_STEP", T, Pp, None, None)[3]
    ops = run("G2_ADD_STEP", T2, [Q[0][0], Q[0][1], Q[1][0], Q[1][1]], Pp, None, None)
    assert proj_to_aff(ops[3]) == O.g2_mul(Q, 3)


# ---- reference drivers (coop.h does exactly this) ------------------------------------------------
def miller_loop(pairs):
    """prod_j f_{|x|,Q_j}(P_j), conjugated; pairs of (P affine G1, Q affine G2)."""
    F = flat12(O.F12_ONE)
    st = []
    for Pg, Qg in pairs:
        st.append(([Qg[0][0], Qg[0][1], Qg[1][0], Qg[1][1], 1, 0], [Qg[0][0], Qg[0][1], Qg[1][0], Qg[1][1]],
                   [(-Pg[0]) % P, Pg[1] % P]))
    bits = bin(O.X_ABS)[3:]
    first = True
    for bit in bits:
        nst = []
        for j, (T, Q, Pp) in enumerate(st):
            if j == 0 and not first:  # the square of f fused with pair 0's doubling step
                ops = run("MILLER_SQR_DBL", F, T, Pp, None, None, None)
                F, T, L = ops[3], ops[4], ops[5]
            else:
                ops = run("G2_DBL_STEP", T, Pp, None, None)
                T, L = ops[2], ops[3]
            F = run("FP12_MUL_LINE", F, L, None)[2]
            nst.append([T, Q, Pp])
        first = False
        st = nst
        if bit == "1":
            for s in st:
                ops = run("G2_ADD_STEP", s[0], s[1], s[2], None, None)
                s[0] = ops[3]
                F = run("FP12_MUL_LINE", F, ops[4], None)[2]
    return O.f12_conj(unflat12(F))


def exp_x(a):
    """a^x for a in the cyclotomic subgroup (x < 0: conjugate)."""
    r = list(a)
    for bit in bin(O.X_ABS)[3:]:
        r = run("FP12_CYC_SQR", r, None)[1]
        if bit == "1":
            r = run("FP12_MUL", r, a, None)[2]
    return flat12(O.f12_conj(unflat12(r)))


def mul(a, b):
    return run("FP12_MUL", a, b, None)[2]


def conj(a):
    return flat12(O.f12_conj(unflat12(a)))


def frob(a, n):
    return run("FP12_FROB%d" % n, a, None)[1]


def final_exp(f):
    """f^(3 (p^12-1)/r), the x-chain of fp12.h final_exponentiation."""
    f = flat12(f)
    inv = flat12(O.f12_inv(unflat12(f)))  # lane-0 scalar inverse on the device
    t = mul(conj(f), inv)
    t = mul(frob(t, 2), t)
    a = mul(exp_x(t), conj(t))
    a = mul(exp_x(a), conj(a))
    b = mul(exp_x(a), frob(a, 1))
    c = mul(exp_x(exp_x(b)), frob(b, 2))
    c = mul(c, conj(b))
    t3 = mul(run("FP12_CYC_SQR", t, None)[1], t)
    return unflat12(mul(c, t3))


def test_pairing_matches_oracle():
    Pg = O.g1_mul(O.G1_GEN, 777)
    Qg = O.g2_mul(O.G2_GEN, 999)
    want = O.f12_pow(O.pairing(Pg, Qg), 3)
    assert final_exp(miller_loop([(Pg, Qg)])) == want


def test_two_pair_check():
    sk = 0x1234567
    msg = b"coop"
    H = O.hash_to_g2(msg)
    pk, sig = O.sk_to_pk(sk), O.sign(sk, msg)
    f = miller_loop([(pk, H), (O.g1_neg(O.G1_GEN), sig)])
    assert final_exp(f) == O.F12_ONE
    f = miller_loop([(pk, O.hash_to_g2(b"other")), (O.g1_neg(O.G1_GEN), sig)])
    assert final_exp(f) != O.F12_ONE
