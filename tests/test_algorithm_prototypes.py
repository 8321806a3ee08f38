"""Python prototypes of the formulas the HIP kernels use, checked against the oracle's definitions.

The device code (lodestar_amd/csrc/*.h) follows these prototypes step for step: homogeneous-projective
Miller loop with sparse (w^0, w^2, w^3) lines, the x-chain hard part of the final exponentiation
(3*(p^4-p^2+1)/r = (x-1)^2 (x+p) (x^2+p^2-1) + 3), the uniform-cost Fp2 square root, and the Jacobian
G1/G2 formulas.  CPU only.
"""
import random

from oracle import bls_oracle as o

P, R, X = o.P, o.R, o.X
B2P = (4, 4)  # b' = 4(1+i)


# ---- Fp2 square root with two Fp exponentiations and no data-dependent branch ----------------
def fp2_sqrt_uniform(a):
    a0, a1 = a
    n = (a0 * a0 + a1 * a1) % P
    alpha = pow(n, (P + 1) // 4, P)
    inv2 = (P + 1) // 2
    delta = (a0 + alpha) * inv2 % P
    if delta == 0:  # only when a1 == 0 and alpha == -a0
        delta = (a0 - alpha) * inv2 % P
    t = pow(delta, (P - 3) // 4, P)
    x0 = t * delta % P
    qr = (x0 * t) % P == 1
    if qr:
        root = (x0, a1 * t % P * inv2 % P)
    else:
        root = ((-a1) * t % P * inv2 % P, x0)
    ok = o.f2_sqr(root) == (a0 % P, a1 % P)
    return ok, root


def test_fp2_sqrt_uniform():
    rng = random.Random(3)
    for k in range(200):
        a = (rng.randrange(P), rng.randrange(P)) if k > 4 else [(0, 0), (4, 0), (P - 4, 0), (0, 9), (7, 0)][k]
        ok, root = fp2_sqrt_uniform(a)
        ref = o.f2_sqrt(a)
        assert ok == (ref is not None)
        if ok:
            assert root in (ref, o.f2_neg(ref))


# ---- Miller loop in homogeneous projective coordinates on the twist --------------------------
def f12_sparse(c0, c2, c3):
    """line = (c0 + c2 v) + (c3 v) w  -- coefficients at w^0, w^2, w^3."""
    return ((c0, c2, o.F2_ZERO), (o.F2_ZERO, c3, o.F2_ZERO))


def dbl_step(T, Pg1):
    X1, Y1, Z1 = T
    xP, yP = Pg1
    A = o.f2_muls(o.f2_mul(X1, Y1), (P + 1) // 2)
    B = o.f2_sqr(Y1)
    C = o.f2_sqr(Z1)
    E = o.f2_mul(C, o.f2_muls(B2P, 3))
    F = o.f2_muls(E, 3)
    X3 = o.f2_mul(A, o.f2_sub(B, F))
    G = o.f2_muls(o.f2_add(B, F), (P + 1) // 2)
    Y3 = o.f2_sub(o.f2_sqr(G), o.f2_muls(o.f2_sqr(E), 3))
    H = o.f2_sub(o.f2_sqr(o.f2_add(Y1, Z1)), o.f2_add(B, C))
    Z3 = o.f2_mul(B, H)
    X2 = o.f2_sqr(X1)
    line = f12_sparse(o.f2_sub(B, E), o.f2_muls(o.f2_muls(X2, 3), (-xP) % P), o.f2_muls(H, yP))
    return (X3, Y3, Z3), line


def add_step(T, Q, Pg1):
    X1, Y1, Z1 = T
    x2, y2 = Q
    xP, yP = Pg1
    theta = o.f2_sub(Y1, o.f2_mul(y2, Z1))
    lam = o.f2_sub(X1, o.f2_mul(x2, Z1))
    C = o.f2_sqr(theta)
    D = o.f2_sqr(lam)
    E = o.f2_mul(D, lam)
    F = o.f2_mul(Z1, C)
    G = o.f2_mul(X1, D)
    H = o.f2_sub(o.f2_add(E, F), o.f2_add(G, G))
    X3 = o.f2_mul(lam, H)
    Y3 = o.f2_sub(o.f2_mul(theta, o.f2_sub(G, H)), o.f2_mul(Y1, E))
    Z3 = o.f2_mul(Z1, E)
    line = f12_sparse(o.f2_sub(o.f2_mul(theta, x2), o.f2_mul(lam, y2)),
                      o.f2_muls(theta, (-xP) % P), o.f2_muls(lam, yP))
    return (X3, Y3, Z3), line


def miller_loop_proj(pairs):
    f = o.F12_ONE
    Ts = [(Q[0], Q[1], o.F2_ONE) for _, Q in pairs]
    for bit in bin(o.X_ABS)[3:]:
        f = o.f12_sqr(f)
        for j, (Pg1, Q) in enumerate(pairs):
            Ts[j], l = dbl_step(Ts[j], Pg1)
            f = o.f12_mul(f, l)
        if bit == "1":
            for j, (Pg1, Q) in enumerate(pairs):
                Ts[j], l = add_step(Ts[j], Q, Pg1)
                f = o.f12_mul(f, l)
    return o.f12_conj(f)


def final_exp_chain(f):
    """Returns f^(3 (p^12-1)/r) using the x-chain for the hard part."""
    t = o.f12_mul(o.f12_conj(f), o.f12_inv(f))
    t = o.f12_mul(o.f12_frob_n(t, 2), t)

    def exp_x(a):  # a^x, x < 0, a cyclotomic
        return o.f12_conj(o.f12_pow(a, o.X_ABS))

    a = o.f12_mul(exp_x(t), o.f12_conj(t))       # t^(x-1)
    a = o.f12_mul(exp_x(a), o.f12_conj(a))       # t^((x-1)^2)
    b = o.f12_mul(exp_x(a), o.f12_frob(a))       # a^(x+p)
    c = o.f12_mul(o.f12_mul(exp_x(exp_x(b)), o.f12_frob_n(b, 2)), o.f12_conj(b))  # b^(x^2+p^2-1)
    t3 = o.f12_mul(o.f12_sqr(t), t)
    return o.f12_mul(c, t3)


def test_hard_part_identity():
    lam = (P ** 4 - P ** 2 + 1) // R
    assert 3 * lam == (X - 1) ** 2 * (X + P) * (X * X + P * P - 1) + 3


def test_projective_miller_and_chain_match_oracle():
    Pg = o.g1_mul(o.G1_GEN, 7)
    Qg = o.g2_mul(o.G2_GEN, 11)
    f_ref = o.miller_loop(Pg, Qg)
    f_new = miller_loop_proj([(Pg, Qg)])
    e_ref = o.final_exponentiation(f_ref)
    assert o.final_exponentiation(f_new) == e_ref
    assert final_exp_chain(f_new) == o.f12_pow(e_ref, 3)
    # two-pair product == 1 for a valid signature relation
    sk = 99
    Hm = o.hash_to_g2(b"abc")
    sig = o.g2_mul(Hm, sk)
    pk = o.g1_mul(o.G1_GEN, sk)
    f2 = miller_loop_proj([(pk, Hm), (o.g1_neg(o.G1_GEN), sig)])
    assert final_exp_chain(f2) == o.F12_ONE


# ---- Jacobian formulas (a = 0) ---------------------------------------------------------------
def jac_dbl(F, Pj):
    X1, Y1, Z1 = Pj
    A = F.sqr(X1); B = F.sqr(Y1); C = F.sqr(B)
    D = F.muls(F.sub(F.sub(F.sqr(F.add(X1, B)), A), C), 2)
    E = F.muls(A, 3); Fv = F.sqr(E)
    X3 = F.sub(Fv, F.muls(D, 2))
    Y3 = F.sub(F.mul(E, F.sub(D, X3)), F.muls(C, 8))
    Z3 = F.muls(F.mul(Y1, Z1), 2)
    return (X3, Y3, Z3)


def jac_madd(F, Pj, Q):
    X1, Y1, Z1 = Pj
    x2, y2 = Q
    Z1Z1 = F.sqr(Z1)
    U2 = F.mul(x2, Z1Z1)
    S2 = F.mul(y2, F.mul(Z1, Z1Z1))
    H = F.sub(U2, X1)
    HH = F.sqr(H)
    I = F.muls(HH, 4)
    J = F.mul(H, I)
    r = F.muls(F.sub(S2, Y1), 2)
    V = F.mul(X1, I)
    X3 = F.sub(F.sub(F.sqr(r), J), F.muls(V, 2))
    Y3 = F.sub(F.mul(r, F.sub(V, X3)), F.muls(F.mul(Y1, J), 2))
    Z3 = F.sub(F.sub(F.sqr(F.add(Z1, H)), Z1Z1), HH)
    return (X3, Y3, Z3)


def jac_to_aff(F, Pj):
    X1, Y1, Z1 = Pj
    zi = F.inv(Z1)
    zi2 = F.sqr(zi)
    return (F.mul(X1, zi2), F.mul(Y1, F.mul(zi2, zi)))


def test_jacobian_formulas():
    for F, G, mul in ((o._Fp, o.G1_GEN, o.g1_mul), (o._Fp2, o.G2_GEN, o.g2_mul)):
        Pa = mul(G, 5)
        Pj = (Pa[0], Pa[1], F.one)
        assert jac_to_aff(F, jac_dbl(F, Pj)) == mul(G, 10)
        assert jac_to_aff(F, jac_madd(F, jac_dbl(F, Pj), G)) == mul(G, 11)


# ---- bucket MSM of the same-message segment (lodestar_amd/csrc/k_msm.hip) ----------------------
def scalar_half_mag(s):
    """curve.h scalar_half_mag: a = 2 s - (2^32 - 1) as (|a|, a < 0)."""
    a = 2 * s - (2 ** 32 - 1)
    return abs(a), a < 0


def msm_bucket_prototype(points, r64s, lam, q, c=16, windows=2, slice_=16):
    """k_msm.hip over the group Z_q (a point is its discrete log, E(P) = lam P): entries by
    (window, digit), bucket sums, slice running sums + d0 * T, window weights 2^(c w)."""
    buckets = {}
    for t, (p, r) in enumerate(zip(points, r64s)):
        for h, s in enumerate((r & 0xFFFFFFFF, r >> 32)):
            mag, neg = scalar_half_mag(s)
            pt = p * lam % q if h else p
            if neg:
                pt = -pt % q
            for w in range(windows):
                d = (mag >> (c * w)) & ((1 << c) - 1)
                if d:
                    buckets[(w, d)] = (buckets.get((w, d), 0) + pt) % q
    total = 0
    for w in range(windows):
        for d0 in range(0, 1 << c, slice_):
            T = A = 0
            for qq in range(slice_ - 1, 0, -1):
                T = (T + buckets.get((w, d0 + qq), 0)) % q
                A = (A + T) % q
            T = (T + buckets.get((w, d0), 0)) % q
            M = 0
            for k in range(c - 1, -1, -1):  # double-and-add over the bits of d0
                M = 2 * M % q
                if (d0 >> k) & 1:
                    M = (M + T) % q
            total = (total + (A + M) * pow(2, c * w, q)) % q
    return total


def test_msm_bucket_prototype_matches_randomised_sum():
    """The MSM's sum equals sum_i r_i P_i with r_i = a_i - b_i x^2 (the scalar randomize_pair applies),
    i.e. the same G2 sum the per-set ladders would form, so the segment check is unchanged."""
    rng = random.Random(7)
    lam = (-X * X) % R  # eigenvalue of E = -psi^2 on G2 (and phi on G1)
    pts = [rng.randrange(1, R) for _ in range(300)]
    rs = [rng.getrandbits(64) | 1 for _ in range(300)]
    rs[:4] = [1, 2 ** 64 - 1, 2 ** 63, 0x0001000000010000]  # extreme halves and zero digits
    want = 0
    for p, r in zip(pts, rs):
        a = 2 * (r & 0xFFFFFFFF) - (2 ** 32 - 1)
        b = 2 * (r >> 32) - (2 ** 32 - 1)
        want = (want + (a - b * X * X) * p) % R
    assert msm_bucket_prototype(pts, rs, lam, R) == want
