"""Generate lodestar_amd/csrc/coop_tables.h: wave-cooperative Fp12 / G2-line programs.

Why: a pairing is a long chain of DEPENDENT Fp12 operations.  Run by one thread it is
latency-bound (~3 us per Fp product on gfx950 at one wave per SIMD, so ~25 ms per pairing
check).  Every such operation is, however, a bilinear (or quadratic) map over Fp whose
Karatsuba form needs 18-54 INDEPENDENT Fp products.  A "program" here is that form, written
out: rounds of Fp products, each product's two operands a signed small-integer linear
combination of operand coordinates / earlier products / constants, then output coordinates as
linear combinations.  One wave runs a program with one lane per product (coop.h), so an Fp12
multiplication costs about one Fp product of latency instead of 54.

The formulas are the same ones lodestar_amd/csrc/fp12.h and pairing.h use per thread (Karatsuba
Fp2/Fp6/Fp12, Granger-Scott cyclotomic squaring, sparse line multiplication, homogeneous
projective doubling/addition steps with line coefficients, Frobenius), executed symbolically.
tests/test_coop_tables.py re-executes every program in Python against the oracle.

Round 4 wrote the hottest of these out as fixed code in coop.h (cyc_sqr, mul_line, sqr_dbl, mul12:
lane terms resolved once, no records, no partial-sum phase); FP12_CYC_SQR, FP12_MUL_LINE,
MILLER_SQR_DBL, G2_DBL_STEP, G2_DBL_PT and FP12_MUL stay here as the specification of the same maps
(the written-out forms follow dbl_step_into's scaling exactly) and are not emitted.  The device
still interprets the Frobenius maps and G2_ADD_STEP: only those go into coop_tables.h
(DEVICE_PROGRAMS).

Program encoding (all indices small; emitted as fixed-size per-lane u32 records -- a product is a
header (term counts) + up to 10 A terms + up to 10 B terms, a partial sum / output a header + up to
7 terms; within a linear form the coefficient +1 terms come first, then the -1 terms (the sign of a
unit term is its position and the device reads the value or its stored negation), then the rare
scaled terms (|coefficient| > 1, sign in bit 4 of the term word) -- a lane fetches its whole record
with a few 16-byte loads, one memory latency per phase, evaluates the unit terms in an unrolled
chain and the scaled ones in a short rolled loop, i.e. only its true number of terms):
  operands 0..5 -> base pointers given at run time (program-specific signature below)
  SRC_Z = 6  -> Z[k], the k-th product of this program (then the partial sums)
  SRC_C = 7  -> CONSTS[k] (Montgomery Fp constants emitted below)
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
SRC_Z, SRC_C = 6, 7
PART_TERMS = 6
OUT_MAX = 7  # longer outputs are split into partial sums of PART_TERMS (short add chains per phase)
OPW = 10  # terms per product operand record (A: 0..9, B: 10..19); 20 x 4 B = five 16-byte loads


# ---- symbolic Fp: linear forms over symbols ----------------------------------------------------
class Lin:
    __slots__ = ("d",)

    def __init__(self, d=None):
        self.d = {k: v for k, v in (d or {}).items() if v}

    def __add__(self, o):
        d = dict(self.d)
        for k, v in o.d.items():
            d[k] = d.get(k, 0) + v
        return Lin(d)

    def __sub__(self, o):
        return self + o.scale(-1)

    def __neg__(self):
        return self.scale(-1)

    def scale(self, k):
        return Lin({s: v * k for s, v in self.d.items()})


def inp(op, i):
    return Lin({("in", op, i): 1})


class Const:
    """Constant pool (plain integers mod p)."""

    def __init__(self):
        self.vals = []
        self.index = {}

    def get(self, v):
        v %= P
        if v not in self.index:
            self.index[v] = len(self.vals)
            self.vals.append(v)
        return Lin({("c", self.index[v]): 1})


CONSTS = Const()
CONSTS.get(0)
ZERO_IDX = CONSTS.index[0]  # the constant 0 (registered first): padding of the records


class Builder:
    def __init__(self, name, signature):
        self.name = name
        self.signature = signature  # list of (operand name, n coords, role)
        self.prods = []  # (Lin, Lin)
        self.outs = []   # (dst operand, coord, Lin)
        self.xparts = []  # explicit partial sums (Lin over products / inputs / constants)
        self.out_max = OUT_MAX  # outputs longer than this are split into partial sums

    def part(self, lin):
        """An explicit partial sum: one lane of the partial-sum phase computes it into Z, so an
        output can use it several times (3 t - 2 z as t + t + t - z - z: unit terms only)."""
        self.xparts.append(lin)
        return Lin({("p", len(self.xparts) - 1): 1})

    def mul(self, a, b):
        self.prods.append((a, b))
        return Lin({("z", len(self.prods) - 1): 1})

    # Fp2 = (Lin, Lin) ---------------------------------------------------------------------------
    def f2mul(self, a, b):
        t0 = self.mul(a[0], b[0])
        t1 = self.mul(a[1], b[1])
        t2 = self.mul(a[0] + a[1], b[0] + b[1])
        return (t0 - t1, t2 - t0 - t1)

    def f2sqr(self, a):
        t0 = self.mul(a[0] + a[1], a[0] - a[1])
        t1 = self.mul(a[0], a[1])
        return (t0, t1.scale(2))

    def f2mulfp(self, a, s):
        return (self.mul(a[0], s), self.mul(a[1], s))

    def f2mulc(self, a, c):  # c: plain (c0, c1) constant
        c0, c1 = c[0] % P, c[1] % P
        if c1 == 0:
            return (self.mul(a[0], CONSTS.get(c0)), self.mul(a[1], CONSTS.get(c0)))
        if c0 == 0:  # (a0 + a1 i) (c1 i) = -a1 c1 + a0 c1 i
            return (-self.mul(a[1], CONSTS.get(c1)), self.mul(a[0], CONSTS.get(c1)))
        return self.f2mul(a, (CONSTS.get(c0), CONSTS.get(c1)))

    # Fp6 = 3 x Fp2, Fp12 = 2 x Fp6 (fp12.h formulas) --------------------------------------------
    def f6mul(self, a, b):
        t0 = self.f2mul(a[0], b[0])
        t1 = self.f2mul(a[1], b[1])
        t2 = self.f2mul(a[2], b[2])
        c0 = f2add(t0, f2xi(f2sub(f2sub(self.f2mul(f2add(a[1], a[2]), f2add(b[1], b[2])), t1), t2)))
        c1 = f2add(f2sub(f2sub(self.f2mul(f2add(a[0], a[1]), f2add(b[0], b[1])), t0), t1), f2xi(t2))
        c2 = f2add(f2sub(f2sub(self.f2mul(f2add(a[0], a[2]), f2add(b[0], b[2])), t0), t2), t1)
        return (c0, c1, c2)

    def f12mul(self, a, b):
        t0 = self.f6mul(a[0], b[0])
        t1 = self.f6mul(a[1], b[1])
        c1 = f6sub(f6sub(self.f6mul(f6add(a[0], a[1]), f6add(b[0], b[1])), t0), t1)
        return (f6add(t0, f6mulv(t1)), c1)

    def f12sqr(self, a):
        t = self.f6mul(a[0], a[1])
        c0 = f6sub(f6sub(self.f6mul(f6add(a[0], a[1]), f6add(a[0], f6mulv(a[1]))), t), f6mulv(t))
        return (c0, f6add(t, t))

    def f6mul_by_01(self, f, a, b):
        t0 = self.f2mul(f[0], a)
        t1 = self.f2mul(f[1], b)
        c1 = f2sub(f2sub(self.f2mul(f2add(f[0], f[1]), f2add(a, b)), t0), t1)
        c0 = f2add(t0, f2xi(self.f2mul(f[2], b)))
        c2 = f2add(t1, self.f2mul(f[2], a))
        return (c0, c1, c2)

    def f6mul_by_1(self, f, c):
        return (f2xi(self.f2mul(f[2], c)), self.f2mul(f[0], c), self.f2mul(f[1], c))

    def f12mul_line(self, f, c0, c2, c3):
        a = self.f6mul_by_01(f[0], c0, c2)
        b = self.f6mul_by_1(f[1], c3)
        e = self.f6mul_by_01(f6add(f[0], f[1]), c0, f2add(c2, c3))
        return (f6add(a, f6mulv(b)), f6sub(f6sub(e, a), b))

    def f12cyc_sqr(self, a):
        # Granger-Scott: three Fp4 squarings over Fp2[y]/(y^2 - xi), y = w^3
        z0, z4, z3 = a[0]
        z2, z1, z5 = a[1]

        def fp4_sqr(x, y):
            tmp = self.f2mul(x, y)
            t0 = f2sub(f2sub(self.f2mul(f2add(x, y), f2add(f2xi(y), x)), tmp), f2xi(tmp))
            return t0, f2add(tmp, tmp)

        t0, t1 = fp4_sqr(z0, z1)
        t2, t3 = fp4_sqr(z2, z3)
        t4, t5 = fp4_sqr(z4, z5)
        # the t's become partial sums, so each output 3 t +- 2 z is five unit terms
        t0, t1, t2, t3, t4 = [(self.part(t[0]), self.part(t[1])) for t in (t0, t1, t2, t3, t4)]
        t5x = f2xi(t5)
        t5x = (self.part(t5x[0]), self.part(t5x[1]))
        n0 = f2sub(f2scale(t0, 3), f2scale(z0, 2))
        n1 = f2add(f2scale(t1, 3), f2scale(z1, 2))
        n2 = f2add(f2scale(t5x, 3), f2scale(z2, 2))
        n3 = f2sub(f2scale(t4, 3), f2scale(z3, 2))
        n4 = f2sub(f2scale(t2, 3), f2scale(z4, 2))
        n5 = f2add(f2scale(t3, 3), f2scale(z5, 2))
        return ((n0, n4, n3), (n2, n1, n5))

    def f12cyc_sqr3(self, a):
        """The same squaring with no partial-sum phase: the 3 of every 3 t +- 2 z is carried by one
        operand of each base product (unit copies: the round has lanes to spare), so each output is
        a signed sum of <= 9 product terms and two copies of z -- one output phase of <= 11 terms."""
        z0, z4, z3 = a[0]
        z2, z1, z5 = a[1]

        def weight(lin):
            return sum(abs(c) for c in lin.d.values())

        def mul3(p, q):
            return self.mul(p.scale(3), q) if weight(p) <= weight(q) else self.mul(p, q.scale(3))

        def f2mul3(x, y):  # 3 x y
            t0 = mul3(x[0], y[0])
            t1 = mul3(x[1], y[1])
            t2 = mul3(x[0] + x[1], y[0] + y[1])
            return (t0 - t1, t2 - t0 - t1)

        def fp4_sqr3(x, y):  # 3 (t0, t1) of fp4_sqr
            tmp = f2mul3(x, y)
            t0 = f2sub(f2sub(f2mul3(f2add(x, y), f2add(f2xi(y), x)), tmp), f2xi(tmp))
            return t0, f2add(tmp, tmp)

        t0, t1 = fp4_sqr3(z0, z1)
        t2, t3 = fp4_sqr3(z2, z3)
        t4, t5 = fp4_sqr3(z4, z5)
        t5x = f2xi(t5)
        n0 = f2sub(t0, f2scale(z0, 2))
        n1 = f2add(t1, f2scale(z1, 2))
        n2 = f2add(t5x, f2scale(z2, 2))
        n3 = f2sub(t4, f2scale(z3, 2))
        n4 = f2sub(t2, f2scale(z4, 2))
        n5 = f2add(t3, f2scale(z5, 2))
        return ((n0, n4, n3), (n2, n1, n5))

    def out_vec(self, op, lins):
        for i, l in enumerate(lins):
            self.outs.append((op, i, l))


def f2add(a, b):
    return (a[0] + b[0], a[1] + b[1])


def f2sub(a, b):
    return (a[0] - b[0], a[1] - b[1])


def f2neg(a):
    return (-a[0], -a[1])


def f2conj(a):
    return (a[0], -a[1])


def f2xi(a):
    return (a[0] - a[1], a[0] + a[1])


def f2scale(a, k):
    return (a[0].scale(k), a[1].scale(k))


def f6add(a, b):
    return tuple(f2add(x, y) for x, y in zip(a, b))


def f6sub(a, b):
    return tuple(f2sub(x, y) for x, y in zip(a, b))


def f6mulv(a):
    return (f2xi(a[2]), a[0], a[1])


def fp12_in(op):
    c = [inp(op, i) for i in range(12)]
    f2 = [(c[2 * k], c[2 * k + 1]) for k in range(6)]
    return ((f2[0], f2[1], f2[2]), (f2[3], f2[4], f2[5]))


def fp12_flat(a):
    out = []
    for six in a:
        for two in six:
            out += [two[0], two[1]]
    return out


def fp2_in(op, k):
    return (inp(op, 2 * k), inp(op, 2 * k + 1))


# ---- programs ----------------------------------------------------------------------------------
def prog_fp12_mul():
    b = Builder("FP12_MUL", [("a", 12, "in"), ("b", 12, "in"), ("c", 12, "out")])
    b.out_vec(2, fp12_flat(b.f12mul(fp12_in(0), fp12_in(1))))
    return b


def prog_fp12_sqr():
    b = Builder("FP12_SQR", [("a", 12, "in"), ("c", 12, "out")])
    b.out_vec(1, fp12_flat(b.f12sqr(fp12_in(0))))
    return b


CYC_DIRECT = int(os.environ.get("GBV_GEN_CYC_DIRECT", "0"))  # 1: no partial-sum phase (measured: no faster)


def prog_cyc_sqr():
    b = Builder("FP12_CYC_SQR", [("a", 12, "in"), ("c", 12, "out")])
    if CYC_DIRECT:
        b.out_max = SUM_TERMS
        b.out_vec(1, fp12_flat(b.f12cyc_sqr3(fp12_in(0))))
    else:
        b.out_vec(1, fp12_flat(b.f12cyc_sqr(fp12_in(0))))
    return b


def prog_mul_line():
    # line operand: 6 coords = c0 (Fp2), c2 (Fp2), c3 (Fp2)
    b = Builder("FP12_MUL_LINE", [("f", 12, "in"), ("l", 6, "in"), ("c", 12, "out")])
    b.out_vec(2, fp12_flat(b.f12mul_line(fp12_in(0), fp2_in(1, 0), fp2_in(1, 1), fp2_in(1, 2))))
    return b


def prog_frob(n):
    from oracle import bls_oracle as O
    b = Builder("FP12_FROB%d" % n, [("a", 12, "in"), ("c", 12, "out")])
    a = fp12_in(0)
    coeffs = [a[0][0], a[0][1], a[0][2], a[1][0], a[1][1], a[1][2]]
    out = []
    for k in range(6):
        e = [O.F2_ZERO] * 6
        e[k] = O.F2_ONE
        img = O.f12_frob_n(((e[0], e[1], e[2]), (e[3], e[4], e[5])), n)
        g = (img[0] + img[1])[k]
        x = coeffs[k] if n % 2 == 0 else f2conj(coeffs[k])
        out.append(b.f2mulc(x, g) if g != (1, 0) else x)
    b.out_vec(1, fp12_flat(((out[0], out[1], out[2]), (out[3], out[4], out[5]))))
    return b


def dbl_step_into(b, t_op, p_op, t_out, l_out):
    """The doubling step T -> 4 [2]T (homogeneous) with its line through P = (-xP, yP), emitted into
    builder b with the given operand indices."""
    X, Y, Z = fp2_in(t_op, 0), fp2_in(t_op, 1), fp2_in(t_op, 2)
    nxp, yp = inp(p_op, 0), inp(p_op, 1)
    A = b.f2mul(X, Y)           # XY (the 1/2 of the unscaled formula is folded into the x4 scaling)
    B = b.f2sqr(Y)
    C = b.f2sqr(Z)
    X2 = b.f2sqr(X)
    YZ2 = b.f2sqr(f2add(Y, Z))
    E = f2scale(f2xi(C), 12)    # C * 3b', b' = 4(1 + i)
    F = f2scale(E, 3)
    H = f2sub(YZ2, f2add(B, C))
    X3 = f2scale(b.f2mul(A, f2sub(B, F)), 2)
    Y3 = f2sub(b.f2sqr(f2add(B, F)), f2scale(b.f2sqr(E), 12))
    Z3 = f2scale(b.f2mul(B, H), 4)
    l0 = f2sub(B, E)
    l2 = b.f2mulfp(f2scale(X2, 3), nxp)
    l3 = b.f2mulfp(H, yp)
    b.out_vec(t_out, [X3[0], X3[1], Y3[0], Y3[1], Z3[0], Z3[1]])
    b.out_vec(l_out, [l0[0], l0[1], l2[0], l2[1], l3[0], l3[1]])


def prog_dbl_step():
    # T (6: x, y, z in Fp2), P (2: -xP, yP)  ->  T' = 4 * [2]T (homogeneous), line (6: c0, c2, c3)
    b = Builder("G2_DBL_STEP", [("t", 6, "in"), ("p", 2, "in"), ("t_out", 6, "out"), ("l", 6, "out")])
    dbl_step_into(b, 0, 1, 2, 3)
    return b


def prog_sqr_dbl():
    # One Miller-loop bit's independent halves in ONE program: f^2 (the 36 products of the Fp12
    # square) and the doubling step of T with its line (11 + 14 products), so the square's products
    # and the doubling's first round share a round (47 lanes) -- one program, its phases and barriers,
    # per bit fewer.  f (12), T (6), P (2) -> f^2 (12), T' (6), line (6); f^2 may overwrite f.
    b = Builder("MILLER_SQR_DBL", [("f", 12, "in"), ("t", 6, "in"), ("p", 2, "in"), ("f_out", 12, "out"),
                                   ("t_out", 6, "out"), ("l", 6, "out")])
    b.out_vec(3, fp12_flat(b.f12sqr(fp12_in(0))))
    dbl_step_into(b, 1, 2, 4, 5)
    return b


def prog_dbl_pt():
    # T (6) -> T' = 4 * [2]T (homogeneous): the doubling step without its line (cofactor clearing and
    # other plain [|x|] multiplications): 19 products in two rounds, 6 outputs
    b = Builder("G2_DBL_PT", [("t", 6, "in"), ("t_out", 6, "out")])
    X, Y, Z = fp2_in(0, 0), fp2_in(0, 1), fp2_in(0, 2)
    A = b.f2mul(X, Y)
    B = b.f2sqr(Y)
    C = b.f2sqr(Z)
    YZ2 = b.f2sqr(f2add(Y, Z))
    E = f2scale(f2xi(C), 12)
    F = f2scale(E, 3)
    H = f2sub(YZ2, f2add(B, C))
    X3 = f2scale(b.f2mul(A, f2sub(B, F)), 2)
    Y3 = f2sub(b.f2sqr(f2add(B, F)), f2scale(b.f2sqr(E), 12))
    Z3 = f2scale(b.f2mul(B, H), 4)
    b.out_vec(1, [X3[0], X3[1], Y3[0], Y3[1], Z3[0], Z3[1]])
    return b


def prog_add_step():
    # T (6), Q affine (4: x, y in Fp2), P (2: -xP, yP) -> T' = T + Q, line (6)
    b = Builder("G2_ADD_STEP", [("t", 6, "in"), ("q", 4, "in"), ("p", 2, "in"), ("t_out", 6, "out"), ("l", 6, "out")])
    X, Y, Z = fp2_in(0, 0), fp2_in(0, 1), fp2_in(0, 2)
    Qx, Qy = fp2_in(1, 0), fp2_in(1, 1)
    nxp, yp = inp(2, 0), inp(2, 1)
    theta = f2sub(Y, b.f2mul(Qy, Z))
    lam = f2sub(X, b.f2mul(Qx, Z))
    C = b.f2sqr(theta)
    D = b.f2sqr(lam)
    E = b.f2mul(D, lam)
    F = b.f2mul(Z, C)
    G = b.f2mul(X, D)
    H = f2sub(f2add(E, F), f2scale(G, 2))
    X3 = b.f2mul(lam, H)
    Y3 = f2sub(b.f2mul(theta, f2sub(G, H)), b.f2mul(Y, E))
    Z3 = b.f2mul(Z, E)
    l0 = f2sub(b.f2mul(theta, Qx), b.f2mul(lam, Qy))
    l2 = b.f2mulfp(theta, nxp)
    l3 = b.f2mulfp(lam, yp)
    b.out_vec(3, [X3[0], X3[1], Y3[0], Y3[1], Z3[0], Z3[1]])
    b.out_vec(4, [l0[0], l0[1], l2[0], l2[1], l3[0], l3[1]])
    return b


PROGRAMS = [prog_fp12_mul, prog_fp12_sqr, prog_cyc_sqr, prog_mul_line, lambda: prog_frob(1), lambda: prog_frob(2),
            prog_dbl_step, prog_add_step, prog_dbl_pt, prog_sqr_dbl]


# ---- scheduling and encoding -------------------------------------------------------------------
def schedule(b):
    """Round of each product = 1 + max round of the products its operands reference."""
    rnd = []
    for a, c in b.prods:
        r = 1
        for lin in (a, c):
            for s in lin.d:
                if s[0] == "z":
                    r = max(r, rnd[s[1]] + 1)
        rnd.append(r)
    order = sorted(range(len(b.prods)), key=lambda k: (rnd[k], k))
    remap = {old: new for new, old in enumerate(order)}
    nr = max(rnd) if rnd else 0
    round_end = [sum(1 for k in rnd if k <= r) for r in range(1, nr + 1)]
    return order, remap, round_end


DUP_MAX = 3  # a term with |coefficient| <= DUP_MAX is emitted as |c| unit terms (no scaling loop)


def encode(b):
    order, remap, round_end = schedule(b)
    nprod = len(b.prods)
    terms = []

    def expand(lin, width):
        """(src, idx, coefficient) list of a linear form; terms with |c| <= DUP_MAX become |c| unit
        copies (no scaling loop on the device) while the record width allows."""
        items = []
        for s_, c in sorted(lin.d.items(), key=lambda kv: str(kv[0])):
            if s_[0] == "in":
                src, idx = s_[1], s_[2]
            elif s_[0] == "z":
                src, idx = SRC_Z, remap[s_[1]]
            elif s_[0] == "p":
                src, idx = SRC_Z, nprod + s_[1]
            elif s_[0] == "zraw":
                src, idx = SRC_Z, s_[1]
            else:
                src, idx = SRC_C, s_[1]
            assert -32768 < c < 32768 and idx < 256
            items.append((src, idx, c))
        budget = width - len(items)
        out = []
        for src, idx, c in items:
            if 1 < abs(c) <= DUP_MAX and abs(c) - 1 <= budget:
                budget -= abs(c) - 1
                out += [(src, idx, 1 if c > 0 else -1)] * abs(c)
            else:
                out.append((src, idx, c))
        return out

    def put(tl):
        start = len(terms)
        terms.extend(tl)
        return start, len(tl)

    prods = []
    for k in order:
        a0, an = put(expand(b.prods[k][0], OPW))
        b0, bn = put(expand(b.prods[k][1], OPW))
        assert an <= OPW and bn <= OPW, (b.name, an, bn)
        prods.append((a0, an, b0, bn))
    # Partial sums (one lane each, stored in Z after the products): the explicit ones, then the
    # pieces of long outputs, so the output phase is two short add chains, not one long one.
    parts = []
    nz = nprod
    for lin in b.xparts:
        tl = expand(lin, SUM_TERMS)
        assert all(t[0] != SRC_Z or t[1] < nprod for t in tl), "a partial sum reads products only"
        assert len(tl) <= SUM_TERMS, (b.name, len(tl))
        t0, tn = put(tl)
        parts.append((t0, tn, nz))
        nz += 1
    outs = []
    for op, i, lin in b.outs:
        tl = expand(lin, b.out_max)
        if len(tl) > b.out_max:  # split: expand freely inside the pieces
            tl = expand(lin, 4 * SUM_TERMS * SUM_TERMS)
        if len(tl) > b.out_max:
            refs = []
            for j in range(0, len(tl), PART_TERMS):
                t0, tn = put(tl[j:j + PART_TERMS])
                parts.append((t0, tn, nz))
                refs.append((SRC_Z, nz, 1))
                nz += 1
            assert len(refs) <= SUM_TERMS, (b.name, len(refs))
            t0, tn = put(refs)
            outs.append((t0, tn, op, i))
        else:
            t0, tn = put(tl)
            outs.append((t0, tn, op, i))
    assert len(outs) <= 64 and len(prods) <= 64 and len(parts) <= 64 and nz <= 128, (b.name, len(outs), len(prods), nz)
    return {"name": b.name, "signature": b.signature, "round_end": round_end, "prods": prods, "parts": parts,
            "outs": outs, "terms": terms, "nz": nz}


def mont(v):
    return v * (1 << 392) % P  # Montgomery radix R = 2^392 (fp.h)


def limbs(v):
    return ["0x%08xu" % ((v >> (32 * i)) & 0xFFFFFFFF) for i in range(12)]


PROD_WORDS, SUM_WORDS, SUM_TERMS = 24, 12, 11


def term_word(t, neg=False):
    src, idx, c = t
    assert 0 <= src < 8 and idx < 256 and 0 < abs(c) < 65536
    return src | (int(neg) << 4) | (idx << 8) | (abs(c) << 16)


ZERO_TERM = SRC_C | (ZERO_IDX << 8) | (1 << 16)


def signed_record(T, t0, tn, width):
    """(npos, nneg, nsc, words): the terms of T[t0:t0+tn] as `width` u32 words (src | neg << 4 |
    idx << 8 | |c| << 16): the unit terms (+1, then -1 with the neg bit) from word 0, then the scaled
    terms (|c| > 1), then the zero constant (ZERO_TERM) as padding."""
    ts = list(T[t0:t0 + tn])
    pos = [t for t in ts if t[2] == 1]
    neg = [t for t in ts if t[2] == -1]
    sc = [t for t in ts if abs(t[2]) > 1]
    assert len(pos) + len(neg) + len(sc) == len(ts) and len(ts) <= width
    words = [term_word(t) for t in pos] + [term_word(t, True) for t in neg] + [term_word(t, t[2] < 0) for t in sc]
    return len(pos), len(neg), len(sc), words + [ZERO_TERM] * (width - len(words))


def phase_umax(T, recs):
    """The wave-uniform trip count of a phase's unit-term loop (its lanes' records recs = [(t0, tn)]):
    the largest unit count.  A lane masks the words past its own count to the zero constant."""
    return max([sum(1 for t in T[t0:t0 + tn] if abs(t[2]) == 1) for t0, tn in recs] or [0])


def emit(progs, path):
    L = ["// GENERATED by tools/gen_coop.py -- do not edit.",
         "// Wave-cooperative programs (see tools/gen_coop.py for the encoding); run by coop.h.",
         "#pragma once", '#include "fp_types.h"', "", "namespace gbv {", "namespace coop {", ""]
    assert len(CONSTS.vals) <= 16
    L.append("constexpr int N_CONSTS = %d;" % len(CONSTS.vals))
    L.append("constexpr uint32_t ZERO_TERM = 0x%xu;  // the constant 0: record padding, masked-off terms" % ZERO_TERM)
    L.append("GBV_COOP_TABLE Fp CONSTS[%d] = {" % max(1, len(CONSTS.vals)))
    for v in CONSTS.vals or [0]:
        L.append("    {{%s}}," % ", ".join(limbs(mont(v))))
    L.append("};")
    for p in progs:
        n = p["name"]
        L.append("")
        L.append("// %s: operands %s; %d products in %d rounds, %d partial sums, %d outputs, %d terms" % (
            n, ", ".join("%d=%s[%d] %s" % (i, s[0], s[1], s[2]) for i, s in enumerate(p["signature"])),
            len(p["prods"]), len(p["round_end"]), len(p["parts"]), len(p["outs"]), len(p["terms"])))
        T = p["terms"]
        prod_recs = []
        for (a0, an, b0, bn) in p["prods"]:
            pa, na, sa, wa = signed_record(T, a0, an, OPW)
            pb, nb, sb, wb = signed_record(T, b0, bn, OPW)
            hdr = pa | (na << 8) | (pb << 16) | (nb << 24)
            prod_recs.append([hdr] + wa + wb + [sa | (sb << 8)] + [0] * (PROD_WORDS - 2 - 2 * OPW))
        prod_recs = prod_recs or [[0] * PROD_WORDS]

        def sum_rec(t0, tn):
            ps, ns, ss, w = signed_record(T, t0, tn, SUM_TERMS)
            return [ps | (ns << 8) | (ss << 16)] + w
        part_recs = [sum_rec(t0, tn) for (t0, tn, _) in p["parts"]] or [[0] * SUM_WORDS]
        out_recs = [sum_rec(t0, tn) for (t0, tn, _, _) in p["outs"]]
        for j, (_, _, z) in enumerate(p["parts"]):
            assert z == len(p["prods"]) + j
        fmt = lambda recs: ",\n    ".join("{" + ", ".join("0x%xu" % w for w in r) + "}" for r in recs)
        L.append("GBV_COOP_TABLE uint32_t %s_PRODS[%d][%d] __attribute__((aligned(16))) = {\n    %s};" % (
            n, len(prod_recs), PROD_WORDS, fmt(prod_recs)))
        L.append("GBV_COOP_TABLE uint32_t %s_PARTS[%d][%d] __attribute__((aligned(16))) = {\n    %s};" % (
            n, len(part_recs), SUM_WORDS, fmt(part_recs)))
        L.append("GBV_COOP_TABLE uint32_t %s_OUTS[%d][%d] __attribute__((aligned(16))) = {\n    %s};" % (
            n, len(out_recs), SUM_WORDS, fmt(out_recs)))
        L.append("GBV_COOP_TABLE uint8_t %s_OUT_DST[%d] = {%s};" % (n, len(p["outs"]), ", ".join(str(o[2]) for o in p["outs"])))
        L.append("GBV_COOP_TABLE uint8_t %s_OUT_IDX[%d] = {%s};" % (n, len(p["outs"]), ", ".join(str(o[3]) for o in p["outs"])))
        re = p["round_end"] + [0] * (6 - len(p["round_end"]))
        assert len(p["round_end"]) <= 6
        amax, bmax, r0 = [], [], 0
        for r1 in p["round_end"]:
            amax.append(phase_umax(T, [(a0, an) for (a0, an, _, _) in p["prods"][r0:r1]]))
            bmax.append(phase_umax(T, [(b0, bn) for (_, _, b0, bn) in p["prods"][r0:r1]]))
            r0 = r1
        amax += [0] * (6 - len(amax))
        bmax += [0] * (6 - len(bmax))
        pmax = phase_umax(T, [(t0, tn) for (t0, tn, _) in p["parts"]])
        omax = phase_umax(T, [(t0, tn) for (t0, tn, _, _) in p["outs"]])
        L.append("GBV_COOP_TABLE Prog %s = {%d, %d, %d, {%s}, {%s}, {%s}, %d, %d, &%s_PRODS[0][0], &%s_PARTS[0][0], &%s_OUTS[0][0], %s_OUT_DST, %s_OUT_IDX};" % (
            n, len(p["round_end"]), len(p["parts"]), len(p["outs"]), ", ".join(map(str, re)), ", ".join(map(str, amax)),
            ", ".join(map(str, bmax)), pmax, omax, n, n, n, n, n))
    L += ["", "}  // namespace coop", "}  // namespace gbv", ""]
    open(path, "w").write("\n".join(L))


def build_all():
    progs = [encode(f()) for f in PROGRAMS]
    return progs, list(CONSTS.vals)


# The programs the device still interprets (coop.h run()): the Frobenius maps and the mixed addition
# step.  The others are specifications of the written-out steps (coop.h cyc_sqr, mul_line, sqr_dbl,
# mul12, the point doublings) and are checked here and by tests/test_coop_tables.py only.
DEVICE_PROGRAMS = ("FP12_FROB1", "FP12_FROB2", "G2_ADD_STEP")


def main():
    progs, consts = build_all()
    out = os.path.join(ROOT, "lodestar_amd", "csrc", "coop_tables.h")
    emit([p for p in progs if p["name"] in DEVICE_PROGRAMS], out)
    for p in progs:
        print("%-16s prods=%2d rounds=%d parts=%2d outs=%2d terms=%4d" % (
            p["name"], len(p["prods"]), len(p["round_end"]), len(p["parts"]), len(p["outs"]), len(p["terms"])))
    print("wrote", os.path.relpath(out, ROOT), "consts", len(consts))


if __name__ == "__main__":
    main()
