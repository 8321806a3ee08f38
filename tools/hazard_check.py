"""Compare tools/hazard_check output with Python Montgomery arithmetic (see the .hip)."""
import sys

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 1 << 384
RINV = pow(R, -1, P)
ONE = R % P


def limbs(x):
    return [(x >> (32 * i)) & 0xFFFFFFFF for i in range(12)]


def unlimbs(v):
    return sum(w << (32 * i) for i, w in enumerate(v))


def expected(t, iters):
    a, b = limbs(ONE), limbs(ONE)
    a[0] ^= (t * 0x9E3779B9) & 0xFFFFFFFF
    a[5] ^= t
    b[3] ^= 0x12345 + t
    a, b = unlimbs(a), unlimbs(b)
    a = a - P if a >= P else a
    b = b - P if b >= P else b
    for _ in range(iters):
        a = a * b * RINV % P
        b = (b + a) % P
        a = (a - b) % P
    return a


def main(path, iters):
    bad = 0
    n = 0
    for line in open(path):
        parts = line.split()
        if len(parts) != 2 or not parts[0].isdigit():
            continue
        t, hexv = int(parts[0]), parts[1]
        n += 1
        if int(hexv, 16) != expected(t, iters):
            bad += 1
    print("%s: %d lanes checked, %d wrong" % (path, n, bad))
    return bad


if __name__ == "__main__":
    sys.exit(1 if main(sys.argv[1], int(sys.argv[2])) else 0)
