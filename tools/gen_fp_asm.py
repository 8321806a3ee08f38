"""Generate lodestar_amd/csrc/fp_asm.h: 384-bit add/sub/reduce carry chains as single inline-asm
blocks for gfx950 (VCC carry chains, no compiler-inserted s_nop padding between links).

Each block takes its operands in VGPRs (the prime's limbs included: VOP2 carry ops read VCC
implicitly, which uses the one constant-bus slot, so SGPR/literal operands are not encodable)."""
import os

N = 12


def regs(base):
    return ["%%%d" % (base + i) for i in range(N)]


def block(name, body, outs, ins, doc):
    lines = ["// %s" % doc, "#define %s(%s) \\" % (name, ", ".join(o for o, _ in outs + ins))]
    lines.append("  asm(" + " \\\n      ".join('"%s\\n\\t"' % l for l in body[:-1]) + ' \\\n      "%s" \\' % body[-1])
    ov = []
    for o, c in outs:
        ov += ['"%s"(%s.v[%d])' % (c, o, i) for i in range(N)]
    iv = []
    for o, _ in ins:
        iv += ['"v"(%s.v[%d])' % (o, i) for i in range(N)]
    lines.append("      : " + ", ".join(ov) + " \\")
    lines.append("      : " + ", ".join(iv) + " \\")
    lines.append('      : "vcc")')
    return "\n".join(lines) + "\n"


def add_reduce():
    s, r = regs(0), regs(12)
    a, b, p = regs(24), regs(36), regs(48)
    body = ["v_add_co_u32 %s, vcc, %s, %s" % (s[0], a[0], b[0])]
    body += ["v_addc_co_u32 %s, vcc, %s, %s, vcc" % (s[i], a[i], b[i]) for i in range(1, N)]
    body += ["v_sub_co_u32 %s, vcc, %s, %s" % (r[0], s[0], p[0])]
    body += ["v_subb_co_u32 %s, vcc, %s, %s, vcc" % (r[i], s[i], p[i]) for i in range(1, N)]
    body += ["v_cndmask_b32 %s, %s, %s, vcc" % (r[i], r[i], s[i]) for i in range(N)]
    return block("GBV_ASM_ADD_MOD", body, [("s", "=&v"), ("r", "=&v")], [("a", "v"), ("b", "v"), ("p", "v")],
                 "r = (a + b) mod p for a, b < p (s is scratch).  36 VALU ops.")


def sub_mod():
    d, m = regs(0), regs(12)
    a, b, p = regs(24), regs(36), regs(48)
    body = ["v_sub_co_u32 %s, vcc, %s, %s" % (d[0], a[0], b[0])]
    body += ["v_subb_co_u32 %s, vcc, %s, %s, vcc" % (d[i], a[i], b[i]) for i in range(1, N)]
    body += ["v_cndmask_b32 %s, 0, %s, vcc" % (m[i], p[i]) for i in range(N)]
    body += ["v_add_co_u32 %s, vcc, %s, %s" % (d[0], d[0], m[0])]
    body += ["v_addc_co_u32 %s, vcc, %s, %s, vcc" % (d[i], d[i], m[i]) for i in range(1, N)]
    return block("GBV_ASM_SUB_MOD", body, [("d", "=&v"), ("m", "=&v")], [("a", "v"), ("b", "v"), ("p", "v")],
                 "d = (a - b) mod p for a, b < p (m is scratch).  36 VALU ops.")


def reduce_once():
    r = regs(0)
    x, p = regs(12), regs(24)
    body = ["v_sub_co_u32 %s, vcc, %s, %s" % (r[0], x[0], p[0])]
    body += ["v_subb_co_u32 %s, vcc, %s, %s, vcc" % (r[i], x[i], p[i]) for i in range(1, N)]
    body += ["v_cndmask_b32 %s, %s, %s, vcc" % (r[i], r[i], x[i]) for i in range(N)]
    return block("GBV_ASM_REDUCE_ONCE", body, [("r", "=&v")], [("x", "v"), ("p", "v")],
                 "r = x < p ? x : x - p for x < 2p.  24 VALU ops.")


def add_raw():
    s = regs(0)
    a, b = regs(12), regs(24)
    body = ["v_add_co_u32 %s, vcc, %s, %s" % (s[0], a[0], b[0])]
    body += ["v_addc_co_u32 %s, vcc, %s, %s, vcc" % (s[i], a[i], b[i]) for i in range(1, N)]
    return block("GBV_ASM_ADD_RAW", body, [("s", "=&v")], [("a", "v"), ("b", "v")],
                 "s = a + b, no reduction (a + b < 2^384; the product input of a lazy sum).  12 VALU ops.")


def sub_raw_k():
    t, d = regs(0), regs(12)
    a, b, k = regs(24), regs(36), regs(48)
    body = ["v_add_co_u32 %s, vcc, %s, %s" % (t[0], a[0], k[0])]
    body += ["v_addc_co_u32 %s, vcc, %s, %s, vcc" % (t[i], a[i], k[i]) for i in range(1, N)]
    body += ["v_sub_co_u32 %s, vcc, %s, %s" % (d[0], t[0], b[0])]
    body += ["v_subb_co_u32 %s, vcc, %s, %s, vcc" % (d[i], t[i], b[i]) for i in range(1, N)]
    return block("GBV_ASM_SUB_RAW_K", body, [("t", "=&v"), ("d", "=&v")], [("a", "v"), ("b", "v"), ("k", "v")],
                 "d = a + k - b, no reduction (b <= k, a + k < 2^384; t is scratch).  24 VALU ops.")


def acc_raw():
    s = regs(0)
    b = regs(12)
    body = ["v_add_co_u32 %s, vcc, %s, %s" % (s[0], s[0], b[0])]
    body += ["v_addc_co_u32 %s, vcc, %s, %s, vcc" % (s[i], s[i], b[i]) for i in range(1, N)]
    return block("GBV_ASM_ACC_RAW", body, [("s", "+v")], [("b", "v")],
                 "s += b in place, no reduction (the accumulator of a lazy sum: no copy out of the asm's\n"
                 "// registers at every term).  12 VALU ops.")


def reduce_ip():
    x, t = regs(0), regs(12)
    p = regs(24)
    body = ["v_sub_co_u32 %s, vcc, %s, %s" % (t[0], x[0], p[0])]
    body += ["v_subb_co_u32 %s, vcc, %s, %s, vcc" % (t[i], x[i], p[i]) for i in range(1, N)]
    body += ["v_cndmask_b32 %s, %s, %s, vcc" % (x[i], t[i], x[i]) for i in range(N)]
    return block("GBV_ASM_REDUCE_IP", body, [("x", "+v"), ("t", "=&v")], [("p", "v")],
                 "x = x < p ? x : x - p in place for x < 2p (t is scratch).  24 VALU ops.")


def main():
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lodestar_amd", "csrc", "fp_asm.h")
    src = ["// GENERATED by tools/gen_fp_asm.py -- do not edit.",
           "// 384-bit modular add/sub carry chains as single gfx950 inline-asm blocks (device only).",
           "#pragma once", "", add_reduce(), sub_mod(), reduce_once(), add_raw(), sub_raw_k(), acc_raw(), reduce_ip()]
    open(out, "w").write("\n".join(src))
    print("wrote", os.path.normpath(out))


if __name__ == "__main__":
    main()
