#!/usr/bin/env python3
"""Generate bls_wc12_tables.h: wave-cooperative Fp12 operations as bilinear
programs (products of linear forms, then linear forms of the products).

Why: the per-request tails of the verification (the Miller loop of
(-g1, S_k) and the final exponentiation) are single Fp12 dependency chains of
~8-10k Fp products; run by one lane they take 15-20 ms whatever the batch
size.  Written as "K independent Fp products + linear combinations", every
Fp12 multiplication / squaring becomes ONE round of parallel products across
the lanes of a wave (K = 18 ... 54), so the chain's latency drops by the
product count per operation.

Each op is derived by running the same tower formulas as bls_field.h
(Karatsuba Fp2/Fp6/Fp12, complex squaring, Granger-Scott cyclotomic squaring,
sparse line multiplication, Frobenius) on symbolic linear forms: a product
records (x = sum a_i A_i, y = sum b_j B_j) and the outputs are forms over the
products and the inputs.  Symbols: A[0..11], B[0..11] are the Fp coefficients
of the two operands in tower order (c0.c0.c0, c0.c0.c1, c0.c1.c0, ...,
c1.c2.c1); products P[0..K).

Usage: python gen_wc12.py OUT.h
"""
import sys
from collections import defaultdict


class Form:
    """Linear form over symbols ('A', i) / ('B', i) / ('P', k) with small int coefficients."""

    def __init__(self, d=None):
        self.d = {k: v for k, v in (d or {}).items() if v}

    @staticmethod
    def sym(kind, i):
        return Form({(kind, i): 1})

    def __add__(self, o):
        r = defaultdict(int, self.d)
        for k, v in o.d.items():
            r[k] += v
        return Form(r)

    def __sub__(self, o):
        r = defaultdict(int, self.d)
        for k, v in o.d.items():
            r[k] -= v
        return Form(r)

    def __neg__(self):
        return Form({k: -v for k, v in self.d.items()})

    def scale(self, c):
        return Form({k: v * c for k, v in self.d.items()})

    def kinds(self):
        return {k[0] for k in self.d}


ZERO = Form()


class Program:
    def __init__(self, square=False):
        self.prods = []  # (x form, y form)
        self.square = square  # B aliases A

    def mul(self, x, y):
        if self.square:
            # x, y both over A; keep them over A (B == A at run time)
            assert x.kinds() <= {"A"} and y.kinds() <= {"A"}, (x.d, y.d)
        else:
            if x.kinds() <= {"B"} and y.kinds() <= {"A"}:
                x, y = y, x
            assert x.kinds() <= {"A"} and y.kinds() <= {"B"}, (x.d, y.d)
        if not x.d or not y.d:
            return ZERO
        self.prods.append((x, y))
        return Form.sym("P", len(self.prods) - 1)


# ---- symbolic tower (same formulas as bls_field.h) --------------------------
class F2:
    def __init__(self, c0, c1):
        self.c0, self.c1 = c0, c1

    def __add__(self, o):
        return F2(self.c0 + o.c0, self.c1 + o.c1)

    def __sub__(self, o):
        return F2(self.c0 - o.c0, self.c1 - o.c1)

    def __neg__(self):
        return F2(-self.c0, -self.c1)

    def conj(self):
        return F2(self.c0, -self.c1)

    def mul_xi(self):
        return F2(self.c0 - self.c1, self.c0 + self.c1)

    def scale(self, c):
        return F2(self.c0.scale(c), self.c1.scale(c))


def f2_mul(P, a, b):
    t0 = P.mul(a.c0, b.c0)
    t1 = P.mul(a.c1, b.c1)
    s = P.mul(a.c0 + a.c1, b.c0 + b.c1)
    return F2(t0 - t1, s - t0 - t1)


def f2_sqr(P, a):
    m = P.mul(a.c0, a.c1)
    return F2(P.mul(a.c0 + a.c1, a.c0 - a.c1), m + m)


class F6:
    def __init__(self, c0, c1, c2):
        self.c = [c0, c1, c2]

    def __add__(self, o):
        return F6(*[x + y for x, y in zip(self.c, o.c)])

    def __sub__(self, o):
        return F6(*[x - y for x, y in zip(self.c, o.c)])

    def __neg__(self):
        return F6(*[-x for x in self.c])

    def mul_v(self):
        return F6(self.c[2].mul_xi(), self.c[0], self.c[1])


def f6_mul(P, a, b):
    a0, a1, a2 = a.c
    b0, b1, b2 = b.c
    t0, t1, t2 = f2_mul(P, a0, b0), f2_mul(P, a1, b1), f2_mul(P, a2, b2)
    c0 = t0 + (f2_mul(P, a1 + a2, b1 + b2) - t1 - t2).mul_xi()
    c1 = f2_mul(P, a0 + a1, b0 + b1) - t0 - t1 + t2.mul_xi()
    c2 = f2_mul(P, a0 + a2, b0 + b2) - t0 - t2 + t1
    return F6(c0, c1, c2)


def f6_mul_01(P, a, b0, b1):
    t0, t1 = f2_mul(P, a.c[0], b0), f2_mul(P, a.c[1], b1)
    c0 = t0 + f2_mul(P, a.c[2], b1).mul_xi()
    c1 = f2_mul(P, a.c[0] + a.c[1], b0 + b1) - t0 - t1
    c2 = t1 + f2_mul(P, a.c[2], b0)
    return F6(c0, c1, c2)


def f6_mul_1(P, a, b1):
    return F6(f2_mul(P, a.c[2], b1).mul_xi(), f2_mul(P, a.c[0], b1), f2_mul(P, a.c[1], b1))


class F12:
    def __init__(self, c0, c1):
        self.c0, self.c1 = c0, c1

    def flat(self):
        out = []
        for f6 in (self.c0, self.c1):
            for f2 in f6.c:
                out += [f2.c0, f2.c1]
        return out


def sym12(kind):
    s = [Form.sym(kind, i) for i in range(12)]
    f2s = [F2(s[2 * k], s[2 * k + 1]) for k in range(6)]
    return F12(F6(*f2s[0:3]), F6(*f2s[3:6]))


def op_mul():
    P = Program()
    a, b = sym12("A"), sym12("B")
    t0, t1 = f6_mul(P, a.c0, b.c0), f6_mul(P, a.c1, b.c1)
    c1 = f6_mul(P, a.c0 + a.c1, b.c0 + b.c1) - t0 - t1
    c0 = t0 + t1.mul_v()
    return P, F12(c0, c1)


def op_sqr():
    P = Program(square=True)
    a = sym12("A")
    t = f6_mul(P, a.c0, a.c1)
    s = f6_mul(P, a.c0 + a.c1, a.c0 + a.c1.mul_v())
    c0 = s - t - t.mul_v()
    c1 = t + t
    return P, F12(c0, c1)


def op_cyc():
    P = Program(square=True)
    f = sym12("A")

    def fp4_sqr(x, y):
        t0, t1 = f2_sqr(P, x), f2_sqr(P, y)
        t2 = f2_sqr(P, x + y)
        return t0 + t1.mul_xi(), t2 - t0 - t1

    def m2(a, b):  # 3a - 2b
        return (a - b).scale(2) + a

    def p2(a, b):  # 3a + 2b
        return (a + b).scale(2) + a

    Ax, Ay = fp4_sqr(f.c0.c[0], f.c1.c[1])
    Bx, By = fp4_sqr(f.c1.c[0], f.c0.c[2])
    Cx, Cy = fp4_sqr(f.c0.c[1], f.c1.c[2])
    c00 = m2(Ax, f.c0.c[0])
    c11 = p2(Ay, f.c1.c[1])
    c10 = p2(Cy.mul_xi(), f.c1.c[0])
    c02 = m2(Cx, f.c0.c[2])
    c01 = m2(Bx, f.c0.c[1])
    c12 = p2(By, f.c1.c[2])
    return P, F12(F6(c00, c01, c02), F6(c10, c11, c12))


def op_line():
    """f * (l0 + l1 v + l4 v w); B[0..5] = l0.c0, l0.c1, l1.c0, l1.c1, l4.c0, l4.c1."""
    P = Program()
    f = sym12("A")
    l0 = F2(Form.sym("B", 0), Form.sym("B", 1))
    l1 = F2(Form.sym("B", 2), Form.sym("B", 3))
    l4 = F2(Form.sym("B", 4), Form.sym("B", 5))
    t0 = f6_mul_01(P, f.c0, l0, l1)
    t1 = f6_mul_1(P, f.c1, l4)
    s = f6_mul_01(P, f.c0 + f.c1, l0, l1 + l4)
    c1 = s - t0 - t1
    c0 = t0 + t1.mul_v()
    return P, F12(c0, c1)


def op_frob(k):
    """f^(p^k): coefficient of w^e (c_i.c_j, e = 2j + i) conjugated k times and
    multiplied by gamma_{k,e}; B holds gamma_{k,e} as Fp2 at B[2e], B[2e+1]."""
    P = Program()
    f = sym12("A")
    slots = [(0, 0), (1, 0), (0, 1), (1, 1), (0, 2), (1, 2)]  # e -> (i, j)
    out = {}
    for e, (i, j) in enumerate(slots):
        x = (f.c0 if i == 0 else f.c1).c[j]
        if k % 2:
            x = x.conj()
        out[(i, j)] = x if e == 0 else f2_mul(P, x, F2(Form.sym("B", 2 * e), Form.sym("B", 2 * e + 1)))
    return P, F12(F6(*[out[(0, j)] for j in range(3)]), F6(*[out[(1, j)] for j in range(3)]))


def op_conj():
    P = Program()
    f = sym12("A")
    return P, F12(f.c0, -f.c1)


OPS = [("MUL", op_mul), ("SQR", op_sqr), ("CYC", op_cyc), ("LINE", op_line), ("FROB1", lambda: op_frob(1)),
       ("FROB2", lambda: op_frob(2)), ("FROB3", lambda: op_frob(3)), ("CONJ", op_conj)]
KIND = {"A": 0, "B": 1, "P": 2}


def enc_terms(form, allowed):
    out = []
    for (kind, idx), c in sorted(form.d.items()):
        assert kind in allowed, (kind, allowed)
        assert -8 <= c <= 8 and c != 0, c
        out.append((c, KIND[kind] << 6 | idx))
    return out


CHUNK = 8  # max sum |c| of one lane's lazily accumulated terms (< 8p < 2^384)


def chunks(term_list):
    """Split an output's terms into runs with sum |c| <= CHUNK."""
    out, cur, w = [], [], 0
    for c, code in term_list:
        if cur and w + abs(c) > CHUNK:
            out.append(cur)
            cur, w = [], 0
        cur.append((c, code))
        w += abs(c)
    if cur:
        out.append(cur)
    return out


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else "bls_wc12_tables.h"
    terms = []  # flat (coef, code)
    lines = ["// GENERATED by gen_wc12.py -- do not edit.", "#pragma once", ""]
    descs = []
    stats = []
    for name, fn in OPS:
        P, out = fn()
        K = len(P.prods)
        assert K <= 64
        xoff, yoff = [], []
        for x, y in P.prods:
            xoff.append(len(terms))
            tx = enc_terms(x, {"A"})
            assert sum(abs(c) for c, _ in tx) <= CHUNK
            terms += tx
            yoff.append(len(terms))
            ty = enc_terms(y, {"A"} if P.square else {"B"})
            assert sum(abs(c) for c, _ in ty) <= CHUNK
            terms += ty
        yoff.append(len(terms))  # sentinel after the last product's y terms
        coff, cs = [], []
        for o in out.flat():
            cs.append(len(coff))
            for ch in chunks(enc_terms(o, {"A", "B", "P"})):
                coff.append(len(terms))
                terms += ch
        cs.append(len(coff))
        coff.append(len(terms))
        nc = len(coff) - 1
        assert nc <= 64, (name, nc)
        descs.append((name, K, P.square, xoff, yoff, nc, coff, cs))
        stats.append("%s: %d products, %d output chunks" % (name, K, nc))
    assert len(terms) < 65536
    lines.append("// " + "; ".join(stats))
    lines.append("#define LB_WC_NTERMS %d" % len(terms))
    lines.append("__device__ __constant__ const int8_t LB_WC_COEF[%d] = {%s};" % (
        len(terms), ", ".join(str(c) for c, _ in terms)))
    lines.append("__device__ __constant__ const uint8_t LB_WC_CODE[%d] = {%s};" % (
        len(terms), ", ".join(str(x) for _, x in terms)))
    lines.append("// per op: K products (lane k: x terms [xoff[k], yoff[k]), y terms up to the next xoff /\n"
                 "// yoff[K]); NC output chunks (lane c: terms [coff[c], coff[c+1]), sum |coef| <= 8);\n"
                 "// output o = sum of chunks [cs[o], cs[o+1])")
    lines.append("struct wc_desc {\n  uint8_t K, square, NC, pad;\n  uint16_t xoff[64], yoff[65], coff[65], cs[13];\n};")
    for i, d in enumerate(descs):
        lines.append("#define LB_WC_%s %d" % (d[0], i))
    lines.append("#define LB_WC_NOPS %d" % len(descs))
    body = []
    for name, K, sq, xoff, yoff, nc, coff, cs in descs:
        pad = lambda v, n: v + [0] * (n - len(v))  # noqa: E731
        body.append("{%d, %d, %d, 0, {%s}, {%s}, {%s}, {%s}}" % (
            K, int(sq), nc, ", ".join(map(str, pad(xoff, 64))), ", ".join(map(str, pad(yoff, 65))),
            ", ".join(map(str, pad(coff, 65))), ", ".join(map(str, cs))))
    lines.append("__device__ __constant__ const wc_desc LB_WC_OPS[%d] = {\n  %s};" % (len(descs), ",\n  ".join(body)))
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(stats))


if __name__ == "__main__":
    main()
