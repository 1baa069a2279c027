"""Fp2 / Fp6 / Fp12 and the G1 / G2 group law as round-program builders.

The formulas are those of the one-lane device code (csrc/bls_field.h,
bls_curve.h, bls_pairing.h) so both paths compute the same points; only the
execution differs: every product below becomes a unit of the round program,
and all products of one tower operation with ready operands share a round.
Data-dependent branches of the device code (exceptional cases of the group
law, square-root cases, sign fixes) are selects on flags here.
"""
from __future__ import annotations

from .dsl import Flag, Fp, Graph, P, select, select_n


# ---------------------------------------------------------------------------
# Fp2 = Fp[u]/(u^2 + 1)
# ---------------------------------------------------------------------------
class Fp2:
    __slots__ = ("c0", "c1")

    def __init__(self, c0: Fp, c1: Fp):
        self.c0, self.c1 = c0, c1

    @property
    def g(self) -> Graph:
        return self.c0.g

    @staticmethod
    def const(g: Graph, v) -> "Fp2":
        return Fp2(g.const(v[0]), g.const(v[1]))

    @staticmethod
    def zero(g: Graph) -> "Fp2":
        return Fp2(g.zero(), g.zero())

    @staticmethod
    def one(g: Graph) -> "Fp2":
        return Fp2(g.one(), g.zero())

    def map2(self, f, o: "Fp2") -> "Fp2":
        return Fp2(f(self.c0, o.c0), f(self.c1, o.c1))

    def __add__(self, o: "Fp2") -> "Fp2":
        return Fp2(self.c0 + o.c0, self.c1 + o.c1)

    def __sub__(self, o: "Fp2") -> "Fp2":
        return Fp2(self.c0 - o.c0, self.c1 - o.c1)

    def __neg__(self) -> "Fp2":
        return Fp2(-self.c0, -self.c1)

    def scale(self, k: int) -> "Fp2":
        return Fp2(self.c0.scale(k), self.c1.scale(k))

    def dbl(self) -> "Fp2":
        return self.scale(2)

    def conj(self) -> "Fp2":
        return Fp2(self.c0, -self.c1)

    def mul_xi(self) -> "Fp2":  # (1 + u) a
        return Fp2(self.c0 - self.c1, self.c0 + self.c1)

    def __mul__(self, o):
        if isinstance(o, int):
            return self.scale(o)
        if isinstance(o, Fp):
            return Fp2(self.c0 * o, self.c1 * o)
        t0 = self.c0 * o.c0
        t1 = self.c1 * o.c1
        t2 = (self.c0 + self.c1) * (o.c0 + o.c1)
        return Fp2(t0 - t1, t2 - t0 - t1)

    def sqr(self) -> "Fp2":
        m = self.c0 * self.c1
        return Fp2((self.c0 + self.c1) * (self.c0 - self.c1), m + m)

    def mul_const(self, v) -> "Fp2":
        return self * Fp2.const(self.g, v)

    def norm(self) -> Fp:
        return self.c0.sqr() + self.c1.sqr()

    def inv(self) -> "Fp2":
        ni = self.g.inv(self.norm())
        return Fp2(self.c0 * ni, -(self.c1 * ni))

    def is_zero(self) -> Flag:
        return self.g.is_zero(self.c0) & self.g.is_zero(self.c1)

    def eq(self, o: "Fp2") -> Flag:
        return (self - o).is_zero()

    def mat(self) -> "Fp2":
        return Fp2(self.c0.mat(), self.c1.mat())


def fp_from_mont(x: Fp) -> Fp:
    """raw value (x R^-1): one product by the raw register 1"""
    return x * x.g.const_raw(1)


def fp_sgn0(x: Fp) -> Flag:
    return x.g.bit0(fp_from_mont(x))


def fp_lex_largest(x: Fp) -> Flag:
    return x.g.gt_half(fp_from_mont(x))


def fp2_sgn0(a: Fp2) -> Flag:
    """RFC 9380 sgn0 for Fp2 (bls_field.h fp2_sgn0)"""
    g = a.g
    s0 = fp_sgn0(a.c0)
    z0 = g.is_zero(a.c0)
    s1 = fp_sgn0(a.c1)
    return s0 | (z0 & s1)


def fp2_lex_largest(a: Fp2) -> Flag:
    """ZCash sign flag: c1 decides unless zero (bls_field.h fp2_lex_largest)"""
    g = a.g
    z1 = g.is_zero(a.c1)
    l0 = fp_lex_largest(a.c0)
    l1 = fp_lex_largest(a.c1)
    return (z1 & l0) | (~z1 & l1)


def select2(f: Flag, a: Fp2, b: Fp2) -> Fp2:
    return select(f, a, b)


# ---------------------------------------------------------------------------
# Fp exponentiations (fixed exponents, square-and-multiply with a window of 3
# like bls_field.h fp_pow_p34: unrolled into the program)
# ---------------------------------------------------------------------------
def fp_pow(x: Fp, e: int, window: int = 0) -> Fp:
    """x^e for a fixed exponent e > 0.

    Default (window 0): right-to-left, depth-optimal for round programs.  The
    squaring chain x, x^2, x^4, ... runs one round per bit and the running
    product takes x^(2^i) one round after it appears, so x^e is ready one round
    after the top squaring: ~log2(e) rounds instead of log2(e) + the window
    products of the left-to-right method (378 + 108 for (p-3)/4), at the price
    of popcount(e) products instead of ~e.bit_length() / 4 (units in otherwise
    idle rows).  window > 0: left-to-right sliding window (fewest products)."""
    if e == 0:
        return x.g.one()
    if window == 0:
        acc = None
        s = x
        for i in range(e.bit_length()):
            if (e >> i) & 1:
                acc = s if acc is None else acc * s
            if i + 1 < e.bit_length():
                s = s.sqr()
        return acc
    bits = bin(e)[2:]
    odd = {1: x}
    if window > 1:
        x2 = x.sqr()
        for k in range(3, 1 << window, 2):
            odd[k] = odd[k - 2] * x2
    acc = None
    i = 0
    n = len(bits)
    while i < n:
        if bits[i] == "0":
            acc = acc.sqr()
            i += 1
            continue
        j = min(n, i + window)
        while bits[j - 1] == "0":
            j -= 1
        val = int(bits[i:j], 2)
        if acc is None:
            acc = odd[val]
        else:
            for _ in range(j - i):
                acc = acc.sqr()
            acc = acc * odd[val]
        i = j
    return acc


P34 = (P - 3) // 4


def fp_sqrt_cand(a: Fp) -> tuple:
    """(s, is_square): s = a^((p+1)/4), square iff s^2 == a (bls_field.h fp_sqrt)"""
    t = fp_pow(a, P34)
    s = t * a
    return s, a.g.is_zero(s.sqr() - a)


# ---------------------------------------------------------------------------
# Fp6 = Fp2[v]/(v^3 - xi), Fp12 = Fp6[w]/(w^2 - v)
# ---------------------------------------------------------------------------
class Fp6:
    __slots__ = ("c0", "c1", "c2")

    def __init__(self, c0: Fp2, c1: Fp2, c2: Fp2):
        self.c0, self.c1, self.c2 = c0, c1, c2

    @staticmethod
    def zero(g) -> "Fp6":
        return Fp6(Fp2.zero(g), Fp2.zero(g), Fp2.zero(g))

    @staticmethod
    def one(g) -> "Fp6":
        return Fp6(Fp2.one(g), Fp2.zero(g), Fp2.zero(g))

    def map2(self, f, o):
        return Fp6(self.c0.map2(f, o.c0), self.c1.map2(f, o.c1), self.c2.map2(f, o.c2))

    def __add__(self, o):
        return Fp6(self.c0 + o.c0, self.c1 + o.c1, self.c2 + o.c2)

    def __sub__(self, o):
        return Fp6(self.c0 - o.c0, self.c1 - o.c1, self.c2 - o.c2)

    def __neg__(self):
        return Fp6(-self.c0, -self.c1, -self.c2)

    def mul_v(self) -> "Fp6":
        return Fp6(self.c2.mul_xi(), self.c0, self.c1)

    def __mul__(self, b: "Fp6") -> "Fp6":
        a = self
        t0 = a.c0 * b.c0
        t1 = a.c1 * b.c1
        t2 = a.c2 * b.c2
        c0 = t0 + ((a.c1 + a.c2) * (b.c1 + b.c2) - t1 - t2).mul_xi()
        c1 = (a.c0 + a.c1) * (b.c0 + b.c1) - t0 - t1 + t2.mul_xi()
        c2 = (a.c0 + a.c2) * (b.c0 + b.c2) - t0 - t2 + t1
        return Fp6(c0, c1, c2)

    def mul_01(self, b0: Fp2, b1: Fp2) -> "Fp6":
        a = self
        t0 = a.c0 * b0
        t1 = a.c1 * b1
        c0 = t0 + (a.c2 * b1).mul_xi()
        c1 = (a.c0 + a.c1) * (b0 + b1) - t0 - t1
        c2 = t1 + a.c2 * b0
        return Fp6(c0, c1, c2)

    def mul_1(self, b1: Fp2) -> "Fp6":
        a = self
        return Fp6((a.c2 * b1).mul_xi(), a.c0 * b1, a.c1 * b1)

    def mul_12(self, y1: Fp2, y2: Fp2) -> "Fp6":
        a = self
        p1 = a.c0 * y1
        p2 = a.c0 * y2
        q1 = a.c1 * y1
        q2 = a.c2 * y2
        s = (a.c1 + a.c2) * (y1 + y2) - q1 - q2
        return Fp6(s.mul_xi(), p1 + q2.mul_xi(), p2 + q1)

    def inv(self) -> "Fp6":
        a = self
        c0 = a.c0.sqr() - (a.c1 * a.c2).mul_xi()
        c1 = a.c2.sqr().mul_xi() - a.c0 * a.c1
        c2 = a.c1.sqr() - a.c0 * a.c2
        t = ((a.c2 * c1) + (a.c1 * c2)).mul_xi() + a.c0 * c0
        t = t.inv()
        return Fp6(c0 * t, c1 * t, c2 * t)

    def mat(self) -> "Fp6":
        return Fp6(self.c0.mat(), self.c1.mat(), self.c2.mat())

    def coeffs(self):
        return [self.c0, self.c1, self.c2]


class Fp12:
    __slots__ = ("c0", "c1")

    def __init__(self, c0: Fp6, c1: Fp6):
        self.c0, self.c1 = c0, c1

    @staticmethod
    def one(g) -> "Fp12":
        return Fp12(Fp6.one(g), Fp6.zero(g))

    @staticmethod
    def from_fps(fps) -> "Fp12":
        """12 Fp in the device's memory order c0.c0.c0, c0.c0.c1, c0.c1.c0, ..., c1.c2.c1"""
        f2 = [Fp2(fps[2 * i], fps[2 * i + 1]) for i in range(6)]
        return Fp12(Fp6(f2[0], f2[1], f2[2]), Fp6(f2[3], f2[4], f2[5]))

    def fps(self):
        out = []
        for c6 in (self.c0, self.c1):
            for c2 in (c6.c0, c6.c1, c6.c2):
                out += [c2.c0, c2.c1]
        return out

    def map2(self, f, o):
        return Fp12(self.c0.map2(f, o.c0), self.c1.map2(f, o.c1))

    def conj(self) -> "Fp12":
        return Fp12(self.c0, -self.c1)

    def __mul__(self, b: "Fp12") -> "Fp12":
        a = self
        t0 = a.c0 * b.c0
        t1 = a.c1 * b.c1
        s = (a.c0 + a.c1) * (b.c0 + b.c1)
        return Fp12(t0 + t1.mul_v(), s - t0 - t1)

    def sqr(self) -> "Fp12":
        a = self
        t = a.c0 * a.c1
        s = (a.c0 + a.c1) * (a.c0 + a.c1.mul_v())
        return Fp12(s - t - t.mul_v(), t + t)

    def cyc_sqr(self, lin: "Fp12" = None) -> "Fp12":
        """Granger-Scott squaring in the cyclotomic subgroup (bls_field.h fp12_cyc_sqr).
        lin: the same value as self, materialized: used for the output's linear
        part (3 a^2 -+ 2 a) so a chain of squarings on lazy values never nests
        forms (its LIN units run in the round of the next squaring's products)."""
        f = self
        fl = self if lin is None else lin

        def fp4_sqr(x: Fp2, y: Fp2):
            t0 = x.sqr()
            t1 = y.sqr()
            t2 = (x + y).sqr() - t0 - t1
            return t0 + t1.mul_xi(), t2

        Ax, Ay = fp4_sqr(f.c0.c0, f.c1.c1)
        Bx, By = fp4_sqr(f.c1.c0, f.c0.c2)
        Cx, Cy = fp4_sqr(f.c0.c1, f.c1.c2)

        def m2b(a, b):  # 3a - 2b
            return a.scale(3) - b.scale(2)

        def p2b(a, b):  # 3a + 2b
            return a.scale(3) + b.scale(2)

        o00 = m2b(Ax, fl.c0.c0)
        o11 = p2b(Ay, fl.c1.c1)
        o10 = p2b(Cy.mul_xi(), fl.c1.c0)
        o02 = m2b(Cx, fl.c0.c2)
        o01 = m2b(Bx, fl.c0.c1)
        o12 = p2b(By, fl.c1.c2)
        return Fp12(Fp6(o00, o01, o02), Fp6(o10, o11, o12))

    def mul_line(self, l0: Fp2, l1: Fp2, l4: Fp2) -> "Fp12":
        """f * ((l0 + l1 v) + (l4 v) w)  (bls_field.h fp12_mul_line)"""
        f = self
        t0 = f.c0.mul_01(l0, l1)
        t1 = f.c1.mul_1(l4)
        s = (f.c0 + f.c1).mul_01(l0, l1 + l4)
        return Fp12(t0 + t1.mul_v(), s - t0 - t1)

    def mul_sparse2(self, x: Fp6, y1: Fp2, y2: Fp2) -> "Fp12":
        """f * ((x0 + x1 v + x2 v^2) + (y1 v + y2 v^2) w)  (bls_field.h fp12_mul_by_sparse2)"""
        f = self
        t0 = f.c0 * x
        t1 = f.c1.mul_12(y1, y2)
        sm = Fp6(x.c0, x.c1 + y1, x.c2 + y2)
        sf = (f.c0 + f.c1) * sm
        return Fp12(t0 + t1.mul_v(), sf - t0 - t1)

    def inv(self) -> "Fp12":
        a = self
        t = a.c0 * a.c0 - (a.c1 * a.c1).mul_v()
        t = t.inv()
        return Fp12(a.c0 * t, -(a.c1 * t))

    def frob(self, k: int, gam) -> "Fp12":
        """f^(p^k), k = 1, 2, 3; gam[e] = gamma_{k,e} (as integer pairs)"""
        g = self.c0.c0.g
        conj = k % 2 == 1
        cs = [self.c0.c0, self.c0.c1, self.c0.c2, self.c1.c0, self.c1.c1, self.c1.c2]
        es = [0, 2, 4, 1, 3, 5]
        out = []
        for c, e in zip(cs, es):
            x = c.conj() if conj else c
            out.append(x if e == 0 else x * Fp2.const(g, gam[e]))
        return Fp12(Fp6(out[0], out[1], out[2]), Fp6(out[3], out[4], out[5]))

    def is_one(self) -> Flag:
        g = self.c0.c0.g
        fs = self.fps()
        f = g.is_zero(fs[0] - g.one())
        for x in fs[1:]:
            f = f & g.is_zero(x)
        return f

    def mat(self) -> "Fp12":
        return Fp12(self.c0.mat(), self.c1.mat())


def line_mul_line(l0, l1, l4, m0, m1, m4):
    """(l0 + l1 v + l4 v w)(m0 + m1 v + m4 v w) -> (x: Fp6, y1, y2) (bls_field.h line_mul_line)"""
    p00 = l0 * m0
    p11 = l1 * m1
    p44 = l4 * m4
    x1 = (l0 + l1) * (m0 + m1) - p00 - p11
    y1 = (l0 + l4) * (m0 + m4) - p00 - p44
    y2 = (l1 + l4) * (m1 + m4) - p11 - p44
    x0 = p00 + p44.mul_xi()
    return Fp6(x0, x1, p11), y1, y2


# ---------------------------------------------------------------------------
# Curves: Jacobian points over Fp (G1) or Fp2 (G2); Z == 0 <=> infinity
# ---------------------------------------------------------------------------
class Ops:
    """Field adaptor so the group law is written once (like bls_curve.h's overloads)."""

    def __init__(self, g: Graph, ext: bool):
        self.g, self.ext = g, ext

    def zero(self):
        return Fp2.zero(self.g) if self.ext else self.g.zero()

    def one(self):
        return Fp2.one(self.g) if self.ext else self.g.one()

    def is_zero(self, a) -> Flag:
        return a.is_zero() if self.ext else self.g.is_zero(a)

    def sqr(self, a):
        return a.sqr()

    def dbl(self, a):
        return a.scale(2)

    def sel(self, f, a, b):
        return select(f, a, b)

    def b3(self, a):
        """3b times a, linear: b = 4 on E1, 4 (1 + u) on E2"""
        return a.mul_xi().scale(12) if self.ext else a.scale(12)


class Jac:
    __slots__ = ("X", "Y", "Z")

    def __init__(self, X, Y, Z):
        self.X, self.Y, self.Z = X, Y, Z

    def neg(self) -> "Jac":
        return Jac(self.X, -self.Y, self.Z)


def jsel(flag: Flag, a: Jac, b: Jac) -> Jac:
    return select(flag, a, b)


def jac_inf(F: Ops) -> Jac:
    return Jac(F.one(), F.one(), F.zero())


def jac_dbl(F: Ops, p: Jac) -> Jac:
    """dbl-2009-l (a = 0); Z3 = 2YZ maps infinity to infinity"""
    Z3 = (p.Y * p.Z).scale(2)
    B = p.Y.sqr()
    A = p.X.sqr()
    C = B.sqr()
    D = ((p.X + B).sqr() - A - C).scale(2)
    E = A.scale(3)
    X3 = E.sqr() - D.scale(2)
    Y3 = E * (D - X3) - C.scale(8)
    return Jac(X3, Y3, Z3)


def jac_add(F: Ops, p: Jac, q: Jac, p_inf=None, q_inf=None) -> Jac:
    """add-2007-bl with the exceptional cases as selects (bls_curve.h jac_add_impl):
    P = O -> Q, Q = O -> P, P == Q -> 2P, P == -Q -> O."""
    Z1Z1 = p.Z.sqr()
    Z2Z2 = q.Z.sqr()
    W = (p.Z + q.Z).sqr() - Z1Z1 - Z2Z2
    S1 = p.Y * (q.Z * Z2Z2)
    S2 = q.Y * (p.Z * Z1Z1)
    U1 = p.X * Z2Z2
    U2 = q.X * Z1Z1
    H = U2 - U1
    Rr = S2 - S1
    I = H.scale(2).sqr()
    J = H * I
    V = U1 * I
    R2 = Rr.scale(2)
    X3 = R2.sqr() - J - V.scale(2)
    Y3 = R2 * (V - X3) - (S1 * J).scale(2)
    Z3 = W * H
    gen = Jac(X3, Y3, Z3)
    pi = F.is_zero(p.Z) if p_inf is None else p_inf
    qi = F.is_zero(q.Z) if q_inf is None else q_inf
    h0 = F.is_zero(H)
    r0 = F.is_zero(Rr)
    dbl = jac_dbl(F, p)
    inf = jac_inf(F)
    return select_n([(pi, q), (qi, p), (h0 & r0, dbl), (h0, inf)], gen)


def jac_add_aff(F: Ops, p: Jac, qx, qy, q_inf=None, p_inf=None, skip=None) -> Jac:
    """madd-2007-bl, p Jacobian + q affine, exceptional cases as selects
    (bls_curve.h jac_add_aff_impl); skip (a flag): return p unchanged"""
    Z1Z1 = p.Z.sqr()
    S2 = qy * (p.Z * Z1Z1)
    U2 = qx * Z1Z1
    H = U2 - p.X
    Rr = S2 - p.Y
    HH = H.sqr()
    Z3 = (p.Z + H).sqr() - Z1Z1 - HH
    I = HH.scale(4)
    J = H * I
    V = p.X * I
    R2 = Rr.scale(2)
    X3 = R2.sqr() - J - V.scale(2)
    Y3 = R2 * (V - X3) - (p.Y * J).scale(2)
    gen = Jac(X3, Y3, Z3)
    pi = F.is_zero(p.Z) if p_inf is None else p_inf
    h0 = F.is_zero(H)
    r0 = F.is_zero(Rr)
    dbl = jac_dbl(F, p)
    inf = jac_inf(F)
    cases = []
    if skip is not None:
        cases.append((skip, p))
    if q_inf is not None:
        cases.append((q_inf, p))
    cases += [(pi, Jac(qx, qy, F.one())), (h0 & r0, dbl), (h0, inf)]
    return select_n(cases, gen)


def jac_eq(F: Ops, p: Jac, q: Jac) -> Flag:
    """bls_curve.h jac_eq: both infinity, or equal affine points"""
    pi = F.is_zero(p.Z)
    qi = F.is_zero(q.Z)
    z1z1 = p.Z.sqr()
    z2z2 = q.Z.sqr()
    ex = F.is_zero(p.X * z2z2 - q.X * z1z1)
    ey = F.is_zero(p.Y * (z2z2 * q.Z) - q.Y * (z1z1 * p.Z))
    both = pi & qi
    neither = ~pi & ~qi
    return both | (neither & ex & ey)


# ---------------------------------------------------------------------------
# Homogeneous projective points (x = X / Z, y = Y / Z) with the complete formulas
# of Renes-Costello-Batina for a = 0 (Algorithms 7 and 9 of "Complete addition
# formulas for prime order elliptic curves", 2016).  They have no exceptional
# case on curves without 2-torsion -- E1(Fp) and E2'(Fp2) of BLS12-381 both have
# odd order -- and every output coordinate has degree <= 4 in the inputs, so a
# doubling or an addition takes TWO rounds (the one-lane Jacobian dbl-2009-l
# takes three, madd four plus the selects of its exceptional cases).  3b enters
# linearly (Ops.b3).  The group law is the same as the one-lane code's; the
# representatives differ, which only the affine values (and the pairing, up to
# factors the final exponentiation kills) ever see.
# ---------------------------------------------------------------------------
class Proj:
    __slots__ = ("X", "Y", "Z")

    def __init__(self, X, Y, Z):
        self.X, self.Y, self.Z = X, Y, Z

    def neg(self) -> "Proj":
        return Proj(self.X, -self.Y, self.Z)


def proj_from_jac(p: Jac) -> Proj:
    """(X, Y, Z) Jacobian -> (X Z, Y, Z^3); infinity (Z = 0) -> (0, Y, 0)"""
    return Proj(p.X * p.Z, p.Y, p.Z.sqr() * p.Z)


def proj_to_jac(p: Proj) -> Jac:
    """(X, Y, Z) homogeneous -> (X Z, Y Z^2, Z); infinity stays Z = 0"""
    return Jac(p.X * p.Z, p.Y * p.Z.sqr(), p.Z)


def proj_dbl(F: Ops, p: Proj) -> Proj:
    """X3 = 2XY(Y^2 - 9bZ^2), Y3 = (Y^2 + 9bZ^2)^2 - 108 b^2 Z^4, Z3 = 8Y^3 Z"""
    B = p.Y.sqr()
    C = p.Z.sqr()
    E = F.b3(C)
    Fq = E.scale(3)
    X3 = ((p.X * p.Y) * (B - Fq)).scale(2)
    Y3 = (B + Fq).sqr() - E.sqr().scale(12)
    Z3 = (B * (p.Y * p.Z)).scale(8)
    return Proj(X3, Y3, Z3)


def proj_add(F: Ops, p: Proj, q: Proj) -> Proj:
    """complete addition (RCB Algorithm 7, a = 0): two rounds of products"""
    t0 = p.X * q.X
    t1 = p.Y * q.Y
    t2 = p.Z * q.Z
    t3 = (p.X + p.Y) * (q.X + q.Y) - t0 - t1
    t4 = (p.Y + p.Z) * (q.Y + q.Z) - t1 - t2
    y3 = (p.X + p.Z) * (q.X + q.Z) - t0 - t2
    t0 = t0.scale(3)
    t2 = F.b3(t2)
    Z3 = t1 + t2
    t1 = t1 - t2
    y3 = F.b3(y3)
    X3 = t3 * t1 - t4 * y3
    Y3 = t1 * Z3 + y3 * t0
    Z3 = Z3 * t4 + t0 * t3
    return Proj(X3, Y3, Z3)


def proj_mul_xabs(F: Ops, p: Proj) -> Proj:
    """[|x|]P: 63 doublings and 5 additions, all complete (P = O gives O)"""
    acc = p
    for i in range(62, -1, -1):
        acc = proj_dbl(F, acc)
        if (X_ABS_T >> i) & 1:
            acc = proj_add(F, acc, p)
    return acc


def proj_eq(F: Ops, p: Proj, q: Proj) -> Flag:
    """equal points (both infinity, or X1 Z2 = X2 Z1 and Y1 Z2 = Y2 Z1 with Z != 0)"""
    pi = F.is_zero(p.Z)
    qi = F.is_zero(q.Z)
    ex = F.is_zero(p.X * q.Z - q.X * p.Z)
    ey = F.is_zero(p.Y * q.Z - q.Y * p.Z)
    return (pi & qi) | (~pi & ~qi & ex & ey)


X_ABS_T = 0xD201000000010000
# 2^384 mod p as a raw register: x * R384_RAW / 2^416 takes this domain's x back to the
# one-lane code's Montgomery form (R = 2^384)
R384_RAW = (1 << 384) % 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
