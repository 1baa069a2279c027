"""The latency path's round programs (build-time).

Three programs, all restating the one-lane device algorithms (csrc/bls_hash.h,
bls_curve.h, bls_pairing.h -- themselves pinned to the oracle) so the two paths
agree point for point:

* ``set_program(single)``: one signature set of a request -- hash_to_G2 of the
  signing root, the signature's decompression and G2 subgroup check, and the
  set's factor of the batch equation as a Miller value.  For a 1-set request
  (core verify: blst ``Signature.verify``, reached from
  BN/chain/bls/maybeBatch.ts:38) the pubkey's G1 subgroup check and the pairs
  (pk, H(m)), (-g1, sig).  For a set of a >= 2-set request (blst
  ``verifyMultipleSignatures``, maybeBatch.ts:19) the pairs (r pk, H(m)) and
  (-r g1, sig): e(-g1, sum_i r_i sig_i) = prod_i e(-r_i g1, sig_i), so the
  random scalar multiplies in G1 (a 32-step GLV ladder on Fp) instead of G2,
  and the request's product needs no sum of G2 points before its Miller loop.
* ``mul_program``: the product of two Miller values (the request's product
  tree across its sets' workgroups).
* ``final_program``: final exponentiation == 1 (the request's verdict).
* ``mtail_program(partial)``: the throughput pipeline's merged check of a whole
  call (the worker's merged batch, BN/chain/bls/multithread/worker.ts:41-96):
  S_all = sum_p 2^p G_p from the bucket MSM's 33 bit sums (k_msm.hip), the
  Miller value of (-g1, S_all), times the call's level-product Horner value,
  then the final exponentiation == 1 -- or, for a two-phase (multi-GPU) call,
  the product itself as the shard's partial.
* ``final_lane_program``: final exponentiation == 1 of a one-lane Fp12 (the
  host combine of the shards' partials, lb_gt_check).
"""
from __future__ import annotations

import importlib.util
import os

from .dsl import Flag, Fp, Graph, P, select, select_n
from .tower import (P34, Fp2, Fp6, Fp12, Jac, Ops, Proj, fp2_lex_largest, fp2_sgn0, fp_pow, jac_add, jac_add_aff,
                    proj_add, proj_dbl, proj_eq, proj_from_jac, proj_mul_xabs, proj_to_jac, R384_RAW,
                    jac_dbl, jac_eq, jac_inf, jsel, line_mul_line)

X_ABS = 0xD201000000010000
_CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc")


def _load_constants() -> dict:
    spec = importlib.util.spec_from_file_location("lb_gen_constants", os.path.join(_CSRC, "gen_constants.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.constants()


C = _load_constants()
HALF = (P + 1) // 2


def c2(g: Graph, name: str) -> Fp2:
    return Fp2.const(g, C[name])


# ---------------------------------------------------------------------------
# square roots (bls_field.h fp2_sqrt, bls_hash.h fp2_sqrt_with_norm_root)
# ---------------------------------------------------------------------------
def fp2_sqrt_in_fp(a0: Fp):
    """fp2_sqrt's a.c1 == 0 branch: sqrt(a0) or u sqrt(-a0)"""
    g = a0.g
    c = fp_pow(a0, P34)
    x0 = a0 * c
    t = x0 * c
    is_qr = g.is_zero(t - g.one()) | g.is_zero(a0)
    z = g.zero()
    return Fp2(select(is_qr, x0, z), select(is_qr, z, x0))


def fp2_sqrt_from_norm_root(a: Fp2, s: Fp) -> Fp2:
    g = a.g
    half = g.const(HALF)
    t = (a.c0 + s) * half
    c = fp_pow(t, P34)
    x0 = t * c
    chk = x0.sqr()
    a1c = (a.c1 * c) * half
    direct = g.is_zero(chk - t)
    return Fp2(select(direct, x0, -a1c), select(direct, a1c, x0))


def fp2_sqrt(a: Fp2):
    """(root, is_square) -- bls_field.h fp2_sqrt"""
    g = a.g
    n = a.norm()
    t = fp_pow(n, P34)
    s = t * n
    ok = g.is_zero(s.sqr() - n)
    main = fp2_sqrt_from_norm_root(a, s)
    z1 = g.is_zero(a.c1)
    r = select(z1, fp2_sqrt_in_fp(a.c0), main)
    return r, z1 | ok


# ---------------------------------------------------------------------------
# Square roots in Fp2 from ONE exponentiation (q = p^2 = 9 mod 16), the round
# programs' form: depth ~log2(p) instead of the norm method's two sequential Fp
# exponentiations (bls_field.h fp2_sqrt).  For U / V (V != 0):
#   y0 = U V^3 (U V^7)^c1,  c1 = (q - 9) / 16   =>   y0^2 = (U / V) zeta,
#   zeta = (U / V)^((q-1)/8) an 8th root of unity: a 4th root (1, -1, i, -i) iff
#   U / V is a square, and then sqrt(U / V) = y0 / sqrt(zeta).
# (U V^7)^c1 splits as w^e0 conj(w)^e1 with c1 = e1 p + e0 (w^p = conj(w)), so ONE
# squaring chain of ~381 Fp2 squarings carries both halves (RFC 9380's
# sqrt_ratio for q = 9 mod 16, restated).  Which root comes out does not matter:
# every caller fixes the sign (sgn0 / lex_largest) afterwards.
# ---------------------------------------------------------------------------
def _f2m(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def _f2pow(a, e):
    r = (1, 0)
    while e:
        if e & 1:
            r = _f2m(r, a)
        a = _f2m(a, a)
        e >>= 1
    return r


def _f2inv(a):
    n = pow((a[0] * a[0] + a[1] * a[1]) % P, P - 2, P)
    return (a[0] * n % P, (-a[1]) * n % P)


def _f2sqrt(a):
    """a square root of a in Fp2 (generator time), or None"""
    if a == (0, 0):
        return (0, 0)
    y0 = _f2m(_f2pow(a, (P * P + 7) // 16), (1, 0))
    for eta in _ETA4:
        y = _f2m(y0, eta)
        if _f2m(y, y) == a:
            return y
    return None


_Q = P * P
_C1 = (_Q - 9) // 16
_E1, _E0 = divmod(_C1, P)
_I = (0, 1)
_RHO = None  # a primitive 8th root of unity with rho^2 = i (found below)
for _c in range(2, 200):
    _r = _f2pow((_c, 1), (_Q - 1) // 8)
    if _f2pow(_r, 4) == (P - 1, 0) and _f2m(_r, _r) == _I:
        _RHO = _r
        break
assert _RHO is not None
_ZETA4 = [(1, 0), (P - 1, 0), _I, (0, P - 1)]                      # 1, -1, i, -i
_SQRT4 = [(1, 0), _I, _RHO, _f2pow(_RHO, 3)]                       # their square roots
_ETA4 = [_f2inv(x) for x in _SQRT4]                                 # y = y0 eta
_ZETA8 = [_f2pow(_RHO, k) for k in (1, 3, 5, 7)]                   # primitive 8th roots
for _z, _sq in zip(_ZETA4, _SQRT4):
    assert _f2m(_sq, _sq) == _z


def fp2_pow_c1(w: Fp2) -> Fp2:
    """w^c1 = w^e0 conj(w)^e1: one squaring chain s_i = w^(2^i); the running product
    takes s_i, conj(s_i) or N(s_i) = s_i conj(s_i) (an Fp scalar) per bit pair."""
    g = w.g
    acc = None
    s = w
    nb = max(_E0.bit_length(), _E1.bit_length())
    for i in range(nb):
        a, b = (_E0 >> i) & 1, (_E1 >> i) & 1
        if a or b:
            if a and b:
                n = s.norm()
                acc = Fp2(n, g.zero()) if acc is None else acc * n
            else:
                m = s if a else s.conj()
                acc = m if acc is None else acc * m
        if i + 1 < nb:
            s = s.sqr()
    return acc


def fp2_sqrt_ratio_y0(U: Fp2, V: Fp2 = None):
    """(y0, A): y0 = U V^3 (U V^7)^c1 and A = y0^2 V (= U zeta); V None means 1"""
    if V is None:
        t = fp2_pow_c1(U)
        y0 = U * t
        return y0, y0.sqr()
    V2 = V.sqr()
    V3 = V2 * V
    V4 = V2.sqr()
    V7 = V4 * V3
    t = fp2_pow_c1(U * V7)
    y0 = (U * V3) * t
    return y0, y0.sqr() * V


def fp2_sqrt1(a: Fp2):
    """(root, is_square) of a (the one-exponentiation method; bls_field.h fp2_sqrt's
    contract: which root is unspecified)"""
    y0, A = fp2_sqrt_ratio_y0(a)
    hits = [(A - a * Fp2.const(a.g, z) if z != (1, 0) else A - a).is_zero() for z in _ZETA4]
    root = select_n([(h, y0 * Fp2.const(a.g, eta)) for h, eta in zip(hits[1:], _ETA4[1:])], y0)
    sq = hits[0] | hits[1] | hits[2] | hits[3]
    return root, sq


# ---------------------------------------------------------------------------
# hash_to_G2 (bls_hash.h): SSWU, 3-isogeny, Q0 + Q1, clear_cofactor
# ---------------------------------------------------------------------------
def map_to_curve_sswu_iso(u: Fp2) -> Proj:
    """Simplified SWU onto E2' and the 3-isogeny to E2 with ONE exponentiation and no
    inversion (the device's map_to_g2_sswu_iso, restated for round programs).
    x1 = n / d (n = -B (tv2 + 1), d = A tv2; tv2 = 0: n = B, d = Z A), g(x1) = U / V with
    U = n^3 + A n d^2 + B d^3, V = d^3; y0 = U V^3 (U V^7)^c1 has y0^2 = g(x1) zeta.
    g(x1) a square (zeta a 4th root): y = y0 / sqrt(zeta), x = x1.  Otherwise zeta is
    a primitive 8th root and g(x2) = (Z u^2)^3 g(x1) is the square:
    y = u^3 y0 sqrt(Z^3 / zeta), x = x2 = Z u^2 x1.  The sign of y follows sgn0(u).
    The isogeny is homogenised in (x_n, d) and lands in homogeneous coordinates."""
    g = u.g
    A = c2(g, "LB_SSWU_A")
    B = c2(g, "LB_SSWU_B")
    Z = c2(g, "LB_SSWU_Z")
    tv1 = Z * u.sqr()
    tv2 = tv1.sqr() + tv1
    exceptional = tv2.is_zero()
    n = select(exceptional, B, -(B * (tv2 + Fp2.one(g))))
    d = select(exceptional, Z * A, A * tv2)
    d2 = d.sqr()
    d3 = d2 * d
    U = n * (n.sqr() + A * d2) + B * d3
    y0, Aq = fp2_sqrt_ratio_y0(U, d3)
    hit4 = [(Aq - U * Fp2.const(g, z) if z != (1, 0) else Aq - U).is_zero() for z in _ZETA4]
    sq1 = hit4[0] | hit4[1] | hit4[2] | hit4[3]
    Zc = C["LB_SSWU_Z"]
    z3 = _f2m(_f2m(Zc, Zc), Zc)
    hit8, ys8 = [], []
    u3y0 = (u.sqr() * u) * y0
    for zeta in _ZETA8:
        k = _f2sqrt(_f2m(z3, _f2inv(zeta)))
        if k is None:
            continue
        hit8.append((Aq - U * Fp2.const(g, zeta)).is_zero())
        ys8.append(u3y0 * Fp2.const(g, k))
    # g(x1) a square: hit4[0] (y0 itself) or one of hit4[1:]; else the hit8 case
    y = select(sq1, select_n([(h, y0 * Fp2.const(g, eta)) for h, eta in zip(hit4[1:], _ETA4[1:])], y0),
               select_n([(h, yy) for h, yy in zip(hit8[1:], ys8[1:])], ys8[0]))
    flip = fp2_sgn0(u) ^ fp2_sgn0(y)
    y = select(flip, -y, y)
    xn = select(sq1, n, tv1 * n)
    return iso_map_g2_frac(xn, d, d2, d3, y)


def iso_map_g2_frac(xn: Fp2, d: Fp2, d2: Fp2, d3: Fp2, y: Fp2) -> Proj:
    """the 3-isogeny at x = xn / d: XN = xn(x) d^3, XD = xd(x) d^2, YN = yn(x) d^3,
    YD = yd(x) d^3; x_E = XN / (XD d), y_E = y YN / YD, so
    (X : Y : Z) = (XN YD : y YN XD d : XD d YD); a kernel point -> (0 : 1 : 0)."""
    g = xn.g

    def k(nm):
        return c2(g, nm)
    XN = ((k("LB_ISO_XNUM3") * xn + k("LB_ISO_XNUM2") * d) * xn + k("LB_ISO_XNUM1") * d2) * xn + \
        k("LB_ISO_XNUM0") * d3
    XD = (xn + k("LB_ISO_XDEN1") * d) * xn + k("LB_ISO_XDEN0") * d2
    YN = ((k("LB_ISO_YNUM3") * xn + k("LB_ISO_YNUM2") * d) * xn + k("LB_ISO_YNUM1") * d2) * xn + \
        k("LB_ISO_YNUM0") * d3
    YD = ((xn + k("LB_ISO_YDEN2") * d) * xn + k("LB_ISO_YDEN1") * d2) * xn + k("LB_ISO_YDEN0") * d3
    kern = XD.is_zero() | YD.is_zero()
    XDd = XD * d
    inf = Proj(Fp2.zero(g), Fp2.one(g), Fp2.zero(g))
    return select(kern, inf, Proj(XN * YD, (y * YN) * XDd, XDd * YD))


def map_to_curve_sswu(u: Fp2):
    """Simplified SWU onto E2' (bls_hash.h map_to_curve_sswu) with no inversion on
    its path: x1 = N / D is kept as a fraction, g(x1) = U / D^3 = W / m with
    W = U conj(D^3) and m = N(D^3) in Fp, so the norm exponentiation runs on
    N(g(x1)) = N(W) / m^2 as N(W)^((p-3)/4) * m^((p+1)/2) (two exponentiations in
    parallel; m^(-2 (p-3)/4) = m^((p+1)/2)) while m^-1 = m^(p-2) runs beside them;
    from there on the values -- g(x), the norm root, x, y -- are the affine ones
    of the one-lane code, so the same root and sign come out."""
    g = u.g
    A = c2(g, "LB_SSWU_A")
    B = c2(g, "LB_SSWU_B")
    Z = c2(g, "LB_SSWU_Z")
    tv1 = Z * u.sqr()
    tv2 = tv1.sqr() + tv1
    exceptional = tv2.is_zero()
    # x1 = (-B/A)(1 + 1/tv2) = N / D;  tv2 == 0: x1 = B / (Z A)
    N = select(exceptional, c2(g, "LB_SSWU_B_OVER_ZA"), (tv2 + Fp2.one(g)) * c2(g, "LB_SSWU_MINUS_B_OVER_A"))
    D = select(exceptional, Fp2.one(g), tv2)
    D2 = D.sqr()
    V = D2 * D
    BV = B * V
    N2 = tv1 * N  # x2 = tv1 x1 = N2 / D
    U1 = N * (N.sqr() + A * D2) + BV
    U2 = N2 * (N2.sqr() + A * D2) + BV
    Vc = V.conj()
    W1 = U1 * Vc
    W2 = U2 * Vc
    m = V.norm()
    nW1 = W1.norm()
    e = fp_pow(nW1, P34) * fp_pow(m, (P + 1) // 2)  # = N(g(x1))^((p-3)/4)
    minv = fp_pow(m, P - 2)
    sq1 = g.is_zero(e.sqr() * nW1 - m.sqr()) | g.is_zero(nW1)
    s1 = (nW1 * e) * minv.sqr()
    nu = u.norm()
    nu3 = nu.sqr() * nu
    s2 = (nu3 * g.const(C["LB_SSWU_NZ3_SQRT"])) * s1
    s = select(sq1, s1, s2)
    gx = select(sq1, W1, W2) * minv
    x = (select(sq1, N, N2) * D.conj()) * (D.norm().sqr() * minv)
    # fp2_sqrt_with_norm_root: gx.c1 == 0 takes fp2_sqrt, i.e. its a.c1 == 0 branch
    # (one exponentiation from gx.c0, beside the main one)
    z1 = g.is_zero(gx.c1)
    y_main = fp2_sqrt_from_norm_root(gx, s)
    y = select(z1, fp2_sqrt_in_fp(gx.c0), y_main)
    flip = fp2_sgn0(u) ^ fp2_sgn0(y)
    y = select(flip, -y, y)
    return x, y


def iso_map_g2(x: Fp2, y: Fp2) -> Proj:
    """3-isogeny E2' -> E2 on the affine SSWU output, to homogeneous coordinates:
    (x yn-free) X = xn yd, Y = y yn xd, Z = xd yd; a kernel point -> (0 : 1 : 0)."""
    g = x.g

    def k(n):
        return c2(g, n)

    xn = ((k("LB_ISO_XNUM3") * x + k("LB_ISO_XNUM2")) * x + k("LB_ISO_XNUM1")) * x + k("LB_ISO_XNUM0")
    xd = (x + k("LB_ISO_XDEN1")) * x + k("LB_ISO_XDEN0")
    yn = ((k("LB_ISO_YNUM3") * x + k("LB_ISO_YNUM2")) * x + k("LB_ISO_YNUM1")) * x + k("LB_ISO_YNUM0")
    yd = ((x + k("LB_ISO_YDEN2")) * x + k("LB_ISO_YDEN1")) * x + k("LB_ISO_YDEN0")
    kern = xd.is_zero() | yd.is_zero()
    Z = xd * yd
    X = xn * yd
    Y = (y * yn) * xd
    inf = Proj(Fp2.zero(g), Fp2.one(g), Fp2.zero(g))
    return select(kern, inf, Proj(X, Y, Z))


def g2_psi(p):
    """psi(x, y) = (conj(x) cx, conj(y) cy): the same map on Jacobian and homogeneous
    coordinates (conj(X) cx / conj(Z)^k for either weight k)"""
    g = p.X.g
    return type(p)(p.X.conj() * c2(g, "LB_PSI_CX"), p.Y.conj() * c2(g, "LB_PSI_CY"), p.Z.conj())


def jac_mul_xabs(F: Ops, p: Jac, p_inf: Flag = None) -> Jac:
    """[|x|]P on the shared-Z curve (bls_curve.h jac_mul_xabs): 63 doublings and
    5 mixed additions of (X, Y); the result's Z times P's Z."""
    qx, qy = p.X, p.Y
    acc = Jac(qx, qy, F.one())
    for i in range(62, -1, -1):
        acc = jac_dbl(F, acc)
        if (X_ABS >> i) & 1:
            acc = jac_add_aff(F, acc, qx, qy)
    acc = Jac(acc.X, acc.Y, acc.Z * p.Z)
    if p_inf is None:
        p_inf = F.is_zero(p.Z)
    return jsel(p_inf, p, acc)


def clear_cofactor_g2(p: Proj) -> Proj:
    """RFC 9380 G.3 (h_eff via psi, bls_hash.h clear_cofactor_g2) with complete
    homogeneous additions: A = [z]P, B = psi(P) - A, D = psi^2(2P) - P - B, h = D - [z]B"""
    F = Ops(p.X.g, True)
    A = proj_mul_xabs(F, p)
    B = proj_add(F, g2_psi(p), A.neg())
    t = g2_psi(g2_psi(proj_dbl(F, p)))
    t = proj_add(F, t, p.neg())
    D = proj_add(F, t, B.neg())
    C = proj_mul_xabs(F, B)
    return proj_add(F, D, C.neg())


def hash_to_g2(u0: Fp2, u1: Fp2) -> Proj:
    q = [map_to_curve_sswu_iso(u) for u in (u0, u1)]
    F = Ops(u0.g, True)
    return clear_cofactor_g2(proj_add(F, q[0], q[1]))


# ---------------------------------------------------------------------------
# subgroup checks (bls_curve.h)
# ---------------------------------------------------------------------------
def g2_in_subgroup(p: Proj, p_inf: Flag) -> Flag:
    """psi(P) == [x]P (bls_curve.h g2_in_subgroup), complete homogeneous ladder"""
    F = Ops(p.X.g, True)
    xp = proj_mul_xabs(F, p).neg()
    return p_inf | proj_eq(F, g2_psi(p), xp)


def g1_in_subgroup(p: Jac, p_inf: Flag) -> Flag:
    """phi(P) == [x^2]P... as bls_curve.h g1_in_subgroup: beta X == -[|x|][|x|]P"""
    g = p.X.g
    F = Ops(g, False)
    q = proj_from_jac(p)
    t = proj_mul_xabs(F, proj_mul_xabs(F, q)).neg()
    ph = Proj(q.X * g.const(C["LB_G1_BETA"]), q.Y, q.Z)
    return p_inf | proj_eq(F, ph, t)


# ---------------------------------------------------------------------------
# [a + b lambda] P on G1 (bls_curve.h jac_mul_glv_xy, shared-Z ladder)
# ---------------------------------------------------------------------------
def g1_glv_mul(p: Jac, a_bits, b_bits) -> Jac:
    """a_bits / b_bits: flags of the 32-bit halves, most significant first."""
    g = p.X.g
    F = Ops(g, False)
    X, Y = p.X, p.Y
    wX = X * g.const(C["LB_G1_BETA"])
    w2X = X * g.const(C["LB_G1_BETA2"])
    acc = jac_inf(F)
    for a, b in zip(a_bits, b_bits):
        acc = jac_dbl(F, acc)
        s1 = a & ~b
        s2 = ~a & b
        s3 = a & b
        nz = a | b
        qx = g.select_n([(s1, X), (s2, wX)], w2X)
        qy = select(s3, -Y, Y)
        acc = jac_add_aff(F, acc, qx, qy, skip=~nz)
    out = Jac(acc.X, acc.Y, acc.Z * p.Z)
    return jsel(F.is_zero(p.Z), p, out)


# ---------------------------------------------------------------------------
# Miller loop of two pairs sharing f (bls_pairing.h miller_dbl_step / miller_add_step)
# with both points projective: no inversion ahead of the loop.
#   P Jacobian (Xp, Yp, Zp): xp = Xp/Zp^2, yp = Yp/Zp^3 -- every line times Zp^3
#     (an Fp scalar) uses (Xp Zp, Yp, Zp^3) instead of (xp, yp, 1);
#   Q Jacobian (X, Y, Z) -> homogeneous (X Z, Y, Z^3) = (Xq, Yq, Zq); the chord of
#     T + Q with th' = Y Zq - Yq Z, la' = X Zq - Xq Z (Zq times the affine-Q
#     values) is the affine-Q chord times Zq^2 (an Fp2 scalar), and with T scaled
#     by Zq the point formulas give Zq^4 times the affine-Q result (the same point).
# Both scalings are killed by the final exponentiation.
# ---------------------------------------------------------------------------
def miller_dbl_step(T, P):
    X, Y, Z = T
    xpz, yp, zp3 = P
    XX = X.sqr()
    Bq = Y.sqr()
    Cq = Z.sqr()
    E = Cq.mul_xi().scale(12)
    Fq = E.scale(3)
    XY = X * Y
    H = (Y + Z).sqr() - Bq - Cq
    l0 = Bq - E
    if zp3 is not None:
        l0 = l0 * zp3
    l1 = -(XX.scale(3) * xpz)
    l4 = H * yp
    X2 = (XY * (Bq - Fq)).scale(2)
    Y2 = (Bq + Fq).sqr() - E.sqr().scale(12)
    Z2 = (Bq * H).scale(4)
    return (X2, Y2, Z2), (l0, l1, l4)


def miller_add_step(T, Q, P):
    X, Y, Z = T
    Xq, Yq, Zq = Q
    xpz, yp, zp3 = P
    if Zq is None:  # affine Q
        th = Y - Yq * Z
        la = X - Xq * Z
        Xs, Ys, Zs = X, Y, Z
        l1 = -(th * xpz)
        l4 = la * yp
    else:
        th = Y * Zq - Yq * Z
        la = X * Zq - Xq * Z
        Xs, Ys, Zs = X * Zq, Y * Zq, Z * Zq
        l1 = -((th * Zq) * xpz)
        l4 = (la * Zq) * yp
    l0 = th * Xq - la * Yq
    if zp3 is not None:
        l0 = l0 * zp3
    Cq = th.sqr()
    D = la.sqr()
    E = la * D
    Fq = Zs * Cq
    G = Xs * D
    H = E + Fq - G.scale(2)
    X2 = la * H
    Y2 = th * (G - H) - Ys * E
    Z2 = Zs * E
    return (X2, Y2, Z2), (l0, l1, l4)


def unit_line(g, void: Flag, line):
    one = Fp2.one(g)
    zero = Fp2.zero(g)
    return (select(void, one, line[0]), select(void, zero, line[1]), select(void, zero, line[2]))


def g1_line_point(p: Jac):
    """(Xp Zp, Yp, Zp^3) of a Jacobian G1 point (zp3 None when Zp is the constant 1)"""
    if p.Z.t == p.X.g.one().t:
        return (p.X, p.Y, None)
    return (p.X * p.Z, p.Y, p.Z.sqr() * p.Z)


def g2_homogeneous(q):
    """(X Z, Y, Z^3) of a Jacobian G2 point (affine: Zq None); a homogeneous one as is"""
    g = q.X.g
    if isinstance(q, Proj):
        return (q.X, q.Y, q.Z)
    if q.Z.c0.t == g.one().t and not q.Z.c1.t:
        return (q.X, q.Y, None)
    return (q.X * q.Z, q.Y, q.Z.sqr() * q.Z)


MILLER_GROUP = 1  # (> 1: the grouped f-chain; rows-bound at 32 rows)


def miller2(pairs, group: int = MILLER_GROUP) -> Fp12:
    """miller2's value with a shorter f-chain: the Horner recurrence f <- f^2 S_t
    (S_t the step's two lines multiplied, line_mul_line) is regrouped by `group`
    consecutive steps, f_end = f_start^(2^d) M with M = the group's lines combined by
    the same Horner rule -- computed beside the chain as the T-chains deliver the
    lines.  The chain itself is then d squarings and ONE product per group (2 rounds
    per squaring, 2 per product) instead of a squaring and a sparse product per step;
    squaring distributes over the product, so the value is the same Fp12 element."""
    if group <= 1:
        return miller2_horner(pairs)
    g = pairs[0][0].X.g
    Ps = [g1_line_point(p) for p, _, _ in pairs]
    Qs = [g2_homogeneous(q) for _, q, _ in pairs]
    Ts = [(q[0], q[1], q[2] if q[2] is not None else Fp2.one(g)) for q in Qs]
    # events (is_dbl, x, y1, y2) in loop order
    events = []
    for i in range(62, -1, -1):
        lines = []
        for k, (_, _, void) in enumerate(pairs):
            Ts[k], ln = miller_dbl_step(Ts[k], Ps[k])
            lines.append(unit_line(g, void, ln))
        events.append((True,) + line_mul_line(*lines[0], *lines[1]))
        if (X_ABS >> i) & 1:
            lines = []
            for k, (_, _, void) in enumerate(pairs):
                Ts[k], ln = miller_add_step(Ts[k], Qs[k], Ps[k])
                lines.append(unit_line(g, void, ln))
            events.append((False,) + line_mul_line(*lines[0], *lines[1]))

    def sparse(x, y1, y2):
        return Fp12(x, Fp6(Fp2.zero(g), y1, y2))
    # the first event starts f (f = 1 before it: its squaring is void)
    f = sparse(*events[0][1:]).mat()
    rest = events[1:]
    for s0 in range(0, len(rest), group):
        grp = rest[s0:s0 + group]
        M, d = None, 0
        for is_dbl, x, y1, y2 in grp:
            if M is None:
                M = sparse(x, y1, y2).mat()
            elif is_dbl:
                M = M.sqr().mat().mul_sparse2(x, y1, y2).mat()
            else:
                M = M.mul_sparse2(x, y1, y2).mat()
            d += 1 if is_dbl else 0
        for _ in range(d):
            f = f.sqr().mat()
        f = (f * M).mat()
    return f.conj()


def miller2_horner(pairs) -> Fp12:
    """prod over two pairs (P: Jacobian G1, Q: Jacobian G2, void) of f_{|x|,Q}(P),
    conjugated (x < 0), up to factors the final exponentiation kills.  A void pair
    (an infinite point) contributes unit lines."""
    g = pairs[0][0].X.g
    Ps = [g1_line_point(p) for p, _, _ in pairs]
    Qs = [g2_homogeneous(q) for _, q, _ in pairs]
    Ts = [(q[0], q[1], q[2] if q[2] is not None else Fp2.one(g)) for q in Qs]
    f = None
    for i in range(62, -1, -1):
        lines = []
        for k, (_, _, void) in enumerate(pairs):
            Ts[k], ln = miller_dbl_step(Ts[k], Ps[k])
            lines.append(unit_line(g, void, ln))
        x, y1, y2 = line_mul_line(*lines[0], *lines[1])
        if f is None:
            # f = l1 l2 as a full Fp12: (x0 + x1 v + x2 v^2) + (y1 v + y2 v^2) w
            f = Fp12(x, Fp6(Fp2.zero(g), y1, y2))
        else:
            f = f.sqr().mat().mul_sparse2(x, y1, y2).mat()
        if (X_ABS >> i) & 1:
            lines = []
            for k, (_, _, void) in enumerate(pairs):
                Ts[k], ln = miller_add_step(Ts[k], Qs[k], Ps[k])
                lines.append(unit_line(g, void, ln))
            x, y1, y2 = line_mul_line(*lines[0], *lines[1])
            f = f.mul_sparse2(x, y1, y2).mat()
    return f.conj()


# ---------------------------------------------------------------------------
# final exponentiation (bls_pairing.h final_exp): f^(3 (p^12 - 1)/r)
# ---------------------------------------------------------------------------
def _gam(k):
    return {e: C["LB_FROB%d_%d" % (k, e)] for e in range(1, 6)}


def fp12_exp_x(a: Fp12) -> Fp12:
    """a^x (x < 0) for cyclotomic a: 63 squarings, one round each -- every
    squaring consumes the previous one's output as forms over its products and
    the materialized value before it, materialized meanwhile (cyc_sqr's lin).
    Right to left: the five products by a^(2^i) (the set bits of |x| below the
    top) run beside the squaring chain instead of inside it."""
    s = a
    s_mat = a
    acc = None
    top = X_ABS.bit_length() - 1
    for i in range(top + 1):
        if (X_ABS >> i) & 1:
            acc = s_mat if acc is None else (acc * s_mat).mat()
        if i < top:
            s = s.cyc_sqr(s_mat)
            s_mat = s.mat()
    return acc.conj()


def final_exp(f: Fp12) -> Fp12:
    t0 = f.conj() * f.inv()
    t0 = t0.mat()
    f2 = (t0.frob(2, _gam(2)) * t0).mat()
    a = (fp12_exp_x(f2) * f2.conj()).mat()
    a = (fp12_exp_x(a) * a.conj()).mat()
    b = (fp12_exp_x(a) * a.frob(1, _gam(1))).mat()
    t0 = fp12_exp_x(fp12_exp_x(b))
    c = (t0 * b.frob(2, _gam(2))).mat()
    c = (c * b.conj()).mat()
    t0 = (f2.cyc_sqr().mat() * f2).mat()
    return c * t0


# ---------------------------------------------------------------------------
# programs
# ---------------------------------------------------------------------------
SET_INPUTS = ["u0c0", "u0c1", "u1c0", "u1c1", "sx0", "sx1", "sy0", "sy1", "pkX", "pkY", "pkZ"]
SET_FLAGS = ["sig_inf", "sig_sign", "sig_comp"] + ["a%d" % i for i in range(32)] + ["b%d" % i for i in range(32)]


def set_program(single: bool) -> Graph:
    g = Graph("set_single" if single else "set_batch")
    v = {n: g.input(n) for n in SET_INPUTS}
    fl = {n: g.input_flag(n) for n in SET_FLAGS}
    F1 = Ops(g, False)
    F2 = Ops(g, True)
    # hash_to_G2 of the signing root (hash_to_field done by the input stage)
    H = hash_to_g2(Fp2(v["u0c0"], v["u0c1"]), Fp2(v["u1c0"], v["u1c1"]))
    # Signature.fromBytes(validate=true): decompression / on-curve, G2 subgroup
    sx = Fp2(v["sx0"], v["sx1"])
    rhs = sx.sqr() * sx + c2(g, "LB_B2")
    yc, sq = fp2_sqrt1(rhs)
    flip = fp2_lex_largest(yc) ^ fl["sig_sign"]
    yc = select(flip, -yc, yc)
    yu = Fp2(v["sy0"], v["sy1"])
    on_u = (yu.sqr() - rhs).is_zero()
    comp = fl["sig_comp"]
    sy = select(comp, yc, yu)
    on_curve = (comp & sq) | (~comp & on_u)
    sig_inf = fl["sig_inf"]
    sig = Jac(sx, sy, Fp2.one(g))
    in_group = g2_in_subgroup(Proj(sx, sy, Fp2.one(g)), sig_inf)
    pk = Jac(v["pkX"], v["pkY"], v["pkZ"])
    pk_inf = g.is_zero(v["pkZ"])
    g1x = g.const(C["LB_G1_X"])
    g1ny = g.const(C["LB_G1_NEG_Y"])
    if single:
        pk_ok = g1_in_subgroup(pk, pk_inf)
        P1 = pk
        P2 = None  # (-g1) affine
    else:
        pk_ok = None
        a = [fl["a%d" % i] for i in range(32)]
        b = [fl["b%d" % i] for i in range(32)]
        P1 = g1_glv_mul(pk, a, b)
        P2 = g1_glv_mul(Jac(g1x, g1ny, g.one()), a, b)
    # the Miller loop takes every point projective (no inversion)
    if P2 is None:
        P2 = Jac(g1x, g1ny, g.one())
        p2_inf = Flag(g, None, False)
    else:
        p2_inf = g.is_zero(P2.Z)
    void1 = g.is_zero(P1.Z) | H.Z.is_zero()
    void2 = sig_inf | p2_inf
    f = miller2([(P1, H, void1), (P2, sig, void2)])
    for k, x in enumerate(f.fps()):
        g.output("f%d" % k, x, canonical=True)  # (the next program's inputs are canonical)
    g.output_flag("on_curve", on_curve)
    g.output_flag("in_group", in_group)
    if pk_ok is not None:
        g.output_flag("pk_in_group", pk_ok)
    return g


def mul_program() -> Graph:
    g = Graph("fp12_mul")
    a = Fp12.from_fps([g.input_raw("a%d" % k) for k in range(12)])
    b = Fp12.from_fps([g.input_raw("b%d" % k) for k in range(12)])
    for k, x in enumerate((a * b).fps()):
        g.output("f%d" % k, x, canonical=True)  # (the next program's inputs are canonical)
    return g


def final_program() -> Graph:
    g = Graph("final_exp")
    f = Fp12.from_fps([g.input_raw("f%d" % k) for k in range(12)])
    g.output_flag("is_one", final_exp(f).is_one())
    return g


# ---------------------------------------------------------------------------
# the throughput pipeline's merged check (bls_host.hip run_pipeline, steps + MSM)
# ---------------------------------------------------------------------------
MSM_POS = 33  # k_msm.hip LB_MSM_POS: bit positions of the MSM's reduction


def miller1(q: Proj, void: Flag) -> Fp12:
    """Miller value of the one pair (-g1, Q), Q homogeneous (conj(f_{|x|,Q}(-g1)), x < 0),
    up to factors the final exponentiation kills; void (Q = O): 1.  -g1 is a constant
    affine point, so its line coordinates enter as constants."""
    g = q.X.g
    P1 = g1_line_point(Jac(g.const(C["LB_G1_X"]), g.const(C["LB_G1_NEG_Y"]), g.one()))
    Q = g2_homogeneous(q)
    T = Q
    f = None
    for i in range(62, -1, -1):
        T, ln = miller_dbl_step(T, P1)
        l0, l1, l4 = unit_line(g, void, ln)
        if f is None:
            f = Fp12(Fp6(l0, l1, Fp2.zero(g)), Fp6(Fp2.zero(g), l4, Fp2.zero(g)))
        else:
            f = f.sqr().mat().mul_line(l0, l1, l4).mat()
        if (X_ABS >> i) & 1:
            T, ln = miller_add_step(T, Q, P1)
            f = f.mul_line(*unit_line(g, void, ln)).mat()
    return f.conj()


def msm_sum(pts) -> Proj:
    """sum_p 2^p G_p (Horner from the top position), complete homogeneous formulas"""
    F = Ops(pts[0].X.g, True)
    acc = pts[-1]
    for p in range(len(pts) - 2, -1, -1):
        acc = proj_add(F, proj_dbl(F, acc), pts[p])
    return acc


def miller1_levels(q: Proj, void: Flag, P) -> Fp12:
    """conj(prod_l (P_l * lines_l)^(2^(62 - l))): the call's 63 level products P_l
    (k_level_prod: the good requests' lane values of level l) folded into the Miller loop
    of the one pair (-g1, Q) -- the value k_horner_all's Horner chain times miller1(q,
    void), with ONE squaring chain for both (conj is multiplicative).  P_l times its
    level's lines is formed beside the chain (the lines depend on the T-chain only), so
    a level costs the chain one squaring and one product."""
    g = q.X.g
    P1 = g1_line_point(Jac(g.const(C["LB_G1_X"]), g.const(C["LB_G1_NEG_Y"]), g.one()))
    Q = g2_homogeneous(q)
    T = Q
    f = None
    for lvl, i in enumerate(range(62, -1, -1)):
        T, ln = miller_dbl_step(T, P1)
        m = P[lvl].mul_line(*unit_line(g, void, ln)).mat()
        if (X_ABS >> i) & 1:
            T, ln = miller_add_step(T, Q, P1)
            m = m.mul_line(*unit_line(g, void, ln)).mat()
        f = m if f is None else (f.sqr().mat() * m).mat()
    return f.conj()


MTAIL_LEVELS = 63  # k_steps.hip: the Horner levels of the step-major accumulation
MTAIL_INPUTS = ["P%d_%d" % (lvl, k) for lvl in range(MTAIL_LEVELS) for k in range(12)] + [
    "G%d_%s" % (p, c) for p in range(MSM_POS) for c in ("X0", "X1", "Y0", "Y1", "Z0", "Z1")]


def mtail_program(partial: bool) -> Graph:
    """inputs: the call's 63 level products P_l over its good requests' lane values
    (k_level_prod) and the MSM's 33 bit sums G_p (Jacobian G2, one-lane Montgomery form);
    S_all = sum 2^p G_p; f = conj(Horner over l of P_l) * Miller(-g1, S_all), the Horner
    chain and the Miller loop's squarings shared (miller1_levels: k_horner_all folded in).
    check: output flag is_one = (final_exp(f) == 1).  partial: f as 12 canonical Fp in
    the one-lane form (R = 2^384), the shard's 576-byte partial before encoding."""
    g = Graph("mtail_partial" if partial else "mtail_check")
    # (the level products come converted to this domain by k_mtail_prep: no conversion unit
    # per input, and no register held by a raw input until its conversion)
    n_p = 12 * MTAIL_LEVELS
    v = [g.input_raw(n) if k < n_p else g.input(n) for k, n in enumerate(MTAIL_INPUTS)]
    P = [Fp12.from_fps(v[12 * lvl:12 * lvl + 12]) for lvl in range(MTAIL_LEVELS)]
    o = 12 * MTAIL_LEVELS
    pts = []
    zero, one = Fp2.zero(g), Fp2.one(g)
    for p in range(MSM_POS):
        X, Y, Z = (Fp2(v[o + 6 * p + 2 * c], v[o + 6 * p + 2 * c + 1]) for c in range(3))
        pts.append(select(Z.is_zero(), Proj(zero, one, zero), proj_from_jac(Jac(X, Y, Z))))
    S = msm_sum(pts)
    f = miller1_levels(S, S.Z.is_zero(), P).mat()
    if partial:
        r384 = g.const_raw(R384_RAW)  # x * R384 / R416: back to the one-lane form
        for k, x in enumerate(f.fps()):
            g.output("f%d" % k, x * r384, canonical=True)
    else:
        g.output_flag("is_one", final_exp(f).is_one())
    return g


SIG_DECODE_INPUTS = ["sx0", "sx1", "sy0", "sy1"]
SIG_DECODE_FLAGS = ["sig_inf", "sig_sign", "sig_comp"]


def sig_decode_program() -> Graph:
    """Signature.fromBytes(validate=true)'s curve arithmetic for a small same-message package
    (bls_host.hip; k_decode_sigs' one-lane chain, ~4 ms, as ~540 rounds on an 8-row workgroup):
    inputs x (and y, uncompressed) in the one-lane form and the encoding's flags as
    k_sm_dec_prep parsed them; outputs y in the one-lane form (the compressed point's root
    with the sign rule, or the given y) and the flags on_curve and in_group -- the same
    formulas as set_program's decompression."""
    g = Graph("sig_decode")
    v = {n: g.input(n) for n in SIG_DECODE_INPUTS}
    fl = {n: g.input_flag(n) for n in SIG_DECODE_FLAGS}
    sx = Fp2(v["sx0"], v["sx1"])
    rhs = sx.sqr() * sx + c2(g, "LB_B2")
    yc, sq = fp2_sqrt1(rhs)
    flip = fp2_lex_largest(yc) ^ fl["sig_sign"]
    yc = select(flip, -yc, yc)
    yu = Fp2(v["sy0"], v["sy1"])
    on_u = (yu.sqr() - rhs).is_zero()
    comp = fl["sig_comp"]
    sy = select(comp, yc, yu)
    on_curve = (comp & sq) | (~comp & on_u)
    in_group = g2_in_subgroup(Proj(sx, sy, Fp2.one(g)), fl["sig_inf"])
    r384 = g.const_raw(R384_RAW)  # x * R384 / R416: back to the one-lane form
    g.output("y0", sy.c0 * r384, canonical=True)
    g.output("y1", sy.c1 * r384, canonical=True)
    g.output_flag("on_curve", on_curve)
    g.output_flag("in_group", in_group)
    return g


def hash_finish_program() -> Graph:
    """hash_to_G2's second half for a lone mid-size call (k_hash_finish's one-lane chain, ~4.7 ms,
    as ~300 rounds on a 16-row workgroup): inputs Q0, Q1 (the two mapped points, Jacobian, one-lane
    form, as k_hash_half writes them; Z = 0 is infinity); output H = clear_cofactor(Q0 + Q1),
    Jacobian in the one-lane form (k_lines_rows' input)."""
    g = Graph("hash_finish")
    F = Ops(g, True)
    zero, one = Fp2.zero(g), Fp2.one(g)
    pts = []
    for i in range(2):
        X, Y, Z = (Fp2(g.input("Q%d_%s0" % (i, c)), g.input("Q%d_%s1" % (i, c))) for c in "XYZ")
        pts.append(select(Z.is_zero(), Proj(zero, one, zero), proj_from_jac(Jac(X, Y, Z))))
    J = proj_to_jac(clear_cofactor_g2(proj_add(F, pts[0], pts[1])))
    r384 = g.const_raw(R384_RAW)  # x * R384 / R416: back to the one-lane form
    for v, c in ((J.X, "X"), (J.Y, "Y"), (J.Z, "Z")):
        g.output("H_%s0" % c, v.c0 * r384, canonical=True)
        g.output("H_%s1" % c, v.c1 * r384, canonical=True)
    return g


def hash_full_program() -> Graph:
    """The whole hash_to_G2 curve part for a lone mid-size call (k_hash_half's SSWU + isogeny
    chains and k_hash_finish's cofactor clearing as ONE program, k_lp_hash): inputs u0, u1 (the
    hash_to_field outputs, one-lane Montgomery form, as k_lp_prep writes them); output
    H = clear_cofactor(map(u0) + map(u1)), Jacobian in the one-lane form."""
    g = Graph("hash_full")
    u = [Fp2(g.input("u%dc0" % i), g.input("u%dc1" % i)) for i in range(2)]
    J = proj_to_jac(hash_to_g2(u[0], u[1]))
    r384 = g.const_raw(R384_RAW)  # x * R384 / R416: back to the one-lane form
    for v, c in ((J.X, "X"), (J.Y, "Y"), (J.Z, "Z")):
        g.output("H_%s0" % c, v.c0 * r384, canonical=True)
        g.output("H_%s1" % c, v.c1 * r384, canonical=True)
    return g


def lines_program() -> Graph:
    """The 68 Miller lines of one pair (r pk, H) for a lone mid-size call (k_lines_rows' one-lane
    T-chain, ~3.3 ms, as ~210 rounds on a 16-row workgroup): inputs P (Jacobian G1) and H
    (Jacobian G2) in the one-lane form; outputs the 68 lines (l0, l1, l4) in loop order, one-lane
    form, as k_lines_rows stores them -- up to Fp2 factors (P and H stay projective: no
    inversion), which the final exponentiation removes; an infinite P or H gives unit lines."""
    g = Graph("lines")
    P = Jac(*(g.input("P_%s" % c) for c in "XYZ"))
    X, Y, Z = (Fp2(g.input("H_%s0" % c), g.input("H_%s1" % c)) for c in "XYZ")
    void = g.is_zero(P.Z) | Z.is_zero()
    Pl = g1_line_point(P)
    Q = g2_homogeneous(Jac(X, Y, Z))
    T = Q
    r384 = g.const_raw(R384_RAW)  # x * R384 / R416: back to the one-lane form
    lines = []
    for i in range(62, -1, -1):
        T, ln = miller_dbl_step(T, Pl)
        lines.append(ln)
        if (X_ABS >> i) & 1:
            T, ln = miller_add_step(T, Q, Pl)
            lines.append(ln)
    for j, ln in enumerate(lines):
        for k, v in enumerate(unit_line(g, void, ln)):
            g.output("L%d_%d0" % (j, k), v.c0 * r384, canonical=True)
            g.output("L%d_%d1" % (j, k), v.c1 * r384, canonical=True)
    return g


MSM_BITS_GROUP = 8  # k_msm.hip: bucket sums per instance of the lone call's bit-sum programs


def msm_bits_program(level: int) -> Graph:
    """A lone call's bit sums G_p = sum of window w's bucket sums B_d with bit k of d set
    (p = 11 w + k), as a tree of round programs over groups of MSM_BITS_GROUP points
    (bls_host.hip run_pipeline; k_msm_bits' 9 dependent one-lane Jacobian additions, ~0.8 ms,
    become three launches of ~10-16 rounds).  level 0: Jacobian points in the one-lane form
    (the bucket sums; Z = 0 is infinity) -> their sum, homogeneous, this domain; level 1:
    homogeneous -> homogeneous; level 2: homogeneous -> Jacobian in the one-lane form (what
    the merged-check program takes as its G_p).  Complete additions (proj_add): no
    exceptional case, infinity included."""
    g = Graph("msm_bits_%d" % level)
    F = Ops(g, True)
    zero, one = Fp2.zero(g), Fp2.one(g)
    pts = []
    for i in range(MSM_BITS_GROUP):
        if level == 0:
            X, Y, Z = (Fp2(g.input("P%d_%s0" % (i, c)), g.input("P%d_%s1" % (i, c))) for c in "XYZ")
            pts.append(select(Z.is_zero(), Proj(zero, one, zero), proj_from_jac(Jac(X, Y, Z))))
        else:
            X, Y, Z = (Fp2(g.input_raw("P%d_%s0" % (i, c)), g.input_raw("P%d_%s1" % (i, c))) for c in "XYZ")
            pts.append(Proj(X, Y, Z))
    while len(pts) > 1:
        pts = [proj_add(F, pts[i], pts[i + 1]) if i + 1 < len(pts) else pts[i] for i in range(0, len(pts), 2)]
    S = pts[0]
    if level == 2:
        J = proj_to_jac(S)
        r384 = g.const_raw(R384_RAW)  # x * R384 / R416: back to the one-lane form
        outs = [(J.X, "X"), (J.Y, "Y"), (J.Z, "Z")]
        for v, c in outs:
            g.output("S_%s0" % c, v.c0 * r384, canonical=True)
            g.output("S_%s1" % c, v.c1 * r384, canonical=True)
    else:
        for v, c in ((S.X, "X"), (S.Y, "Y"), (S.Z, "Z")):
            g.output("S_%s0" % c, v.c0, canonical=True)
            g.output("S_%s1" % c, v.c1, canonical=True)
    return g


RTAIL_INPUTS = ["F%d" % k for k in range(12)] + ["S_x0", "S_x1", "S_y0", "S_y1"]


def rtail_program() -> Graph:
    """One request's tail after a failed merged check (the per-request re-verification,
    worker.ts:74-85): inputs F_k (its Miller value, one-lane fp12) and S_k = sum r_i sigma_i
    (affine G2, one-lane form; input flag S_inf: S_k = O); output flag is_one =
    (final_exp(F_k * Miller(-g1, S_k)) == 1) -- k_lines_S + k_tail's one-wave chain as one
    round program per request (k_lp_rtail)."""
    g = Graph("rtail_check")
    v = [g.input(n) for n in RTAIL_INPUTS]
    s_inf = g.input_flag("S_inf")
    F = Fp12.from_fps(v[:12])
    S = Proj(Fp2(v[12], v[13]), Fp2(v[14], v[15]), Fp2.one(g))
    f = (F * miller1(S, s_inf)).mat()
    g.output_flag("is_one", final_exp(f).is_one())
    return g


def final_lane_program() -> Graph:
    """final exponentiation == 1 of a one-lane Fp12 (canonical, R = 2^384)"""
    g = Graph("final_exp_lane")
    f = Fp12.from_fps([g.input("f%d" % k) for k in range(12)])
    g.output_flag("is_one", final_exp(f).is_one())
    return g
