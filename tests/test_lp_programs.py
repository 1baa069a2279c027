"""CPU checks of the latency path's round programs (lodestar_amd/lpgen): every
program is compiled exactly as the build does and executed by the big-integer
executor of its ENCODED words (lpgen.compile.Program.run: the device's
arithmetic, value bounds asserted), against the oracle: hash_to_G2 inside the
set programs (through the Miller value's final exponentiation), decompression
and subgroup flags, core verify and the batch form with a random scalar, the
Fp12 product and the final exponentiation."""
import functools

import pytest

from lodestar_amd.lpgen import bls, compile as lpc
from oracle import bls12_381 as O
from tests.lp_helper import P, f12_fps, f12_from_out, mont, mont416, sample_sets, set_inputs


@functools.lru_cache(maxsize=None)
def prog(name):
    g = {"single": lambda: bls.set_program(True), "batch": lambda: bls.set_program(False),
         "mul": bls.mul_program, "final": bls.final_program}[name]()
    return lpc.compile_graph(g, rows=32)


def run_set(single, pk, msg, sig, raw=0):
    fps, flags = set_inputs(pk, msg, sig, raw)
    outs, oflags = prog("single" if single else "batch").run([mont(v) for v in fps], flags)
    return f12_from_out(outs), oflags


def test_program_shapes():
    for name in ("single", "batch", "mul", "final"):
        p = prog(name)
        assert p.stats["regs"] <= 1024 and p.stats["flags"] <= 512
    assert prog("single").n_rounds < 2600 and prog("final").n_rounds < 520


def test_final_exp_program():
    one = O.f12_mul(O.miller_loop(O.G1, O.G2), O.miller_loop(O.E1.neg(O.G1), O.G2))
    not_one = O.miller_loop(O.G1, O.G2)
    for f, want in ((one, 1), (not_one, 0)):
        _, fl = prog("final").run([mont416(v) for v in f12_fps(f)], [])
        assert fl == [want]
        assert bool(want) == O.f12_is_one(O.final_exp(f))


def test_mul_program():
    a = O.miller_loop(O.G1, O.G2)
    b = O.miller_loop(O.g1_mul(O.G1, 5), O.G2)
    outs, _ = prog("mul").run([mont416(v) for v in f12_fps(a) + f12_fps(b)], [])
    assert f12_from_out(outs) == O.f12_mul(a, b)


@pytest.mark.parametrize("single", [True, False])
def test_set_program_valid_and_wrong_message(single):
    pks, msgs, sigs = sample_sets(2)
    raw = 0 if single else 0xDEADBEEF12345678
    f, fl = run_set(single, pks[0], msgs[0], sigs[0], raw)
    assert all(fl) and O.f12_is_one(O.final_exp(f))
    f, fl = run_set(single, pks[0], msgs[1], sigs[0], raw)  # wrong message
    assert all(fl) and not O.f12_is_one(O.final_exp(f))
    # the Miller value itself: e(pk, H) e(-g1, sig) up to the final exponentiation
    if single:
        f, _ = run_set(True, pks[1], msgs[1], sigs[1])
        H = O.hash_to_g2(msgs[1])
        ref = O.f12_mul(O.miller_loop(pks[1], H), O.miller_loop(O.E1.neg(O.G1), O.signature_from_bytes(sigs[1])))
        assert O.final_exp(f) == O.final_exp(ref)


def test_set_program_uncompressed_and_not_on_curve():
    pks, msgs, sigs = sample_sets(1)
    s = O.signature_from_bytes(sigs[0])
    f, fl = run_set(True, pks[0], msgs[0], O.g2_to_bytes(s, compressed=False))
    assert all(fl) and O.f12_is_one(O.final_exp(f))
    # an x with no point on the curve: on_curve flag clear
    b = bytearray(sigs[0])
    for k in range(1, 50):
        b[95] = (b[95] + 1) & 255
        x1 = int.from_bytes(bytes(b[:48]), "big") & ((1 << 381) - 1)
        x0 = int.from_bytes(bytes(b[48:]), "big")
        rhs = O.f2_add(O.f2_mul(O.f2_sqr((x0, x1)), (x0, x1)), (4, 4))
        if not O.f2_is_square(rhs):
            break
    _, fl = run_set(True, pks[0], msgs[0], bytes(b))
    assert fl[0] == 0


def test_set_program_not_in_subgroup():
    # a point on E2 outside G2: a hashed point before cofactor clearing
    pks, msgs, _ = sample_sets(1)
    u = O.hash_to_field_fp2(b"not in G2", 2, O.DST_POP)
    q = O.iso_map_g2(O.map_to_curve_sswu(u[0]))
    assert O.E2.on_curve(q) and not O.g2_in_subgroup(q)
    _, fl = run_set(True, pks[0], msgs[0], O.g2_to_bytes(q))
    assert fl[0] == 1 and fl[1] == 0


def test_set_program_pk_not_in_g1():
    pks, msgs, sigs = sample_sets(1)
    # a point on E1 outside G1 (x = 0 is not on E1: search small x)
    x = 1
    while True:
        rhs = (x * x * x + 4) % P
        if pow(rhs, (P - 1) // 2, P) == 1:
            y = pow(rhs, (P + 1) // 4, P)
            if not O.g1_in_subgroup((x, y)):
                break
        x += 1
    _, fl = run_set(True, (x, y), msgs[0], sigs[0])
    assert fl[2] == 0
    _, fl = run_set(True, pks[0], msgs[0], sigs[0])
    assert fl[2] == 1


def test_batch_scalar_in_g1():
    """sum over a 2-set batch: prod f_i -> final exp == 1 iff both valid"""
    pks, msgs, sigs = sample_sets(2)
    fs = [run_set(False, pks[i], msgs[i], sigs[i], 0x1111 * (i + 3) + (i << 40))[0] for i in range(2)]
    assert O.f12_is_one(O.final_exp(O.f12_mul(fs[0], fs[1])))
    bad = run_set(False, pks[1], msgs[0], sigs[1], 0x5555)[0]
    assert not O.f12_is_one(O.final_exp(O.f12_mul(fs[0], bad)))


@functools.lru_cache(maxsize=None)
def sswu_prog():
    """map_to_curve_sswu_iso alone (u in, homogeneous (X : Y : Z) out)"""
    from lodestar_amd.lpgen.dsl import Graph
    from lodestar_amd.lpgen.tower import Fp2
    g = Graph("sswu")
    u = Fp2(g.input("u0"), g.input("u1"))
    q = bls.map_to_curve_sswu_iso(u)
    for nm, c in (("X", q.X), ("Y", q.Y), ("Z", q.Z)):
        g.output(nm + "0", c.c0)
        g.output(nm + "1", c.c1)
    return lpc.compile_graph(g, rows=32)


def test_sswu_iso_program_vs_oracle():
    """the one-exponentiation SSWU + 3-isogeny (both square branches, the sign fix,
    u = 0's exceptional x1, u in Fp) == the oracle's RFC 9380 map, point for point"""
    import random
    from tests.lp_helper import RINV
    rnd = random.Random(5)
    us = [(0, 0), (1, 0), (0, 1), (P - 1, 3)] + [(rnd.randrange(P), rnd.randrange(P)) for _ in range(16)]
    us += list(O.hash_to_field_fp2(b"\x01" * 32, 2, O.DST_POP))
    n_sq = 0
    for u in us:
        outs, _ = sswu_prog().run([mont(u[0]), mont(u[1])], [])
        v = [x * RINV % P for x in outs]
        X, Y, Z = (v[0], v[1]), (v[2], v[3]), (v[4], v[5])
        ref = O.iso_map_g2(O.map_to_curve_sswu(u))
        if ref is None:
            assert O.f2_is_zero(Z)
            continue
        zi = O.f2_inv(Z)
        assert (O.f2_mul(X, zi), O.f2_mul(Y, zi)) == ref, u
        n_sq += 1
    assert n_sq >= 20


@pytest.mark.parametrize("single", [True, False])
def test_set_then_mul_then_final_chain(single):
    """the programs chained as k_lp_verify runs them: set outputs -> fp12_mul -> final_exp
    (each program's outputs are canonical, the next one's inputs assume so)"""
    pks, msgs, sigs = sample_sets(2)
    outs = []
    for k in range(2):
        fps, flags = set_inputs(pks[k], msgs[k], sigs[k], 0x1234567890ABCDEF + k)
        o, _ = prog("single" if single else "batch").run([mont(v) for v in fps], flags)
        assert all(v < P for v in o)
        outs.append(o)
    if single:
        for o in outs:
            assert prog("final").run(o, [])[1] == [1]
        return
    prod, _ = prog("mul").run(outs[0] + outs[1], [])
    assert all(v < P for v in prod)
    assert prog("final").run(prod, [])[1] == [1]


# ---- the throughput pipeline's merged check (mtail) and the combine's final exponentiation
@functools.lru_cache(maxsize=None)
def mtail_prog(partial):
    return lpc.compile_graph(bls.mtail_program(partial), rows=32)


def _jac_inputs(pt, z):
    """G2 point (affine, or None = O) as one-lane Jacobian inputs with Z = z"""
    if pt is None:
        return [1, 0, 1, 0, 0, 0]
    (x0, x1), (y0, y1) = pt
    z2 = z * z % P
    z3 = z2 * z % P
    # Jacobian over Fp2 with z in Fp: X = x z^2, Y = y z^3
    return [x0 * z2 % P, x1 * z2 % P, y0 * z3 % P, y1 * z3 % P, z, 0]


def _mtail_inputs(levels, pts, seed=7):
    """levels: the 63 level products P_l (raw inputs, this domain: k_mtail_prep converts);
    pts: the 33 bit sums (one-lane Montgomery inputs)"""
    import random
    rnd = random.Random(seed)
    vals = [mont416(v) for lv in levels for v in f12_fps(lv)]
    g = []
    for pt in pts:
        g += _jac_inputs(pt, rnd.randrange(1, P))
    return vals + [mont(v) for v in g]


def _levels_for(h):
    """level products whose value conj(prod_l P_l^(2^(62 - l))) is h: P_62 = conj(h), the rest 1"""
    one = O.f12_mul(O.f12_inv(h), h)
    return [one] * (bls.MTAIL_LEVELS - 1) + [O.f12_conj(h)]


def _horner_value(levels):
    """conj(prod_l P_l^(2^(62 - l))) by the oracle (k_horner_all's value)"""
    acc = levels[0]
    for lv in levels[1:]:
        acc = O.f12_mul(O.f12_sqr(acc), lv)
    return O.f12_conj(acc)


def _msm_points(n_inf=3):
    """33 bit sums: multiples of G2, a few infinite; S = sum 2^p G_p"""
    pts, S = [], None
    for p in range(bls.MSM_POS):
        if p in (0, 5, 32)[:n_inf]:
            pts.append(None)
            continue
        g = O.g2_mul(O.G2, 1000 + 37 * p)
        pts.append(g)
        t = O.g2_mul(g, 1 << p)
        S = t if S is None else O.g2_add(S, t)
    return pts, S


def test_mtail_programs_against_oracle():
    """check: final_exp(h * Miller(-g1, S_all)) == 1 exactly when h cancels e(-g1, S_all);
    partial: the same product (up to the factors the final exponentiation kills)"""
    pts, S = _msm_points()
    good = O.miller_loop(O.G1, S)      # e(g1, S) e(-g1, S) = 1
    bad = O.miller_loop(O.G1, O.g2_add(S, O.G2))
    for h, want in ((good, 1), (bad, 0)):
        _, fl = mtail_prog(False).run(_mtail_inputs(_levels_for(h), pts), [])
        assert fl == [want]
        outs, _ = mtail_prog(True).run(_mtail_inputs(_levels_for(h), pts), [])
        f = tuple(tuple((outs[6 * a + 2 * b] * pow(1 << 384, -1, P) % P,
                         outs[6 * a + 2 * b + 1] * pow(1 << 384, -1, P) % P) for b in range(3)) for a in range(2))
        assert all(o < P for o in outs)  # canonical one-lane form
        assert O.f12_is_one(O.final_exp(f)) == bool(want)
    # S_all = O (every bit sum infinite): the Miller factor is 1
    inf_pts = [None] * bls.MSM_POS
    one = O.f12_mul(O.miller_loop(O.G1, O.G2), O.miller_loop(O.E1.neg(O.G1), O.G2))
    _, fl = mtail_prog(False).run(_mtail_inputs(_levels_for(one), inf_pts), [])
    assert fl == [1]
    _, fl = mtail_prog(False).run(_mtail_inputs(_levels_for(O.miller_loop(O.G1, O.G2)), inf_pts), [])
    assert fl == [0]


def test_mtail_horner_over_levels():
    """The folded Horner chain: 63 distinct level products (Miller values of small multiples
    of the generators) -- the partial equals conj(Horner over the P_l) * Miller(-g1, S_all)
    up to the factors the final exponentiation kills, and the check passes exactly when
    that product is 1 after the final exponentiation."""
    pts, S = _msm_points()
    levels = [O.miller_loop(O.g1_mul(O.G1, 3 + lv), O.g2_mul(O.G2, 5 + 2 * lv)) for lv in range(bls.MTAIL_LEVELS)]
    want_f = O.f12_mul(_horner_value(levels), O.miller_loop(O.E1.neg(O.G1), S))
    outs, _ = mtail_prog(True).run(_mtail_inputs(levels, pts), [])
    f = tuple(tuple((outs[6 * a + 2 * b] * pow(1 << 384, -1, P) % P,
                     outs[6 * a + 2 * b + 1] * pow(1 << 384, -1, P) % P) for b in range(3)) for a in range(2))
    assert O.f12_eq(O.final_exp(f), O.final_exp(want_f))
    _, fl = mtail_prog(False).run(_mtail_inputs(levels, pts), [])
    assert fl == [int(O.f12_is_one(O.final_exp(want_f)))]


def test_final_lane_program():
    g = lpc.compile_graph(bls.final_lane_program(), rows=32)
    one = O.f12_mul(O.miller_loop(O.G1, O.G2), O.miller_loop(O.E1.neg(O.G1), O.G2))
    for f, want in ((one, 1), (O.miller_loop(O.G1, O.G2), 0)):
        _, fl = g.run([mont(v) for v in f12_fps(f)], [])
        assert fl == [want]


def test_rtail_program_against_oracle():
    """One request's tail of a failed merged check (k_lp_rtail): final_exp(F_k * Miller(-g1,
    S_k)) == 1 exactly when F_k cancels e(-g1, S_k); S_k = O (input flag): the Miller factor
    is 1."""
    g = lpc.compile_graph(bls.rtail_program(), rows=32)
    S = O.g2_mul(O.G2, 12345)
    good = O.miller_loop(O.G1, S)
    bad = O.miller_loop(O.G1, O.g2_add(S, O.G2))
    (x0, x1), (y0, y1) = S
    for f, want in ((good, 1), (bad, 0)):
        _, fl = g.run([mont(v) for v in f12_fps(f) + [x0, x1, y0, y1]], [0])
        assert fl == [want]
    one = O.f12_mul(O.miller_loop(O.G1, O.G2), O.miller_loop(O.E1.neg(O.G1), O.G2))
    _, fl = g.run([mont(v) for v in f12_fps(one) + [0, 0, 0, 0]], [1])
    assert fl == [1]
    _, fl = g.run([mont(v) for v in f12_fps(good) + [0, 0, 0, 0]], [1])
    assert fl == [0]


def test_msm_bits_programs_against_oracle():
    """A lone call's MSM bit sums as three levels of round programs (k_lp_msm_bits): 8 one-lane
    Jacobian bucket sums per level-0 instance -- some infinite, as k_msm_buckets writes them
    (Z = 0) or as k_msm_bits_prep pads a position (all zero) -- summed 8:1 three times; the
    level-2 output, one-lane Jacobian, equals the oracle's sum of the 64 points."""
    import random
    rnd = random.Random(11)
    progs = [lpc.compile_graph(bls.msm_bits_program(k), rows=32) for k in range(3)]
    assert [p.stats["regs"] <= 512 for p in progs] == [True] * 3
    pts = []
    for i in range(64):
        pts.append(None if i % 9 == 4 else O.g2_mul(O.G2, 7 + 13 * i))
    want = None
    for q in pts:
        if q is not None:
            want = q if want is None else O.g2_add(want, q)
    lvl1 = []
    for grp in range(8):
        ins = []
        for j in range(8):
            q = pts[8 * grp + j]
            if q is None and j % 2:  # (the prep kernel's padding: every coordinate zero)
                ins += [0] * 6
            else:
                ins += [mont(v) for v in _jac_inputs(q, rnd.randrange(1, P))]
        outs, _ = progs[0].run(ins, [])
        assert len(outs) == 6 and all(v < P for v in outs)
        lvl1 += outs
    lvl2, _ = progs[1].run(lvl1, [])
    inf416 = [0, 0, mont416(1), 0, 0, 0]  # homogeneous (0 : 1 : 0)
    outs, _ = progs[2].run(lvl2 + inf416 * 7, [])
    r = pow(1 << 384, -1, P)
    X0, X1, Y0, Y1, Z0, Z1 = (v * r % P for v in outs)
    # affine x = X / Z^2, y = Y / Z^3 over Fp2
    def f2mul(a, b):
        return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)

    def f2inv(a):
        n = pow((a[0] * a[0] + a[1] * a[1]) % P, -1, P)
        return (a[0] * n % P, -a[1] * n % P)
    Z = (Z0, Z1)
    zi = f2inv(Z)
    zi2 = f2mul(zi, zi)
    x = f2mul((X0, X1), zi2)
    y = f2mul((Y0, Y1), f2mul(zi2, zi))
    assert (x, y) == want
    # every point infinite: the sum is infinity (Z = 0)
    outs0, _ = progs[0].run([0] * 48, [])
    outs1, _ = progs[1].run(outs0 + inf416 * 7, [])
    outs2, _ = progs[2].run(outs1 + inf416 * 7, [])
    assert outs2[4] == 0 and outs2[5] == 0


def test_sig_decode_program_against_oracle():
    """A small same-message package's signature decode (k_lp_dec): for compressed and
    uncompressed encodings of valid signatures, an x with no curve point, a curve point
    outside G2 and the infinity encoding -- the program's y (one-lane form), on_curve and
    in_group equal the oracle's g2_from_bytes / g2_in_subgroup (the byte-level rules stay
    with k_sm_dec_prep, as in k_lp_prep)."""
    g = lpc.compile_graph(bls.sig_decode_program(), rows=8)
    assert g.stats["regs"] <= 128
    _, _, sigs = sample_sets(2)
    r384 = pow(1 << 384, -1, P)

    def run(x, y, flags):
        outs, ofl = g.run([mont(v) for v in (x[0], x[1], y[0], y[1])], flags)
        return (outs[0] * r384 % P, outs[1] * r384 % P), ofl
    cases = []
    for s in sigs:
        pt = O.g2_from_bytes(s)
        cases.append((s, pt))
        cases.append((O.g2_to_bytes(pt, False), pt))
    for s, pt in cases:
        comp = len(s) == 96
        sign = (s[0] >> 5) & 1 if comp else 0
        y, ofl = run(pt[0], pt[1] if not comp else (0, 0), [0, sign, int(comp)])
        assert y == pt[1] and ofl == [1, 1]
    # an x whose x^3 + b has no root: not on the curve (compressed); a curve point outside G2
    k = 1
    while O.f2_sqrt(O.f2_add(O.f2_mul(O.f2_sqr((k, 0)), (k, 0)), (4, 4))) is not None:
        k += 1
    _, ofl = run((k, 0), (0, 0), [0, 0, 1])
    assert ofl[0] == 0
    k = 1
    while True:
        x = (k, 1)
        y = O.f2_sqrt(O.f2_add(O.f2_mul(O.f2_sqr(x), x), (4, 4)))
        if y is not None and not O.g2_in_subgroup((x, y)):
            break
        k += 1
    yo, ofl = run(x, (0, 0), [0, int(O.f2_lex_largest(y)), 1])
    assert yo == y and ofl == [1, 0]
    _, ofl = run(x, y, [0, 0, 0])  # (uncompressed: the same point as given)
    assert ofl == [1, 0]
    _, ofl = run(x, O.f2_add(y, (1, 0)), [0, 0, 0])  # uncompressed, y off the curve
    assert ofl[0] == 0
    _, ofl = run((0, 0), (0, 0), [1, 0, 1])  # infinity: in the group
    assert ofl[1] == 1


@pytest.mark.parametrize("rows", [16, 8])
def test_hash_finish_program_against_oracle(rows):
    """A lone mid-size call's hash finish (k_lp_hf): Q0, Q1 -- the two mapped points of a
    message, as one-lane Jacobian inputs with arbitrary Z -- give H = clear_cofactor(Q0 + Q1),
    output Jacobian in the one-lane form, equal to the oracle's hash_to_g2; Q0 = -Q1 gives
    infinity (Z = 0).  Compiled for 16 rows and for the default narrow 8-row workgroup."""
    import random
    rnd = random.Random(5)
    g = lpc.compile_graph(bls.hash_finish_program(), rows=rows)
    assert g.stats["regs"] <= 128
    r384 = pow(1 << 384, -1, P)

    def f2mul(a, b):
        return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)

    def f2inv(a):
        n = pow((a[0] * a[0] + a[1] * a[1]) % P, -1, P)
        return (a[0] * n % P, -a[1] * n % P)
    for msg in (b"\x00" * 32, bytes(range(32))):
        u0, u1 = O.hash_to_field_fp2(msg, 2, O.DST_POP)
        q0 = O.iso_map_g2(O.map_to_curve_sswu(u0))
        q1 = O.iso_map_g2(O.map_to_curve_sswu(u1))
        ins = _jac_inputs(q0, rnd.randrange(1, P)) + _jac_inputs(q1, rnd.randrange(1, P))
        outs, _ = g.run([mont(v) for v in ins], [])
        X0, X1, Y0, Y1, Z0, Z1 = (v * r384 % P for v in outs)
        zi = f2inv((Z0, Z1))
        zi2 = f2mul(zi, zi)
        assert (f2mul((X0, X1), zi2), f2mul((Y0, Y1), f2mul(zi2, zi))) == O.hash_to_g2(msg)
    q = O.g2_mul(O.G2, 7)
    qn = (q[0], ((-q[1][0]) % P, (-q[1][1]) % P))
    outs, _ = g.run([mont(v) for v in _jac_inputs(q, 3) + _jac_inputs(qn, 5)], [])
    assert outs[4] == 0 and outs[5] == 0


def test_hash_full_program_against_oracle():
    """LB_LP_HASH_FULL's program (k_lp_hash): u0, u1 -- hash_to_field's outputs in the one-lane
    Montgomery form -- give H = clear_cofactor(map(u0) + map(u1)) as one-lane Jacobian, equal to
    the oracle's hash_to_g2 (8 rows, the kernel's workgroup)."""
    g = lpc.compile_graph(bls.hash_full_program(), rows=8)
    assert g.stats["regs"] <= 384
    r384 = pow(1 << 384, -1, P)

    def f2mul(a, b):
        return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)

    def f2inv(a):
        n = pow((a[0] * a[0] + a[1] * a[1]) % P, -1, P)
        return (a[0] * n % P, -a[1] * n % P)
    for msg in (b"\x00" * 32, bytes(range(32)), b"\xff" * 32):
        u0, u1 = O.hash_to_field_fp2(msg, 2, O.DST_POP)
        outs, _ = g.run([mont(v) for v in (u0[0], u0[1], u1[0], u1[1])], [])
        X0, X1, Y0, Y1, Z0, Z1 = (v * r384 % P for v in outs)
        zi = f2inv((Z0, Z1))
        zi2 = f2mul(zi, zi)
        assert (f2mul((X0, X1), zi2), f2mul((Y0, Y1), f2mul(zi2, zi))) == O.hash_to_g2(msg)


def test_lines_program_against_oracle():
    """A lone mid-size call's lines (k_lp_lines): the 68 lines of (P, H) from projective inputs,
    multiplied as k_step_acc does (a squaring per level, (l0, l1, l4) at c0.c0, c0.c1, c1.c1),
    conjugated, give the oracle's pairing after the final exponentiation; an infinite P gives
    unit lines."""
    import random
    rnd = random.Random(9)
    g = lpc.compile_graph(bls.lines_program(), rows=16)
    assert g.stats["regs"] <= 512
    r384 = pow(1 << 384, -1, P)
    Pt = O.g1_mul(O.G1, 12345)
    Hq = O.g2_mul(O.G2, 678)
    zp, zh = rnd.randrange(1, P), rnd.randrange(1, P)
    px, py = Pt
    ins = [px * zp * zp % P, py * pow(zp, 3, P) % P, zp] + _jac_inputs(Hq, zh)
    outs, _ = g.run([mont(v) for v in ins], [])
    vals = [v * r384 % P for v in outs]
    zero2 = (0, 0)
    f = None
    j = 0
    for i in range(62, -1, -1):
        for rep in range(2):
            if rep == 1 and not (bls.X_ABS >> i) & 1:
                break
            l0, l1, l4 = ((vals[6 * j + 2 * k], vals[6 * j + 2 * k + 1]) for k in range(3))
            line = ((l0, l1, zero2), (zero2, l4, zero2))
            if rep == 0 and f is not None:
                f = O.f12_sqr(f)
            f = line if f is None else O.f12_mul(f, line)
            j += 1
    assert j == 68
    assert O.f12_eq(O.final_exp(O.f12_conj(f)), O.final_exp(O.miller_loop(Pt, Hq)))
    outs, _ = g.run([mont(v) for v in [1, 1, 0] + _jac_inputs(Hq, zh)], [])  # P = O
    vals = [v * r384 % P for v in outs]
    assert all(vals[6 * j:6 * j + 6] == [1, 0, 0, 0, 0, 0] for j in range(68))
