"""The wave-cooperative Fp12 programs (lodestar_amd/csrc/gen_wc12.py: K parallel
Fp products + linear combinations per operation) evaluated on random inputs
against the oracle's Fp12 arithmetic.  CPU only: this pins the tables the
GPU's k_tail kernel executes."""
import importlib.util
import os
import random

import pytest

from oracle import bls12_381 as O

P = O.P
_spec = importlib.util.spec_from_file_location(
    "gen_wc12", os.path.join(os.path.dirname(__file__), "..", "lodestar_amd", "csrc", "gen_wc12.py"))
G = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(G)


def flat(f12):
    out = []
    for f6 in f12:
        for f2 in f6:
            out += [f2[0], f2[1]]
    return out


def unflat(v):
    f2 = [(v[2 * k], v[2 * k + 1]) for k in range(6)]
    return ((f2[0], f2[1], f2[2]), (f2[3], f2[4], f2[5]))


def run(prog_fn, A, B):
    prog, out = prog_fn()
    env = {}

    def ev(form):
        acc = 0
        for (kind, i), c in form.d.items():
            v = A[i] if kind == "A" else B[i] if kind == "B" else env[i]
            acc += c * v
        return acc % P

    for k, (x, y) in enumerate(prog.prods):
        env[k] = ev(x) * ev(y) % P
    return [ev(o) for o in out.flat()]


def rnd12(r):
    return [r.randrange(P) for _ in range(12)]


@pytest.fixture(scope="module")
def rng():
    return random.Random(2024)


def test_mul(rng):
    for _ in range(3):
        a, b = rnd12(rng), rnd12(rng)
        assert run(G.op_mul, a, b) == flat(O.f12_mul(unflat(a), unflat(b)))


def test_sqr(rng):
    a = rnd12(rng)
    assert run(G.op_sqr, a, a) == flat(O.f12_mul(unflat(a), unflat(a)))


def test_cyclotomic_sqr(rng):
    f = unflat(rnd12(rng))
    f = O.f12_mul(O.f12_conj(f), O.f12_inv(f))          # ^(p^6 - 1)
    f = O.f12_mul(O.f12_pow(f, P * P), f)               # ^(p^2 + 1): cyclotomic
    a = flat(f)
    assert run(G.op_cyc, a, a) == flat(O.f12_mul(f, f))


def test_line(rng):
    a = rnd12(rng)
    l0, l1, l4 = [(rng.randrange(P), rng.randrange(P)) for _ in range(3)]
    b = [l0[0], l0[1], l1[0], l1[1], l4[0], l4[1]] + [0] * 6
    line = ((l0, l1, O.F2_ZERO), (O.F2_ZERO, l4, O.F2_ZERO))
    assert run(G.op_line, a, b) == flat(O.f12_mul(unflat(a), line))


@pytest.mark.parametrize("k", [1, 2, 3])
def test_frobenius(rng, k):
    a = rnd12(rng)
    xi = (1, 1)
    gam = [O.f2_pow(xi, e * (P ** k - 1) // 6) for e in range(6)]
    b = [c for g in gam for c in g]
    assert run({1: lambda: G.op_frob(1), 2: lambda: G.op_frob(2), 3: lambda: G.op_frob(3)}[k], a, b) == \
        flat(O.f12_pow(unflat(a), P ** k))


def test_conj(rng):
    a = rnd12(rng)
    assert run(G.op_conj, a, a) == flat(O.f12_conj(unflat(a)))
