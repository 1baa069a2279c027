"""GPU checks of the field primitives added for lazy reduction (fp_mulw, fp_redc,
the lazy Fp2 product) and of the register-window exponentiation, on edge cases
no hashed input reaches: 0, 1, p - 1, all-ones limbs, and inputs up to 2p where
the documented bound allows them.  Expected values are Python big integers.
The HIP side is tests/native/field_selftest.hip (built by build(); test-only)."""
import ctypes
import os
import random

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# (LB_FIELD_SELFTEST: another build of the same self-test)
LIB = os.environ.get("LB_FIELD_SELFTEST") or os.path.join(ROOT, "tests", "native", "libfield_selftest.so")
P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 1 << 384
RINV = pow(R, -1, P)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        pytest.fail("tests/native/libfield_selftest.so missing: run __graft_entry__.build()")
    L = ctypes.CDLL(LIB)
    L.lbt_field_op.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    return L


def limbs(vals, n):
    out = np.zeros((len(vals), n), np.uint32)
    for i, v in enumerate(vals):
        for j in range(n):
            out[i, j] = (v >> (32 * j)) & 0xFFFFFFFF
    return out


def ints(arr):
    return [sum(int(x) << (32 * j) for j, x in enumerate(row)) for row in arr]


def run(lib, op, a, b, wout):
    n = a.shape[0]
    out = np.zeros((n, wout), np.uint32)
    a = np.ascontiguousarray(a)
    bp = None
    if b is not None:
        b = np.ascontiguousarray(b)
        bp = b.ctypes.data
    rc = lib.lbt_field_op(op, n, a.ctypes.data, bp, out.ctypes.data)
    assert rc == 0, rc
    return out


EDGE = [0, 1, 2, P - 1, P - 2, (P - 1) // 2, (1 << 381) - 1, (1 << 352) - 1, 0xFFFFFFFF, 1 << 380]


def edge_and_random(k, bound, seed):
    rng = random.Random(seed)
    vals = [v % bound for v in EDGE] + [rng.randrange(bound) for _ in range(k)]
    return vals


def test_fp2_mul_lazy(lib):
    """Karatsuba with lazy reduction: inputs < p (the tower keeps them there) and up
    to 2p (the bound the reduction argument allows), output canonical."""
    rng = random.Random(5)
    cases = []
    for bound in (P, 2 * P):
        vals = edge_and_random(60, bound, 9 + bound % 7)
        for _ in range(300):
            cases.append(tuple(rng.choice(vals) for _ in range(4)))
    a = np.concatenate([limbs([c[0] for c in cases], 12), limbs([c[1] for c in cases], 12)], axis=1)
    b = np.concatenate([limbs([c[2] for c in cases], 12), limbs([c[3] for c in cases], 12)], axis=1)
    out = run(lib, 0, a, b, 24)
    r0, r1 = ints(out[:, :12]), ints(out[:, 12:])
    for (a0, a1, b0, b1), c0, c1 in zip(cases, r0, r1):
        assert c0 == (a0 * b0 - a1 * b1) * RINV % P, (a0, a1, b0, b1)
        assert c1 == (a0 * b1 + a1 * b0) * RINV % P, (a0, a1, b0, b1)


def test_mulw_redc(lib):
    xs = edge_and_random(200, R, 1)
    ys = list(reversed(edge_and_random(200, R, 2)))
    w = run(lib, 1, limbs(xs, 12), limbs(ys, 12), 24)
    assert ints(w) == [x * y for x, y in zip(xs, ys)]
    rng = random.Random(3)
    ws = [0, 1, P * R - 1, P * P, 2 * P * P - 1, R - 1, R * R // 16] + [rng.randrange(P * R) for _ in range(300)]
    r = run(lib, 2, limbs(ws, 24), None, 12)
    assert ints(r) == [v * RINV % P for v in ws]


def test_pow_p34(lib):
    """a^((p-3)/4) on Montgomery representatives (register-window exponentiation)."""
    xs = edge_and_random(200, P, 4)
    r = run(lib, 3, limbs([x * R % P for x in xs], 12), None, 12)
    e = (P - 3) // 4
    assert ints(r) == [pow(x, e, P) * R % P for x in xs]


def test_fp_mul(lib):
    xs = edge_and_random(200, P, 6)
    ys = edge_and_random(200, P, 7)
    r = run(lib, 4, limbs(xs, 12), limbs(ys, 12), 12)
    assert ints(r) == [x * y * RINV % P for x, y in zip(xs, ys)]


def test_fp_sqr(lib):
    xs = edge_and_random(200, P, 8)
    r = run(lib, 5, limbs(xs, 12), None, 12)
    assert ints(r) == [x * x * RINV % P for x in xs]

