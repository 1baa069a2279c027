"""GPU checks of the row-cooperative Fp layer (lodestar_amd/csrc/bls_coop.h): the
Montgomery product, the signed normalization + quotient reduction behind every
linear form of the latency path, canonicalisation and the row predicates, on
edge cases (0, p - 1, values just under 2^383, all-ones limbs, maximal negative
partials) and random inputs.  Expected values are Python big integers.  The
HIP side is tests/native/coop_selftest.hip (built by build(); test-only)."""
import ctypes
import os
import random

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tests", "native", "libcoop_selftest.so")
P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 1 << 384
RINV = pow(R, -1, P)
B383 = 1 << 383

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        pytest.fail("tests/native/libcoop_selftest.so missing: run __graft_entry__.build()")
    L = ctypes.CDLL(LIB)
    vp = ctypes.c_void_p
    L.lbt_coop_op.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                              ctypes.c_uint32, ctypes.POINTER(ctypes.c_float)]
    return L


def rows(vals):
    out = np.zeros((len(vals), 16), np.uint32)
    for i, v in enumerate(vals):
        for j in range(16):
            out[i, j] = (v >> (32 * j)) & 0xFFFFFFFF
    return out


def ints(arr):
    return [sum(int(x) << (32 * j) for j, x in enumerate(row)) for row in arr]


def call(lib, op, a, b=None, c=None, d=None, aux=None, k=0, waves=1):
    n = a.shape[0]
    out = np.zeros((n, 16), np.uint32)
    out2 = np.zeros((n, 16), np.uint32)
    aux_out = np.zeros((n, 4), np.uint32)
    cyc = np.zeros(n, np.uint64)
    ms = ctypes.c_float(0)
    ptr = lambda x: None if x is None else np.ascontiguousarray(x).ctypes.data  # noqa: E731
    keep = [np.ascontiguousarray(x) for x in (a, b, c, d, aux) if x is not None]
    rc = lib.lbt_coop_op(op, n, k, ptr(keep[0]), ptr(b), ptr(c), ptr(d), ptr(aux), out.ctypes.data, out2.ctypes.data,
                         aux_out.ctypes.data, cyc.ctypes.data, waves, ctypes.byref(ms))
    assert rc == 0, rc
    return out, out2, aux_out, cyc, ms.value


EDGE = [0, 1, 2, P - 1, P, P + 1, 2 * P, 3 * P - 1, 4 * P + 5, B383 - 1, B383 - P, (1 << 352) - 1, 0xFFFFFFFF,
        (1 << 381) - 1, int("ff" * 47, 16)]


def sample(k, seed, bound=B383):
    rng = random.Random(seed)
    v = [e for e in EDGE if e < bound]
    while len(v) < k:
        v.append(rng.randrange(bound))
    return v[:k]


def test_mont_mul(lib):
    a = sample(256, 1)
    b = sample(256, 2)[::-1]
    out = ints(call(lib, 0, rows(a), rows(b))[0])
    for x, y, o in zip(a, b, out):
        assert o < B383 and o % P == x * y * RINV % P, (hex(x), hex(y), hex(o))


def test_product_chain_and_timing(lib):
    a = sample(64, 3)
    b = sample(64, 4, P)
    k = 2000
    out, _, _, cyc, ms = call(lib, 1, rows(a), rows(b), k=k)
    for x, y, o in zip(a, b, ints(out)):
        want = x * pow(y * RINV, k, P) % P
        assert o < B383 and o % P == want
    per = float(np.median(cyc)) / k
    print(f"\ncoop mont_mul chain: {per:.1f} s_memtime ticks per product ({ms:.3f} ms for {k} products, 16 rows)")


def test_linear_form_normalize_reduce(lib):
    rng = random.Random(5)
    n = 512
    vals = [sample(n, 10 + t) for t in range(4)]
    aux = np.zeros((n, 8), np.int32)
    for i in range(n):
        cf = [rng.choice([1, -1, 2, -2, 3, -3, 6, -6, 12, -12, 24, 64, -64]) for _ in range(4)]
        if i < 8:  # maximal negative weight
            cf = [-64, -64, -64, -64]
        negw = sum(-c for c in cf if c < 0)
        K = (negw * B383 + P - 1) // P  # K p >= the negative terms' bound
        aux[i, :4] = cf
        aux[i, 4] = K
    out, out2, _, _, _ = call(lib, 2, rows(vals[0]), rows(vals[1]), rows(vals[2]), rows(vals[3]), aux)
    T = ints(out)
    Rd = ints(out2)
    for i in range(n):
        exact = sum(int(aux[i, t]) * vals[t][i] for t in range(4)) + int(aux[i, 4]) * P
        assert exact >= 0
        assert T[i] == exact, i
        assert Rd[i] % P == exact % P and Rd[i] < 11 * P // 10, i


def test_canon_and_predicates(lib):
    v = sample(300, 7) + [0, P, 2 * P, 3 * P, 4 * P, (P - 1) // 2, (P + 1) // 2, P - 1 + 4 * P]
    v = [x for x in v if x < B383]
    out, _, aux_out, _, _ = call(lib, 3, rows(v))
    for x, c, f in zip(v, ints(out), aux_out):
        cv = x % P
        assert c == cv
        assert int(f[0]) == (cv == 0)
        assert int(f[1]) == (cv > (P - 1) // 2)
        assert int(f[2]) == (cv & 1)


def test_sub_cmp(lib):
    a = sample(200, 8, P)
    b = sample(200, 9, P)
    a += [5, P - 1, 0]
    b += [5, P - 1, 1]
    out, _, aux_out, _, _ = call(lib, 4, rows(a), rows(b))
    for x, y, o, f in zip(a, b, ints(out), aux_out):
        assert int(f[0]) == (x >= y)
        assert o == (x - y) % (1 << 512)


def test_row_inversion(lib):
    """row_inv_raw (the latency path's INV unit): random values, 0, 1, p - 1, small and
    large powers of two; four rows of a wave invert one after the other."""
    vals = sample(60, 21, P) + [0, 1, P - 1, 2, 1 << 380, P - 2, (1 << 255) + 7, 3]
    out, _, _, cyc, ms = call(lib, 5, rows(vals))
    for x, o in zip(vals, ints(out)):
        assert o == (pow(x, -1, P) if x else 0), hex(x)
    print(f"\nrow inversion: {float(np.median(cyc)):.0f} s_memtime ticks per wave (4 rows), {ms:.3f} ms")
