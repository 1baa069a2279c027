"""The carry-free column products (tools/microbench/fp_cols.h, an experiment kept out of the library: 13 digits of 30 bits,
Montgomery radix 2^384) against Python big integers, on the host (g++ build of the same
header): mul / sqr (a, b < p -> a b 2^-384 mod p, fully reduced), mulw (a, b < 2^384 -> the
exact 768-bit product) and redc (w < p 2^384 -> w 2^-384 mod p, fully reduced), on edge values
(0, 1, p - 1, 2^384 - 1 for mulw, p 2^384 - 1 for redc, all-ones limbs) and random ones.
DESIGN.md §4 "Field core": measured on MI355X, only the squaring came out faster, and the gfx950
build of the converting bodies disagreed with this host build on the device self-test, so the
library keeps its product-scanning asm."""
import ctypes
import os
import random
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 1 << 384
RINV = pow(R, -1, P)


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("cols") / "libfp_cols_host.so")
    src = os.path.join(ROOT, "tests", "native", "fp_cols_host.cpp")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", out, src])
    return ctypes.CDLL(out)


def _arr(v, n):
    return (ctypes.c_uint32 * n)(*[(v >> (32 * i)) & 0xFFFFFFFF for i in range(n)])


def _val(a, n):
    return sum(int(a[i]) << (32 * i) for i in range(n))


def test_columns_against_big_ints(lib):
    rnd = random.Random(11)
    edge_p = [0, 1, 2, P - 1, P - 2, (P - 1) // 2, 2 ** 380, sum(0xFFFFFFFF << (32 * i) for i in range(11))]
    vals = edge_p + [rnd.randrange(P) for _ in range(400)]
    r = (ctypes.c_uint32 * 12)()
    w = (ctypes.c_uint32 * 24)()
    for k, a in enumerate(vals):
        b = vals[(7 * k + 3) % len(vals)]
        lib.cols_mul(r, _arr(a, 12), _arr(b, 12))
        assert _val(r, 12) == a * b * RINV % P, (a, b)
        lib.cols_sqr(r, _arr(a, 12))
        assert _val(r, 12) == a * a * RINV % P, a
    wide = [0, 1, R - 1, R - 2, P, 2 * P, 2 * P - 1] + [rnd.randrange(R) for _ in range(300)]
    for k, a in enumerate(wide):
        b = wide[(5 * k + 1) % len(wide)]
        lib.cols_mulw(w, _arr(a, 12), _arr(b, 12))
        assert _val(w, 24) == a * b, (a, b)
    reds = [0, 1, P * R - 1, P * R // 2, (P - 1) * (P - 1), 4 * P * P] + [rnd.randrange(P * R) for _ in range(300)]
    for x in reds:
        lib.cols_redc(r, _arr(x, 24))
        assert _val(r, 12) == x * RINV % P, x
    # operands beyond the contract, up to 2^384 (as callers pass lazily reduced values): the
    # result stays < 2^384 and congruent (the asm bodies' behaviour), canonical when < 2p
    big = [R - 1, R - 2, 5 * P, 9 * P + 7] + [rnd.randrange(R) for _ in range(200)]
    for k, a in enumerate(big):
        b = big[(3 * k + 1) % len(big)]
        for fn, args, want in ((lib.cols_mul, (_arr(a, 12), _arr(b, 12)), a * b),
                               (lib.cols_sqr, (_arr(a, 12),), a * a)):
            fn(r, *args)
            v = _val(r, 12)
            assert v < R and v % P == want * RINV % P, (a, b)
            if (want + ((-want * pow(P, -1, R)) % R) * P) // R < 2 * P:
                assert v < P
        for x in (a * a, a * b, R * R - 1):
            lib.cols_redc(r, _arr(x % (R * R), 24))
            v = _val(r, 12)
            assert v < R and v % P == (x % (R * R)) * RINV % P
