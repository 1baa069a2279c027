"""GPU parity of the merged check's bucket MSM (k_msm.hip, lb_g2_msm):
sum_i (a_i + b_i lambda) P_i, a_i / b_i the 32-bit halves of the batch scalar,
against the CPU oracle's G2 arithmetic.  Bit-exact (uncompressed affine bytes).

The points are [k_i] G2 for known k_i (made by lb_g2_mul, itself pinned to the
oracle in test_gpu_parity.py), so the expected sum is ONE oracle scalar
multiplication: [sum_i k_i (a_i + b_i lambda) mod r] G2.
"""
import random

import pytest

from oracle import batch as OB
from oracle import bls12_381 as O

pytestmark = pytest.mark.gpu

G2_BYTES = O.g2_to_bytes(O.G2, compressed=False)
INF_BYTES = bytes([0x40]) + bytes(191)


def _points(device, ks):
    return device.g2_mul([G2_BYTES] * len(ks), ks)


def _expect(ks, raws):
    s = 0
    for k, w in zip(ks, raws):
        s += k * ((w & 0xFFFFFFFF) + (w >> 32) * OB.GLV_LAMBDA)
    s %= O.R
    pt = O.g2_mul(O.G2, s) if s else None
    return INF_BYTES if pt is None else O.g2_to_bytes(pt, compressed=False)


def test_msm_empty_and_single(device):
    assert device.g2_msm([], []) == INF_BYTES
    pts = _points(device, [7])
    assert device.g2_msm(pts, [1]) == pts[0]
    assert device.g2_msm(pts, [0]) == INF_BYTES  # zero scalar: every digit zero
    for raw in (2, 1 << 32, (1 << 32) + 1, 0xFFFFFFFF, 0xFFFFFFFFFFFFFFFF, 1024, 1025, 2047, 2048,
                (1024 << 11) | 1024, (1023 << 22) | (1024 << 11) | 1025):
        assert device.g2_msm(pts, [raw]) == _expect([7], [raw]), hex(raw)


def test_msm_digit_edges(device):
    """Scalars at every signed-digit boundary of the 11-bit windows (carries into
    the next window, the top window's digit 1024, zero windows)."""
    rng = random.Random(5)
    edges = [0, 1, 1023, 1024, 1025, 2046, 2047]
    raws = []
    for _ in range(300):
        lo = 0
        for w in range(3):
            lo |= (rng.choice(edges) & (0x3FF if w == 2 else 0x7FF)) << (11 * w)
        hi = 0
        for w in range(3):
            hi |= (rng.choice(edges) & (0x3FF if w == 2 else 0x7FF)) << (11 * w)
        raws.append((hi << 32) | lo)
    ks = [rng.randrange(1, 1 << 40) for _ in raws]
    pts = _points(device, ks)
    assert device.g2_msm(pts, raws) == _expect(ks, raws)


def test_msm_duplicates_and_cancellation(device):
    """Equal points in one bucket (the mixed addition's doubling case), P and -P
    with equal scalars (cancellation to infinity inside a bucket)."""
    pts = _points(device, [3])
    raw = 0x0000012300000456
    assert device.g2_msm(pts * 300, [raw] * 300) == _expect([3] * 300, [raw] * 300)
    neg = pts[0]
    # -P: the same x, y negated (uncompressed: x || y)
    x, y = O.g2_from_bytes(neg)
    negp = O.g2_to_bytes((x, O.f2_neg(y)), compressed=False)
    assert device.g2_msm([neg, negp] * 50, [raw] * 100) == INF_BYTES
    assert device.g2_msm([neg, negp, neg], [raw, raw, raw]) == _expect([3], [raw])


@pytest.mark.parametrize("n", [2, 100, 5000, 40000])
def test_msm_random(device, n):
    rng = random.Random(n)
    ks = [rng.randrange(1, 1 << 60) for _ in range(n)]
    raws = [rng.randrange(1, 1 << 64) for _ in range(n)]
    pts = _points(device, ks)
    assert device.g2_msm(pts, raws) == _expect(ks, raws)


def test_msm_batch_scalars(device):
    """The pipeline's scalars: the DRBG of a seed (lb_batch_scalars), 8192 points."""
    seed = bytes(range(32))
    n = 8192
    raws = device.batch_scalars(seed, 0, n)
    assert raws[:4] == [OB.batch_scalar_raw(seed, i) for i in range(4)]
    rng = random.Random(9)
    ks = [rng.randrange(1, 1 << 62) for _ in range(n)]
    pts = _points(device, ks)
    assert device.g2_msm(pts, raws) == _expect(ks, raws)
