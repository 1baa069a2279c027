"""CPU checks of the step-major Miller accumulation's index arithmetic (k_steps.hip):
the size-descending row layout, the lane -> lines assignment, the level tags and the
two Horner stages.  Restated in Python over integers (exponents of 2 stand in for the
Fp12 squarings), so every line of every pair is shown to reach the final product with
the exponent 2^(62 - lvl(j)) that miller_loop gives it (bls_pairing.h)."""
import random

import pytest

X_ABS = 0xD201000000010000
LINES = 68


def step_table():
    """lvl[j] for the 68 lines (doubling line of bit i = 62..0, then the addition line
    when bit i of |x| is set) and first[l] = first line of level l (first[63] = 68)."""
    lvl, first = [], [0] * 64
    for i in range(62, -1, -1):
        first[62 - i] = len(lvl)
        lvl.append(62 - i)
        if (X_ABS >> i) & 1:
            lvl.append(62 - i)
    first[63] = len(lvl)
    return lvl, first


LVL, FIRST = step_table()


def rows_layout(sizes):
    """k_rows_hist / k_rows_scan / k_rows_pos: positions in size-descending order and
    row offsets (rowoff[i] = sum_{i' < i} #requests with more than i' sets)."""
    n_sets = sum(sizes)
    hist = [0] * (n_sets + 1)
    for z in sizes:
        hist[z] += 1
    gt = [0] * (n_sets + 1)
    acc = 0
    for z in range(n_sets, -1, -1):
        gt[z] = acc
        acc += hist[z]
    rowoff, acc = [0] * (n_sets + 1), 0
    for i in range(n_sets + 1):
        rowoff[i] = acc
        acc += gt[i]
    cursor = [0] * (n_sets + 1)
    pos, inv = [0] * len(sizes), [0] * len(sizes)
    for k, z in enumerate(sizes):
        p = gt[z] + cursor[z]
        cursor[z] += 1
        pos[k], inv[p] = p, k
    rows = max([z for z in sizes if z > 0], default=0)
    return rowoff, pos, inv, rows


def slot_row(rowoff, rows, q):
    lo, hi = 0, rows
    while hi - lo > 1:
        mid = (lo + hi) // 2
        if rowoff[mid] <= q:
            lo = mid
        else:
            hi = mid
    return lo, q - rowoff[lo]


def level_lanes(n, lvl):
    def ceil_lane(j):
        a = FIRST[j] * n - (LINES - 1)
        return 0 if a <= 0 else (a + LINES - 1) // LINES
    lo, hi = ceil_lane(lvl), min(ceil_lane(lvl + 1), n)
    return min(lo, hi), hi


def lane_lines(n, lane):
    """The in-lane Horner of k_step_acc: per line of the lane, the number of squarings
    applied to it inside the lane, and the level the lane's product is tagged with."""
    t0 = LINES * lane
    j, i = divmod(t0, n)
    cur = LVL[j]
    out = []  # (pair i, line j, squarings after it inside the lane)
    c = 0
    while c < LINES:
        if LVL[j] != cur:
            out = [(p, jj, s + 1) for (p, jj, s) in out]  # one squaring of the accumulator
            cur = LVL[j]
        out.append((i, j, 0))
        c += 1
        i += 1
        if i >= n:
            i, j = 0, j + 1
    return out, cur


@pytest.mark.parametrize("sizes", [[128] * 8, [1, 2, 3, 67, 68, 69, 128, 300, 0], [5] * 3 + [1] * 9,
                                   [1200, 3] + [20] * 8])
def test_rows_are_a_bijection_and_lanes_cover_every_line_once(sizes):
    rowoff, pos, inv, rows = rows_layout(sizes)
    n_sets = sum(sizes)
    seen = set()
    for k, z in enumerate(sizes):
        for i in range(z):
            q = rowoff[i] + pos[k]
            assert 0 <= q < n_sets and q not in seen
            seen.add(q)
            assert slot_row(rowoff, rows, q) == (i, pos[k])  # the kernels' inverse map
            assert inv[pos[k]] == k
    assert len(seen) == n_sets
    for k, z in enumerate(sizes):
        cover = {}
        for lane in range(z):
            lines, tag = lane_lines(z, lane)
            lo, hi = level_lanes(z, tag)
            assert lo <= lane < hi  # k_level_prod / k_req_horner find the lane at its level
            for (p, j, s) in lines:
                assert (p, j) not in cover
                # the Horner over levels squares the lane value 62 - tag more times
                cover[(p, j)] = s + 62 - tag
        assert len(cover) == LINES * z
        for (p, j), e in cover.items():
            assert e == 62 - LVL[j]  # exactly miller_loop's exponent 2^(62 - lvl(j))


def test_level_lanes_partition_every_request():
    rnd = random.Random(3)
    for n in [1, 2, 3, 67, 68, 69, 127, 128, 129, 1000] + [rnd.randrange(1, 5000) for _ in range(20)]:
        got = []
        for lvl in range(63):
            lo, hi = level_lanes(n, lvl)
            got += list(range(lo, hi))
        assert got == list(range(n))


def test_step_table():
    assert len(LVL) == LINES and FIRST[63] == LINES
    assert sum(1 for a, b in zip(LVL, LVL[1:]) if a == b) == 5  # the five addition lines
