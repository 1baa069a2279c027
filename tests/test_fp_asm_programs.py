"""CPU checks of the generated carry-chain asm (lodestar_amd/csrc/gen_fp_asm.py).

The lazy-reduction Fp2 product combines three double-width products with
interleaved carry chains written as raw gfx950 asm.  This interprets those
instruction lists on Python integers (one lane) and checks them against big-int
arithmetic, including the wait-state rule the scheduler enforces: a VALU-written
carry mask is read no sooner than two instructions after it is written.
"""
import os
import random
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "lodestar_amd", "csrc"))
import gen_fp_asm as G  # noqa: E402

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 1 << 384
M32 = (1 << 32) - 1


def run(lines, regs):
    """Execute asm lines over regs (name -> int); returns regs."""
    written = {}
    pos = 0

    def val(tok):
        tok = tok.strip()
        if tok.startswith("%["):
            return regs[tok[2:-1]]
        return int(tok, 0)

    def read_carry(tok):
        name = tok.strip()
        assert name in written, f"carry {name} read before written"
        assert pos - written[name] - 1 >= 2, f"wait-state violation on {name} at {pos}"
        return regs[name[2:-1]]

    for ln in lines:
        op, _, rest = ln.partition(" ")
        args = [a.strip() for a in rest.split(",")] if rest else []
        if op == "s_nop":
            pos += int(args[0]) + 1
            continue
        d = args[0][2:-1]
        if op == "v_add_co_u32_e64":
            s = val(args[2]) + val(args[3])
            regs[d], regs[args[1][2:-1]] = s & M32, s >> 32
            written[args[1]] = pos
        elif op == "v_addc_co_u32_e64":
            s = val(args[2]) + val(args[3]) + read_carry(args[4])
            regs[d], regs[args[1][2:-1]] = s & M32, s >> 32
            written[args[1]] = pos
        elif op == "v_sub_co_u32_e64":
            s = val(args[2]) - val(args[3])
            regs[d], regs[args[1][2:-1]] = s & M32, int(s < 0)
            written[args[1]] = pos
        elif op == "v_subb_co_u32_e64":
            s = val(args[2]) - val(args[3]) - read_carry(args[4])
            regs[d], regs[args[1][2:-1]] = s & M32, int(s < 0)
            written[args[1]] = pos
        elif op == "v_cndmask_b32_e64":
            regs[d] = val(args[2]) if read_carry(args[3]) else val(args[1])
        else:
            raise AssertionError(f"unknown op {op}")
        pos += 1
    return regs


def limbs(x, n):
    return [(x >> (32 * j)) & M32 for j in range(n)]


def unlimbs(regs, prefix, n):
    return sum(regs[f"{prefix}{j}"] << (32 * j) for j in range(n))


def kcombine(a0, a1, b0, b1):
    T0, T1, T2 = a0 * b0, a1 * b1, (a0 + a1) * (b0 + b1)
    regs = {}
    for i, T in enumerate((T0, T1, T2)):
        for j, v in enumerate(limbs(T, 24)):
            regs[f"t{i}_{j}"] = v
    for j, v in enumerate(limbs(P, 12)):
        regs[f"p_{j}"] = v
    run(G.kcombine_program(), regs)
    return unlimbs(regs, "t0_", 24), unlimbs(regs, "t2_", 24)


def check_kcombine(a0, a1, b0, b1):
    W0, W1 = kcombine(a0, a1, b0, b1)
    assert W0 == (a0 * b0 - a1 * b1) % (P * R)
    assert W1 == a0 * b1 + a1 * b0
    assert W0 < P * R and W1 < P * R  # REDC input bound -> output < 2p


def test_kcombine_random():
    rng = random.Random(7)
    for _ in range(300):
        check_kcombine(*(rng.randrange(P) for _ in range(4)))


@pytest.mark.parametrize("a0,a1,b0,b1", [
    (0, 0, 0, 0), (P - 1, P - 1, P - 1, P - 1), (0, P - 1, 0, P - 1), (P - 1, 0, P - 1, 0),
    (1, P - 1, 1, P - 1), (P - 1, 1, 1, P - 1), (5, 5, 7, 7),
])
def test_kcombine_edges(a0, a1, b0, b1):
    check_kcombine(a0, a1, b0, b1)


def test_plain_add2():
    rng = random.Random(3)
    for _ in range(200):
        a0, a1, b0, b1 = (rng.randrange(P) for _ in range(4))
        regs = {}
        for x, v in (("s", a0), ("t", b0), ("sb", a1), ("tb", b1)):
            for j, l in enumerate(limbs(v, 12)):
                regs[f"{x}{j}"] = l
        run(G.plain_add2_program(), regs)
        assert unlimbs(regs, "s", 12) == a0 + a1
        assert unlimbs(regs, "t", 12) == b0 + b1


def redc_model(w):
    """The column recurrence of gen_redc on integers."""
    pl = limbs(P, 12)
    pinv = (-pow(P, -1, 1 << 32)) % (1 << 32)
    assert pinv == 0xFFFCFFFD
    wl = limbs(w, 24)
    m, t = [], []
    A = wl[0]
    for k in range(23):
        if k < 12:
            A += sum(m[j] * pl[k - j] for j in range(k))
            m.append((A & M32) * pinv & M32)
            A += m[k] * pl[0]
            assert A & M32 == 0
        else:
            A += sum(m[j] * pl[k - j] for j in range(k - 11, 12))
            t.append(A & M32)
        A = (A >> 32) + wl[k + 1]
    t.append(A & M32)
    assert A >> 32 == 0
    r = sum(v << (32 * j) for j, v in enumerate(t))
    assert r < 2 * P
    return r - P if r >= P else r


def test_redc_recurrence():
    rng = random.Random(11)
    Rinv = pow(R, -1, P)
    for w in [0, 1, P * R - 1, P * P, 2 * P * P] + [rng.randrange(P * R) for _ in range(200)]:
        assert redc_model(w) == w * Rinv % P
