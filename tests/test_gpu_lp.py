"""GPU checks of the latency path's round-program interpreter (k_lp.hip) via
lb_lp_program_run: every output of the device must equal, bit for bit, the CPU
executor of the same encoded program (lpgen.compile.Program.run), and the
verdict chain must match the oracle.  Also prints the per-program kernel time
of one instance (the latency a lone set pays for each stage)."""
import numpy as np
import pytest

from tests.lp_helper import (LB_PROG_FINAL, LB_PROG_MUL, LB_PROG_SET_BATCH, LB_PROG_SET_SINGLE, f12_fps,
                             f12_from_out, mont, mont416, sample_sets, set_inputs)
from tests.test_lp_programs import prog
from oracle import bls12_381 as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from lodestar_amd.native import Device
    d = Device(0)
    yield d
    d.close()


def rec(vals):
    a = np.zeros((len(vals), 16), np.uint32)
    for i, v in enumerate(vals):
        for j in range(12):
            a[i, j] = (v >> (32 * j)) & 0xFFFFFFFF
    return a


def ints(a):
    return [sum(int(x) << (32 * j) for j, x in enumerate(r[:13])) for r in a]  # 13 limbs: R = 2^416 values


def run_both(dev, pid, name, cases):
    """cases: [(montgomery fp inputs, flags)] -> device outputs, after checking the CPU executor agrees"""
    p = prog(name)
    ins = np.stack([rec(fp) for fp, _ in cases])
    fl = np.array([f for _, f in cases], np.uint32) if cases[0][1] else np.zeros((len(cases), 0), np.uint32)
    out, ofl, ms = dev.lp_program_run(pid, ins, fl, len(p.out_names), len(p.outflag_names))
    for i, (fp, f) in enumerate(cases):
        want, wfl = p.run(fp, f)
        assert ints(out[i]) == want, (name, i)
        assert [int(x) for x in ofl[i]] == wfl, (name, i)
    return out, ofl, ms


def test_lp_mul_and_final(dev):
    a = O.miller_loop(O.G1, O.G2)
    b = O.miller_loop(O.E1.neg(O.G1), O.G2)
    out, _, ms = run_both(dev, LB_PROG_MUL, "mul", [([mont416(v) for v in f12_fps(a) + f12_fps(b)], [])])
    ab = f12_from_out(ints(out[0]))
    assert ab == O.f12_mul(a, b)
    _, ofl, ms_f = run_both(dev, LB_PROG_FINAL, "final", [([mont416(v) for v in f12_fps(ab)], []),
                                                          ([mont416(v) for v in f12_fps(a)], [])])
    assert [int(x) for x in ofl[:, 0]] == [1, 0]
    print(f"\nlp mul {ms:.3f} ms, final_exp {ms_f:.3f} ms (2 instances)")


@pytest.mark.parametrize("single", [True, False])
def test_lp_set_programs(dev, single):
    pks, msgs, sigs = sample_sets(3)
    raw = 0 if single else 0x0123456789ABCDEF
    cases = []
    for i in range(3):
        fp, f = set_inputs(pks[i], msgs[i if i < 2 else 0], sigs[i], raw)
        cases.append(([mont(v) for v in fp], f))
    pid = LB_PROG_SET_SINGLE if single else LB_PROG_SET_BATCH
    out, ofl, ms = run_both(dev, pid, "single" if single else "batch", cases)
    verdicts = [O.f12_is_one(O.final_exp(f12_from_out(ints(out[i])))) for i in range(3)]
    assert verdicts == [True, True, False]
    assert all(int(x) == 1 for x in ofl.reshape(-1))
    # one instance alone: the latency of the stage
    _, _, ms1 = dev.lp_program_run(pid, np.stack([rec(cases[0][0])]), np.array([cases[0][1]], np.uint32),
                                   12, len(prog("single" if single else "batch").outflag_names))
    print(f"\nlp set program ({'single' if single else 'batch'}): {ms1:.3f} ms for one set, {ms:.3f} ms for 3")
