"""Device vs CPU executor on pieces of the final-exponentiation program (GPU
debugging aid for the latency path): each piece is compiled as a program of its
own, run on the device through lb_lp_program_run and by the executor, and every
output (value and flag) compared.  Prints one line per piece; exits 1 on any
mismatch.  Usage: python tools/lp_debug.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from lodestar_amd.lpgen import bls, compile as lpc  # noqa: E402
from lodestar_amd.lpgen.dsl import Graph  # noqa: E402
from lodestar_amd.lpgen.tower import Fp2, Fp6, Fp12  # noqa: E402

P = bls.P
R416 = 1 << 416


def rec(vals):
    a = np.zeros((len(vals), 16), np.uint32)
    for i, v in enumerate(vals):
        for j in range(13):
            a[i, j] = (v >> (32 * j)) & 0xFFFFFFFF
    return a


def ints(a):
    return [sum(int(x) << (32 * j) for j, x in enumerate(r[:13])) for r in a]


def piece(name, build, n_in):
    g = Graph(name)
    xs = [g.input_raw("x%d" % k) for k in range(n_in)]
    outs, flags = build(g, xs)
    for k, o in enumerate(outs):
        g.output("o%d" % k, o)
    for k, f in enumerate(flags):
        g.output_flag("f%d" % k, f)
    return lpc.compile_graph(g, rows=32)


def f12(xs):
    return Fp12.from_fps(xs)


def main():
    from lodestar_amd.native import Device
    import random
    rnd = random.Random(1)
    vals = [rnd.randrange(P) * R416 % P for _ in range(12)]
    pieces = [
        ("mul", lambda g, x: ([x[0] * x[1]], []), 2),
        ("canon_iszero", lambda g, x: ([], [g.is_zero(x[0] - x[0]), g.is_zero(x[0])]), 1),
        ("fp_inv", lambda g, x: ([g.inv(x[0])], []), 1),
        ("fp2_inv", lambda g, x: ((lambda v: [v.c0, v.c1])(Fp2(x[0], x[1]).inv()), []), 2),
        ("fp12_inv", lambda g, x: (f12(x).inv().fps(), []), 12),
        ("easy", lambda g, x: ((f12(x).conj() * f12(x).inv()).mat().fps(), []), 12),
        ("cyc_sqr", lambda g, x: (f12(x).cyc_sqr().mat().fps(), []), 12),
        ("exp_x", lambda g, x: (bls.fp12_exp_x(f12(x)).fps(), []), 12),
        ("is_one", lambda g, x: ([], [f12(x).is_one()]), 12),
        ("final_values", lambda g, x: (bls.final_exp(f12(x)).mat().fps(), []), 12),
        ("final", lambda g, x: ([], [bls.final_exp(f12(x)).is_one()]), 12),
    ]
    dev = Device(0) if "--cpu" not in sys.argv else None
    bad = 0
    for name, build, n_in in pieces:
        p = piece(name, build, n_in)
        ins = rec(vals[:n_in])[None, :, :]
        want, wfl = p.run(vals[:n_in], [])
        if dev is None:
            print(name, p.n_rounds, "cpu only", wfl)
            continue
        out, ofl, ms = dev.lp_program_run(p.words, ins, np.zeros((1, 0), np.uint32), len(p.out_names),
                                          len(p.outflag_names))
        got = ints(out[0]) if len(p.out_names) else []
        gfl = [int(x) for x in ofl[0]] if len(p.outflag_names) else []
        ok = got == want and gfl == wfl
        bad += not ok
        first = next((k for k, (a, b) in enumerate(zip(got, want)) if a != b), None)
        print(f"{name:14s} rounds {p.n_rounds:4d} {'OK' if ok else 'MISMATCH'} first_bad_out={first} "
              f"flags dev={gfl} cpu={wfl} {ms:.3f} ms", flush=True)
        if name == "fp_inv" and not ok:
            c = vals[0]
            R384, R416_ = 1 << 384, 1 << 416
            d = got[0]
            hyp = {"dev_mod_p==want": d % P == want[0], "dev<p": d < P,
                   "dev==R384^2/c": d % P == R384 * R384 * pow(c, -1, P) % P,
                   "dev==R416^2/c": d % P == R416_ * R416_ * pow(c, -1, P) % P,
                   "dev*c/R416": d * c * pow(R416_, -1, P) % P, "R416 mod p": R416_ % P}
            print("  fp_inv dev", hex(d), "want", hex(want[0]), hyp, flush=True)
    if dev is not None:
        dev.close()
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
