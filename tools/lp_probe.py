"""Latency-path round costs on the GPU (diagnostic; writes gpurun_out/lp_probe.json).

* synthetic chains: N rounds of one Fp product (x = x^2), of one linear unit,
  of 32 products per round -> microseconds per round of each kind;
* the embedded set/final programs with per-round s_memtime stamps of instance 0,
  summarised by round composition (rounds holding an inversion / a product /
  only linear units / only predicates and flag ops)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from lodestar_amd.lpgen import compile as lpc  # noqa: E402
from lodestar_amd.lpgen.dsl import Graph  # noqa: E402
from lodestar_amd.native import Device  # noqa: E402

TICK_GHZ = 0.1  # s_memtime on gfx950 counts at the 100 MHz reference clock? calibrated below


def chain(kind, n, width=1):
    g = Graph("chain_%s_%d" % (kind, width))
    xs = [g.input("x%d" % i) for i in range(width)]
    for _ in range(n):
        if kind == "mul":
            xs = [x * x for x in xs]
        else:
            xs = [(x + x + x).mat() for x in xs]
    for i, x in enumerate(xs):
        g.output("o%d" % i, x)
    return lpc.compile_graph(g, rows=32)


def composition(words):
    n_rounds = words[1]
    n_const, n_in, n_inflag, n_out, n_outflag = words[4:9]
    boff = (10 + 14 * n_const + n_in + n_inflag + n_out + n_outflag + 3) & ~3
    kinds = []
    for r in range(n_rounds):
        bw, nu = words[boff], words[boff + 1]
        ops = {words[boff + 4 + lpc.REC_WORDS * u] & 15 for u in range(nu)}
        boff += bw
        if 3 in ops:
            k = "inv"
        elif 0 in ops:
            k = "mul"
        elif 1 in ops or 2 in ops or 4 in ops:
            k = "lin/sel"
        else:
            k = "pred/flag"
        kinds.append((k, nu, bw))
    return kinds


def unit_features(words):
    """per round, per unit: (op, ext, nx, ny, ext_terms) from the encoded blocks"""
    n_rounds = words[1]
    n_const, n_in, n_inflag, n_out, n_outflag = words[4:9]
    boff = (10 + 14 * n_const + n_in + n_inflag + n_out + n_outflag + 3) & ~3
    out = []
    for r in range(n_rounds):
        bw, nu = words[boff], words[boff + 1]
        us = []
        for u in range(nu):
            w0 = words[boff + 4 + lpc.REC_WORDS * u]
            op = w0 & 15
            if (w0 >> 18) & 1:
                base = boff + words[boff + 4 + lpc.REC_WORDS * u + 2]
                e0 = words[base]
                op, nops, nfl = e0 & 15, (e0 >> 4) & 7, (e0 >> 7) & 7
                o = base + 1 + nfl
                ts = []
                for _ in range(nops):
                    ts.append(words[o] & 255)
                    o += 1 + (words[o] & 255)
                us.append((op, 1, 0, 0, tuple(ts)))
            else:
                us.append((op, 0, (w0 >> 4) & 31, (w0 >> 9) & 31, ()))
        out.append(us)
        boff += bw
    return out


def wave_table(feats, st):
    """mean run_unit ticks of a wave by its content: key = (kinds present, max inline terms, ext terms)"""
    nw = (st.shape[1] - 6) // 6
    tab = {}
    for r, us in enumerate(feats):
        for w in range(nw):
            mine = us[4 * w:4 * w + 4]
            if not mine:
                continue
            dt = int(st[r, 6 + nw + w]) - int(st[r, 6 + w])
            u0 = 6 + 2 * nw + 4 * w
            inner = [int(st[r, u0 + k]) - int(st[r, 6 + w]) if st[r, u0 + k] else -1 for k in range(4)]
            kinds = tuple(sorted({("ext%d" % u[0]) if u[1] else ("op%d" % u[0]) for u in mine}))
            mt = max((max(u[2], u[3]) for u in mine if not u[1]), default=0)
            et = max((sum(u[4]) for u in mine if u[1]), default=0)
            key = "%s|t%d|e%d" % ("+".join(kinds), mt, (et + 7) // 8 * 8)
            e = tab.setdefault(key, [0, 0, [0, 0, 0, 0], [0, 0, 0, 0]])
            e[0] += 1
            e[1] += dt
            for k in range(4):
                if inner[k] >= 0:
                    e[2][k] += inner[k]
                    e[3][k] += 1
    return {k: {"n": v[0], "ticks": round(v[1] / v[0]),
                "regs_x_y_prod": [round(v[2][i] / v[3][i]) if v[3][i] else None for i in range(4)]}
            for k, v in sorted(tab.items(), key=lambda kv: -kv[1][0])}


def main():
    dev = Device(0)
    out = {}
    rng = np.random.default_rng(1)
    for kind, width in (("mul", 1), ("lin", 1), ("mul", 32), ("mul", 4)):
        p = chain(kind, 2000, width)
        ins = np.zeros((1, width, 16), np.uint32)
        ins[0, :, :11] = rng.integers(0, 2 ** 32, (width, 11), dtype=np.uint64).astype(np.uint32)
        ms_list = []
        for _ in range(3):
            _, _, ms = dev.lp_program_run(p.words, ins, np.zeros((1, 0), np.uint32), width, 0)
            ms_list.append(ms)
        ms = min(ms_list)
        out["chain_%s_w%d" % (kind, width)] = {"rounds": p.n_rounds, "ms": ms, "us_per_round": 1000 * ms / p.n_rounds}
        print(kind, width, p.n_rounds, "rounds", "%.3f ms" % ms, "%.3f us/round" % (1000 * ms / p.n_rounds), flush=True)
    # the embedded programs with stamps
    from lodestar_amd.lpgen import bls
    from tests.lp_helper import mont, sample_sets, set_inputs
    pks, msgs, sigs = sample_sets(1)
    fp, fl = set_inputs(pks[0], msgs[0], sigs[0])
    rec = np.zeros((1, 11, 16), np.uint32)
    for i, v in enumerate(fp):
        mv = mont(v)
        for j in range(12):
            rec[0, i, j] = (mv >> (32 * j)) & 0xFFFFFFFF
    gen = {"set_single": bls.set_program(True), "final": bls.final_program()}
    for name, pid in (("set_single", 0), ("final", 3)):
        p = lpc.compile_graph(gen[name], rows=32)
        kinds = composition(p.words)
        if name == "final":
            rec_f = np.zeros((1, 12, 16), np.uint32)
            rec_f[0, :, 0] = 1
            ins, flg, no, nof = rec_f, np.zeros((1, 0), np.uint32), 0, 1
        else:
            ins, flg, no, nof = rec, np.array([fl], np.uint32), 12, 3
        best = None
        for _ in range(3):
            t0 = time.time()
            _, _, ms, st = dev.lp_program_run(p.words, ins, flg, no, nof, stamps=True)
            if best is None or ms < best[0]:
                best = (ms, st.copy())
        ms, st = best
        st = st.astype(np.int64)
        d = np.diff(st[:, 5])
        # in-round segments: catch-up, ring store, issue + descriptor loads, run_unit, barrier; loop gap
        seg = np.diff(st[:, :6], axis=1)
        gap = st[1:, 0] - st[:-1, 5]
        seg_names = ["catchup", "ring_store", "issue", "run_unit", "barrier"]
        out[name + "_segments"] = {
            "mean_ticks": {n: float(seg[:, k].mean()) for k, n in enumerate(seg_names)},
            "median_ticks": {n: float(np.median(seg[:, k])) for k, n in enumerate(seg_names)},
            "loop_gap_mean": float(gap.mean()),
            "by_kind_mean": {kk: {n: float(seg[[i for i, x in enumerate(kinds) if x[0] == kk], k].mean())
                                  for k, n in enumerate(seg_names)}
                             for kk in sorted({x[0] for x in kinds})}}
        print(name + "_segments", json.dumps(out[name + "_segments"]), flush=True)
        out[name + "_waves"] = wave_table(unit_features(p.words), st)
        for k, v in list(out[name + "_waves"].items())[:40]:
            print("  wave", name, k, v, flush=True)
        summ = {}
        for (k, nu, bw), dt in zip(kinds[1:], d):
            s = summ.setdefault(k, [0, 0])
            s[0] += 1
            s[1] += int(dt)
        out[name] = {"rounds": p.n_rounds, "ms": ms, "us_per_round": 1000 * ms / p.n_rounds,
                     "ticks_total": int(st[-1, 5]) - int(st[0, 0]),
                     "by_kind": {k: {"rounds": v[0], "ticks": v[1], "ticks_per_round": v[1] / max(v[0], 1)}
                                 for k, v in summ.items()},
                     "slowest_rounds": [(int(i) + 1, kinds[int(i) + 1][0], int(d[i])) for i in np.argsort(d)[-8:]]}
        print(name, json.dumps(out[name]), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "lp_probe.json"), "w") as f:
        json.dump(out, f, indent=1)
    dev.close()


if __name__ == "__main__":
    main()
