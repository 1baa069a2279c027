"""Count Fp products per pipeline stage (the roofline's algorithmic-op figure).

Build (CPU container):  python tools/opcount.py --build
Run (GPU box):          python tools/opcount.py --run  -> profiles/op_counts.json

Uses a separate build of the same sources with -DLB_COUNT_OPS (every fp_mul /
fp_sqr does one device atomicAdd).  The counts are exact for the data used:
the only data-dependent branches are the 64-bit scalar bits (add or not) and
the SSWU square/non-square path, both averaged over 256 random sets.  An Fp
inversion (binary GCD, bls_inv.h) counts as 10 products: its 3,000 v_mad_u64_u32
(25 rounds x 120) / 288, plus the one product that returns it to Montgomery form.
"""
import argparse
import ctypes
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# (LB_OPCOUNT_DIR: a directory that travels to the GPU box; tools/opcount_build does not)
OUT_DIR = os.environ.get("LB_OPCOUNT_DIR", os.path.join(ROOT, "tools", "opcount_build"))
MADS_PER_FPMUL = 288  # 12x12 limb products + 12x12 reduction products (bls_fp_ps.h)
MADS_PER_FPSQR = 224  # 66 cross (+2 doubled lone cross) + 12 squares + 144 reduction products


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--run", action="store_true")
    ap.add_argument("--sets", type=int, default=1024)
    ap.add_argument("--per-request", type=int, default=128)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "op_counts.json"))
    ap.add_argument("--workloads", action="store_true",
                    help="count BASELINE.json's C4 shard (at 1/8 scale, same proportions) and C5 epoch shapes in "
                         "the default organisation -> profiles/op_counts_workloads.json (bench.py config_legs)")
    ap.add_argument("--wl-out", default=os.path.join(ROOT, "profiles", "op_counts_workloads.json"))
    a = ap.parse_args()
    from lodestar_amd import build as b
    if a.build:
        print(b.build_opcount(OUT_DIR))
    if not a.run:
        return
    if a.workloads:
        return count_workloads(a.wl_out)
    import numpy as np
    # the bench's organisation (stored lines + multi-pair accumulation, merged check)
    os.environ["LB_MILLER"] = "lines"
    from lodestar_amd import native
    native.library_path = lambda: os.path.join(OUT_DIR, "liblodestar_bls_count.so")
    native._lib = None
    lib = native.load_library()
    lib.lb_opcount_stages.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    n = a.sets
    r_order = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
    sks = [(int.from_bytes(hashlib.sha256(i.to_bytes(32, "little")).digest(), "little") % r_order).to_bytes(32, "big")
           for i in range(n)]
    msgs = [hashlib.sha256(b"opcount" + i.to_bytes(8, "little")).digest() for i in range(n)]

    def count(acc, split=0):
        # LB_ACC=steps (default): step-major lanes + level products + one Horner chain (k_steps.hip);
        # LB_ACC=pairs: k_miller_acc with LB_ACC_SPLIT=0: two pairs per lane (calls overlapped) or
        # 1: requests split in halves, one pair per lane (what a lone call ran in that organisation)
        os.environ["LB_ACC"] = acc
        os.environ["LB_ACC_SPLIT"] = str(split)
        dev = native.Device(0)
        pks = dev.sk_to_pk(sks)
        sigs = dev.sign(sks, msgs)
        blob, offs = native.pack_blobs(sigs)
        req = np.arange(0, n + 1, a.per_request, dtype=np.uint32)
        res = dev.verify_requests(req, np.frombuffer(b"".join(pks), np.uint8), None,
                                  np.frombuffer(b"".join(msgs), np.uint8), blob, offs, bytes(32))
        assert res.valid.all(), res.valid
        names = [nm for nm, _ in dev.last_stage_times(raw=True)]
        buf = (ctypes.c_ulonglong * 32)()
        k = lib.lb_opcount_stages(dev._h, buf, 32)
        per = {}
        tot_mul = tot_sqr = 0
        for i in range(k):
            # low half counts 144-mad halves (a Montgomery product is two)
            muls, sqrs = (int(buf[i]) & 0xFFFFFFFF) / 2, int(buf[i]) >> 32
            tot_mul += muls
            tot_sqr += sqrs
            e = per.setdefault(names[i], {"fp_mul_total": 0, "fp_sqr_total": 0, "fp_mul_per_set": 0.0,
                                          "mads_per_set": 0.0})  # (a stage's launches summed)
            e["fp_mul_total"] += muls
            e["fp_sqr_total"] += sqrs
            e["fp_mul_per_set"] += (muls + sqrs) / n
            e["mads_per_set"] += (muls * MADS_PER_FPMUL + sqrs * MADS_PER_FPSQR) / n
        return per, tot_mul, tot_sqr

    per, tot_mul, tot_sqr = count("steps")
    pairs, p_mul, p_sqr = count("pairs", 0)
    lone, _, _ = count("pairs", 1)
    n_req = n // a.per_request
    out = {"sets": n, "requests": n_req, "sets_per_request": a.per_request, "mads_per_fp_mul": MADS_PER_FPMUL,
           "mads_per_fp_sqr": MADS_PER_FPSQR,
           "organisation": "LB_MILLER=lines, merged check, steps organisation of the Miller accumulation "
                           "(k_step_acc + k_level_prod + k_horner_all, k_steps.hip)",
           "stages": per, "fp_mul_per_set_total": (tot_mul + tot_sqr) / n,
           "mads_per_set_total": (tot_mul * MADS_PER_FPMUL + tot_sqr * MADS_PER_FPSQR) / n,
           "pairs_organisation": "LB_ACC=pairs LB_ACC_SPLIT=0: k_miller_acc, two pairs per lane (rounds 2-3)",
           "pairs_stages": pairs,
           "pairs_mads_per_set_total": (p_mul * MADS_PER_FPMUL + p_sqr * MADS_PER_FPSQR) / n,
           "lone_call_organisation": "LB_ACC=pairs LB_ACC_SPLIT=1: requests split in halves, one pair per lane "
                                     "(what a lone call ran in the pairs organisation)",
           "lone_call_stages": {k: {"mads_per_set": v["mads_per_set"]} for k, v in lone.items()}}
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


def count_workloads(out_path=os.path.join(ROOT, "profiles", "op_counts_workloads.json")):
    """Every Fp product of one call of each config shape (tools/workloads.py), in the
    organisation the library picks for it (no LB_MILLER override), pubkeys by validator
    index from a 65,536-key table: the mads per set bench.py's config legs price."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import workloads as W
    from lodestar_amd import native
    native.library_path = lambda: os.path.join(OUT_DIR, "liblodestar_bls_count.so")
    native._lib = None
    lib = native.load_library()
    lib.lb_opcount_stages.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    dev = native.Device(0)
    keys = W.make_keys(dev, 65536)
    assert dev.pubkey_table_append(keys.pks) == 65536
    shapes = {"c4_shard": lambda: W.c4_shard(dev, keys, singles=112712 // 8, aggregates=4096 // 8),
              "c5": lambda: W.c5_epoch(dev, keys, invalid_rate=0.0)}
    out = {"mads_per_fp_mul": MADS_PER_FPMUL, "mads_per_fp_sqr": MADS_PER_FPSQR,
           "note": "counting build (-DLB_COUNT_OPS), one call per shape, default organisation, all sets valid; "
                   "c4_shard at 1/8 scale (14,089 singles + 512 AggregateAndProof triples of 488 keys)"}
    for name, make in shapes.items():
        p = make()
        blob, offs = p.blobs()
        r = dev.verify_requests(p.req_off, None, p.pk_off, p.msg_array(), blob, offs, bytes(32), pk_indices=p.idx)
        assert r.valid.all(), name
        names = [nm for nm, _ in dev.last_stage_times(raw=True)]
        buf = (ctypes.c_ulonglong * 32)()
        k = lib.lb_opcount_stages(dev._h, buf, 32)
        per, tm, ts = {}, 0, 0
        for i in range(k):
            muls, sqrs = (int(buf[i]) & 0xFFFFFFFF) / 2, int(buf[i]) >> 32
            tm += muls
            ts += sqrs
            e = per.setdefault(names[i], {"mads_per_set": 0.0})  # (a stage's launches summed)
            e["mads_per_set"] += (muls * MADS_PER_FPMUL + sqrs * MADS_PER_FPSQR) / p.n_sets
        out[name] = {"sets": p.n_sets, "requests": p.n_req, "pubkeys": int(len(p.idx)),
                     "keys_per_set": len(p.idx) / p.n_sets, "stages": per,
                     "mads_per_set_total": (tm * MADS_PER_FPMUL + ts * MADS_PER_FPSQR) / p.n_sets}
        print(name, out[name]["mads_per_set_total"], flush=True)
    dev.close()
    with open(out_path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
