"""Summarise tools/pmc.sh passes into profiles/pmc_traffic.json (per pipeline
stage: kernel, counters averaged per launch, HBM bytes per launch).

hbm_bytes_per_launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: FETCH_SIZE and
WRITE_SIZE are KiB from the L2's memory-side request counters; on gfx950
FETCH_SIZE reports half the bytes of wide coalesced reads
(/opt/skills/guides/MI355X_MICROARCH.md, HBM section), hence the factor 2
(an upper bound for narrower accesses).

usage: python tools/pmc_summarize.py PMC_DIR [OUT.json]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

STAGE_OF = {  # pipeline stage (bench.py stage_ms key) -> kernel base name
    "hash_half": "k_hash_half", "hash_finish": "k_hash_finish", "req_flags": "k_req_flags",
    "pubkeys": "k_pubkeys_single", "scalar_pk": "k_scalar_pk", "lines": ("k_lines_rows", "k_lines"),
    "decode_sigs": "k_decode_sigs", "scalar_sig": "k_scalar_sig", "sum_tree": "k_sum_tree",
    "miller_acc": "k_miller_acc", "merge": "k_merge", "lines_S": "k_lines_S", "tail": "k_tail",
    "miller_wave": "k_pair_wc", "pubkeys_agg": "k_pubkeys_agg",
    "msm_digits": "k_msm_scalars", "msm_chunks": "k_msm_chunks", "msm_buckets": "k_msm_buckets",
    "msm_bits": "k_msm_bits", "msm_final": "k_msm_final", "msm_scatter": "k_msm_scatter",
    "step_acc": "k_step_acc", "level_prod": ("k_level_part", "k_level_prod"), "level_wc": "k_level_wc",
    "horner_all": "k_horner_all",
    "req_status": "k_req_status", "req_horner": "k_req_horner", "lines_all": "k_lines_S",
    "mtail": "k_lp_mtail", "rtail": "k_lp_rtail",
}


# Algorithmic HBM bytes per SET of each per-set stage (C2: one pubkey and one
# 96-byte signature per set): what the stage must read and write, no spills.
# Jacobian G1 = 144 B, Jacobian G2 = 288 B, a stored line = 288 B (68 per pair).
ALG_BYTES_PER_SET = {
    "hash_half": 32 + 2 * 288,        # message -> Q0, Q1
    "hash_finish": 2 * 288 + 288,     # Q0, Q1 -> H(m)
    "pubkeys": 96 + 144 + 1,          # encoding -> point + status
    "scalar_pk": 144 + 144 + 1,       # pk -> r pk (+ G1 check flag)
    "decode_sigs": 96 + 288 + 1,      # compressed signature -> point + status
    "scalar_sig": 288 + 288,          # sigma -> r sigma
    "lines": 144 + 288 + 68 * 288,    # r pk, H -> 68 lines
    "miller_acc": 68 * 288 + 2,       # lines (+ statuses) -> per-request F_k
    "step_acc": 68 * 288 + 576,       # a lane's 68 lines -> its level product G (one lane per set)
    "level_prod": 576,                # every G read once
    # bucket MSM: 6 entries per set (2 half-points x 3 windows), each a 4-byte sorted
    # index and the point's affine (x, y) = 192 B, and 6/16 chunk partials (288 B)
    "msm_chunks": 6 * (4 + 192) + 6 * 288 // 16,
}
N_SETS = 65536


def kernel_key(name):
    """'void lb::k_lines<1>(unsigned int, ...)' -> 'k_lines'"""
    n = name.split("(")[0].replace("void ", "").replace("lb::", "").strip()
    return n.split("<")[0]


def main():
    d = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                              "pmc_traffic.json")
    vals = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [per-launch values]
    full = {}
    files = glob.glob(os.path.join(d, "pass*", "**", "*counter_collection.csv"), recursive=True)
    files += glob.glob(os.path.join(d, "pass*_counter_collection.csv"))  # flattened copies under profiles/
    for f in files:
        for row in csv.DictReader(open(f)):
            k = kernel_key(row["Kernel_Name"])
            full[k] = row["Kernel_Name"]
            vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    res = {"_note": __doc__.strip().split("\n\n")[1].replace("\n", " ")}
    for stage, prefixes in STAGE_OF.items():
        found = [p for p in (prefixes if isinstance(prefixes, tuple) else (prefixes,)) if p in vals]
        if not found:
            continue
        k = found[0]
        c = {n: sum(v) / len(v) for n, v in vals[k].items()}
        ent = {"kernel": full[k].split("(")[0], "counters": {n: round(x, 3) for n, x in c.items()}}
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            ent["hbm_bytes_per_launch"] = int((2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024)
            if stage in ALG_BYTES_PER_SET:
                alg = ALG_BYTES_PER_SET[stage] * N_SETS
                ent["algorithmic_bytes_per_launch"] = alg
                ent["traffic_over_algorithmic"] = round(ent["hbm_bytes_per_launch"] / alg, 2)
        if "SQ_INSTS_VALU" in c and "SQ_WAVES" in c and c["SQ_WAVES"]:
            ent["valu_insts_per_wave"] = round(c["SQ_INSTS_VALU"] / c["SQ_WAVES"])
        if c.get("SQ_LDS_IDX_ACTIVE"):
            # extra LDS cycles from bank conflicts / all LDS-array cycles (MI355X_MICROARCH.md LDS section)
            ent["lds_bank_conflict_frac"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0.0) / c["SQ_LDS_IDX_ACTIVE"], 5)
        res[stage] = ent
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1)[:3000])


if __name__ == "__main__":
    main()
