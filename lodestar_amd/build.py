"""Build the HIP library in-tree for gfx950 (hipcc cross-compiles without a GPU)."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "liblodestar_bls.so")
# one translation unit per stage group, compiled in parallel and linked into one .so
UNITS = ["k_final.hip", "k_pairing.hip", "k_aux.hip", "k_hash.hip", "k_miller.hip", "k_scalar.hip", "k_sets.hip",
         "k_prod.hip", "k_tail.hip", "k_ssz.hip", "k_msm.hip", "k_steps.hip", "k_lp.hip", "lp_blob.hip",
         "bls_host.hip"]
HEADERS = ["bls_kernels.h", "bls_inv.h", "bls_field.h", "bls_fp_ps.h", "bls_curve.h", "bls_hash.h", "bls_pairing.h",
           "bls_wc12.h", "bls_wc12_tables.h", "gen_constants.py", "gen_fp_asm.py", "gen_wc12.py"]
# headers / generated files only some units depend on (a regenerated program blob must
# not rebuild every kernel unit)
UNIT_DEPS = {"k_lp.hip": ["bls_coop.h", "bls_lp.h", "bls_lp_progs.h"], "lp_blob.hip": ["lp_programs.bin"],
             "bls_host.hip": ["bls_lp.h", "bls_lp_progs.h"]}
LPGEN = os.path.join(HERE, "lpgen")
LP_BLOB = os.path.join(CSRC, "lp_programs.bin")
SOURCES = UNITS + HEADERS + ["bls_all.hip"] + sorted({d for v in UNIT_DEPS.values() for d in v})
OBJ_DIR = os.path.join(ROOT, "build", "obj")
HEADER = os.path.join(ROOT, "include", "lodestar_bls.h")
ARCH = os.environ.get("LB_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _newest_source_mtime() -> float:
    paths = [os.path.join(CSRC, s) for s in SOURCES] + [HEADER, os.path.abspath(__file__)]
    return max(os.path.getmtime(p) for p in paths if os.path.exists(p))


def gen_constants() -> str:
    """Generated headers: curve constants and the product-scanning field multiply."""
    for header, script in (("bls_constants.h", "gen_constants.py"), ("bls_fp_ps.h", "gen_fp_asm.py"),
                           ("bls_wc12_tables.h", "gen_wc12.py")):
        out = os.path.join(CSRC, header)
        gen = os.path.join(CSRC, script)
        if not os.path.exists(out) or os.path.getmtime(out) < os.path.getmtime(gen):
            subprocess.check_call([sys.executable, gen, out])
    # the latency path's round programs (lp_programs.bin + bls_lp_progs.h) from lpgen/
    gen = os.path.join(CSRC, "gen_lp.py")
    srcs = [gen, os.path.join(CSRC, "gen_constants.py")] + [os.path.join(LPGEN, f) for f in os.listdir(LPGEN)
                                                            if f.endswith(".py")]
    outs = [LP_BLOB, os.path.join(CSRC, "bls_lp_progs.h")]
    if not all(os.path.exists(o) for o in outs) or min(os.path.getmtime(o) for o in outs) < max(
            os.path.getmtime(x) for x in srcs):
        subprocess.check_call([sys.executable, gen, CSRC])
    return os.path.join(CSRC, "bls_constants.h")


FLAGS = ["-O3", "-std=c++17", "-fPIC"]


def blob_define() -> str:
    return '-DLB_LP_BLOB_PATH="%s"' % LP_BLOB


def hipcc_cmd(out: str, extra=()) -> list:
    """Single-TU build of the whole library (op-counting variant)."""
    return [HIPCC, f"--offload-arch={ARCH}", *FLAGS, "-shared", blob_define(), "-o", out,
            os.path.join(CSRC, "bls_all.hip"), *extra]


def _unit_deps_mtime(unit: str) -> float:
    paths = [os.path.join(CSRC, unit)] + [os.path.join(CSRC, h) for h in HEADERS + UNIT_DEPS.get(unit, [])] + [HEADER]
    return max(os.path.getmtime(p) for p in paths if os.path.exists(p))


def build(force: bool = False, verbose: bool = False, jobs: int = 0, lib: str = LIB, obj_dir: str = OBJ_DIR,
          extra=(), blob: str = None) -> str:
    """Compile every unit for gfx950 (in parallel, each unit only when stale) and link the .so."""
    gen_constants()
    LIB = lib  # noqa: N806
    OBJ_DIR = obj_dir  # noqa: N806
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= _newest_source_mtime():
        return LIB
    os.makedirs(OBJ_DIR, exist_ok=True)
    objs, todo = [], []
    for u in UNITS:
        o = os.path.join(OBJ_DIR, os.path.splitext(u)[0] + ".o")
        objs.append(o)
        if force or not os.path.exists(o) or os.path.getmtime(o) < _unit_deps_mtime(u):
            unit_flags = [(blob_define() if blob is None else '-DLB_LP_BLOB_PATH="%s"' % blob)] if u == "lp_blob.hip" else []
            todo.append([HIPCC, f"--offload-arch={ARCH}", *FLAGS, *extra, *unit_flags, "-c", "-o", o,
                         os.path.join(CSRC, u)])
    jobs = jobs or max(1, min(len(todo), os.cpu_count() or 1, 16))
    procs = []
    for cmd in todo:
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append((cmd, subprocess.Popen(cmd)))
        while sum(p.poll() is None for _, p in procs) >= jobs:
            procs[0][1].wait() if procs[0][1].poll() is None else None
            import time
            time.sleep(0.2)
    failed = [c for c, p in procs if p.wait() != 0]
    if failed:
        raise RuntimeError("hipcc failed: " + " | ".join(" ".join(c) for c in failed))
    link = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB + ".tmp", *objs]
    if verbose:
        print(" ".join(link), flush=True)
    subprocess.check_call(link)
    os.replace(LIB + ".tmp", LIB)
    return LIB


def build_variant(name: str, extra, verbose: bool = False, blob: str = None) -> str:
    """Same library with extra compile flags, under build/variants/NAME/ (select it
    at run time with LB_LIBRARY=<path>); for tuning experiments only."""
    d = os.path.join(ROOT, "build", "variants", name)
    return build(verbose=verbose, lib=os.path.join(d, "liblodestar_bls.so"), obj_dir=os.path.join(d, "obj"),
                 extra=tuple(extra), blob=blob)


def build_opcount(out_dir: str) -> str:
    """Variant with every Fp product counted (tools/opcount.py); never shipped."""
    gen_constants()
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, "liblodestar_bls_count.so")
    subprocess.check_call(hipcc_cmd(out, extra=("-DLB_COUNT_OPS",)))
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
