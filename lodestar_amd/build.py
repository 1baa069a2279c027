"""Build the HIP library in-tree for gfx950 (hipcc cross-compiles without a GPU)."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "liblodestar_bls.so")
SOURCES = ["bls_kernels.hip", "bls_field.h", "bls_curve.h", "bls_hash.h", "bls_pairing.h", "gen_constants.py"]
HEADER = os.path.join(ROOT, "include", "lodestar_bls.h")
ARCH = os.environ.get("LB_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _newest_source_mtime() -> float:
    paths = [os.path.join(CSRC, s) for s in SOURCES] + [HEADER, os.path.abspath(__file__)]
    return max(os.path.getmtime(p) for p in paths if os.path.exists(p))


def gen_constants() -> str:
    out = os.path.join(CSRC, "bls_constants.h")
    gen = os.path.join(CSRC, "gen_constants.py")
    if not os.path.exists(out) or os.path.getmtime(out) < os.path.getmtime(gen):
        subprocess.check_call([sys.executable, gen, out])
    return out


def hipcc_cmd(out: str, extra=()) -> list:
    return [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
            "-o", out, os.path.join(CSRC, "bls_kernels.hip"), *extra]


def build(force: bool = False, verbose: bool = False) -> str:
    gen_constants()
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= _newest_source_mtime():
        return LIB
    cmd = hipcc_cmd(LIB + ".tmp")
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(LIB + ".tmp", LIB)
    return LIB


def build_opcount(out_dir: str) -> str:
    """Variant with every Fp product counted (tools/opcount.py); never shipped."""
    gen_constants()
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, "liblodestar_bls_count.so")
    subprocess.check_call(hipcc_cmd(out, extra=("-DLB_COUNT_OPS",)))
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
