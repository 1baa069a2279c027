"""Build the C restatement of the oracle (test infrastructure only).

    python -m oracle.build_c      -> oracle/c/libbls_oracle.so

gcc -O3 on oracle/c/bls_oracle.c with the constants generated from the pinned
Python oracle (oracle/gen_c_consts.py).  Portable x86-64-v2 code so the .so
built here also runs on the GPU box's host CPU (bench.py cpu_baseline leg).
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CDIR = os.path.join(HERE, "c")
SRC = os.path.join(CDIR, "bls_oracle.c")
CONSTS = os.path.join(CDIR, "bls_oracle_consts.h")
LIB = os.path.join(CDIR, "libbls_oracle.so")        # x86-64-v2: runs on any x86-64 host
LIB_V3 = os.path.join(CDIR, "libbls_oracle_v3.so")  # x86-64-v3 (AVX2/BMI2 mulx): picked when the host has it


def build(force: bool = False, verbose: bool = False) -> str:
    gen = os.path.join(HERE, "gen_c_consts.py")
    oracle_py = os.path.join(HERE, "bls12_381.py")
    if force or not os.path.exists(CONSTS) or os.path.getmtime(CONSTS) < max(os.path.getmtime(gen),
                                                                            os.path.getmtime(oracle_py)):
        subprocess.check_call([sys.executable, gen, CONSTS], cwd=os.path.dirname(HERE))
    deps = [SRC, CONSTS, os.path.abspath(__file__)]
    for lib, march in ((LIB, "x86-64-v2"), (LIB_V3, "x86-64-v3")):
        if not force and os.path.exists(lib) and os.path.getmtime(lib) >= max(os.path.getmtime(p) for p in deps):
            continue
        cmd = ["gcc", "-O3", f"-march={march}", "-std=gnu11", "-shared", "-fPIC", "-pthread", "-Wall",
               "-Wno-unused-function", "-o", lib + ".tmp", SRC]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)
        os.replace(lib + ".tmp", lib)
    return LIB


def host_supports_v3() -> bool:
    try:
        flags = next(l for l in open("/proc/cpuinfo") if l.startswith("flags")).split()
    except (OSError, StopIteration):
        return False
    return all(f in flags for f in ("avx2", "bmi2", "fma", "movbe"))


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
