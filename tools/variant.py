"""Tuning variants of the library that differ in a few units only: reuse the
main build's objects, recompile UNITS with extra flags, link under
build/variants/NAME/liblodestar_bls.so (select with LB_LIBRARY=...).
usage: python tools/variant.py NAME unit.hip[,unit.hip] -DFLAG ..."""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from lodestar_amd import build as B  # noqa: E402


def main():
    name, units, extra = sys.argv[1], sys.argv[2].split(","), sys.argv[3:]
    B.build()
    d = os.path.join(ROOT, "build", "variants", name)
    od = os.path.join(d, "obj")
    os.makedirs(od, exist_ok=True)
    objs = []
    procs = []
    for u in B.UNITS:
        o = os.path.join(od, os.path.splitext(u)[0] + ".o")
        objs.append(o)
        if u in units:
            cmd = [B.HIPCC, f"--offload-arch={B.ARCH}", *B.FLAGS, *extra, "-c", "-o", o, os.path.join(B.CSRC, u)]
            procs.append(subprocess.Popen(cmd))
        else:
            shutil.copy2(os.path.join(B.OBJ_DIR, os.path.basename(o)), o)
    if any(p.wait() for p in procs):
        raise SystemExit("hipcc failed")
    lib = os.path.join(d, "liblodestar_bls.so")
    subprocess.check_call([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", lib, *objs])
    print(lib)


if __name__ == "__main__":
    main()
