"""Build a variant library whose latency path runs ROWS rows per workgroup (ROWS x 16
threads; programs compiled for ROWS rows with no block cap, which only the LDS-ring
interpreter needs): build/variants/lpROWS/liblodestar_bls.so, selected with LB_LIBRARY.
Usage: python tools/lp_rows_variant.py ROWS"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from lodestar_amd import build as B  # noqa: E402


def main():
    rows = int(sys.argv[1])
    name = "lp%d" % rows
    gen_dir = os.path.join(ROOT, "build", "variants", name, "gen")
    os.makedirs(gen_dir, exist_ok=True)
    env = dict(os.environ, LB_LP_GEN_ROWS=str(rows), LB_LP_GEN_CAP=str(1 << 20))
    subprocess.check_call([sys.executable, os.path.join(B.CSRC, "gen_lp.py"), gen_dir], env=env)
    hdr = os.path.join(gen_dir, "bls_lp_progs.h")
    print(B.build_variant(name, ["-DLB_LP_ROWS=%d" % rows, '-DLB_LP_PROGS_HEADER="%s"' % hdr],
                          blob=os.path.join(gen_dir, "lp_programs.bin")))


if __name__ == "__main__":
    main()
