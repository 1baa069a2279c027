"""Build the N-API addon (addon.cc -> lodestar_bls.node) against the node
headers in /usr/include/node (N-API is ABI-stable: the same addon loads in any
node >= 12.22 that offers N-API 8, including the node 20 line the reference
requires).  Links liblodestar_bls.so from the package directory (rpath
$ORIGIN/..), so the addon loads wherever the package is unpacked."""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
ROOT = os.path.dirname(PKG)
OUT = os.path.join(HERE, "lodestar_bls.node")
NODE_INCLUDE = os.environ.get("NODE_INCLUDE", "/usr/include/node")


def available() -> bool:
    return os.path.exists(os.path.join(NODE_INCLUDE, "node_api.h")) and shutil.which("g++") is not None


def build(force: bool = False, verbose: bool = False) -> str:
    src = os.path.join(HERE, "addon.cc")
    deps = [src, os.path.join(ROOT, "include", "lodestar_bls.h"), os.path.join(PKG, "liblodestar_bls.so")]
    if not force and os.path.exists(OUT) and os.path.getmtime(OUT) >= max(os.path.getmtime(p) for p in deps):
        return OUT
    cmd = ["g++", "-std=c++17", "-O2", "-fPIC", "-shared", "-Wall", "-Wno-unused-function",
           "-DNODE_GYP_MODULE_NAME=lodestar_bls", f"-I{NODE_INCLUDE}", f"-I{os.path.join(ROOT, 'include')}",
           src, "-o", OUT + ".tmp", f"-L{PKG}", "-llodestar_bls", "-Wl,-rpath,$ORIGIN/..", "-pthread"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
