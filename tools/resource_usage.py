"""Per-kernel register / LDS / spill / occupancy table of the gfx950 build
(hipcc -Rpass-analysis=kernel-resource-usage, device-only compile of each unit).
Usage: python tools/resource_usage.py [unit.hip ...] > profiles/resource_usage_rNN.txt"""
import os
import re
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from lodestar_amd import build as B  # noqa: E402


def usage(unit, extra=()):
    cmd = [B.HIPCC, f"--offload-arch={B.ARCH}", *B.FLAGS, *extra, "--offload-device-only", "-c", "-o", "/dev/null",
           "-Rpass-analysis=kernel-resource-usage", os.path.join(B.CSRC, unit)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    out, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"kernel": m.group(1)}
            out.append(cur)
            continue
        m = re.search(r"remark:\s+([\w \[\]/]+?): (\S+) \[", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = m.group(2)
    return unit, out


def main():
    units = sys.argv[1:] or [u for u in B.UNITS if u != "bls_host.hip"]
    with ThreadPoolExecutor(8) as ex:
        res = list(ex.map(usage, units))
    keys = ["VGPRs", "AGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]", "SGPRs Spill", "VGPRs Spill",
            "LDS Size [bytes/block]"]
    print("kernel | " + " | ".join(keys))
    for unit, ks in res:
        for k in ks:
            if "__device_stub" in k["kernel"]:
                continue
            print(f"{k['kernel'][:60]} | " + " | ".join(str(k.get(x, "-")) for x in keys))


if __name__ == "__main__":
    main()
