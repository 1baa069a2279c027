"""Debugging aid (not collected by pytest): one valid set through the latency path
with LB_LP_DUMP=1 (the library prints set 0's program inputs, flags and Miller
value on stderr), and the inputs the CPU tests build for the same set on stdout,
for comparison.  Usage: LB_LP_DUMP=1 python tests/debug_lp_dump.py 2> dump.txt > want.txt"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from lodestar_amd.native import Device, pack_blobs  # noqa: E402
from oracle import bls12_381 as O  # noqa: E402
from tests.lp_helper import mont, sample_sets, set_inputs  # noqa: E402


def main():
    pks, msgs, sigs = sample_sets(1)
    fps, flags = set_inputs(pks[0], msgs[0], sigs[0])
    print("want_in", " ".join("%x" % mont(v) for v in fps))
    print("want_fl", " ".join(str(f) for f in flags))
    dev = Device(0)
    dev.set_latency_path(1 << 20)
    blob, offs = pack_blobs([sigs[0]])
    import tempfile
    tmp = tempfile.TemporaryFile(mode="w+")
    sys.stderr.flush()
    saved = os.dup(2)
    os.dup2(tmp.fileno(), 2)
    try:
        r = dev.verify_requests(np.array([0, 1], np.uint32), np.frombuffer(O.g1_to_bytes(pks[0], False), np.uint8),
                                None, np.frombuffer(msgs[0], np.uint8), blob, offs, bytes(32))
    finally:
        os.dup2(saved, 2)
    print("verdict", list(r.valid), list(r.errors), list(r.set_status))
    tmp.seek(0)
    words = [int(x, 16) for x in tmp.read().split("lb_lp_dump")[1].split()]
    F = np.array(words[11 * 16 + 67:11 * 16 + 67 + 192], np.uint32).reshape(1, 12, 16)
    _, ofl, ms = dev.lp_program_run(3, F, np.zeros((1, 0), np.uint32), 0, 1)
    print("final program on the dumped F:", ofl.tolist(), ms)
    dev.close()


if __name__ == "__main__":
    main()
