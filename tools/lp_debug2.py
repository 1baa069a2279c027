"""GPU debugging aid for the small-call path: valid requests of 1, 2, 3, 4 and 8 sets
(and a 1-set and 2-set request in one call) through the latency path and the
throughput pipeline; prints verdicts, rejection codes and set statuses."""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from bench import make_workload
    from lodestar_amd.native import Device, pack_blobs
    lp = Device(0)
    lp.set_latency_path(1 << 20)
    tp = Device(0)
    tp.set_latency_path(0)
    sks, pks, msgs, sigs = make_workload(lp, 16, 0, hashlib.sha256(b"dbg").digest())
    seed = hashlib.sha256(b"s").digest()
    for sizes in ([1], [2], [3], [4], [8], [1, 2], [2, 1, 1]):
        n = sum(sizes)
        req = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint32)
        blob, offs = pack_blobs(sigs[:n])
        args = (req, np.frombuffer(b"".join(pks[:n]), np.uint8), None, np.frombuffer(b"".join(msgs[:n]), np.uint8),
                blob, offs, seed)
        a = lp.verify_requests(*args)
        b = tp.verify_requests(*args)
        print(sizes, "lp", list(a.valid), list(a.errors), list(a.set_status), "| tp", list(b.valid), list(b.errors),
              list(b.set_status), flush=True)
    lp.close()
    tp.close()


if __name__ == "__main__":
    main()
