"""Two-phase (multi-GPU combine) calls on the C2 workload, one process: device-resident
inputs as bench.py --gpus N, one call and 16 in flight; reports verdict counts."""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")


def main():
    import numpy as np
    import torch

    from bench import make_workload
    from lodestar_amd.native import Device
    dev = Device(0)
    n = 65536
    sks, pks, msgs, sigs = make_workload(dev, n, 0, hashlib.sha256(b"lodestar-mi355x-bench").digest())
    cuda = torch.device("cuda", 0)
    d_pk = torch.from_numpy(np.frombuffer(b"".join(pks), np.uint8).copy()).to(cuda)
    d_msg = torch.from_numpy(np.frombuffer(b"".join(msgs), np.uint8).copy()).to(cuda)
    d_sig = torch.from_numpy(np.frombuffer(b"".join(sigs), np.uint8).copy()).to(cuda)
    so = np.arange(0, 96 * (n + 1), 96, dtype=np.uint32)
    ro = np.arange(0, n + 1, 128, dtype=np.uint32)
    nr = len(ro) - 1
    d_so = torch.from_numpy(so.view(np.int32)).to(cuda)
    d_ro = torch.from_numpy(ro.view(np.int32)).to(cuda)
    d_seed = torch.from_numpy(np.frombuffer(hashlib.sha256(b"batch-rand").digest(), np.uint8).copy()).to(cuda)
    nbuf = 16
    d_valid = [torch.zeros(nr, dtype=torch.uint8, device=cuda) for _ in range(nbuf)]
    d_err = [torch.zeros(nr, dtype=torch.uint8, device=cuda) for _ in range(nbuf)]
    torch.cuda.synchronize()

    def submit(k, partial):
        return dev.verify_requests_device_async(nr, n, d_ro.data_ptr(), d_pk.data_ptr(), None, d_msg.data_ptr(),
                                                d_sig.data_ptr(), d_so.data_ptr(), d_seed.data_ptr(),
                                                d_valid[k % nbuf].data_ptr(), d_err[k % nbuf].data_ptr(),
                                                partial=partial)

    def counts(k):
        torch.cuda.synchronize()
        v = d_valid[k % nbuf].cpu().numpy()
        e = d_err[k % nbuf].cpu().numpy()
        return int(v.sum()), int((e != 0).sum())

    out = {}
    for b in d_valid:
        b.zero_()
    t = submit(0, False)
    dev.wait(t)
    out["one_call"] = counts(0)
    d_valid[0].zero_()
    t = submit(0, True)
    part = dev.partial_wait_t(t)
    ok = dev.gt_check([part])
    dev.finish_t(t, ok)
    dev.wait(t)
    out["one_two_phase"] = (ok,) + counts(0)
    for b in d_valid:
        b.zero_()
    pend, res = [], []
    for k in range(32):
        pend.append((k, submit(k, True)))
        if len(pend) >= nbuf:
            kk, tt = pend.pop(0)
            p = dev.partial_wait_t(tt)
            okk = dev.gt_check([p])
            dev.finish_t(tt, okk)
            dev.wait(tt)
            res.append((kk, okk) + counts(kk))
    for kk, tt in pend:
        p = dev.partial_wait_t(tt)
        okk = dev.gt_check([p])
        dev.finish_t(tt, okk)
        dev.wait(tt)
        res.append((kk, okk) + counts(kk))
    out["inflight16"] = res
    for env in ("LB_ACC=pairs",):
        pass
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
