"""The two-phase contract under LB_TP_RELEASE=1 (the default; include/lodestar_bls.h,
"Contract of the default flow"), VERDICT r5 #3 / ADVICE r5:

- a released call's outputs are provisional until lb_wait; at most 256 two-phase calls
  may be unfinished: the 257th is refused with LB_ERR_RESOURCES (nothing enqueued)
  instead of overwriting a record whose provisional "valid" verdicts only it can turn
  into final ones;
- a failed combined check (an invalid set in the shard) still yields per-request false
  after the release, for host and device buffers;
- a failure of the failed combine's re-run is an error from lb_verify_requests_finish
  AND from lb_wait (never the provisional verdicts), and through node it rejects the
  finish() promise (napi/addon.cc Kind::Finish).
Expected verdicts come from the oracle's core_verify of each set (oracle/bls12_381.py)."""
import hashlib
import json
import os
import shutil
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _sets(dev, n=8, bad=()):
    from oracle import bls12_381 as O
    sks = [O.interop_secret_key(i).to_bytes(32, "big") for i in range(n)]
    msgs = [hashlib.sha256(b"tp-ring" + bytes([i])).digest() for i in range(n)]
    pks = dev.sk_to_pk(sks)
    sigs = dev.sign(sks, msgs)
    msgs = [hashlib.sha256(b"wrong").digest() if i in bad else m for i, m in enumerate(msgs)]
    # the expectation from the oracle, set by set
    expect = [O.core_verify(O.sk_to_pk(int.from_bytes(sks[i], "big")), msgs[i], O.signature_from_bytes(sigs[i]))
              for i in range(n)]
    return pks, msgs, sigs, expect


def _args(pks, msgs, sigs, per_req):
    from lodestar_amd.native import pack_blobs
    n = len(msgs)
    req = np.arange(0, n + 1, per_req, dtype=np.uint32)
    blob, offs = pack_blobs(sigs)
    return (req, np.frombuffer(b"".join(pks), np.uint8), None, np.frombuffer(b"".join(msgs), np.uint8), blob, offs,
            hashlib.sha256(b"tp-seed").digest())


def test_ring_refuses_the_257th_unfinished_call():
    from lodestar_amd.native import Device, LodestarBlsError
    dev = Device(0)
    try:
        pks, msgs, sigs, expect = _sets(dev, 4)
        assert all(expect)
        args = _args(pks, msgs, sigs, 2)
        calls = []
        refused = None
        for k in range(300):
            try:
                calls.append(dev.verify_requests_async(*args, partial=True))
            except LodestarBlsError as e:
                refused = (k, str(e))
                break
        assert refused is not None, "300 unfinished two-phase calls accepted"
        k, msg = refused
        print("\nrefused at call", k + 1, ":", msg)
        assert k == 256 and "(-5)" in msg and "two-phase ring full" in msg, refused
        # tickets consecutive: the refused call took none (nothing enqueued)
        assert [c.ticket for c in calls] == list(range(calls[0].ticket, calls[0].ticket + 256))
        # finishing + waiting for the oldest frees exactly its entry
        first = calls[0]
        assert dev.gt_check([dev.partial_wait(first)])
        dev.verify_finish(first, True)
        r = dev.wait_call(first)
        assert r.valid.tolist() == [1, 1]
        calls.append(dev.verify_requests_async(*args, partial=True))
        with pytest.raises(LodestarBlsError, match="two-phase ring full"):
            dev.verify_requests_async(*args, partial=True)
        # every other call: its own combine, then final verdicts
        for c in calls[1:]:
            ok = dev.gt_check([dev.partial_wait(c)])
            assert ok
            dev.verify_finish(c, ok)
            assert dev.wait_call(c).valid.tolist() == [1, 1]
        # a finish of a ticket whose record was reused is a no-op, not an error
        dev.finish_t(first.ticket, True)
    finally:
        dev.close()


def _device_call(dev, args, torch, cuda):
    req, pk, _, mg, blob, offs, seed = args
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x).copy()).to(cuda)  # noqa: E731
    d = [t(req.view(np.int32)), t(pk), t(mg), t(blob), t(offs.view(np.int32)), t(np.frombuffer(seed, np.uint8))]
    d_valid = torch.zeros(len(req) - 1, dtype=torch.uint8, device=cuda)
    d_err = torch.zeros(len(req) - 1, dtype=torch.uint8, device=cuda)
    torch.cuda.synchronize()
    tk = dev.verify_requests_device_async(len(req) - 1, int(req[-1]), d[0].data_ptr(), d[1].data_ptr(), None,
                                          d[2].data_ptr(), d[3].data_ptr(), d[4].data_ptr(), d[5].data_ptr(),
                                          d_valid.data_ptr(), d_err.data_ptr(), partial=True)
    ok = dev.gt_check([dev.partial_wait_t(tk)])
    dev.finish_t(tk, ok)
    dev.wait(tk)
    return ok, [bool(v) for v in d_valid.cpu().numpy()], d_err.cpu().numpy()


def test_failed_combine_after_release_host_and_device():
    """A failed combine gives per-request false after the release (host buffers, then device
    buffers on a fresh context: the provisional outputs are overwritten by the re-run); the
    call after a failed combine takes the legacy mode (kTpPause) with the same verdicts."""
    import torch
    from lodestar_amd.native import Device
    cuda = torch.device("cuda", 0)
    dev = Device(0)
    try:
        pks, msgs, sigs, expect = _sets(dev, 8, bad={5})
        want = [all(expect[0:4]), all(expect[4:8])]
        assert want == [True, False]
        args = _args(pks, msgs, sigs, 4)
        # host buffers, release mode (a fresh context)
        pc = dev.verify_requests_async(*args, partial=True)
        ok = dev.gt_check([dev.partial_wait(pc)])
        assert not ok
        dev.verify_finish(pc, ok)
        r = dev.wait_call(pc)
        assert [bool(v) for v in r.valid] == want and r.batch_retries == 1
        # the next calls after the failure: legacy mode, same verdicts (device, then host)
        ok, got, err = _device_call(dev, args, torch, cuda)
        assert not ok and got == want and not err.any()
        pc = dev.verify_requests_async(*args, partial=True)
        ok = dev.gt_check([dev.partial_wait(pc)])
        dev.verify_finish(pc, ok)
        assert [bool(v) for v in dev.wait_call(pc).valid] == want
    finally:
        dev.close()
    dev = Device(0)
    try:  # device buffers, release mode
        ok, got, err = _device_call(dev, args, torch, cuda)
        assert not ok and got == want and not err.any()
    finally:
        dev.close()


PROBE_FAULT = r"""
import json, sys, hashlib
sys.path.insert(0, %r)
sys.path.insert(0, %r)
import numpy as np
from lodestar_amd.native import Device, LodestarBlsError
from test_gpu_twophase import _sets, _args
dev = Device(0)
pks, msgs, sigs, expect = _sets(dev, 4, bad={1})
pc = dev.verify_requests_async(*_args(pks, msgs, sigs, 2), partial=True)
ok = dev.gt_check([dev.partial_wait(pc)])
out = {"ok": ok}
try:
    dev.verify_finish(pc, ok)
    out["finish"] = "no error"
except LodestarBlsError as e:
    out["finish"] = str(e)
try:
    r = dev.wait_call(pc)
    out["wait"] = [int(v) for v in r.valid]
except LodestarBlsError as e:
    out["wait"] = str(e)
dev.close()
print(json.dumps(out))
"""


def test_failed_rerun_is_an_error_not_verdicts():
    env = dict(os.environ, LB_FAULT_RERUN="1")
    r = subprocess.run([sys.executable, "-c", PROBE_FAULT % (ROOT, os.path.join(ROOT, "tests"))], env=env,
                       capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    print("\n", out)
    assert out["ok"] is False
    assert "LB_FAULT_RERUN" in out["finish"] and "(-2)" in out["finish"], out
    assert isinstance(out["wait"], str) and "not verdicts" in out["wait"], out


@pytest.mark.skipif(shutil.which("node") is None, reason="node not installed")
def test_finish_error_rejects_through_node(tmp_path):
    """napi/addon.cc: a failing lb_verify_requests_finish rejects finish()'s promise."""
    from lodestar_amd.native import Device
    dev = Device(0)
    try:
        pks, msgs, sigs, _ = _sets(dev, 4, bad={1})
    finally:
        dev.close()
    for name, items in (("pks", pks), ("msgs", msgs), ("sigs", sigs)):
        (tmp_path / (name + ".bin")).write_bytes(b"".join(items))
    env = dict(os.environ, LB_FAULT_RERUN="1")
    r = subprocess.run(["node", os.path.join(ROOT, "tests", "js", "finish_error.js"), str(tmp_path)], env=env,
                       capture_output=True, text=True, timeout=180, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    rep = json.loads(r.stdout.strip().splitlines()[-1])
    print("\n", rep)
    assert rep["gt_ok"] is False and rep["rejected"] and rep["code"] == "LB_ERR_DEVICE", rep
