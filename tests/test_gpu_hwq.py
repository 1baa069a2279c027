"""lb_create's hardware-queue guard: every HIP hardware queue
reserves scratch for the library's largest private segment at full occupancy, so
lb_create prices EVERY queue the context opens -- plain streams (pooled into
GPU_MAX_HW_QUEUES queues), CU-masked streams (a queue each), the priority lane and
the aux stream -- against the budget of the largest configuration seen to run, and
refuses one above it with LB_ERR_RESOURCES and the arithmetic, before any stream
exists (instead of failing later inside a dispatch with
HSA_STATUS_ERROR_OUT_OF_RESOURCES, profiles/ab_r03/r03g_q24_fail.txt).
The refused configurations are never run (no stream is created for them)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROBE = r"""
import json, sys
sys.path.insert(0, %r)
from lodestar_amd import native
out = {}
per_q, lane = native.scratch_per_queue(0)
out["per_queue"], out["lane"] = per_q, lane
try:
    d = native.Device(0)
    out["slots"] = d.slots()
    out["hw_queues"] = d.hw_queues()
    d.close()
except native.LodestarBlsError as e:
    out["error"] = str(e)
print(json.dumps(out))
""" % ROOT


def _probe(queues, **env_extra):
    env = dict(os.environ, GPU_MAX_HW_QUEUES=str(queues))
    for k in ("LB_SLOTS", "LB_PRIO_DYN_SLOTS", "LB_PRIO_CUS", "LB_PRIO_DYN", "LB_SCRATCH_BUDGET_GB"):
        env.pop(k, None)
    env.update(env_extra)
    r = subprocess.run([sys.executable, "-c", PROBE], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_hw_queue_guard():
    # the default configuration: 16 plain + 2 CU-masked + 2 high-priority queues
    at_cap = _probe(16)
    print("\n16 queues (default):", at_cap)
    assert at_cap.get("slots") == 16, at_cap
    assert at_cap["hw_queues"] == 20, at_cap
    assert at_cap["lane"] > 0 and at_cap["per_queue"] % (at_cap["lane"] * 64 * 32) == 0
    # GPU_MAX_HW_QUEUES above the slot cap: refused before any stream exists
    over = _probe(17)
    print("17 queues:", over)
    assert "error" in over and "failed with -5" in over["error"] and "scratch" in over["error"], over
    # one more CU-masked queue than the default: 21 queues, over the budget, refused
    masked = _probe(16, LB_PRIO_DYN_SLOTS="3")
    print("16 + 3 masked:", masked)
    assert "error" in masked and "failed with -5" in masked["error"], masked
    assert "3 CU-masked" in masked["error"] and "21 hardware queues" in masked["error"], masked


def test_sync_call_keeps_two_streams_with_prio_dyn():
    """a synchronous call above the latency path's size borrows slot 1's
    stream (the two-stream DAG); with LB_PRIO_DYN on, pick_streams used to overwrite
    it, so the call ran on one stream."""
    code = r"""
import json, sys, os
sys.path.insert(0, %r)
import numpy as np
from lodestar_amd import native
from oracle import bls12_381 as O
import hashlib
d = native.Device(0)
d.set_latency_path(0)
sks = [O.interop_secret_key(i) for i in range(8)]
sk_be = [s.to_bytes(32, "big") for s in sks]
msgs = [hashlib.sha256(bytes([i])).digest() for i in range(8)]
pks = d.sk_to_pk(sk_be)
sigs = d.sign(sk_be, msgs)
blob, offs = native.pack_blobs(sigs)
# the priority lane in use (LB_PRIO_DYN: the throughput streams switch to their masked pair)
d.set_latency_path(1024)
r0 = d.verify_requests(np.array([0, 1], np.uint32), np.frombuffer(b"".join(pks[:1]), np.uint8), None,
                       np.frombuffer(b"".join(msgs[:1]), np.uint8), blob[:96], offs[:2], bytes(32))
d.set_latency_path(0)
r = d.verify_requests(np.array([0, 4, 8], np.uint32), np.frombuffer(b"".join(pks), np.uint8), None,
                      np.frombuffer(b"".join(msgs), np.uint8), blob, offs, bytes(32))
print(json.dumps({"valid": [int(v) for v in r.valid] + [int(r0.valid[0])], "streams": d.last_call_streams()}))
d.close()
""" % ROOT
    env = dict(os.environ, LB_PRIO_DYN="1", GPU_MAX_HW_QUEUES="16")
    env.pop("LB_SLOTS", None)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=180, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    print("\n", out)
    assert out["valid"] == [1, 1, 1], out
    assert out["streams"] == 2, out
