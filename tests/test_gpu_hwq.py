"""lb_create's hardware-queue cap: every HIP hardware queue
reserves scratch for the library's largest private segment at full occupancy, so
GPU_MAX_HW_QUEUES above 16 is refused with LB_ERR_RESOURCES and a message that
prices the reservation, instead of failing later inside a dispatch
(HSA_STATUS_ERROR_OUT_OF_RESOURCES, profiles/ab_r03/r03g_q24_fail.txt).
The refusal happens before any stream exists; 16 (the cap) must still work."""
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
    d.close()
except native.LodestarBlsError as e:
    out["error"] = str(e)
print(json.dumps(out))
""" % ROOT


def _probe(queues):
    env = dict(os.environ, GPU_MAX_HW_QUEUES=str(queues))
    env.pop("LB_SLOTS", None)
    r = subprocess.run([sys.executable, "-c", PROBE], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_hw_queue_cap():
    at_cap = _probe(16)
    print("\n16 queues:", at_cap)
    assert at_cap.get("slots") == 16, at_cap
    assert at_cap["lane"] > 0 and at_cap["per_queue"] == at_cap["lane"] * 64 * 32 * (at_cap["per_queue"] // (at_cap["lane"] * 64 * 32))
    over = _probe(17)
    print("17 queues:", over)
    assert "error" in over and "failed with -5" in over["error"] and "scratch" in over["error"], over
