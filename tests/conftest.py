import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")
    config.addinivalue_line("markers", "slow: long CPU-oracle cases")


@pytest.fixture(scope="session")
def device():
    from lodestar_amd.native import Device
    dev = Device(0)
    yield dev
    dev.close()


@pytest.fixture(scope="session", params=["lane", "lines", "wave", "lp"])
def device_modes(request):
    """A context per verification organisation.  Throughput pipeline (latency
    path off): one pair per lane (k_miller_sets), stored lines + multi-pair
    accumulation (k_lines / k_miller_acc, which the library otherwise picks only
    for calls of >= 1025 sets) and stored lines + one wave per pair (k_lines /
    k_pair_wc).  "lp": every call on the latency path (k_lp_verify, one
    workgroup per set running the round programs), whatever its size."""
    import os
    from lodestar_amd.native import Device
    old = os.environ.get("LB_MILLER")
    os.environ["LB_MILLER"] = "auto" if request.param == "lp" else request.param
    try:
        dev = Device(0)
        dev.set_latency_path(1 << 20 if request.param == "lp" else 0)
    finally:
        if old is None:
            os.environ.pop("LB_MILLER", None)
        else:
            os.environ["LB_MILLER"] = old
    yield dev
    dev.close()


def load_golden(name):
    import json
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)
