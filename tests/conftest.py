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


def load_golden(name):
    import json
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)
