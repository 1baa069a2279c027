"""The Lodestar-side host: the N-API addon and the JS BlsGpuVerifier, run under
node (tests/js/).  CPU: scheduling semantics with a mock backend, addon loading,
argument marshalling and error -> rejection.  GPU: the golden verdict tables
replayed through the addon on cuda:0."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NODE = shutil.which("node")
ADDON = os.path.join(ROOT, "lodestar_amd", "napi", "lodestar_bls.node")

pytestmark = pytest.mark.skipif(NODE is None, reason="node not installed")


def _node(script, timeout=120):
    r = subprocess.run([NODE, os.path.join(ROOT, "tests", "js", script)], capture_output=True, text=True,
                       timeout=timeout, cwd=ROOT)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_js_verifier_scheduling():
    out = _node("test_host.js")
    assert "0 failed" in out


@pytest.fixture(scope="module")
def addon_built():
    if not os.path.exists(ADDON):
        from lodestar_amd.napi import build as nb
        if not nb.available():
            pytest.skip("node headers not available")
        nb.build()
    return ADDON


def test_addon_loads_and_marshals(addon_built):
    assert "addon ok" in _node("test_addon.js")


@pytest.mark.gpu
def test_addon_gpu_replay(addon_built):
    out = _node("gpu_replay.js", timeout=300)
    assert '"verify_requests"' in out and '"sharded"' in out


@pytest.mark.gpu
def test_addon_e2e_multithread_under_load(addon_built, tmp_path):
    """BNT/e2e/chain/bls/multithread.test.ts:85-129 through the real addon on the GPU,
    with 16 C2-sized packages in flight through the same verifier (tests/js/e2e_multithread.js)."""
    import hashlib
    import json

    from lodestar_amd.native import Device
    from oracle import bls12_381 as O
    n = 4096
    dev = Device(0)
    try:
        sks = [O.interop_secret_key(i).to_bytes(32, "big") for i in range(n)]
        msgs = [hashlib.sha256(b"e2e-load" + i.to_bytes(4, "little")).digest() for i in range(n)]
        pks = dev.sk_to_pk(sks)
        sigs = dev.sign(sks, msgs)
    finally:
        dev.close()
    for name, items in (("pks", pks), ("msgs", msgs), ("sigs", sigs)):
        (tmp_path / (name + ".bin")).write_bytes(b"".join(items))
    r = subprocess.run([NODE, os.path.join(ROOT, "tests", "js", "e2e_multithread.js"), str(tmp_path)],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    rep = json.loads(r.stdout.strip().splitlines()[-1])
    print("\n", json.dumps(rep))
    assert len(rep["cases"]) == 8 and rep["load_sets_done"] >= 16 * 65536
