"""GPU signing roots (lb_signing_roots_*) bit-exact against the reference-pinned
vectors of tests/golden/ssz.json and the SSZ oracle."""
import hashlib
import random

import pytest

from oracle import ssz as S
from tests.conftest import load_golden

pytestmark = pytest.mark.gpu
G = load_golden("ssz.json")


def test_attestation_signing_roots_mainnet(device):
    data = [bytes.fromhex(a["ssz"]) for a in G["attestations"]]
    got = device.signing_roots_attestation(data, bytes.fromhex(G["domain_attester"]))
    assert [g.hex() for g in got] == [a["signing_root"] for a in G["attestations"]]
    # per-object domains (stride 32)
    doms = [hashlib.sha256(bytes([i])).digest() for i in range(len(data))]
    got = device.signing_roots_attestation(data, doms)
    assert got == [S.compute_signing_root(S.attestation_data_root(d), dm) for d, dm in zip(data, doms)]


def test_block_proposer_signing_roots(device):
    fr = [[bytes.fromhex(x) for x in b["field_roots"]] for b in G["blocks"]]
    got = device.signing_roots_chunks(fr, bytes.fromhex(G["domain_proposer"]))
    assert [g.hex() for g in got] == [b["signing_root"] for b in G["blocks"]]


def test_deposit_signing_root_kat(device):
    d = G["deposit"]
    got = device.signing_roots_chunks([[bytes.fromhex(x) for x in d["field_roots"]]], bytes.fromhex(d["domain"]))
    assert got[0].hex() == d["signing_root"]


@pytest.mark.parametrize("m", [1, 2, 3, 5, 8, 9, 16])
def test_chunks_random_vs_oracle(device, m):
    rnd = random.Random(m)
    objs = [[rnd.randbytes(32) for _ in range(m)] for _ in range(300)]
    doms = [rnd.randbytes(32) for _ in range(300)]
    got = device.signing_roots_chunks(objs, doms)
    assert got == [S.signing_root_from_field_roots(o, d) for o, d in zip(objs, doms)]


def test_attestations_random_large_vs_oracle(device):
    rnd = random.Random(5)
    data = [rnd.randbytes(128) for _ in range(5000)]
    dom = rnd.randbytes(32)
    got = device.signing_roots_attestation(data, dom)
    idx = rnd.sample(range(5000), 200)
    for i in idx:
        assert got[i] == S.compute_signing_root(S.attestation_data_root(data[i]), dom)


def test_device_signing_roots_feed_verification(device):
    """Signing roots computed in HBM become the messages of a device-resident
    verify call (no host round trip): attestations signed over their roots verify."""
    import numpy as np
    import torch

    from oracle import bls12_381 as O
    rnd = random.Random(11)
    n = 40
    data = [rnd.randbytes(128) for _ in range(n)]
    dom = rnd.randbytes(32)
    roots = [S.compute_signing_root(S.attestation_data_root(d), dom) for d in data]
    sks = [O.interop_secret_key(i).to_bytes(32, "big") for i in range(n)]
    sigs = device.sign(sks, roots)
    pks = device.sk_to_pk(sks)
    cuda = torch.device("cuda", 0)
    t = lambda b: torch.from_numpy(np.frombuffer(b, np.uint8).copy()).to(cuda)  # noqa: E731
    d_data, d_dom, d_msgs = t(b"".join(data)), t(dom), torch.zeros(32 * n, dtype=torch.uint8, device=cuda)
    device.signing_roots_attestation_device(n, d_data.data_ptr(), d_dom.data_ptr(), 0, d_msgs.data_ptr())
    assert d_msgs.cpu().numpy().tobytes() == b"".join(roots)
    d_pks, d_sigs = t(b"".join(pks)), t(b"".join(sigs))
    d_sigoff = torch.from_numpy(np.arange(0, 96 * (n + 1), 96, dtype=np.uint32).view(np.int32)).to(cuda)
    d_req = torch.from_numpy(np.array([0, 20, n], np.uint32).view(np.int32)).to(cuda)
    d_seed = torch.zeros(32, dtype=torch.uint8, device=cuda)
    d_valid = torch.zeros(2, dtype=torch.uint8, device=cuda)
    d_err = torch.zeros(2, dtype=torch.uint8, device=cuda)
    device.verify_requests_device(2, n, d_req.data_ptr(), d_pks.data_ptr(), None, d_msgs.data_ptr(),
                                  d_sigs.data_ptr(), d_sigoff.data_ptr(), d_seed.data_ptr(), d_valid.data_ptr(),
                                  d_err.data_ptr())
    assert d_valid.cpu().tolist() == [1, 1] and d_err.cpu().tolist() == [0, 0]
