"""getBlockSignatureSets on the GPU: SSZ blocks -> sets with
GPU-computed signing roots and validator-index pubkeys -> one verify request per
block (verifyBlocksSignatures.ts:38-55).  Roots against oracle/ssz.py and the
reference's mainnet fixture; verdicts against the C oracle over the same sets."""
import json
import os

import numpy as np
import pytest

import blocks_helper as BH
from lodestar_amd import block_sets as B

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
NV = 96


@pytest.fixture(scope="module")
def backend():
    from lodestar_amd.verifier import DeviceBackend
    sys_path_tools()
    import workloads as W
    b = DeviceBackend(0, seed_source=lambda: bytes(range(32)))
    keys = W.make_keys(b.dev, NV)
    assert b.dev.pubkey_table_append(keys.pks) == NV
    yield b, keys
    b.close()


def sys_path_tools():
    import sys
    p = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools")
    if p not in sys.path:
        sys.path.insert(0, p)


def test_mainnet_block_roots_on_gpu(backend):
    b, _ = backend
    blocks = json.load(open(os.path.join(GOLD, "blocks_ssz.json")))["blocks"]
    sizes = {}
    for blk in blocks:
        for a in B.parse_signed_block(bytes.fromhex(blk["ssz"]), "phase0").attestations:
            n = (len(a.aggregation_bits) - 1) * 8 + a.aggregation_bits[-1].bit_length() - 1
            sizes[(int.from_bytes(a.data[0:8], "little"), int.from_bytes(a.data[8:16], "little"))] = n
    gpu = B.BlockSignatureSetBuilder(b.dev, B.MAINNET, lambda s, i: list(range(sizes[(s, i)])))
    cpu = B.BlockSignatureSetBuilder(BH.OracleRoots(), B.MAINNET, lambda s, i: list(range(sizes[(s, i)])))
    ssz = [bytes.fromhex(x["ssz"]) for x in blocks]
    got, want = gpu.build(ssz), cpu.build(ssz)
    assert [[s.signing_root for s in x] for x in got] == [[s.signing_root for s in x] for x in want]
    gold = json.load(open(os.path.join(GOLD, "ssz.json")))
    assert [s.signing_root.hex() for x in got for s in x[1:-1]] == [a["signing_root"] for a in gold["attestations"]]


def _chain():
    return (BH.Chain(bytes(range(32)), [(0, bytes(4)), (2, bytes([1, 0, 0, 0]))]),
            B.ChainConfig(bytes(range(32)), [(0, bytes(4), "phase0"), (2, bytes([1, 0, 0, 0]), "altair")]))


def test_block_import_end_to_end(backend):
    """Four blocks (two phase0, two altair with a sync aggregate) carrying every operation
    kind; block 2's first attestation signature is replaced by another valid signature.
    Verdicts per block through the device path equal the C oracle's."""
    from oracle import c_oracle as C
    from lodestar_amd.native import pack_blobs
    b, keys = backend
    chain, config = _chain()
    committee, sync = BH.committee_of(NV), BH.sync_committee_of(NV)
    blocks, parent = [], bytes(32)
    for n, slot in enumerate([40, 41, 70, 71]):
        corrupt = n == 2

        def sign(sks, roots, corrupt=corrupt):
            sig = W_sign(b.dev, sks, roots)
            if corrupt and len(sig) > 8:
                sig[1 + 2 + 2] = sig[0]  # first attestation (after randao, 1 proposer slashing, 1 attester slashing)
            return sig
        ssz, expected, root, _ = BH.make_block(sign, keys.sks, chain, slot, (7 * n) % NV, parent, committee, sync,
                                               n_atts=6, n_exits=2, n_prop_sl=1, n_att_sl=1, n_deposits=1,
                                               sync_participants=200, seed=n)
        blocks.append(ssz)
        parent = root
    sets = B.BlockSignatureSetBuilder(b.dev, config, committee, sync).build(blocks)
    valid, errors = b.verify_requests(sets)
    assert valid == [True, True, False, True]
    # C oracle over the same sets, pubkeys as bytes
    flat = [s for blk in sets for s in blk]
    req_off = np.cumsum([0] + [len(x) for x in sets]).astype(np.uint32)
    idx = [[s.pubkey.index] if s.pubkey is not None else [k.index for k in s.pubkeys] for s in flat]
    pk_off = np.cumsum([0] + [len(i) for i in idx]).astype(np.uint32)
    pks = np.frombuffer(b"".join(keys.pks[i] for ix in idx for i in ix), np.uint8)
    blob, offs = pack_blobs([s.signature for s in flat])
    v, e = C.verify_requests(req_off, pks, pk_off, np.frombuffer(b"".join(s.signing_root for s in flat), np.uint8),
                             blob, offs, bytes(range(32)), threads=16)
    assert list(v) == [int(x) for x in valid] and list(e) == list(errors)


def W_sign(dev, sks, roots):
    sys_path_tools()
    import workloads as W
    return W.sign_many(dev, sks, roots)
