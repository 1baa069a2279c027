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


def _chain5():
    vers = [bytes([k, 0, 0, 9]) for k in range(5)]
    ep = [0, 2, 3, 4, 5]
    return (BH.Chain(bytes(range(32)), [(ep[k], vers[k]) for k in range(5)]),
            B.ChainConfig(bytes(range(32)), [(ep[k], vers[k], B.FORKS[k]) for k in range(5)]))


def test_fork_blocks_end_to_end(backend):
    """A bellatrix, a capella and a deneb block (execution payloads, BLS-to-execution changes
    whose own keys ride beside validator-index keys in one mixed package, blob commitments),
    plus a capella block with one corrupted BLS-change signature: per-block verdicts through
    the device path equal the C oracle's; the change keys are decompressed + validated on the GPU."""
    from oracle import bls12_381 as O
    from oracle import c_oracle as C
    from lodestar_amd.native import pack_blobs
    b, keys = backend
    chain, config = _chain5()
    committee, sync = BH.committee_of(NV), BH.sync_committee_of(NV)
    pk48 = lambda sk: O.g1_to_bytes(O.sk_to_pk(sk), compressed=True)  # noqa: E731
    blocks, parent = [], bytes(32)
    for n, slot in enumerate([3 * 32 + 5, 4 * 32 + 5, 5 * 32 + 5, 4 * 32 + 9]):
        corrupt = n == 3

        def sign(sks, roots, corrupt=corrupt):
            sig = W_sign(b.dev, sks, roots)
            if corrupt and len(sks) == 2 and len(sig) == 2:  # the block's two BLS changes
                sig[1] = sig[0]
            return sig
        ssz, expected, root, _ = BH.make_block(sign, keys.sks, chain, slot, (5 * n + 1) % NV, parent, committee,
                                               sync, n_atts=4, n_exits=1, n_prop_sl=1, n_att_sl=1, n_deposits=1,
                                               sync_participants=150, seed=n, pk48=pk48, n_changes=2)
        blocks.append(ssz)
        parent = root
    sets = B.BlockSignatureSetBuilder(b.dev, config, committee, sync).build(blocks)
    assert [len(x) for x in sets] == [12, 14, 14, 14]  # randao, 2 + 2 slashing sets, 4 atts, exit, proposer, sync (+ 2 changes)
    valid, errors = b.verify_requests(sets)
    assert valid == [True, True, True, False]
    flat = [s for blk in sets for s in blk]
    req_off = np.cumsum([0] + [len(x) for x in sets]).astype(np.uint32)
    kb = []
    for s in flat:
        ks = [s.pubkey] if s.pubkey is not None else s.pubkeys
        kb.append([keys.pks[k.index] if k.index is not None else k.uncompressed for k in ks])
    pk_off = np.cumsum([0] + [len(x) for x in kb]).astype(np.uint32)
    pks = np.frombuffer(b"".join(k for x in kb for k in x), np.uint8)
    blob, offs = pack_blobs([s.signature for s in flat])
    v, e = C.verify_requests(req_off, pks, pk_off, np.frombuffer(b"".join(s.signing_root for s in flat), np.uint8),
                             blob, offs, bytes(range(32)), threads=16)
    assert list(v) == [int(x) for x in valid] and list(e) == list(errors)


def test_bellatrix_reference_block_on_gpu(backend):
    """The reference's real bellatrix block: its signing roots on the GPU equal the CPU
    restatement's, and every signature in it (block, randao, attestations, sync aggregate)
    decodes and passes the G2 subgroup check on the GPU."""
    b, _ = backend
    ssz = open(os.path.join(GOLD, "goerli_shadow_fork_block_13249.ssz"), "rb").read()
    blk = B.parse_signed_block(ssz, "bellatrix")
    sizes = {}
    for a in blk.attestations:
        n = (len(a.aggregation_bits) - 1) * 8 + a.aggregation_bits[-1].bit_length() - 1
        sizes[(int.from_bytes(a.data[0:8], "little"), int.from_bytes(a.data[8:16], "little"))] = n
    cfg = B.ChainConfig(bytes(32), [(0, bytes(4), "phase0"), (0, bytes([1, 0, 0, 0]), "altair"),
                                    (0, bytes([2, 0, 0, 0]), "bellatrix")])
    comm = lambda s, i: list(range(sizes[(s, i)]))  # noqa: E731
    sync = lambda s: list(range(512))  # noqa: E731
    got = B.BlockSignatureSetBuilder(b.dev, cfg, comm, sync).build([ssz])[0]
    want = B.BlockSignatureSetBuilder(BH.OracleRoots(), cfg, comm, sync).build([ssz])[0]
    assert [s.signing_root for s in got] == [s.signing_root for s in want]
    sigs = [blk.signature, blk.randao_reveal, blk.sync_signature] + [a.signature for a in blk.attestations]
    status, _ = b.dev.decode_signatures(sigs)
    assert status == [0] * len(sigs)
