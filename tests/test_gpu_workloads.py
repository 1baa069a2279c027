"""Full-size configs on the GPU against the C oracle (BASELINE.json C4 / C5).

* C4: one GPU's full shard of the 1M-set gossip replay -- 125,000 sets
  (112,712 single attestations + 4,096 AggregateAndProof triples whose third
  set aggregates 488 keys, 2.1 M pubkeys by validator index), 977 requests of
  <= 128 sets, invalid sets injected -- verdicts and rejection codes request
  by request against the C oracle over the same sets (pubkeys as bytes).
* C5: a 32-block epoch of block import (147 sets per block, one request per
  block, 128 x 488-key attestations + a 512-key sync aggregate per block,
  invalid sets at 1e-3): per-block verdicts, per-set decode statuses and the
  merged check's fallback, against the C oracle.
Reference shapes: ST/signatureSets/index.ts:26-73, verifyBlocksSignatures.ts:38-55,
BN/chain/validation/aggregateAndProof.ts:200.
"""
import hashlib
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import workloads as W  # noqa: E402

pytestmark = pytest.mark.gpu
THREADS = 16  # the GPU box's CPU share


@pytest.fixture(scope="module")
def table_device():
    """A context whose device pubkey table holds 65,536 interop validators."""
    from lodestar_amd.native import Device
    dev = Device(0)
    keys = W.make_keys(dev, 65536)
    assert dev.pubkey_table_append(keys.pks) == 65536
    yield dev, keys
    dev.close()


def _oracle(p: W.Packed, keys: W.Keys, seed: bytes):
    from oracle import c_oracle as C
    blob, offs = p.blobs()
    return C.verify_requests(p.req_off, p.pk_bytes(keys), p.pk_off, p.msg_array(), blob, offs, seed, threads=THREADS)


def test_c4_full_shard_vs_c_oracle(table_device):
    dev, keys = table_device
    p = W.c4_shard(dev, keys, n_invalid=24)
    assert p.n_sets == 125000 and len(p.idx) == 112712 + 4096 * (2 + 488)
    seed = hashlib.sha256(b"c4").digest()
    blob, offs = p.blobs()
    res = dev.verify_requests(p.req_off, None, p.pk_off, p.msg_array(), blob, offs, seed, pk_indices=p.idx)
    valid, err = _oracle(p, keys, seed)
    assert list(res.errors) == list(err)
    assert list(res.valid) == list(valid)
    # exactly the requests holding an injected set are false (merged check -> per-request tails)
    assert {k for k, v in enumerate(res.valid) if not v} == p.expect_invalid_requests
    assert res.batch_retries == 1
    # the same shard through the byte path (worker wire format) and the async host API
    pc = dev.verify_requests_async(p.req_off, p.pk_bytes(keys), p.pk_off, p.msg_array(), blob, offs, seed)
    res2 = dev.wait_call(pc)
    assert list(res2.valid) == list(valid) and list(res2.errors) == list(err)


def test_c4_all_valid_shard_passes_merged(table_device):
    dev, keys = table_device
    p = W.c4_shard(dev, keys, singles=20000, aggregates=512, seed=3)
    blob, offs = p.blobs()
    res = dev.verify_requests(p.req_off, None, p.pk_off, p.msg_array(), blob, offs, bytes(32), pk_indices=p.idx)
    assert res.valid.all() and not res.errors.any()
    assert res.batch_retries == 0 and res.batch_sigs_success == p.n_sets


def test_c5_epoch_vs_c_oracle(table_device):
    from oracle import c_oracle as C
    dev, keys = table_device
    p = W.c5_epoch(dev, keys)
    assert p.n_req == 32 and p.n_sets == 32 * 147
    seed = hashlib.sha256(b"c5").digest()
    blob, offs = p.blobs()
    res = dev.verify_requests(p.req_off, None, p.pk_off, p.msg_array(), blob, offs, seed, pk_indices=p.idx)
    valid, err = _oracle(p, keys, seed)
    assert list(res.valid) == list(valid) and list(res.errors) == list(err)
    assert [bool(v) for v in res.valid] == [k not in p.expect_invalid_requests for k in range(32)]
    assert 0 < len(p.expect_invalid_requests) < 32
    # per-set status == the oracle's Signature.fromBytes(validate=true) status
    st, _ = C.decode_signatures(p.sigs)
    assert list(res.set_status) == st
    assert res.batch_retries == 1


def test_c5_block_verdicts_through_verifier(table_device):
    """verifyBlocksSignatures: one verifySignatureSets per block, no opts
    (verifyBlocksSignatures.ts:38-40), through BlsGpuVerifier with index keys."""
    import asyncio

    from lodestar_amd.verifier import BlsGpuVerifier, DeviceBackend, PublicKey, SignatureSet, SignatureSetType
    dev, keys = table_device
    p = W.c5_epoch(dev, keys, blocks=4, seed=19)
    backend = DeviceBackend(0, seed_source=lambda: bytes(32))
    assert backend.sync_pubkeys(keys.pks) == 65536

    def block_sets(k):
        out = []
        for i in range(int(p.req_off[k]), int(p.req_off[k + 1])):
            ix = [PublicKey(index=int(v)) for v in p.idx[p.pk_off[i]:p.pk_off[i + 1]]]
            out.append(SignatureSet(SignatureSetType.single, p.msgs[i], p.sigs[i], pubkey=ix[0]) if len(ix) == 1 else
                       SignatureSet(SignatureSetType.aggregate, p.msgs[i], p.sigs[i], pubkeys=ix))
        return out

    async def main():
        v = BlsGpuVerifier(backends=[backend])
        got = await asyncio.gather(*[v.verify_signature_sets(block_sets(k)) for k in range(p.n_req)])
        await v.close()
        return got
    got = asyncio.run(main())
    assert got == [k not in p.expect_invalid_requests for k in range(p.n_req)]
