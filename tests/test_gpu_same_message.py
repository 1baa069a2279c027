"""Batched same-message jobs on the GPU (lb_verify_same_message_batch) and the
single-thread verifier.

The reference turns every same-message job into ONE aggregated set inside a
worker package (jobItemWorkReq sameMessage, jobItem.ts:64-86; index.ts:455-489)
and retries a failed job set by set (jobItemSameMessageToMultiSet,
jobItem.ts:93-125).  Here all jobs of a package go to the device in one call.
Expected verdicts are known by construction (every set is signed by its own
key unless corrupted) and sampled against the C oracle.
"""
import asyncio
import hashlib
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import workloads as W  # noqa: E402
from lodestar_amd.verifier import (BlsGpuSingleThreadVerifier, BlsGpuVerifier, DeviceBackend,  # noqa: E402
                                   PublicKey, VerifySignatureOpts, single_set)
from oracle import bls12_381 as O  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def keyed():
    from lodestar_amd.native import Device
    dev = Device(0)
    keys = W.make_keys(dev, 16384)
    assert dev.pubkey_table_append(keys.pks) == len(keys.pks)
    yield dev, keys
    dev.close()


def test_same_message_batch_full_package(keyed):
    """512 jobs x 128 sets (65,536 sets, one device call), 40 corrupted sets."""
    dev, keys = keyed
    jobs, expect = W.same_message_jobs(dev, keys, n_jobs=512, per_job=128, n_invalid=40)
    res, fast, (retried, ok_sets) = dev.verify_same_message_batch(jobs, bytes(32), by_index=True)
    assert res == expect
    bad_jobs = {j for j, e in enumerate(expect) if not all(e)}
    assert [not f for f in fast] == [j in bad_jobs for j in range(512)]
    assert retried == len(bad_jobs) and ok_sets == 128 * (512 - len(bad_jobs))
    # the byte path (96-byte pubkeys) gives the same verdicts
    jb = [([keys.pks[i] for i in ix], s, m) for ix, s, m in jobs[:64]]
    res_b, _, _ = dev.verify_same_message_batch(jb, bytes(32))
    assert res_b == expect[:64]


def test_same_message_batch_vs_c_oracle_sample(keyed):
    """Each set of a few corrupted jobs re-verified alone by the C oracle."""
    from lodestar_amd.native import pack_blobs
    from oracle import c_oracle as C
    dev, keys = keyed
    jobs, expect = W.same_message_jobs(dev, keys, n_jobs=24, per_job=32, seed=5, n_invalid=9)
    res, _, _ = dev.verify_same_message_batch(jobs, bytes(32), by_index=True)
    flat = [(keys.pks[i], s, m) for ix, sigs, m in jobs for i, s in zip(ix, sigs)]
    blob, offs = pack_blobs([s for _, s, _ in flat])
    n = len(flat)
    valid, err = C.verify_requests(np.arange(n + 1, dtype=np.uint32), np.frombuffer(b"".join(p for p, _, _ in flat),
                                                                                   np.uint8),
                                   None, np.frombuffer(b"".join(m for _, _, m in flat), np.uint8), blob, offs,
                                   bytes(32), threads=16)
    assert [v for r in res for v in r] == [bool(x) for x in valid] == [v for e in expect for v in e]


def test_same_message_edge_jobs(keyed):
    """Empty job in the middle, 1-set jobs, a job whose only set is malformed, and
    a cancelling pair (plain sums accept it, as the reference's aggregate does)."""
    dev, keys = keyed
    root = hashlib.sha256(b"edge").digest()
    s = W.sign_many(dev, keys.sks[:4], [root] * 4)
    # cancelling pair: sig0 + D and sig1 - D: both individually invalid, their sum valid
    d = O.g2_mul(O.G2, 99991)
    s0 = O.g2_to_bytes(O.E2.add(O.signature_from_bytes(s[0]), d))
    s1 = O.g2_to_bytes(O.E2.add(O.signature_from_bytes(s[1]), O.E2.neg(d)))
    jobs = [([0, 1], [s[0], s[1]], root), ([], [], root), ([2], [s[2]], root), ([3], [bytes([10]) * 96], root),
            ([0, 1], [s0, s1], root)]
    res, fast, _ = dev.verify_same_message_batch(jobs, bytes(32), by_index=True)
    assert res == [[True, True], [], [True], [False], [True, True]]
    assert fast == [True, False, True, False, True]


def test_reference_same_message_table_single_thread(keyed):
    """bls.test.ts:69-85 through BlsGpuSingleThreadVerifier (singleThread.ts:37-81)."""
    sks = [O.keygen(bytes([i]) * 32) for i in range(3)]
    pks = [PublicKey(O.g1_to_bytes(O.sk_to_pk(sk), compressed=False)) for sk in sks]
    root = bytes([100]) * 32
    sigs = [O.g2_to_bytes(O.sign(sk, root)) for sk in sks]

    async def main():
        v = BlsGpuSingleThreadVerifier(DeviceBackend(0, seed_source=lambda: bytes(32)))
        assert await v.verify_signature_sets_same_message(list(zip(pks, sigs)), root) == [True, True, True]
        bad = list(sigs)
        bad[1] = O.g2_to_bytes(O.sign(sks[1], bytes([101]) * 32))
        assert await v.verify_signature_sets_same_message(list(zip(pks, bad)), root) == [True, False, True]
        bad[1] = bytes([10]) * 96
        assert await v.verify_signature_sets_same_message(list(zip(pks, bad)), root) == [True, False, True]
        # verifySignatureSets (bls.test.ts:36-52)
        mk = [single_set(pks[i], bytes([i]) * 32, O.g2_to_bytes(O.sign(sks[i], bytes([i]) * 32))) for i in range(3)]
        assert await v.verify_signature_sets(mk) is True
        mk[1].signing_root = bytes([10]) * 32
        assert await v.verify_signature_sets(mk) is False
        mk[1].signing_root = bytes([1]) * 32
        mk[2].signature = bytes([10]) * 96
        assert await v.verify_signature_sets(mk) is False
        assert v.can_accept_work()
        await v.close()
    asyncio.run(main())


def test_verify_on_main_thread_path(keyed):
    """index.ts:174-187: verifyOnMainThread verifies synchronously (gossip block
    proposer signature, BN/chain/validation/block.ts:146)."""
    sks = [O.keygen(bytes([i + 7]) * 32) for i in range(2)]
    pks = [PublicKey(O.g1_to_bytes(O.sk_to_pk(sk), compressed=False)) for sk in sks]

    async def main():
        b = DeviceBackend(0, seed_source=lambda: bytes(32))
        v = BlsGpuVerifier(backends=[b])
        opts = VerifySignatureOpts(verify_on_main_thread=True)
        good = [single_set(pks[i], bytes([i]) * 32, O.g2_to_bytes(O.sign(sks[i], bytes([i]) * 32))) for i in range(2)]
        assert await v.verify_signature_sets(good, opts) is True
        assert await v.verify_signature_sets(good[:1], opts) is True
        good[0].signing_root = bytes([9]) * 32
        assert await v.verify_signature_sets(good, opts) is False
        assert v.pool_metrics.histogram("lodestar_bls_thread_pool_main_thread_time_seconds")[0] == 3
        assert v.metrics["dispatches"] == 0  # never went through the queue
        await v.close()
    asyncio.run(main())


def test_pool_same_message_jobs_share_one_device_call(keyed):
    """Several same-message jobs buffered into one package -> one batched device call."""
    dev, keys = keyed
    jobs, expect = W.same_message_jobs(dev, keys, n_jobs=6, per_job=20, seed=9, n_invalid=2)

    async def main():
        b = DeviceBackend(0, seed_source=lambda: bytes(32))
        b.sync_pubkeys(keys.pks)
        calls = []
        orig = b.submit_same_message
        b.submit_same_message = lambda js, priority=False: (calls.append(len(js)), orig(js, priority))[1]
        v = BlsGpuVerifier(backends=[b])
        opts = VerifySignatureOpts(batchable=True)
        outs = await asyncio.gather(*[
            v.verify_signature_sets_same_message([(PublicKey(index=i), s) for i, s in zip(ix, sigs)], m, opts)
            for ix, sigs, m in jobs])
        await v.close()
        return outs, calls
    outs, calls = asyncio.run(main())
    assert outs == expect
    assert calls == [6]


def test_same_message_async_packages_in_flight(keyed):
    """lb_verify_same_message_batch_async: four packages (two with corrupted sets, whose
    failed jobs are re-verified set by set when the package retires, on its own slot)
    in flight beside a default-request call, retired out of order; verdicts, fast-path
    flags and retry counts as by construction, and one package's sets re-verified alone
    by the C oracle."""
    from lodestar_amd.native import pack_blobs
    from oracle import c_oracle as C
    dev, keys = keyed
    pkgs = [W.same_message_jobs(dev, keys, n_jobs=64, per_job=32, seed=20 + k, n_invalid=(0, 7, 0, 3)[k])
            for k in range(4)]
    pend = [dev.verify_same_message_batch_async(jobs, bytes([k]) * 32, by_index=True)
            for k, (jobs, _) in enumerate(pkgs)]
    # a default-request call in flight between them
    jobs0 = pkgs[0][0]
    flat = [(keys.pks[i], s, m) for ix, sigs, m in jobs0[:8] for i, s in zip(ix, sigs)]
    blob, offs = pack_blobs([s for _, s, _ in flat])
    n = len(flat)
    pc = dev.verify_requests_async(np.arange(0, n + 1, 32, dtype=np.uint32),
                                   np.frombuffer(b"".join(p for p, _, _ in flat), np.uint8), None,
                                   np.frombuffer(b"".join(m for _, _, m in flat), np.uint8), blob, offs, bytes(32))
    for k in (2, 0, 3, 1):
        res, fast, (retried, ok_sets), _ = dev.wait_same_message(pend[k])
        jobs, expect = pkgs[k]
        assert res == expect, k
        bad = {j for j, e in enumerate(expect) if not all(e)}
        assert [not f for f in fast] == [j in bad for j in range(len(jobs))]
        assert retried == len(bad) and ok_sets == sum(len(e) for j, e in enumerate(expect) if j not in bad)
    assert list(dev.wait_call(pc).valid) == [1] * 8
    # package 1 (7 corrupted sets) set by set against the C oracle
    jobs, expect = pkgs[1]
    flat = [(keys.pks[i], s, m) for ix, sigs, m in jobs for i, s in zip(ix, sigs)]
    blob, offs = pack_blobs([s for _, s, _ in flat])
    n = len(flat)
    valid, _ = C.verify_requests(np.arange(n + 1, dtype=np.uint32), np.frombuffer(b"".join(p for p, _, _ in flat),
                                                                                 np.uint8),
                                 None, np.frombuffer(b"".join(m for _, _, m in flat), np.uint8), blob, offs,
                                 bytes(32), threads=16)
    assert [bool(x) for x in valid] == [v for e in expect for v in e]


def test_same_message_async_edge_jobs_bytes(keyed):
    """The edge jobs of test_same_message_edge_jobs through the async entry with 96-byte
    pubkeys (phase-2 keys are rows of the package's own key bytes), plus an
    infinite signature in a 1-set job (core verify rejects it in phase 2)."""
    dev, keys = keyed
    root = hashlib.sha256(b"edge-async").digest()
    s = W.sign_many(dev, keys.sks[:4], [root] * 4)
    d = O.g2_mul(O.G2, 7919)
    s0 = O.g2_to_bytes(O.E2.add(O.signature_from_bytes(s[0]), d))
    s1 = O.g2_to_bytes(O.E2.add(O.signature_from_bytes(s[1]), O.E2.neg(d)))
    inf = bytes([0xC0]) + bytes(95)
    pk = keys.pks
    jobs = [([pk[0], pk[1]], [s[0], s[1]], root), ([], [], root), ([pk[2]], [s[2]], root),
            ([pk[3]], [bytes([10]) * 96], root), ([pk[0], pk[1]], [s0, s1], root), ([pk[2]], [inf], root),
            ([pk[3], pk[2]], [s[3], s0], root)]
    p = dev.verify_same_message_batch_async(jobs, bytes(32))
    res, fast, (retried, ok_sets), _ = dev.wait_same_message(p)
    assert res == [[True, True], [], [True], [False], [True, True], [False], [True, False]]
    assert fast == [True, False, True, False, True, False, False]
    assert retried == 3 and ok_sets == 5
