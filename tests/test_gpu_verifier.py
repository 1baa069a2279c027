"""The reference's verifier tests, replayed through BlsGpuVerifier on the GPU.

* test/unit/chain/bls/bls.test.ts:10-88 (keys SecretKey.fromKeygen(Buffer.alloc(32, i)))
* test/e2e/chain/bls/multithread.test.ts:9-130 (keys SecretKey.fromBytes(Buffer.alloc(32, i+1)),
  8 concurrent calls, sync/async/batchable x priority, an invalid zero signature must not poison
  valid sets)
"""
import asyncio

import pytest

from lodestar_amd.verifier import BlsGpuVerifier, DeviceBackend, PublicKey, VerifySignatureOpts, single_set
from oracle import bls12_381 as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def backend():
    b = DeviceBackend(0, seed_source=lambda: bytes(32))
    yield b
    b.close()


def keyset_keygen(n):
    sks = [O.keygen(bytes([i]) * 32) for i in range(n)]
    return sks, [PublicKey(O.g1_to_bytes(O.sk_to_pk(sk), compressed=False)) for sk in sks]


def run(coro):
    return asyncio.run(coro)


def test_bls_test_ts_verify_signature_sets(backend):
    sks, pks = keyset_keygen(3)

    def make():
        return [single_set(pks[i], bytes([i]) * 32, O.g2_to_bytes(O.sign(sks[i], bytes([i]) * 32)))
                for i in range(3)]

    async def main():
        v = BlsGpuVerifier(backends=[backend])
        assert await v.verify_signature_sets(make()) is True
        s = make()
        s[1].signing_root = bytes([10]) * 32  # wrong signing root
        assert await v.verify_signature_sets(s) is False
        s = make()
        s[1].signature = bytes([10]) * 96  # malformed
        assert await v.verify_signature_sets(s) is False
    run(main())


def test_bls_test_ts_same_message(backend):
    sks, pks = keyset_keygen(3)
    root = bytes([100]) * 32

    async def main():
        v = BlsGpuVerifier(backends=[backend])
        sigs = [O.g2_to_bytes(O.sign(sk, root)) for sk in sks]
        assert await v.verify_signature_sets_same_message(list(zip(pks, sigs)), root) == [True, True, True]
        bad = list(sigs)
        bad[1] = O.g2_to_bytes(O.sign(sks[1], bytes(32)))
        assert await v.verify_signature_sets_same_message(list(zip(pks, bad)), root) == [True, False, True]
        bad[1] = bytes([10]) * 96
        assert await v.verify_signature_sets_same_message(list(zip(pks, bad)), root) == [True, False, True]
    run(main())


def test_multithread_test_ts_concurrency_and_invalid_does_not_poison(backend):
    sks = [int.from_bytes(bytes([i + 1]) * 32, "big") % O.R for i in range(3)]
    pks = [PublicKey(O.g1_to_bytes(O.sk_to_pk(sk), compressed=False)) for sk in sks]
    msgs = [bytes([i + 1]) * 32 for i in range(3)]
    sigs = [O.g2_to_bytes(O.sign(sk, m)) for sk, m in zip(sks, msgs)]
    sets = [single_set(pks[i], msgs[i], sigs[i]) for i in range(3)]

    async def main():
        v = BlsGpuVerifier(backends=[backend])
        calls = []
        for batchable in (False, True):
            for priority in (False, True):
                opts = VerifySignatureOpts(batchable=batchable, priority=priority)
                calls += [v.verify_signature_sets(sets, opts) for _ in range(2)]
        assert await asyncio.gather(*calls) == [True] * 8
        invalid = single_set(pks[0], msgs[0], bytes(32))
        r = await asyncio.gather(v.verify_signature_sets([invalid], VerifySignatureOpts(batchable=True)),
                                 *[v.verify_signature_sets([s], VerifySignatureOpts(batchable=True)) for s in sets])
        assert r == [False, True, True, True]
    run(main())
