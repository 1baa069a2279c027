"""BlsGpuVerifier scheduling semantics on CPU with a mock backend (the pattern
of the reference's test/mocks/mockedBls.ts): chunking, buffering, priority,
same-message flattening, rejection rules, close()."""
import asyncio

import pytest

from lodestar_amd.native import EmptyAggregateError
from lodestar_amd.verifier import (MAX_BUFFER_WAIT_MS, BlsGpuVerifier, PublicKey, QueueError, VerifySignatureOpts,
                                   aggregate_set, chunkify_maximize_chunk_size, single_set)

GOOD = b"\x01" * 96
BAD = b"\x02" * 96
PK = PublicKey(bytes(96))


class MockBackend:
    """valid iff every set carries GOOD; zero-pubkey aggregate -> error 1."""

    def __init__(self):
        self.dispatches = []
        self.same_message_calls = []

    def verify_requests(self, requests):
        self.dispatches.append([len(r) for r in requests])
        valid, errs = [], []
        for r in requests:
            empty = any(s.pubkeys is not None and len(s.pubkeys) == 0 for s in r)
            errs.append(1 if empty else 0)
            valid.append(bool(r) and all(s.signature == GOOD for s in r))
        return valid, errs

    def verify_same_message(self, pubkeys, signatures, message):
        self.same_message_calls.append(len(signatures))
        return [s == GOOD for s in signatures]


def sets(n, bad=()):
    return [single_set(PK, bytes([i % 256]) * 32, BAD if i in bad else GOOD) for i in range(n)]


def run(coro):
    return asyncio.run(coro)


def test_chunkify_matches_reference():
    assert [len(c) for c in chunkify_maximize_chunk_size(list(range(300)), 128)] == [150, 150]
    assert [len(c) for c in chunkify_maximize_chunk_size(list(range(100)), 128)] == [100]


def test_verify_all_valid_and_one_invalid():
    async def main():
        b = MockBackend()
        v = BlsGpuVerifier(backends=[b])
        assert await v.verify_signature_sets(sets(3)) is True
        assert await v.verify_signature_sets(sets(3, bad={1})) is False
        await v.close()
    run(main())


def test_large_call_is_chunked_into_jobs_of_le_128():
    async def main():
        b = MockBackend()
        v = BlsGpuVerifier(backends=[b])
        assert await v.verify_signature_sets(sets(300)) is True
        assert sorted(x for d in b.dispatches for x in d) == [150, 150]
        await v.close()
    run(main())


def test_batchable_calls_are_buffered_and_merged():
    async def main():
        b = MockBackend()
        v = BlsGpuVerifier(backends=[b])
        opts = VerifySignatureOpts(batchable=True)
        r = await asyncio.gather(v.verify_signature_sets(sets(3), opts), v.verify_signature_sets(sets(4), opts),
                                 v.verify_signature_sets(sets(2, bad={0}), opts))
        assert r == [True, True, False]
        assert b.dispatches == [[3, 4, 2]]  # one package, three verdicts
        await v.close()
    run(main())


def test_buffer_flushes_above_32_sigs_without_waiting():
    async def main():
        b = MockBackend()
        v = BlsGpuVerifier(backends=[b])
        loop = asyncio.get_running_loop()
        t0 = loop.time()
        assert await v.verify_signature_sets(sets(33), VerifySignatureOpts(batchable=True))
        assert loop.time() - t0 < MAX_BUFFER_WAIT_MS / 1000 / 2
        await v.close()
    run(main())


def test_batchable_waits_for_buffer_timeout():
    async def main():
        b = MockBackend()
        v = BlsGpuVerifier(backends=[b])
        loop = asyncio.get_running_loop()
        t0 = loop.time()
        assert await v.verify_signature_sets(sets(2), VerifySignatureOpts(batchable=True))
        assert loop.time() - t0 >= MAX_BUFFER_WAIT_MS / 1000 * 0.9
        await v.close()
    run(main())


def test_priority_jobs_run_first():
    async def main():
        b = MockBackend()
        v = BlsGpuVerifier(backends=[b], max_sets_per_dispatch=1)
        v._idle = []  # hold dispatch until both are queued
        f1 = asyncio.ensure_future(v.verify_signature_sets(sets(2)))
        f2 = asyncio.ensure_future(v.verify_signature_sets(sets(5), VerifySignatureOpts(priority=True)))
        await asyncio.sleep(0.01)
        v._idle = [0]
        v._run_job()
        await asyncio.gather(f1, f2)
        assert b.dispatches[0] == [5]
        await v.close()
    run(main())


def test_empty_aggregate_rejects_the_job():
    async def main():
        b = MockBackend()
        v = BlsGpuVerifier(backends=[b])
        with pytest.raises(EmptyAggregateError):
            await v.verify_signature_sets([aggregate_set([], bytes(32), GOOD)])
        await v.close()
    run(main())


def test_empty_sets_are_false_like_reference():
    """chunkify([]) -> [[]] -> one job of 0 sets -> maybeBatch throws "Empty
    signature set" -> caught -> false (index.ts:191-213, maybeBatch.ts:31-33)."""
    async def main():
        v = BlsGpuVerifier(backends=[MockBackend()])
        assert await v.verify_signature_sets([]) is False
        await v.close()
    run(main())


def test_same_message_flattens_chunks():
    async def main():
        b = MockBackend()
        v = BlsGpuVerifier(backends=[b])
        pairs = [(PK, GOOD)] * 299 + [(PK, BAD)]
        out = await v.verify_signature_sets_same_message(pairs, bytes(32))
        assert out == [True] * 299 + [False]
        assert sorted(b.same_message_calls) == [150, 150]  # chunkify(300, 128)
        assert await v.verify_signature_sets_same_message([], bytes(32)) == []
        await v.close()
    run(main())


def test_verify_on_main_thread_is_synchronous():
    async def main():
        b = MockBackend()
        v = BlsGpuVerifier(backends=[b])
        assert await v.verify_signature_sets(sets(2), VerifySignatureOpts(verify_on_main_thread=True))
        assert b.dispatches == [[2]]
        await v.close()
    run(main())


def test_close_rejects_queued_jobs_and_new_work():
    async def main():
        v = BlsGpuVerifier(backends=[MockBackend()])
        fut = asyncio.ensure_future(v.verify_signature_sets(sets(2), VerifySignatureOpts(batchable=True)))
        await asyncio.sleep(0)
        await v.close()
        with pytest.raises(QueueError):
            await fut
        with pytest.raises(QueueError):
            await v.verify_signature_sets(sets(1))
    run(main())


def test_can_accept_work():
    async def main():
        v = BlsGpuVerifier(backends=[MockBackend()])
        assert v.can_accept_work()
        v._idle = []
        assert not v.can_accept_work()
        v._idle = [0]
        await v.close()
    run(main())


def test_multiple_backends_share_load():
    async def main():
        bs = [MockBackend(), MockBackend()]
        v = BlsGpuVerifier(backends=bs, max_sets_per_dispatch=128)
        r = await asyncio.gather(*[v.verify_signature_sets(sets(128)) for _ in range(6)])
        assert all(r)
        assert all(len(b.dispatches) > 0 for b in bs)
        await v.close()
    run(main())


# ---- index-addressed keys (device pubkey table) ------------------
def test_public_key_index_or_bytes():
    from lodestar_amd.verifier import PublicKey
    assert PublicKey(index=3).index == 3
    with pytest.raises(ValueError):
        PublicKey()
    with pytest.raises(ValueError):
        PublicKey(b"\0" * 95, index=1)


class FakeDev:
    """Stand-in for native.Device (no GPU): records the arrays a call ships."""

    def __init__(self, slow=0.0):
        self.calls = []
        self.slow = slow
        self.closed = False
        self.active = 0

    def verify_requests_async(self, req_off, pks, pk_off, msgs, blob, offs, seed, pk_indices=None, partial=False):
        import numpy as np
        from lodestar_amd.native import PendingCall
        assert not self.closed, "call on a destroyed context"
        self.calls.append((pks, None if pk_indices is None else list(pk_indices), list(pk_off)))
        n = len(req_off) - 1
        self.active += 1
        return PendingCall(len(self.calls), n, 0, np.ones(max(n, 1), np.uint8), np.zeros(max(n, 1), np.uint8),
                           np.zeros(1, np.uint8), None, partial)

    def wait_call(self, pc):
        import time as _t

        import numpy as np
        from lodestar_amd.native import VerifyResult
        assert not self.closed, "wait on a destroyed context"
        _t.sleep(self.slow)
        self.active -= 1
        return VerifyResult(pc.valid[:pc.n_req], pc.err[:pc.n_req], np.zeros(0, np.uint8), 0.0)

    def verify_same_message_batch_async(self, jobs, seed, by_index=False):
        import numpy as np
        from lodestar_amd.native import PendingSameMessage
        assert not self.closed, "call on a destroyed context"
        self.active += 1
        return PendingSameMessage(0, len(jobs), None, None, np.zeros(1, np.uint32), list(jobs))

    def wait_same_message(self, pc):
        assert not self.closed, "wait on a destroyed context"
        self.active -= 1
        jobs = pc.keep
        return ([[True] * len(s) for _, s, _ in jobs], [True] * len(jobs), (0, sum(len(s) for _, s, _ in jobs)),
                0.0)

    def last_stage_times(self):
        return [("pubkeys_agg", 0.5)]

    def pubkey_table_size(self):
        return 10

    def pubkey_table_read(self, first, n):
        return [bytes([first]) * 96]

    def close(self):
        assert self.active == 0, "context destroyed with a call in flight"
        self.closed = True


def test_device_backend_ships_indices_when_every_key_has_one():
    from lodestar_amd.verifier import DeviceBackend, PublicKey, aggregate_set, single_set

    b = DeviceBackend(seed_source=lambda: bytes(32), dev=FakeDev())
    s1 = single_set(PublicKey(index=4), bytes(32), bytes(96))
    s2 = aggregate_set([PublicKey(index=1), PublicKey(index=2)], bytes(32), bytes(96))
    assert b.verify_requests([[s1, s2]]) == ([True], [0])
    pks, idx, pk_off = b.dev.calls[-1]
    assert pks is None and idx == [4, 1, 2] and pk_off == [0, 1, 3]
    # mixed (a capella block's BLS-change key beside validator keys): indices for the table
    # keys, flagged row indices (LB_PK_ROW_FLAG) for the keys shipped as bytes
    s3 = single_set(PublicKey(bytes([7]) * 96), bytes(32), bytes(96))
    b.verify_requests([[s1, s3, s2]])
    pks, idx, _ = b.dev.calls[-1]
    assert idx == [4, 0x80000000, 1, 2] and pks.tobytes() == bytes([7]) * 96
    # no index at all: the encodings
    b.verify_requests([[s3]])
    pks, idx, _ = b.dev.calls[-1]
    assert idx is None and pks.tobytes() == bytes([7]) * 96
    b.close()


def test_signing_root_length_is_checked():
    from lodestar_amd.verifier import DeviceBackend, PublicKey, single_set

    b = DeviceBackend(seed_source=lambda: bytes(32), dev=FakeDev())
    with pytest.raises(ValueError):
        b.verify_requests([[single_set(PublicKey(index=1), bytes(31), bytes(96))]])
    b.close()

    async def main():
        v = BlsGpuVerifier(backends=[MockBackend()])
        with pytest.raises(ValueError):
            await v.verify_signature_sets([single_set(PK, bytes(33), GOOD)])
        await v.close()
    run(main())


def test_close_waits_for_calls_in_flight():
    """close() must never destroy the context under a running call
    (index.ts:244-265 awaits the workers)."""
    from lodestar_amd.verifier import DeviceBackend

    async def main():
        dev = FakeDev(slow=0.2)
        v = BlsGpuVerifier(backends=[DeviceBackend(seed_source=lambda: bytes(32), dev=dev)])
        futs = [asyncio.ensure_future(v.verify_signature_sets(sets(3))) for _ in range(6)]
        await asyncio.sleep(0.05)  # dispatched, the fake device still busy
        await v.close()
        assert dev.closed and dev.active == 0
        done = [f.result() if not f.exception() else f.exception() for f in futs]
        assert all(d is True or isinstance(d, QueueError) for d in done)
    run(main())


def test_device_backend_keeps_several_calls_in_flight():
    from lodestar_amd.verifier import DeviceBackend

    dev = FakeDev(slow=0.05)
    b = DeviceBackend(seed_source=lambda: bytes(32), dev=dev, capacity=4)
    futs = [b.submit_requests([sets(2)]) for _ in range(8)]
    assert [f.result()[0] for f in futs] == [[True]] * 8
    b.close()


def test_worker_batch_stats_match_reference_chunking():
    """worker.ts:41-85: batchable requests in chunks of >= 16, one retry per failed chunk."""
    from lodestar_amd.verifier import worker_batch_stats
    assert worker_batch_stats([3] * 10, [True] * 10, [True] * 10) == (0, 30)
    assert worker_batch_stats([3] * 10, [True] * 10, [True] * 9 + [False]) == (1, 0)
    # 40 batchable requests -> chunkify(40, 16) = 2 chunks of 20; one bad request fails one chunk
    v = [True] * 40
    v[25] = False
    assert worker_batch_stats([2] * 40, [True] * 40, v) == (1, 40)
    # non-batchable requests never count
    assert worker_batch_stats([5, 5], [False, False], [False, True]) == (0, 0)


# ---- metrics parity (lodestar.ts:380-495 names, index.ts update sites) -------------
def test_pool_metrics_reference_names():
    from lodestar_amd import metrics as M

    async def main():
        b = MockBackend()
        v = BlsGpuVerifier(backends=[b])
        assert await v.verify_signature_sets(sets(300), VerifySignatureOpts(batchable=True, priority=True)) is True
        with pytest.raises(EmptyAggregateError):
            await v.verify_signature_sets([aggregate_set([], bytes(32), GOOD)])
        out = await v.verify_signature_sets_same_message([(PK, GOOD), (PK, BAD)], bytes(32))
        assert out == [True, False]
        pm = v.pool_metrics
        assert pm.get(M.TOTAL_SIG_SETS) == 301
        assert pm.get(M.BATCHABLE_SIG_SETS) == 300 and pm.get(M.PRIORITIZED_SIG_SETS) == 300
        assert pm.get(M.SIG_SETS_STARTED, type="default") == 301
        assert pm.get(M.SIG_SETS_STARTED, type="same_message") == 2
        assert pm.get(M.JOBS_STARTED, type="default") == 3
        assert pm.get(M.ERROR_AGGREGATE_SETS, type="default") == 1
        assert pm.get(M.ERROR_JOBS_SETS) == 1 and pm.get(M.SUCCESS_JOBS_SETS) == 301
        assert pm.get(M.SAME_MESSAGE_RETRY_JOBS) == 1 and pm.get(M.SAME_MESSAGE_RETRY_SETS) == 2
        assert pm.get(M.BATCH_RETRIES) == 0 and pm.get(M.BATCH_SIGS_SUCCESS) == 300  # one passing chunk
        assert pm.histogram(M.JOB_WAIT_TIME)[0] == 4
        names = set(pm.collect())
        assert "lodestar_bls_thread_pool_sig_sets_total" in names
        assert 'lodestar_bls_thread_pool_jobs_started_total{type="default"}' in names
        await v.close()
    run(main())


class SlotDev(FakeDev):
    """FakeDev with the library's slot accounting: a two-phase call holds its slot from
    submission until verify_finish; more than `slots` calls holding slots at once would
    make the library reuse (and silently resume) a pending partial."""

    def __init__(self, slots=2, slow=0.02):
        super().__init__(slow=slow)
        self.slots, self.pending, self.max_used = slots, 0, 0

    def verify_requests_async(self, *a, partial=False, **k):
        assert self.active + self.pending < self.slots, "a slot holding a pending partial was reused"
        pc = super().verify_requests_async(*a, partial=partial, **k)
        if partial:
            self.active -= 1
            self.pending += 1
        self.max_used = max(self.max_used, self.active + self.pending)
        return pc

    def partial_wait(self, pc):
        return bytes(576)

    def verify_finish(self, pc, ok):
        self.pending -= 1
        self.active += 1

    def verify_same_message_batch_async(self, jobs, seed, by_index=False):
        assert self.active + self.pending < self.slots, "a slot holding a pending partial was reused"
        pc = super().verify_same_message_batch_async(jobs, seed, by_index)
        self.max_used = max(self.max_used, self.active + self.pending)
        return pc


def test_partial_call_holds_its_slot_until_finished():
    """pending two-phase calls count against the backend's capacity, so
    neither a later package nor an interleaved same-message call resumes them early."""
    from lodestar_amd.verifier import DeviceBackend, PublicKey, single_set

    dev = SlotDev(slots=2)
    b = DeviceBackend(seed_source=lambda: bytes(32), dev=dev, capacity=2)
    req = [[single_set(PublicKey(index=1), bytes(32), bytes(96))]]
    pc = b.submit_requests(req, partial=True).result()
    later = [b.submit_requests(req) for _ in range(3)]
    sm = b.submit_same_message([([PublicKey(index=2)], [bytes(96)], bytes(32))])
    assert sm.result()[0] == [[True]]
    for f in later:
        assert f.result()[0] == [True]
    assert dev.pending == 1  # still waiting for its host verdict
    assert b.finish(pc, True).result()[0] == [True]
    assert dev.max_used <= 2 and dev.pending == 0
    b.close()
