"""Multi-GPU sharding logic on CPU: shard boundaries, in-process fan-out, and a
world_size-2 torch.distributed (gloo) run whose verdicts equal the unsharded ones."""
import os
import random

import pytest
import torch.multiprocessing as mp

from lodestar_amd.sharding import ShardedVerifier, shard_requests, verify_distributed


class TableBackend:
    """Deterministic stand-in for a GPU: a request is valid iff none of its
    sets is marked bad (the verdict rule verify_requests implements)."""

    def __init__(self):
        self.seen = []

    def verify_requests(self, requests):
        self.seen.append([r[0]["id"] if r else None for r in requests])
        return [bool(r) and all(not s["bad"] for s in r) for r in requests], \
               [1 if any(s.get("empty_agg") for s in r) else 0 for r in requests]


class TwoPhaseBackend(TableBackend):
    """TableBackend with the two-phase protocol of DeviceBackend: the 576-byte
    "partial" of a shard is 1 iff none of its requests holds a bad set (the
    multiplicative combine in miniature), gt_check = AND of the partials."""

    def __init__(self):
        super().__init__()
        self.finished = []

    def submit_requests(self, requests, partial=False, priority=False):
        import concurrent.futures
        from types import SimpleNamespace
        f = concurrent.futures.Future()
        v, e = self.verify_requests(requests)
        if partial:
            ok = all(not s["bad"] for r in requests for s in r)
            f.set_result(SimpleNamespace(backend=self, partial=bytes([ok]) + bytes(575), verdicts=(v, e)))
        else:
            f.set_result((v, e, None))
        return f

    def gt_check(self, partials):
        import concurrent.futures
        self.gt_checks = getattr(self, "gt_checks", 0) + 1
        f = concurrent.futures.Future()
        f.set_result(all(p[0] == 1 for p in partials))
        return f

    def finish(self, call, ok):
        import concurrent.futures
        self.finished.append(ok)
        f = concurrent.futures.Future()
        f.set_result((*call.verdicts, None))
        return f


def make_requests(seed=0, n=37):
    rnd = random.Random(seed)
    reqs, k = [], 0
    for _ in range(n):
        size = rnd.choice([0, 1, 2, 5, 128, 3])
        reqs.append([{"id": k + j, "bad": rnd.random() < 0.05, "empty_agg": rnd.random() < 0.01}
                     for j in range(size)])
        k += size
    return reqs


@pytest.mark.parametrize("shards", [1, 2, 3, 4, 8])
def test_shards_cover_every_request_once(shards):
    sizes = [len(r) for r in make_requests(1)]
    sh = shard_requests(sizes, shards)
    assert len(sh) == shards
    assert sh[0][0] == 0 and sh[-1][1] == len(sizes)
    for (a, b), (c, d) in zip(sh, sh[1:]):
        assert b == c and a <= b
    total = sum(sizes)
    for a, b in sh:  # balance: no shard above its fair share by more than one request
        assert sum(sizes[a:b]) <= total / shards + max(sizes)


def test_shard_more_shards_than_requests():
    sh = shard_requests([3, 4], 8)
    assert sum(b - a for a, b in sh) == 2


def test_sharded_verifier_equals_single():
    reqs = make_requests(2)
    single = TableBackend().verify_requests(reqs)
    backs = [TableBackend() for _ in range(4)]
    assert ShardedVerifier(backs).verify_requests(reqs) == single
    assert sum(len(b.seen) for b in backs) >= 1


@pytest.mark.parametrize("bad", [False, True])
def test_sharded_verifier_combines_partials(bad):
    reqs = make_requests(4)
    for r in reqs:
        for st in r:
            st["bad"] = False
            st["empty_agg"] = False
    if bad:
        next(r for r in reqs if r)[0]["bad"] = True
    want = TableBackend().verify_requests(reqs)
    backs = [TwoPhaseBackend() for _ in range(3)]
    sv = ShardedVerifier(backs)
    assert sv.combine
    assert sv.verify_requests(reqs) == want
    assert sv.last_combine["merged_ok"] is (not bad) and sv.last_combine["n_partials"] == 3
    assert all(b.finished == [not bad] for b in backs)


class FailingBackend(TwoPhaseBackend):
    """Phase 1 raises (a device error on this GPU)."""

    def submit_requests(self, requests, partial=False, priority=False):
        import concurrent.futures
        f = concurrent.futures.Future()
        f.set_exception(RuntimeError("device lost"))
        return f


def test_sharded_verifier_resumes_the_other_shards_when_one_fails():
    """a failing shard must not leave the others' partials pending."""
    reqs = make_requests(5)
    backs = [TwoPhaseBackend(), FailingBackend(), TwoPhaseBackend()]
    with pytest.raises(RuntimeError, match="device lost"):
        ShardedVerifier(backs).verify_requests(reqs)
    assert backs[0].finished == [False] and backs[2].finished == [False]


def _worker(rank, world, port, reqs, out_q, two_phase=False, fail_rank=-1):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b = (FailingBackend() if rank == fail_rank else TwoPhaseBackend()) if two_phase else TableBackend()
    try:
        v, e = verify_distributed(reqs, b.verify_requests, rank, world, backend=b if two_phase else None)
        out_q.put((rank, v, e, b.seen, getattr(b, "gt_checks", None)))
    except Exception as ex:  # noqa: BLE001
        out_q.put((rank, "error", str(ex), None, None))
    dist.barrier()
    dist.destroy_process_group()


def test_verify_distributed_fails_on_every_rank_together():
    """A rank whose shard raises joins the collectives with an error flag: every rank
    raises instead of the others blocking in all_gather."""
    reqs = make_requests(6)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 31500 + random.Random(os.getpid()).randrange(2000)
    procs = [ctx.Process(target=_worker, args=(r, 2, port, reqs, q, True, 1)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[1] for r in res] == ["error", "error"]
    assert "device lost" in res[1][2] and "rank(s) [1]" in res[0][2]


@pytest.mark.parametrize("two_phase", [False, True])
def test_verify_distributed_gloo_world2(two_phase):
    reqs = make_requests(3)
    want = TableBackend().verify_requests(reqs)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + random.Random(os.getpid()).randrange(2000)
    procs = [ctx.Process(target=_worker, args=(r, 2, port + (7 if two_phase else 0), reqs, q, two_phase))
             for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    shards = shard_requests([len(r) for r in reqs], 2)
    for rank, v, e, seen, checks in res:
        assert (v, e) == want
        if two_phase:  # the combined check runs once, on rank 0
            assert checks == (1 if rank == 0 else None)
        lo, hi = shards[rank]
        assert len(seen[0]) == hi - lo  # each rank verified only its own shard


def test_packed_requests_slice_rebases_offsets():
    """PackedRequests.slice(lo, hi): requests [lo, hi) as a call of their own."""
    import numpy as np
    from lodestar_amd.sharding import PackedRequests, shard_requests
    rng = np.random.default_rng(1)
    sizes = rng.integers(1, 6, 40)
    req_off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint32)
    n = int(req_off[-1])
    keys_per_set = rng.integers(1, 4, n)
    pk_off = np.concatenate([[0], np.cumsum(keys_per_set)]).astype(np.uint32)
    idx = np.arange(int(pk_off[-1]), dtype=np.uint32) * 7
    sig_len = rng.choice([96, 192], n)
    sig_off = np.concatenate([[0], np.cumsum(sig_len)]).astype(np.uint32)
    blob = (np.arange(int(sig_off[-1])) % 251).astype(np.uint8)
    msgs = (np.arange(32 * n) % 253).astype(np.uint8)
    p = PackedRequests(req_off, pk_off, msgs, blob, sig_off, idx=idx)
    parts = [p.slice(lo, hi) for lo, hi in shard_requests(sizes.tolist(), 3)]
    assert sum(q.n_req for q in parts) == 40
    assert np.array_equal(np.concatenate([q.msgs for q in parts]), msgs)
    assert np.array_equal(np.concatenate([q.idx for q in parts]), idx)
    assert np.array_equal(np.concatenate([q.sig_blob for q in parts]), blob)
    for q in parts:
        assert q.req_off[0] == 0 and q.pk_off[0] == 0 and q.sig_off[0] == 0
        assert int(q.sig_off[-1]) == len(q.sig_blob) and int(q.pk_off[-1]) == len(q.idx)
        assert int(q.req_off[-1]) * 32 == len(q.msgs) == 32 * (len(q.sig_off) - 1)


def test_packed_requests_slice_mixed_rows():
    """A mixed package (validator indices + byte keys named by LB_PK_ROW_FLAG
    indices): each slice keeps exactly the rows it names, renumbered from 0, so
    every key resolves to the same bytes / index as in the whole package."""
    import numpy as np
    from lodestar_amd.native import LB_PK_ROW_FLAG
    from lodestar_amd.sharding import PackedRequests, shard_requests
    rng = np.random.default_rng(2)
    sizes = rng.integers(1, 5, 30)
    req_off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint32)
    n = int(req_off[-1])
    pk_off = np.arange(n + 1, dtype=np.uint32)
    is_row = rng.random(n) < 0.3
    rows = rng.integers(0, 256, (int(is_row.sum()), 96)).astype(np.uint8)
    idx = np.where(is_row, 0, rng.integers(0, 1000, n)).astype(np.uint32)
    idx[is_row] = LB_PK_ROW_FLAG | np.arange(int(is_row.sum()), dtype=np.uint32)
    sig_off = np.arange(n + 1, dtype=np.uint32) * 96
    p = PackedRequests(req_off, pk_off, np.zeros(32 * n, np.uint8), np.zeros(96 * n, np.uint8), sig_off,
                       idx=idx, pks=rows.reshape(-1))

    def resolve(q):
        out = []
        for v in q.idx:
            v = int(v)
            out.append(bytes(q.pks.reshape(-1, 96)[v ^ LB_PK_ROW_FLAG]) if v & LB_PK_ROW_FLAG else v)
        return out
    whole = resolve(p)
    got = []
    for lo, hi in shard_requests(sizes.tolist(), 4):
        q = p.slice(lo, hi)
        n_rows = int(((q.idx & LB_PK_ROW_FLAG) != 0).sum())
        assert n_rows == 0 or len(q.pks) == 96 * n_rows
        got += resolve(q)
    assert got == whole
