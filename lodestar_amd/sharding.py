"""Multi-GPU sharding of verification requests.

Sets are independent and the batch equation is multiplicative, so a batch of
requests shards across GPUs with no data-path collective: each GPU gets a
contiguous range of whole requests (a request -- one BlsWorkReq of <= 128
sets, multithread/index.ts:57 -- is never split) and runs it up to its merged
Miller product P_g (576 bytes, lb_verify_requests_partial_async).  The host
gathers the <= 8 partials and checks final_exp(prod_g P_g) == 1 ONCE
(lb_gt_check); every shard then resumes with that verdict: all requests valid
with no further work, or -- only when the combined check fails -- each shard
verifies its requests alone (worker.ts:74-85 after a failed merged batch).
RCCL over xGMI is not used: per GPU the exchange is 576 bytes.

* ``shard_requests``: balance ranges by set count.
* ``ShardedVerifier``: one process driving several local GPUs (one lb_ctx and
  one submission thread per GPU), with the Fp12-partial combine.
* ``verify_distributed``: one process per GPU under torch.distributed (gloo,
  host memory): the partials are all-gathered (576 B per rank), rank 0 runs the
  combined check and broadcasts it, then the verdict bytes are gathered.
"""
from __future__ import annotations

import threading
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

GT_BYTES = 576  # LB_GT_BYTES: one Fp12 partial


def shard_requests(request_sizes: Sequence[int], n_shards: int) -> List[Tuple[int, int]]:
    """Split requests [0, n) into n_shards contiguous [lo, hi) ranges of
    roughly equal set counts; every request lands in exactly one shard."""
    n = len(request_sizes)
    if n_shards <= 0:
        raise ValueError("n_shards must be positive")
    total = int(sum(request_sizes))
    bounds = [0]
    acc = 0
    k = 1
    for i, s in enumerate(request_sizes):
        acc += int(s)
        while k < n_shards and acc * n_shards >= total * k and bounds[-1] <= i:
            bounds.append(i + 1)
            k += 1
    while len(bounds) < n_shards:
        bounds.append(n)
    bounds.append(n)
    return [(bounds[j], bounds[j + 1]) for j in range(n_shards)]


def slice_requests(requests: Sequence, lo: int, hi: int) -> list:
    return list(requests[lo:hi])


@dataclass
class PackedRequests:
    """Requests already in the C-ABI layout (lb_request_batch): the shape a gossip
    replay of ~1 M sets takes without one Python object per set or per key.
    ``idx`` holds validator indices (device pubkey table) when not None, else
    ``pks`` the 96-byte keys; with both, a mixed package: ``idx`` entries carrying
    LB_PK_ROW_FLAG name rows of ``pks`` (keys without a validator index).
    ``msgs`` is n_sets x 32 bytes."""
    req_off: np.ndarray
    pk_off: np.ndarray
    msgs: np.ndarray
    sig_blob: np.ndarray
    sig_off: np.ndarray
    idx: Optional[np.ndarray] = None
    pks: Optional[np.ndarray] = None

    @property
    def n_req(self) -> int:
        return len(self.req_off) - 1

    def request_sizes(self) -> np.ndarray:
        return np.diff(self.req_off.astype(np.int64))

    def slice(self, lo: int, hi: int) -> "PackedRequests":
        """Requests [lo, hi) as a call of their own (offsets rebased)."""
        a, b = int(self.req_off[lo]), int(self.req_off[hi])
        ka, kb = int(self.pk_off[a]), int(self.pk_off[b])
        sa, sb = int(self.sig_off[a]), int(self.sig_off[b])
        idx, pks = None, None
        if self.idx is not None and self.pks is not None:
            # mixed: keep the rows this slice names, renumbered from 0
            from .native import LB_PK_ROW48_FLAG, LB_PK_ROW_FLAG, LB_PK_ROW_MASK
            idx = self.idx[ka:kb].astype(np.uint32)
            flagged = (idx & LB_PK_ROW_FLAG) != 0
            rows = (idx[flagged] & np.uint32(LB_PK_ROW_MASK)).astype(np.int64)
            # (a compressed row keeps its LB_PK_ROW48_FLAG)
            idx[flagged] = (np.uint32(LB_PK_ROW_FLAG) | (idx[flagged] & np.uint32(LB_PK_ROW48_FLAG)) |
                            np.arange(len(rows), dtype=np.uint32))
            pks = self.pks.reshape(-1, 96)[rows].reshape(-1) if len(rows) else np.zeros(1, np.uint8)
        elif self.idx is not None:
            idx = self.idx[ka:kb]
        elif self.pks is not None:
            pks = self.pks[96 * ka:96 * kb]
        return PackedRequests(
            (self.req_off[lo:hi + 1] - a).astype(np.uint32), (self.pk_off[a:b + 1] - ka).astype(np.uint32),
            self.msgs[32 * a:32 * b], self.sig_blob[sa:sb] if sb > sa else np.zeros(1, np.uint8),
            (self.sig_off[a:b + 1] - sa).astype(np.uint32), idx, pks)


def _two_phase(backend) -> bool:
    return all(hasattr(backend, a) for a in ("submit_requests", "finish", "gt_check"))


class ShardedVerifier:
    """Verify a list of requests on several local GPUs concurrently.

    ``backends[g]`` offers ``verify_requests(requests) -> (valid, errors)``;
    when every backend also offers the two-phase protocol
    (lodestar_amd.verifier.DeviceBackend: ``submit_requests(partial=True)``,
    ``finish``, ``gt_check``) and ``combine`` is set, the shards' Fp12 partials
    are combined on the host with ONE final exponentiation (north_star).
    ``last_combine`` records the combined check of the last call.
    """

    def __init__(self, backends: Sequence[object], combine: bool = True):
        self.backends = list(backends)
        self.combine = combine and all(_two_phase(b) for b in self.backends)
        self.last_combine: Optional[dict] = None

    def verify_packed(self, p: PackedRequests) -> Tuple[List[bool], List[int]]:
        """verify_requests for requests already packed (PackedRequests): each shard's
        slice goes to its backend's submit_packed; the same two-phase combine."""
        shards = shard_requests(p.request_sizes().tolist(), len(self.backends))
        if not self.combine:
            raise ValueError("verify_packed needs two-phase backends (DeviceBackend)")
        return self._verify_combined(p, shards, packed=True)

    def verify_requests(self, requests: Sequence) -> Tuple[List[bool], List[int]]:
        shards = shard_requests([len(r) for r in requests], len(self.backends))
        if self.combine:
            return self._verify_combined(requests, shards)
        out_valid: List[bool] = [False] * len(requests)
        out_err: List[int] = [0] * len(requests)
        errors: List[BaseException] = []

        def run(g, lo, hi):
            try:
                if hi > lo:
                    r = self.backends[g].verify_requests(list(requests[lo:hi]))
                    out_valid[lo:hi] = r[0]
                    out_err[lo:hi] = r[1]
            except BaseException as ex:  # surfaced after join
                errors.append(ex)

        threads = [threading.Thread(target=run, args=(g, lo, hi)) for g, (lo, hi) in enumerate(shards)]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        if errors:
            raise errors[0]
        return out_valid, out_err

    def _verify_combined(self, requests, shards, packed: bool = False):
        live = [(g, lo, hi) for g, (lo, hi) in enumerate(shards) if hi > lo]
        # phase 1: every GPU runs its shard up to the merged Miller product
        futs = [(g, lo, hi, self.backends[g].submit_packed(requests.slice(lo, hi), partial=True) if packed else
                 self.backends[g].submit_requests(list(requests[lo:hi]), partial=True))
                for g, lo, hi in live]
        calls, errors = [], []
        for g, lo, hi, f in futs:
            try:
                calls.append((g, lo, hi, f.result()))
            except BaseException as ex:  # noqa: BLE001 -- re-raised below, after the others are resumed
                errors.append(ex)
        if errors:
            # never leave a shard's slot holding a partial: resume every call that got one
            # (merged_ok = False: each runs its own per-request tails), then fail the call
            for _, _, _, c in calls:
                try:
                    c.backend.finish(c, False).result()
                except BaseException:  # noqa: BLE001
                    pass
            raise errors[0]
        # host combine: prod of the <= 8 partials, one final exponentiation on the GPU of the
        # largest shard (shards are balanced, so the check lands on a different GPU per call
        # rather than always on GPU 0)
        partials = [c.partial for _, _, _, c in calls]
        if calls:
            gi = max(range(len(calls)), key=lambda i: (calls[i][2] - calls[i][1], -i))
            ok = bool(self.backends[calls[gi][0]].gt_check(partials).result())
        else:
            ok = True
        self.last_combine = {"merged_ok": ok, "n_partials": len(partials)}
        # phase 2: resume every shard with the combined verdict
        fins = [(lo, hi, c.backend.finish(c, ok)) for _, lo, hi, c in calls]
        n = requests.n_req if packed else len(requests)
        out_valid: List[bool] = [False] * n
        out_err: List[int] = [0] * n
        for lo, hi, f in fins:
            v, e, _ = f.result()
            out_valid[lo:hi] = v
            out_err[lo:hi] = e
        return out_valid, out_err


def verify_distributed(requests: Sequence, verify_local: Optional[Callable[[list], Tuple[List[bool], List[int]]]],
                       rank: int, world: int, backend: Optional[object] = None) -> Tuple[List[bool], List[int]]:
    """torch.distributed version (one process per GPU): every rank holds the
    same request list and verifies its own shard.  With a two-phase ``backend``
    the ranks all-gather their 576-byte partials (gloo, host memory), rank 0 runs
    the ONE combined check and broadcasts its verdict, and every rank resumes its
    shard; otherwise ``verify_local`` verifies the shard alone.  All ranks
    receive every verdict (gloo all_gather of one int per request).  A rank whose
    shard raises still joins every collective (with an error flag), so all ranks
    fail together instead of leaving the others blocked."""
    import torch
    import torch.distributed as dist
    shards = shard_requests([len(r) for r in requests], world)
    lo, hi = shards[rank]
    err: Optional[BaseException] = None
    v: List[bool] = []
    e: List[int] = []
    if backend is not None and _two_phase(backend):
        call = None
        try:
            call = backend.submit_requests(list(requests[lo:hi]), partial=True).result() if hi > lo else None
        except BaseException as ex:  # noqa: BLE001
            err = ex
        part = torch.zeros(GT_BYTES + 2, dtype=torch.uint8)
        if call is not None:
            part[:GT_BYTES] = torch.frombuffer(bytearray(call.partial), dtype=torch.uint8)
            part[GT_BYTES] = 1
        part[GT_BYTES + 1] = 1 if err is not None else 0
        parts = [torch.zeros(GT_BYTES + 2, dtype=torch.uint8) for _ in range(world)]
        dist.all_gather(parts, part)
        any_err = any(int(p[GT_BYTES + 1]) for p in parts)
        verdict = torch.zeros(1, dtype=torch.int32)
        if rank == 0 and not any_err:
            partials = [bytes(p[:GT_BYTES].tolist()) for p in parts if int(p[GT_BYTES]) == 1]
            try:
                verdict[0] = 1 if bool(backend.gt_check(partials).result()) else 0
            except BaseException as ex:  # noqa: BLE001
                err, verdict[0] = ex, -1
        dist.broadcast(verdict, 0)
        any_err = any_err or int(verdict[0]) < 0
        if call is not None:
            try:
                v, e, _ = backend.finish(call, (not any_err) and int(verdict[0]) == 1).result()
            except BaseException as ex:  # noqa: BLE001
                err = err or ex
    else:
        try:
            v, e = verify_local(list(requests[lo:hi])) if hi > lo else ([], [])
        except BaseException as ex:  # noqa: BLE001
            err = ex
    n = len(requests)
    mine = torch.zeros(n + 1, dtype=torch.int32)
    if hi > lo and err is None:
        mine[lo:hi] = torch.tensor([int(x) | (int(y) << 8) for x, y in zip(v, e)], dtype=torch.int32)
    mine[n] = 1 if err is not None else 0
    gathered = [torch.zeros(n + 1, dtype=torch.int32) for _ in range(world)]
    dist.all_gather(gathered, mine)
    if err is not None:
        raise err
    bad = [r for r in range(world) if int(gathered[r][n])]
    if bad:
        raise RuntimeError(f"verify_distributed: rank(s) {bad} failed")
    combined = np.zeros(n, dtype=np.int32)
    for r, (a, b) in enumerate(shards):
        combined[a:b] = gathered[r].numpy()[a:b]
    return [bool(x & 0xFF) for x in combined], [int(x >> 8) for x in combined]
