"""BlsGpuVerifier: the IBlsVerifier surface over the MI355X C ABI.

Mirrors packages/beacon-node/src/chain/bls/interface.ts:25-68 and the job
scheduling of BlsMultiThreadWorkerPool (chain/bls/multithread/index.ts:114-580)
with GPUs in place of worker threads:

* verify_signature_sets(sets, opts) -> bool           (index.ts:163-213)
* verify_signature_sets_same_message(sets, msg, opts) -> [bool]  (index.ts:218-242)
* close()                                             (index.ts:244-265)
* can_accept_work()                                   (index.ts:155-161)

Scheduling rules kept from the reference:
* sets are chunked with chunkify_maximize_chunk_size(sets, 128) into jobs (index.ts:191-205)
* batchable jobs are buffered until MAX_BUFFER_WAIT_MS = 100 ms or more than
  MAX_BUFFERED_SIGS = 32 sigs are buffered (index.ts:327-343); priority jobs
  go to the queue front (index.ts:544-555)
* an aggregate set with no pubkeys rejects its job (index.ts:403-409)
* a same-message job that fails is retried set by set (index.ts:473-484,557-568)
* verify_on_main_thread verifies synchronously on the caller's thread (index.ts:174-187)

What changes for a GPU: a dispatch ("package") may hold many more than 128
sig sets (max_sets_per_dispatch, default 65,536) because the GPU needs tens of
thousands of sets in flight; every job still gets its own verdict, computed
per request on the device (lb_verify_requests), so merging never changes a
verdict (worker.ts:74-85 guarantees the same on CPU by re-verifying).
"""
from __future__ import annotations

import asyncio
import concurrent.futures
import enum
import os
import threading
import time
from collections import deque
from dataclasses import dataclass, field
from typing import Callable, Deque, List, Optional, Sequence, Tuple, Union

import numpy as np

from . import metrics as M
from .native import (LB_PK_ROW_FLAG, PendingSameMessage, LB_REQ_BAD_PUBKEY, LB_REQ_EMPTY_AGGREGATE, BadPubkeyError, Device, EmptyAggregateError,
                     pack_blobs)

MAX_SIGNATURE_SETS_PER_JOB = 128      # index.ts:57
MAX_BUFFERED_SIGS = 32                # index.ts:66
MAX_BUFFER_WAIT_MS = 100              # index.ts:75
MAX_JOBS_CAN_ACCEPT_WORK = 512        # index.ts:80
BATCHABLE_MIN_PER_CHUNK = 16          # worker.ts:17


class SignatureSetType(str, enum.Enum):
    single = "single"
    aggregate = "aggregate"


@dataclass
class PublicKey:
    """A G1 public key: its 96-byte uncompressed encoding (what jobItemWorkReq
    ships to the worker, jobItem.ts:59 / index.ts:144) and/or its validator
    index in the device-resident pubkey table (the index2pubkey mirror,
    state-transition/src/cache/pubkeyCache.ts:56-77; see sync_pubkeys).  A
    package whose keys all carry an index ships 4-byte indices instead of
    points and is aggregated on the GPU from the table."""
    uncompressed: bytes = b""
    index: Optional[int] = None

    def __post_init__(self):
        if self.index is None and len(self.uncompressed) != 96:
            raise ValueError("PublicKey expects the 96-byte uncompressed encoding or a validator index")
        if self.uncompressed and len(self.uncompressed) != 96:
            raise ValueError("PublicKey expects the 96-byte uncompressed encoding")


@dataclass
class SignatureSet:
    """ISignatureSet (packages/state-transition/src/util/signatureSets.ts:5-24)."""
    type: SignatureSetType
    signing_root: bytes
    signature: bytes
    pubkey: Optional[PublicKey] = None          # single
    pubkeys: Optional[List[PublicKey]] = None   # aggregate


def single_set(pubkey: PublicKey, signing_root: bytes, signature: bytes) -> SignatureSet:
    return SignatureSet(SignatureSetType.single, signing_root, signature, pubkey=pubkey)


def aggregate_set(pubkeys: Sequence[PublicKey], signing_root: bytes, signature: bytes) -> SignatureSet:
    return SignatureSet(SignatureSetType.aggregate, signing_root, signature, pubkeys=list(pubkeys))


@dataclass
class VerifySignatureOpts:
    batchable: bool = False
    verify_on_main_thread: bool = False
    priority: bool = False


class QueueErrorCode(str, enum.Enum):
    QUEUE_ABORTED = "QUEUE_ERROR_QUEUE_ABORTED"


class QueueError(Exception):
    def __init__(self, code: QueueErrorCode):
        super().__init__(code.value)
        self.code = code


def chunkify_maximize_chunk_size(arr: Sequence, min_per_chunk: int) -> List[list]:
    """multithread/utils.ts:4-19."""
    chunk_count = len(arr) // min_per_chunk
    if chunk_count <= 1:
        return [list(arr)]
    per_chunk = -(-len(arr) // chunk_count)
    return [list(arr[i:i + per_chunk]) for i in range(0, len(arr), per_chunk)]


class JobType(str, enum.Enum):
    default = "default"
    same_message = "same_message"


@dataclass
class _Job:
    type: JobType
    future: asyncio.Future
    opts: VerifySignatureOpts
    sets: list
    message: Optional[bytes] = None
    added: float = field(default_factory=time.monotonic)

    def sig_sets(self) -> int:
        """jobItemSigSets (jobItem.ts:39-46): a same-message job counts as 1."""
        return len(self.sets) if self.type == JobType.default else 1


def worker_batch_stats(request_sizes: Sequence[int], batchable: Sequence[bool],
                       valid: Sequence[bool]) -> Tuple[int, int]:
    """(batchRetries, batchSigsSuccess) exactly as the reference worker counts
    them for one package (multithread/worker.ts:41-85): batchable requests are
    split with chunkifyMaximizeChunkSize(batchable, 16) and each chunk is one
    merged verifySignatureSetsMaybeBatch; a chunk passes iff all its sets verify
    (every request in it valid) -- then its sets count as batchSigsSuccess --
    else it is one batchRetry.  The GPU verifies a whole package in one merged
    check instead, so the device's own merged-check stats differ; the pool
    metrics report these, the reference's, so dashboards read the same."""
    idx = [k for k, b in enumerate(batchable) if b]
    retries = sigs_ok = 0
    if not idx:
        return 0, 0
    for chunk in chunkify_maximize_chunk_size(idx, BATCHABLE_MIN_PER_CHUNK):
        n = sum(request_sizes[k] for k in chunk)
        if n > 0 and all(valid[k] for k in chunk):
            sigs_ok += n
        else:
            retries += 1
    return retries, sigs_ok


@dataclass
class CallStats:
    """Per-call bookkeeping a backend reports with its verdicts."""
    batch_retries: int = 0        # device merged check (0/1) or same-message jobs retried set by set
    batch_sigs_success: int = 0
    device_ms: float = 0.0
    t_start: float = 0.0          # the submission thread picked the call up ("worker start")
    t_end: float = 0.0            # verdicts ready on the submission thread ("worker end")
    stage_ms: Optional[dict] = None


class DeviceBackend:
    """One GPU (one lb_ctx) behind ONE host submission thread (SURVEY §8b:
    "one host submission thread per GPU"): the context is not thread-safe, so
    every library call runs on that thread.  Callers get
    ``concurrent.futures.Future``s; up to ``capacity`` calls (the library's
    slots, one per HIP hardware queue) are kept in flight, so one package's
    tails overlap the next package's per-set stages -- the reference pool's
    several workers (multithread/index.ts:47,362-519) in one device."""

    def __init__(self, device: int = 0, seed_source: Callable[[], bytes] = lambda: os.urandom(32),
                 capacity: Optional[int] = None, dev: Optional[object] = None):
        self.dev = dev if dev is not None else Device(device)  # dev: an injected stand-in (host tests)
        self.device = device
        self.seed_source = seed_source
        # the library's calls in flight (lb_slots: one per HIP hardware queue of the process)
        self.capacity = capacity or (self.dev.slots() if hasattr(self.dev, "slots") else
                                     max(1, int(os.environ.get("LB_SLOTS", "4"))))
        self._q: Deque[tuple] = deque()
        self._cv = threading.Condition()
        self._closing = False
        self._thread = threading.Thread(target=self._loop, name=f"lb-gpu{device}", daemon=True)
        self._thread.start()

    # ---- submission thread ----------------------------------------------------------
    def _put(self, kind: str, payload, front: bool = False) -> concurrent.futures.Future:
        fut: concurrent.futures.Future = concurrent.futures.Future()
        with self._cv:
            if self._closing:
                raise QueueError(QueueErrorCode.QUEUE_ABORTED)
            (self._q.appendleft if front else self._q.append)((kind, payload, fut))
            self._cv.notify()
        return fut

    def _loop(self) -> None:
        inflight: Deque[tuple] = deque()  # (PendingCall, future, post, CallStats)
        # two-phase calls handed out and not yet finished hold a library slot too: they
        # count against capacity, so no later call reuses (and silently resumes) their slot
        self._partials = 0
        while True:
            with self._cv:
                while not self._q and not inflight and not self._closing:
                    self._cv.wait()
                # a finish never needs a free slot (it resumes its own)
                head_is_finish = bool(self._q) and self._q[0][0] == "finish"
                room = len(inflight) + self._partials < self.capacity
                item = self._q.popleft() if self._q and (room or head_is_finish) else None
                if item is None and not inflight and self._closing and not self._q:
                    break
                if item is None and not inflight and self._q:
                    # every slot holds a partial waiting for its host verdict: hand out the
                    # next call anyway (the library then resumes the oldest with merged_ok = 0)
                    item = self._q.popleft()
            if item is not None:
                kind, payload, fut = item
                if not fut.set_running_or_notify_cancel():
                    continue
                cs = CallStats(t_start=time.monotonic())
                try:
                    if kind in ("requests", "packed"):
                        requests, partial = payload
                        pc, post = (self._submit_requests(requests, partial) if kind == "requests" else
                                    self._submit_packed(requests, partial))
                        if partial:
                            self._partials += 1
                            try:
                                part = self.dev.partial_wait(pc)
                            except BaseException:
                                self._partials -= 1
                                self.dev.verify_finish(pc, False)
                                raise
                            fut.set_result(PartialCall(self, pc, post, cs, part))
                        else:
                            inflight.append((pc, fut, post, cs))
                    elif kind == "finish":
                        call, ok = payload
                        self._partials = max(0, self._partials - 1)
                        self.dev.verify_finish(call.pc, ok)
                        inflight.append((call.pc, fut, call.post, call.stats))
                    elif kind == "same_message":
                        # one package of same-message jobs, in flight like any call: its
                        # per-set retries run when it retires, on its own slot
                        pc, post = self._submit_same_message(payload)
                        inflight.append((pc, fut, post, cs))
                    else:  # synchronous library calls (same-message batch, table sync, gt check, ...)
                        fut.set_result(payload(cs))
                except BaseException as e:  # noqa: BLE001 -- surfaced through the future
                    fut.set_exception(e)
                continue
            pc, fut, post, cs = inflight.popleft()
            try:
                if isinstance(pc, PendingSameMessage):
                    res, fast, (retried, ok_sets), dev_ms = self.dev.wait_same_message(pc)
                    cs.batch_retries, cs.batch_sigs_success, cs.device_ms = retried, ok_sets, dev_ms
                    cs.stage_ms = dict(self.dev.last_stage_times())
                    cs.t_end = time.monotonic()
                    fut.set_result((res, fast, cs))
                    continue
                res = self.dev.wait_call(pc)
                cs.batch_retries, cs.batch_sigs_success, cs.device_ms = (res.batch_retries, res.batch_sigs_success,
                                                                         res.device_ms)
                cs.stage_ms = dict(self.dev.last_stage_times())
                cs.t_end = time.monotonic()
                fut.set_result(post(res, cs))
            except BaseException as e:  # noqa: BLE001
                fut.set_exception(e)
        self.dev.close()

    def _submit_requests(self, requests: List[List[SignatureSet]], partial: bool):
        keys_all, pk_off, msgs, sigs, req_off = [], [0], [], [], [0]
        for req in requests:
            for s in req:
                keys = [s.pubkey] if s.type == SignatureSetType.single else (s.pubkeys or [])
                keys_all.extend(keys)
                pk_off.append(len(keys_all))
                if len(s.signing_root) != 32:
                    raise ValueError("signing_root must be 32 bytes")
                msgs.append(bytes(s.signing_root))
                sigs.append(bytes(s.signature))
            req_off.append(len(msgs))
        blob, offs = pack_blobs(sigs)
        # validator indices when every key has one (device table); a mixed package (e.g. a
        # capella block's BLS-change keys beside validator keys) ships the byte keys as rows
        # named by flagged indices (LB_PK_ROW_FLAG); with no index at all, the encodings
        n_idx = sum(1 for k in keys_all if k.index is not None)
        idx = pks = None
        if keys_all and n_idx == len(keys_all):
            idx = np.array([k.index for k in keys_all], np.uint32)
        elif n_idx:
            rows: List[bytes] = []
            ix = []
            for k in keys_all:
                if k.index is not None:
                    ix.append(k.index)
                else:
                    ix.append(LB_PK_ROW_FLAG | len(rows))
                    rows.append(k.uncompressed)
            idx = np.array(ix, np.uint32)
            pks = np.frombuffer(b"".join(rows), np.uint8)
        else:
            pks = np.frombuffer(b"".join(self._key_bytes(keys_all)) or b"\0", np.uint8)
        pc = self.dev.verify_requests_async(np.array(req_off, np.uint32), pks, np.array(pk_off, np.uint32),
                                            np.frombuffer(b"".join(msgs) or b"\0", np.uint8), blob, offs,
                                            self.seed_source(), pk_indices=idx, partial=partial)

        def post(res, cs):
            return [bool(v) for v in res.valid], [int(e) for e in res.errors], cs
        return pc, post

    def _submit_packed(self, p, partial: bool):
        # (with both idx and pks: a mixed package, flagged indices naming rows of pks)
        pc = self.dev.verify_requests_async(p.req_off, p.pks, p.pk_off, p.msgs,
                                            p.sig_blob, p.sig_off, self.seed_source(), pk_indices=p.idx,
                                            partial=partial)

        def post(res, cs):
            return [bool(v) for v in res.valid], [int(e) for e in res.errors], cs
        return pc, post

    def _key_bytes(self, keys: Sequence[PublicKey]) -> List[bytes]:
        """96-byte encodings; index-only keys are read back from the device table
        (mixed packages only).  An index outside the table -> an all-zero
        encoding, which decodes as a bad pubkey (LB_REQ_BAD_PUBKEY)."""
        size = None
        out = []
        for k in keys:
            if k.uncompressed:
                out.append(k.uncompressed)
                continue
            size = self.dev.pubkey_table_size() if size is None else size
            out.append(self.dev.pubkey_table_read(k.index, 1)[0] if 0 <= k.index < size else bytes(96))
        return out

    # ---- API used by BlsGpuVerifier / ShardedVerifier --------------------------------
    def submit_requests(self, requests: List[List[SignatureSet]], partial: bool = False,
                        priority: bool = False) -> concurrent.futures.Future:
        """Future of (valid, errors, CallStats); with partial=True a PartialCall
        (the shard's 576-byte Fp12 partial, to be finished with finish())."""
        return self._put("requests", (list(requests), partial), front=priority)

    def submit_packed(self, p, partial: bool = False, priority: bool = False) -> concurrent.futures.Future:
        """submit_requests for requests already in the C-ABI layout
        (sharding.PackedRequests): no per-set packing on the host."""
        return self._put("packed", (p, partial), front=priority)

    def finish(self, call: "PartialCall", merged_ok: bool) -> concurrent.futures.Future:
        return self._put("finish", (call, merged_ok), front=True)

    def gt_check(self, partials: Sequence[bytes]) -> concurrent.futures.Future:
        return self._put("call", lambda cs: self.dev.gt_check(list(partials)), front=True)

    def _submit_same_message(self, jobs):
        by_index = all(k.index is not None for pks, _, _ in jobs for k in pks)
        dj = [([k.index for k in pks] if by_index else self._key_bytes(pks), list(sigs), bytes(msg))
              for pks, sigs, msg in jobs]
        return self.dev.verify_same_message_batch_async(dj, self.seed_source(), by_index=by_index), None

    def submit_same_message(self, jobs: Sequence[Tuple[Sequence[PublicKey], Sequence[bytes], bytes]],
                            priority: bool = False) -> concurrent.futures.Future:
        """Future of (per-job verdict lists, per-job fast flags, CallStats): all
        same-message jobs of a package in one device call, kept in flight beside
        the other packages (lb_verify_same_message_batch_async)."""
        return self._put("same_message", list(jobs), front=priority)

    def verify_requests(self, requests: List[List[SignatureSet]]) -> Tuple[List[bool], List[int]]:
        """Blocking convenience (tests, ShardedVerifier without the combine)."""
        valid, errors, _ = self.submit_requests(requests).result()
        return valid, errors

    def verify_same_message(self, pubkeys: Sequence[PublicKey], signatures: Sequence[bytes],
                            message: bytes) -> List[bool]:
        res, _, _ = self.submit_same_message([(list(pubkeys), list(signatures), message)]).result()
        return res[0]

    def sync_pubkeys(self, pubkeys: Sequence[bytes]) -> int:
        """syncPubkeys (pubkeyCache.ts:56-77): append validators' keys (48-byte
        compressed, as the state holds them) to the device table; returns its size."""
        return self._put("call", lambda cs: self.dev.pubkey_table_append(list(pubkeys))).result()

    def close(self) -> None:
        """Finish every queued and in-flight call, then release the device
        (from the submission thread, after its last call -- never under one)."""
        with self._cv:
            self._closing = True
            self._cv.notify()
        if threading.current_thread() is not self._thread:
            self._thread.join()


@dataclass
class PartialCall:
    """A shard stopped at its merged Miller product (two-phase call)."""
    backend: DeviceBackend
    pc: object
    post: Callable
    stats: CallStats
    partial: bytes


class BlsGpuVerifier:
    """IBlsVerifier over one or more GPUs (BlsMultiThreadWorkerPool with GPUs as
    workers; each GPU backend takes up to ``capacity`` packages at once)."""

    def __init__(self, backends: Optional[Sequence[object]] = None, devices: Optional[Sequence[int]] = None,
                 blsVerifyAllMultiThread: bool = False, max_sets_per_dispatch: int = 65536,
                 loop: Optional[asyncio.AbstractEventLoop] = None):
        if backends is None:
            devices = list(devices) if devices is not None else [0]
            backends = [DeviceBackend(d) for d in devices]
        self.backends = list(backends)
        if not self.backends:
            raise ValueError("at least one backend/device is required")
        self.verify_all_multi_thread = blsVerifyAllMultiThread
        self.max_sets_per_dispatch = max_sets_per_dispatch
        self._jobs: Deque[_Job] = deque()
        self._buffered: Optional[dict] = None
        # one idle entry per package a backend can hold in flight (index.ts: one per worker)
        self._idle = [bi for bi, b in enumerate(self.backends) for _ in range(max(1, getattr(b, "capacity", 1)))]
        self._capacity = len(self._idle)
        self._running: set = set()  # dispatch tasks in flight (awaited by close())
        self._closed = False
        self._loop = loop
        self.metrics = {"total_sig_sets": 0, "batchable_sig_sets": 0, "prioritized_sig_sets": 0,
                        "jobs_started": 0, "dispatches": 0, "same_message_retry_jobs": 0,
                        "same_message_retry_sets": 0, "aggregated_pubkeys": 0}
        # the reference's metric names (lodestar.ts:380-495), see lodestar_amd/metrics.py
        self.pool_metrics = M.BlsPoolMetrics()

    def sync_pubkeys(self, pubkeys: Sequence[bytes]) -> int:
        """Append validators' pubkeys to every GPU's device table (index2pubkey
        mirror, pubkeyCache.ts:56-77); sets may then carry PublicKey(index=i)."""
        sizes = [b.sync_pubkeys(pubkeys) for b in self.backends]
        if len(set(sizes)) != 1:
            raise RuntimeError(f"pubkey tables out of sync across devices: {sizes}")
        return sizes[0]

    # ---- IBlsVerifier --------------------------------------------------------------
    def can_accept_work(self) -> bool:
        """index.ts:155-161: workersBusy < poolSize && jobs < MAX_JOBS_CAN_ACCEPT_WORK."""
        return len(self._idle) > 0 and len(self._jobs) < MAX_JOBS_CAN_ACCEPT_WORK

    async def verify_signature_sets(self, sets: List[SignatureSet],
                                    opts: Optional[VerifySignatureOpts] = None) -> bool:
        opts = opts or VerifySignatureOpts()
        pm = self.pool_metrics
        n_agg = sum(len(s.pubkeys or []) for s in sets if s.type == SignatureSetType.aggregate)
        self.metrics["aggregated_pubkeys"] += n_agg
        pm.inc(M.AGGREGATED_PUBKEYS, n_agg)
        self.metrics["total_sig_sets"] += len(sets)
        pm.inc(M.TOTAL_SIG_SETS, len(sets))
        if opts.priority:
            self.metrics["prioritized_sig_sets"] += len(sets)
            pm.inc(M.PRIORITIZED_SIG_SETS, len(sets))
        if opts.batchable:
            self.metrics["batchable_sig_sets"] += len(sets)
            pm.inc(M.BATCHABLE_SIG_SETS, len(sets))
        for s in sets:
            if len(s.signing_root) != 32:
                raise ValueError("signing_root must be 32 bytes")
        if opts.verify_on_main_thread and not self.verify_all_multi_thread:
            # synchronous, on the caller's thread (index.ts:174-187): blocks it, as the reference blocks the main thread
            t0 = time.monotonic()
            try:
                return self._verify_now(sets)
            finally:
                pm.observe(M.MAIN_THREAD_TIME, time.monotonic() - t0)
        loop = self._get_loop()
        futs = []
        for chunk in chunkify_maximize_chunk_size(sets, MAX_SIGNATURE_SETS_PER_JOB):
            fut = loop.create_future()
            self._queue(_Job(JobType.default, fut, opts, chunk))
            futs.append(fut)
        results = await asyncio.gather(*futs)
        if len(results) == 0:
            raise RuntimeError("Empty results array")
        return all(r is True for r in results)

    async def verify_signature_sets_same_message(self, sets: List[Tuple[PublicKey, bytes]], message: bytes,
                                                 opts: Optional[VerifySignatureOpts] = None) -> List[bool]:
        opts = opts or VerifySignatureOpts()
        if len(message) != 32:
            raise ValueError("message must be 32 bytes")
        loop = self._get_loop()
        futs = []
        for chunk in chunkify_maximize_chunk_size(sets, MAX_SIGNATURE_SETS_PER_JOB):
            fut = loop.create_future()
            self._queue(_Job(JobType.same_message, fut, opts, chunk, message=bytes(message)))
            futs.append(fut)
        results = await asyncio.gather(*futs)
        return [v for r in results for v in r]

    async def close(self) -> None:
        """index.ts:244-265: abort queued jobs, then wait for the packages already
        on a GPU and release the devices (never while a call is in flight)."""
        if self._buffered is not None and self._buffered.get("timer") is not None:
            self._buffered["timer"].cancel()
        for job in self._jobs:
            if not job.future.done():
                job.future.set_exception(QueueError(QueueErrorCode.QUEUE_ABORTED))
        self._jobs.clear()
        if self._buffered is not None:
            for job in self._buffered["jobs"] + self._buffered["prioritized"]:
                if not job.future.done():
                    job.future.set_exception(QueueError(QueueErrorCode.QUEUE_ABORTED))
            self._buffered = None
        self._closed = True
        if self._running:
            await asyncio.gather(*list(self._running), return_exceptions=True)
        loop = self._get_loop()
        for b in self.backends:
            close = getattr(b, "close", None)
            if close:
                await loop.run_in_executor(None, close)

    # ---- scheduling -------------------------------------------------------------------
    def _get_loop(self):
        if self._loop is None:
            self._loop = asyncio.get_running_loop()
        return self._loop

    def _queue(self, job: _Job) -> None:
        if self._closed:
            raise QueueError(QueueErrorCode.QUEUE_ABORTED)
        loop = self._get_loop()
        if job.opts.batchable:
            if self._buffered is None:
                self._buffered = {"jobs": [], "prioritized": [], "sig_count": 0,
                                  "timer": loop.call_later(MAX_BUFFER_WAIT_MS / 1000, self._run_buffered)}
            (self._buffered["prioritized"] if job.opts.priority else self._buffered["jobs"]).append(job)
            self._buffered["sig_count"] += job.sig_sets()
            if self._buffered["sig_count"] > MAX_BUFFERED_SIGS:
                self._buffered["timer"].cancel()
                self._run_buffered()
        else:
            if job.opts.priority:
                self._jobs.appendleft(job)
            else:
                self._jobs.append(job)
            loop.call_soon(self._run_job)

    def _run_buffered(self) -> None:
        if self._buffered is None:
            return
        for job in self._buffered["jobs"]:
            self._jobs.append(job)
        for job in self._buffered["prioritized"]:
            self._jobs.appendleft(job)
        self._buffered = None
        self._get_loop().call_soon(self._run_job)

    def _prepare_work(self) -> List[_Job]:
        jobs, total = [], 0
        while total < self.max_sets_per_dispatch and self._jobs:
            job = self._jobs.popleft()
            jobs.append(job)
            total += job.sig_sets()
        return jobs

    def _run_job(self) -> None:
        if self._closed or not self._idle or not self._jobs:
            return
        jobs = self._prepare_work()
        if not jobs:
            return
        bi = self._idle.pop(0)
        self.metrics["dispatches"] += 1
        self.metrics["jobs_started"] += len(jobs)
        pm, now = self.pool_metrics, time.monotonic()
        pm.inc(M.JOB_GROUPS_STARTED)  # index.ts:433-437
        for t in (JobType.default, JobType.same_message):
            pm.inc(M.JOBS_STARTED, sum(1 for j in jobs if j.type == t), type=t.value)
            pm.inc(M.SIG_SETS_STARTED, sum(len(j.sets) for j in jobs if j.type == t), type=t.value)
        for j in jobs:
            pm.observe(M.JOB_WAIT_TIME, now - j.added)  # index.ts:396
        pm.set(M.WORKERS_BUSY, self._capacity - len(self._idle))
        pm.set(M.QUEUE_LENGTH, len(self._jobs))
        task = self._get_loop().create_task(self._dispatch(bi, jobs))
        self._running.add(task)
        task.add_done_callback(self._running.discard)
        if self._idle and self._jobs:  # more packages while GPUs have free slots
            self._get_loop().call_soon(self._run_job)

    async def _dispatch(self, bi: int, jobs: List[_Job]) -> None:
        """One package on backend bi: default jobs as requests of one call, all
        same-message jobs in one batched call; the event loop never blocks."""
        backend = self.backends[bi]
        loop = self._get_loop()
        t_dispatch = time.monotonic()
        default_idx = [i for i, j in enumerate(jobs) if j.type == JobType.default]
        same_idx = [i for i, j in enumerate(jobs) if j.type == JobType.same_message]
        prio = any(j.opts.priority for j in jobs)
        try:
            waits = []
            if default_idx:
                reqs = [jobs[i].sets for i in default_idx]
                if hasattr(backend, "submit_requests"):
                    waits.append(asyncio.wrap_future(backend.submit_requests(reqs, priority=prio)))
                else:
                    waits.append(loop.run_in_executor(None, _sync_requests, backend, reqs))
            if same_idx:
                sm = [([p for p, _ in jobs[i].sets], [s for _, s in jobs[i].sets], jobs[i].message) for i in same_idx]
                if hasattr(backend, "submit_same_message"):
                    waits.append(asyncio.wrap_future(backend.submit_same_message(sm, priority=prio)))
                else:
                    waits.append(loop.run_in_executor(None, _sync_same_message, backend, sm))
            outs = await asyncio.gather(*waits)
        except Exception as e:  # device failure rejects every job of the package (index.ts:503-512)
            self._idle.append(bi)
            self.pool_metrics.set(M.WORKERS_BUSY, self._capacity - len(self._idle))
            for job in jobs:
                if not job.future.done():
                    job.future.set_exception(e)
            loop.call_soon(self._run_job)
            return
        t_back = time.monotonic()
        self._idle.append(bi)
        pm = self.pool_metrics
        pm.set(M.WORKERS_BUSY, self._capacity - len(self._idle))
        results: List[tuple] = [None] * len(jobs)  # type: ignore[list-item]
        stats: List[CallStats] = []
        k = 0
        if default_idx:
            valid, errors, cs = outs[k]
            k += 1
            stats.append(cs)
            for n, i in enumerate(default_idx):
                results[i] = ("ok", valid[n]) if errors[n] == 0 else ("err", errors[n])
            # the reference worker's merged-batch accounting for this package (worker.ts:41-85)
            retries, sigs_ok = worker_batch_stats([len(jobs[i].sets) for i in default_idx],
                                                  [jobs[i].opts.batchable for i in default_idx],
                                                  [bool(valid[n]) and errors[n] == 0 for n in range(len(default_idx))])
            pm.inc(M.BATCH_RETRIES, retries)
            pm.inc(M.BATCH_SIGS_SUCCESS, sigs_ok)
        if same_idx:
            verdicts, fast, cs = outs[k]
            stats.append(cs)
            for n, i in enumerate(same_idx):
                results[i] = ("same", verdicts[n], fast[n])
            # same-message jobs are batchable requests of one set in the worker (jobItem.ts:75-86)
            retries, sigs_ok = worker_batch_stats([1] * len(same_idx), [jobs[i].opts.batchable for i in same_idx],
                                                  list(fast))
            pm.inc(M.BATCH_RETRIES, retries)
            pm.inc(M.BATCH_SIGS_SUCCESS, sigs_ok)
            if cs.stage_ms and "sm_decode" in cs.stage_ms:  # jobItem.ts:72-74, on the GPU here
                pm.observe(M.SIG_DESERIALIZATION_MAIN_THREAD, cs.stage_ms["sm_decode"] / 1e3)
        # index.ts:479-502 (workerId = the GPU backend): worker time, latency to / from the worker
        started = sum(len(j.sets) for j in jobs)
        for cs in stats:
            if cs.t_end:
                pm.inc(M.JOBS_WORKER_TIME, cs.t_end - cs.t_start, workerId=bi)
                if started:
                    pm.observe(M.TIME_PER_SIG_SET, (cs.t_end - cs.t_start) / started)
                pm.observe(M.LATENCY_TO_WORKER, max(0.0, cs.t_start - t_dispatch))
                pm.observe(M.LATENCY_FROM_WORKER, max(0.0, t_back - cs.t_end))
            if cs.stage_ms and "pubkeys_agg" in cs.stage_ms:  # utils.ts:13 main-thread aggregation, on the GPU here
                pm.observe(M.PUBKEYS_AGGREGATION_MAIN_THREAD, cs.stage_ms["pubkeys_agg"] / 1e3)
        pm.inc(M.SUCCESS_JOBS_SETS, sum(j.sig_sets() for j, r in zip(jobs, results) if r[0] != "err"))
        pm.inc(M.ERROR_JOBS_SETS, sum(j.sig_sets() for j, r in zip(jobs, results) if r[0] == "err"))
        for job, r in zip(jobs, results):
            if job.future.done():
                continue
            if r[0] == "ok":
                job.future.set_result(bool(r[1]))
            elif r[0] == "err":
                if r[1] == LB_REQ_EMPTY_AGGREGATE:  # index.ts:403-409
                    pm.inc(M.ERROR_AGGREGATE_SETS, len(job.sets), type=job.type.value)
                err = EmptyAggregateError("EMPTY_AGGREGATE_ARRAY") if r[1] == LB_REQ_EMPTY_AGGREGATE else \
                    BadPubkeyError("invalid pubkey encoding") if r[1] == LB_REQ_BAD_PUBKEY else RuntimeError(str(r[1]))
                job.future.set_exception(err)
            else:
                verdicts, fast = list(r[1]), r[2]
                if not fast and job.sets:
                    self.metrics["same_message_retry_jobs"] += 1
                    self.metrics["same_message_retry_sets"] += len(job.sets)
                    pm.inc(M.SAME_MESSAGE_RETRY_JOBS)  # index.ts:566-567
                    pm.inc(M.SAME_MESSAGE_RETRY_SETS, len(job.sets))
                job.future.set_result(verdicts)
        loop.call_soon(self._run_job)

    def _verify_now(self, sets: List[SignatureSet]) -> bool:
        valid, errors = self.backends[0].verify_requests([sets])[:2]
        if errors[0] == LB_REQ_EMPTY_AGGREGATE:
            raise EmptyAggregateError("EMPTY_AGGREGATE_ARRAY")
        if errors[0] != 0:
            raise BadPubkeyError("invalid pubkey encoding")
        return valid[0]


def _sync_requests(backend, reqs):
    out = backend.verify_requests(reqs)
    return (out[0], out[1], out[2] if len(out) > 2 else CallStats())


def _sync_same_message(backend, jobs):
    verdicts = [backend.verify_same_message(pks, sigs, msg) for pks, sigs, msg in jobs]
    fast = [bool(v) and all(v) for v in verdicts]
    return verdicts, fast, CallStats()


class BlsGpuSingleThreadVerifier:
    """BlsSingleThreadVerifier (chain/bls/singleThread.ts:10-89) on one GPU: no
    queue, no buffering; every call verifies synchronously on the caller's
    thread (chain.ts:206-208 picks it with blsVerifyAllMainThread).
    verifySignatureSets: aggregate + maybeBatch of the call's sets as one
    request.  verifySignatureSetsSameMessage: aggregate pubkeys and validated
    signatures, one verify; on failure each set alone (a malformed signature ->
    false).  Metrics: blsSingleThread.* and the main-thread timer."""

    def __init__(self, backend: Optional[object] = None, device: int = 0):
        self.backend = backend if backend is not None else DeviceBackend(device)
        self.pool_metrics = M.BlsPoolMetrics()

    async def verify_signature_sets(self, sets: List[SignatureSet],
                                    opts: Optional[VerifySignatureOpts] = None) -> bool:
        pm = self.pool_metrics
        pm.inc(M.AGGREGATED_PUBKEYS, sum(len(s.pubkeys or []) for s in sets if s.type == SignatureSetType.aggregate))
        t0 = time.monotonic()
        valid, errors = self.backend.verify_requests([list(sets)])[:2]
        if errors[0] == LB_REQ_EMPTY_AGGREGATE:
            raise EmptyAggregateError("EMPTY_AGGREGATE_ARRAY")  # getAggregatedPubkey throws (singleThread.ts:20-24)
        if errors[0] != 0:
            raise BadPubkeyError("invalid pubkey encoding")
        dt = time.monotonic() - t0
        pm.observe(M.MAIN_THREAD_TIME, dt)
        pm.observe(M.SINGLE_THREAD_TIME, dt)
        if sets:
            pm.observe(M.SINGLE_THREAD_TIME_PER_SIGSET, dt / len(sets))
        return bool(valid[0])

    async def verify_signature_sets_same_message(self, sets: List[Tuple[PublicKey, bytes]], message: bytes,
                                                 opts: Optional[VerifySignatureOpts] = None) -> List[bool]:
        if len(sets) == 0:  # bls.PublicKey.aggregate([]) throws (singleThread.ts:43)
            raise EmptyAggregateError("EMPTY_AGGREGATE_ARRAY")
        t0 = time.monotonic()
        out = self.backend.verify_same_message([p for p, _ in sets], [s for _, s in sets], message)
        self.pool_metrics.observe(M.MAIN_THREAD_TIME, time.monotonic() - t0)
        return list(out)

    async def close(self) -> None:
        close = getattr(self.backend, "close", None)
        if close:
            close()

    def can_accept_work(self) -> bool:
        return True  # blocking verification: no throttle (singleThread.ts:84-88)
