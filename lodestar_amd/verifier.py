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
import enum
import os
import threading
import time
from collections import deque
from dataclasses import dataclass, field
from typing import Callable, Deque, List, Optional, Sequence, Tuple, Union

import numpy as np

from . import metrics as M
from .native import (LB_REQ_BAD_PUBKEY, LB_REQ_EMPTY_AGGREGATE, BadPubkeyError, Device, EmptyAggregateError,
                     pack_blobs)

MAX_SIGNATURE_SETS_PER_JOB = 128      # index.ts:57
MAX_BUFFERED_SIGS = 32                # index.ts:66
MAX_BUFFER_WAIT_MS = 100              # index.ts:75
MAX_JOBS_CAN_ACCEPT_WORK = 512        # index.ts:80


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


class DeviceBackend:
    """Thin adapter: jobs -> one lb_verify_requests call per package."""

    def __init__(self, device: int = 0, seed_source: Callable[[], bytes] = lambda: os.urandom(32)):
        self.dev = Device(device)
        self.seed_source = seed_source
        self.lock = threading.Lock()

    def sync_pubkeys(self, pubkeys: Sequence[bytes]) -> int:
        """syncPubkeys (pubkeyCache.ts:56-77): append validators' keys (48-byte
        compressed, as the state holds them) to the device table; returns its size."""
        with self.lock:
            return self.dev.pubkey_table_append(list(pubkeys))

    def verify_requests(self, requests: List[List[SignatureSet]]) -> Tuple[List[bool], List[int]]:
        keys_all, pk_off, msgs, sigs, req_off = [], [0], [], [], [0]
        for req in requests:
            for s in req:
                keys = [s.pubkey] if s.type == SignatureSetType.single else (s.pubkeys or [])
                keys_all.extend(keys)
                pk_off.append(len(keys_all))
                msgs.append(bytes(s.signing_root))
                sigs.append(bytes(s.signature))
            req_off.append(len(msgs))
        blob, offs = pack_blobs(sigs)
        # validator indices when every key has one (device table), else the encodings
        by_index = bool(keys_all) and all(k.index is not None for k in keys_all)
        idx = np.array([k.index for k in keys_all], np.uint32) if by_index else None
        with self.lock:
            pks = None if by_index else np.frombuffer(b"".join(self._key_bytes(keys_all)) or b"\0", np.uint8)
            res = self.dev.verify_requests(np.array(req_off, np.uint32), pks, np.array(pk_off, np.uint32),
                                           np.frombuffer(b"".join(msgs) or b"\0", np.uint8), blob, offs,
                                           self.seed_source(), pk_indices=idx)
        self.last_stats = (res.batch_retries, res.batch_sigs_success)
        return [bool(v) for v in res.valid], [int(e) for e in res.errors]

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

    def verify_same_message(self, pubkeys: Sequence[PublicKey], signatures: Sequence[bytes],
                            message: bytes) -> List[bool]:
        with self.lock:
            out, _ = self.dev.verify_same_message(self._key_bytes(pubkeys), list(signatures), message,
                                                  self.seed_source())
        return out

    def close(self):
        self.dev.close()


class BlsGpuVerifier:
    """IBlsVerifier over one or more GPUs (one backend per GPU)."""

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
        self._idle = list(range(len(self.backends)))
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
        if opts.verify_on_main_thread and not self.verify_all_multi_thread:
            # synchronous, on the caller's thread (index.ts:174-187)
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
        loop = self._get_loop()
        futs = []
        for chunk in chunkify_maximize_chunk_size(sets, MAX_SIGNATURE_SETS_PER_JOB):
            fut = loop.create_future()
            self._queue(_Job(JobType.same_message, fut, opts, chunk, message=bytes(message)))
            futs.append(fut)
        results = await asyncio.gather(*futs)
        return [v for r in results for v in r]

    async def close(self) -> None:
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
        for b in self.backends:
            close = getattr(b, "close", None)
            if close:
                close()

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
        bi = self._idle.pop()
        self.metrics["dispatches"] += 1
        self.metrics["jobs_started"] += len(jobs)
        pm, now = self.pool_metrics, time.monotonic()
        pm.inc(M.JOB_GROUPS_STARTED)  # index.ts:433-437
        for t in (JobType.default, JobType.same_message):
            pm.inc(M.JOBS_STARTED, sum(1 for j in jobs if j.type == t), type=t.value)
            pm.inc(M.SIG_SETS_STARTED, sum(len(j.sets) for j in jobs if j.type == t), type=t.value)
        for j in jobs:
            pm.observe(M.JOB_WAIT_TIME, now - j.added)  # index.ts:396
        pm.set(M.WORKERS_BUSY, len(self.backends) - len(self._idle))
        pm.set(M.QUEUE_LENGTH, len(self._jobs))
        loop = self._get_loop()
        task = loop.run_in_executor(None, self._execute, bi, jobs)
        task.add_done_callback(lambda f, bi=bi, jobs=jobs: self._on_done(f, bi, jobs))

    def _execute(self, bi: int, jobs: List[_Job]):
        """Runs on an executor thread (the event loop never blocks on the GPU)."""
        backend = self.backends[bi]
        t0 = time.monotonic()
        out = [None] * len(jobs)
        default_idx = [i for i, j in enumerate(jobs) if j.type == JobType.default]
        if default_idx:
            valid, errors = backend.verify_requests([jobs[i].sets for i in default_idx])
            for k, i in enumerate(default_idx):
                out[i] = ("ok", valid[k]) if errors[k] == 0 else ("err", errors[k])
        for i, j in enumerate(jobs):
            if j.type == JobType.same_message:
                out[i] = ("same", backend.verify_same_message([p for p, _ in j.sets], [s for _, s in j.sets],
                                                              j.message))
        stats = getattr(backend, "last_stats", (0, 0)) if default_idx else (0, 0)
        return out, time.monotonic() - t0, stats

    def _on_done(self, fut, bi: int, jobs: List[_Job]) -> None:
        self._idle.append(bi)
        pm = self.pool_metrics
        pm.set(M.WORKERS_BUSY, len(self.backends) - len(self._idle))
        try:
            results, elapsed, (retries, sigs_ok) = fut.result()
        except Exception as e:  # device failure rejects every job of the package (index.ts:503-512)
            for job in jobs:
                if not job.future.done():
                    job.future.set_exception(e)
            self._get_loop().call_soon(self._run_job)
            return
        # index.ts:495-502 (workerId = the GPU backend)
        started = sum(len(j.sets) for j in jobs)
        pm.inc(M.JOBS_WORKER_TIME, elapsed, workerId=bi)
        if started:
            pm.observe(M.TIME_PER_SIG_SET, elapsed / started)
        pm.inc(M.SUCCESS_JOBS_SETS, sum(j.sig_sets() for j, (k, _) in zip(jobs, results) if k != "err"))
        pm.inc(M.ERROR_JOBS_SETS, sum(j.sig_sets() for j, (k, _) in zip(jobs, results) if k == "err"))
        pm.inc(M.BATCH_RETRIES, retries)
        pm.inc(M.BATCH_SIGS_SUCCESS, sigs_ok)
        for job, (kind, val) in zip(jobs, results):
            if job.future.done():
                continue
            if kind == "ok":
                job.future.set_result(bool(val))
            elif kind == "err":
                if val == LB_REQ_EMPTY_AGGREGATE:  # index.ts:403-409
                    pm.inc(M.ERROR_AGGREGATE_SETS, len(job.sets), type=job.type.value)
                err = EmptyAggregateError("EMPTY_AGGREGATE_ARRAY") if val == LB_REQ_EMPTY_AGGREGATE else \
                    BadPubkeyError("invalid pubkey encoding") if val == LB_REQ_BAD_PUBKEY else RuntimeError(str(val))
                job.future.set_exception(err)
            else:
                verdicts = list(val)
                if not all(verdicts):
                    self.metrics["same_message_retry_jobs"] += 1
                    self.metrics["same_message_retry_sets"] += len(job.sets)
                    pm.inc(M.SAME_MESSAGE_RETRY_JOBS)  # index.ts:566-567
                    pm.inc(M.SAME_MESSAGE_RETRY_SETS, len(job.sets))
                job.future.set_result(verdicts)
        self._get_loop().call_soon(self._run_job)

    def _verify_now(self, sets: List[SignatureSet]) -> bool:
        valid, errors = self.backends[0].verify_requests([sets])
        if errors[0] == LB_REQ_EMPTY_AGGREGATE:
            raise EmptyAggregateError("EMPTY_AGGREGATE_ARRAY")
        if errors[0] != 0:
            raise BadPubkeyError("invalid pubkey encoding")
        return valid[0]
