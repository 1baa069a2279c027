"""ctypes binding of ``liblodestar_bls.so`` (the C ABI in include/lodestar_bls.h).

The product path has no CPU fallback: if the HIP library is missing or no
GPU is visible, constructing :class:`Device` raises.  (The CPU checker lives in
``oracle/`` and is only ever used by tests and the bench's cpu_baseline leg.)
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

_LIB_NAME = "liblodestar_bls.so"
_HERE = os.path.dirname(os.path.abspath(__file__))

LB_OK = 0
LB_ERR_INVALID_ARGUMENT = -1
LB_ERR_DEVICE = -2
LB_ERR_NO_DEVICE = -3
LB_ERR_OUT_OF_MEMORY = -4

LB_REQ_OK = 0
LB_REQ_EMPTY_AGGREGATE = 1
LB_REQ_BAD_PUBKEY = 2

SET_STATUS_NAMES = {0: "OK", 1: "BAD_ENCODING", 2: "NOT_ON_CURVE", 3: "NOT_IN_GROUP", 4: "PK_INFINITY",
                    5: "EMPTY_AGGREGATE", 6: "ZERO_SIGNATURE"}

# Every symbol include/lodestar_bls.h declares (checked by tests/test_capi_symbols.py)
EXPORTED_SYMBOLS = (
    "lb_create", "lb_destroy", "lb_last_error", "lb_slots", "lb_device_count", "lb_verify_requests",
    "lb_verify_requests_device", "lb_verify_same_message", "lb_aggregate_pubkeys", "lb_aggregate_signatures",
    "lb_hash_to_g2", "lb_decode_signatures", "lb_pairing", "lb_batch_scalars", "lb_g1_mul", "lb_g2_mul", "lb_g2_msm", "lb_verify_same_message_batch_async",
    "lb_last_stage_times", "lb_sk_to_pk", "lb_sign", "lb_verify_requests_device_async", "lb_wait",
    "lb_pubkey_table_append", "lb_pubkey_table_size", "lb_pubkey_table_read", "lb_pubkey_table_truncate",
    "lb_aggregate_pubkeys_indexed", "lb_signing_roots_attestation", "lb_signing_roots_chunks",
    "lb_signing_roots_attestation_device", "lb_verify_requests_async", "lb_verify_requests_partial_async",
    "lb_partial_wait", "lb_gt_check", "lb_verify_requests_finish", "lb_verify_same_message_batch",
    "lb_pubkeys_from_bytes", "lb_poll", "lb_set_latency_path", "lb_lp_program_run", "lb_scratch_per_queue",
    "lb_verify_requests_priority_async", "lb_partial_poll", "lb_hw_queues", "lb_last_call_streams",
    "lb_create_lane", "lb_mark_priority", "lb_last_latency_clocks",
)

LB_BATCH_DEVICE = 1
LB_GT_BYTES = 576
LB_PK_ROW_FLAG = 0x80000000  # mixed packages: an index naming a row of the call's 96-byte pubkeys
LB_PK_ROW48_FLAG = 0x40000000  # ... whose row holds a 48-byte compressed encoding
LB_PK_ROW_MASK = 0x3FFFFFFF


class LodestarBlsError(RuntimeError):
    pass


class EmptyAggregateError(LodestarBlsError):
    """Mirrors @chainsafe/bls EMPTY_AGGREGATE_ARRAY (a rejected job, not a false verdict)."""


class BadPubkeyError(LodestarBlsError):
    """Pubkey bytes PublicKey.fromBytes would throw on (worker.ts:110-116)."""


def library_path() -> str:
    # LB_LIBRARY: an alternative build of the same library (tuning experiments,
    # lodestar_amd/build.py build_variant); never a CPU fallback
    return os.environ.get("LB_LIBRARY") or os.path.join(_HERE, _LIB_NAME)


class _RequestBatch(ctypes.Structure):
    _fields_ = [
        ("n_requests", ctypes.c_uint32),
        ("n_sets", ctypes.c_uint32),
        ("request_offsets", ctypes.c_void_p),
        ("request_batchable", ctypes.c_void_p),
        ("pubkeys", ctypes.c_void_p),
        ("pk_offsets", ctypes.c_void_p),
        ("messages", ctypes.c_void_p),
        ("signatures", ctypes.c_void_p),
        ("sig_offsets", ctypes.c_void_p),
        ("seed", ctypes.c_void_p),
        ("pubkey_indices", ctypes.c_void_p),
    ]


class _SameMessageBatch(ctypes.Structure):
    _fields_ = [
        ("n_jobs", ctypes.c_uint32),
        ("n_sets", ctypes.c_uint32),
        ("job_offsets", ctypes.c_void_p),
        ("pubkeys", ctypes.c_void_p),
        ("pubkey_indices", ctypes.c_void_p),
        ("signatures", ctypes.c_void_p),
        ("sig_offsets", ctypes.c_void_p),
        ("messages", ctypes.c_void_p),
        ("seed", ctypes.c_void_p),
    ]


class _Stats(ctypes.Structure):
    _fields_ = [("batch_retries", ctypes.c_uint32), ("batch_sigs_success", ctypes.c_uint32),
                ("device_ms", ctypes.c_double)]


_lib = None


def load_library() -> ctypes.CDLL:
    """Load the HIP library (raises if it was not built -- no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    path = library_path()
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64, and
    # when /opt/rocm's is loaded first (by this library) torch's HIP
    # initialisation fails later in the same process ("No HIP GPUs are
    # available").  Loading torch first makes both share torch's runtime, the
    # order bench.py and the tests use.
    if os.environ.get("LB_NO_TORCH_PRELOAD") != "1":
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    if not os.path.exists(path):
        raise LodestarBlsError(
            f"{path} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = ctypes.CDLL(path)
    vp, u32, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
    lib.lb_create.argtypes = [i32, ctypes.POINTER(vp)]
    lib.lb_create_lane.argtypes = [i32, ctypes.POINTER(vp)]
    lib.lb_mark_priority.argtypes = [vp]
    lib.lb_last_latency_clocks.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64)]
    lib.lb_destroy.argtypes = [vp]
    lib.lb_last_error.argtypes = [vp]
    lib.lb_last_error.restype = ctypes.c_char_p
    lib.lb_slots.argtypes = [vp]
    lib.lb_hw_queues.argtypes = [vp]
    lib.lb_last_call_streams.argtypes = [vp]
    lib.lb_device_count.argtypes = []
    lib.lb_scratch_per_queue.argtypes = [i32, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(u32)]
    lib.lb_verify_requests.argtypes = [vp, ctypes.POINTER(_RequestBatch), vp, vp, vp, ctypes.POINTER(_Stats)]
    lib.lb_verify_requests_device.argtypes = [vp, ctypes.POINTER(_RequestBatch), vp, vp, vp, ctypes.POINTER(_Stats)]
    lib.lb_verify_same_message.argtypes = [vp, u32, vp, vp, vp, vp, vp, vp, ctypes.POINTER(u32)]
    lib.lb_aggregate_pubkeys.argtypes = [vp, u32, vp, vp, vp]
    lib.lb_aggregate_signatures.argtypes = [vp, u32, vp, vp, vp, ctypes.POINTER(ctypes.c_int32)]
    lib.lb_hash_to_g2.argtypes = [vp, u32, vp, vp]
    lib.lb_decode_signatures.argtypes = [vp, u32, vp, vp, vp, vp]
    lib.lb_pairing.argtypes = [vp, u32, vp, vp, vp]
    lib.lb_batch_scalars.argtypes = [vp, vp, u32, u32, vp]
    lib.lb_g1_mul.argtypes = [vp, u32, vp, vp, vp]
    lib.lb_g2_mul.argtypes = [vp, u32, vp, vp, vp]
    lib.lb_g2_msm.argtypes = [vp, u32, vp, vp, vp]
    lib.lb_verify_requests_device_async.argtypes = [vp, ctypes.POINTER(_RequestBatch), vp, vp, vp,
                                                    ctypes.POINTER(ctypes.c_uint64)]
    lib.lb_wait.argtypes = [vp, ctypes.c_uint64, ctypes.POINTER(_Stats)]
    lib.lb_poll.argtypes = [vp, ctypes.c_uint64, ctypes.POINTER(ctypes.c_int32)]
    lib.lb_verify_requests_async.argtypes = [vp, ctypes.POINTER(_RequestBatch), vp, vp, vp,
                                             ctypes.POINTER(ctypes.c_uint64)]
    lib.lb_partial_poll.argtypes = [vp, ctypes.c_uint64, ctypes.POINTER(ctypes.c_int32)]
    lib.lb_verify_requests_priority_async.argtypes = [vp, ctypes.POINTER(_RequestBatch), vp, vp, vp,
                                                      ctypes.POINTER(ctypes.c_uint64)]
    lib.lb_verify_requests_partial_async.argtypes = [vp, ctypes.POINTER(_RequestBatch), u32, vp, vp, vp,
                                                     ctypes.POINTER(ctypes.c_uint64)]
    lib.lb_partial_wait.argtypes = [vp, ctypes.c_uint64, vp]
    lib.lb_gt_check.argtypes = [vp, u32, vp, ctypes.POINTER(ctypes.c_int32)]
    lib.lb_verify_requests_finish.argtypes = [vp, ctypes.c_uint64, i32]
    lib.lb_verify_same_message_batch.argtypes = [vp, ctypes.POINTER(_SameMessageBatch), vp, vp,
                                                 ctypes.POINTER(_Stats)]
    lib.lb_verify_same_message_batch_async.argtypes = [vp, ctypes.POINTER(_SameMessageBatch), vp, vp,
                                                       ctypes.POINTER(ctypes.c_uint64)]
    lib.lb_sk_to_pk.argtypes = [vp, u32, vp, vp]
    lib.lb_pubkey_table_append.argtypes = [vp, u32, vp, u32, ctypes.POINTER(ctypes.c_int32)]
    lib.lb_pubkeys_from_bytes.argtypes = [vp, u32, vp, u32, vp, vp]
    lib.lb_pubkey_table_size.argtypes = [vp, ctypes.POINTER(u32)]
    lib.lb_pubkey_table_read.argtypes = [vp, u32, u32, vp]
    lib.lb_pubkey_table_truncate.argtypes = [vp, u32]
    lib.lb_aggregate_pubkeys_indexed.argtypes = [vp, u32, vp, vp, vp]
    lib.lb_signing_roots_attestation.argtypes = [vp, u32, vp, vp, u32, vp]
    lib.lb_signing_roots_chunks.argtypes = [vp, u32, u32, vp, vp, u32, vp]
    lib.lb_signing_roots_attestation_device.argtypes = [vp, u32, vp, vp, u32, vp]
    lib.lb_sign.argtypes = [vp, u32, vp, vp, vp]
    lib.lb_last_stage_times.argtypes = [vp, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_char_p), i32]
    lib.lb_set_latency_path.argtypes = [vp, u32]
    lib.lb_lp_program_run.argtypes = [vp, u32, vp, ctypes.c_size_t, u32, vp, vp, vp, vp, ctypes.POINTER(ctypes.c_float),
                                      vp]
    for name in EXPORTED_SYMBOLS:
        getattr(lib, name).restype = getattr(lib, name).restype or ctypes.c_int
    _lib = lib
    return lib


def _ptr(a: Optional[np.ndarray]) -> Optional[int]:
    return None if a is None else a.ctypes.data


def _u8(b) -> np.ndarray:
    if isinstance(b, np.ndarray):
        return np.ascontiguousarray(b, dtype=np.uint8)
    return np.frombuffer(bytes(b), dtype=np.uint8).copy()


def pack_blobs(items: Sequence[bytes]) -> Tuple[np.ndarray, np.ndarray]:
    """Concatenate variable-length byte strings -> (blob, offsets[n+1])."""
    offs = np.zeros(len(items) + 1, dtype=np.uint32)
    if len(items):
        offs[1:] = np.cumsum(np.fromiter((len(x) for x in items), dtype=np.uint64, count=len(items)))
    total = int(offs[-1])
    if not total:
        return np.zeros(1, np.uint8), offs
    try:
        joined = b"".join(items)  # bytes-like items: no per-item copy
    except TypeError:
        joined = b"".join(bytes(x) for x in items)
    return np.frombuffer(joined, dtype=np.uint8).copy(), offs


@dataclass
class VerifyResult:
    valid: np.ndarray          # uint8 per request
    errors: np.ndarray         # uint8 per request (LB_REQ_*)
    set_status: np.ndarray     # uint8 per set (LB_SET_*)
    device_ms: float
    batch_retries: int = 0     # worker.ts:80 (merged check failed -> per-request re-verification)
    batch_sigs_success: int = 0  # worker.ts:71 (sets verified inside a passing merged check)


@dataclass
class PendingCall:
    """An enqueued host-buffer call: its ticket, the output arrays the library
    fills when the call retires and the input arrays it reads until then."""
    ticket: int
    n_req: int
    n_sets: int
    valid: np.ndarray
    err: np.ndarray
    sst: np.ndarray
    keep: object
    partial: bool = False


@dataclass
class PendingSameMessage:
    """An enqueued same-message package: its ticket, the verdict / fast-path arrays
    the library fills when it retires, and the inputs it reads until then."""
    ticket: int
    n_jobs: int
    out: np.ndarray
    fast: np.ndarray
    job_off: np.ndarray
    keep: object


class Device:
    """One lb_ctx bound to one GPU (one per process per GPU)."""

    def __init__(self, device: int = 0):
        self.lib = load_library()
        h = ctypes.c_void_p()
        rc = self.lib.lb_create(device, ctypes.byref(h))
        if rc != LB_OK:
            msg = self.lib.lb_last_error(None).decode(errors="replace")
            raise LodestarBlsError(f"lb_create({device}) failed with {rc}: {msg}")
        self._h = h
        self.device = device

    # -- lifecycle ---------------------------------------------------------
    def slots(self) -> int:
        """Calls the library keeps in flight (lb_slots: one per HIP hardware queue)."""
        return int(self.lib.lb_slots(self._h))

    def hw_queues(self) -> int:
        """HIP hardware queues this context opens (lb_hw_queues, priced by lb_create)."""
        return int(self.lib.lb_hw_queues(self._h))

    def last_latency_clocks(self):
        """(kernel ms by s_memrealtime at 100 MHz, shader clock MHz) of the last latency-path call"""
        c = (ctypes.c_uint64 * 4)()
        self._check(self.lib.lb_last_latency_clocks(self._h, c), "lb_last_latency_clocks")
        rt = c[2] - c[0]
        return (rt / 1e5, (c[3] - c[1]) / rt * 100.0) if rt > 0 and c[2] >= c[0] else (None, None)

    def last_call_streams(self) -> int:
        """Distinct streams of the last submitted verify call (2 = the two-stream DAG)."""
        return int(self.lib.lb_last_call_streams(self._h))

    def close(self) -> None:
        if self._h:
            self.lib.lb_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int, what: str) -> None:
        if rc != LB_OK:
            msg = self.lib.lb_last_error(self._h).decode(errors="replace")
            raise LodestarBlsError(f"{what} failed ({rc}): {msg}")

    # -- hot path ------------------------------------------------------------
    @staticmethod
    def _host_batch(request_offsets, pubkeys, pk_offsets, messages, sig_blob, sig_offsets, seed, batchable=None,
                    pk_indices=None):
        """(batch struct, arrays it points into, n_req, n_sets) for a host-buffer call."""
        request_offsets = np.ascontiguousarray(request_offsets, dtype=np.uint32)
        n_req = len(request_offsets) - 1
        n_sets = int(request_offsets[-1]) if n_req >= 0 else 0
        pubkeys = _u8(pubkeys) if pubkeys is not None and len(pubkeys) else np.zeros(1, np.uint8)
        messages = _u8(messages) if len(messages) else np.zeros(1, np.uint8)
        if len(messages) < 32 * n_sets:
            raise ValueError(f"messages: {len(messages)} bytes for {n_sets} sets (32 bytes each)")
        sig_blob = _u8(sig_blob) if len(sig_blob) else np.zeros(1, np.uint8)
        sig_offsets = np.ascontiguousarray(sig_offsets, dtype=np.uint32)
        if len(sig_offsets) != n_sets + 1:
            raise ValueError("sig_offsets must have n_sets + 1 entries")
        pk_offsets = None if pk_offsets is None else np.ascontiguousarray(pk_offsets, dtype=np.uint32)
        if batchable is not None:
            batchable = np.ascontiguousarray(batchable, dtype=np.uint8)
        seed_a = _u8(seed)
        if len(seed_a) != 32:
            raise ValueError("seed must be 32 bytes")
        if pk_indices is not None:
            pk_indices = np.ascontiguousarray(pk_indices, dtype=np.uint32)
            if len(pk_indices) == 0:
                pk_indices = np.zeros(1, np.uint32)
        b = _RequestBatch(n_req, n_sets, _ptr(request_offsets), _ptr(batchable), _ptr(pubkeys), _ptr(pk_offsets),
                          _ptr(messages), _ptr(sig_blob), _ptr(sig_offsets), _ptr(seed_a), _ptr(pk_indices))
        keep = (request_offsets, pubkeys, messages, sig_blob, sig_offsets, pk_offsets, batchable, seed_a, pk_indices)
        return b, keep, n_req, n_sets

    def verify_requests(self, request_offsets: np.ndarray, pubkeys: np.ndarray, pk_offsets: Optional[np.ndarray],
                        messages: np.ndarray, sig_blob: np.ndarray, sig_offsets: np.ndarray, seed: bytes,
                        batchable: Optional[np.ndarray] = None,
                        pk_indices: Optional[np.ndarray] = None) -> VerifyResult:
        """pk_indices (u32 validator indices into the device pubkey table) replaces pubkeys when given."""
        b, keep, n_req, n_sets = self._host_batch(request_offsets, pubkeys, pk_offsets, messages, sig_blob,
                                                  sig_offsets, seed, batchable, pk_indices)
        valid = np.zeros(max(n_req, 1), np.uint8)
        err = np.zeros(max(n_req, 1), np.uint8)
        sst = np.zeros(max(n_sets, 1), np.uint8)
        st = _Stats()
        rc = self.lib.lb_verify_requests(self._h, ctypes.byref(b), _ptr(valid), _ptr(err), _ptr(sst), ctypes.byref(st))
        self._check(rc, "lb_verify_requests")
        del keep
        return VerifyResult(valid[:n_req], err[:n_req], sst[:n_sets], st.device_ms, int(st.batch_retries),
                            int(st.batch_sigs_success))

    def verify_requests_async(self, request_offsets, pubkeys, pk_offsets, messages, sig_blob, sig_offsets, seed,
                              batchable=None, pk_indices=None, partial: bool = False,
                              priority: bool = False) -> "PendingCall":
        """lb_verify_requests_async (or the two-phase lb_verify_requests_partial_async,
        or with priority=True the priority lane, lb_verify_requests_priority_async):
        enqueue and return at once; wait_call() gives the verdicts."""
        if partial and priority:
            raise ValueError("a two-phase call cannot take the priority lane")
        b, keep, n_req, n_sets = self._host_batch(request_offsets, pubkeys, pk_offsets, messages, sig_blob,
                                                  sig_offsets, seed, batchable, pk_indices)
        pc = PendingCall(0, n_req, n_sets, np.zeros(max(n_req, 1), np.uint8), np.zeros(max(n_req, 1), np.uint8),
                         np.zeros(max(n_sets, 1), np.uint8), keep, partial)
        t = ctypes.c_uint64(0)
        if partial:
            rc = self.lib.lb_verify_requests_partial_async(self._h, ctypes.byref(b), 0, _ptr(pc.valid), _ptr(pc.err),
                                                           _ptr(pc.sst), ctypes.byref(t))
            self._check(rc, "lb_verify_requests_partial_async")
        else:
            fn = self.lib.lb_verify_requests_priority_async if priority else self.lib.lb_verify_requests_async
            rc = fn(self._h, ctypes.byref(b), _ptr(pc.valid), _ptr(pc.err), _ptr(pc.sst), ctypes.byref(t))
            self._check(rc, "lb_verify_requests_priority_async" if priority else "lb_verify_requests_async")
        pc.ticket = int(t.value)
        return pc

    def wait_call(self, pc: "PendingCall") -> VerifyResult:
        st = _Stats()
        self._check(self.lib.lb_wait(self._h, pc.ticket, ctypes.byref(st)), "lb_wait")
        pc.keep = None
        return VerifyResult(pc.valid[:pc.n_req], pc.err[:pc.n_req], pc.sst[:pc.n_sets], st.device_ms,
                            int(st.batch_retries), int(st.batch_sigs_success))

    # -- multi-GPU combine (two-phase calls) ----------------------------
    def partial_wait(self, pc: "PendingCall") -> bytes:
        """The shard's merged Miller product (576 bytes) once it is ready."""
        return self.partial_wait_t(pc.ticket)

    def verify_finish(self, pc: "PendingCall", merged_ok: bool) -> None:
        self.finish_t(pc.ticket, merged_ok)

    def gt_check(self, partials: Sequence[bytes]) -> bool:
        """final_exp(prod of the partials) == 1 (the host-side combine, run on this GPU)."""
        if any(len(p) != LB_GT_BYTES for p in partials):
            raise ValueError("partials are 576 bytes each")
        blob = _u8(b"".join(partials)) if partials else np.zeros(1, np.uint8)
        out = ctypes.c_int32(0)
        self._check(self.lib.lb_gt_check(self._h, len(partials), _ptr(blob), ctypes.byref(out)), "lb_gt_check")
        return bool(out.value)

    def _same_message_batch(self, jobs, seed: bytes, by_index: bool, rows=None):
        """The lb_same_message_batch of a package, its output arrays and the
        input arrays the library reads (kept alive until the call retires).  rows (with
        by_index): a mixed package's 96-byte key rows, named by LB_PK_ROW_FLAG indices."""
        nj = len(jobs)
        job_off = np.zeros(nj + 1, np.uint32)
        for j, (pks, sigs, msg) in enumerate(jobs):
            if len(pks) != len(sigs):
                raise ValueError("one signature per pubkey")
            if len(msg) != 32:
                raise ValueError("signing root must be 32 bytes")
            job_off[j + 1] = job_off[j] + len(pks)
        ns = int(job_off[-1])
        blob, offs = pack_blobs([s for _, sigs, _ in jobs for s in sigs])
        msgs = _u8(b"".join(bytes(m) for _, _, m in jobs))
        if by_index:
            idx = (np.concatenate([np.asarray(pks, dtype=np.uint32).reshape(-1) for pks, _, _ in jobs])
                   if ns else np.zeros(1, np.uint32))
            pk = _u8(rows) if rows is not None else None
        else:
            pk = _u8(b"".join(bytes(k) for pks, _, _ in jobs for k in pks) or b"\0")
            idx = None
        sd = _u8(seed)
        b = _SameMessageBatch(nj, ns, _ptr(job_off), _ptr(pk), _ptr(idx), _ptr(blob), _ptr(offs), _ptr(msgs),
                              _ptr(sd))
        out = np.zeros(max(ns, 1), np.uint8)
        fast = np.zeros(max(nj, 1), np.uint8)
        return b, out, fast, job_off, (job_off, pk, idx, blob, offs, msgs, sd)

    @staticmethod
    def _same_message_result(out, fast, job_off, nj, st):
        ns = int(job_off[-1])
        flat = out[:ns].astype(bool).tolist()
        bounds = job_off.tolist()
        res = [flat[bounds[j]:bounds[j + 1]] for j in range(nj)]
        return res, fast[:nj].astype(bool).tolist(), (int(st.batch_retries), int(st.batch_sigs_success))

    def verify_same_message_batch(self, jobs: Sequence[Tuple[Sequence, Sequence[bytes], bytes]], seed: bytes,
                                  by_index: bool = False,
                                  rows=None) -> Tuple[List[List[bool]], List[bool], Tuple[int, int]]:
        """jobs: (pubkeys, signatures, message) per same-message job; pubkeys are
        96-byte encodings, or validator indices when by_index.  Returns per-set
        verdicts per job, the per-job fast-path flags and (retried jobs, sets
        verified by a passing aggregate)."""
        nj = len(jobs)
        if nj == 0:
            return [], [], (0, 0)
        b, out, fast, job_off, keep = self._same_message_batch(jobs, seed, by_index, rows)
        st = _Stats()
        rc = self.lib.lb_verify_same_message_batch(self._h, ctypes.byref(b), _ptr(out), _ptr(fast), ctypes.byref(st))
        self._check(rc, "lb_verify_same_message_batch")
        del keep
        return self._same_message_result(out, fast, job_off, nj, st)

    def verify_same_message_batch_async(self, jobs: Sequence[Tuple[Sequence, Sequence[bytes], bytes]], seed: bytes,
                                        by_index: bool = False) -> "PendingSameMessage":
        """lb_verify_same_message_batch_async: enqueue the package on the next slot of
        the ring of calls in flight and return at once; wait_same_message() gives
        what verify_same_message_batch returns."""
        nj = len(jobs)
        b, out, fast, job_off, keep = self._same_message_batch(jobs, seed, by_index) if nj else (
            _SameMessageBatch(0, 0, None, None, None, None, None, None, None), np.zeros(1, np.uint8),
            np.zeros(1, np.uint8), np.zeros(1, np.uint32), None)
        t = ctypes.c_uint64(0)
        rc = self.lib.lb_verify_same_message_batch_async(self._h, ctypes.byref(b), _ptr(out), _ptr(fast),
                                                         ctypes.byref(t))
        self._check(rc, "lb_verify_same_message_batch_async")
        return PendingSameMessage(int(t.value), nj, out, fast, job_off, keep)

    def prepare_same_message(self, jobs, seed: bytes, by_index: bool = False):
        """A package packed once (bench: the same package resubmitted without re-packing)."""
        return (len(jobs),) + self._same_message_batch(jobs, seed, by_index)

    def verify_same_message_prepared_async(self, prep) -> "PendingSameMessage":
        nj, b, _, _, job_off, keep = prep
        out = np.zeros(max(int(job_off[-1]), 1), np.uint8)
        fast = np.zeros(max(nj, 1), np.uint8)
        t = ctypes.c_uint64(0)
        rc = self.lib.lb_verify_same_message_batch_async(self._h, ctypes.byref(b), _ptr(out), _ptr(fast),
                                                         ctypes.byref(t))
        self._check(rc, "lb_verify_same_message_batch_async")
        return PendingSameMessage(int(t.value), nj, out, fast, job_off, keep)

    def wait_same_message(self, pc: "PendingSameMessage"):
        st = _Stats()
        self._check(self.lib.lb_wait(self._h, pc.ticket, ctypes.byref(st)), "lb_wait")
        pc.keep = None
        res = self._same_message_result(pc.out, pc.fast, pc.job_off, pc.n_jobs, st)
        return res + (float(st.device_ms),)

    def verify_requests_device(self, n_req: int, n_sets: int, d_req_off: int, d_pubkeys: int, d_pk_off: Optional[int],
                               d_msgs: int, d_sigs: int, d_sig_off: int, d_seed: int, d_valid: int, d_err: int,
                               d_set_status: Optional[int] = None, d_pk_idx: Optional[int] = None) -> float:
        """All arguments are device pointers (ints).  Returns device_ms."""
        b = _RequestBatch(n_req, n_sets, d_req_off, None, d_pubkeys, d_pk_off, d_msgs, d_sigs, d_sig_off, d_seed,
                          d_pk_idx)
        st = _Stats()
        rc = self.lib.lb_verify_requests_device(self._h, ctypes.byref(b), d_valid, d_err, d_set_status,
                                                ctypes.byref(st))
        self._check(rc, "lb_verify_requests_device")
        return st.device_ms

    def verify_requests_device_async(self, n_req: int, n_sets: int, d_req_off: int, d_pubkeys: int,
                                     d_pk_off: Optional[int], d_msgs: int, d_sigs: int, d_sig_off: int, d_seed: int,
                                     d_valid: int, d_err: int, d_set_status: Optional[int] = None,
                                     d_pk_idx: Optional[int] = None, partial: bool = False) -> int:
        """Enqueue; returns a ticket for wait().  All arguments are device pointers.
        partial=True: the two-phase call (partial_wait_t / finish_t before wait)."""
        b = _RequestBatch(n_req, n_sets, d_req_off, None, d_pubkeys, d_pk_off, d_msgs, d_sigs, d_sig_off, d_seed,
                          d_pk_idx)
        t = ctypes.c_uint64(0)
        if partial:
            rc = self.lib.lb_verify_requests_partial_async(self._h, ctypes.byref(b), LB_BATCH_DEVICE, d_valid, d_err,
                                                           d_set_status, ctypes.byref(t))
            self._check(rc, "lb_verify_requests_partial_async")
        else:
            rc = self.lib.lb_verify_requests_device_async(self._h, ctypes.byref(b), d_valid, d_err, d_set_status,
                                                          ctypes.byref(t))
            self._check(rc, "lb_verify_requests_device_async")
        return int(t.value)

    def partial_wait_t(self, ticket: int) -> bytes:
        out = np.zeros(LB_GT_BYTES, np.uint8)
        self._check(self.lib.lb_partial_wait(self._h, ticket, _ptr(out)), "lb_partial_wait")
        return out.tobytes()

    def partial_ready(self, ticket: int) -> bool:
        """True when partial_wait_t(ticket) would return at once (lb_partial_poll)."""
        r = ctypes.c_int32(0)
        self._check(self.lib.lb_partial_poll(self._h, ticket, ctypes.byref(r)), "lb_partial_poll")
        return bool(r.value)

    def finish_t(self, ticket: int, merged_ok: bool) -> None:
        self._check(self.lib.lb_verify_requests_finish(self._h, ticket, 1 if merged_ok else 0),
                    "lb_verify_requests_finish")

    def poll(self, ticket: int) -> bool:
        """True when wait(ticket) would return without blocking (lb_poll)."""
        done = ctypes.c_int32(0)
        self._check(self.lib.lb_poll(self._h, ticket, ctypes.byref(done)), "lb_poll")
        return bool(done.value)

    def wait(self, ticket: int) -> float:
        """lb_wait on a ticket; returns device_ms (the call's stats in self.last_stats)."""
        st = _Stats()
        self._check(self.lib.lb_wait(self._h, ticket, ctypes.byref(st)), "lb_wait")
        self.last_stats = (int(st.batch_retries), int(st.batch_sigs_success))
        return st.device_ms

    def verify_same_message(self, pubkeys: Sequence[bytes], signatures: Sequence[bytes], message: bytes,
                            seed: bytes) -> Tuple[List[bool], bool]:
        n = len(pubkeys)
        if n == 0:
            return [], False
        pk = _u8(b"".join(pubkeys))
        blob, offs = pack_blobs(signatures)
        msg = _u8(message)
        sd = _u8(seed)
        out = np.zeros(n, np.uint8)
        fast = ctypes.c_uint32(0)
        rc = self.lib.lb_verify_same_message(self._h, n, _ptr(pk), _ptr(blob), _ptr(offs), _ptr(msg), _ptr(sd),
                                             _ptr(out), ctypes.byref(fast))
        self._check(rc, "lb_verify_same_message")
        return [bool(x) for x in out], bool(fast.value)

    def aggregate_pubkeys(self, pubkeys: Sequence[bytes]) -> bytes:
        if len(pubkeys) == 0:
            raise EmptyAggregateError("EMPTY_AGGREGATE_ARRAY")
        pk = _u8(b"".join(pubkeys))
        out = np.zeros(96, np.uint8)
        st = np.zeros(1, np.uint8)
        rc = self.lib.lb_aggregate_pubkeys(self._h, len(pubkeys), _ptr(pk), _ptr(out), _ptr(st))
        self._check(rc, "lb_aggregate_pubkeys")
        if st[0] != 0:
            raise BadPubkeyError(SET_STATUS_NAMES.get(int(st[0]), str(st[0])))
        return out.tobytes()

    def aggregate_signatures(self, signatures: Sequence[bytes]) -> Tuple[bytes, int]:
        if len(signatures) == 0:
            raise EmptyAggregateError("EMPTY_AGGREGATE_ARRAY")
        blob, offs = pack_blobs(signatures)
        out = np.zeros(192, np.uint8)
        bad = ctypes.c_int32(-1)
        rc = self.lib.lb_aggregate_signatures(self._h, len(signatures), _ptr(blob), _ptr(offs), _ptr(out),
                                              ctypes.byref(bad))
        self._check(rc, "lb_aggregate_signatures")
        return out.tobytes(), int(bad.value)

    def pubkeys_from_bytes(self, pubkeys: Sequence[bytes]) -> Tuple[List[bytes], List[int]]:
        """PublicKey.fromBytes(b, affine, validate=true) on the GPU for keys of one length
        (48 or 96): (96-byte uncompressed encodings, per-key status; 0 = valid)."""
        n = len(pubkeys)
        if n == 0:
            return [], []
        pk_len = len(pubkeys[0])
        if pk_len not in (48, 96) or any(len(p) != pk_len for p in pubkeys):
            raise ValueError("pubkeys_from_bytes expects keys of one encoding length (48 or 96)")
        blob = _u8(b"".join(pubkeys))
        out = np.zeros(n * 96, np.uint8)
        st = np.zeros(n, np.uint8)
        self._check(self.lib.lb_pubkeys_from_bytes(self._h, n, _ptr(blob), pk_len, _ptr(out), _ptr(st)),
                    "lb_pubkeys_from_bytes")
        return [out[i * 96:(i + 1) * 96].tobytes() for i in range(n)], [int(x) for x in st]

    # -- device-resident pubkey table (index2pubkey mirror) -------------------------
    def pubkey_table_append(self, pubkeys: Sequence[bytes]) -> int:
        """syncPubkeys: append keys (all 48-byte compressed or all 96-byte uncompressed);
        returns the new table size.  Raises BadPubkeyError(index) if one fails to decode."""
        n = len(pubkeys)
        if n == 0:
            return self.pubkey_table_size()
        pk_len = len(pubkeys[0])
        if any(len(p) != pk_len for p in pubkeys):
            raise ValueError("pubkey_table_append expects keys of one encoding length")
        blob = _u8(b"".join(pubkeys))
        bad = ctypes.c_int32(-1)
        rc = self.lib.lb_pubkey_table_append(self._h, n, _ptr(blob), pk_len, ctypes.byref(bad))
        if rc == LB_ERR_INVALID_ARGUMENT and bad.value >= 0:
            raise BadPubkeyError(f"pubkey {bad.value} fails to decode")
        self._check(rc, "lb_pubkey_table_append")
        return self.pubkey_table_size()

    def pubkey_table_size(self) -> int:
        n = ctypes.c_uint32(0)
        self._check(self.lib.lb_pubkey_table_size(self._h, ctypes.byref(n)), "lb_pubkey_table_size")
        return int(n.value)

    def pubkey_table_read(self, first: int, n: int) -> List[bytes]:
        out = np.zeros(max(n, 1) * 96, np.uint8)
        self._check(self.lib.lb_pubkey_table_read(self._h, first, n, _ptr(out)), "lb_pubkey_table_read")
        return [out[i * 96:(i + 1) * 96].tobytes() for i in range(n)]

    def pubkey_table_truncate(self, n: int) -> None:
        self._check(self.lib.lb_pubkey_table_truncate(self._h, n), "lb_pubkey_table_truncate")

    def aggregate_pubkeys_indexed(self, indices: Sequence[int]) -> bytes:
        if len(indices) == 0:
            raise EmptyAggregateError("EMPTY_AGGREGATE_ARRAY")
        idx = np.ascontiguousarray(indices, dtype=np.uint32)
        out = np.zeros(96, np.uint8)
        st = np.zeros(1, np.uint8)
        rc = self.lib.lb_aggregate_pubkeys_indexed(self._h, len(idx), _ptr(idx), _ptr(out), _ptr(st))
        self._check(rc, "lb_aggregate_pubkeys_indexed")
        if st[0] != 0:
            raise BadPubkeyError(SET_STATUS_NAMES.get(int(st[0]), str(st[0])))
        return out.tobytes()

    # -- signing roots (computeSigningRoot, state-transition/src/util/signingRoot.ts:7-13) --
    def signing_roots_attestation(self, data128: Sequence[bytes], domains) -> List[bytes]:
        """n SSZ AttestationData (128 B each); domains: one 32-byte domain or a list of n."""
        n = len(data128)
        if n == 0:
            return []
        shared = isinstance(domains, (bytes, bytearray))
        dom = _u8(bytes(domains) if shared else b"".join(domains))
        d = _u8(b"".join(data128))
        assert len(d) == 128 * n and len(dom) == (32 if shared else 32 * n)
        out = np.zeros(32 * n, np.uint8)
        self._check(self.lib.lb_signing_roots_attestation(self._h, n, _ptr(d), _ptr(dom), 0 if shared else 32,
                                                          _ptr(out)), "lb_signing_roots_attestation")
        return [out[32 * i:32 * (i + 1)].tobytes() for i in range(n)]

    def signing_roots_attestation_device(self, n: int, d_data: int, d_domains: int, domain_stride: int,
                                         d_out: int) -> None:
        """Device pointers in and out (roots straight into a verify call's messages buffer)."""
        self._check(self.lib.lb_signing_roots_attestation_device(self._h, n, d_data, d_domains, domain_stride, d_out),
                    "lb_signing_roots_attestation_device")

    def signing_roots_chunks(self, field_roots: Sequence[Sequence[bytes]], domains) -> List[bytes]:
        """n objects given as m field roots (32 B each, same m for all)."""
        n = len(field_roots)
        if n == 0:
            return []
        m = len(field_roots[0])
        assert all(len(f) == m for f in field_roots)
        shared = isinstance(domains, (bytes, bytearray))
        dom = _u8(bytes(domains) if shared else b"".join(domains))
        c = _u8(b"".join(b"".join(f) for f in field_roots))
        assert len(c) == 32 * m * n
        out = np.zeros(32 * n, np.uint8)
        self._check(self.lib.lb_signing_roots_chunks(self._h, n, m, _ptr(c), _ptr(dom), 0 if shared else 32,
                                                     _ptr(out)), "lb_signing_roots_chunks")
        return [out[32 * i:32 * (i + 1)].tobytes() for i in range(n)]

    # -- stage-level entry points (parity tests) ---------------------------------
    def hash_to_g2(self, messages: Sequence[bytes]) -> List[bytes]:
        n = len(messages)
        m = _u8(b"".join(messages))
        out = np.zeros(max(n, 1) * 192, np.uint8)
        self._check(self.lib.lb_hash_to_g2(self._h, n, _ptr(m), _ptr(out)), "lb_hash_to_g2")
        return [out[i * 192:(i + 1) * 192].tobytes() for i in range(n)]

    def decode_signatures(self, signatures: Sequence[bytes]) -> Tuple[List[int], List[bytes]]:
        n = len(signatures)
        blob, offs = pack_blobs(signatures)
        st = np.zeros(max(n, 1), np.uint8)
        out = np.zeros(max(n, 1) * 192, np.uint8)
        self._check(self.lib.lb_decode_signatures(self._h, n, _ptr(blob), _ptr(offs), _ptr(st), _ptr(out)),
                    "lb_decode_signatures")
        return [int(x) for x in st[:n]], [out[i * 192:(i + 1) * 192].tobytes() for i in range(n)]

    def decode_signatures_packed(self, blob: np.ndarray, offs: np.ndarray, out: Optional[np.ndarray] = None
                                 ) -> np.ndarray:
        """lb_decode_signatures on an already packed blob (pack_blobs): the per-signature
        statuses (0 = valid: Signature.fromBytes(bytes, affine, validate=true) accepts it);
        the affine points land in `out` (n x 192 bytes) when given."""
        n = len(offs) - 1
        st = np.zeros(max(n, 1), np.uint8)
        if out is None or len(out) < max(n, 1) * 192:
            out = np.zeros(max(n, 1) * 192, np.uint8)
        self._check(self.lib.lb_decode_signatures(self._h, n, _ptr(blob), _ptr(offs), _ptr(st), _ptr(out)),
                    "lb_decode_signatures")
        return st[:n]

    def pairing(self, g1s: Sequence[bytes], g2s: Sequence[bytes]) -> List[bytes]:
        n = len(g1s)
        a = _u8(b"".join(g1s))
        b = _u8(b"".join(g2s))
        out = np.zeros(max(n, 1) * 576, np.uint8)
        self._check(self.lib.lb_pairing(self._h, n, _ptr(a), _ptr(b), _ptr(out)), "lb_pairing")
        return [out[i * 576:(i + 1) * 576].tobytes() for i in range(n)]

    def batch_scalars(self, seed: bytes, first: int, n: int) -> List[int]:
        sd = _u8(seed)
        out = np.zeros(max(n, 1), np.uint64)
        self._check(self.lib.lb_batch_scalars(self._h, _ptr(sd), first, n, _ptr(out)), "lb_batch_scalars")
        return [int(x) for x in out[:n]]

    def g1_mul(self, pts: Sequence[bytes], ks: Sequence[int]) -> List[bytes]:
        n = len(pts)
        a = _u8(b"".join(pts))
        k = np.array(ks, dtype=np.uint64)
        out = np.zeros(max(n, 1) * 96, np.uint8)
        self._check(self.lib.lb_g1_mul(self._h, n, _ptr(a), _ptr(k), _ptr(out)), "lb_g1_mul")
        return [out[i * 96:(i + 1) * 96].tobytes() for i in range(n)]

    def g2_mul(self, pts: Sequence[bytes], ks: Sequence[int]) -> List[bytes]:
        n = len(pts)
        a = _u8(b"".join(pts))
        k = np.array(ks, dtype=np.uint64)
        out = np.zeros(max(n, 1) * 192, np.uint8)
        self._check(self.lib.lb_g2_mul(self._h, n, _ptr(a), _ptr(k), _ptr(out)), "lb_g2_mul")
        return [out[i * 192:(i + 1) * 192].tobytes() for i in range(n)]

    def g2_msm(self, pts: Sequence[bytes], raw: Sequence[int]) -> bytes:
        """sum_i (a_i + b_i lambda) P_i (a_i / b_i = low / high 32 bits of raw[i]) through
        the merged check's bucket MSM; 192-byte uncompressed points in and out."""
        n = len(pts)
        a = _u8(b"".join(pts)) if n else np.zeros(1, np.uint8)
        k = np.array(list(raw) or [0], dtype=np.uint64)
        out = np.zeros(192, np.uint8)
        self._check(self.lib.lb_g2_msm(self._h, n, _ptr(a), _ptr(k), _ptr(out)), "lb_g2_msm")
        return out.tobytes()

    def sk_to_pk(self, sks_be32: Sequence[bytes]) -> List[bytes]:
        n = len(sks_be32)
        k = _u8(b"".join(sks_be32))
        out = np.zeros(max(n, 1) * 96, np.uint8)
        self._check(self.lib.lb_sk_to_pk(self._h, n, _ptr(k), _ptr(out)), "lb_sk_to_pk")
        return [out[i * 96:(i + 1) * 96].tobytes() for i in range(n)]

    def sign(self, sks_be32: Sequence[bytes], messages: Sequence[bytes]) -> List[bytes]:
        n = len(sks_be32)
        k = _u8(b"".join(sks_be32))
        m = _u8(b"".join(messages))
        out = np.zeros(max(n, 1) * 96, np.uint8)
        self._check(self.lib.lb_sign(self._h, n, _ptr(k), _ptr(m), _ptr(out)), "lb_sign")
        return [out[i * 96:(i + 1) * 96].tobytes() for i in range(n)]

    def set_latency_path(self, max_sets: int) -> None:
        """Calls of at most max_sets sets take the latency path (0: never)."""
        self._check(self.lib.lb_set_latency_path(self._h, max_sets), "lb_set_latency_path")

    def lp_program_run(self, prog, inputs: np.ndarray, flags: np.ndarray, n_out: int, n_outflag: int,
                       stamps: bool = False):
        """One latency-path round program on n instances (lb_lp_program_run): prog = an
        embedded program id or an encoded program (list of u32 words); inputs (n, n_in, 16)
        u32 limb records, flags (n, n_inflag) u32 -> (out (n, n_out, 16), out_flags
        (n, n_outflag), kernel ms[, per-round s_memtime stamps of instance 0])."""
        inputs = np.ascontiguousarray(inputs, dtype=np.uint32)
        n = inputs.shape[0]
        fl = np.ascontiguousarray(flags, dtype=np.uint32) if flags is not None and flags.size else None
        out = np.zeros((n, max(n_out, 1), 16), np.uint32)
        ofl = np.zeros((n, max(n_outflag, 1)), np.uint32)
        ms = ctypes.c_float(0)
        words = None
        if not isinstance(prog, int):
            words = np.ascontiguousarray(np.array(prog, dtype=np.uint32))
        n_rounds = int(words[1]) if words is not None else 4096
        st = np.zeros((n_rounds, 6 + 6 * 8), np.uint64) if stamps else None  # LB_LP_STAMPS points per round
        self._check(self.lib.lb_lp_program_run(self._h, 0 if words is not None else prog, _ptr(words),
                                               0 if words is None else words.size, n, _ptr(inputs), _ptr(fl),
                                               _ptr(out), _ptr(ofl) if n_outflag else None, ctypes.byref(ms),
                                               _ptr(st)), "lb_lp_program_run")
        res = (out[:, :n_out], ofl[:, :n_outflag], float(ms.value))
        return res + (st,) if stamps else res

    def last_stage_times(self, raw: bool = False) -> List[Tuple[str, float]]:
        ms = (ctypes.c_float * 32)()
        names = (ctypes.c_char_p * 32)()
        n = self.lib.lb_last_stage_times(self._h, ms, names, 32)
        if raw:  # one entry per launch, in launch order (tools/opcount.py pairs them with its counters)
            return [(names[i].decode(), float(ms[i])) for i in range(min(n, 32))]
        # a stage launched more than once in a call (level_wc's passes) is reported once, summed
        out: dict = {}
        for i in range(min(n, 32)):
            nm = names[i].decode()
            out[nm] = out.get(nm, 0.0) + float(ms[i])
        return list(out.items())


def scratch_per_queue(device: int = 0) -> Tuple[int, int]:
    """(scratch bytes one hardware queue reserves, largest private bytes per lane)."""
    lib = load_library()
    b, lane = ctypes.c_uint64(0), ctypes.c_uint32(0)
    rc = lib.lb_scratch_per_queue(device, ctypes.byref(b), ctypes.byref(lane))
    if rc != LB_OK:
        raise LodestarBlsError(f"lb_scratch_per_queue failed ({rc})")
    return int(b.value), int(lane.value)


def device_count() -> int:
    return int(load_library().lb_device_count())
