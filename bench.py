"""Benchmark: verified BLS signature sets/sec on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1], the single-GPU config the metric is quoted
on): 65,536 distinct-message single-pubkey attestation sets per GPU, submitted
as 512 requests x 128 sets (MAX_SIGNATURE_SETS_PER_JOB, packages/beacon-node/
src/chain/bls/multithread/index.ts:57), each request verified with
verifySignatureSetsMaybeBatch semantics.  A "step" = one call over the whole
65,536-set batch with inputs already resident in HBM.  Synthetic data: interop
secret keys (packages/state-transition/src/util/interop.ts:19-23), messages
sha256(seed || LE64(i)), signatures from the GPU signer (parity-checked
against the oracle by tests and smoke()).

Multi-GPU (--gpus N): one process per GPU.  Without WORLD_SIZE in the
environment, bench.py starts the N ranks itself (child processes, before any
GPU call); under torchrun it is one of them.  Each rank verifies its own
65,536 sets per step (weak scaling, no data-path collective): every step runs
as a two-phase call up to the rank's merged Miller product, the 576-byte Fp12
partials of all ranks are all-gathered over gloo (host memory), the
combined check final_exp(prod) == 1 runs once, on rank 0's GPU, and its
verdict is broadcast
(north_star: partials combined on the host).  value = total sets
over all ranks / max-over-ranks time.

Secondary legs (N = 1, after the timed region; reported, never `value`):
host-buffer API throughput (PCIe included), same-message gossip jobs (512
jobs x 128 sets per call), an adversarial leg (one wrong-message set per call),
the C1 CPU p50 of one 128-set job, p50 latency of one 128-set request on the
GPU, the CPU baseline.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
# HIP hardware queues per process (HIP's default, and the box's environment, is 4).
# The library keeps one call in flight per queue (lb_create: GPU_MAX_HW_QUEUES slots,
# up to 16); each call's merged check ends in one-wave kernels (MSM bit sums, final
# exponentiation) during which its queue's share of the GPU idles, so more calls in
# flight fill the SIMDs better: 2.74 / 2.89 / 2.98 / 3.03 M sets/s at 4 / 8 / 12 / 16
# (profiles/ab_r03/hwq, hwq2).  Set before HIP initialises (torch import); the N-API
# addon does the same for a Lodestar process (LB_HW_QUEUES overrides both).
# (clamped to 16: lb_create refuses more, each queue reserving scratch for the largest
# private segment at full occupancy)
os.environ["GPU_MAX_HW_QUEUES"] = str(max(1, min(16, int(os.environ.get("LB_HW_QUEUES", "16")))))
sys.path.insert(0, ROOT)

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
# Roofline peak: v_mad_u64_u32 is quarter-rate on gfx950: 32 per clk per CU at
# 2.4 GHz over 256 CUs = 19.66 Tmad/s.  Measured: 1.877e13/s = 30.55 per clk per CU
# (tools/microbench/mad_rate.hip, 8 waves/SIMD; profiles/prof_r03e/mad_rate.txt).
# The larger of the two (the nominal one) prices every fraction.
PEAK_MAD_PER_S = max(256 * 32 * 2.4e9, 1.877e13)


def interop_sk_be(i: int) -> bytes:
    d = hashlib.sha256(i.to_bytes(32, "little")).digest()
    return (int.from_bytes(d, "little") % R_ORDER).to_bytes(32, "big")


def make_workload(dev, n_sets: int, first_index: int, seed: bytes):
    sks = [interop_sk_be(first_index + i) for i in range(n_sets)]
    msgs = [hashlib.sha256(seed + (first_index + i).to_bytes(8, "little")).digest() for i in range(n_sets)]
    pks, sigs = [], []
    chunk = 16384
    for s in range(0, n_sets, chunk):
        pks += dev.sk_to_pk(sks[s:s + chunk])
        sigs += dev.sign(sks[s:s + chunk], msgs[s:s + chunk])
    return sks, pks, msgs, sigs


def cpu_baseline_c(pks, msgs, sigs, seconds: float, threads: int, per_request: int):
    """Time the C oracle (oracle/c/bls_oracle.c, the CPU restatement of the same
    verification, kind "port") on `threads` host threads: rounds of one
    128-set request per thread from the same workload until ~`seconds` have
    passed.  Returns (sets/s, sets done, elapsed, build variant)."""
    from oracle import c_oracle as C
    n_req_round = threads
    n_sets = n_req_round * per_request
    req_off = np.arange(0, n_sets + 1, per_request, dtype=np.uint32)
    pk = np.frombuffer(b"".join(pks[:n_sets]), np.uint8)
    mg = np.frombuffer(b"".join(msgs[:n_sets]), np.uint8)
    blob, offs = C.pack_blobs(sigs[:n_sets])
    seed = hashlib.sha256(b"batch-rand").digest()
    done, t0 = 0, time.time()
    while True:
        valid, err = C.verify_requests(req_off, pk, None, mg, blob, offs, seed, threads)
        assert valid.all() and not err.any(), "CPU oracle rejected a valid request"
        done += n_sets
        if time.time() - t0 >= seconds:
            break
    el = time.time() - t0
    return done / el, done, el, C.variant()


def cpu_c1_p50(pks, msgs, sigs, per_request: int, reps: int):
    """C1 (BASELINE.json configs[0]): one 128-set verifySignatureSets job as one
    worker thread runs it (worker.ts:30-108 on one core), p50 over `reps`."""
    from oracle import c_oracle as C
    req_off = np.array([0, per_request], np.uint32)
    pk = np.frombuffer(b"".join(pks[:per_request]), np.uint8)
    mg = np.frombuffer(b"".join(msgs[:per_request]), np.uint8)
    blob, offs = C.pack_blobs(sigs[:per_request])
    lat = []
    for _ in range(reps):
        t1 = time.perf_counter()
        valid, _ = C.verify_requests(req_off, pk, None, mg, blob, offs, bytes(32), 1)
        lat.append((time.perf_counter() - t1) * 1e3)
        assert valid.all()
    return float(np.median(lat))


def launch_ranks(a) -> int:
    """--gpus N without a launcher: one child process per GPU (started before
    this process touches the GPU), RANK/LOCAL_RANK/WORLD_SIZE in their env;
    rank 0 prints the JSON line.  Returns the worst exit code."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    # ranks sharing a GPU (a rehearsal on fewer GPUs than ranks): their contexts' HIP
    # hardware queues add up on that GPU, and past what its queue scheduler maps at once it
    # time-slices them -- 2 ranks x 20 queues on one GPU ran at 0.6-1.0 M sets/s, 2 x 12 at
    # 3.36 M (profiles/r05/rehearsal/).  Each rank then gets a share of the 16 calls in flight.
    qenv = {}
    try:
        import torch  # (device_count does not initialise the GPU on this image)
        ndev = torch.cuda.device_count()
    except Exception:
        ndev = 0
    share = -(-a.gpus // ndev) if ndev else 1
    if share > 1 and "LB_HW_QUEUES" not in os.environ:
        qenv["LB_HW_QUEUES"] = str(max(4, 16 // share))
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus), LOCAL_WORLD_SIZE=str(a.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), **qenv)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rcs = [p.wait() for p in procs]
    return max(abs(rc) for rc in rcs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--sets", type=int, default=65536)
    ap.add_argument("--per-request", type=int, default=128)
    ap.add_argument("--latency-reps", type=int, default=10)
    ap.add_argument("--iso-reps", type=int, default=3,
                    help="sync calls after the timed region whose stage times price the dominant kernel")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-legs", action="store_true", help="skip the secondary legs (host API, same-message, ...)")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the C3 / C4 shard / C5 / perf-suite size legs (config_legs)")
    ap.add_argument("--node-rounds", type=int, default=96,
                    help="node leg: rounds of 512 x 128-set jobs (one 65,536-set package each) queued at once "
                         "(enough packages past the 16 in flight that filling and draining the pipe is small)")
    ap.add_argument("--sync", action="store_true", help="one call at a time (no overlap between steps)")
    ap.add_argument("--combine", choices=["auto", "on", "off"], default="auto",
                    help="two-phase calls + host combine of the ranks' Fp12 partials (auto: on -- at N = 1 too, "
                         "where it measured 3.61-3.63 vs 3.53 M sets/s one-phase: the slot is released at the "
                         "partial and the final exponentiation runs beside the calls, profiles/r05/combine_ab/; "
                         "off: every call one-phase)")
    ap.add_argument("--inflight", type=int,
                    default=int(os.environ.get("LB_SLOTS", min(16, max(4, int(os.environ["GPU_MAX_HW_QUEUES"]))))),
                    help="calls kept in flight (= library slots, env LB_SLOTS)")
    ap.add_argument("--node-data", help=argparse.SUPPRESS)  # (internal: the node leg's input child)
    a = ap.parse_args()

    if a.node_data:
        node_data_main(a.node_data, a.sets)
        return
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a))
    # the node leg first, while this process holds no HIP queue (node_leg)
    node_res = None
    if int(os.environ.get("WORLD_SIZE", "1")) == 1 and not a.no_legs:
        _progress("node leg")
        node_res = node_leg(a.sets, a.node_rounds)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # barrier, max-over-ranks and the 576-byte partials; no data-path collective.  Gloo's
        # C++ side prints "[Gloo] Rank r is connected ..." on stdout: route fd 1 to stderr
        # meanwhile, so rank 0's stdout carries only the JSON line
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo")
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    ndev = torch.cuda.device_count()
    gpu = local % max(ndev, 1)  # one process per GPU; ranks > devices only when rehearsing
    torch.cuda.set_device(gpu)
    from lodestar_amd.native import Device
    dev = Device(gpu)
    combine = a.combine == "on" or (a.combine == "auto" and not a.sync)

    n = a.sets
    seed = hashlib.sha256(b"lodestar-mi355x-bench").digest()
    t_gen = time.time()
    sks, pks, msgs, sigs = make_workload(dev, n, rank * n, seed)
    t_gen = time.time() - t_gen

    cuda = torch.device("cuda", gpu)
    d_pk = torch.from_numpy(np.frombuffer(b"".join(pks), np.uint8).copy()).to(cuda)
    d_msg = torch.from_numpy(np.frombuffer(b"".join(msgs), np.uint8).copy()).to(cuda)
    d_sig = torch.from_numpy(np.frombuffer(b"".join(sigs), np.uint8).copy()).to(cuda)
    sig_off = np.arange(0, 96 * (n + 1), 96, dtype=np.uint32)
    req_off = np.arange(0, n + 1, a.per_request, dtype=np.uint32)
    if req_off[-1] != n:
        req_off = np.append(req_off, np.uint32(n))
    n_req = len(req_off) - 1
    d_sigoff = torch.from_numpy(sig_off.view(np.int32)).to(cuda)
    d_reqoff = torch.from_numpy(req_off.view(np.int32)).to(cuda)
    d_seed = torch.from_numpy(np.frombuffer(hashlib.sha256(b"batch-rand").digest(), np.uint8).copy()).to(cuda)
    # one output buffer per in-flight call (the library keeps one call per slot)
    nbuf = max(1, a.inflight)
    # (+ a quarter more: the two-phase flow keeps that many more calls outstanding)
    d_valid = [torch.zeros(n_req, dtype=torch.uint8, device=cuda) for _ in range(nbuf + nbuf // 4)]
    d_err = [torch.zeros(n_req, dtype=torch.uint8, device=cuda) for _ in range(nbuf + nbuf // 4)]
    torch.cuda.synchronize()

    def submit(k, msg_ptr=None, partial=False):
        return dev.verify_requests_device_async(n_req, n, d_reqoff.data_ptr(), d_pk.data_ptr(), None,
                                                msg_ptr or d_msg.data_ptr(), d_sig.data_ptr(), d_sigoff.data_ptr(),
                                                d_seed.data_ptr(), d_valid[k % len(d_valid)].data_ptr(),
                                                d_err[k % len(d_err)].data_ptr(), partial=partial)

    def step(k=0, nr=n_req, ns=n):
        # synchronous call (library slot 0: two-stream DAG, lowest latency)
        dev.verify_requests_device(nr, ns, d_reqoff.data_ptr(), d_pk.data_ptr(), None, d_msg.data_ptr(),
                                   d_sig.data_ptr(), d_sigoff.data_ptr(), d_seed.data_ptr(),
                                   d_valid[k % len(d_valid)].data_ptr(), d_err[k % len(d_err)].data_ptr())

    combined = {"checks": 0, "passed": 0, "partials_per_check": 0, "gather_ms": 0.0, "check_ms": 0.0}

    def resolve(t):
        """Two-phase step: this rank's partial, all ranks' partials gathered on the
        host (gloo), one final exponentiation on this GPU, resume with the verdict."""
        part = dev.partial_wait_t(t)
        t1 = time.perf_counter()
        if world > 1:
            mine = torch.frombuffer(bytearray(part), dtype=torch.uint8)
            parts = [torch.zeros(576, dtype=torch.uint8) for _ in range(world)]
            dist.all_gather(parts, mine)
            partials = [bytes(p.numpy().tobytes()) for p in parts]
        else:
            partials = [part]
        t2 = time.perf_counter()
        if world > 1:
            # ONE combined final exponentiation (rank 0's GPU), its verdict broadcast
            flag = torch.zeros(1, dtype=torch.int32)
            if rank == 0:
                flag[0] = 1 if dev.gt_check(partials) else 0
            dist.broadcast(flag, 0)
            ok = bool(int(flag[0]))
        else:
            ok = dev.gt_check(partials)
        t3 = time.perf_counter()
        dev.finish_t(t, ok)
        dev.wait(t)
        combined["checks"] += 1
        combined["passed"] += int(ok)
        combined["partials_per_check"] = len(partials)
        combined["gather_ms"] += (t2 - t1) * 1e3
        combined["check_ms"] += (t3 - t2) * 1e3

    for k in range(a.warmup):
        step(k)
    # every slot's first C2-sized call sizes its workspace (~1.9 GB hipMalloc, bls_host.hip
    # ensure_ws): one async call per slot in flight here, so no timed step pays for it
    # (the W steps above run synchronously on slot 0 and the priority lane)
    if not a.sync:
        for t in [submit(k, partial=combine) for k in range(nbuf)]:
            resolve(t) if combine else dev.wait(t)
    if combine:  # warm the two-phase path too (every rank takes part in each gather)
        resolve(submit(0, partial=True))
        combined.update(checks=0, passed=0, gather_ms=0.0, check_ms=0.0)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    _progress("timed region")
    t0 = time.perf_counter()
    stage_acc = {}
    n_acc = [0]

    def accumulate():
        n_acc[0] += 1
        for name, ms in dev.last_stage_times():
            stage_acc[name] = stage_acc.get(name, 0.0) + ms

    pending = []
    if combine and not a.sync:
        # two-phase steps with the combine off the submit loop: this thread keeps `nbuf`
        # calls in flight; a resolver thread takes each call in order through partial ->
        # all-gather -> one final exponentiation -> finish -> retire.  The context is not
        # thread-safe: every library call holds `lock`, and the resolver polls
        # (lb_partial_poll / lb_poll) instead of blocking in the library with it held.
        import queue
        import threading
        lock = threading.Lock()
        # calls outstanding: the library's slots plus a quarter more -- a two-phase call frees
        # its slot when its partial is ready (LB_TP_RELEASE, default), so the calls waiting
        # for the combine do not keep the GPU's slots idle (without the release a submit
        # would wait in the library for a slot held by a call the resolver has yet to finish)
        extra = nbuf // 4 if os.environ.get("LB_TP_RELEASE", "1") != "0" else 0
        free = threading.Semaphore(nbuf + extra)
        todo = queue.Queue()
        failed = []

        def poll_until(fn, t):
            while True:
                with lock:
                    if fn(t):
                        return
                time.sleep(0.0002)

        def resolver():
            try:
                while True:
                    t = todo.get()
                    if t is None:
                        return
                    poll_until(dev.partial_ready, t)
                    with lock:
                        part = dev.partial_wait_t(t)
                    t1 = time.perf_counter()
                    if world > 1:
                        mine = torch.frombuffer(bytearray(part), dtype=torch.uint8)
                        parts = [torch.zeros(576, dtype=torch.uint8) for _ in range(world)]
                        dist.all_gather(parts, mine)
                        partials = [bytes(p.numpy().tobytes()) for p in parts]
                    else:
                        partials = [part]
                    t2 = time.perf_counter()
                    if world > 1:
                        flag = torch.zeros(1, dtype=torch.int32)
                        if rank == 0:
                            flag[0] = 1 if dev.gt_check(partials) else 0
                        dist.broadcast(flag, 0)
                        ok_t = bool(int(flag[0]))
                    else:
                        # (lb_gt_check uses only the context's aux buffers and stream: no lock,
                        # the submit loop goes on meanwhile -- include/lodestar_bls.h)
                        ok_t = dev.gt_check(partials)
                    t3 = time.perf_counter()
                    with lock:
                        dev.finish_t(t, ok_t)
                    poll_until(dev.poll, t)
                    with lock:
                        dev.wait(t)
                        accumulate()
                    combined["checks"] += 1
                    combined["passed"] += int(ok_t)
                    combined["partials_per_check"] = len(partials)
                    combined["gather_ms"] += (t2 - t1) * 1e3
                    combined["check_ms"] += (t3 - t2) * 1e3
                    free.release()
            except BaseException as e:  # surfaced after the join
                failed.append(e)
                for _ in range(nbuf):
                    free.release()

        th = threading.Thread(target=resolver, daemon=True)
        th.start()
        for k in range(a.steps):
            free.acquire()
            if failed:
                break
            with lock:
                t = submit(k, partial=True)
            todo.put(t)
        todo.put(None)
        th.join()
        if failed:
            raise failed[0]
    for k in range(a.steps if not (combine and not a.sync) else 0):
        if a.sync and not combine:
            step(k)
            accumulate()
        else:
            pending.append(submit(k, partial=combine))
            if len(pending) >= (1 if a.sync else nbuf):
                t = pending.pop(0)
                resolve(t) if combine else dev.wait(t)
                accumulate()
    for t in pending:
        resolve(t) if combine else dev.wait(t)
        accumulate()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    # (only the output buffers the timed steps wrote: with fewer steps than calls in flight the
    # rest were never used)
    used = sorted({k % len(d_valid) for k in range(a.steps)})
    ok = all(bool(d_valid[i].cpu().numpy().all()) for i in used) and \
        not any(bool(d_err[i].cpu().numpy().any()) for i in used)

    # the same call, one at a time and on ONE stream (a context with LB_DAG=0: no kernel of
    # the other DAG branch and no other call beside it): every kernel's duration alone on the
    # GPU (the roofline of the dominant kernel is priced on these)
    iso = {}
    if a.iso_reps > 0:
        # (and no priority-lane CU reservation: a second context's CU-masked streams cost the
        # later legs of this process a third of their throughput)
        saved = {k: os.environ.get(k) for k in ("LB_DAG", "LB_PRIO_CUS")}
        os.environ["LB_DAG"] = "0"
        os.environ["LB_PRIO_CUS"] = "0"
        try:
            iso_dev = Device(gpu)
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        for k in range(a.iso_reps + 1):  # (+1: the context's first call is a warm-up)
            iso_dev.verify_requests_device(n_req, n, d_reqoff.data_ptr(), d_pk.data_ptr(), None, d_msg.data_ptr(),
                                           d_sig.data_ptr(), d_sigoff.data_ptr(), d_seed.data_ptr(),
                                           d_valid[k % nbuf].data_ptr(), d_err[k % nbuf].data_ptr())
            if k:
                for name, ms in iso_dev.last_stage_times():
                    iso.setdefault(name, []).append(ms)
        iso_dev.close()
    iso_ms = {k: float(np.median(v)) for k, v in iso.items()}

    # p50 latency of one 128-set batch (one request)
    lat = []
    if a.latency_reps > 0:
        step(0, 1, a.per_request)
        for _ in range(a.latency_reps):
            t1 = time.perf_counter()
            step(0, 1, a.per_request)
            lat.append((time.perf_counter() - t1) * 1e3)
    p50 = float(np.median(lat)) if lat else None
    lat_stages = {name: round(ms, 3) for name, ms in dev.last_stage_times()} if lat else None
    # p50 of ONE set (the verifyOnMainThread shape: a 1-set request, core verify,
    # BN/chain/validation/block.ts:146) and of one 128-set request through the
    # synchronous host-buffer entry point (numpy in, verdicts out, PCIe included)
    lat1, lat_host, lat1_clk = [], [], []
    if a.latency_reps > 0:
        d_req1 = torch.tensor([0, 1], dtype=torch.int32, device=cuda)

        def one_set():
            dev.verify_requests_device(1, 1, d_req1.data_ptr(), d_pk.data_ptr(), None, d_msg.data_ptr(),
                                       d_sig.data_ptr(), d_sigoff.data_ptr(), d_seed.data_ptr(),
                                       d_valid[0].data_ptr(), d_err[0].data_ptr())
        pk_h = np.frombuffer(b"".join(pks[:a.per_request]), np.uint8)
        mg_h = np.frombuffer(b"".join(msgs[:a.per_request]), np.uint8)
        sg_h = np.frombuffer(b"".join(sigs[:a.per_request]), np.uint8)
        ro_h = np.array([0, a.per_request], np.uint32)
        so_h = sig_off[:a.per_request + 1]
        seed_h = hashlib.sha256(b"batch-rand").digest()
        one_set()
        assert dev.verify_requests(ro_h, pk_h, None, mg_h, sg_h, so_h, seed_h).valid.all()
        for _ in range(a.latency_reps):
            t1 = time.perf_counter()
            one_set()
            lat1.append((time.perf_counter() - t1) * 1e3)
            lat1_clk.append(dev.last_latency_clocks())
            t1 = time.perf_counter()
            dev.verify_requests(ro_h, pk_h, None, mg_h, sg_h, so_h, seed_h)
            lat_host.append((time.perf_counter() - t1) * 1e3)
    p50_1 = float(np.median(lat1)) if lat1 else None
    p50_host = float(np.median(lat_host)) if lat_host else None

    # the same two latencies while `nbuf` 65,536-set calls stay in flight (a node under
    # gossip load): the small calls take the library's priority lane (a slot of its own on
    # a highest-priority stream, lb_verify_requests_device of <= lp_max sets); every
    # iteration retires the oldest call and submits the next, so the load never drains
    loaded = None
    if a.latency_reps > 0 and world == 1:  # (one-phase background calls, after the timed region)
        # (the window opens before the first background call is submitted and closes when the
        # last retires: every one of the kk calls ran inside it, and all kk are counted --
        # the window used to open after nbuf calls were already in flight)
        t_load = time.perf_counter()
        pend = [submit(k) for k in range(nbuf)]
        kk = nbuf
        ll1, ll128 = [], []
        for r in range(2 * a.latency_reps):
            t1 = time.perf_counter()
            if r % 2:
                step(0, 1, a.per_request)
                ll128.append((time.perf_counter() - t1) * 1e3)
            else:
                one_set()
                ll1.append((time.perf_counter() - t1) * 1e3)
            dev.wait(pend.pop(0))
            pend.append(submit(kk))
            kk += 1
        for t in pend:
            dev.wait(t)
        el_load = time.perf_counter() - t_load
        loaded = {"p50_ms_1set": round(float(np.median(ll1)), 3),
                  "p50_ms_128set_batch": round(float(np.median(ll128)), 3),
                  "calls_in_flight": nbuf, "background_sets_per_s": round(n * kk / el_load, 1),
                  "background_calls": kk, "window_s": round(el_load, 3),
                  "ratio_1set_vs_idle": round(float(np.median(ll1)) / p50_1, 2) if p50_1 else None,
                  "ratio_128set_vs_idle": round(float(np.median(ll128)) / p50, 2) if p50 else None,
                  "lane": "priority slot (highest-priority stream) + latency path"}

    legs = {}
    if world == 1 and not a.no_legs:
        _progress("secondary legs")
        legs = secondary_legs(a, dev, torch, cuda, pks, msgs, sigs, sks, submit, nbuf, n, n_req, req_off, sig_off,
                              (d_reqoff.data_ptr(), d_pk.data_ptr(), d_sig.data_ptr(), d_sigoff.data_ptr(),
                               d_seed.data_ptr()))
        if not a.no_configs:
            legs.update(config_legs(a, dev, torch, cuda, sks, pks, msgs, sigs, nbuf))
        if node_res is not None:
            legs["node"] = node_res

    if rank != 0:
        if world > 1:
            dist.barrier()
        return
    total_sets = n * world * a.steps
    value = total_sets / elapsed
    stage_ms = {k: v / max(n_acc[0], 1) for k, v in stage_acc.items()}
    roof = roofline(iso_ms, stage_ms, n, value, a.iso_reps, n_req)
    cpu = None
    c1 = None
    if not a.no_cpu_baseline and world == 1:
        _progress("cpu baseline")
        # the box's CPU share is 16 threads per GPU (os.cpu_count() shows the whole host)
        threads = max(1, min(16, os.cpu_count() or 1))
        rate, done, el, variant = cpu_baseline_c(pks, msgs, sigs, a.cpu_seconds, threads, a.per_request)
        cpu = {"value": round(rate, 2), "unit": "sets/s", "cores": threads, "kind": "port",
               "sample": f"{done} sets of the same workload ({a.per_request}-set requests, same verdict rules) "
                         f"verified by the C restatement oracle/c/bls_oracle.c ({variant}, {threads} threads, "
                         f"{el:.1f} s); blst itself cannot run here (no node>=20 / @chainsafe/blst); the "
                         f"reference's own anchor is ~0.9 ms/set/core (metrics/metrics/lodestar.ts:470)"}
        c1 = {"config": "C1: verifySignatureSets on one 128-set job (BASELINE.json configs[0])",
              "cpu_p50_ms": round(cpu_c1_p50(pks, msgs, sigs, a.per_request, 7), 3), "cpu_threads": 1,
              "cpu_kind": "port (oracle/c/bls_oracle.c, one worker thread)",
              "gpu_p50_ms": round(p50, 3) if p50 is not None else None}
    out = {
        "metric": "verified signature sets/sec",
        "value": round(value, 2),
        "unit": "sets/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(elapsed / a.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (interop keys, sha256 messages, GPU-signed)",
        "config": {"workload": f"C2: {n} distinct-message single-pubkey sets per GPU, {n_req} requests x "
                               f"{a.per_request} sets, verifySignatureSetsMaybeBatch semantics",
                   "sets_per_gpu": n, "sets_per_request": a.per_request, "parallelism": f"shard{world}"},
        "requested_gpus": a.gpus,
        "ranks_joined": world,
        "p50_ms_128set_batch": round(p50, 3) if p50 is not None else None,
        "p50_stage_ms": lat_stages,
        "p50_ms_1set": round(p50_1, 3) if p50_1 is not None else None,
        # the latency path's kernel alone (s_memrealtime inside k_lp_verify) and its shader clock
        "p50_1set_kernel": ({"ms": round(float(np.median([c[0] for c in lat1_clk if c[0]])), 3),
                             "clock_mhz": round(float(np.median([c[1] for c in lat1_clk if c[0]])), 1)}
                            if any(c[0] for c in lat1_clk) else None),
        "p50_ms_128set_host": round(p50_host, 3) if p50_host is not None else None,
        "latency_under_load": loaded,
        "all_valid": ok,
        "overlap": "sync" if a.sync else f"{nbuf} calls in flight",
        "combine": ({"mode": ("two-phase calls; per-step all-gather of the ranks' 576-byte Fp12 partials (gloo), "
                              "one final exponentiation on rank 0's GPU (lb_gt_check), verdict broadcast; "
                              "the combine runs on a resolver thread beside the submit loop") if world > 1 else
                             ("two-phase calls (the multi-GPU flow at N = 1): each call's 576-byte Fp12 partial, "
                              "its final exponentiation (lb_gt_check) and finish on a resolver thread beside the "
                              "submit loop; the call's slot is released at the partial"),
                     "checks": combined["checks"], "passed": combined["passed"],
                     "partials_per_check": combined["partials_per_check"],
                     "gather_ms_avg": round(combined["gather_ms"] / max(combined["checks"], 1), 3),
                     "check_ms_avg": round(combined["check_ms"] / max(combined["checks"], 1), 3)}
                    if combine else None),
        "stage_ms": {k: round(v, 3) for k, v in stage_ms.items()},
        "iso_stage_ms": {k: round(v, 3) for k, v in iso_ms.items()},
        "roofline": roof,
        "cpu_baseline": cpu,
        "c1": c1,
        **legs,
        "datagen_s": round(t_gen, 2),
    }
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()


# Algorithmic work priced at the lowest count the same kernel reaches (the
# default k_step_acc takes one line at a time, 631,170 mads/set; with lines paired the same
# accumulation needs 554,850 -- DESIGN.md §4 table), so a frac never credits redundant work
ALGO_MIN_MADS_PER_SET = {"step_acc": 554850.0}
ALGO_MIN_PIPELINE_SAVING = 631170.0 - 554850.0


def roofline(iso_ms, stage_ms, n, value, iso_reps, n_req):
    """Dominant kernel's integer-MAD roofline (achieved = algorithmic mads of one
    launch / its HIP-event duration, one call at a time) + the pipeline's."""
    counts_path = os.path.join(ROOT, "profiles", "op_counts.json")
    timing = iso_ms if iso_ms else stage_ms
    cands = [k for k in timing if k not in ("start", "h2d", "d2h")]
    if not cands or not os.path.exists(counts_path):
        return None
    dom = max(cands, key=lambda k: timing[k])
    oc = json.load(open(counts_path))
    pairs_org = os.environ.get("LB_ACC") == "pairs"
    st = (oc.get("pairs_stages", oc["stages"]) if pairs_org else oc["stages"]).get(dom)
    if not st:
        return None
    per_set = st.get("mads_per_set", st["fp_mul_per_set"] * oc["mads_per_fp_mul"])
    # the iso launches are lone calls: k_miller_acc then splits requests in halves (one pair per
    # lane, its own Fp12 squarings), so its work per set is that organisation's count
    lone = oc.get("lone_call_stages", {}).get(dom) if iso_ms and pairs_org else None
    per_set_pipe = per_set
    split_env = os.environ.get("LB_ACC_SPLIT")  # bls_host.hip: 1 always, 0 never,
    split = split_env != "0" and (split_env == "1" or n_req >= 64)  # default: lone calls from 64 requests
    if lone and split:
        per_set = lone["mads_per_set"]
    executed = per_set
    if not pairs_org and dom in ALGO_MIN_MADS_PER_SET:
        per_set = min(per_set, ALGO_MIN_MADS_PER_SET[dom])
        if os.environ.get("LB_STEP_MODE", "1") in ("0", "1"):  # paired lines (the default LDS build)
            executed = per_set
    mads = per_set * n
    achieved = mads / (timing[dom] * 1e-3) / 1e12
    peak = PEAK_MAD_PER_S / 1e12
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc_path):
        traffic = json.load(open(pmc_path)).get(dom, {}).get("hbm_bytes_per_launch")
    roof = {"bound": "valu", "kernel": dom, "achieved": round(achieved, 4), "peak": round(peak, 3),
            "unit": "Tmad/s", "frac": round(achieved / peak, 5), "traffic": traffic,
            "algorithmic_mads_per_launch": mads, "executed_mads_per_set": round(executed),
            "launch_ms": round(timing[dom], 3),
            "timing": "median of %d one-at-a-time single-stream calls after the timed region (LB_DAG=0: "
                      "the kernel alone on the GPU; HIP events on its stream)" % iso_reps
                      if iso_ms else "timed region, calls overlapped"}
    if executed != per_set_pipe:
        roof["organisation"] = ("lone call: requests split in halves, one pair per lane "
                                "(profiles/op_counts.json lone_call_stages)")
        roof["mads_per_set_launch"] = round(per_set)
        roof["mads_per_set_two_pairs_per_lane"] = round(per_set_pipe)
        roof["frac_at_two_pairs_per_lane_count"] = round(per_set_pipe * n / (timing[dom] * 1e-3) / 1e12 / peak, 5)
    if iso_ms:
        # every kernel with an op count, each alone on the GPU: ms and fraction of the mad peak
        stages = oc.get("pairs_stages", oc["stages"]) if pairs_org else oc["stages"]
        ka = {}
        for k, ms in sorted(iso_ms.items(), key=lambda x: -x[1]):
            m = stages.get(k, {}).get("mads_per_set")
            if m and not pairs_org and k in ALGO_MIN_MADS_PER_SET:
                m = min(m, ALGO_MIN_MADS_PER_SET[k])
            if m and ms > 0.5:
                ka[k] = {"ms": round(ms, 3), "frac": round(m * n / (ms * 1e-3) / 1e12 / peak, 4)}
        roof["kernels_alone"] = ka
    if iso_ms and dom in stage_ms:
        # the same kernel while other calls' kernels share the CUs (timed region, two pairs per lane)
        roof["in_pipeline_launch_ms"] = round(stage_ms[dom], 3)
        roof["in_pipeline_frac"] = round(min(per_set_pipe, per_set) * n / (stage_ms[dom] * 1e-3) / 1e12 / peak, 5)
    tot_key = "pairs_mads_per_set_total" if pairs_org and "pairs_mads_per_set_total" in oc else "mads_per_set_total"
    if tot_key in oc:
        # whole pipeline: every v_mad_u64_u32 the algorithm needs per set x sets/s
        tot = oc[tot_key] - (0 if pairs_org else ALGO_MIN_PIPELINE_SAVING)
        pipe = value * tot / 1e12
        roof["pipeline_achieved"] = round(pipe, 4)
        roof["pipeline_frac"] = round(pipe / peak, 5)
        roof["mads_per_set"] = round(tot)
    return roof


def compress_g1(unc: bytes) -> bytes:
    """ZCash compression of a 96-byte uncompressed G1 encoding (x with the 0x80 flag, 0x20
    when y is the lexicographically larger root)"""
    p = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
    if unc[0] & 0x40:
        return bytes([0xC0]) + bytes(47)
    y = int.from_bytes(unc[48:96], "big")
    return bytes([unc[0] | 0x80 | (0x20 if 2 * y > p else 0)]) + unc[1:48]


def c4_aggregates(dev, sks, n_agg: int = 1024, k: int = 488):
    """C4's aggregate attestations (committees of ~488 keys): n_agg committees of
    k validator indices, a message each, the aggregate signature = a signature by the sum
    of the committee's secret keys (= the sum of their signatures)"""
    n = len(sks)
    ints = [int.from_bytes(s, "big") for s in sks]
    idx = np.array([(a * k + q) * 7 % n for a in range(n_agg) for q in range(k)], np.uint32)
    msgs = [hashlib.sha256(b"c4-agg" + a.to_bytes(4, "little")).digest() for a in range(n_agg)]
    agg_sk = [(sum(ints[int(i)] for i in idx[a * k:(a + 1) * k]) % R_ORDER).to_bytes(32, "big") for a in range(n_agg)]
    sigs = []
    for s in range(0, n_agg, 16384):
        sigs += dev.sign(agg_sk[s:s + 16384], msgs[s:s + 16384])
    return idx, msgs, sigs


def write_node_inputs(d, pks, msgs, sigs, agg):
    for name, items in (("pks", pks), ("msgs", msgs), ("sigs", sigs)):
        with open(os.path.join(d, name + ".bin"), "wb") as f:
            f.write(b"".join(items))
    with open(os.path.join(d, "pks_c.bin"), "wb") as f:
        f.write(b"".join(compress_g1(k) for k in pks))
    agg_idx, agg_msgs, agg_sigs = agg
    with open(os.path.join(d, "agg_idx.bin"), "wb") as f:
        f.write(agg_idx.tobytes())
    with open(os.path.join(d, "agg_msgs.bin"), "wb") as f:
        f.write(b"".join(agg_msgs))
    with open(os.path.join(d, "agg_sigs.bin"), "wb") as f:
        f.write(b"".join(agg_sigs))


def node_data_main(d, n_sets):
    """--node-data DIR (a child process): the node leg's inputs -- the C2 workload of the
    main measurement and the C4 aggregates -- written to DIR; exits, releasing its queues."""
    from lodestar_amd.native import Device
    dev = Device(0)
    sks, pks, msgs, sigs = make_workload(dev, n_sets, 0, hashlib.sha256(b"lodestar-mi355x-bench").digest())
    agg = c4_aggregates(dev, sks)
    dev.close()
    write_node_inputs(d, pks, msgs, sigs, agg)


def node_leg(n_sets: int, rounds: int = 4):
    """The Lodestar path (tools/bench_node.js): BlsGpuVerifier in node -> N-API addon ->
    lb_verify_requests_async, pubkeys by index; throughput and p50 latencies; C4-shaped
    AggregateAndProof triples with keys as PublicKey objects.  Run BEFORE this process
    opens a HIP queue, the inputs made by a child process: HIP keeps a process's hardware
    queues after its streams are destroyed, and the node process's queues beside another
    process's oversubscribe the GPU's queue scheduler (priority calls under load:
    1-set p50 1.4-2.3x idle and 128-set spikes of 100-500 ms with this process's queues
    alive, 1.14-1.18x / 1.24-1.31x without; profiles/r05/node_q/)."""
    import shutil
    import tempfile
    if not shutil.which("node") or not os.path.exists(os.path.join(ROOT, "lodestar_amd", "napi", "lodestar_bls.node")):
        return None
    with tempfile.TemporaryDirectory() as d:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--node-data", d, "--sets", str(n_sets)],
                           capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            return {"error": "node inputs: " + r.stderr[-500:]}
        try:
            out = subprocess.run(["node", os.path.join(ROOT, "tools", "bench_node.js"), d, str(rounds)],
                                 capture_output=True, text=True, timeout=300)
        except subprocess.TimeoutExpired:
            return {"error": "timeout"}
    if out.returncode != 0:
        return {"error": out.stderr[-500:]}
    return json.loads(out.stdout.strip().splitlines()[-1])


def secondary_legs(a, dev, torch, cuda, pks, msgs, sigs, sks, submit, nbuf, n, n_req, req_off, sig_off, dev_ptrs):
    legs = {}
    reps = max(4, a.steps // 2)
    # (1) host-buffer API (what BlsGpuVerifier calls): numpy inputs, pinned staging, PCIe both ways
    pk_h = np.frombuffer(b"".join(pks), np.uint8)
    mg_h = np.frombuffer(b"".join(msgs), np.uint8)
    blob_h = np.frombuffer(b"".join(sigs), np.uint8)
    seed = hashlib.sha256(b"batch-rand").digest()
    pcs = [dev.verify_requests_async(req_off, pk_h, None, mg_h, blob_h, sig_off, seed) for _ in range(nbuf)]
    for pc in pcs:
        assert dev.wait_call(pc).valid.all()
    t1 = time.perf_counter()
    pend = []
    for _ in range(reps):
        pend.append(dev.verify_requests_async(req_off, pk_h, None, mg_h, blob_h, sig_off, seed))
        if len(pend) >= nbuf:
            dev.wait_call(pend.pop(0))
    allv = True
    for pc in pend:
        allv &= bool(dev.wait_call(pc).valid.all())
    el = time.perf_counter() - t1
    legs["host_api"] = {"sets_per_s": round(n * reps / el, 1), "calls": reps, "all_valid": allv,
                        "api": f"lb_verify_requests_async, host buffers, {nbuf} calls in flight (PCIe included)"}
    # (1b) the same with pubkeys by validator index into the device table (what the node
    # leg's BlsGpuVerifier sends): the library side of the Lodestar path without JS
    base = dev.pubkey_table_size()
    dev.pubkey_table_append(pks)
    idx = np.arange(base, base + n, dtype=np.uint32)
    pend, allv = [], True
    t1 = time.perf_counter()
    for _ in range(reps):
        pend.append(dev.verify_requests_async(req_off, None, None, mg_h, blob_h, sig_off, seed, pk_indices=idx))
        if len(pend) >= nbuf:
            allv &= bool(dev.wait_call(pend.pop(0)).valid.all())
    for pc in pend:
        allv &= bool(dev.wait_call(pc).valid.all())
    el = time.perf_counter() - t1
    legs["host_api_indexed"] = {"sets_per_s": round(n * reps / el, 1), "calls": reps, "all_valid": allv,
                                "api": f"lb_verify_requests_async, host buffers, pubkeys by validator index, "
                                       f"{nbuf} calls in flight"}
    # (2) adversarial: one wrong-message set per call -> merged check fails, every request's tail runs
    bad = bytearray(b"".join(msgs))
    bad[32 * (n // 2):32 * (n // 2) + 32] = hashlib.sha256(b"wrong").digest()
    d_bad = torch.from_numpy(np.frombuffer(bytes(bad), np.uint8).copy()).to(cuda)
    torch.cuda.synchronize()
    dev.wait(submit(0, d_bad.data_ptr()))
    t1 = time.perf_counter()
    pend = []
    for k in range(reps):
        pend.append(submit(k, d_bad.data_ptr()))
        if len(pend) >= nbuf:
            dev.wait(pend.pop(0))
    for t in pend:
        dev.wait(t)
    torch.cuda.synchronize()
    el = time.perf_counter() - t1
    legs["adversarial"] = {"sets_per_s": round(n * reps / el, 1), "calls": reps,
                           "case": "one wrong-message set per 65,536-set call: merged check fails, 512 per-request "
                                   "tails (worker.ts:74-85 retry)"}
    # (2b) the same through the two-phase flow (what bench.py times and the multi-GPU path runs):
    # the combined check fails for every call.  LB_TP_RELEASE=1 (default) re-verifies the
    # shard as a one-phase call; LB_TP_RELEASE=0 keeps the slot and runs only the per-request
    # tails on the products already computed (the cost of the release's re-run)
    from lodestar_amd.native import Device

    def two_phase_bad(d):
        def one(k):
            tk = d.verify_requests_device_async(n_req, n, d_reqoff_, d_pk_, None, d_bad.data_ptr(), d_sig_, d_sigoff_,
                                                d_seed_, d_valid_[k % len(d_valid_)], d_err_[k % len(d_err_)],
                                                partial=True)
            return tk

        def resolve(tk):
            ok_ = d.gt_check([d.partial_wait_t(tk)])
            assert not ok_
            d.finish_t(tk, ok_)
            d.wait(tk)
        resolve(one(0))
        t1_ = time.perf_counter()
        pend_ = []
        for k in range(reps):
            pend_.append(one(k))
            if len(pend_) >= nbuf:
                resolve(pend_.pop(0))
        for tk in pend_:
            resolve(tk)
        torch.cuda.synchronize()
        return n * reps / (time.perf_counter() - t1_)
    d_reqoff_, d_pk_, d_sig_, d_sigoff_, d_seed_ = dev_ptrs
    keep_ =[torch.zeros(n_req, dtype=torch.uint8, device=cuda) for _ in range(2 * nbuf)]
    d_valid_ = [x.data_ptr() for x in keep_[:nbuf]]
    d_err_ = [x.data_ptr() for x in keep_[nbuf:]]
    rel = two_phase_bad(dev)
    bad_row = (n // 2) // a.per_request
    got = keep_[0].cpu().numpy()
    assert not got[bad_row] and got.sum() == n_req - 1, "two-phase adversarial verdicts"
    other = {}
    for name, env in (("release_only", {"LB_TP_PAUSE": "0"}), ("legacy", {"LB_TP_RELEASE": "0"})):
        saved = {k: os.environ.get(k) for k in list(env) + ["LB_PRIO_CUS"]}
        os.environ.update(env, LB_PRIO_CUS="0")
        try:
            od = Device(dev.device)
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        try:
            other[name] = two_phase_bad(od)
        finally:
            od.close()
    legs["adversarial_two_phase"] = {
        "sets_per_s": round(rel, 1), "sets_per_s_release_only": round(other["release_only"], 1),
        "sets_per_s_legacy": round(other["legacy"], 1), "calls": reps,
        "case": "one wrong-message set per 65,536-set two-phase call: the combined check fails every time. "
                "Default context: released calls, and after a failed combine the next 32 two-phase calls in the "
                "legacy mode (LB_TP_PAUSE); release_only (LB_TP_PAUSE=0): every failed shard re-verified as a "
                "one-phase call; legacy (LB_TP_RELEASE=0): the slot held, only the per-request tails run"}
    # (3) same-message gossip jobs: 512 attestation-data groups x 128 validators per call, pubkeys by index
    from lodestar_amd.native import Device  # noqa: F401
    n_jobs, per_job = 512, 128
    roots = [hashlib.sha256(b"attdata" + j.to_bytes(4, "little")).digest() for j in range(n_jobs)]
    if dev.pubkey_table_size() < len(pks):
        dev.pubkey_table_append(pks)
    rng = np.random.default_rng(3)
    members = [rng.choice(len(pks), per_job, replace=False) for _ in range(n_jobs)]
    flat_sk = [sks[int(v)] for m in members for v in m]
    flat_msg = [roots[j] for j in range(n_jobs) for _ in range(per_job)]
    sm_sigs = []
    for s in range(0, len(flat_sk), 16384):
        sm_sigs += dev.sign(flat_sk[s:s + 16384], flat_msg[s:s + 16384])
    jobs = [([int(v) for v in members[j]], sm_sigs[j * per_job:(j + 1) * per_job], roots[j]) for j in range(n_jobs)]
    res, fast, _ = dev.verify_same_message_batch(jobs, seed, by_index=True)
    assert all(fast) and all(all(r) for r in res)
    lat = []
    for _ in range(max(3, reps // 2)):
        t1 = time.perf_counter()
        dev.verify_same_message_batch(jobs, seed, by_index=True)
        lat.append(time.perf_counter() - t1)
    sm_stage = {k: round(v, 3) for k, v in dev.last_stage_times()}
    legs["same_message"] = {"sets_per_s": round(n_jobs * per_job / float(np.median(lat)), 1),
                            "ms_per_call": round(float(np.median(lat)) * 1e3, 3), "jobs": n_jobs,
                            "sets_per_job": per_job,
                            "api": "lb_verify_same_message_batch (host buffers, validator indices, one call)",
                            "stage_ms": sm_stage}
    # (4) the same packages kept in flight (lb_verify_same_message_batch_async, what the pool's
    # submission thread does): packed once, nbuf packages in flight, PCIe included
    prep = dev.prepare_same_message(jobs, seed, by_index=True)
    for pc in [dev.verify_same_message_prepared_async(prep) for _ in range(nbuf)]:
        assert all(dev.wait_same_message(pc)[1])
    t1 = time.perf_counter()
    pend, allv = [], True
    for _ in range(reps):
        pend.append(dev.verify_same_message_prepared_async(prep))
        if len(pend) >= nbuf:
            allv &= all(dev.wait_same_message(pend.pop(0))[1])
    for pc in pend:
        allv &= all(dev.wait_same_message(pc)[1])
    el = time.perf_counter() - t1
    legs["same_message_inflight"] = {"sets_per_s": round(n_jobs * per_job * reps / el, 1), "packages": reps,
                                     "all_fast": bool(allv), "jobs": n_jobs, "sets_per_job": per_job,
                                     "api": f"lb_verify_same_message_batch_async, {nbuf} packages in flight "
                                            "(host buffers, validator indices)"}
    return legs


def _progress(msg):
    """A line on stderr per leg (a long run shows it is alive; stdout carries only the JSON line)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _p50(fn, reps):
    ts = []
    for _ in range(reps):
        t1 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t1) * 1e3)
    return float(np.median(ts))


def _config_roof(oc_w, key, sets_per_s, keys_per_set):
    """A config's whole-pipeline fraction of the mad peak: its own measured mads per set
    (tools/opcount.py --workload, profiles/op_counts_workloads.json) x sets/s."""
    c = (oc_w or {}).get(key)
    if not c:
        return None
    tot = c["mads_per_set_total"]
    return {"bound": "valu", "unit": "Tmad/s", "mads_per_set": round(tot), "keys_per_set": round(keys_per_set, 2),
            "achieved": round(sets_per_s * tot / 1e12, 4), "peak": round(PEAK_MAD_PER_S / 1e12, 3),
            "frac": round(sets_per_s * tot / PEAK_MAD_PER_S, 5),
            "counts": "profiles/op_counts_workloads.json[%s] (counting build, this config's shape)" % key}


def config_legs(a, dev, torch, cuda, sks, pks, msgs, sigs, nbuf):
    """Every other BASELINE.json config and the reference's perf-suite sizes
    (BNT/perf/bls/bls.test.ts:56-122), timed after the C2 measurement (reported, never
    `value`):
      c3       2048-key committee aggregation (PublicKey.aggregate, chain/bls/utils.ts:13) and
               the 512-key sync-committee aggregate verify (one 1-set request);
      c4_shard one GPU's 1/8 of the 1 M mixed gossip sets (125,000 sets: 112,712 attestations +
               4,096 AggregateAndProof triples with 488-key aggregates, 977 requests of 128),
               pubkeys by validator index, device-resident inputs, `nbuf` calls in flight; plus
               the node leg's C4 package shape (220 x 128 singles + 1,024 triples) through the
               Python host, the GPU-bound ceiling of node's c4_public_key_objects leg;
      c5       the 32-block epoch of block import (147 sets per block: proposer, RANDAO, 128
               aggregates of 488 keys, the 512-key sync aggregate, 16 exits; one request per
               block, verifyBlocksSignatures.ts:38-55) with invalid sets injected at 1e-3 --
               the blocks holding one are false, every other block true;
      sizes    verifyMultipleSignatures {3, 8, 32, 64, 128} (one request), same-message
               {3, ..., 128} (one job), aggregatePubkeys {32, 128}, deserializing 10k / 100k
               signatures with validation."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import workloads as W
    from lodestar_amd.native import pack_blobs
    out = {}
    reps = max(5, a.latency_reps)
    nv = len(pks)
    seed = hashlib.sha256(b"batch-rand").digest()
    oc_w = None
    p = os.path.join(ROOT, "profiles", "op_counts_workloads.json")
    if os.path.exists(p):
        oc_w = json.load(open(p))
    # validator i's key at table index i (the secondary legs appended the C2 keys to a fresh table)
    if dev.pubkey_table_size() == 0:
        dev.pubkey_table_append(pks)
    assert dev.pubkey_table_read(0, 1)[0] == pks[0] and dev.pubkey_table_size() >= nv
    keys = W.Keys([int.from_bytes(s, "big") for s in sks], list(pks))
    rng = np.random.default_rng(5)

    _progress("config legs: C3")
    # ---- C3 ------------------------------------------------------------------------------
    t_gen = time.time()
    com = rng.choice(nv, 2048, replace=False).astype(np.uint32)
    com_b = [pks[int(i)] for i in com]
    agg = dev.aggregate_pubkeys(com_b)
    assert agg == dev.aggregate_pubkeys_indexed(com)
    sync = rng.choice(nv, 512, replace=False).astype(np.uint32)
    root = hashlib.sha256(b"sync-committee-c3").digest()
    sync_sig = W.sign_many(dev, [sum(keys.sks[int(i)] for i in sync) % R_ORDER], [root])[0]
    blob1, offs1 = pack_blobs([sync_sig])
    req1, pko1 = np.array([0, 1], np.uint32), np.array([0, 512], np.uint32)
    mg1 = np.frombuffer(root, np.uint8)

    def sync_verify():
        r = dev.verify_requests(req1, None, pko1, mg1, blob1, offs1, seed, pk_indices=sync)
        assert bool(r.valid[0]) and not r.errors.any()
    sync_verify()
    sync_verify_b = np.frombuffer(b"".join(pks[int(i)] for i in sync), np.uint8)

    def sync_verify_bytes():
        r = dev.verify_requests(req1, sync_verify_b, pko1, mg1, blob1, offs1, seed)
        assert bool(r.valid[0])
    sync_verify_bytes()
    out["c3"] = {"config": "C3: 2048-key committee aggregation + 512-key sync-committee aggregate verify",
                 "aggregate_2048_bytes_p50_ms": round(_p50(lambda: dev.aggregate_pubkeys(com_b), reps), 3),
                 "aggregate_2048_indexed_p50_ms": round(_p50(lambda: dev.aggregate_pubkeys_indexed(com), reps), 3),
                 "sync_aggregate_512_verify_indexed_p50_ms": round(_p50(sync_verify, reps), 3),
                 "sync_aggregate_512_verify_bytes_p50_ms": round(_p50(sync_verify_bytes, reps), 3),
                 "sync_verify_stage_ms": {k: round(v, 3) for k, v in dev.last_stage_times()},
                 "api": "lb_aggregate_pubkeys[_indexed]; lb_verify_requests (host buffers, one 1-set request of "
                        "512 keys: the latency path)",
                 "datagen_s": round(time.time() - t_gen, 2)}

    _progress("config legs: C4 shard")
    # ---- C4: one GPU's shard ---------------------------------------------------------------
    t_gen = time.time()
    c4 = W.c4_shard(dev, keys)
    gen_c4 = time.time() - t_gen
    blob4, offs4 = c4.blobs()
    mg4 = c4.msg_array()
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x).copy()).to(cuda)  # noqa: E731
    d_req, d_pko, d_idx = t(c4.req_off.view(np.int32)), t(c4.pk_off.view(np.int32)), t(c4.idx.view(np.int32))
    d_msg, d_sig, d_sigo, d_seed = t(mg4), t(blob4), t(offs4.view(np.int32)), t(np.frombuffer(seed, np.uint8))
    nr4, ns4 = c4.n_req, c4.n_sets
    outs = [(torch.zeros(nr4, dtype=torch.uint8, device=cuda), torch.zeros(nr4, dtype=torch.uint8, device=cuda))
            for _ in range(nbuf)]
    torch.cuda.synchronize()

    def submit4(k):
        v, e = outs[k % nbuf]
        return dev.verify_requests_device_async(nr4, ns4, d_req.data_ptr(), 0, d_pko.data_ptr(), d_msg.data_ptr(),
                                                d_sig.data_ptr(), d_sigo.data_ptr(), d_seed.data_ptr(), v.data_ptr(),
                                                e.data_ptr(), d_pk_idx=d_idx.data_ptr())
    for tk in [submit4(k) for k in range(nbuf)]:  # every slot's workspace sized for the shard
        dev.wait(tk)
    calls4 = max(nbuf, 2 * a.steps // 3)
    t1 = time.perf_counter()
    pend = []
    for k in range(calls4):
        pend.append(submit4(k))
        if len(pend) >= nbuf:
            dev.wait(pend.pop(0))
    for tk in pend:
        dev.wait(tk)
    torch.cuda.synchronize()
    el4 = time.perf_counter() - t1
    ok4 = all(bool(v.cpu().numpy().all()) and not bool(e.cpu().numpy().any()) for v, e in outs)
    lone4 = _p50(lambda: dev.verify_requests_device(nr4, ns4, d_req.data_ptr(), 0, d_pko.data_ptr(), d_msg.data_ptr(),
                                                    d_sig.data_ptr(), d_sigo.data_ptr(), d_seed.data_ptr(),
                                                    outs[0][0].data_ptr(), outs[0][1].data_ptr(),
                                                    d_pk_idx=d_idx.data_ptr()), 3)
    st4 = {k: round(v, 3) for k, v in dev.last_stage_times()}
    host4 = _p50(lambda: dev.verify_requests(c4.req_off, None, c4.pk_off, mg4, blob4, offs4, seed, pk_indices=c4.idx),
                 3)
    rate4 = ns4 * calls4 / el4
    kps4 = len(c4.idx) / ns4
    # the node leg's C4 package shape through the Python host (bench_node.js c4Leg): 220 jobs of
    # 128 single sets + 1,024 (selection proof, aggregator signature, 488-key aggregate) triples
    n_agg = 1024
    trip = [int(q) for q in np.nonzero(np.diff(c4.pk_off) > 1)[0][:n_agg]]
    singles = [int(q) for q in np.nonzero(np.diff(c4.pk_off) == 1)[0][:220 * 128 + 2 * n_agg]]
    sel = singles[:220 * 128]
    rest = singles[220 * 128:]
    order = sel + [q for a_ in range(n_agg) for q in (rest[2 * a_], rest[2 * a_ + 1], trip[a_])]
    req_n = np.array([0] + [128 * (j + 1) for j in range(220)] + [220 * 128 + 3 * (a_ + 1) for a_ in range(n_agg)],
                     np.uint32)
    pk_n = np.zeros(len(order) + 1, np.uint32)
    pk_n[1:] = np.cumsum([int(c4.pk_off[q + 1] - c4.pk_off[q]) for q in order])
    idx_n = np.concatenate([c4.idx[c4.pk_off[q]:c4.pk_off[q + 1]] for q in order]).astype(np.uint32)
    mg_n = np.frombuffer(b"".join(c4.msgs[q] for q in order), np.uint8)
    blob_n, offs_n = pack_blobs([c4.sigs[q] for q in order])
    pcs = [dev.verify_requests_async(req_n, None, pk_n, mg_n, blob_n, offs_n, seed, pk_indices=idx_n)
           for _ in range(nbuf)]
    assert all(bool(dev.wait_call(pc).valid.all()) for pc in pcs)
    t1 = time.perf_counter()
    pend, okn, calls_n = [], True, 2 * nbuf
    for _ in range(calls_n):
        pend.append(dev.verify_requests_async(req_n, None, pk_n, mg_n, blob_n, offs_n, seed, pk_indices=idx_n))
        if len(pend) >= nbuf:
            okn &= bool(dev.wait_call(pend.pop(0)).valid.all())
    for pc in pend:
        okn &= bool(dev.wait_call(pc).valid.all())
    el_n = time.perf_counter() - t1
    out["c4_shard"] = {
        "config": "C4: one GPU's 1/8 of 1M mixed gossip sets (BASELINE.json configs[3])",
        "sets": ns4, "requests": nr4, "pubkeys": int(len(c4.idx)), "keys_per_set": round(kps4, 2),
        "sets_per_s": round(rate4, 1), "ms_per_call": round(el4 / calls4 * 1e3, 3), "calls": calls4,
        "all_valid": ok4, "lone_call_ms": round(lone4, 3), "lone_call_stage_ms": st4,
        "host_indexed_call_ms": round(host4, 3), "host_indexed_sets_per_s": round(ns4 / host4 * 1e3, 1),
        "api": f"lb_verify_requests_device_async, validator indices, device-resident inputs, {nbuf} calls in flight",
        "roofline": _config_roof(oc_w, "c4_shard", rate4, kps4),
        "node_package_shape_python_host": {
            "sets_per_call": len(order), "requests": len(req_n) - 1, "calls": calls_n,
            "sets_per_s": round(len(order) * calls_n / el_n, 1), "all_valid": okn,
            "api": f"lb_verify_requests_async, host buffers, validator indices, {nbuf} calls in flight: the "
                   "package node's c4_public_key_objects leg sends, without JS"},
        "datagen_s": round(gen_c4, 2)}
    del d_req, d_pko, d_idx, d_msg, d_sig, d_sigo, outs

    _progress("config legs: C5 epoch")
    # ---- C5: block import, one 32-block epoch ----------------------------------------------
    t_gen = time.time()
    c5 = W.c5_epoch(dev, keys)
    gen_c5 = time.time() - t_gen
    blob5, offs5 = c5.blobs()
    mg5 = c5.msg_array()
    want = [k not in c5.expect_invalid_requests for k in range(c5.n_req)]

    def c5_host():
        r = dev.verify_requests(c5.req_off, None, c5.pk_off, mg5, blob5, offs5, seed, pk_indices=c5.idx)
        assert [bool(v) for v in r.valid] == want, "C5 block verdicts"
        return r
    r5 = c5_host()
    host5 = _p50(c5_host, reps)
    st5_host = {k: round(v, 3) for k, v in dev.last_stage_times()}
    d5 = [t(c5.req_off.view(np.int32)), t(c5.pk_off.view(np.int32)), t(c5.idx.view(np.int32)), t(mg5), t(blob5),
          t(offs5.view(np.int32)), t(np.frombuffer(seed, np.uint8))]
    v5 = torch.zeros(c5.n_req, dtype=torch.uint8, device=cuda)
    e5 = torch.zeros(c5.n_req, dtype=torch.uint8, device=cuda)
    torch.cuda.synchronize()

    def c5_dev():
        return dev.verify_requests_device(c5.n_req, c5.n_sets, d5[0].data_ptr(), 0, d5[1].data_ptr(), d5[3].data_ptr(),
                                          d5[4].data_ptr(), d5[5].data_ptr(), d5[6].data_ptr(), v5.data_ptr(),
                                          e5.data_ptr(), d_pk_idx=d5[2].data_ptr())
    c5_dev()
    dev5 = _p50(c5_dev, reps)
    st5 = {k: round(v, 3) for k, v in dev.last_stage_times()}
    assert [bool(v) for v in v5.cpu().numpy()] == want, "C5 block verdicts (device inputs)"
    kps5 = len(c5.idx) / c5.n_sets
    out["c5"] = {
        "config": "C5: block import, 32-block epoch, 147 sets per block, invalid sets injected at 1e-3",
        "blocks": c5.n_req, "sets": c5.n_sets, "pubkeys": int(len(c5.idx)), "keys_per_set": round(kps5, 2),
        "invalid_blocks": sorted(c5.expect_invalid_requests), "verdicts_match": True,
        "batch_retries": r5.batch_retries,
        "epoch_ms_p50_device_inputs": round(dev5, 3), "sets_per_s": round(c5.n_sets / dev5 * 1e3, 1),
        "epoch_ms_p50_host_indexed": round(host5, 3),
        "stage_ms": st5, "stage_ms_host": st5_host,
        "roofline": _config_roof(oc_w, "c5", c5.n_sets / dev5 * 1e3, kps5),
        "api": "lb_verify_requests_device (one synchronous call per epoch, validator indices, inputs in HBM) and "
               "lb_verify_requests (host buffers)",
        "datagen_s": round(gen_c5, 2)}
    # the same epoch before the injection: every block valid, no per-request failure path
    b5v, o5v = pack_blobs(c5.clean_sigs)
    m5v = np.frombuffer(b"".join(c5.clean_msgs), np.uint8)

    def c5_valid():
        r = dev.verify_requests(c5.req_off, None, c5.pk_off, m5v, b5v, o5v, seed, pk_indices=c5.idx)
        assert r.valid.all()
    c5_valid()
    out["c5"]["all_valid_epoch_ms_p50_host_indexed"] = round(_p50(c5_valid, reps), 3)
    out["c5"]["all_valid_stage_ms_host"] = {k: round(v, 3) for k, v in dev.last_stage_times()}
    del d5, v5, e5

    _progress("config legs: perf-suite sizes")
    # ---- the reference's perf-suite sizes (bls.test.ts:56-122) ------------------------------
    sizes = {}
    lat1 = []
    for nset in (1, 3, 8, 32, 64, 128):
        ro = np.array([0, nset], np.uint32)
        pk_h = np.frombuffer(b"".join(pks[:nset]), np.uint8)
        mg_h = np.frombuffer(b"".join(msgs[:nset]), np.uint8)
        bl, of = pack_blobs(sigs[:nset])

        def one():
            r = dev.verify_requests(ro, pk_h, None, mg_h, bl, of, seed)
            assert bool(r.valid[0])
        one()
        ms = _p50(one, reps)
        key = "verify_1" if nset == 1 else f"verifyMultipleSignatures_{nset}"
        sizes[key] = {"p50_ms": round(ms, 3), "sets_per_s": round(nset / ms * 1e3, 1)}
    root_sm = hashlib.sha256(b"same-message-perf").digest()
    sm_sigs = W.sign_many(dev, keys.sks[:128], [root_sm] * 128)
    for nset in (3, 8, 32, 64, 128):
        def sm():
            v, fast = dev.verify_same_message(pks[:nset], sm_sigs[:nset], root_sm, seed)
            assert all(v) and fast
        sm()
        ms = _p50(sm, reps)
        sizes[f"sameMessage_{nset}"] = {"p50_ms": round(ms, 3), "sets_per_s": round(nset / ms * 1e3, 1)}
    for nk in (32, 128):
        ks = pks[:nk]
        sizes[f"aggregatePubkeys_{nk}"] = {"p50_ms": round(_p50(lambda: dev.aggregate_pubkeys(ks), reps), 3)}
    for nsig in (10_000, 100_000):
        bl, of = pack_blobs([sigs[i % 256] for i in range(nsig)])  # (getSet(i % 256), bls.test.ts:82)
        buf = np.zeros(nsig * 192, np.uint8)
        assert not dev.decode_signatures_packed(bl, of, buf).any()
        ms = _p50(lambda: dev.decode_signatures_packed(bl, of, buf), reps)
        sizes[f"deserializing_{nsig}"] = {"p50_ms": round(ms, 3), "signatures_per_s": round(nsig / ms * 1e3, 1)}
    out["sizes"] = {"suite": "BNT/perf/bls/bls.test.ts:56-122 shapes (one call each, host buffers, synchronous; "
                             "1..128-set calls take the latency path)", **sizes}
    return out


if __name__ == "__main__":
    main()
