"""Multi-GPU path on one GPU: the two-phase calls that return each
shard's 576-byte Fp12 partial, the host combine (one final exponentiation for
all shards), ShardedVerifier over two contexts and verify_distributed as two
ranks (two processes) sharing cuda:0, against the unsharded verdicts; plus the
asynchronous host-buffer API with more calls than slots.
"""
import hashlib
import os
import random

import numpy as np
import pytest

from lodestar_amd.native import Device, LodestarBlsError, pack_blobs
from lodestar_amd.verifier import DeviceBackend, PublicKey, SignatureSet, SignatureSetType

pytestmark = pytest.mark.gpu


def _interop_sk_be(i):
    from oracle import bls12_381 as O
    return O.interop_secret_key(i).to_bytes(32, "big")


@pytest.fixture(scope="module")
def workload(device):
    """64 requests of 1..40 sets over 96 keys, some aggregates; `bad` holds the
    request indices with an injected wrong message."""
    rnd = random.Random(17)
    sks = [_interop_sk_be(i) for i in range(96)]
    pks = device.sk_to_pk(sks)
    reqs_plan = []
    for k in range(64):
        reqs_plan.append([rnd.sample(range(96), rnd.choice([1, 1, 1, 3])) for _ in range(rnd.randint(1, 40))])
    flat = [(k, ix) for k, r in enumerate(reqs_plan) for ix in r]
    msgs = [hashlib.sha256(b"mg" + j.to_bytes(4, "little")).digest() for j in range(len(flat))]
    from oracle import bls12_381 as O
    agg_sk = [(sum(int.from_bytes(sks[i], "big") for i in ix) % O.R).to_bytes(32, "big") for _, ix in flat]
    sigs = device.sign(agg_sk, msgs)
    requests = []
    j = 0
    for r in reqs_plan:
        req = []
        for ix in r:
            keys = [PublicKey(pks[i]) for i in ix]
            req.append(SignatureSet(SignatureSetType.single, msgs[j], sigs[j], pubkey=keys[0]) if len(keys) == 1 else
                       SignatureSet(SignatureSetType.aggregate, msgs[j], sigs[j], pubkeys=keys))
            j += 1
        requests.append(req)
    return requests


def _corrupt(requests, which):
    import copy
    out = copy.deepcopy(requests)
    for k in which:
        out[k][0].signing_root = bytes(32)
    return out


def _single_verdicts(requests):
    b = DeviceBackend(0, seed_source=lambda: bytes(32))
    try:
        return b.verify_requests(requests)
    finally:
        b.close()


@pytest.mark.parametrize("bad", [(), (5, 40)])
def test_sharded_verifier_fp12_combine(workload, bad):
    from lodestar_amd.sharding import ShardedVerifier
    reqs = _corrupt(workload, bad)
    want = _single_verdicts(reqs)
    assert want[0] == [k not in bad for k in range(len(reqs))]
    backs = [DeviceBackend(0, seed_source=lambda: bytes(32)) for _ in range(2)]
    try:
        sv = ShardedVerifier(backs)
        assert sv.combine
        assert sv.verify_requests(reqs) == want
        assert sv.last_combine == {"merged_ok": not bad, "n_partials": 2}
    finally:
        for b in backs:
            b.close()


def test_partials_device_api(device, workload):
    """lb_verify_requests_partial_async / lb_partial_wait / lb_gt_check /
    lb_verify_requests_finish directly: a valid shard's partial final-exps to 1,
    an invalid shard's does not, the product of both does not, empty -> 1."""
    reqs_ok = workload[:20]
    reqs_bad = _corrupt(workload[20:40], [3])

    def pack(reqs):
        pks, pk_off, msgs, sigs, req_off = [], [0], [], [], [0]
        for r in reqs:
            for s in r:
                keys = [s.pubkey] if s.pubkey is not None else s.pubkeys
                pks += [k.uncompressed for k in keys]
                pk_off.append(len(pks))
                msgs.append(s.signing_root)
                sigs.append(s.signature)
            req_off.append(len(msgs))
        blob, offs = pack_blobs(sigs)
        return (np.array(req_off, np.uint32), np.frombuffer(b"".join(pks), np.uint8), np.array(pk_off, np.uint32),
                np.frombuffer(b"".join(msgs), np.uint8), blob, offs)

    seed = bytes(32)
    a, b = pack(reqs_ok), pack(reqs_bad)
    pa = device.verify_requests_async(*a, seed, partial=True)
    pb = device.verify_requests_async(*b, seed, partial=True)
    Pa, Pb = device.partial_wait(pa), device.partial_wait(pb)
    assert len(Pa) == len(Pb) == 576
    assert device.gt_check([Pa]) is True
    assert device.gt_check([Pb]) is False
    assert device.gt_check([Pa, Pb]) is False
    assert device.gt_check([]) is True
    one = bytes(47) + b"\x01" + bytes(528)
    assert device.gt_check([one, Pa]) is True
    with pytest.raises(LodestarBlsError):
        device.gt_check([b"\xff" * 576])
    device.verify_finish(pa, True)   # combined verdict for shard a alone: valid
    device.verify_finish(pb, False)  # failed combine: per-request tails
    ra, rb = device.wait_call(pa), device.wait_call(pb)
    assert ra.valid.all() and ra.batch_retries == 0
    assert [bool(v) for v in rb.valid] == [k != 3 for k in range(20)] and rb.batch_retries == 1
    # a two-phase call waited for without finish resumes with merged_ok = 0 (verdicts still right)
    pc = device.verify_requests_async(*b, seed, partial=True)
    assert [bool(v) for v in device.wait_call(pc).valid] == [k != 3 for k in range(20)]


def test_async_host_api_more_calls_than_slots(device, workload):
    """lb_verify_requests_async: 10 calls in flight over 4 slots == the sync API, per call."""
    calls, want = [], []
    for t in range(10):
        reqs = _corrupt(workload[t * 5:t * 5 + 8], [t % 8] if t % 3 == 0 else [])
        want.append([not (t % 3 == 0 and k == t % 8) for k in range(len(reqs))])
        calls.append(reqs)

    def pack(reqs):
        pks, pk_off, msgs, sigs, req_off = [], [0], [], [], [0]
        for r in reqs:
            for s in r:
                keys = [s.pubkey] if s.pubkey is not None else s.pubkeys
                pks += [k.uncompressed for k in keys]
                pk_off.append(len(pks))
                msgs.append(s.signing_root)
                sigs.append(s.signature)
            req_off.append(len(msgs))
        blob, offs = pack_blobs(sigs)
        return (np.array(req_off, np.uint32), np.frombuffer(b"".join(pks), np.uint8), np.array(pk_off, np.uint32),
                np.frombuffer(b"".join(msgs), np.uint8), blob, offs)
    pcs = [device.verify_requests_async(*pack(r), bytes(32)) for r in calls]
    got = [[bool(v) for v in device.wait_call(pc).valid] for pc in pcs]
    assert got == want


def _rank(rank, world, port, reqs, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from lodestar_amd.sharding import verify_distributed
    b = DeviceBackend(0, seed_source=lambda: bytes(32))
    try:
        v, e = verify_distributed(reqs, None, rank, world, backend=b)
        q.put((rank, v, e))
        dist.barrier()
    finally:
        b.close()
        dist.destroy_process_group()


@pytest.mark.parametrize("bad", [(), (7,)])
def test_verify_distributed_two_ranks_one_gpu(workload, bad):
    """Two processes (ranks) on cuda:0: partials all-gathered over gloo, the same
    combined check on every rank, verdicts == the unsharded call."""
    import torch.multiprocessing as mp
    reqs = _corrupt(workload, bad)
    want = _single_verdicts(reqs)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + random.Random(os.getpid() + len(bad)).randrange(1000)
    procs = [ctx.Process(target=_rank, args=(r, 2, port, reqs, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, v, e in res:
        assert (v, e) == want


def test_async_lone_call_borrows_a_stream(device, workload):
    """A lone async call runs as the two-stream DAG on an idle slot's stream (lower
    latency); the next calls (one of which lands on the lent slot) wait for it and
    every verdict stays right; a two-phase call never borrows."""
    reqs = _corrupt(workload[:12], [4])
    want = [k != 4 for k in range(12)]
    pks, pk_off, msgs, sigs, req_off = [], [0], [], [], [0]
    for r in reqs:
        for s in r:
            keys = [s.pubkey] if s.pubkey is not None else s.pubkeys
            pks += [k.uncompressed for k in keys]
            pk_off.append(len(pks))
            msgs.append(s.signing_root)
            sigs.append(s.signature)
        req_off.append(len(msgs))
    blob, offs = pack_blobs(sigs)
    args = (np.array(req_off, np.uint32), np.frombuffer(b"".join(pks), np.uint8), np.array(pk_off, np.uint32),
            np.frombuffer(b"".join(msgs), np.uint8), blob, offs)
    for _ in range(3):
        pcs = [device.verify_requests_async(*args, bytes(32))]
        pcs += [device.verify_requests_async(*args, bytes(32)) for _ in range(device.slots() + 1)]
        assert all([bool(v) for v in device.wait_call(pc).valid] == want for pc in pcs)
    pp = device.verify_requests_async(*args, bytes(32), partial=True)
    lone = device.verify_requests_async(*args, bytes(32))
    assert [bool(v) for v in device.wait_call(lone).valid] == want
    device.verify_finish(pp, False)
    assert [bool(v) for v in device.wait_call(pp).valid] == want


def _pack_requests(reqs):
    pks, pk_off, msgs, sigs, req_off = [], [0], [], [], [0]
    for r in reqs:
        for s in r:
            keys = [s.pubkey] if s.pubkey is not None else s.pubkeys
            pks += [k.uncompressed for k in keys]
            pk_off.append(len(pks))
            msgs.append(s.signing_root)
            sigs.append(s.signature)
        req_off.append(len(msgs))
    blob, offs = pack_blobs(sigs)
    return (np.array(req_off, np.uint32), np.frombuffer(b"".join(pks), np.uint8), np.array(pk_off, np.uint32),
            np.frombuffer(b"".join(msgs), np.uint8), blob, offs)


def _dev_env(**env):
    from lodestar_amd.native import Device
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return Device(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.parametrize("gt_lp", ["1", "0"])
def test_partials_round_program_tail(workload, gt_lp):
    """Two-phase calls whose merged product comes from the round program (the bucket MSM
    forced on, LB_MTAIL=1: k_lp_mtail's partial form) and from the one-lane chain
    (LB_MTAIL=0): each mode's shard partials combine to the right verdict, partials of
    the two modes combine with each other (they differ only by factors the final
    exponentiation kills), and lb_gt_check's final exponentiation as a round program
    (LB_GT_LP=1) agrees with the one-wave chain (0)."""
    seed = bytes(32)
    ok_a, ok_b = _pack_requests(workload[:32]), _pack_requests(workload[32:])
    bad = _pack_requests(_corrupt(workload[32:], [7]))
    parts = {}
    for mtail in ("1", "0"):
        dev = _dev_env(LB_MSM_MIN="1", LB_MILLER="lines", LB_MTAIL=mtail, LB_GT_LP=gt_lp)
        try:
            pcs = [dev.verify_requests_async(*x, seed, partial=True) for x in (ok_a, ok_b, bad)]
            parts[mtail] = [dev.partial_wait(pc) for pc in pcs]
            Pa, Pb, Pbad = parts[mtail]
            assert dev.gt_check([Pa, Pb]) is True
            assert dev.gt_check([Pa, Pbad]) is False
            dev.verify_finish(pcs[0], True)
            dev.verify_finish(pcs[1], True)
            dev.verify_finish(pcs[2], False)
            r = [dev.wait_call(pc) for pc in pcs]
            assert r[0].valid.all() and r[1].valid.all()
            assert [bool(v) for v in r[2].valid] == [k != 7 for k in range(len(workload) - 32)]
        finally:
            dev.close()
    dev = _dev_env(LB_GT_LP=gt_lp)
    try:
        assert dev.gt_check([parts["1"][0], parts["0"][1]]) is True
        assert dev.gt_check([parts["0"][0], parts["1"][2]]) is False
    finally:
        dev.close()
