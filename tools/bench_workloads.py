"""Secondary workloads (BASELINE.json configs C3 and one GPU's shard of C4), with
pubkeys shipped as bytes (the worker wire format) vs as validator indices into
the device-resident pubkey table.

C3: aggregate a 2048-key committee (PublicKey.aggregate, chain/bls/utils.ts:13)
    and verify a 512-key sync-committee aggregate set (1-set request).
C4 shard: 1M mixed sets / 8 GPUs = 125,000 sets per GPU: 112,712 single
    attestations + 4,096 AggregateAndProofs x (selection proof, aggregator
    signature, aggregate attestation over 488 keys), in 128-set requests.
    Each is timed (a) through the host-buffer API (PCIe included, how the
    beacon node would call it) with 96-byte pubkeys, (b) the same with u32
    indices, (c) device-resident indices (inputs in HBM).

Usage (GPU box): python tools/bench_workloads.py [--reps 5] > profiles/workloads_rNN.json
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


def interop_sk(i: int) -> int:
    d = hashlib.sha256(i.to_bytes(32, "little")).digest()
    return int.from_bytes(d, "little") % R_ORDER


def be(k: int) -> bytes:
    return k.to_bytes(32, "big")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--validators", type=int, default=65536)
    ap.add_argument("--singles", type=int, default=112712)
    ap.add_argument("--aggregates", type=int, default=4096)
    ap.add_argument("--committee", type=int, default=488)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()

    import torch
    from lodestar_amd.native import Device, pack_blobs

    dev = Device(0)
    rng = np.random.default_rng(7)
    nv = a.validators
    t0 = time.time()
    sks = [interop_sk(i) for i in range(nv)]
    pks = []
    for s in range(0, nv, 16384):
        pks += dev.sk_to_pk([be(k) for k in sks[s:s + 16384]])
    assert dev.pubkey_table_append(pks) == nv
    gen_keys_s = time.time() - t0

    def sign_many(sk_list, msgs):
        out = []
        for s in range(0, len(sk_list), 16384):
            out += dev.sign([be(k) for k in sk_list[s:s + 16384]], msgs[s:s + 16384])
        return out

    # ---- C3 -------------------------------------------------------------------------
    com = rng.choice(nv, 2048, replace=False).astype(np.uint32)
    agg_bytes = dev.aggregate_pubkeys([pks[i] for i in com])
    agg_idx = dev.aggregate_pubkeys_indexed(com)
    assert agg_bytes == agg_idx
    t_b, t_i = [], []
    for _ in range(a.reps):
        t1 = time.perf_counter()
        dev.aggregate_pubkeys([pks[i] for i in com])
        t_b.append((time.perf_counter() - t1) * 1e3)
        t1 = time.perf_counter()
        dev.aggregate_pubkeys_indexed(com)
        t_i.append((time.perf_counter() - t1) * 1e3)
    sync = rng.choice(nv, 512, replace=False).astype(np.uint32)
    root = hashlib.sha256(b"sync-committee").digest()
    sync_sig = sign_many([sum(sks[i] for i in sync) % R_ORDER], [root])[0]
    blob, offs = pack_blobs([sync_sig])
    req1, pko1 = np.array([0, 1], np.uint32), np.array([0, 512], np.uint32)
    lat_sync = []
    for _ in range(a.reps):
        t1 = time.perf_counter()
        r = dev.verify_requests(req1, None, pko1, np.frombuffer(root, np.uint8), blob, offs, bytes(32), pk_indices=sync)
        lat_sync.append((time.perf_counter() - t1) * 1e3)
        assert bool(r.valid[0])
    c3 = {"aggregate_2048_bytes_ms_p50": round(float(np.median(t_b)), 3),
          "aggregate_2048_indexed_ms_p50": round(float(np.median(t_i)), 3),
          "sync_aggregate_512_verify_indexed_ms_p50": round(float(np.median(lat_sync)), 3),
          "aggregate_bit_exact_bytes_vs_indexed": True}

    # ---- C4 shard -------------------------------------------------------------------
    t0 = time.time()
    sets = []  # (indices, msg, sk)
    single_v = rng.integers(0, nv, a.singles)
    for k, v in enumerate(single_v):
        sets.append(([int(v)], hashlib.sha256(b"att" + k.to_bytes(8, "little")).digest(), sks[v]))
    for g in range(a.aggregates):
        agg_v = int(rng.integers(0, nv))
        members = rng.choice(nv, a.committee, replace=False)
        sets.append(([agg_v], hashlib.sha256(b"sel" + g.to_bytes(8, "little")).digest(), sks[agg_v]))
        sets.append(([agg_v], hashlib.sha256(b"aap" + g.to_bytes(8, "little")).digest(), sks[agg_v]))
        sets.append(([int(m) for m in members], hashlib.sha256(b"agg" + g.to_bytes(8, "little")).digest(),
                     sum(sks[m] for m in members) % R_ORDER))
    order = rng.permutation(len(sets))  # gossip arrival order
    sets = [sets[i] for i in order]
    n = len(sets)
    msgs = [m for _, m, _ in sets]
    sigs = sign_many([k for _, _, k in sets], msgs)
    idx = np.array([i for ix, _, _ in sets for i in ix], np.uint32)
    pk_off = np.zeros(n + 1, np.uint32)
    pk_off[1:] = np.cumsum([len(ix) for ix, _, _ in sets])
    req_off = np.arange(0, n + 1, 128, dtype=np.uint32)
    if req_off[-1] != n:
        req_off = np.append(req_off, np.uint32(n))
    pk_bytes = np.frombuffer(b"".join(pks[i] for i in idx), np.uint8)
    mg = np.frombuffer(b"".join(msgs), np.uint8)
    blob, offs = pack_blobs(sigs)
    gen_c4_s = time.time() - t0

    def host_call(by_index):
        return dev.verify_requests(req_off, None if by_index else pk_bytes, pk_off, mg, blob, offs, bytes(32),
                                   pk_indices=idx if by_index else None)

    res = {}
    for name, by_index in (("host_bytes", False), ("host_indexed", True)):
        r = host_call(by_index)
        assert r.valid.all() and not r.errors.any(), name
        ts = []
        for _ in range(a.reps):
            t1 = time.perf_counter()
            host_call(by_index)
            ts.append(time.perf_counter() - t1)
        res[name] = {"sets_per_s": round(n / float(np.median(ts)), 1), "ms": round(float(np.median(ts)) * 1e3, 3),
                     "h2d_pubkey_bytes": int(idx.nbytes if by_index else pk_bytes.nbytes)}
        if by_index:
            res[name]["stage_ms"] = {k: round(v, 3) for k, v in dev.last_stage_times()}
    # device-resident indices, calls in flight
    cuda = torch.device("cuda", 0)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(cuda)  # noqa: E731
    d_req, d_pko, d_idx = t(req_off.view(np.int32)), t(pk_off.view(np.int32)), t(idx.view(np.int32))
    d_msg, d_sig, d_sigo = t(mg), t(blob), t(offs.view(np.int32))
    d_seed = t(np.zeros(32, np.uint8))
    nr = len(req_off) - 1
    outs = [(torch.zeros(nr, dtype=torch.uint8, device=cuda), torch.zeros(nr, dtype=torch.uint8, device=cuda))
            for _ in range(3)]
    torch.cuda.synchronize()

    def submit(k):
        v, e = outs[k % 3]
        return dev.verify_requests_device_async(nr, n, d_req.data_ptr(), 0, d_pko.data_ptr(), d_msg.data_ptr(),
                                                d_sig.data_ptr(), d_sigo.data_ptr(), d_seed.data_ptr(), v.data_ptr(),
                                                e.data_ptr(), d_pk_idx=d_idx.data_ptr())
    dev.wait(submit(0))
    steps = max(a.reps, 3)
    t1 = time.perf_counter()
    pend = []
    for k in range(steps):
        pend.append(submit(k))
        if len(pend) >= 3:
            dev.wait(pend.pop(0))
    for p in pend:
        dev.wait(p)
    torch.cuda.synchronize()
    el = time.perf_counter() - t1
    ok = all(bool(v.cpu().numpy().all()) and not bool(e.cpu().numpy().any()) for v, e in outs)
    res["device_indexed_inflight"] = {"sets_per_s": round(n * steps / el, 1), "ms_per_call": round(el / steps * 1e3, 3),
                                      "all_valid": ok}
    # signing roots of the shard's attestations (the step before the verifier)
    att = [rng.bytes(128) for _ in range(n)]
    dom = rng.bytes(32)
    dev.signing_roots_attestation(att, dom)
    ts = []
    for _ in range(a.reps):
        t1 = time.perf_counter()
        dev.signing_roots_attestation(att, dom)
        ts.append(time.perf_counter() - t1)
    ssz = {"attestation_signing_roots": n, "host_call_ms_p50": round(float(np.median(ts)) * 1e3, 3),
           "roots_per_s": round(n / float(np.median(ts)), 1)}
    # ---- C5: block import, one 32-block epoch --------------------------------------
    # per block: proposer + RANDAO + 128 aggregate attestations (488 keys) + sync
    # aggregate (512 keys) + 16 exits = 147 sets, one request (verifySignatureSets
    # per block); signing roots computed on the GPU; invalid sets injected at 1e-3
    # (wrong message, malformed signature bytes) -> exactly those blocks are false.
    t0 = time.time()
    dom = rng.bytes(32)
    blocks, all_sets = 32, []
    att_data = [rng.bytes(128) for _ in range(blocks * 128)]
    att_roots = dev.signing_roots_attestation(att_data, dom)
    hdr = dev.signing_roots_chunks([[rng.bytes(32) for _ in range(5)] for _ in range(blocks)], dom)
    rnd_roots = dev.signing_roots_chunks([[int(e).to_bytes(8, "little") + bytes(24)] for e in range(blocks)], dom)
    exit_roots = dev.signing_roots_chunks([[int(e).to_bytes(8, "little") + bytes(24),
                                            int(v).to_bytes(8, "little") + bytes(24)]
                                           for e, v in zip(range(blocks * 16), rng.integers(0, nv, blocks * 16))], dom)
    sync_roots = dev.signing_roots_chunks([[rng.bytes(32)] for _ in range(blocks)], dom)
    for bi in range(blocks):
        prop = int(rng.integers(0, nv))
        bs = [([prop], hdr[bi]), ([prop], rnd_roots[bi])]
        for k in range(128):
            bs.append(([int(m) for m in rng.choice(nv, a.committee, replace=False)], att_roots[bi * 128 + k]))
        bs.append(([int(m) for m in rng.choice(nv, 512, replace=False)], sync_roots[bi]))
        for k in range(16):
            bs.append(([int(rng.integers(0, nv))], exit_roots[bi * 16 + k]))
        all_sets.append(bs)
    flat = [st for bs in all_sets for st in bs]
    c5_sigs = sign_many([sum(sks[i] for i in ix) % R_ORDER for ix, _ in flat], [m for _, m in flat])
    c5_msgs = [m for _, m in flat]
    bad_blocks = set()
    for j in rng.choice(len(flat), max(2, len(flat) // 1000), replace=False):
        j = int(j)
        bad_blocks.add(j // 147)
        if j % 2:
            c5_msgs[j] = hashlib.sha256(b"wrong" + j.to_bytes(4, "little")).digest()
        else:
            c5_sigs[j] = bytes([10]) * 96  # Buffer.alloc(96, 10), bls.test.ts:48
    c5_idx = np.array([i for ix, _ in flat for i in ix], np.uint32)
    c5_pko = np.zeros(len(flat) + 1, np.uint32)
    c5_pko[1:] = np.cumsum([len(ix) for ix, _ in flat])
    c5_req = np.arange(0, len(flat) + 1, 147, dtype=np.uint32)
    c5_blob, c5_offs = pack_blobs(c5_sigs)
    c5_mg = np.frombuffer(b"".join(c5_msgs), np.uint8)
    gen_c5_s = time.time() - t0
    r = dev.verify_requests(c5_req, None, c5_pko, c5_mg, c5_blob, c5_offs, bytes(32), pk_indices=c5_idx)
    expect = [bi not in bad_blocks for bi in range(blocks)]
    assert [bool(v) for v in r.valid] == expect, "C5 block verdicts"
    ts = []
    for _ in range(a.reps):
        t1 = time.perf_counter()
        dev.verify_requests(c5_req, None, c5_pko, c5_mg, c5_blob, c5_offs, bytes(32), pk_indices=c5_idx)
        ts.append(time.perf_counter() - t1)
    c5 = {"blocks": blocks, "sets": len(flat), "pubkeys": int(len(c5_idx)), "invalid_blocks": sorted(bad_blocks),
          "verdicts_match": True, "batch_retries": r.batch_retries, "epoch_ms_p50": round(float(np.median(ts)) * 1e3, 3),
          "sets_per_s": round(len(flat) / float(np.median(ts)), 1), "datagen_s": round(gen_c5_s, 2)}

    out = {"workloads": "C3 + C4 shard (1/8 of 1M mixed sets) + C5 epoch", "validators_in_table": nv, "ssz": ssz,
           "c5_block_import": c5,
           "c3": c3,
           "c4_shard": {"sets": n, "requests": nr, "pubkeys": int(len(idx)), "singles": a.singles,
                        "aggregate_and_proofs": a.aggregates, "committee": a.committee, **res},
           "datagen_s": {"keys": round(gen_keys_s, 2), "c4": round(gen_c4_s, 2)}}
    print(json.dumps(out), flush=True)
    dev.close()


if __name__ == "__main__":
    main()
