"""Synthetic workloads of BASELINE.json configs C4 and C5 (shared by the GPU
parity tests, bench.py's config legs and tools/opcount.py --workloads).

Keys are the interop keys sk_i = LE(sha256(LE32(i))) mod r
(packages/state-transition/src/util/interop.ts:19-23); signatures come from the
GPU signer (lb_sign, pinned bit-for-bit to the oracle by the KAT tests);
aggregate signatures are signed with the summed secret key, so they equal
Signature.aggregate of the members' signatures.

C4 shard (1M mixed sets / 8 GPUs = 125,000 per GPU): 112,712 single
    attestations + 4,096 AggregateAndProofs x (selection proof, aggregator
    signature, aggregate attestation over `committee` = 488 keys), shuffled into
    gossip arrival order, 128-set requests (index.ts:57).  Shapes:
    BN/chain/validation/aggregateAndProof.ts:200, ST/signatureSets/*.
C5 epoch (block import, verifyBlocksSignatures.ts:38-55): 32 blocks of
    proposer + RANDAO + 128 aggregate attestations (488 keys) + sync aggregate
    (512 keys) + 16 exits = 147 sets, one request per block
    (getBlockSignatureSets, ST/signatureSets/index.ts:26-73); signing roots
    computed on the GPU; invalid sets injected at 1e-3 (a wrong message as
    bls.test.ts:42, Buffer.alloc(96, 10) as bls.test.ts:48).
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass, field
from typing import List, Optional, Set

import numpy as np

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


def interop_sk(i: int) -> int:
    d = hashlib.sha256(i.to_bytes(32, "little")).digest()
    return int.from_bytes(d, "little") % R_ORDER


def be(k: int) -> bytes:
    return k.to_bytes(32, "big")


@dataclass
class Keys:
    sks: List[int]
    pks: List[bytes]  # 96-byte uncompressed


def make_keys(dev, n: int) -> Keys:
    sks = [interop_sk(i) for i in range(n)]
    pks: List[bytes] = []
    for s in range(0, n, 16384):
        pks += dev.sk_to_pk([be(k) for k in sks[s:s + 16384]])
    return Keys(sks, pks)


def sign_many(dev, sks: List[int], msgs: List[bytes]) -> List[bytes]:
    out: List[bytes] = []
    for s in range(0, len(sks), 16384):
        out += dev.sign([be(k) for k in sks[s:s + 16384]], msgs[s:s + 16384])
    return out


@dataclass
class Packed:
    """A call in the C-ABI layout (lb_request_batch)."""
    req_off: np.ndarray
    pk_off: np.ndarray
    idx: np.ndarray            # validator indices, pk_off[-1] of them
    msgs: List[bytes]
    sigs: List[bytes]
    expect_invalid_requests: Set[int] = field(default_factory=set)
    clean_msgs: Optional[List[bytes]] = None  # (c5_epoch: messages / signatures before the injection)
    clean_sigs: Optional[List[bytes]] = None

    @property
    def n_sets(self) -> int:
        return len(self.msgs)

    @property
    def n_req(self) -> int:
        return len(self.req_off) - 1

    def blobs(self):
        from lodestar_amd.native import pack_blobs
        return pack_blobs(self.sigs)

    def msg_array(self) -> np.ndarray:
        return np.frombuffer(b"".join(self.msgs), np.uint8)

    def pk_bytes(self, keys: Keys) -> np.ndarray:
        return np.frombuffer(b"".join(keys.pks[i] for i in self.idx), np.uint8)


def _pack(sets, req_size: Optional[int], req_off: Optional[np.ndarray] = None) -> Packed:
    n = len(sets)
    idx = np.array([i for ix, _, _ in sets for i in ix], np.uint32)
    pk_off = np.zeros(n + 1, np.uint32)
    pk_off[1:] = np.cumsum([len(ix) for ix, _, _ in sets])
    if req_off is None:
        req_off = np.arange(0, n + 1, req_size, dtype=np.uint32)
        if req_off[-1] != n:
            req_off = np.append(req_off, np.uint32(n))
    return Packed(req_off, pk_off, idx, [m for _, m, _ in sets], [s for _, _, s in sets])


def inject_invalid(p: Packed, positions, rng) -> None:
    """Corrupt set j (alternating kinds): a wrong signing root (bls.test.ts:42), malformed
    bytes Buffer.alloc(96, 10) (bls.test.ts:48), 32 zero bytes (multithread.test.ts:114-121),
    the infinite signature 0xc0.. (ST/constants/constants.ts:5-8, false in a 1-set request)."""
    for t, j in enumerate(positions):
        j = int(j)
        kind = t % 4
        if kind == 0:
            p.msgs[j] = hashlib.sha256(b"wrong" + j.to_bytes(4, "little")).digest()
        elif kind == 1:
            p.sigs[j] = bytes([10]) * 96
        elif kind == 2:
            p.sigs[j] = bytes(32)
        else:
            p.sigs[j] = bytes([0xC0]) + bytes(95)
        k = int(np.searchsorted(p.req_off, j, side="right")) - 1
        p.expect_invalid_requests.add(k)


def c4_shard(dev, keys: Keys, singles: int = 112712, aggregates: int = 4096, committee: int = 488, seed: int = 7,
             n_invalid: int = 0) -> Packed:
    rng = np.random.default_rng(seed)
    nv = len(keys.sks)
    sks = keys.sks
    plan = []  # (indices, msg, signing key)
    for k, v in enumerate(rng.integers(0, nv, singles)):
        plan.append(([int(v)], hashlib.sha256(b"att" + k.to_bytes(8, "little")).digest(), sks[v]))
    for g in range(aggregates):
        agg_v = int(rng.integers(0, nv))
        members = rng.choice(nv, committee, replace=False)
        plan.append(([agg_v], hashlib.sha256(b"sel" + g.to_bytes(8, "little")).digest(), sks[agg_v]))
        plan.append(([agg_v], hashlib.sha256(b"aap" + g.to_bytes(8, "little")).digest(), sks[agg_v]))
        plan.append(([int(m) for m in members], hashlib.sha256(b"agg" + g.to_bytes(8, "little")).digest(),
                     sum(sks[m] for m in members) % R_ORDER))
    order = rng.permutation(len(plan))  # gossip arrival order
    plan = [plan[i] for i in order]
    sigs = sign_many(dev, [k for _, _, k in plan], [m for _, m, _ in plan])
    p = _pack([(ix, m, s) for (ix, m, _), s in zip(plan, sigs)], 128)
    if n_invalid:
        inject_invalid(p, rng.choice(len(plan), n_invalid, replace=False), rng)
    return p


def c5_epoch(dev, keys: Keys, blocks: int = 32, committee: int = 488, seed: int = 11,
             invalid_rate: float = 1e-3) -> Packed:
    rng = np.random.default_rng(seed)
    nv = len(keys.sks)
    dom = rng.bytes(32)
    att_roots = dev.signing_roots_attestation([rng.bytes(128) for _ in range(blocks * 128)], dom)
    hdr = dev.signing_roots_chunks([[rng.bytes(32) for _ in range(5)] for _ in range(blocks)], dom)
    rnd_roots = dev.signing_roots_chunks([[int(e).to_bytes(8, "little") + bytes(24)] for e in range(blocks)], dom)
    exit_roots = dev.signing_roots_chunks([[int(e).to_bytes(8, "little") + bytes(24),
                                            int(v).to_bytes(8, "little") + bytes(24)]
                                           for e, v in zip(range(blocks * 16), rng.integers(0, nv, blocks * 16))],
                                          dom)
    sync_roots = dev.signing_roots_chunks([[rng.bytes(32)] for _ in range(blocks)], dom)
    plan = []
    for bi in range(blocks):
        prop = int(rng.integers(0, nv))
        plan += [([prop], hdr[bi]), ([prop], rnd_roots[bi])]
        for k in range(128):
            plan.append(([int(m) for m in rng.choice(nv, committee, replace=False)], att_roots[bi * 128 + k]))
        plan.append(([int(m) for m in rng.choice(nv, 512, replace=False)], sync_roots[bi]))
        for k in range(16):
            plan.append(([int(rng.integers(0, nv))], exit_roots[bi * 16 + k]))
    per_block = 147
    sigs = sign_many(dev, [sum(keys.sks[i] for i in ix) % R_ORDER for ix, _ in plan], [m for _, m in plan])
    req_off = np.arange(0, len(plan) + 1, per_block, dtype=np.uint32)
    p = _pack([(ix, m, s) for (ix, m), s in zip(plan, sigs)], None, req_off)
    p.clean_msgs, p.clean_sigs = list(p.msgs), list(p.sigs)  # (the same epoch before the injection)
    if invalid_rate <= 0:
        return p
    n_bad = max(2, int(round(len(plan) * invalid_rate)))
    pos = rng.choice(len(plan), n_bad, replace=False)
    # only the two kinds the reference's bls.test.ts uses for block import (wrong root, malformed)
    for t, j in enumerate(pos):
        j = int(j)
        if t % 2 == 0:
            p.msgs[j] = hashlib.sha256(b"wrong" + j.to_bytes(4, "little")).digest()
        else:
            p.sigs[j] = bytes([10]) * 96
        p.expect_invalid_requests.add(j // per_block)
    return p


def same_message_jobs(dev, keys: Keys, n_jobs: int = 512, per_job: int = 128, seed: int = 13, n_invalid: int = 0):
    """Gossip attestations grouped by AttestationData (validateGossipAttestationsSameAttData,
    BN/chain/validation/attestation.ts:82-176): job j = per_job distinct validators
    signing one root.  Invalid sets: another validator's signature over the same root
    (validateGossipAttestationsSameAttData.test.ts:91), malformed bytes, the infinite
    signature.  Returns (jobs as (indices, sigs, message), expected per-set verdicts)."""
    rng = np.random.default_rng(seed)
    nv = len(keys.sks)
    roots = [hashlib.sha256(b"attdata" + j.to_bytes(4, "little")).digest() for j in range(n_jobs)]
    members = [rng.choice(nv, per_job, replace=False) for _ in range(n_jobs)]
    sigs = sign_many(dev, [keys.sks[int(v)] for m in members for v in m],
                     [roots[j] for j in range(n_jobs) for _ in range(per_job)])
    jobs, expect = [], []
    for j in range(n_jobs):
        s = sigs[j * per_job:(j + 1) * per_job]
        jobs.append(([int(v) for v in members[j]], list(s), roots[j]))
        expect.append([True] * per_job)
    if n_invalid:
        for t, f in enumerate(rng.choice(n_jobs * per_job, n_invalid, replace=False)):
            j, i = divmod(int(f), per_job)
            kind = t % 3
            if kind == 0:
                jobs[j][1][i] = jobs[j][1][(i + 1) % per_job]
            elif kind == 1:
                jobs[j][1][i] = bytes([10]) * 96
            else:
                jobs[j][1][i] = bytes([0xC0]) + bytes(95)
            expect[j][i] = False
    return jobs, expect
