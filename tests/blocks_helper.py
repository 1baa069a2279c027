"""Test helper (TEST INFRASTRUCTURE): SSZ encoding of phase0/altair SignedBeaconBlocks
and an independent restatement of their hash_tree_root from the structured fields
(oracle/ssz.py primitives), plus a synthetic signed-block generator for the
getBlockSignatureSets tests.  The product parser (lodestar_amd/block_sets.py) reads
the bytes; this side never parses, it builds -- so the two meet only at the roots.

Layouts: SignedBeaconBlock{message: BeaconBlock, signature}, BeaconBlock{slot,
proposer_index, parent_root, state_root, body}, BeaconBlockBody phase0 {randao_reveal,
eth1_data, graffiti, proposer_slashings, attester_slashings, attestations, deposits,
voluntary_exits} (+ sync_aggregate in altair) -- the consensus-spec containers the
reference's @lodestar/types ssz definitions follow (packages/types/src/phase0/sszTypes.ts,
altair/sszTypes.ts).
"""
from __future__ import annotations

import hashlib
import os
import sys
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence, Tuple

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import ssz as S  # noqa: E402

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
le32 = lambda v: int(v).to_bytes(4, "little")  # noqa: E731
le64 = lambda v: int(v).to_bytes(8, "little")  # noqa: E731


def var_list(elems: Sequence[bytes]) -> bytes:
    off = 4 * len(elems)
    head, body = b"", b""
    for e in elems:
        head += le32(off + len(body))
        body += e
    return head + body


@dataclass
class Att:
    bits: bytes          # bitlist with delimiter
    data: bytes          # 128
    sig: bytes

    def ssz(self) -> bytes:
        return le32(228) + self.data + self.sig + self.bits

    def root(self) -> bytes:
        return S.merkleize([S.bitlist_root(self.bits, 2048), S.attestation_data_root(self.data),
                            S.bytes_vector_root(self.sig)])


@dataclass
class Indexed:
    indices: List[int]
    data: bytes
    sig: bytes

    def ssz(self) -> bytes:
        return le32(228) + self.data + self.sig + b"".join(le64(i) for i in self.indices)

    def root(self) -> bytes:
        packed = S.pack_bytes(b"".join(le64(i) for i in self.indices))
        return S.merkleize([S.mix_in_length(S.merkleize(packed, 512), len(self.indices)),
                            S.attestation_data_root(self.data), S.bytes_vector_root(self.sig)])


def header(slot, proposer, parent, state, body_root) -> bytes:
    return le64(slot) + le64(proposer) + parent + state + body_root


def header_root(h: bytes) -> bytes:
    return S.merkleize([S.u64(int.from_bytes(h[0:8], "little")), S.u64(int.from_bytes(h[8:16], "little")),
                        h[16:48], h[48:80], h[80:112]])


@dataclass
class Body:
    randao: bytes
    eth1: bytes = field(default_factory=lambda: bytes(72))
    graffiti: bytes = field(default_factory=lambda: bytes(32))
    proposer_slashings: List[Tuple[bytes, bytes, bytes, bytes]] = field(default_factory=list)  # h1, s1, h2, s2
    attester_slashings: List[Tuple[Indexed, Indexed]] = field(default_factory=list)
    attestations: List[Att] = field(default_factory=list)
    deposits: List[bytes] = field(default_factory=list)  # 1240 bytes each
    exits: List[Tuple[int, int, bytes]] = field(default_factory=list)
    sync: Optional[Tuple[bytes, bytes]] = None  # (64-byte bits, sig) altair

    def ssz(self) -> bytes:
        fixed = 220 + (160 if self.sync is not None else 0)
        parts = [b"".join(h1 + s1 + h2 + s2 for h1, s1, h2, s2 in self.proposer_slashings),
                 var_list([le32(8) + le32(8 + len(a.ssz())) + a.ssz() + b.ssz() for a, b in self.attester_slashings]),
                 var_list([a.ssz() for a in self.attestations]),
                 b"".join(self.deposits),
                 b"".join(le64(e) + le64(v) + s for e, v, s in self.exits)]
        offs, o = b"", fixed
        for p in parts:
            offs += le32(o)
            o += len(p)
        tail = b"" if self.sync is None else self.sync[0] + self.sync[1]
        return self.randao + self.eth1 + self.graffiti + offs + tail + b"".join(parts)

    def root(self) -> bytes:
        ml = lambda xs, lim: S.mix_in_length(S.merkleize(xs, lim), len(xs))  # noqa: E731
        sh = lambda h, s: S.merkleize([header_root(h), S.bytes_vector_root(s)])  # noqa: E731

        def dep(d):
            dd = d[1056:]
            return S.merkleize([S.merkleize([d[32 * i:32 * i + 32] for i in range(33)]),
                                S.merkleize([S.bytes_vector_root(dd[0:48]), dd[48:80],
                                             S.u64(int.from_bytes(dd[80:88], "little")),
                                             S.bytes_vector_root(dd[88:184])])])
        e = self.eth1
        fields = [S.bytes_vector_root(self.randao),
                  S.merkleize([e[0:32], S.u64(int.from_bytes(e[32:40], "little")), e[40:72]]),
                  self.graffiti,
                  ml([S.merkleize([sh(h1, s1), sh(h2, s2)]) for h1, s1, h2, s2 in self.proposer_slashings], 16),
                  ml([S.merkleize([a.root(), b.root()]) for a, b in self.attester_slashings], 2),
                  ml([a.root() for a in self.attestations], 128),
                  ml([dep(d) for d in self.deposits], 16),
                  ml([S.merkleize([S.merkleize([S.u64(ep), S.u64(v)]), S.bytes_vector_root(s)])
                      for ep, v, s in self.exits], 16)]
        if self.sync is not None:
            fields.append(S.merkleize([S.merkleize(S.pack_bytes(self.sync[0])), S.bytes_vector_root(self.sync[1])]))
        return S.merkleize(fields)


def signed_block_ssz(slot, proposer, parent, state, body: Body, sig: bytes) -> bytes:
    msg = le64(slot) + le64(proposer) + parent + state + le32(84) + body.ssz()
    return le32(100) + sig + msg


def block_root(slot, proposer, parent, state, body: Body) -> bytes:
    return header_root(header(slot, proposer, parent, state, body.root()))


# ---- the reference's mainnet JSON blocks -> SSZ ----------------------------------------
def _hx(s):
    return bytes.fromhex(s[2:] if s.startswith("0x") else s)


def json_block_to_ssz(b: dict) -> bytes:
    m = b["message"]
    bd = m["body"]
    for k in ("proposer_slashings", "attester_slashings", "deposits", "voluntary_exits"):
        assert not bd[k], "fixture blocks carry attestations only"
    e = bd["eth1_data"]
    body = Body(_hx(bd["randao_reveal"]), _hx(e["deposit_root"]) + le64(e["deposit_count"]) + _hx(e["block_hash"]),
                _hx(bd["graffiti"]),
                attestations=[Att(_hx(a["aggregation_bits"]), S.attestation_data_ssz(a["data"]), _hx(a["signature"]))
                              for a in bd["attestations"]])
    return signed_block_ssz(int(m["slot"]), int(m["proposer_index"]), _hx(m["parent_root"]), _hx(m["state_root"]),
                            body, _hx(b["signature"]))


# ---- synthetic signed blocks -------------------------------------------------------------
class Chain:
    """Fork schedule + domains restated from the spec (compute_domain), independent of the product."""

    def __init__(self, gvr: bytes, forks: List[Tuple[int, bytes]]):
        self.gvr, self.forks = gvr, forks

    def domain(self, dt: bytes, slot: int) -> bytes:
        v = [ver for ep, ver in self.forks if slot // 32 >= ep][-1]
        return S.compute_domain(dt, v, self.gvr)

    def altair(self, slot: int) -> bool:
        return len([1 for ep, _ in self.forks if slot // 32 >= ep]) >= 2


def committee_of(n_validators: int, size: int = 24) -> Callable[[int, int], List[int]]:
    def f(slot, index):
        h = hashlib.sha256(b"committee" + le64(slot) + le64(index)).digest()
        start = int.from_bytes(h[:4], "little") % n_validators
        return [(start + 7 * k) % n_validators for k in range(size)]
    return f


def sync_committee_of(n_validators: int) -> Callable[[int], List[int]]:
    return lambda slot: [(slot // 8192 * 31 + 13 * k) % n_validators for k in range(512)]


def make_block(sign, sks: List[int], chain: Chain, slot: int, proposer: int, parent: bytes, committee, sync_committee,
               n_atts=3, n_exits=1, n_prop_sl=1, n_att_sl=1, n_deposits=1, sync_participants=100, seed=0):
    """sign(list of int sks, list of 32-byte roots) -> signatures.  Returns (ssz, expected sets as
    (validator indices, signing root), block root).  Every signature is valid."""
    rng = hashlib.sha256(b"blk" + le64(slot) + le64(seed)).digest()
    todo: List[Tuple[List[int], bytes]] = []   # expected sets in the reference's order
    dom = chain.domain
    epoch = slot // 32
    todo.append(([proposer], S.compute_signing_root(S.u64(epoch), dom(bytes([2, 0, 0, 0]), slot))))
    prop_sl = []
    for k in range(n_prop_sl):
        pi = (proposer + 5 + k) % len(sks)
        hs = [header(slot - 1, pi, hashlib.sha256(rng + bytes([k, j])).digest(), bytes(32), bytes(32)) for j in (0, 1)]
        roots = [S.compute_signing_root(header_root(h), dom(bytes(4), slot - 1)) for h in hs]
        prop_sl.append((hs, roots, pi))
        todo += [([pi], r) for r in roots]
    att_sl = []
    for k in range(n_att_sl):
        pair = []
        for j in (0, 1):
            ix = sorted({(proposer + 3 * t + j + k) % len(sks) for t in range(6)})
            data = le64(slot - 2) + le64(j) + hashlib.sha256(rng + b"as" + bytes([k, j])).digest() + \
                le64(epoch - 1) + bytes(32) + le64(epoch) + bytes(32)
            r = S.compute_signing_root(S.attestation_data_root(data), dom(bytes([1, 0, 0, 0]), epoch * 32))
            pair.append((ix, data, r))
            todo.append((ix, r))
        att_sl.append(pair)
    atts = []
    for k in range(n_atts):
        aslot, aindex = slot - 1, k
        members = committee(aslot, aindex)
        bits = [(rng[(k + t) % 32] >> (t % 8)) & 1 or t == 0 for t in range(len(members))]
        raw = bytearray((len(members) + 8) // 8)
        for t, bt in enumerate(bits):
            if bt:
                raw[t // 8] |= 1 << (t % 8)
        raw[len(members) // 8] |= 1 << (len(members) % 8)
        data = le64(aslot) + le64(aindex) + hashlib.sha256(rng + b"bb" + bytes([k])).digest() + \
            le64(max(epoch - 1, 0)) + bytes(32) + le64(aslot // 32) + hashlib.sha256(b"t").digest()
        r = S.compute_signing_root(S.attestation_data_root(data), dom(bytes([1, 0, 0, 0]), (aslot // 32) * 32))
        ix = sorted(members[t] for t, bt in enumerate(bits) if bt)
        atts.append((bytes(raw), data, ix, r))
        todo.append((ix, r))
    exits = []
    for k in range(n_exits):
        v = (proposer + 11 + k) % len(sks)
        r = S.compute_signing_root(S.merkleize([S.u64(epoch), S.u64(v)]), dom(bytes([4, 0, 0, 0]), epoch * 32))
        exits.append((epoch, v, r))
        todo.append(([v], r))
    n_block_sets = len(todo)
    sigs = sign([sum(sks[i] for i in ix) % R_ORDER for ix, _ in todo], [r for _, r in todo])
    it = iter(sigs)
    randao = next(it)
    ps_enc = []
    for hs, _, _ in prop_sl:
        ps_enc.append((hs[0], next(it), hs[1], next(it)))
    as_enc = []
    for pair in att_sl:
        as_enc.append(tuple(Indexed(ix, data, next(it)) for ix, data, _ in pair))
    at_enc = [Att(raw, data, next(it)) for raw, data, _, _ in atts]
    ex_enc = [(ep, v, next(it)) for ep, v, _ in exits]
    deposits = [hashlib.sha256(rng + b"dep" + bytes([k])).digest() * 38 + bytes(24) for k in range(n_deposits)]
    body = Body(randao, hashlib.sha256(rng).digest() + le64(7) + bytes(32), b"graffiti".ljust(32, b"\0"),
                ps_enc, as_enc, at_enc, deposits, ex_enc)
    sync_set = None
    if chain.altair(slot):
        members = sync_committee(slot)
        bits = bytearray(64)
        for t in range(sync_participants):
            p = (t * 37 + seed) % 512
            bits[p // 8] |= 1 << (p % 8)
        part = [members[t] for t in range(512) if (bits[t // 8] >> (t % 8)) & 1]
        if part:
            r = S.compute_signing_root(parent, dom(bytes([7, 0, 0, 0]), max(slot, 1) - 1))
            sync_sig = sign([sum(sks[i] for i in part) % R_ORDER], [r])[0]
            sync_set = (part, r)
        else:
            sync_sig = bytes([0xC0]) + bytes(95)
        body.sync = (bytes(bits), sync_sig)
    state = hashlib.sha256(rng + b"state").digest()
    broot = block_root(slot, proposer, parent, state, body)
    prop_root = S.compute_signing_root(broot, dom(bytes(4), slot))
    bsig = sign([sks[proposer]], [prop_root])[0]
    expected = todo[:n_block_sets] + [([proposer], prop_root)] + ([sync_set] if sync_set else [])
    return signed_block_ssz(slot, proposer, parent, state, body, bsig), expected, broot, body


class OracleRoots:
    """The roots backend computed on the CPU with oracle/ssz.py (CPU tests)."""

    def signing_roots_attestation(self, data, domains):
        doms = [domains] * len(data) if isinstance(domains, (bytes, bytearray)) else domains
        return [S.compute_signing_root(S.attestation_data_root(d), dm) for d, dm in zip(data, doms)]

    def signing_roots_chunks(self, field_roots, domains):
        doms = [domains] * len(field_roots) if isinstance(domains, (bytes, bytearray)) else domains
        return [S.signing_root_from_field_roots(f, dm) for f, dm in zip(field_roots, doms)]
