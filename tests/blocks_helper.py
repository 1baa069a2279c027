"""Test helper (TEST INFRASTRUCTURE): SSZ encoding of phase0 ... deneb SignedBeaconBlocks
and an independent restatement of their hash_tree_root from the structured fields
(oracle/ssz.py primitives), plus a synthetic signed-block generator for the
getBlockSignatureSets tests.  The product parser (lodestar_amd/block_sets.py) reads
the bytes; this side never parses, it builds -- so the two meet only at the roots.

Layouts: SignedBeaconBlock{message: BeaconBlock, signature}, BeaconBlock{slot,
proposer_index, parent_root, state_root, body}, BeaconBlockBody phase0 {randao_reveal,
eth1_data, graffiti, proposer_slashings, attester_slashings, attestations, deposits,
voluntary_exits} (+ sync_aggregate in altair, + execution_payload in bellatrix, +
bls_to_execution_changes in capella, + blob_kzg_commitments in deneb) -- the
consensus-spec containers the reference's @lodestar/types ssz definitions follow
(packages/types/src/{phase0,altair,bellatrix,capella,deneb}/sszTypes.ts).
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


FORK_NAMES = ("phase0", "altair", "bellatrix", "capella", "deneb")


def seq(fork: str) -> int:
    return FORK_NAMES.index(fork)


@dataclass
class Payload:
    """ExecutionPayload (bellatrix/capella/deneb) from structured fields."""
    fork: str
    parent_hash: bytes
    fee_recipient: bytes          # 20
    state_root: bytes
    receipts_root: bytes
    logs_bloom: bytes             # 256
    prev_randao: bytes
    block_number: int
    gas_limit: int
    gas_used: int
    timestamp: int
    extra_data: bytes
    base_fee_per_gas: int
    block_hash: bytes
    transactions: List[bytes] = field(default_factory=list)
    withdrawals: List[Tuple[int, int, bytes, int]] = field(default_factory=list)  # index, validator, address, amount
    blob_gas_used: int = 0
    excess_blob_gas: int = 0

    def ssz(self) -> bytes:
        capella = seq(self.fork) >= seq("capella")
        fixed = 508 + (4 if capella else 0) + (16 if self.fork == "deneb" else 0)
        txs = var_list(self.transactions)
        wds = b"".join(le64(i) + le64(v) + a + le64(am) for i, v, a, am in self.withdrawals)
        head = (self.parent_hash + self.fee_recipient + self.state_root + self.receipts_root + self.logs_bloom +
                self.prev_randao + le64(self.block_number) + le64(self.gas_limit) + le64(self.gas_used) +
                le64(self.timestamp) + le32(fixed) + self.base_fee_per_gas.to_bytes(32, "little") + self.block_hash +
                le32(fixed + len(self.extra_data)))
        if capella:
            head += le32(fixed + len(self.extra_data) + len(txs))
        if self.fork == "deneb":
            head += le64(self.blob_gas_used) + le64(self.excess_blob_gas)
        assert len(head) == fixed
        return head + self.extra_data + txs + (wds if capella else b"")

    def root(self) -> bytes:
        tx_roots = [S.mix_in_length(S.merkleize(S.pack_bytes(t) if t else [], 1 << 25), len(t))
                    for t in self.transactions]
        f = [self.parent_hash, S.bytes_vector_root(self.fee_recipient), self.state_root, self.receipts_root,
             S.bytes_vector_root(self.logs_bloom), self.prev_randao, S.u64(self.block_number), S.u64(self.gas_limit),
             S.u64(self.gas_used), S.u64(self.timestamp),
             S.mix_in_length(S.merkleize(S.pack_bytes(self.extra_data) if self.extra_data else [], 1),
                             len(self.extra_data)),
             self.base_fee_per_gas.to_bytes(32, "little"), self.block_hash,
             S.mix_in_length(S.merkleize(tx_roots, 1 << 20), len(tx_roots))]
        if seq(self.fork) >= seq("capella"):
            f.append(S.mix_in_length(S.merkleize([S.merkleize([S.u64(i), S.u64(v), S.bytes_vector_root(a), S.u64(am)])
                                                  for i, v, a, am in self.withdrawals], 16), len(self.withdrawals)))
        if self.fork == "deneb":
            f += [S.u64(self.blob_gas_used), S.u64(self.excess_blob_gas)]
        return S.merkleize(f)


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
    sync: Optional[Tuple[bytes, bytes]] = None  # (64-byte bits, sig) altair+
    fork: Optional[str] = None                  # None: phase0, or altair when sync is set
    payload: Optional[Payload] = None           # bellatrix+
    bls_changes: List[Tuple[int, bytes, bytes, bytes]] = field(default_factory=list)  # vi, pk48, address, sig
    blobs: List[bytes] = field(default_factory=list)  # deneb: 48-byte commitments

    def _fork(self) -> str:
        return self.fork or ("altair" if self.sync is not None else "phase0")

    def ssz(self) -> bytes:
        fk = seq(self._fork())
        fixed = 220 + (160 if fk >= 1 else 0) + 4 * max(0, fk - 1)
        parts = [b"".join(h1 + s1 + h2 + s2 for h1, s1, h2, s2 in self.proposer_slashings),
                 var_list([le32(8) + le32(8 + len(a.ssz())) + a.ssz() + b.ssz() for a, b in self.attester_slashings]),
                 var_list([a.ssz() for a in self.attestations]),
                 b"".join(self.deposits),
                 b"".join(le64(e) + le64(v) + s for e, v, s in self.exits)]
        late = []
        if fk >= 2:
            late.append(self.payload.ssz())
        if fk >= 3:
            late.append(b"".join(le64(v) + pk + a + sg for v, pk, a, sg in self.bls_changes))
        if fk >= 4:
            late.append(b"".join(self.blobs))
        offs, o = [], fixed
        for q in parts + late:
            offs.append(le32(o))
            o += len(q)
        tail = b"" if fk == 0 else self.sync[0] + self.sync[1]
        return (self.randao + self.eth1 + self.graffiti + b"".join(offs[:5]) + tail + b"".join(offs[5:]) +
                b"".join(parts) + b"".join(late))

    def root(self) -> bytes:
        fk = seq(self._fork())
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
        if fk >= 1:
            fields.append(S.merkleize([S.merkleize(S.pack_bytes(self.sync[0])), S.bytes_vector_root(self.sync[1])]))
        if fk >= 2:
            fields.append(self.payload.root())
        if fk >= 3:
            fields.append(ml([S.merkleize([bls_change_root(v, pk, a), S.bytes_vector_root(sg)])
                              for v, pk, a, sg in self.bls_changes], 16))
        if fk >= 4:
            fields.append(ml([S.bytes_vector_root(c) for c in self.blobs], 4096))
        return S.merkleize(fields)


def bls_change_root(vi: int, pk48: bytes, addr: bytes) -> bytes:
    return S.merkleize([S.u64(vi), S.bytes_vector_root(pk48), S.bytes_vector_root(addr)])


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
    """Fork schedule + domains restated from the spec (compute_domain), independent of the product.
    forks: [(epoch, version)] in fork order phase0, altair, bellatrix, capella, deneb."""

    def __init__(self, gvr: bytes, forks: List[Tuple[int, bytes]]):
        self.gvr, self.forks = gvr, forks

    def _index(self, slot: int) -> int:
        return len([1 for ep, _ in self.forks if slot // 32 >= ep]) - 1

    def domain(self, dt: bytes, slot: int) -> bytes:
        """The message's own fork (every synthetic message sits in its block's fork)."""
        return S.compute_domain(dt, self.forks[self._index(slot)][1], self.gvr)

    def domain_at(self, dt: bytes, fork: str) -> bytes:
        return S.compute_domain(dt, self.forks[seq(fork)][1], self.gvr)

    def fork(self, slot: int) -> str:
        return FORK_NAMES[self._index(slot)]

    def altair(self, slot: int) -> bool:
        return self._index(slot) >= 1


def committee_of(n_validators: int, size: int = 24) -> Callable[[int, int], List[int]]:
    def f(slot, index):
        h = hashlib.sha256(b"committee" + le64(slot) + le64(index)).digest()
        start = int.from_bytes(h[:4], "little") % n_validators
        return [(start + 7 * k) % n_validators for k in range(size)]
    return f


def sync_committee_of(n_validators: int) -> Callable[[int], List[int]]:
    return lambda slot: [(slot // 8192 * 31 + 13 * k) % n_validators for k in range(512)]


def make_block(sign, sks: List[int], chain: Chain, slot: int, proposer: int, parent: bytes, committee, sync_committee,
               n_atts=3, n_exits=1, n_prop_sl=1, n_att_sl=1, n_deposits=1, sync_participants=100, seed=0,
               pk48=None, n_changes=2, n_txs=3, n_withdrawals=2, n_blobs=2):
    """sign(list of int sks, list of 32-byte roots) -> signatures.  Returns (ssz, expected sets as
    (validator indices, signing root), block root, body).  Every signature is valid.  A BLS-to-execution
    change set (capella+, needs pk48(sk) -> 48-byte compressed pubkey) is expected as
    (("pk48", key), root)."""
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
    fork = chain.fork(slot)
    for k in range(n_exits):
        v = (proposer + 11 + k) % len(sks)
        # EIP-7044: from deneb on, exits are signed with the capella fork version
        exit_dom = chain.domain_at(bytes([4, 0, 0, 0]), "capella") if fork == "deneb" else \
            dom(bytes([4, 0, 0, 0]), epoch * 32)
        r = S.compute_signing_root(S.merkleize([S.u64(epoch), S.u64(v)]), exit_dom)
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
                ps_enc, as_enc, at_enc, deposits, ex_enc, fork=fork)
    if seq(fork) >= seq("bellatrix"):
        hx = lambda t: hashlib.sha256(rng + t).digest()  # noqa: E731
        body.payload = Payload(fork, hx(b"ph"), hx(b"fr")[:20], hx(b"sr"), hx(b"rr"), hx(b"lb") * 8, hx(b"pr"),
                               1000 + slot, 30_000_000, 12_345_678, 1_700_000_000 + 12 * slot, b"lodestar-amd",
                               7 * 10 ** 9, hx(b"bh"),
                               [hx(b"tx" + bytes([k])) * (k + 1) + bytes([k]) for k in range(n_txs)],
                               [(slot * 16 + k, (proposer + k) % len(sks), hx(b"wa" + bytes([k]))[:20], 32 * 10 ** 9 + k)
                                for k in range(n_withdrawals)] if seq(fork) >= seq("capella") else [],
                               131072 if fork == "deneb" else 0, 262144 if fork == "deneb" else 0)
    change_sets = []
    if seq(fork) >= seq("capella") and pk48 is not None:
        csks = [(int.from_bytes(hashlib.sha256(rng + b"wsk" + bytes([k])).digest(), "big") % (R_ORDER - 1)) + 1
                for k in range(n_changes)]
        msgs = []
        for k, csk in enumerate(csks):
            vi, pk, addr = (proposer + 21 + k) % len(sks), pk48(csk), hashlib.sha256(rng + b"ea" + bytes([k])).digest()[:20]
            r = S.compute_signing_root(bls_change_root(vi, pk, addr), chain.domain_at(bytes([10, 0, 0, 0]), "phase0"))
            msgs.append((vi, pk, addr, r))
        csigs = sign(csks, [m[3] for m in msgs])
        body.bls_changes = [(vi, pk, addr, sg) for (vi, pk, addr, _), sg in zip(msgs, csigs)]
        change_sets = [(("pk48", pk), r) for _, pk, _, r in msgs]
    if fork == "deneb":
        body.blobs = [bytes([0xC0 | k]) + hashlib.sha256(rng + b"kzg" + bytes([k])).digest() + bytes(15)
                      for k in range(n_blobs)]
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
    expected = todo[:n_block_sets] + [([proposer], prop_root)] + ([sync_set] if sync_set else []) + change_sets
    return signed_block_ssz(slot, proposer, parent, state, body, bsig), expected, broot, body


class OracleRoots:
    """The roots backend computed on the CPU with oracle/ssz.py (CPU tests)."""

    def pubkeys_from_bytes(self, keys48):
        from oracle import bls12_381 as O
        out, st = [], []
        for k in keys48:
            try:
                p = O.g1_from_bytes(k)
                ok = p is not None and O.g1_in_subgroup(p)
            except ValueError:
                ok = False
            out.append(O.g1_to_bytes(p, compressed=False) if ok else bytes([0x40]) + bytes(95))
            st.append(0 if ok else 3)
        return out, st

    def signing_roots_attestation(self, data, domains):
        doms = [domains] * len(data) if isinstance(domains, (bytes, bytearray)) else domains
        return [S.compute_signing_root(S.attestation_data_root(d), dm) for d, dm in zip(data, doms)]

    def signing_roots_chunks(self, field_roots, domains):
        doms = [domains] * len(field_roots) if isinstance(domains, (bytes, bytearray)) else domains
        return [S.signing_root_from_field_roots(f, dm) for f, dm in zip(field_roots, doms)]
