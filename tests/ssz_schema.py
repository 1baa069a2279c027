"""Test helper (TEST INFRASTRUCTURE): a generic, schema-driven SSZ decoder / encoder /
hash_tree_root, and the SignedBeaconBlock schemas of phase0 ... deneb written from
the consensus-spec containers that the reference's @lodestar/types follows
(packages/types/src/{phase0,altair,bellatrix,capella,deneb}/sszTypes.ts, mainnet
preset packages/params/src/presets/mainnet.ts).

It shares no code with the product parser (lodestar_amd/block_sets.py, hand-written
offsets per fork) and none with tests/blocks_helper.py (which only builds): a block
decoded here and re-hashed must give the product's body and block roots, and
re-encoding must give the original bytes back.
"""
from __future__ import annotations

import hashlib
import struct
from typing import List, Sequence, Tuple

ZERO = bytes(32)
_ZH = [ZERO]
for _ in range(64):
    _ZH.append(hashlib.sha256(_ZH[-1] * 2).digest())


def _merkle(chunks: Sequence[bytes], limit: int) -> bytes:
    depth = max(limit - 1, 0).bit_length()
    layer = list(chunks)
    for d in range(depth):
        if len(layer) & 1:
            layer.append(_ZH[d])
        layer = [hashlib.sha256(layer[i] + layer[i + 1]).digest() for i in range(0, len(layer), 2)]
    return layer[0] if layer else _ZH[depth]


def _pack(b: bytes) -> List[bytes]:
    b = b + bytes(-len(b) % 32)
    return [b[i:i + 32] for i in range(0, len(b), 32)]


def _mix(root: bytes, n: int) -> bytes:
    return hashlib.sha256(root + n.to_bytes(32, "little")).digest()


class T:
    fixed = True
    size = 0

    def decode(self, b: bytes):
        raise NotImplementedError

    def encode(self, v) -> bytes:
        raise NotImplementedError

    def root(self, v) -> bytes:
        raise NotImplementedError


class Uint(T):
    def __init__(self, nbytes):
        self.size = nbytes

    def decode(self, b):
        assert len(b) == self.size
        return int.from_bytes(b, "little")

    def encode(self, v):
        return int(v).to_bytes(self.size, "little")

    def root(self, v):
        return self.encode(v) + bytes(32 - self.size)


class ByteVector(T):
    def __init__(self, n):
        self.size = n

    def decode(self, b):
        assert len(b) == self.size
        return bytes(b)

    def encode(self, v):
        return bytes(v)

    def root(self, v):
        return _merkle(_pack(v), (self.size + 31) // 32)


class ByteList(T):
    fixed = False

    def __init__(self, limit):
        self.limit = limit

    def decode(self, b):
        assert len(b) <= self.limit
        return bytes(b)

    def encode(self, v):
        return bytes(v)

    def root(self, v):
        return _mix(_merkle(_pack(v) if v else [], (self.limit + 31) // 32), len(v))


class Bitvector(ByteVector):
    def __init__(self, nbits):
        super().__init__((nbits + 7) // 8)


class Bitlist(T):
    fixed = False

    def __init__(self, limit):
        self.limit = limit

    def decode(self, b):
        assert b and b[-1]
        return bytes(b)

    def encode(self, v):
        return bytes(v)

    def root(self, v):
        n = (len(v) - 1) * 8 + v[-1].bit_length() - 1
        raw = bytearray(v)
        raw[-1] ^= 1 << (v[-1].bit_length() - 1)
        data = bytes(raw[:(n + 7) // 8])
        return _mix(_merkle(_pack(data) if data else [], (self.limit + 255) // 256), n)


def _decode_seq(elem: T, b: bytes, count=None) -> list:
    if elem.fixed:
        assert len(b) % elem.size == 0
        n = len(b) // elem.size
        assert count is None or n == count
        return [elem.decode(b[i * elem.size:(i + 1) * elem.size]) for i in range(n)]
    if not b:
        return []
    first = struct.unpack_from("<I", b, 0)[0]
    n = first // 4
    offs = [struct.unpack_from("<I", b, 4 * i)[0] for i in range(n)] + [len(b)]
    assert all(offs[i] <= offs[i + 1] for i in range(n))
    return [elem.decode(b[offs[i]:offs[i + 1]]) for i in range(n)]


def _encode_seq(elem: T, vals) -> bytes:
    parts = [elem.encode(v) for v in vals]
    if elem.fixed:
        return b"".join(parts)
    head, o = b"", 4 * len(parts)
    for p in parts:
        head += o.to_bytes(4, "little")
        o += len(p)
    return head + b"".join(parts)


class Vector(T):
    def __init__(self, elem: T, n: int):
        self.elem, self.n = elem, n
        self.fixed = elem.fixed
        self.size = elem.size * n if elem.fixed else 0

    def decode(self, b):
        return _decode_seq(self.elem, b, self.n)

    def encode(self, v):
        return _encode_seq(self.elem, v)

    def root(self, v):
        return _merkle([self.elem.root(x) for x in v], self.n)


class List(T):
    fixed = False

    def __init__(self, elem: T, limit: int):
        self.elem, self.limit = elem, limit

    def decode(self, b):
        v = _decode_seq(self.elem, b)
        assert len(v) <= self.limit
        return v

    def encode(self, v):
        return _encode_seq(self.elem, v)

    def root(self, v):
        if isinstance(self.elem, Uint):  # packed basic elements
            data = b"".join(self.elem.encode(x) for x in v)
            lim = (self.limit * self.elem.size + 31) // 32
            return _mix(_merkle(_pack(data) if data else [], lim), len(v))
        return _mix(_merkle([self.elem.root(x) for x in v], self.limit), len(v))


class Container(T):
    def __init__(self, fields: List[Tuple[str, T]]):
        self.fields = fields
        self.fixed = all(t.fixed for _, t in fields)
        self.size = sum(t.size if t.fixed else 4 for _, t in fields)

    def decode(self, b):
        out, o, var = {}, 0, []
        for name, t in self.fields:
            if t.fixed:
                out[name] = t.decode(b[o:o + t.size])
                o += t.size
            else:
                var.append((name, t, struct.unpack_from("<I", b, o)[0]))
                o += 4
        assert not var or var[0][2] == o
        for k, (name, t, a) in enumerate(var):
            end = var[k + 1][2] if k + 1 < len(var) else len(b)
            out[name] = t.decode(b[a:end])
        return out

    def encode(self, v):
        head, tail = [], []
        fixed_len = self.size
        for name, t in self.fields:
            if t.fixed:
                head.append(t.encode(v[name]))
            else:
                head.append(None)
                tail.append(t.encode(v[name]))
        o, ti, out = fixed_len, 0, b""
        for hpart in head:
            if hpart is None:
                out += o.to_bytes(4, "little")
                o += len(tail[ti])
                ti += 1
            else:
                out += hpart
        return out + b"".join(tail)

    def root(self, v):
        return _merkle([t.root(v[name]) for name, t in self.fields], len(self.fields))


# ---- the beacon-chain containers (mainnet preset) ---------------------------------------
U64, B32 = Uint(8), ByteVector(32)
SIG, PK = ByteVector(96), ByteVector(48)
Checkpoint = Container([("epoch", U64), ("root", B32)])
AttestationData = Container([("slot", U64), ("index", U64), ("beacon_block_root", B32), ("source", Checkpoint),
                             ("target", Checkpoint)])
BeaconBlockHeader = Container([("slot", U64), ("proposer_index", U64), ("parent_root", B32), ("state_root", B32),
                               ("body_root", B32)])
SignedBeaconBlockHeader = Container([("message", BeaconBlockHeader), ("signature", SIG)])
ProposerSlashing = Container([("signed_header_1", SignedBeaconBlockHeader), ("signed_header_2", SignedBeaconBlockHeader)])
IndexedAttestation = Container([("attesting_indices", List(U64, 2048)), ("data", AttestationData), ("signature", SIG)])
AttesterSlashing = Container([("attestation_1", IndexedAttestation), ("attestation_2", IndexedAttestation)])
Attestation = Container([("aggregation_bits", Bitlist(2048)), ("data", AttestationData), ("signature", SIG)])
DepositData = Container([("pubkey", PK), ("withdrawal_credentials", B32), ("amount", U64), ("signature", SIG)])
Deposit = Container([("proof", Vector(B32, 33)), ("data", DepositData)])
VoluntaryExit = Container([("epoch", U64), ("validator_index", U64)])
SignedVoluntaryExit = Container([("message", VoluntaryExit), ("signature", SIG)])
Eth1Data = Container([("deposit_root", B32), ("deposit_count", U64), ("block_hash", B32)])
SyncAggregate = Container([("sync_committee_bits", Bitvector(512)), ("sync_committee_signature", SIG)])
Withdrawal = Container([("index", U64), ("validator_index", U64), ("address", ByteVector(20)), ("amount", U64)])
BLSToExecutionChange = Container([("validator_index", U64), ("from_bls_pubkey", PK),
                                  ("to_execution_address", ByteVector(20))])
SignedBLSToExecutionChange = Container([("message", BLSToExecutionChange), ("signature", SIG)])

_PAYLOAD_COMMON = [("parent_hash", B32), ("fee_recipient", ByteVector(20)), ("state_root", B32),
                   ("receipts_root", B32), ("logs_bloom", ByteVector(256)), ("prev_randao", B32),
                   ("block_number", U64), ("gas_limit", U64), ("gas_used", U64), ("timestamp", U64),
                   ("extra_data", ByteList(32)), ("base_fee_per_gas", Uint(32)), ("block_hash", B32),
                   ("transactions", List(ByteList(1 << 30), 1 << 20))]
PAYLOAD = {
    "bellatrix": Container(_PAYLOAD_COMMON),
    "capella": Container(_PAYLOAD_COMMON + [("withdrawals", List(Withdrawal, 16))]),
    "deneb": Container(_PAYLOAD_COMMON + [("withdrawals", List(Withdrawal, 16)), ("blob_gas_used", U64),
                                          ("excess_blob_gas", U64)]),
}

_BODY0 = [("randao_reveal", SIG), ("eth1_data", Eth1Data), ("graffiti", B32),
          ("proposer_slashings", List(ProposerSlashing, 16)), ("attester_slashings", List(AttesterSlashing, 2)),
          ("attestations", List(Attestation, 128)), ("deposits", List(Deposit, 16)),
          ("voluntary_exits", List(SignedVoluntaryExit, 16))]
_BODY1 = _BODY0 + [("sync_aggregate", SyncAggregate)]
BODY = {
    "phase0": Container(_BODY0),
    "altair": Container(_BODY1),
    "bellatrix": Container(_BODY1 + [("execution_payload", PAYLOAD["bellatrix"])]),
    "capella": Container(_BODY1 + [("execution_payload", PAYLOAD["capella"]),
                                   ("bls_to_execution_changes", List(SignedBLSToExecutionChange, 16))]),
    "deneb": Container(_BODY1 + [("execution_payload", PAYLOAD["deneb"]),
                                 ("bls_to_execution_changes", List(SignedBLSToExecutionChange, 16)),
                                 ("blob_kzg_commitments", List(PK, 4096))]),
}


def signed_block_type(fork: str) -> Container:
    block = Container([("slot", U64), ("proposer_index", U64), ("parent_root", B32), ("state_root", B32),
                       ("body", BODY[fork])])
    return Container([("message", block), ("signature", SIG)])
