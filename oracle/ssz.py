"""CPU restatement of the SSZ hash_tree_root / signing-root step (TEST INFRASTRUCTURE:
only tests/ and the golden-fixture scripts use it, never the product path).

Reference: computeSigningRoot (packages/state-transition/src/util/signingRoot.ts:7-13),
getAttestationDataSigningRoot (state-transition/src/signatureSets/indexedAttestation.ts:10-19),
computeDomain / ForkData (state-transition/src/util/domain.ts).  The SSZ library
itself (@chainsafe/ssz) is not vendored in /root/reference; this restates the
published SSZ merkleization (32-byte chunks, zero-padded power-of-two trees,
mix_in_length for lists/bitlists) and is pinned by the reference's own data: the
first four mainnet blocks of test/unit/sync/backfill/blocks.json, whose
parent_root links (checked by verify.test.ts:25-31) equal hash_tree_root of the
previous block, so the 45 attestations they carry pin the AttestationData roots,
and the interop deposit KAT (genesisState.test.ts:51-55) pins the signing step.
"""
from __future__ import annotations

import hashlib
from typing import List, Optional, Sequence

ZERO = bytes(32)


def h(b: bytes) -> bytes:
    return hashlib.sha256(b).digest()


def _zero_hashes(n: int) -> List[bytes]:
    z = [ZERO]
    for _ in range(n):
        z.append(h(z[-1] + z[-1]))
    return z


ZH = _zero_hashes(64)


def _next_pow2(n: int) -> int:
    w = 1
    while w < n:
        w <<= 1
    return w


def merkleize(chunks: Sequence[bytes], limit: Optional[int] = None) -> bytes:
    """SSZ merkleize: pad to next_pow2(limit or len) with zero chunks."""
    n = len(chunks) if limit is None else limit
    assert len(chunks) <= n
    width = _next_pow2(max(n, 1))
    depth = width.bit_length() - 1
    layer = list(chunks)
    for d in range(depth):
        if len(layer) % 2:
            layer.append(ZH[d])
        layer = [h(layer[i] + layer[i + 1]) for i in range(0, len(layer), 2)]
    return layer[0] if layer else ZH[depth]


def mix_in_length(root: bytes, length: int) -> bytes:
    return h(root + length.to_bytes(32, "little"))


def u64(v: int) -> bytes:
    return int(v).to_bytes(8, "little") + bytes(24)


def pack_bytes(b: bytes) -> List[bytes]:
    b = bytes(b)
    if len(b) % 32:
        b += bytes(32 - len(b) % 32)
    return [b[i:i + 32] for i in range(0, len(b), 32)]


def bytes_vector_root(b: bytes) -> bytes:
    return merkleize(pack_bytes(b)) if len(b) > 32 else bytes(b) + bytes(32 - len(b))


def bitlist_root(bits_with_delimiter: bytes, limit_bits: int) -> bytes:
    b = bytearray(bits_with_delimiter)
    assert b and b[-1] != 0, "bitlist must carry its delimiter bit"
    last = b[-1].bit_length() - 1
    length = (len(b) - 1) * 8 + last
    b[-1] &= ~(1 << last) & 0xFF
    if b and b[-1] == 0 and length % 8 == 0:
        b = b[:-1]
    return mix_in_length(merkleize(pack_bytes(bytes(b)), (limit_bits + 255) // 256), length)


def _hx(s: str) -> bytes:
    return bytes.fromhex(s[2:] if s.startswith("0x") else s)


# ---- phase0 containers ------------------------------------------------------------
def checkpoint_root(epoch: int, root: bytes) -> bytes:
    return merkleize([u64(epoch), bytes(root)])


def attestation_data_ssz(d: dict) -> bytes:
    """phase0.AttestationData JSON -> 128-byte SSZ serialization."""
    return (int(d["slot"]).to_bytes(8, "little") + int(d["index"]).to_bytes(8, "little") +
            _hx(d["beacon_block_root"]) +
            int(d["source"]["epoch"]).to_bytes(8, "little") + _hx(d["source"]["root"]) +
            int(d["target"]["epoch"]).to_bytes(8, "little") + _hx(d["target"]["root"]))


def attestation_data_root(ser: bytes) -> bytes:
    assert len(ser) == 128
    return merkleize([ser[0:8] + bytes(24), ser[8:16] + bytes(24), ser[16:48],
                      checkpoint_root(int.from_bytes(ser[48:56], "little"), ser[56:88]),
                      checkpoint_root(int.from_bytes(ser[88:96], "little"), ser[96:128])])


MAX_VALIDATORS_PER_COMMITTEE = 2048


def attestation_root(a: dict) -> bytes:
    return merkleize([bitlist_root(_hx(a["aggregation_bits"]), MAX_VALIDATORS_PER_COMMITTEE),
                      attestation_data_root(attestation_data_ssz(a["data"])),
                      bytes_vector_root(_hx(a["signature"]))])


def block_body_root_phase0(body: dict) -> bytes:
    for k in ("proposer_slashings", "attester_slashings", "deposits", "voluntary_exits"):
        assert not body[k], f"{k}: only empty lists restated"
    e = body["eth1_data"]
    eth1 = merkleize([_hx(e["deposit_root"]), u64(int(e["deposit_count"])), _hx(e["block_hash"])])
    atts = [attestation_root(a) for a in body["attestations"]]
    empty = lambda limit: mix_in_length(merkleize([], limit), 0)  # noqa: E731
    return merkleize([bytes_vector_root(_hx(body["randao_reveal"])), eth1, _hx(body["graffiti"]),
                      empty(16), empty(2), mix_in_length(merkleize(atts, 128), len(atts)), empty(16), empty(16)])


def block_field_roots_phase0(m: dict) -> List[bytes]:
    """phase0.BeaconBlock field roots [slot, proposer_index, parent_root, state_root, body_root]."""
    return [u64(int(m["slot"])), u64(int(m["proposer_index"])), _hx(m["parent_root"]), _hx(m["state_root"]),
            block_body_root_phase0(m["body"])]


def block_root_phase0(m: dict) -> bytes:
    return merkleize(block_field_roots_phase0(m))


# ---- domains and signing roots ------------------------------------------------------
def compute_domain(domain_type: bytes, fork_version: bytes, genesis_validators_root: bytes) -> bytes:
    """computeDomain: domain_type || hash_tree_root(ForkData{version, gvr})[:28]."""
    fork_data_root = merkleize([bytes(fork_version) + bytes(28), bytes(genesis_validators_root)])
    return bytes(domain_type) + fork_data_root[:28]


def compute_signing_root(object_root: bytes, domain: bytes) -> bytes:
    """hash_tree_root(SigningData{object_root, domain}) (signingRoot.ts:7-13)."""
    return merkleize([bytes(object_root), bytes(domain)])


def signing_root_from_field_roots(field_roots: Sequence[bytes], domain: bytes) -> bytes:
    return compute_signing_root(merkleize(list(field_roots)), domain)
