"""getBlockSignatureSets on the GPU: the signature sets of
SSZ-encoded SignedBeaconBlocks, ready for the verifier with validator-index
pubkeys (the device pubkey table) and signing roots computed on the GPU.

Reference: getBlockSignatureSets (packages/state-transition/src/signatureSets/
index.ts:26-73) and the per-kind builders in the same directory --
randao.ts:19-33, proposerSlashings.ts:9-33, attesterSlashings.ts:8-37,
indexedAttestation.ts:10-48, voluntaryExits.ts:19-42, proposer.ts:16-33 -- plus
getSyncCommitteeSignatureSet (state-transition/src/block/processSyncCommittee.ts:88-111).
Set order and contents follow the reference: randao, proposer slashings (2 sets
each), attester slashings (2 aggregate sets each), attestations (one aggregate
set each), voluntary exits, the block proposer signature (unless
skip_proposer_signature), the sync aggregate (altair+, only with participants;
without any, the signature must be the infinity point or building throws), the
BLS-to-execution changes (capella+).

What runs where: the SSZ block is parsed and its body hashed on the host
(hashlib, as the reference hashes on the main thread); every signing root --
the block's, the RANDAO epoch's, each exit's and slashing header's, every
attestation's AttestationData (the bulk: up to 128 per block) -- is computed
on the GPU in two batched calls per package of blocks (lb_signing_roots_chunks
and lb_signing_roots_attestation with per-object domains); the attesting
indices come from the caller's committee lookup (EpochCache.getBeaconCommittee
in the reference, state-transition/src/cache/epochCache.ts) and travel as
validator indices, so the GPU aggregates the committee pubkeys from its table.

Forks: phase0, altair, bellatrix, capella and deneb block layouts (the execution
payload, the capella BLS-to-execution changes -- which add their own sets,
blsToExecutionChange.ts:1-45 -- and the deneb blob KZG commitments enter the
body root).  Domains follow config.getDomain(stateSlot, type, messageSlot) with
the state at the block's slot (only its fork or the previous one may sign).
"""
from __future__ import annotations

import hashlib
import struct
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

from .verifier import PublicKey, SignatureSet, SignatureSetType

SLOTS_PER_EPOCH = 32
DOMAIN_BEACON_PROPOSER = bytes([0, 0, 0, 0])
DOMAIN_BEACON_ATTESTER = bytes([1, 0, 0, 0])
DOMAIN_RANDAO = bytes([2, 0, 0, 0])
DOMAIN_VOLUNTARY_EXIT = bytes([4, 0, 0, 0])
DOMAIN_SYNC_COMMITTEE = bytes([7, 0, 0, 0])
# list limits (packages/params/src/presets/mainnet.ts)
MAX_PROPOSER_SLASHINGS = 16
MAX_ATTESTER_SLASHINGS = 2
MAX_ATTESTATIONS = 128
MAX_DEPOSITS = 16
MAX_VOLUNTARY_EXITS = 16
MAX_VALIDATORS_PER_COMMITTEE = 2048
SYNC_COMMITTEE_SIZE = 512
ZERO32 = bytes(32)


class SszError(ValueError):
    pass


# ---- SSZ merkleization (hashlib) -------------------------------------------------
def _h(b: bytes) -> bytes:
    return hashlib.sha256(b).digest()


_ZH = [ZERO32]
for _ in range(64):
    _ZH.append(_h(_ZH[-1] + _ZH[-1]))


def merkleize(chunks: Sequence[bytes], limit: Optional[int] = None) -> bytes:
    n = len(chunks)
    size = max(n, 1) if limit is None else max(limit, 1)
    depth = (size - 1).bit_length()
    layer = list(chunks)
    for d in range(depth):
        if len(layer) % 2:
            layer.append(_ZH[d])
        layer = [_h(layer[i] + layer[i + 1]) for i in range(0, len(layer), 2)]
    return layer[0] if layer else _ZH[depth]


def mix_in_length(root: bytes, length: int) -> bytes:
    return _h(root + length.to_bytes(32, "little"))


def _u64(v: int) -> bytes:
    return v.to_bytes(8, "little") + bytes(24)


def _chunks(b: bytes) -> List[bytes]:
    if len(b) % 32:
        b = b + bytes(32 - len(b) % 32)
    return [b[i:i + 32] for i in range(0, len(b), 32)] or [ZERO32]


def _bytes_root(b: bytes) -> bytes:
    return merkleize(_chunks(b))


def _bitlist_root(bits: bytes, limit_bits: int) -> Tuple[bytes, int]:
    """(root, length) of an SSZ bitlist given its serialization (delimiter bit included)."""
    if not bits or bits[-1] == 0:
        raise SszError("bitlist without delimiter")
    n = (len(bits) - 1) * 8 + bits[-1].bit_length() - 1
    raw = bytearray(bits)
    raw[-1] &= ~(1 << (bits[-1].bit_length() - 1)) & 0xFF
    data = bytes(raw[:(n + 7) // 8])
    root = merkleize(_chunks(data) if data else [], (limit_bits + 255) // 256)
    return mix_in_length(root, n), n


def _bitlist_bits(bits: bytes) -> List[int]:
    n = (len(bits) - 1) * 8 + bits[-1].bit_length() - 1
    return [i for i in range(n) if (bits[i // 8] >> (i % 8)) & 1]


# ---- SSZ reading -------------------------------------------------------------------
def _offsets(buf: bytes, n_fixed: int, starts_at: int, n_var: int, total: int) -> List[Tuple[int, int]]:
    offs = [struct.unpack_from("<I", buf, starts_at + 4 * i)[0] for i in range(n_var)]
    if n_var and offs[0] != n_fixed:
        raise SszError("first offset does not point past the fixed part")
    ends = offs[1:] + [total]
    for a, b in zip(offs, ends):
        if a > b or b > total:
            raise SszError("offsets out of order")
    return list(zip(offs, ends))


def _fixed_list(b: bytes, size: int, limit: int) -> List[bytes]:
    if len(b) % size or len(b) // size > limit:
        raise SszError("bad fixed-size list")
    return [b[i:i + size] for i in range(0, len(b), size)]


def _var_list(b: bytes, limit: int) -> List[bytes]:
    if not b:
        return []
    first = struct.unpack_from("<I", b, 0)[0]
    if first % 4 or first // 4 > limit or first > len(b):
        raise SszError("bad variable-size list")
    n = first // 4
    offs = [struct.unpack_from("<I", b, 4 * i)[0] for i in range(n)] + [len(b)]
    return [b[offs[i]:offs[i + 1]] for i in range(n)]


@dataclass
class Attestation:
    aggregation_bits: bytes
    data: bytes  # 128-byte SSZ AttestationData
    signature: bytes

    @staticmethod
    def parse(b: bytes) -> "Attestation":
        if len(b) < 228:
            raise SszError("attestation too short")
        off = struct.unpack_from("<I", b, 0)[0]
        if off != 228:
            raise SszError("attestation offset")
        return Attestation(b[228:], b[4:132], b[132:228])

    def root(self) -> bytes:
        bits_root, _ = _bitlist_root(self.aggregation_bits, MAX_VALIDATORS_PER_COMMITTEE)
        return merkleize([bits_root, attestation_data_root(self.data), _bytes_root(self.signature)])


@dataclass
class IndexedAttestation:
    attesting_indices: List[int]
    data: bytes
    signature: bytes

    @staticmethod
    def parse(b: bytes) -> "IndexedAttestation":
        if len(b) < 228 or struct.unpack_from("<I", b, 0)[0] != 228:
            raise SszError("indexed attestation")
        idx = b[228:]
        if len(idx) % 8 or len(idx) // 8 > MAX_VALIDATORS_PER_COMMITTEE:
            raise SszError("attesting indices")
        return IndexedAttestation([struct.unpack_from("<Q", idx, i)[0] for i in range(0, len(idx), 8)], b[4:132],
                                  b[132:228])

    def root(self) -> bytes:
        packed = b"".join(i.to_bytes(8, "little") for i in self.attesting_indices)
        ir = mix_in_length(merkleize(_chunks(packed) if packed else [], MAX_VALIDATORS_PER_COMMITTEE * 8 // 32),
                           len(self.attesting_indices))
        return merkleize([ir, attestation_data_root(self.data), _bytes_root(self.signature)])


def attestation_data_root(d: bytes) -> bytes:
    """AttestationData{slot, index, beacon_block_root, source: Checkpoint, target: Checkpoint}."""
    cp = lambda o: merkleize([d[o:o + 8] + bytes(24), d[o + 8:o + 40]])  # noqa: E731
    return merkleize([d[0:8] + bytes(24), d[8:16] + bytes(24), d[16:48], cp(48), cp(88)])


def header_field_roots(h: bytes) -> List[bytes]:
    """BeaconBlockHeader (112 bytes) -> its 5 field roots."""
    return [h[0:8] + bytes(24), h[8:16] + bytes(24), h[16:48], h[48:80], h[80:112]]


FORKS = ("phase0", "altair", "bellatrix", "capella", "deneb")
# fixed part of BeaconBlockBody per fork: phase0 randao(96) eth1(72) graffiti(32) + 5 offsets;
# altair + SyncAggregate(64 + 96); bellatrix + ExecutionPayload offset; capella +
# bls_to_execution_changes offset; deneb + blob_kzg_commitments offset
BODY_FIXED = {"phase0": 220, "altair": 380, "bellatrix": 384, "capella": 388, "deneb": 392}
# fixed part of ExecutionPayload: 14 fields (508 B) + capella withdrawals offset + deneb blob gas (2 x u64)
PAYLOAD_FIXED = {"bellatrix": 508, "capella": 512, "deneb": 528}
MAX_BYTES_PER_TRANSACTION = 1 << 30
MAX_TRANSACTIONS_PER_PAYLOAD = 1 << 20
MAX_EXTRA_DATA_BYTES = 32
MAX_WITHDRAWALS_PER_PAYLOAD = 16
MAX_BLS_TO_EXECUTION_CHANGES = 16
MAX_BLOB_COMMITMENTS_PER_BLOCK = 4096
DOMAIN_BLS_TO_EXECUTION_CHANGE = bytes([10, 0, 0, 0])
G2_POINT_AT_INFINITY = bytes([0xC0]) + bytes(95)


def fork_seq(fork: str) -> int:
    return FORKS.index(fork)


def execution_payload_root(p: bytes, fork: str) -> bytes:
    """hash_tree_root(ExecutionPayload) of the bellatrix / capella / deneb layout
    (packages/types/src/{bellatrix,capella,deneb}/sszTypes.ts ExecutionPayload)."""
    fixed = PAYLOAD_FIXED[fork]
    if len(p) < fixed:
        raise SszError("execution payload too short")
    offs = [436, 504] + ([508] if fork_seq(fork) >= fork_seq("capella") else [])
    var = _var_fields(p, fixed, offs)
    extra, txs = var[0], var[1]
    if len(extra) > MAX_EXTRA_DATA_BYTES:
        raise SszError("extra_data too long")
    tx_roots = []
    for tx in _var_list(txs, MAX_TRANSACTIONS_PER_PAYLOAD):
        if len(tx) > MAX_BYTES_PER_TRANSACTION:
            raise SszError("transaction too long")
        tx_roots.append(mix_in_length(merkleize(_chunks(tx) if tx else [], MAX_BYTES_PER_TRANSACTION // 32), len(tx)))
    fields = [p[0:32], p[32:52] + bytes(12), p[52:84], p[84:116], merkleize(_chunks(p[116:372])), p[372:404],
              p[404:412] + bytes(24), p[412:420] + bytes(24), p[420:428] + bytes(24), p[428:436] + bytes(24),
              mix_in_length(merkleize(_chunks(extra) if extra else [], 1), len(extra)), p[440:472], p[472:504],
              mix_in_length(merkleize(tx_roots, MAX_TRANSACTIONS_PER_PAYLOAD), len(tx_roots))]
    if fork_seq(fork) >= fork_seq("capella"):
        ws = _fixed_list(var[2], 44, MAX_WITHDRAWALS_PER_PAYLOAD)
        fields.append(mix_in_length(merkleize([merkleize([w[0:8] + bytes(24), w[8:16] + bytes(24), w[16:36] + bytes(12),
                                                          w[36:44] + bytes(24)]) for w in ws],
                                              MAX_WITHDRAWALS_PER_PAYLOAD), len(ws)))
    if fork == "deneb":
        fields += [p[512:520] + bytes(24), p[520:528] + bytes(24)]
    return merkleize(fields)


def _var_fields(buf: bytes, n_fixed: int, positions: Sequence[int]) -> List[bytes]:
    """The variable-size fields of a container whose offsets sit at `positions`."""
    offs = [struct.unpack_from("<I", buf, q)[0] for q in positions]
    if offs and offs[0] != n_fixed:
        raise SszError("first offset does not point past the fixed part")
    ends = offs[1:] + [len(buf)]
    for a, b in zip(offs, ends):
        if a > b or b > len(buf):
            raise SszError("offsets out of order")
    return [buf[a:b] for a, b in zip(offs, ends)]


def bls_change_message_fields(c: bytes) -> List[bytes]:
    """BLSToExecutionChange{validator_index, from_bls_pubkey, to_execution_address} field roots."""
    return [c[0:8] + bytes(24), merkleize(_chunks(c[8:56])), c[56:76] + bytes(12)]


@dataclass
class SignedBlock:
    fork: str
    slot: int
    proposer_index: int
    parent_root: bytes
    state_root: bytes
    body_root: bytes
    signature: bytes
    randao_reveal: bytes
    proposer_slashings: List[bytes]          # 416 bytes each: 2 x SignedBeaconBlockHeader
    attester_slashings: List[Tuple[IndexedAttestation, IndexedAttestation]]
    attestations: List[Attestation]
    voluntary_exits: List[bytes]             # 112 bytes each: VoluntaryExit (16) + signature
    sync_bits: Optional[bytes] = None        # altair+: 64 bytes
    sync_signature: Optional[bytes] = None
    execution_payload_root: Optional[bytes] = None   # bellatrix+
    bls_to_execution_changes: List[bytes] = field(default_factory=list)  # capella+: 172 bytes each
    blob_kzg_commitments: List[bytes] = field(default_factory=list)      # deneb: 48 bytes each

    def field_roots(self) -> List[bytes]:
        return [_u64(self.slot), _u64(self.proposer_index), self.parent_root, self.state_root, self.body_root]

    def root(self) -> bytes:
        return merkleize(self.field_roots())


def parse_signed_block(ssz: bytes, fork: str) -> SignedBlock:
    """SSZ SignedBeaconBlock of `fork` (phase0 ... deneb) -> SignedBlock with the body root computed."""
    if fork not in FORKS:
        raise SszError(f"unsupported fork {fork}")
    seq = fork_seq(fork)
    if len(ssz) < 100 or struct.unpack_from("<I", ssz, 0)[0] != 100:
        raise SszError("SignedBeaconBlock header")
    sig = ssz[4:100]
    m = ssz[100:]
    if len(m) < 84 or struct.unpack_from("<I", m, 80)[0] != 84:
        raise SszError("BeaconBlock header")
    slot, proposer = struct.unpack_from("<QQ", m, 0)
    parent, state = m[16:48], m[48:80]
    body = m[84:]
    fixed = BODY_FIXED[fork]
    if len(body) < fixed:
        raise SszError("body too short")
    randao, eth1, graffiti = body[0:96], body[96:168], body[168:200]
    positions = [200, 204, 208, 212, 216] + [380, 384, 388][:max(0, seq - 1)]
    var = _var_fields(body, fixed, positions)
    ps, ats, att, dep, ex = var[:5]
    prop_sl = _fixed_list(ps, 416, MAX_PROPOSER_SLASHINGS)
    att_sl = []
    for s in _var_list(ats, MAX_ATTESTER_SLASHINGS):
        if len(s) < 8:
            raise SszError("attester slashing")
        o1, o2 = struct.unpack_from("<II", s, 0)
        if o1 != 8 or o2 < o1 or o2 > len(s):
            raise SszError("attester slashing offsets")
        att_sl.append((IndexedAttestation.parse(s[o1:o2]), IndexedAttestation.parse(s[o2:])))
    atts = [Attestation.parse(a) for a in _var_list(att, MAX_ATTESTATIONS)]
    deps = _fixed_list(dep, 1240, MAX_DEPOSITS)
    exits = _fixed_list(ex, 112, MAX_VOLUNTARY_EXITS)
    sync_bits = sync_sig = payload_root = None
    changes: List[bytes] = []
    blobs: List[bytes] = []
    # body root (BeaconBlockBody hash_tree_root)
    sh = lambda h_: merkleize([merkleize(header_field_roots(h_[:112])), _bytes_root(h_[112:208])])  # noqa: E731
    ps_root = mix_in_length(merkleize([merkleize([sh(p[:208]), sh(p[208:])]) for p in prop_sl],
                                      MAX_PROPOSER_SLASHINGS), len(prop_sl))
    as_root = mix_in_length(merkleize([merkleize([a.root(), b.root()]) for a, b in att_sl], MAX_ATTESTER_SLASHINGS),
                            len(att_sl))
    at_root = mix_in_length(merkleize([a.root() for a in atts], MAX_ATTESTATIONS), len(atts))

    def deposit_root(d: bytes) -> bytes:
        proof = merkleize([d[32 * i:32 * i + 32] for i in range(33)])
        dd = d[1056:]
        data = merkleize([_bytes_root(dd[0:48]), dd[48:80], dd[80:88] + bytes(24), _bytes_root(dd[88:184])])
        return merkleize([proof, data])
    dp_root = mix_in_length(merkleize([deposit_root(d) for d in deps], MAX_DEPOSITS), len(deps))
    ex_root = mix_in_length(merkleize([merkleize([merkleize([e[0:8] + bytes(24), e[8:16] + bytes(24)]),
                                                  _bytes_root(e[16:112])]) for e in exits], MAX_VOLUNTARY_EXITS),
                            len(exits))
    eth1_root = merkleize([eth1[0:32], eth1[32:40] + bytes(24), eth1[40:72]])
    fields = [_bytes_root(randao), eth1_root, graffiti, ps_root, as_root, at_root, dp_root, ex_root]
    if seq >= fork_seq("altair"):
        sync_bits, sync_sig = body[220:284], body[284:380]
        fields.append(merkleize([merkleize(_chunks(sync_bits)), _bytes_root(sync_sig)]))
    if seq >= fork_seq("bellatrix"):
        payload_root = execution_payload_root(var[5], fork)
        fields.append(payload_root)
    if seq >= fork_seq("capella"):
        changes = _fixed_list(var[6], 172, MAX_BLS_TO_EXECUTION_CHANGES)
        fields.append(mix_in_length(merkleize([merkleize([merkleize(bls_change_message_fields(c[:76])),
                                                          _bytes_root(c[76:172])]) for c in changes],
                                              MAX_BLS_TO_EXECUTION_CHANGES), len(changes)))
    if seq >= fork_seq("deneb"):
        blobs = _fixed_list(var[7], 48, MAX_BLOB_COMMITMENTS_PER_BLOCK)
        fields.append(mix_in_length(merkleize([_bytes_root(c) for c in blobs], MAX_BLOB_COMMITMENTS_PER_BLOCK),
                                    len(blobs)))
    return SignedBlock(fork, slot, proposer, parent, state, merkleize(fields), sig, randao, prop_sl, att_sl, atts,
                       exits, sync_bits, sync_sig, payload_root, changes, blobs)


# ---- domains -----------------------------------------------------------------------------
@dataclass
class ChainConfig:
    """The parts of BeaconConfig the set builders read: the fork schedule (epoch,
    version, name) and genesis_validators_root -- config.getDomain / getDomainAtFork /
    getDomainForVoluntaryExit (packages/config/src/genesisConfig/index.ts:28-87)."""
    genesis_validators_root: bytes
    forks: List[Tuple[int, bytes, str]] = field(default_factory=lambda: [(0, bytes(4), "phase0")])

    def _fork_index(self, epoch: int) -> int:
        cur = 0
        for i, f in enumerate(self.forks):
            if epoch >= f[0]:
                cur = i
        return cur

    def fork_at_epoch(self, epoch: int) -> Tuple[bytes, str]:
        f = self.forks[self._fork_index(epoch)]
        return f[1], f[2]

    def fork_epoch(self, name: str) -> Optional[int]:
        for ep, _, nm in self.forks:
            if nm == name:
                return ep
        return None

    def _domain(self, domain_type: bytes, version: bytes) -> bytes:
        fork_data_root = _h(version + bytes(28) + self.genesis_validators_root)
        return domain_type + fork_data_root[:28]

    def domain(self, domain_type: bytes, state_slot: int, message_slot: Optional[int] = None) -> bytes:
        """getDomain(stateSlot, domainType, messageSlot): only the fork of the state's slot
        or the one before it may sign -- the previous fork when the message's epoch
        precedes the state fork's epoch (genesisConfig/index.ts:28-53)."""
        i = self._fork_index(state_slot // SLOTS_PER_EPOCH)
        epoch = (state_slot if message_slot is None else message_slot) // SLOTS_PER_EPOCH
        if epoch < self.forks[i][0] and i > 0:
            i -= 1
        return self._domain(domain_type, self.forks[i][1])

    def domain_at_fork(self, name: str, domain_type: bytes) -> bytes:
        """getDomainAtFork (genesisConfig/index.ts:55-72)."""
        for _, ver, nm in self.forks:
            if nm == name:
                return self._domain(domain_type, ver)
        raise ValueError(f"fork {name} not in the schedule")

    def domain_voluntary_exit(self, state_slot: int, message_slot: int) -> bytes:
        """getDomainForVoluntaryExit: from deneb on the domain is fixed to capella's
        (EIP-7044, genesisConfig/index.ts:76-86)."""
        deneb = self.fork_epoch("deneb")
        if deneb is None or state_slot < deneb * SLOTS_PER_EPOCH:
            return self.domain(DOMAIN_VOLUNTARY_EXIT, state_slot, message_slot)
        return self.domain_at_fork("capella", DOMAIN_VOLUNTARY_EXIT)


MAINNET = ChainConfig(bytes.fromhex("4b363db94e286120d76eb905340fdd4e54bfe9f06bf33ff6cf5ad27f511bfe95"),
                      [(0, bytes.fromhex("00000000"), "phase0"), (74240, bytes.fromhex("01000000"), "altair"),
                       (144896, bytes.fromhex("02000000"), "bellatrix"), (194048, bytes.fromhex("03000000"), "capella"),
                       (269568, bytes.fromhex("04000000"), "deneb")])


# ---- the builder -------------------------------------------------------------------------
class BlockSignatureSetBuilder:
    """getBlockSignatureSets for a package of blocks.

    roots: the GPU (lodestar_amd.native.Device) or any object with its
    signing_roots_attestation / signing_roots_chunks methods.
    committee(slot, index) -> validator indices of that beacon committee;
    sync_committee(slot) -> the 512 validator indices of the sync committee (altair)."""

    def __init__(self, roots, config: ChainConfig, committee: Callable[[int, int], Sequence[int]],
                 sync_committee: Optional[Callable[[int], Sequence[int]]] = None):
        self.roots = roots
        self.config = config
        self.committee = committee
        self.sync_committee = sync_committee

    def build(self, signed_blocks: Sequence[bytes], skip_proposer_signature: bool = False) -> List[List[SignatureSet]]:
        blocks = []
        for ssz in signed_blocks:
            # the fork of a block is the fork at its slot (bytes 100:108 are BeaconBlock.slot)
            slot = struct.unpack_from("<Q", ssz, 100)[0] if len(ssz) >= 108 else 0
            blocks.append(parse_signed_block(ssz, self.config.fork_at_epoch(slot // SLOTS_PER_EPOCH)[1]))
        cfg = self.config
        # every object to sign, in the reference's per-block order
        chunk_jobs: Dict[int, List[Tuple[List[bytes], bytes]]] = {}  # m -> [(field roots, domain)]
        att_jobs: List[Tuple[bytes, bytes]] = []                     # (128-byte data, domain)
        change_keys: List[bytes] = []                                # 48-byte fromBlsPubkey of every change
        plan: List[List[tuple]] = []

        def chunk(fields: List[bytes], domain: bytes) -> tuple:
            lst = chunk_jobs.setdefault(len(fields), [])
            lst.append((fields, domain))
            return ("c", len(fields), len(lst) - 1)

        def att(data: bytes, state_slot: int) -> tuple:
            # indexedAttestation.ts:16 / attesterSlashings.ts:32: the target epoch's start slot
            target_epoch = struct.unpack_from("<Q", data, 88)[0]
            att_jobs.append((data, cfg.domain(DOMAIN_BEACON_ATTESTER, state_slot, target_epoch * SLOTS_PER_EPOCH)))
            return ("a", len(att_jobs) - 1)

        for b in blocks:
            p = []
            st = b.slot  # the state the block is processed on is at the block's slot
            # randao.ts:19-33: signing root of the block's epoch (ssz.Epoch)
            p.append((chunk([_u64(b.slot // SLOTS_PER_EPOCH)], cfg.domain(DOMAIN_RANDAO, st, b.slot)),
                      [b.proposer_index], b.randao_reveal))
            # proposerSlashings.ts:9-33: both headers, pubkey of header1's proposer
            for ps in b.proposer_slashings:
                pi = struct.unpack_from("<Q", ps, 8)[0]
                for hdr in (ps[:208], ps[208:]):
                    hslot = struct.unpack_from("<Q", hdr, 0)[0]
                    p.append((chunk(header_field_roots(hdr[:112]), cfg.domain(DOMAIN_BEACON_PROPOSER, st, hslot)),
                              [pi], hdr[112:208]))
            # attesterSlashings.ts:8-37: both indexed attestations
            for a1, a2 in b.attester_slashings:
                for ia in (a1, a2):
                    p.append((att(ia.data, st), list(ia.attesting_indices), ia.signature))
            # indexedAttestation.ts:40-48 with epochCtx.getIndexedAttestation: committee members whose bit is set
            for a in b.attestations:
                aslot, aindex = struct.unpack_from("<QQ", a.data, 0)
                members = list(self.committee(aslot, aindex))
                bits = _bitlist_bits(a.aggregation_bits)
                nbits = (len(a.aggregation_bits) - 1) * 8 + a.aggregation_bits[-1].bit_length() - 1
                if nbits != len(members):
                    raise SszError("aggregation_bits length != committee size")
                p.append((att(a.data, st), sorted(members[i] for i in bits), a.signature))
            # voluntaryExits.ts:19-42 (getDomainForVoluntaryExit: capella's domain from deneb on)
            for e in b.voluntary_exits:
                epoch, vi = struct.unpack_from("<QQ", e, 0)
                p.append((chunk([_u64(epoch), _u64(vi)], cfg.domain_voluntary_exit(st, epoch * SLOTS_PER_EPOCH)),
                          [vi], e[16:112]))
            # proposer.ts:16-33
            if not skip_proposer_signature:
                p.append((chunk(b.field_roots(), cfg.domain(DOMAIN_BEACON_PROPOSER, st, b.slot)),
                          [b.proposer_index], b.signature))
            # processSyncCommittee.ts:88-111: participants sign the parent root at the previous slot
            if fork_seq(b.fork) >= fork_seq("altair") and b.sync_bits is not None:
                if self.sync_committee is None:
                    raise ValueError("altair+ blocks need sync_committee(slot)")
                members = list(self.sync_committee(b.slot))
                part = [members[i] for i in range(SYNC_COMMITTEE_SIZE) if (b.sync_bits[i // 8] >> (i % 8)) & 1]
                if part:
                    prev = max(b.slot, 1) - 1
                    p.append((chunk([b.parent_root], cfg.domain(DOMAIN_SYNC_COMMITTEE, st, prev)), part,
                              b.sync_signature))
                elif b.sync_signature != G2_POINT_AT_INFINITY:
                    # no participants: only the infinity signature is valid (processSyncCommittee.ts:94-101)
                    raise ValueError("Empty sync committee signature is not infinity")
            # blsToExecutionChange.ts:19-45: fixed phase0 domain, the change's own (48-byte) pubkey
            for c in b.bls_to_execution_changes:
                change_keys.append(c[8:56])
                p.append((chunk(bls_change_message_fields(c[:76]),
                                cfg.domain_at_fork("phase0", DOMAIN_BLS_TO_EXECUTION_CHANGE)),
                          ("k", len(change_keys) - 1), c[76:172]))
            plan.append(p)
        # all signing roots on the GPU: one call per container width + one for the attestations
        roots_c: Dict[int, List[bytes]] = {}
        for m, jobs in chunk_jobs.items():
            roots_c[m] = self.roots.signing_roots_chunks([f for f, _ in jobs], [d for _, d in jobs])
        roots_a = self.roots.signing_roots_attestation([d for d, _ in att_jobs], [dm for _, dm in att_jobs]) \
            if att_jobs else []
        # PublicKey.fromBytes(fromBlsPubkey, affine, validate=true) on the GPU; the reference throws
        keys96: List[bytes] = []
        if change_keys:
            keys96, status = self.roots.pubkeys_from_bytes(change_keys)
            for i, stt in enumerate(status):
                if stt != 0:
                    raise ValueError(f"BLS-to-execution change {i}: invalid from_bls_pubkey (status {stt})")
        out = []
        for p in plan:
            sets = []
            for ref, idx, sig in p:
                root = roots_c[ref[1]][ref[2]] if ref[0] == "c" else roots_a[ref[1]]
                if isinstance(idx, tuple):  # a BLS change: its own pubkey, no validator index
                    sets.append(SignatureSet(SignatureSetType.single, root, bytes(sig),
                                             pubkey=PublicKey(uncompressed=keys96[idx[1]])))
                    continue
                keys = [PublicKey(index=int(i)) for i in idx]
                sets.append(SignatureSet(SignatureSetType.single, root, bytes(sig), pubkey=keys[0]) if len(keys) == 1
                            else SignatureSet(SignatureSetType.aggregate, root, bytes(sig), pubkeys=keys))
            out.append(sets)
        return out
