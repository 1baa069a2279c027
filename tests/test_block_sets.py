"""getBlockSignatureSets host logic on the CPU: the product's SSZ
parser and body hashing against the reference's mainnet blocks (their parent_root
chain, verify.test.ts:25-31), and the set list against an independent restatement
(tests/blocks_helper.py), with signing roots from oracle/ssz.py standing in for the GPU.
The same builder with the GPU computing the roots: tests/test_gpu_block_sets.py."""
import json
import os
import struct

import pytest

import blocks_helper as BH
import ssz_schema as SC
from lodestar_amd import block_sets as B

GOLD = os.path.join(os.path.dirname(__file__), "golden")
BLOCKS = json.load(open(os.path.join(GOLD, "blocks_ssz.json")))["blocks"]
SSZ_GOLD = json.load(open(os.path.join(GOLD, "ssz.json")))


def test_mainnet_blocks_parse_and_root_chain():
    for i, b in enumerate(BLOCKS):
        blk = B.parse_signed_block(bytes.fromhex(b["ssz"]), "phase0")
        assert (blk.slot, blk.proposer_index) == (b["slot"], b["proposer_index"])
        assert len(blk.attestations) == b["n_attestations"]
        assert blk.parent_root.hex() == b["parent_root"]
        if i + 1 < len(BLOCKS):  # hash_tree_root(block i) == parent_root of block i+1 (reference data)
            assert blk.root().hex() == BLOCKS[i + 1]["parent_root"]


def test_mainnet_block_sets_match_reference_roots():
    """Sets of the fixture blocks: randao, one per attestation, proposer.  The attestation
    and proposer signing roots equal the fixture's (mainnet domains)."""
    builder = B.BlockSignatureSetBuilder(BH.OracleRoots(), B.MAINNET, _committee_by_bits())
    sets = builder.build([bytes.fromhex(b["ssz"]) for b in BLOCKS])
    att_roots = [a["signing_root"] for a in SSZ_GOLD["attestations"]]
    k = 0
    for i, (b, s) in enumerate(zip(BLOCKS, sets)):
        assert len(s) == 1 + b["n_attestations"] + 1
        assert s[0].pubkey.index == b["proposer_index"] and s[-1].pubkey.index == b["proposer_index"]
        for st in s[1:-1]:
            assert st.signing_root.hex() == att_roots[k]
            k += 1
        if i < 3:
            assert s[-1].signing_root.hex() == SSZ_GOLD["blocks"][i]["signing_root"]
    assert k == len(att_roots)
    # skipProposerSignature (index.ts:57-59)
    assert [len(x) for x in builder.build([bytes.fromhex(BLOCKS[0]["ssz"])], skip_proposer_signature=True)] == \
        [1 + BLOCKS[0]["n_attestations"]]


class _committee_by_bits:
    """A committee whose size matches each attestation's bitlist (the fixture has no state)."""

    def __init__(self):
        self.sizes = {}
        for b in BLOCKS:
            for a in B.parse_signed_block(bytes.fromhex(b["ssz"]), "phase0").attestations:
                slot, index = struct.unpack_from("<QQ", a.data, 0)
                n = (len(a.aggregation_bits) - 1) * 8 + a.aggregation_bits[-1].bit_length() - 1
                self.sizes[(slot, index)] = n

    def __call__(self, slot, index):
        return [100 * index + t for t in range(self.sizes[(slot, index)])]


def _sign_stub(sks, roots):
    return [bytes([0xA0 | (i % 16)]) + bytes(95) for i in range(len(sks))]


CHAIN = BH.Chain(bytes(range(32)), [(0, bytes(4)), (2, bytes([1, 0, 0, 0]))])
CONFIG = B.ChainConfig(bytes(range(32)), [(0, bytes(4), "phase0"), (2, bytes([1, 0, 0, 0]), "altair")])


@pytest.mark.parametrize("slot", [40, 70])  # phase0 (epoch 1), altair (epoch 2)
def test_synthetic_block_all_operations(slot):
    sks = list(range(1, 65))
    committee, sync = BH.committee_of(64), BH.sync_committee_of(64)
    ssz, expected, root, body = BH.make_block(_sign_stub, sks, CHAIN, slot, 9, bytes([3]) * 32, committee, sync,
                                              n_atts=4, n_exits=2, n_prop_sl=2, n_att_sl=2, n_deposits=2)
    blk = B.parse_signed_block(ssz, "altair" if slot >= 64 else "phase0")
    assert blk.body_root == body.root()
    assert blk.root() == root
    builder = B.BlockSignatureSetBuilder(BH.OracleRoots(), CONFIG, committee, sync)
    (sets,) = builder.build([ssz])
    assert len(sets) == len(expected) == 1 + 4 + 4 + 4 + 2 + 1 + (1 if slot >= 64 else 0)
    for st, (ix, r) in zip(sets, expected):
        got = [st.pubkey.index] if st.pubkey is not None else [k.index for k in st.pubkeys]
        assert got == ix and st.signing_root == r


def test_sync_aggregate_without_participants_adds_no_set():
    sks = list(range(1, 65))
    committee, sync = BH.committee_of(64), BH.sync_committee_of(64)
    ssz, expected, _, _ = BH.make_block(_sign_stub, sks, CHAIN, 80, 4, bytes(32), committee, sync, n_atts=1,
                                        n_exits=0, n_prop_sl=0, n_att_sl=0, n_deposits=0, sync_participants=0)
    (sets,) = B.BlockSignatureSetBuilder(BH.OracleRoots(), CONFIG, committee, sync).build([ssz])
    assert len(sets) == len(expected) == 3


def test_malformed_blocks_raise():
    good = bytes.fromhex(BLOCKS[1]["ssz"])
    for bad in (good[:50], good[:100 + 84 + 100], b"\x00\x00\x00\x00" + good[4:]):
        with pytest.raises(B.SszError):
            B.parse_signed_block(bad, "phase0")
    # body offsets out of order
    body0 = 100 + 84
    t = bytearray(good)
    struct.pack_into("<I", t, body0 + 200 + 8, 10 ** 6)
    with pytest.raises(B.SszError):
        B.parse_signed_block(bytes(t), "phase0")
    # an attestation whose bitlist does not match the committee
    builder = B.BlockSignatureSetBuilder(BH.OracleRoots(), B.MAINNET, lambda s, i: [1, 2, 3])
    with pytest.raises(B.SszError):
        builder.build([good])
    with pytest.raises(B.SszError):
        B.parse_signed_block(good, "bellatrix")
    with pytest.raises(B.SszError):
        B.parse_signed_block(good, "electra")


def test_domains_follow_fork_schedule():
    from oracle import ssz as S
    assert CONFIG.domain(B.DOMAIN_RANDAO, 63) == S.compute_domain(bytes([2, 0, 0, 0]), bytes(4), bytes(range(32)))
    assert CONFIG.domain(B.DOMAIN_RANDAO, 64) == S.compute_domain(bytes([2, 0, 0, 0]), bytes([1, 0, 0, 0]),
                                                                  bytes(range(32)))
    assert B.MAINNET.domain(B.DOMAIN_BEACON_ATTESTER, 0).hex() == SSZ_GOLD["domain_attester"]


# ---- bellatrix / capella / deneb ------------------------------------
GVR5 = bytes(range(32, 64))
VERS5 = [bytes([k, 0, 0, 9]) for k in range(5)]
EPOCHS5 = [0, 2, 3, 4, 5]                                                   # fork k from epoch EPOCHS5[k]
CHAIN5 = BH.Chain(GVR5, [(EPOCHS5[k], VERS5[k]) for k in range(5)])
CONFIG5 = B.ChainConfig(GVR5, [(EPOCHS5[k], VERS5[k], B.FORKS[k]) for k in range(5)])
BELLATRIX_SSZ = open(os.path.join(GOLD, "goerli_shadow_fork_block_13249.ssz"), "rb").read()


def _pk48(sk):
    from oracle import bls12_381 as O
    return O.g1_to_bytes(O.sk_to_pk(sk), compressed=True)


def _pk96(pk48):
    from oracle import bls12_381 as O
    return O.g1_to_bytes(O.g1_from_bytes(pk48), compressed=False)


@pytest.mark.parametrize("fork_k", range(5))
def test_synthetic_block_every_fork(fork_k):
    """A block of each fork with every operation kind (execution payload with
    transactions and withdrawals, BLS-to-execution changes, blob commitments): the
    product parser's body / block roots equal the builder's restatement and the generic
    schema decoder's, and the set list equals the expected one."""
    slot = 32 * EPOCHS5[fork_k] + 9 if fork_k else 40
    sks = list(range(1, 65))
    committee, sync = BH.committee_of(64), BH.sync_committee_of(64)
    ssz, expected, root, body = BH.make_block(_sign_stub, sks, CHAIN5, slot, 9, bytes([5]) * 32, committee, sync,
                                              n_atts=3, n_exits=2, n_prop_sl=1, n_att_sl=1, n_deposits=1,
                                              pk48=_pk48)
    fork = B.FORKS[fork_k]
    blk = B.parse_signed_block(ssz, fork)
    assert blk.body_root == body.root() and blk.root() == root
    typ = SC.signed_block_type(fork)
    dec = typ.decode(ssz)
    assert typ.encode(dec) == ssz
    assert SC.BODY[fork].root(dec["message"]["body"]) == blk.body_root
    assert len(blk.bls_to_execution_changes) == (2 if fork_k >= 3 else 0)
    assert len(blk.blob_kzg_commitments) == (2 if fork_k >= 4 else 0)
    (sets,) = B.BlockSignatureSetBuilder(BH.OracleRoots(), CONFIG5, committee, sync).build([ssz])
    assert len(sets) == len(expected)
    for st, (ix, r) in zip(sets, expected):
        if isinstance(ix, tuple):  # BLS change: its own key, decompressed + validated
            assert st.pubkey.index is None and st.pubkey.uncompressed == _pk96(ix[1])
        else:
            got = [st.pubkey.index] if st.pubkey is not None else [k.index for k in st.pubkeys]
            assert got == ix
        assert st.signing_root == r


def test_bellatrix_reference_block_parses_and_rehashes():
    """The reference's real bellatrix block (goerli shadow fork, slot 13249): the product
    parser and the generic schema decoder agree on every root; re-encoding is byte-exact."""
    blk = B.parse_signed_block(BELLATRIX_SSZ, "bellatrix")
    assert (blk.slot, blk.proposer_index) == (13249, 18462)
    typ = SC.signed_block_type("bellatrix")
    dec = typ.decode(BELLATRIX_SSZ)
    assert typ.encode(dec) == BELLATRIX_SSZ
    body = dec["message"]["body"]
    assert SC.PAYLOAD["bellatrix"].root(body["execution_payload"]) == blk.execution_payload_root
    assert SC.BODY["bellatrix"].root(body) == blk.body_root
    assert len(blk.attestations) == len(body["attestations"]) > 0
    assert len(body["execution_payload"]["transactions"]) > 0
    # the block root three ways
    msg = dec["message"]
    hdr = {"slot": msg["slot"], "proposer_index": msg["proposer_index"], "parent_root": msg["parent_root"],
           "state_root": msg["state_root"], "body_root": SC.BODY["bellatrix"].root(body)}
    assert SC.BeaconBlockHeader.root(hdr) == blk.root()
    # a body byte flipped inside the payload changes the product's root
    t = bytearray(BELLATRIX_SSZ)
    t[100 + 84 + 3870 + 40] ^= 1  # fee_recipient (the payload starts at body offset 3870)
    assert B.parse_signed_block(bytes(t), "bellatrix").body_root != blk.body_root


def test_mainnet_blocks_match_schema_decoder():
    typ = SC.signed_block_type("phase0")
    for b in BLOCKS:
        ssz = bytes.fromhex(b["ssz"])
        dec = typ.decode(ssz)
        assert typ.encode(dec) == ssz
        assert SC.BODY["phase0"].root(dec["message"]["body"]) == B.parse_signed_block(ssz, "phase0").body_root


def test_deneb_exit_domain_is_capella():
    """getDomainForVoluntaryExit: from deneb on the exit domain is capella's (EIP-7044)."""
    from oracle import ssz as S
    d = CONFIG5.domain_voluntary_exit(32 * 5 + 3, 0)
    assert d == S.compute_domain(bytes([4, 0, 0, 0]), VERS5[3], GVR5)
    assert CONFIG5.domain_voluntary_exit(32 * 4 + 3, 32 * 4) == S.compute_domain(bytes([4, 0, 0, 0]), VERS5[3], GVR5)
    assert CONFIG5.domain_voluntary_exit(32 * 3 + 3, 0) == S.compute_domain(bytes([4, 0, 0, 0]), VERS5[1], GVR5)


def test_domain_uses_state_fork_or_previous():
    """config.getDomain(stateSlot, type, messageSlot) (genesisConfig/index.ts:28-53): a
    message from a later fork inside a phase0 block signs with phase0's version."""
    from oracle import ssz as S
    mainnet_altair = 74240 * 32
    # a phase0 state slot, message slot in altair: still phase0
    assert B.MAINNET.domain(B.DOMAIN_BEACON_PROPOSER, mainnet_altair - 5, mainnet_altair + 100) == \
        S.compute_domain(bytes(4), bytes(4), B.MAINNET.genesis_validators_root)
    # an altair state slot, message from phase0: previous fork
    assert B.MAINNET.domain(B.DOMAIN_BEACON_PROPOSER, mainnet_altair + 5, mainnet_altair - 40) == \
        S.compute_domain(bytes(4), bytes(4), B.MAINNET.genesis_validators_root)
    # capella state, message from altair: only current (capella) or previous (bellatrix)
    cap = 194048 * 32
    assert B.MAINNET.domain(B.DOMAIN_RANDAO, cap + 1, 74240 * 32 + 1) == \
        S.compute_domain(bytes([2, 0, 0, 0]), bytes([2, 0, 0, 0]), B.MAINNET.genesis_validators_root)
    assert B.MAINNET.domain_at_fork("phase0", B.DOMAIN_BLS_TO_EXECUTION_CHANGE) == \
        S.compute_domain(bytes([10, 0, 0, 0]), bytes(4), B.MAINNET.genesis_validators_root)


def test_phase0_block_with_future_proposer_slashing_uses_phase0_domain():
    """A proposer slashing whose headers carry a slot of the next fork, inside a block of
    the earlier fork: the set's domain is the block's fork."""
    from oracle import ssz as S
    sks = list(range(1, 65))
    committee, sync = BH.committee_of(64), BH.sync_committee_of(64)
    ssz, _, _, body = BH.make_block(_sign_stub, sks, CHAIN, 40, 4, bytes(32), committee, sync, n_atts=0, n_exits=0,
                                    n_prop_sl=1, n_att_sl=0, n_deposits=0)
    # rewrite the slashing headers' slot to 70 (altair under CONFIG), re-encode the block
    h1, s1, h2, s2 = body.proposer_slashings[0]
    body.proposer_slashings = [(BH.le64(70) + h1[8:], s1, BH.le64(70) + h2[8:], s2)]
    m = BH.signed_block_ssz(40, 4, bytes(32), ssz[100 + 48:100 + 80], body, bytes(96))
    (sets,) = B.BlockSignatureSetBuilder(BH.OracleRoots(), CONFIG, committee, sync).build([m])
    dom = S.compute_domain(bytes(4), bytes(4), bytes(range(32)))
    assert sets[1].signing_root == S.compute_signing_root(BH.header_root(BH.le64(70) + h1[8:]), dom)


def test_empty_sync_aggregate_requires_infinity_signature():
    """processSyncCommittee.ts:94-101: no participants and a non-infinity signature throws."""
    sks = list(range(1, 65))
    committee, sync = BH.committee_of(64), BH.sync_committee_of(64)
    ssz, _, _, _ = BH.make_block(_sign_stub, sks, CHAIN, 80, 4, bytes(32), committee, sync, n_atts=1,
                                 n_exits=0, n_prop_sl=0, n_att_sl=0, n_deposits=0, sync_participants=0)
    builder = B.BlockSignatureSetBuilder(BH.OracleRoots(), CONFIG, committee, sync)
    assert len(builder.build([ssz])[0]) == 3
    # the same block with a non-infinity sync signature (the last 96 bytes of the sync aggregate)
    body0 = 100 + 84
    t = bytearray(ssz)
    t[body0 + 284] = 0xA0
    with pytest.raises(ValueError, match="not infinity"):
        builder.build([bytes(t)])
