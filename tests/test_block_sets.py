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


def test_domains_follow_fork_schedule():
    from oracle import ssz as S
    assert CONFIG.domain(B.DOMAIN_RANDAO, 63) == S.compute_domain(bytes([2, 0, 0, 0]), bytes(4), bytes(range(32)))
    assert CONFIG.domain(B.DOMAIN_RANDAO, 64) == S.compute_domain(bytes([2, 0, 0, 0]), bytes([1, 0, 0, 0]),
                                                                  bytes(range(32)))
    assert B.MAINNET.domain(B.DOMAIN_BEACON_ATTESTER, 0).hex() == SSZ_GOLD["domain_attester"]
