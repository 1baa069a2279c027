"""SSZ signing-root oracle (oracle/ssz.py) against the committed reference vectors
(tests/golden/ssz.json: mainnet block parent_root links, interop deposit KAT)."""
import hashlib

from oracle import ssz as S
from tests.conftest import load_golden

G = load_golden("ssz.json")
K = load_golden("kats.json")


def test_block_roots_equal_reference_parent_roots():
    for b in G["blocks"]:
        assert S.merkleize([bytes.fromhex(x) for x in b["field_roots"]]).hex() == b["reference_block_root"]


def test_attestation_roots_and_signing_roots():
    dom = bytes.fromhex(G["domain_attester"])
    for a in G["attestations"]:
        root = S.attestation_data_root(bytes.fromhex(a["ssz"]))
        assert root.hex() == a["object_root"]
        assert S.compute_signing_root(root, dom).hex() == a["signing_root"]


def test_deposit_signing_root_matches_kat():
    d = G["deposit"]
    got = S.signing_root_from_field_roots([bytes.fromhex(x) for x in d["field_roots"]], bytes.fromhex(d["domain"]))
    assert got.hex() == d["signing_root"] == K["deposit"]["signing_root"]


def test_merkleize_edge_cases():
    c = [hashlib.sha256(bytes([i])).digest() for i in range(5)]
    assert S.merkleize(c[:1]) == c[0]
    assert S.merkleize(c[:2]) == S.h(c[0] + c[1])
    assert S.merkleize(c[:3]) == S.h(S.h(c[0] + c[1]) + S.h(c[2] + bytes(32)))
    assert S.merkleize([], 4) == S.ZH[2]
