"""Pin the CPU oracle to the reference's own known-answer data.

CPU only.  Each test names the reference file that holds the vector.
"""
import hashlib
import random

import pytest

from oracle import batch as OB
from oracle import bls12_381 as O
from tests.conftest import load_golden

KATS = load_golden("kats.json")


def test_interop_pubkeys_all_100():
    """packages/state-transition/test-cache/interop-pubkeys.json (interop.ts:19-23)."""
    for i, pk_hex in enumerate(KATS["interop_pubkeys"]):
        assert O.g1_to_bytes(O.sk_to_pk(O.interop_secret_key(i))).hex() == pk_hex, i


def test_interop_pubkeys_roundtrip_uncompressed():
    for pk_hex in KATS["interop_pubkeys"][:16]:
        pt = O.g1_from_bytes(bytes.fromhex(pk_hex))
        assert O.g1_in_subgroup(pt)
        assert O.g1_from_bytes(O.g1_to_bytes(pt, compressed=False)) == pt


def test_deposit_signature_kat():
    """packages/beacon-node/test/e2e/interop/genesisState.test.ts:51-55 (hash_to_G2 + sign + compress)."""
    d = KATS["deposit"]
    sk = O.interop_secret_key(d["interop_index"])
    assert O.g1_to_bytes(O.sk_to_pk(sk)).hex() == d["pubkey"]
    assert d["withdrawal_credentials"] == "00fad2a6bfb0e7f1f0f45460944fbd8dfa7f37da06a4d13b3983cc90bb46963b"
    root = bytes.fromhex(d["signing_root"])
    assert O.g2_to_bytes(O.sign(sk, root)).hex() == d["signature"]
    sig = O.signature_from_bytes(bytes.fromhex(d["signature"]))
    assert O.core_verify(O.sk_to_pk(sk), root, sig)
    assert not O.core_verify(O.sk_to_pk(sk), bytes(32), sig)


def test_mainnet_signatures_deserialize_and_subgroup():
    """packages/beacon-node/test/unit/sync/backfill/blocks.json: 53 real G2 signatures."""
    sigs = KATS["mainnet_signatures"]
    assert len(sigs) == 53
    for s in sigs:
        pt = O.signature_from_bytes(bytes.fromhex(s))
        assert O.g2_to_bytes(pt).hex() == s


def test_valid_g2_point_oppool():
    """test/unit/chain/opPools/aggregatedAttestationPool.test.ts:24-27."""
    assert O.signature_from_bytes(bytes.fromhex(KATS["valid_g2_oppool"])) is not None


def test_negative_kats():
    """Buffer.alloc(96,10) must throw (bls.test.ts:48-49); 32 zero bytes -> false (multithread.test.ts:114-121)."""
    for h in KATS["malformed_signatures"]:
        with pytest.raises(O.DeserializeError):
            O.signature_from_bytes(bytes.fromhex(h))
    assert O.signature_from_bytes(bytes.fromhex(KATS["g2_infinity"])) is None  # G2_POINT_AT_INFINITY


def test_rfc9380_expand_message_xmd():
    """RFC 9380 K.1 (SHA-256, DST QUUX-V01-CS02-with-expander-SHA256-128)."""
    dst = b"QUUX-V01-CS02-with-expander-SHA256-128"
    assert O.expand_message_xmd(b"", dst, 0x20).hex() == \
        "68a985b87eb6b46952128911f2a4412bbc302a9d759667f87f7a21d803f07235"
    assert O.expand_message_xmd(b"abc", dst, 0x20).hex() == \
        "d8ccab23b5985ccea865c6c97b6e5b8350e794e603b4b97902f53a8a0d605615"


def test_rfc9380_hash_to_g2_empty_message():
    """RFC 9380 J.10.1 BLS12381G2_XMD:SHA-256_SSWU_RO_, msg = ''."""
    dst = b"QUUX-V01-CS02-with-BLS12381G2_XMD:SHA-256_SSWU_RO_"
    u = O.hash_to_field_fp2(b"", 2, dst)
    assert u[0][0] == 0x03dbc2cce174e91ba93cbb08f26b917f98194a2ea08d1cce75b2b9cc9f21689d80bd79b594a613d0a68eb807dfdc1cf8
    assert u[0][1] == 0x05a2acec64114845711a54199ea339abd125ba38253b70a92c876df10598bd1986b739cad67961eb94f7076511b3b39a
    h = O.hash_to_g2(b"", dst)
    assert h[0][0] == 0x0141ebfbdca40eb85b87142e130ab689c673cf60f1a3e98d69335266f30d9b8d4ac44c1038e9dcdd5393faf5c41fb78a
    assert h[0][1] == 0x05cb8437535e20ecffaef7752baddf98034139c38452458baeefab379ba13dff5bf5dd71b72418717047f5b0f37da03d


def test_isogeny_maps_onto_e2_and_is_homomorphic():
    rnd = random.Random(3)
    a = O.map_to_curve_sswu((rnd.randrange(O.P), rnd.randrange(O.P)))
    b = O.map_to_curve_sswu((rnd.randrange(O.P), rnd.randrange(O.P)))
    assert O.E2.on_curve(O.iso_map_g2(a))
    assert O.iso_map_g2(O.E2_ISO.add(a, b)) == O.E2.add(O.iso_map_g2(a), O.iso_map_g2(b))


def test_pairing_bilinear_and_order_r():
    e = O.pairing(O.G1, O.G2)
    assert e != O.F12_ONE
    assert O.f12_pow(e, O.R) == O.F12_ONE
    assert O.pairing(O.g1_mul(O.G1, 12345), O.g2_mul(O.G2, 678)) == O.f12_pow(e, 12345 * 678)


def test_final_exp_chain_identity():
    """3 (p^4 - p^2 + 1)/r = (x-1)^2 (x+p) (x^2+p^2-1) + 3 (used by the GPU final exponentiation)."""
    x, p, r = O.X_PARAM, O.P, O.R
    assert (x - 1) ** 2 * (x + p) * (x * x + p * p - 1) + 3 == 3 * (p ** 4 - p ** 2 + 1) // r


def test_g2_subgroup_check_psi_equivalence():
    """psi(P) == [x]P (GPU test) agrees with [r]P == O (definition) on members and non-members."""
    rnd = random.Random(9)
    for k in (1, 2, 999):
        P = O.g2_mul(O.G2, k)
        assert O.psi(P) == O.g2_mul(P, O.X_PARAM)
    n_non = 0
    while n_non < 3:
        x = (rnd.randrange(O.P), rnd.randrange(O.P))
        y = O.f2_sqrt(O.f2_add(O.f2_mul(O.f2_sqr(x), x), (4, 4)))
        if y is None:
            continue
        P = (x, y)
        assert (O.psi(P) == O.g2_mul(P, O.X_PARAM)) == O.g2_in_subgroup(P)
        n_non += 1


def test_batch_scalar_drbg():
    seed = bytes(range(32))
    w = OB.batch_scalar_raw(seed, 5)
    assert w == int.from_bytes(hashlib.sha256(seed + (5).to_bytes(4, "little")).digest()[:8], "little")
    r = OB.batch_scalar(seed, 5)
    assert r == ((w & 0xFFFFFFFF) + (w >> 32) * OB.GLV_LAMBDA) % O.R


def test_glv_eigenvalues():
    """lambda = -x^2 is the eigenvalue of phi on G1 and of -psi^2 on G2 (the
    endomorphisms the device's jac_mul_glv uses)."""
    lam = OB.GLV_LAMBDA
    assert (lam * lam + lam + 1) % O.R == 0
    P = O.g1_mul(O.G1, 12345)
    # the two primitive cube roots of unity mod p; one of them is the device's beta
    g = next(c for c in range(2, 100) if pow(c, (O.P - 1) // 3, O.P) != 1)
    w = pow(g, (O.P - 1) // 3, O.P)
    lam_P = O.g1_mul(P, lam)
    assert sum((P[0] * b % O.P, P[1]) == lam_P for b in (w, w * w % O.P)) == 1
    Q = O.g2_mul(O.G2, 6789)
    assert O.E2.neg(O.psi(O.psi(Q))) == O.g2_mul(Q, lam)


def test_chunkify_maximize_chunk_size():
    """multithread/utils.ts:4-19 semantics."""
    assert OB.chunkify_maximize_chunk_size(list(range(10)), 16) == [list(range(10))]
    assert OB.chunkify_maximize_chunk_size(list(range(31)), 16) == [list(range(31))]
    chunks = OB.chunkify_maximize_chunk_size(list(range(33)), 16)
    assert [len(c) for c in chunks] == [17, 16]
    chunks = OB.chunkify_maximize_chunk_size(list(range(300)), 128)
    assert [len(c) for c in chunks] == [150, 150]


def test_golden_verdict_scenarios_match_semantics_of_3set_batch():
    """Spot-check one golden verdict scenario on the CPU (the GPU suite replays all)."""
    v = load_golden("vectors.json")["verify_requests"][0]
    sets = []
    for st in v["requests"][0]:
        pk = O.g1_from_bytes(bytes.fromhex(st["pks"][0]))
        sets.append((pk, bytes.fromhex(st["msg"]), bytes.fromhex(st["sig"])))
    assert OB.verify_signature_sets_maybe_batch(sets) == v["expect"][0]


def test_expand_message_zpad_state_constant():
    """bls_hash.h expand_message_xmd_32 starts from the SHA-256 state after the all-zero
    Z_pad block (a constant): that state, completed with the padding block of a 64-byte
    message, must give hashlib's sha256(64 zero bytes)."""
    import hashlib
    import os
    import re
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lodestar_amd", "csrc",
                            "bls_hash.h")).read()
    m = re.search(r"uint32_t st\[8\] = \{([^}]*)\};", src)
    st = [int(x.strip().rstrip("u"), 16) for x in m.group(1).split(",")]
    K = [int(x) for x in (
        "1116352408 1899447441 3049323471 3921009573 961987163 1508970993 2453635748 2870763221 3624381080 "
        "310598401 607225278 1426881987 1925078388 2162078206 2614888103 3248222580 3835390401 4022224774 "
        "264347078 604807628 770255983 1249150122 1555081692 1996064986 2554220882 2821834349 2952996808 "
        "3210313671 3336571891 3584528711 113926993 338241895 666307205 773529912 1294757372 1396182291 "
        "1695183700 1986661051 2177026350 2456956037 2730485921 2820302411 3259730800 3345764771 3516065817 "
        "3600352804 4094571909 275423344 430227734 506948616 659060556 883997877 958139571 1322822218 "
        "1537002063 1747873779 1955562222 2024104815 2227730452 2361852424 2428436474 2756734187 3204031479 "
        "3329325298").split()]
    M = 0xFFFFFFFF

    def rotr(x, n):
        return ((x >> n) | (x << (32 - n))) & M

    def compress(state, block):
        w = list(block) + [0] * 48
        for i in range(16, 64):
            s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3)
            s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10)
            w[i] = (w[i - 16] + s0 + w[i - 7] + s1) & M
        a, b, c, d, e, f, g, h = state
        for i in range(64):
            t1 = (h + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + K[i] + w[i]) & M
            t2 = ((rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c))) & M
            h, g, f, e, d, c, b, a = g, f, e, (d + t1) & M, c, b, a, (t1 + t2) & M
        return [(x + y) & M for x, y in zip(state, [a, b, c, d, e, f, g, h])]

    digest = compress(st, [0x80000000] + [0] * 14 + [512])
    assert b"".join(x.to_bytes(4, "big") for x in digest) == hashlib.sha256(bytes(64)).digest()
