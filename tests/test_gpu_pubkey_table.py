"""Device-resident pubkey table: the index2pubkey mirror
(state-transition/src/cache/pubkeyCache.ts:56-77) and index-addressed sets.

Parity: table entries re-encode bit-exactly to the oracle's encodings of the
reference's 100 interop pubkeys (interop-pubkeys.json, decoded from the 48-byte
compressed form the state holds); index-addressed aggregation equals the
oracle's G1 sum; index-addressed verification gives the same verdicts and
rejection codes as the byte path (and as the oracle) request by request.
"""
import hashlib

import numpy as np
import pytest

from lodestar_amd.native import BadPubkeyError, Device, EmptyAggregateError, LB_REQ_BAD_PUBKEY, \
    LB_REQ_EMPTY_AGGREGATE, pack_blobs
from lodestar_amd.verifier import BlsGpuVerifier, DeviceBackend, PublicKey, VerifySignatureOpts, aggregate_set, \
    single_set
from oracle import bls12_381 as O
from tests.conftest import load_golden

pytestmark = pytest.mark.gpu

KATS = load_golden("kats.json")
N_KEYS = 100


@pytest.fixture(scope="module")
def tdev():
    """A fresh context whose table holds the 100 interop validators (compressed, as in the state)."""
    dev = Device(0)
    size = dev.pubkey_table_append([bytes.fromhex(h) for h in KATS["interop_pubkeys"]])
    assert size == N_KEYS
    yield dev
    dev.close()


def sk_be(i):
    return O.interop_secret_key(i).to_bytes(32, "big")


def oracle_pk(i):
    return O.sk_to_pk(O.interop_secret_key(i))


def test_table_entries_reencode_to_interop_kats(tdev):
    out = tdev.pubkey_table_read(0, N_KEYS)
    for i, unc in enumerate(out):
        assert unc == O.g1_to_bytes(O.g1_from_bytes(bytes.fromhex(KATS["interop_pubkeys"][i])), compressed=False)
        assert O.g1_to_bytes(O.g1_from_bytes(unc)).hex() == KATS["interop_pubkeys"][i]


def test_append_rejects_bad_key_atomically(tdev):
    good = bytes.fromhex(KATS["interop_pubkeys"][0])
    bad = bytes([0x80]) + bytes([0xff]) * 47  # x >= p
    with pytest.raises(BadPubkeyError, match="pubkey 1 "):
        tdev.pubkey_table_append([good, bad, good])
    assert tdev.pubkey_table_size() == N_KEYS


def test_append_uncompressed_grow_and_truncate():
    dev = Device(0)
    try:
        pks = dev.sk_to_pk([sk_be(i) for i in range(5000)])  # forces a table reallocation (> 4096)
        assert dev.pubkey_table_append(pks[:3000]) == 3000
        assert dev.pubkey_table_append(pks[3000:]) == 5000
        assert dev.pubkey_table_read(0, 2) == pks[:2]
        assert dev.pubkey_table_read(4998, 2) == pks[4998:]
        dev.pubkey_table_truncate(10)
        assert dev.pubkey_table_size() == 10
        assert dev.pubkey_table_read(9, 1) == pks[9:10]
    finally:
        dev.close()


def test_aggregate_by_index_matches_bytes_and_oracle(tdev):
    idx = [3, 17, 17, 42, 99, 0]  # duplicates are summed, as PublicKey.aggregate does
    got = tdev.aggregate_pubkeys_indexed(idx)
    acc = None
    for i in idx:
        acc = oracle_pk(i) if acc is None else O.g1_add(acc, oracle_pk(i))
    assert got == O.g1_to_bytes(acc, compressed=False)
    assert got == tdev.aggregate_pubkeys([tdev.pubkey_table_read(i, 1)[0] for i in idx])
    assert tdev.aggregate_pubkeys_indexed([7]) == O.g1_to_bytes(oracle_pk(7), compressed=False)
    with pytest.raises(EmptyAggregateError):
        tdev.aggregate_pubkeys_indexed([])
    with pytest.raises(BadPubkeyError):
        tdev.aggregate_pubkeys_indexed([1, N_KEYS])


def _requests(tdev):
    """Mixed requests over the table: singles, committee aggregates, a wrong
    message, an out-of-range index, an empty aggregate, 1-set requests."""
    msgs = [hashlib.sha256(b"table" + bytes([i])).digest() for i in range(N_KEYS)]
    sigs = tdev.sign([sk_be(i) for i in range(N_KEYS)], msgs)
    root = hashlib.sha256(b"committee").digest()
    com_sig = {}

    def committee(ix):
        key = tuple(ix)
        if key not in com_sig:
            parts = tdev.sign([sk_be(i) for i in ix], [root] * len(ix))
            agg, bad = tdev.aggregate_signatures(parts)
            assert bad == -1
            com_sig[key] = agg
        return com_sig[key]

    reqs = []  # list of requests; a set = (indices, msg, sig)
    reqs.append([([i], msgs[i], sigs[i]) for i in range(0, 10)])                         # valid singles
    reqs.append([([i], msgs[i], sigs[i]) for i in range(10, 20)] +
                [(list(range(20, 84)), root, committee(list(range(20, 84))))])          # + 64-key aggregate
    bad = [([i], msgs[i], sigs[i]) for i in range(30, 36)]
    bad[2] = ([32], msgs[33], sigs[32])                                                 # wrong message
    reqs.append(bad)
    reqs.append([([5], msgs[5], sigs[5]), ([N_KEYS + 7], msgs[6], sigs[6])])            # index out of range
    reqs.append([([1], msgs[1], sigs[1]), ([], msgs[2], sigs[2])])                      # empty aggregate
    reqs.append([([77], msgs[77], sigs[77])])                                           # 1-set core verify
    reqs.append([(list(range(0, 100, 3)), root, committee(list(range(0, 100, 3))))])    # 1-set aggregate
    reqs.append([([50], msgs[51], sigs[50])])                                           # 1-set, wrong
    return reqs


def _pack(reqs):
    idx, pk_off, msgs, sigs, req_off = [], [0], [], [], [0]
    for r in reqs:
        for ix, m, s in r:
            idx += ix
            pk_off.append(len(idx))
            msgs.append(m)
            sigs.append(s)
        req_off.append(len(msgs))
    blob, offs = pack_blobs(sigs)
    return (np.array(req_off, np.uint32), np.array(idx, np.uint32), np.array(pk_off, np.uint32),
            np.frombuffer(b"".join(msgs), np.uint8), blob, offs)


def test_verify_by_index_matches_byte_path(tdev):
    reqs = _requests(tdev)
    req_off, idx, pk_off, msgs, blob, offs = _pack(reqs)
    seed = hashlib.sha256(b"seed").digest()
    by_idx = tdev.verify_requests(req_off, None, pk_off, msgs, blob, offs, seed, pk_indices=idx)
    table = tdev.pubkey_table_read(0, N_KEYS)
    pk_bytes = b"".join(table[i] if i < N_KEYS else bytes(96) for i in idx)
    by_bytes = tdev.verify_requests(req_off, np.frombuffer(pk_bytes, np.uint8), pk_off, msgs, blob, offs, seed)
    assert list(by_idx.valid) == list(by_bytes.valid)
    assert list(by_idx.errors) == list(by_bytes.errors)
    assert [bool(v) for v in by_idx.valid] == [True, True, False, False, False, True, True, False]
    assert list(by_idx.errors) == [0, 0, 0, LB_REQ_BAD_PUBKEY, LB_REQ_EMPTY_AGGREGATE, 0, 0, 0]


@pytest.mark.parametrize("n_req", [64])
def test_verify_by_index_merged_call_with_invalid(tdev, n_req):
    """>= 8 requests take the merged check; one injected invalid set must only
    fail its own request (the merged-failure fallback)."""
    # (the merged check is the throughput pipeline's: a call this small would otherwise take
    # the latency path, which checks each request on its own and never retries)
    tdev.set_latency_path(0)
    base = _requests(tdev)[:2]
    reqs = [list(base[k % 2]) for k in range(n_req)]
    r = reqs[37]
    ix, m, s = r[3]
    r[3] = (ix, hashlib.sha256(b"other").digest(), s)
    req_off, idx, pk_off, msgs, blob, offs = _pack(reqs)
    res = tdev.verify_requests(req_off, None, pk_off, msgs, blob, offs, bytes(32), pk_indices=idx)
    assert [bool(v) for v in res.valid] == [k != 37 for k in range(n_req)]
    assert (res.batch_retries, res.batch_sigs_success) == (1, 0)  # worker.ts:80 merged batch retried
    # all valid: the merged check passes and covers every set (worker.ts:71)
    reqs[37][3] = (ix, m, s)
    req_off, idx, pk_off, msgs, blob, offs = _pack(reqs)
    res = tdev.verify_requests(req_off, None, pk_off, msgs, blob, offs, bytes(32), pk_indices=idx)
    assert res.valid.all()
    assert (res.batch_retries, res.batch_sigs_success) == (0, int(req_off[-1]))
    # the latency path: the same verdicts, no merged batch
    tdev.set_latency_path(1024)
    reqs[37][3] = (ix, hashlib.sha256(b"other").digest(), s)
    req_off, idx, pk_off, msgs, blob, offs = _pack(reqs)
    res = tdev.verify_requests(req_off, None, pk_off, msgs, blob, offs, bytes(32), pk_indices=idx)
    assert [bool(v) for v in res.valid] == [k != 37 for k in range(n_req)]
    assert res.batch_retries == 0


def test_bls_gpu_verifier_index_keys():
    backend = DeviceBackend(0, seed_source=lambda: bytes(32))
    try:
        v = BlsGpuVerifier(backends=[backend])
        assert v.sync_pubkeys([bytes.fromhex(h) for h in KATS["interop_pubkeys"][:40]]) == 40
        msgs = [hashlib.sha256(b"v" + bytes([i])).digest() for i in range(40)]
        sigs = backend.dev.sign([sk_be(i) for i in range(40)], msgs)
        root = hashlib.sha256(b"agg").digest()
        agg_sig, _ = backend.dev.aggregate_signatures(backend.dev.sign([sk_be(i) for i in range(8)], [root] * 8))
        import asyncio

        async def main():
            sets = [single_set(PublicKey(index=i), msgs[i], sigs[i]) for i in range(20)]
            sets.append(aggregate_set([PublicKey(index=i) for i in range(8)], root, agg_sig))
            assert await v.verify_signature_sets(sets, VerifySignatureOpts(batchable=True)) is True
            wrong = list(sets)
            wrong[4] = single_set(PublicKey(index=5), msgs[4], sigs[4])
            assert await v.verify_signature_sets(wrong) is False
            # mixed package: index-only keys next to byte keys
            mixed = [single_set(PublicKey(O.g1_to_bytes(oracle_pk(30), compressed=False)), msgs[30], sigs[30]),
                     single_set(PublicKey(index=31), msgs[31], sigs[31])]
            assert await v.verify_signature_sets(mixed) is True
            with pytest.raises(BadPubkeyError):
                await v.verify_signature_sets([single_set(PublicKey(index=400), msgs[0], sigs[0])] + sets[:2])
        asyncio.run(main())
    finally:
        backend.close()


def test_infinity_key_in_table_gives_false_not_error():
    """fromBytes accepts the infinity encoding (no validation in syncPubkeys); a set
    over it is false (BLST_PK_IS_INFINITY caught in maybeBatch), not a rejection."""
    dev = Device(0)
    try:
        inf48 = bytes([0xC0]) + bytes(47)
        keys = [bytes.fromhex(h) for h in KATS["interop_pubkeys"][:3]] + [inf48]
        assert dev.pubkey_table_append(keys) == 4
        assert dev.pubkey_table_read(3, 1)[0] == bytes([0x40]) + bytes(95)
        msgs = [hashlib.sha256(bytes([i])).digest() for i in range(4)]
        sigs = dev.sign([sk_be(i) for i in range(3)], msgs[:3]) + [bytes([0xC0]) + bytes(95)]
        blob, offs = pack_blobs(sigs)
        req_off = np.array([0, 3, 4, 5], np.uint32)
        pk_off = np.array([0, 1, 2, 3, 4], np.uint32)
        # request 2 re-uses set 3's key with another set's data: (idx 3, msg 0, sig 0)
        sigs2, msgs2 = sigs + [sigs[0]], msgs + [msgs[0]]
        blob, offs = pack_blobs(sigs2)
        res = dev.verify_requests(req_off, None, np.array([0, 1, 2, 3, 4, 5], np.uint32),
                                  np.frombuffer(b"".join(msgs2), np.uint8), blob, offs, bytes(32),
                                  pk_indices=np.array([0, 1, 2, 3, 3], np.uint32))
        assert [bool(v) for v in res.valid] == [True, False, False]
        assert list(res.errors) == [0, 0, 0]
    finally:
        dev.close()
