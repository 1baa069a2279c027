"""Compressed (48-byte) pubkeys in a call: LB_PK_ROW48_FLAG rows, decompressed on the
GPU with PublicKey.fromBytes(48 B) semantics (the JS host ships a key as such when a
@chainsafe/bls PublicKey gives its compressed form, or the caller passes 48 bytes;
VERDICT r4 #1).  Requests and same-message packages mixing compressed rows,
uncompressed rows and table indices, against the oracle's verdicts."""
import hashlib

import numpy as np
import pytest

from lodestar_amd import native
from oracle import bls12_381 as O

pytestmark = pytest.mark.gpu

F, F48 = native.LB_PK_ROW_FLAG, native.LB_PK_ROW48_FLAG


@pytest.fixture(scope="module")
def env():
    dev = native.Device(0)
    n = 12
    sks = [O.interop_secret_key(i) for i in range(n)]
    pts = [O.sk_to_pk(sk) for sk in sks]
    unc = [O.g1_to_bytes(p, compressed=False) for p in pts]
    comp = [O.g1_to_bytes(p, compressed=True) for p in pts]
    msgs = [hashlib.sha256(b"row48" + bytes([i])).digest() for i in range(n)]
    sigs = [O.g2_to_bytes(O.sign(sk, m)) for sk, m in zip(sks, msgs)]
    base = dev.pubkey_table_size()
    dev.pubkey_table_append(unc[:4])
    yield dev, unc, comp, msgs, sigs, base
    dev.close()


def _row(b):
    return bytes(b) + bytes(96 - len(b))


@pytest.mark.parametrize("lp", [0, 1024])
def test_requests_with_compressed_rows(env, lp):
    dev, unc, comp, msgs, sigs, base = env
    dev.set_latency_path(lp)
    try:
        not_on_curve = bytearray(comp[5])
        for k in range(1, 256):  # an x with no point on the curve
            not_on_curve[47] = comp[5][47] ^ k
            try:
                O.g1_from_bytes(bytes(not_on_curve))
            except O.DeserializeError:
                break
        rows = [_row(comp[4]), _row(unc[5]), _row(comp[6]), _row(comp[7]), _row(comp[8]), _row(bytes(not_on_curve)),
                _row(bytes([0xc0]) + bytes(47))]
        # request 0: [compressed 4] [uncompressed 5] [aggregate: table 0 + compressed 6 + table 1]
        # request 1: [compressed 7] alone (core verify through the row)      -> valid
        # request 2: [compressed 8 over message 9]                          -> false
        # request 3: [a row that is no point]                              -> LB_REQ_BAD_PUBKEY
        # request 4: [the compressed infinity]                             -> false (infinite pubkey)
        parts = [O.sign(O.interop_secret_key(i), msgs[0]) for i in (0, 6, 1)]
        agg_sig = O.g2_to_bytes(O.g2_add(O.g2_add(parts[0], parts[1]), parts[2]))
        idx = [F | F48 | 0, F | 1, base + 0, F | F48 | 2, base + 1, F | F48 | 3, F | F48 | 4, F | F48 | 5, F | F48 | 6]
        pk_off = [0, 1, 2, 5, 6, 7, 8, 9]
        set_msgs = [msgs[4], msgs[5], msgs[0], msgs[7], msgs[9], msgs[1], msgs[2]]
        set_sigs = [sigs[4], sigs[5], agg_sig, sigs[7], sigs[8], sigs[1], sigs[2]]
        req_off = np.array([0, 3, 4, 5, 6, 7], np.uint32)
        blob, offs = native.pack_blobs(set_sigs)
        r = dev.verify_requests(req_off, np.frombuffer(b"".join(rows), np.uint8), np.array(pk_off, np.uint32),
                                np.frombuffer(b"".join(set_msgs), np.uint8), blob, offs, bytes(32),
                                pk_indices=np.array(idx, np.uint32))
        assert [int(v) for v in r.valid] == [1, 1, 0, 0, 0], (r.valid, r.errors)
        assert [int(e) for e in r.errors] == [0, 0, 0, native.LB_REQ_BAD_PUBKEY, 0], r.errors
    finally:
        dev.set_latency_path(1024)


def test_same_message_with_compressed_rows(env):
    dev, unc, comp, msgs, sigs, base = env
    root = hashlib.sha256(b"same root").digest()
    sm_sigs = [O.g2_to_bytes(O.sign(O.interop_secret_key(i), root)) for i in range(8)]
    rows = [_row(comp[5]), _row(unc[6]), _row(comp[7])]
    # job 0: table 0, compressed 5, uncompressed 6, compressed 7 -> all valid (fast path)
    # job 1: table 1, compressed 5 with key 2's signature        -> [True, False] (per-set retry)
    jobs = [([base + 0, F | F48 | 0, F | 1, F | F48 | 2], [sm_sigs[0], sm_sigs[5], sm_sigs[6], sm_sigs[7]], root),
            ([base + 1, F | F48 | 0], [sm_sigs[1], sm_sigs[2]], root)]
    res, fast, _ = dev.verify_same_message_batch(jobs, bytes(32), by_index=True,
                                                 rows=np.frombuffer(b"".join(rows), np.uint8))
    assert res == [[True, True, True, True], [True, False]], res
    assert fast == [True, False], fast
