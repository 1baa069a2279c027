"""BASELINE C4 composed in full on the one GPU we have: the 1M-set mainnet gossip
replay (8 x 125,000-set C4 shards: singles + AggregateAndProof triples with
488-key aggregates by validator index) verified as ONE sharded call over 8
contexts on cuda:0 -- what 8 MI355X run, one context each:
every shard stops at its 576-byte Fp12 partial, the host multiplies the 8
partials and runs ONE final exponentiation, every shard resumes with that
verdict (failed -> its per-request tails).  Reference: the pool's fan-out of
one package over workers, BN/chain/bls/multithread/index.ts:191-205.

* ShardedVerifier over 8 DeviceBackends (Python host), packed requests;
* verifyPackedSharded over 8 N-API addon contexts (node, the Lodestar host);
checked against the 8 shards verified unsharded, the known injection positions,
and a >= 2,000-set C-oracle sample (every injected request + random ones).
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import workloads as W  # noqa: E402

pytestmark = pytest.mark.gpu
N_SHARDS = 8


@pytest.fixture(scope="module")
def replay():
    """8 C4 shards (distinct seeds, 3 injected invalid sets each) concatenated into
    one packed call of 1,000,000 sets, plus the per-shard unsharded verdicts."""
    from lodestar_amd.native import Device
    from lodestar_amd.sharding import PackedRequests
    dev = Device(0)
    keys = W.make_keys(dev, 65536)
    assert dev.pubkey_table_append(keys.pks) == 65536
    shards = [W.c4_shard(dev, keys, seed=100 + g, n_invalid=3) for g in range(N_SHARDS)]
    per_shard = []
    for p in shards:
        blob, offs = p.blobs()
        r = dev.verify_requests(p.req_off, None, p.pk_off, p.msg_array(), blob, offs, bytes(32), pk_indices=p.idx)
        per_shard.append((list(r.valid), list(r.errors)))
    dev.close()
    req_off, pk_off, idx, msgs, sigs, expect_bad = [np.zeros(1, np.uint32)], [np.zeros(1, np.uint32)], [], [], [], set()
    r0 = s0 = k0 = 0
    for p in shards:
        req_off.append(p.req_off[1:] + s0)
        pk_off.append(p.pk_off[1:] + k0)
        idx.append(p.idx)
        msgs += p.msgs
        sigs += p.sigs
        expect_bad |= {r0 + k for k in p.expect_invalid_requests}
        r0 += p.n_req
        s0 += p.n_sets
        k0 += len(p.idx)
    from lodestar_amd.native import pack_blobs
    blob, offs = pack_blobs(sigs)
    packed = PackedRequests(np.concatenate(req_off).astype(np.uint32), np.concatenate(pk_off).astype(np.uint32),
                            np.frombuffer(b"".join(msgs), np.uint8), blob, offs,
                            idx=np.concatenate(idx).astype(np.uint32))
    want_v = [v for v, _ in per_shard for v in v]
    want_e = [e for _, e in per_shard for e in e]
    return keys, packed, msgs, sigs, expect_bad, (want_v, want_e)


@pytest.mark.timeout(900)
def test_c4_million_sets_8_contexts_python(replay):
    from lodestar_amd.sharding import ShardedVerifier
    from lodestar_amd.verifier import DeviceBackend
    keys, packed, _, _, expect_bad, (want_v, want_e) = replay
    assert int(packed.req_off[-1]) == N_SHARDS * 125000 and len(expect_bad) > 0
    backs = [DeviceBackend(0, seed_source=lambda: bytes(32), capacity=2) for _ in range(N_SHARDS)]
    try:
        for b in backs:
            assert b.sync_pubkeys(keys.pks) == 65536
        sv = ShardedVerifier(backs)
        valid, errors = sv.verify_packed(packed)
        assert sv.last_combine == {"merged_ok": False, "n_partials": N_SHARDS}
        assert [bool(v) for v in valid] == [bool(v) for v in want_v]
        assert errors == [int(e) for e in want_e]
        assert {k for k, v in enumerate(valid) if not v} == expect_bad
        # the requests before the first injection, sharded the same way: the combined
        # check of 8 partials passes and no shard runs a tail
        m = min(expect_bad)
        assert m >= N_SHARDS
        v2, e2 = sv.verify_packed(packed.slice(0, m))
        assert sv.last_combine == {"merged_ok": True, "n_partials": N_SHARDS}
        assert all(v2) and not any(e2)
    finally:
        for b in backs:
            b.close()


@pytest.mark.timeout(900)
def test_c4_million_sets_8_addon_contexts_node(replay):
    keys, packed, _, _, expect_bad, (want_v, want_e) = replay
    with tempfile.TemporaryDirectory() as d:
        for name, arr in (("req_off", packed.req_off), ("pk_off", packed.pk_off), ("idx", packed.idx),
                          ("msgs", packed.msgs), ("sigs", packed.sig_blob), ("sig_off", packed.sig_off)):
            np.ascontiguousarray(arr).tofile(os.path.join(d, name + ".bin"))
        np.frombuffer(b"".join(keys.pks), np.uint8).tofile(os.path.join(d, "keys.bin"))
        out = subprocess.run(["node", os.path.join(ROOT, "tests", "js", "c4_sharded.js"), d, str(N_SHARDS)],
                             capture_output=True, text=True, timeout=800)
    assert out.returncode == 0, out.stderr[-2000:]
    r = json.loads(out.stdout.strip().splitlines()[-1])
    valid = list(bytes.fromhex(r["valid"]))
    errors = list(bytes.fromhex(r["errors"]))
    assert r["mergedOk"] is False and r["tableSizes"] == [65536] * N_SHARDS
    assert [bool(v) for v in valid] == [bool(v) for v in want_v]
    assert errors == [int(e) for e in want_e]
    assert {k for k, v in enumerate(valid) if not v} == expect_bad


@pytest.mark.timeout(900)
def test_c4_million_sets_c_oracle_sample(replay):
    """Every request holding an injected set plus random others, >= 2,000 sets, re-verified
    by the C oracle (96-byte keys) == the sharded verdicts (== the unsharded ones)."""
    from lodestar_amd.native import pack_blobs
    from oracle import c_oracle as C
    keys, packed, msgs, sigs, expect_bad, (want_v, want_e) = replay
    rng = np.random.default_rng(4)
    pick = sorted(set(expect_bad) | set(int(k) for k in rng.choice(packed.n_req, 24, replace=False)))
    req_off, pk_off, pks, ms, ss = [0], [0], [], [], []
    for k in pick:
        for i in range(int(packed.req_off[k]), int(packed.req_off[k + 1])):
            ix = packed.idx[int(packed.pk_off[i]):int(packed.pk_off[i + 1])]
            pks += [keys.pks[int(j)] for j in ix]
            pk_off.append(len(pks))
            ms.append(msgs[i])
            ss.append(sigs[i])
        req_off.append(len(ms))
    assert len(ms) >= 2000
    blob, offs = pack_blobs(ss)
    valid, err = C.verify_requests(np.array(req_off, np.uint32), np.frombuffer(b"".join(pks), np.uint8),
                                   np.array(pk_off, np.uint32), np.frombuffer(b"".join(ms), np.uint8), blob, offs,
                                   hashlib.sha256(b"c4-sample").digest(), threads=16)
    assert [bool(v) for v in valid] == [bool(want_v[k]) for k in pick]
    assert [int(e) for e in err] == [int(want_e[k]) for k in pick]
    assert [bool(v) for v in valid] == [k not in expect_bad for k in pick]
