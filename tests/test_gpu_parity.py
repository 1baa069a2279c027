"""GPU parity: the HIP path (through the C ABI) against the CPU oracle's golden
fixtures and the reference's own KATs.  Bit-exact for every byte/integer output.

Run on an MI355X:  python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
"""
import hashlib
import random

import numpy as np
import pytest

from lodestar_amd.native import pack_blobs
from oracle import batch as OB
from oracle import bls12_381 as O
from tests.conftest import load_golden

pytestmark = pytest.mark.gpu

KATS = load_golden("kats.json")
VEC = load_golden("vectors.json")
R_ORDER = O.R


def interop_sk_be(i):
    return O.interop_secret_key(i).to_bytes(32, "big")


def run_requests(dev, requests, seed=bytes(32)):
    """requests: [[{"pks": [hex], "msg": hex, "sig": hex}, ...], ...] -> VerifyResult"""
    pks, pk_off, msgs, sigs, req_off = [], [0], [], [], [0]
    for req in requests:
        for st in req:
            pks += [bytes.fromhex(p) for p in st["pks"]]
            pk_off.append(len(pks))
            msgs.append(bytes.fromhex(st["msg"]))
            sigs.append(bytes.fromhex(st["sig"]))
        req_off.append(len(msgs))
    blob, offs = pack_blobs(sigs)
    return dev.verify_requests(np.array(req_off, np.uint32), np.frombuffer(b"".join(pks) or b"\0", np.uint8),
                               np.array(pk_off, np.uint32), np.frombuffer(b"".join(msgs) or b"\0", np.uint8), blob,
                               offs, seed)


# ---- reference KATs --------------------------------------------------------------
def test_sk_to_pk_interop_kat(device):
    """GPU keygen reproduces all 100 interop pubkeys (interop-pubkeys.json)."""
    out = device.sk_to_pk([interop_sk_be(i) for i in range(100)])
    for i, unc in enumerate(out):
        pt = O.g1_from_bytes(unc)
        assert O.g1_to_bytes(pt).hex() == KATS["interop_pubkeys"][i], i


def test_sign_deposit_kat(device):
    """GPU hash_to_G2 + sign reproduce the interop deposit signature (genesisState.test.ts:51-55)."""
    d = KATS["deposit"]
    sig = device.sign([interop_sk_be(0)], [bytes.fromhex(d["signing_root"])])[0]
    assert sig.hex() == d["signature"]


def test_mainnet_signatures_decode(device):
    sigs = [bytes.fromhex(s) for s in KATS["mainnet_signatures"]] + [bytes.fromhex(KATS["valid_g2_oppool"])]
    st, dec = device.decode_signatures(sigs)
    assert st == [0] * len(sigs)
    for s, d in zip(sigs, dec):
        assert O.g2_to_bytes(O.g2_from_bytes(d)) == s


def test_negative_kats_decode(device):
    st, _ = device.decode_signatures([bytes.fromhex(h) for h in KATS["malformed_signatures"]])
    assert st == [1, 1]


# ---- stage vectors (golden, oracle-generated) ------------------------------------------
def test_hash_to_g2_golden(device):
    out = device.hash_to_g2([bytes.fromhex(v["msg"]) for v in VEC["hash_to_g2"]])
    assert [o.hex() for o in out] == [v["point"] for v in VEC["hash_to_g2"]]


def test_signature_decode_golden(device):
    cases = VEC["sig_decode"]
    st, dec = device.decode_signatures([bytes.fromhex(c["bytes"]) for c in cases])
    for c, s, d in zip(cases, st, dec):
        assert s == c["status"], c["name"]
        if c["point"] is not None:
            assert d.hex() == c["point"], c["name"]


def test_pairing_golden(device):
    cases = VEC["pairing"]
    out = device.pairing([bytes.fromhex(c["g1"]) for c in cases], [bytes.fromhex(c["g2"]) for c in cases])
    assert [o.hex() for o in out] == [c["gt"] for c in cases]


def test_scalar_mul_golden(device):
    g1 = VEC["g1_mul"]
    out = device.g1_mul([bytes.fromhex(c["p"]) for c in g1], [int(c["k"]) for c in g1])
    assert [o.hex() for o in out] == [c["out"] for c in g1]
    g2 = VEC["g2_mul"]
    out = device.g2_mul([bytes.fromhex(c["p"]) for c in g2], [int(c["k"]) for c in g2])
    assert [o.hex() for o in out] == [c["out"] for c in g2]


def test_batch_scalars_golden(device):
    v = VEC["batch_scalars"]
    out = device.batch_scalars(bytes.fromhex(v["seed"]), v["first"], len(v["values"]))
    assert [str(x) for x in out] == v["values"]


def test_aggregate_pubkeys_golden(device):
    v = VEC["aggregate_pubkeys"]
    assert device.aggregate_pubkeys([bytes.fromhex(p) for p in v["pubkeys"]]).hex() == v["out"]


def test_aggregate_signatures_golden(device):
    v = VEC["aggregate_signatures"]
    out, bad = device.aggregate_signatures([bytes.fromhex(s) for s in v["signatures"]])
    assert bad == -1 and out.hex() == v["out"]


# ---- verdict scenarios (maybeBatch / worker semantics) -----------------------------------
@pytest.mark.parametrize("idx", range(len(VEC["verify_requests"])))
def test_verify_requests_scenarios(device_modes, idx):
    sc = VEC["verify_requests"][idx]
    res = run_requests(device_modes, sc["requests"])
    errors = sc.get("errors", [0] * len(sc["expect"]))
    assert list(res.errors) == errors, sc["name"]
    for e, v, err in zip(sc["expect"], res.valid, errors):
        if err == 0:
            assert bool(v) == e, sc["name"]


@pytest.mark.parametrize("idx", range(len(VEC["same_message"])))
def test_same_message_scenarios(device, idx):
    sc = VEC["same_message"][idx]
    verdicts, fast = device.verify_same_message([bytes.fromhex(p) for p in sc["pubkeys"]],
                                                [bytes.fromhex(s) for s in sc["signatures"]],
                                                bytes.fromhex(sc["message"]), bytes(32))
    assert verdicts == sc["expect"], sc["name"]
    assert fast == sc["fast_path"], sc["name"]


def test_same_message_empty(device):
    assert device.verify_same_message([], [], bytes(32), bytes(32)) == ([], False)


def test_aggregate_empty_rejects(device):
    from lodestar_amd.native import EmptyAggregateError
    with pytest.raises(EmptyAggregateError):
        device.aggregate_pubkeys([])


# ---- random cases vs the live oracle --------------------------------------------------
def test_sign_matches_oracle_random(device):
    rnd = random.Random(77)
    sks = [rnd.randrange(1, R_ORDER) for _ in range(6)]
    msgs = [bytes(rnd.getrandbits(8) for _ in range(32)) for _ in range(6)]
    out = device.sign([k.to_bytes(32, "big") for k in sks], msgs)
    for k, m, s in zip(sks, msgs, out):
        assert s == O.g2_to_bytes(O.sign(k, m))


def test_random_batches_vs_oracle(device_modes):
    """Random mixes of valid / wrong-message / malformed sets: verdicts equal oracle.batch."""
    device = device_modes
    rnd = random.Random(1234)
    n = 24
    sks = [interop_sk_be(i) for i in range(n)]
    pks = device.sk_to_pk(sks)
    msgs = [hashlib.sha256(b"rb" + bytes([i])).digest() for i in range(n)]
    sigs = device.sign(sks, msgs)
    reqs, expect = [], []
    i = 0
    while i < n:
        k = rnd.choice([1, 2, 3, 5])
        req = []
        for j in range(i, min(n, i + k)):
            sig = sigs[j]
            msg = msgs[j]
            roll = rnd.random()
            if roll < 0.15:
                msg = hashlib.sha256(b"other" + bytes([j])).digest()
            elif roll < 0.22:
                sig = bytes([rnd.getrandbits(8) for _ in range(96)])
            req.append({"pks": [pks[j].hex()], "msg": msg.hex(), "sig": sig.hex()})
        reqs.append(req)
        i += k
    res = run_requests(device, reqs)
    for req, v in zip(reqs, res.valid):
        want = all(OB.individually_valid(bytes.fromhex(s["pks"][0]), bytes.fromhex(s["msg"]), bytes.fromhex(s["sig"]))
                   for s in req) if req else False
        assert bool(v) == want


# ---- full-size properties (BASELINE.json config sizes) -----------------------------------
def _gen(device, n, tag):
    sks = [interop_sk_be(i) for i in range(n)]
    msgs = [hashlib.sha256(tag + i.to_bytes(8, "little")).digest() for i in range(n)]
    pks, sigs = [], []
    for s in range(0, n, 8192):
        pks += device.sk_to_pk(sks[s:s + 8192])
        sigs += device.sign(sks[s:s + 8192], msgs[s:s + 8192])
    return pks, msgs, sigs


def test_c2_full_size_with_injected_invalids(device):
    """65,536 sets (BASELINE configs[1]) in 512 requests of 128: all valid except the
    requests holding injected invalid sets (wrong message / malformed)."""
    n, per = 65536, 128
    pks, msgs, sigs = _gen(device, n, b"c2")
    rnd = random.Random(42)
    bad = sorted(rnd.sample(range(n), 20))
    msgs2, sigs2 = list(msgs), list(sigs)
    for t, j in enumerate(bad):
        if t % 2:
            msgs2[j] = bytes(32)
        else:
            sigs2[j] = bytes([10]) * 96
    blob, offs = pack_blobs(sigs2)
    res = device.verify_requests(np.arange(0, n + 1, per, dtype=np.uint32), np.frombuffer(b"".join(pks), np.uint8),
                                 None, np.frombuffer(b"".join(msgs2), np.uint8), blob, offs, bytes(32))
    bad_req = {j // per for j in bad}
    assert [k for k in range(n // per) if not res.valid[k]] == sorted(bad_req)
    assert not res.errors.any()


def test_c3_committee_aggregation_2048(device):
    """2048-pubkey aggregation -> 96-byte uncompressed, bit-exact vs the oracle (config C3)."""
    n = 2048
    sks = [interop_sk_be(i) for i in range(n)]
    pks = device.sk_to_pk(sks)
    got = device.aggregate_pubkeys(pks)
    ssum = sum(O.interop_secret_key(i) for i in range(n)) % R_ORDER
    assert got == O.g1_to_bytes(O.sk_to_pk(ssum), compressed=False)


def test_c3_sync_aggregate_512(device):
    """512-key same-message sync aggregate: aggregate set verifies; one wrong key fails."""
    n = 512
    sks = [interop_sk_be(i) for i in range(n)]
    pks = device.sk_to_pk(sks)
    msg = hashlib.sha256(b"sync").digest()
    sigs = device.sign(sks, [msg] * n)
    agg_sig, bad = device.aggregate_signatures(sigs)
    assert bad == -1
    blob, offs = pack_blobs([agg_sig, agg_sig])
    pk_all = b"".join(pks) + b"".join(pks[:-1]) + pks[0]
    res = device.verify_requests(np.array([0, 1, 2], np.uint32), np.frombuffer(pk_all, np.uint8),
                                 np.array([0, n, 2 * n], np.uint32), np.frombuffer(msg * 2, np.uint8), blob, offs,
                                 bytes(32))
    assert list(res.valid) == [1, 0]


# ---- mixed block-import / gossip workloads vs the C oracle (configs C4 / C5 shapes) ----------
def _mixed_workload(device, n_keys=512, n_sets=1500, seed=5, inject=True):
    """Single sets, committee aggregates (2..64 pubkeys, same message, 192-byte
    aggregated signature), and injected failures: wrong message, malformed
    signatures (Buffer.alloc(96, 10), 32 zero bytes), infinite signature,
    bad pubkey bytes, empty aggregate.  Requests of 1..128 sets."""
    rnd = random.Random(seed)
    sks = [interop_sk_be(i) for i in range(n_keys)]
    pks = device.sk_to_pk(sks)
    # plan the sets, then sign everything in one device call
    plan, msgs = [], []
    for j in range(n_sets):
        msgs.append(hashlib.sha256(b"mixed" + j.to_bytes(4, "little")).digest())
        plan.append(rnd.sample(range(n_keys), rnd.randint(2, 64)) if rnd.random() < 0.15 else [rnd.randrange(n_keys)])
    flat_sig = device.sign([sks[m] for p in plan for m in p], [msgs[j] for j, p in enumerate(plan) for _ in p])
    set_pks, sigs, at = [], [], 0
    for p in plan:
        part = flat_sig[at:at + len(p)]
        at += len(p)
        set_pks.append([pks[m] for m in p])
        if len(p) == 1:
            sigs.append(part[0])
        else:
            msig, bad = device.aggregate_signatures(part)
            assert bad == -1
            sigs.append(msig)
    for j in rnd.sample(range(n_sets), 40 if inject else 0):
        kind = rnd.randrange(6)
        if kind == 0:
            msgs[j] = bytes(32)
        elif kind == 1:
            sigs[j] = bytes([10]) * 96
        elif kind == 2:
            sigs[j] = bytes(32)
        elif kind == 3:
            sigs[j] = bytes([0xC0]) + bytes(95)
        elif kind == 4:
            set_pks[j] = [bytes(rnd.getrandbits(8) for _ in range(96))]
        else:
            set_pks[j] = []
    req_off = [0]
    while req_off[-1] < n_sets:
        req_off.append(min(n_sets, req_off[-1] + rnd.choice([1, 1, 2, 3, 16, 64, 128])))
    flat, pk_off = [], [0]
    for s in set_pks:
        flat += s
        pk_off.append(len(flat))
    blob, offs = pack_blobs(sigs)
    return (np.array(req_off, np.uint32), np.frombuffer(b"".join(flat), np.uint8), np.array(pk_off, np.uint32),
            np.frombuffer(b"".join(msgs), np.uint8), blob, offs)


@pytest.fixture(scope="module")
def mixed_workload(device):
    return _mixed_workload(device)


def test_mixed_workload_vs_c_oracle(device_modes, mixed_workload):
    """GPU verdicts and rejection codes == the C oracle's, request by request."""
    from oracle import c_oracle as C
    args = mixed_workload
    seed = hashlib.sha256(b"mixed-seed").digest()
    res = device_modes.verify_requests(*args, seed)
    valid, err = C.verify_requests(*args, seed, threads=16)
    assert list(res.errors) == list(err)
    assert list(res.valid) == list(valid)
    assert 0 < int(valid.sum()) < len(valid)  # the injections hit some requests, not all


@pytest.mark.parametrize("split,tail_prio", [("1", "0"), ("0", "0"), ("0", "1")])
def test_mixed_workload_split_halves_vs_c_oracle(mixed_workload, split, tail_prio):
    """The pair-major Miller accumulation (k_miller_acc, LB_ACC=pairs) with every
    request split in two halves (k_split_requests / k_join_halves, LB_ACC_SPLIT=1)
    and never split, both forced onto the stored-lines organisation, and the merged
    check on the shared high-priority stream (LB_TAIL_PRIO=1): verdicts and
    rejection codes == the C oracle's (1-set requests have an empty half)."""
    import os

    from lodestar_amd.native import Device
    from oracle import c_oracle as C
    old = {k: os.environ.get(k) for k in ("LB_MILLER", "LB_ACC_SPLIT", "LB_TAIL_PRIO", "LB_ACC")}
    os.environ.update(LB_MILLER="lines", LB_ACC_SPLIT=split, LB_TAIL_PRIO=tail_prio, LB_ACC="pairs")
    try:
        dev = Device(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    try:
        seed = hashlib.sha256(b"split-seed").digest()
        res = dev.verify_requests(*mixed_workload, seed)
        valid, err = C.verify_requests(*mixed_workload, seed, threads=16)
        assert list(res.errors) == list(err)
        assert list(res.valid) == list(valid)
        if split == "1":
            assert "join_halves" in dict(dev.last_stage_times())
    finally:
        dev.close()


def _device_with_env(**env):
    import os

    from lodestar_amd.native import Device
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return Device(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.parametrize("wide", ["1", "lanes", "0", "chunk1", "chunk16"])
@pytest.mark.parametrize("mtail", ["1", "0"])
@pytest.mark.parametrize("inject", [True, False])
def test_mixed_workload_bucket_msm_vs_c_oracle(device, inject, mtail, wide):
    """The merged check's sum of r_i sig_i from the bucket MSM (k_msm.hip), forced
    onto this 1,500-set call (LB_MSM_MIN=1; by default calls of >= 1025 sets):
    with injected failures the merged check fails and the per-request tails take
    their S_k from the per-set ladders; without, the merged check passes on the
    MSM's sum alone.  The merged check itself runs as the round program (LB_MTAIL=1,
    k_lp_mtail: S_all from the MSM's bit sums, its Miller value, the final
    exponentiation) or as the one-lane / one-wave chain (msm_final, lines of S_all,
    k_tail).  A lone call's wide forms (the merged check on 64 rows, the MSM's sums over
    more lanes, its bit sums as three levels of round programs) and the narrow ones of calls
    sharing the GPU (LB_WIDE_TAIL=0, LB_MSM_LANES=0); "lanes": the bit sums by k_msm_bits'
    256 threads instead of the programs (LB_MSM_BITS_LP=0).  A lone call of this size accumulates
    chunks of <= 4 entries; "chunk1" / "chunk16": chunks of one entry (LB_MSM_T_LONE=1) / the
    shared calls' 16 (LB_MSM_SHORT=0; with the hash as k_hash_half + the hash finish's 16-row program,
    LB_LP_HASH_FULL=0 / LB_LP_NARROW=0, instead of the default whole-hash program).  Verdicts and rejection codes == the C oracle's."""
    from oracle import c_oracle as C
    args = mixed_workload_cache(device, inject)
    seed = hashlib.sha256(b"msm-seed").digest()
    w = "0" if wide == "0" else "1"
    chunks = {"chunk1": {"LB_MSM_T_LONE": "1"}, "chunk16": {"LB_MSM_SHORT": "0", "LB_LP_NARROW": "0", "LB_LP_HASH_FULL": "0"}}.get(wide, {})
    dev = _device_with_env(LB_MSM_MIN="1", LB_MILLER="lines", LB_MTAIL=mtail, LB_WIDE_TAIL=w, LB_MSM_LANES=w,
                           LB_MSM_BITS_LP="0" if wide == "lanes" else "1", **chunks)
    try:
        res = dev.verify_requests(*args, seed)
        stages = dict(dev.last_stage_times())
        valid, err = C.verify_requests(*args, seed, threads=16)
        assert list(res.errors) == list(err)
        assert list(res.valid) == list(valid)
        assert "msm_chunks" in stages
        assert ("mtail" in stages) == (mtail == "1") and ("msm_final" in stages) == (mtail == "0")
        if inject:
            assert res.batch_retries == 1 and "scalar_sig" in stages
        else:
            assert all(valid) and res.batch_retries == 0
    finally:
        dev.close()


_MIXED = {}


def mixed_workload_cache(device, inject):
    if inject not in _MIXED:
        _MIXED[inject] = _mixed_workload(device, inject=inject)
    return _MIXED[inject]


@pytest.mark.parametrize("mode,waves", [("0", "1"), ("1", "1"), ("0", "2")])
def test_mixed_workload_step_variants_vs_c_oracle(device, mode, waves):
    """The k_step_acc variants besides the default (one line at a time, two waves):
    paired lines at one and two waves/SIMD, the accumulator in LDS (LB_STEP_MODE /
    LB_STEP_WAVES), merged check failing and passing: verdicts == the C oracle's."""
    from oracle import c_oracle as C
    for inject in (True, False):
        args = mixed_workload_cache(device, inject)
        seed = hashlib.sha256(b"step-variant" + mode.encode() + waves.encode()).digest()
        dev = _device_with_env(LB_MILLER="lines", LB_MSM_MIN="1", LB_STEP_MODE=mode, LB_STEP_WAVES=waves)
        try:
            res = dev.verify_requests(*args, seed)
            valid, err = C.verify_requests(*args, seed, threads=16)
            assert list(res.errors) == list(err)
            assert list(res.valid) == list(valid)
            assert res.batch_retries == (1 if inject else 0)
        finally:
            dev.close()


@pytest.mark.parametrize("msm,merge", [("0", "8"), ("1", "8"), ("0", "0"), ("1", "1")])
@pytest.mark.parametrize("inject", [True, False])
def test_mixed_workload_steps_vs_c_oracle(device, msm, merge, inject):
    """The step-major Miller accumulation (k_steps.hip: requests ordered by size,
    68 consecutive lines per lane, level products, one Horner chain), forced onto
    this 1,500-set call of ragged requests (1 .. 128 sets): merged check with S_all
    from the per-request sums (LB_MSM_MIN=0) or the bucket MSM (1), merged check
    passing (no injections) or failing (per-request Horner values, k_req_horner), and
    no merged check at all (LB_MERGE_MIN=0: every request's tail).  Verdicts and
    rejection codes == the C oracle's."""
    from oracle import c_oracle as C
    args = mixed_workload_cache(device, inject)
    seed = hashlib.sha256(b"steps-seed" + msm.encode() + merge.encode()).digest()
    dev = _device_with_env(LB_MILLER="lines", LB_MSM_MIN=msm, LB_MERGE_MIN=merge)
    try:
        res = dev.verify_requests(*args, seed)
        stages = dict(dev.last_stage_times())
        valid, err = C.verify_requests(*args, seed, threads=16)
        assert list(res.errors) == list(err)
        assert list(res.valid) == list(valid)
        assert "step_acc" in stages and "miller_acc" not in stages
        if merge != "0":
            # (the bucket MSM's merged check runs as the mtail round program, which folds the
            # Horner chain over the level products into its Miller loop: no k_horner_all)
            assert ("horner_all" in stages) == (msm == "0") and ("mtail" in stages) == (msm == "1")
            assert "level_prod" in stages and "level_wc" in stages  # (the two-stage level products)
            assert "req_horner" in stages  # (skips itself when the check passes)
            assert res.batch_retries == (1 if inject else 0)
        else:
            assert "req_horner" in stages and "horner_all" not in stages
    finally:
        dev.close()


@pytest.mark.parametrize("split", ["", "1", "2"])
@pytest.mark.parametrize("level", ["1", "0"])
@pytest.mark.parametrize("layout", ["mixed", "one_large"])
def test_steps_uniform_and_single_requests_vs_c_oracle(device, layout, level, split):
    """Row layout edge cases of the steps organisation: equal-size requests (the
    coalesced C2 shape), one-set requests (a lane runs the whole Miller loop), a
    request larger than 68 sets next to small ones, an empty request; and a
    1,200-set request beside small ones (its lanes of a level spread over all the
    threads of k_level_part / k_level_prod).  The level products both ways: lane
    products + wave-cooperative passes (LB_LEVEL=1, default) and k_level_prod's
    one-lane LDS tree (LB_LEVEL=0); the lanes of the accumulation split in 4 (a lone
    call of this size, default), 2 or not at all (LB_STEP_SPLIT): 17, 34 or 68 lines a
    lane."""
    from oracle import c_oracle as C
    req_off, pks, pk_off, msgs, blob, offs = mixed_workload_cache(device, layout == "mixed")
    n = len(pk_off) - 1
    sizes = [128] * 6 + [1] * 40 + [300, 0, 2, 67, 68, 69] if layout == "mixed" else [3, 1200] + [20] * 8
    off = [0]
    for z in sizes:
        off.append(min(n, off[-1] + z))
    off[-1] = n
    seed = hashlib.sha256(b"steps-rows").digest()
    env = {"LB_STEP_SPLIT": split} if split else {}
    if split == "1":  # (and the signatures decoded by k_decode_sigs instead of the round programs)
        env["LB_LP_DECODE"] = "0"
    dev = _device_with_env(LB_MILLER="lines", LB_LEVEL=level, **env)
    try:
        ro = np.array(off, np.uint32)
        res = dev.verify_requests(ro, pks, pk_off, msgs, blob, offs, seed)
        valid, err = C.verify_requests(ro, pks, pk_off, msgs, blob, offs, seed, threads=16)
        assert list(res.errors) == list(err)
        assert list(res.valid) == list(valid)
        stages = dict(dev.last_stage_times())
        assert "step_acc" in stages and "level_prod" in stages and ("level_wc" in stages) == (level == "1")
        if layout == "one_large":  # all valid: the merged check itself must pass (no per-request retry)
            assert all(valid) and res.batch_retries == 0
    finally:
        dev.close()


def test_poll_reports_completion_without_blocking(device, mixed_workload):
    """lb_poll (the N-API worker's non-blocking retire test): False while a call
    runs, True once its device work is done, True for a retired ticket; the
    verdicts through poll-then-wait equal a plain wait's."""
    import time
    seed = hashlib.sha256(b"poll-seed").digest()
    ref = device.verify_requests(*mixed_workload, seed)
    pc = device.verify_requests_async(*mixed_workload, seed)
    seen_busy = not device.poll(pc.ticket)
    t0 = time.time()
    while not device.poll(pc.ticket):
        assert time.time() - t0 < 60
        time.sleep(0.0005)
    res = device.wait_call(pc)
    assert seen_busy  # a 1,500-set call takes milliseconds: the first poll saw it running
    assert device.poll(pc.ticket)  # retired
    assert list(res.valid) == list(ref.valid) and list(res.errors) == list(ref.errors)


@pytest.mark.parametrize("inject", [True, False])
@pytest.mark.parametrize("n_req_sets", [(1, 1000), (0, 960)])
def test_lone_mid_call_pipeline_vs_c_oracle(device, inject, n_req_sets):
    """A lone call of lp_lone_max (896) < n_sets <= lp_max_sets (1,024) leaves the latency path
    for the pipeline's steps + MSM + merged-check program, merged whatever its request count
    (run_pipeline's lone_mid): a mixed 960-set workload of 1..128-set requests, and one request
    of 1,000 single sets.  Verdicts and rejection codes == the C oracle's; the default context
    (no explicit latency-path bound)."""
    from oracle import c_oracle as C
    from lodestar_amd.native import Device
    one, n = n_req_sets
    args = _mixed_workload(device, n_keys=256, n_sets=n, seed=23, inject=inject)
    if one:
        args = (np.array([0, n], np.uint32),) + tuple(args[1:])
    seed = hashlib.sha256(b"lone-mid").digest()
    dev = Device(0)
    try:
        res = dev.verify_requests(*args, seed)
        stages = dict(dev.last_stage_times())
        valid, err = C.verify_requests(*args, seed, threads=16)
        assert list(res.errors) == list(err)
        assert list(res.valid) == list(valid)
        assert "lp_verify" not in stages and "mtail" in stages and "msm_chunks" in stages
    finally:
        dev.close()
