"""CPU oracle: verdict semantics of Lodestar's BLS hot path.

TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke(), bench.py's
cpu_baseline leg).  Restates, on top of ``oracle.bls12_381``:

* ``verify_signature_sets_maybe_batch``  -- packages/beacon-node/src/chain/bls/maybeBatch.ts:16-46
* ``verify_multiple_signatures``         -- blst verifyMultipleAggregateSignatures as called at
  maybeBatch.ts:19-26 (Pairing.mul_n_aggregate with 64-bit scalars, commit, finalverify);
  the scalars come from the deterministic DRBG shared with the GPU
  (r_i = LE64(SHA-256(seed || LE32(i))[0..8]), 0 -> 1) instead of crypto.randomBytes
* ``verify_many_signature_sets``         -- multithread/worker.ts:30-108
* ``verify_same_message``                -- multithread/index.ts:218-242 + jobItem.ts:64-125
                                            (and singleThread.ts:37-81, same verdicts)
* ``chunkify_maximize_chunk_size``       -- multithread/utils.ts:4-19
"""
from __future__ import annotations

import hashlib
from typing import List, Optional, Sequence, Tuple

from . import bls12_381 as O

MIN_SET_COUNT_TO_BATCH = 2          # maybeBatch.ts:4
BATCHABLE_MIN_PER_CHUNK = 16        # worker.ts:17
MAX_SIGNATURE_SETS_PER_JOB = 128    # index.ts:57


# GLV eigenvalue shared by phi on G1 and -psi^2 on G2 (the maps the subgroup
# checks use): lambda = -x^2 mod r
GLV_LAMBDA = (-(O.X_PARAM * O.X_PARAM)) % O.R


def batch_scalar_raw(seed: bytes, i: int) -> int:
    """64-bit DRBG output w_i = LE64(SHA-256(seed || LE32(i))[0..8]), 0 -> 1
    (what the device's lb_batch_scalars returns)."""
    d = hashlib.sha256(bytes(seed) + int(i).to_bytes(4, "little")).digest()
    v = int.from_bytes(d[:8], "little")
    return v if v else 1


def batch_scalar(seed: bytes, i: int) -> int:
    """Batch scalar r_i = (w_i mod 2^32) + (w_i >> 32) * lambda (mod r).

    Like blst's 8 random bytes per set (maybeBatch.ts:19 -> mul_n_aggregate)
    this takes 2^64 distinct values (a + b lambda with a, b < 2^32 never
    collide: the lattice {(a, b): a + b lambda = 0 mod r} has no vector shorter
    than ~2^64), so the small-exponent batch test keeps its 2^-64 soundness;
    the split lets the device multiply with two 32-bit halves (GLV)."""
    w = batch_scalar_raw(seed, i)
    return ((w & 0xFFFFFFFF) + (w >> 32) * GLV_LAMBDA) % O.R


class BlsThrow(Exception):
    """Something @chainsafe/bls / blst would throw (caught by maybeBatch -> false)."""


def _pk(pk):
    """Accept an affine point, None (infinity) or 96/48-byte encoding."""
    if pk is None or isinstance(pk, tuple):
        return pk
    try:
        return O.g1_from_bytes(bytes(pk))
    except O.DeserializeError as e:
        raise BlsThrow(str(e))


def _sig(b: bytes):
    try:
        return O.signature_from_bytes(bytes(b), validate=True)
    except O.DeserializeError as e:
        raise BlsThrow(str(e))


def verify_multiple_signatures(sets, seed: bytes, index_base: int = 0) -> bool:
    """prod e(r_i pk_i, H(m_i)) * e(-g1, sum r_i sig_i) == 1 ; infinite pk -> throw."""
    f = O.F12_ONE
    S = None
    for i, (pk, msg, sig) in enumerate(sets):
        if pk is None:
            raise BlsThrow("BLST_PK_IS_INFINITY")
        r = batch_scalar(seed, index_base + i)
        S = O.E2.add(S, O.g2_mul(sig, r) if sig is not None else None)
        f = O.f12_mul(f, O.miller_loop(O.g1_mul(pk, r), O.hash_to_g2(msg)))
    if S is not None:
        f = O.f12_mul(f, O.miller_loop(O.E1.neg(O.G1), S))
    return O.f12_is_one(O.final_exp(f))


def core_verify_single(pk, msg: bytes, sig_bytes: bytes) -> bool:
    """``sig = Signature.fromBytes(bytes, affine, true); sig.verify(pk, msg)``
    (infinite signature -> ZeroSignatureError, infinite pk -> false)."""
    sig = _sig(sig_bytes)
    if sig is None:
        raise BlsThrow("ZeroSignatureError")
    return O.core_verify(pk, msg, sig)


def verify_signature_sets_maybe_batch(sets, seed: bytes = bytes(32), index_base: int = 0) -> bool:
    """sets: [(pubkey point | bytes, message, signature bytes)]  (maybeBatch.ts:16-46)."""
    try:
        if len(sets) >= MIN_SET_COUNT_TO_BATCH:
            dec = [(_pk(pk), bytes(m), _sig(s)) for pk, m, s in sets]
            return verify_multiple_signatures(dec, seed, index_base)
        if len(sets) == 0:
            raise BlsThrow("Empty signature set")
        return all(core_verify_single(_pk(pk), bytes(m), s) for pk, m, s in sets)
    except BlsThrow:
        return False


def individually_valid(pk, msg: bytes, sig_bytes: bytes) -> bool:
    """Validity of one set on its own (what every batch verdict reduces to)."""
    return verify_signature_sets_maybe_batch([(pk, msg, sig_bytes)])


def chunkify_maximize_chunk_size(arr: Sequence, min_per_chunk: int) -> List[list]:
    """multithread/utils.ts:4-19."""
    chunk_count = len(arr) // min_per_chunk
    if chunk_count <= 1:
        return [list(arr)]
    per_chunk = -(-len(arr) // chunk_count)
    return [list(arr[i:i + per_chunk]) for i in range(0, len(arr), per_chunk)]


def verify_many_signature_sets(work_reqs, seed: bytes = bytes(32)):
    """worker.ts:30-108.  work_reqs: [(batchable: bool, sets)] -> (results, batch_retries, batch_sigs_success)."""
    results: List[Optional[bool]] = [None] * len(work_reqs)
    batch_retries = 0
    batch_sigs_success = 0
    batchable = [(i, sets) for i, (b, sets) in enumerate(work_reqs) if b]
    non_batchable = [(i, sets) for i, (b, sets) in enumerate(work_reqs) if not b]
    if batchable:
        for chunk in chunkify_maximize_chunk_size(batchable, BATCHABLE_MIN_PER_CHUNK):
            all_sets = [s for _, sets in chunk for s in sets]
            if verify_signature_sets_maybe_batch(all_sets, seed):
                for idx, sets in chunk:
                    batch_sigs_success += len(sets)
                    results[idx] = True
            else:
                batch_retries += 1
                non_batchable.extend(chunk)
    for idx, sets in non_batchable:
        results[idx] = verify_signature_sets_maybe_batch(sets, seed)
    return results, batch_retries, batch_sigs_success


def verify_same_message(sets: Sequence[Tuple[object, bytes]], message: bytes) -> Tuple[List[bool], bool]:
    """One same-message job: [(pubkey, signature bytes)] -> (per-set verdicts, fast_path_ok).

    jobItemWorkReq(sameMessage) validates every signature (a throw -> retry each
    set alone), aggregates pubkeys and signatures with plain sums and verifies
    the single aggregated set; false -> retry each set alone (jobItem.ts:93-125).
    """
    if len(sets) == 0:
        return [], False
    pks = [_pk(pk) for pk, _ in sets]
    try:
        sigs = [_sig(s) for _, s in sets]
        agg_pk = O.aggregate_g1(pks)
        agg_sig = O.aggregate_g2(sigs)
        agg_bytes = O.g2_to_bytes(agg_sig, compressed=False)
        if verify_signature_sets_maybe_batch([(agg_pk, message, agg_bytes)]):
            return [True] * len(sets), True
    except BlsThrow:
        pass
    return [verify_signature_sets_maybe_batch([(pk, message, s)]) for pk, (_, s) in zip(pks, sets)], False
