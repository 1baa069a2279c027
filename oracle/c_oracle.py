"""ctypes front end of the C oracle (oracle/c/bls_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/ and bench.py's cpu_baseline leg,
never by lodestar_amd/.  The entry points mirror lodestar_amd.native.Device so
the same scenario helpers drive both.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import build_c

_lib = None


def variant() -> str:
    """Which build load() picks on this host."""
    return "x86-64-v3" if (os.path.exists(build_c.LIB_V3) and build_c.host_supports_v3()) else "x86-64-v2"


def load(build_if_missing: bool = True):
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(build_c.LIB) and build_if_missing:
        build_c.build()
    path = build_c.LIB_V3 if (os.path.exists(build_c.LIB_V3) and build_c.host_supports_v3()) else build_c.LIB
    lib = ctypes.CDLL(path)
    vp, u32, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
    lib.lbo_verify_requests.argtypes = [u32, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32]
    lib.lbo_hash_to_g2.argtypes = [u32, vp, vp]
    lib.lbo_decode_signatures.argtypes = [u32, vp, vp, vp, vp]
    lib.lbo_pairing.argtypes = [u32, vp, vp, vp]
    lib.lbo_sk_to_pk.argtypes = [u32, vp, vp]
    lib.lbo_sign.argtypes = [u32, vp, vp, vp]
    _lib = lib
    return lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _u8(b: bytes):
    return np.frombuffer(bytes(b) or b"\0", np.uint8)


def pack_blobs(items: Sequence[bytes]) -> Tuple[np.ndarray, np.ndarray]:
    offs = np.zeros(len(items) + 1, np.uint32)
    for i, s in enumerate(items):
        offs[i + 1] = offs[i] + len(s)
    return _u8(b"".join(items)), offs


def verify_requests(req_off, pubkeys, pk_off, messages, sig_blob, sig_off, seed: bytes, threads: int = 1):
    """Same arguments as Device.verify_requests -> (valid[n_req], errors[n_req])."""
    lib = load()
    req_off = np.ascontiguousarray(req_off, np.uint32)
    n_req = len(req_off) - 1
    valid = np.zeros(max(n_req, 1), np.uint8)
    err = np.zeros(max(n_req, 1), np.uint8)
    pk_off = None if pk_off is None else np.ascontiguousarray(pk_off, np.uint32)
    seed_a = _u8(seed)
    rc = lib.lbo_verify_requests(n_req, _p(req_off), _p(np.ascontiguousarray(pubkeys, np.uint8)), _p(pk_off),
                                 _p(np.ascontiguousarray(messages, np.uint8)),
                                 _p(np.ascontiguousarray(sig_blob, np.uint8)),
                                 _p(np.ascontiguousarray(sig_off, np.uint32)), _p(seed_a), _p(valid), _p(err),
                                 int(threads))
    assert rc == 0
    return valid[:n_req], err[:n_req]


def hash_to_g2(msgs: Sequence[bytes]) -> List[bytes]:
    lib = load()
    out = np.zeros(192 * len(msgs), np.uint8)
    lib.lbo_hash_to_g2(len(msgs), _p(_u8(b"".join(msgs))), _p(out))
    return [out[192 * i:192 * (i + 1)].tobytes() for i in range(len(msgs))]


def decode_signatures(sigs: Sequence[bytes]) -> Tuple[List[int], List[bytes]]:
    lib = load()
    blob, offs = pack_blobs(sigs)
    st = np.zeros(max(len(sigs), 1), np.uint8)
    out = np.zeros(192 * max(len(sigs), 1), np.uint8)
    lib.lbo_decode_signatures(len(sigs), _p(blob), _p(offs), _p(st), _p(out))
    return [int(s) for s in st[:len(sigs)]], [out[192 * i:192 * (i + 1)].tobytes() for i in range(len(sigs))]


def pairing(g1s: Sequence[bytes], g2s: Sequence[bytes]) -> List[bytes]:
    lib = load()
    out = np.zeros(576 * len(g1s), np.uint8)
    lib.lbo_pairing(len(g1s), _p(_u8(b"".join(g1s))), _p(_u8(b"".join(g2s))), _p(out))
    return [out[576 * i:576 * (i + 1)].tobytes() for i in range(len(g1s))]


def sk_to_pk(sks_be32: Sequence[bytes]) -> List[bytes]:
    lib = load()
    out = np.zeros(96 * len(sks_be32), np.uint8)
    lib.lbo_sk_to_pk(len(sks_be32), _p(_u8(b"".join(sks_be32))), _p(out))
    return [out[96 * i:96 * (i + 1)].tobytes() for i in range(len(sks_be32))]


def sign(sks_be32: Sequence[bytes], msgs: Sequence[bytes]) -> List[bytes]:
    """96-byte compressed signatures sk * H(m)."""
    lib = load()
    out = np.zeros(96 * len(sks_be32), np.uint8)
    lib.lbo_sign(len(sks_be32), _p(_u8(b"".join(sks_be32))), _p(_u8(b"".join(msgs))), _p(out))
    return [out[96 * i:96 * (i + 1)].tobytes() for i in range(len(sks_be32))]


def run_requests(requests, seed: bytes = bytes(32), threads: int = 1):
    """requests: [[{"pks": [hex], "msg": hex, "sig": hex}, ...], ...] (tests/golden format)."""
    pks, pk_off, msgs, sigs, req_off = [], [0], [], [], [0]
    for req in requests:
        for st in req:
            pks += [bytes.fromhex(p) for p in st["pks"]]
            pk_off.append(len(pks))
            msgs.append(bytes.fromhex(st["msg"]))
            sigs.append(bytes.fromhex(st["sig"]))
        req_off.append(len(msgs))
    blob, offs = pack_blobs(sigs)
    return verify_requests(np.array(req_off, np.uint32), _u8(b"".join(pks)), np.array(pk_off, np.uint32),
                           _u8(b"".join(msgs)), blob, offs, seed, threads)
