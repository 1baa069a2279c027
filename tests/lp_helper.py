"""Inputs of the latency path's set programs built from the oracle (test
infrastructure): hash_to_field of the signing root, the signature's x
coordinate and flags, the pubkey, the GLV halves of the batch scalar."""
import hashlib

from oracle import bls12_381 as O

P = O.P
R = 1 << 384       # the one-lane code's Montgomery radix: the set programs' inputs
R416 = 1 << 416    # the latency path's radix: Miller values between programs
RINV = pow(R416, -1, P)
LB_PROG_SET_SINGLE, LB_PROG_SET_BATCH, LB_PROG_MUL, LB_PROG_FINAL = range(4)


def mont(v):
    return v % P * R % P


def mont416(v):
    return v % P * R416 % P


def set_inputs(pk, msg: bytes, sig_bytes: bytes, raw_scalar: int = 0):
    """(fp inputs as field values, flag inputs) of one set; sig_bytes compressed (96)
    or uncompressed (192), already past the byte-level checks."""
    u = O.hash_to_field_fp2(msg, 2, O.DST_POP)
    comp = len(sig_bytes) == 96
    inf = (sig_bytes[0] & 0x40) != 0
    sign = (sig_bytes[0] >> 5) & 1 if comp else 0
    x1 = int.from_bytes(sig_bytes[:48], "big") & ((1 << 381) - 1)
    x0 = int.from_bytes(sig_bytes[48:96], "big")
    y1 = y0 = 0
    if not comp:
        y1 = int.from_bytes(sig_bytes[96:144], "big")
        y0 = int.from_bytes(sig_bytes[144:192], "big")
    if inf:
        x0 = x1 = y0 = y1 = 0
    if pk is None:
        px, py, pz = 1, 1, 0
    elif len(pk) == 3:
        px, py, pz = pk
    else:
        px, py, pz = pk[0], pk[1], 1
    fps = [u[0][0], u[0][1], u[1][0], u[1][1], x0, x1, y0, y1, px, py, pz]
    a, b = raw_scalar & 0xFFFFFFFF, raw_scalar >> 32
    flags = [int(inf), sign, int(comp)] + [(a >> (31 - i)) & 1 for i in range(32)] + \
            [(b >> (31 - i)) & 1 for i in range(32)]
    return fps, flags


def f12_from_out(vals):
    """12 outputs (Montgomery, R = 2^416) -> oracle Fp12"""
    v = [x * RINV % P for x in vals]
    f2 = [(v[2 * i], v[2 * i + 1]) for i in range(6)]
    return ((f2[0], f2[1], f2[2]), (f2[3], f2[4], f2[5]))


def f12_fps(f):
    out = []
    for c6 in f:
        for c2 in c6:
            out += [c2[0], c2[1]]
    return out


def sample_sets(n: int, seed: bytes = b"lp"):
    sks = [O.interop_secret_key(i) for i in range(n)]
    msgs = [hashlib.sha256(seed + bytes([i])).digest() for i in range(n)]
    pks = [O.sk_to_pk(sk) for sk in sks]
    sigs = [O.g2_to_bytes(O.sign(sk, m)) for sk, m in zip(sks, msgs)]
    return pks, msgs, sigs
