"""Ad-hoc GPU-vs-oracle check used during bring-up (the real parity suite is tests/)."""
import os
import sys
import time
import random
import hashlib

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import bls12_381 as O  # noqa: E402
from lodestar_amd.native import Device  # noqa: E402


def gt_bytes(f):
    out = b""
    for c6 in f:
        for c2 in c6:
            out += c2[0].to_bytes(48, "big") + c2[1].to_bytes(48, "big")
    return out


def main():
    t0 = time.time()
    dev = Device(0)
    print("device ok", time.time() - t0, flush=True)
    rnd = random.Random(5)
    msgs = [bytes(rnd.getrandbits(8) for _ in range(32)) for _ in range(4)]
    t = time.time()
    hs = dev.hash_to_g2(msgs)
    print("hash_to_g2 gpu", time.time() - t, flush=True)
    ok = sum(hs[i] == O.g2_to_bytes(O.hash_to_g2(m), compressed=False) for i, m in enumerate(msgs))
    print("hash_to_g2 parity", ok, "/", len(msgs), flush=True)
    seed = bytes(range(32))
    sc = dev.batch_scalars(seed, 0, 4)
    exp = []
    for i in range(4):
        d = hashlib.sha256(seed + i.to_bytes(4, "little")).digest()
        v = int.from_bytes(d[:8], "little")
        exp.append(v if v else 1)
    print("scalars parity", sc == exp, flush=True)
    sks = [O.interop_secret_key(i) for i in range(4)]
    pks = [O.sk_to_pk(sk) for sk in sks]
    sigs = [O.sign(sk, m) for sk, m in zip(sks, msgs)]
    g1m = dev.g1_mul([O.g1_to_bytes(p, False) for p in pks], sc)
    print("g1_mul parity", all(g1m[i] == O.g1_to_bytes(O.g1_mul(pks[i], sc[i]), False) for i in range(4)), flush=True)
    g2m = dev.g2_mul([O.g2_to_bytes(s, False) for s in sigs], sc)
    print("g2_mul parity", all(g2m[i] == O.g2_to_bytes(O.g2_mul(sigs[i], sc[i]), False) for i in range(4)), flush=True)
    comp = [O.g2_to_bytes(s) for s in sigs]
    st, dec = dev.decode_signatures(comp + [bytes([10]) * 96, bytes(32)])
    print("decode status", st, "parity", all(dec[i] == O.g2_to_bytes(sigs[i], False) for i in range(4)), flush=True)
    t = time.time()
    gts = dev.pairing([O.g1_to_bytes(pks[0], False)], [O.g2_to_bytes(sigs[0], False)])
    print("pairing gpu", time.time() - t, flush=True)
    print("pairing parity", gts[0] == gt_bytes(O.pairing(pks[0], sigs[0])), flush=True)
    # verify: 2 requests, second has a wrong message
    import numpy as np
    from lodestar_amd.native import pack_blobs
    pkb = np.frombuffer(b"".join(O.g1_to_bytes(p, False) for p in pks), np.uint8)
    msgs2 = list(msgs)
    msgs2[3] = bytes(32)
    mb = np.frombuffer(b"".join(msgs2), np.uint8)
    blob, offs = pack_blobs(comp)
    res = dev.verify_requests(np.array([0, 2, 4], np.uint32), pkb, None, mb, blob, offs, seed)
    print("verify", res.valid, res.errors, res.set_status, res.device_ms, flush=True)
    print(dev.last_stage_times())


if __name__ == "__main__":
    main()
