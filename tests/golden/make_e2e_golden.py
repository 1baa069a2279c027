"""Fixture of the reference's e2e pool test (BNT/e2e/chain/bls/multithread.test.ts:26-47):
three keys sk_i = Buffer.alloc(32, i + 1), messages Buffer.alloc(32, i + 1), their
signatures, the same-message signatures over Buffer.alloc(32, 100), and the invalid
32-zero-byte signature of its "first is invalid" case (:114).  Generated with the
oracle (the reference's @chainsafe/bls is not in the container); keys are given in
both encodings so the replay can hand them over as PublicKey-shaped objects.

    python tests/golden/make_e2e_golden.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import bls12_381 as O  # noqa: E402


def main():
    same = bytes([100]) * 32
    sets, same_sets = [], []
    for i in range(3):
        sk = int.from_bytes(bytes([i + 1]) * 32, "big")  # SecretKey.fromBytes(Buffer.alloc(32, i + 1))
        assert 0 < sk < O.R
        pk = O.sk_to_pk(sk)
        msg = bytes([i + 1]) * 32
        sets.append({"pk_uncompressed": O.g1_to_bytes(pk, compressed=False).hex(),
                     "pk_compressed": O.g1_to_bytes(pk).hex(), "message": msg.hex(),
                     "signature": O.g2_to_bytes(O.sign(sk, msg)).hex()})
        same_sets.append({"signature": O.g2_to_bytes(O.sign(sk, same)).hex()})
    out = {"_source": "BNT/e2e/chain/bls/multithread.test.ts:26-47,114 restated; tests/golden/make_e2e_golden.py",
           "sets": sets, "same_message": same.hex(), "same_message_sets": same_sets,
           "invalid_signature": bytes(32).hex()}
    with open(os.path.join(HERE, "e2e_multithread.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
