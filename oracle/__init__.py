"""CPU oracle (test infrastructure only; see bls12_381.py header)."""
