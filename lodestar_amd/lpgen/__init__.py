"""Round programs of the latency path (build-time generator).

A latency-path kernel (lodestar_amd/csrc/k_lp.hip) runs one straight-line
program per verified set on one workgroup: a sequence of *rounds*, each a set
of independent *units* executed one per 16-lane row (bls_coop.h: one Fp
element per row) between two workgroup barriers.  A unit forms linear
combinations of LDS-resident Fp registers and multiplies them (or selects,
inverts, tests a predicate), so a round is one Fp product deep no matter how
many of the tower's products it holds.  The verification's latency is then
the depth of its product DAG (~2k rounds) instead of the ~12k serial products
of a one-lane chain.

``dsl``      graph of Fp / flag nodes with lazy linear forms
``tower``    Fp2 / Fp6 / Fp12 and the curve arithmetic on top of it
``bls``      the per-set, product and final-exponentiation programs
``compile``  list scheduling, register allocation, encoding, and a big-integer
             executor of the encoded program (the CPU check of every program)
"""
