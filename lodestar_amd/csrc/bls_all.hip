// Single-translation-unit build of the whole library (op-counting variant,
// tools/opcount.py): one device global counter shared by every kernel.
#include "k_sets.hip"
#include "k_hash.hip"
#include "k_scalar.hip"
#include "k_miller.hip"
#include "k_prod.hip"
#include "k_final.hip"
#include "k_pairing.hip"
#include "k_aux.hip"
#include "k_tail.hip"
#include "k_ssz.hip"
#include "k_msm.hip"
#include "bls_host.hip"
