// Host build of tools/microbench/fp_cols.h for tests/test_fp_cols.py: the column
// products as plain C++ (g++), checked against Python big integers.
#define __device__
#define __constant__
#include "../../lodestar_amd/csrc/bls_constants.h"
#define LB_HD static inline
#include "../../tools/microbench/fp_cols.h"

extern "C" {
void cols_mul(uint32_t* r, const uint32_t* a, const uint32_t* b) { lb::cols::mul(r, a, b); }
void cols_sqr(uint32_t* r, const uint32_t* a) { lb::cols::sqr(r, a); }
void cols_mulw(uint32_t* w, const uint32_t* a, const uint32_t* b) { lb::cols::mulw(w, a, b); }
void cols_redc(uint32_t* r, const uint32_t* w) { lb::cols::redc(r, w); }
}
