// Host driver for lodestar_amd/csrc/bls_inv.h (the device inversion compiled
// for the CPU): reads hex inputs (one per line, < p) and prints y^-1 mod p in
// hex.  Used by tests/test_fp_inv.py against Python big integers.
#include <cstdio>
#include <cstring>
#include <string>
#include <iostream>

#include "../../lodestar_amd/csrc/bls_inv.h"

int main() {
  std::string line;
  while (std::getline(std::cin, line)) {
    if (line.empty()) continue;
    uint32_t y[12] = {0}, r[12];
    // big-endian hex (96 digits) -> little-endian limbs
    for (int j = 0; j < 12; j++) {
      const std::string w = line.substr(line.size() - 8 * (j + 1), 8);
      y[j] = (uint32_t)std::stoul(w, nullptr, 16);
    }
    lb_inv::inv_raw(r, y);
    for (int j = 11; j >= 0; j--) printf("%08x", r[j]);
    printf("\n");
  }
  return 0;
}
