// Signing roots on the GPU (the step before the verifier):
// computeSigningRoot(type, obj, domain) = hash_tree_root(SigningData{objectRoot, domain})
// (packages/state-transition/src/util/signingRoot.ts:7-13), with the SSZ
// merkleization of @chainsafe/ssz restated: 32-byte chunks, basic uint64
// fields packed little-endian into one chunk, containers merkleized over
// their field roots zero-padded to the next power of two.
//
// One lane per object; SHA-256 of two chunks = two compressions (the second
// is the constant padding block).  Integer VALU work only, ~20 compressions
// per attestation: hash-bound, not memory-bound (160 B in, 32 B out).
#include "bls_kernels.h"

namespace lb {

struct chunk {
  uint32_t w[8];  // 32 bytes as big-endian SHA-256 words
};

LB_DEV void chunk_load(chunk& c, const uint8_t* p, int nbytes) {
  for (int i = 0; i < 8; i++) c.w[i] = 0;
  for (int i = 0; i < nbytes; i++) c.w[i >> 2] |= (uint32_t)p[i] << (24 - 8 * (i & 3));
}

LB_DEV void chunk_store(uint8_t* p, const chunk& c) {
  for (int i = 0; i < 32; i++) p[i] = (uint8_t)(c.w[i >> 2] >> (24 - 8 * (i & 3)));
}

// sha256(a || b)
LB_DEV void hash2(chunk& out, const chunk& a, const chunk& b) {
  uint32_t st[8], w[16];
  sha256_init(st);
  for (int i = 0; i < 8; i++) {
    w[i] = a.w[i];
    w[8 + i] = b.w[i];
  }
  sha256_compress(st, w);
  for (int i = 0; i < 16; i++) w[i] = 0;
  w[0] = 0x80000000u;
  w[15] = 512u;  // message length in bits
  sha256_compress(st, w);
  for (int i = 0; i < 8; i++) out.w[i] = st[i];
}

// merkleize(chunks[0..m)), m <= 16: zero chunks pad to the next power of two
// (a single chunk is its own root)
LB_DEV void merkleize(chunk& root, chunk* c, int m) {
  int width = 1;
  while (width < m) width <<= 1;
  for (int i = m; i < width; i++)
    for (int k = 0; k < 8; k++) c[i].w[k] = 0;
  for (; width > 1; width >>= 1)
    for (int i = 0; i < width / 2; i++) hash2(c[i], c[2 * i], c[2 * i + 1]);
  root = c[0];
}

// phase0.AttestationData (SSZ, 128 bytes): slot u64 | index u64 |
// beacon_block_root | source {epoch u64, root} | target {epoch u64, root};
// getAttestationDataSigningRoot (state-transition/src/signatureSets/indexedAttestation.ts:10-19).
__global__ void __launch_bounds__(TPB) k_signing_root_att(uint32_t n, const uint8_t* __restrict__ data,
                                                          const uint8_t* __restrict__ domains, uint32_t dstride,
                                                          uint8_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* d = data + (size_t)i * 128;
  chunk c[8], e, r;
  chunk_load(c[0], d, 8);        // slot
  chunk_load(c[1], d + 8, 8);    // index
  chunk_load(c[2], d + 16, 32);  // beacon_block_root
  chunk_load(e, d + 48, 8);      // source Checkpoint
  chunk_load(r, d + 56, 32);
  hash2(c[3], e, r);
  chunk_load(e, d + 88, 8);      // target Checkpoint
  chunk_load(r, d + 96, 32);
  hash2(c[4], e, r);
  chunk root, dom;
  merkleize(root, c, 5);
  chunk_load(dom, domains + (size_t)i * dstride, 32);
  hash2(root, root, dom);  // SigningData{objectRoot, domain}
  chunk_store(out + (size_t)i * 32, root);
}

// Any container whose m <= 16 field roots the caller supplies (block headers,
// RANDAO epochs, exits, deposit messages ...): merkleize + SigningData.
__global__ void __launch_bounds__(TPB) k_signing_root_chunks(uint32_t n, uint32_t m, const uint8_t* __restrict__ chunks,
                                                             const uint8_t* __restrict__ domains, uint32_t dstride,
                                                             uint8_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  chunk c[16], root, dom;
  for (uint32_t j = 0; j < m; j++) chunk_load(c[j], chunks + ((size_t)i * m + j) * 32, 32);
  merkleize(root, c, (int)m);
  chunk_load(dom, domains + (size_t)i * dstride, 32);
  hash2(root, root, dom);
  chunk_store(out + (size_t)i * 32, root);
}

}  // namespace lb
