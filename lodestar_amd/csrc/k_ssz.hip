// Signing-root kernels: batched SHA-256 over SSZ nodes.  One thread per
// node / object; the work is integer VALU (rotates, xor3, bfi, add3), ~2.4k VALU ops per 64-byte
// digest against 96 bytes of HBM traffic, so the launches are compute-bound, not HBM-bound.
//   k_ssz_digest64        persistent-merkle-tree hasher.digest64 over n 64-byte inputs; one tree level
//                         of gbv_merkle_roots per launch (siblings are adjacent in object-major layout)
//   k_ssz_signing_roots   computeSigningRoot from object roots (signingRoot.ts:7-13)
//   k_ssz_att_signing_roots  getAttestationDataSigningRoot (beacon-node/src/chain/validation/
//                         attestation.ts:657-665) from the 128-byte SSZ AttestationData: 9 digests
#include <hip/hip_runtime.h>
#include "ssz.h"

namespace gbv {

__device__ __forceinline__ void ld_le(uint32_t* w, const uint4* p, int n16) {
#pragma unroll
  for (int i = 0; i < n16; ++i) {
    uint4 v = p[i];
    w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
  }
}
__device__ __forceinline__ void st_root(uint4* p, u32x8 r) {
  p[0] = make_uint4(__builtin_bswap32(r[0]), __builtin_bswap32(r[1]), __builtin_bswap32(r[2]), __builtin_bswap32(r[3]));
  p[1] = make_uint4(__builtin_bswap32(r[4]), __builtin_bswap32(r[5]), __builtin_bswap32(r[6]), __builtin_bswap32(r[7]));
}
__device__ __forceinline__ u32x8 domain_of(const uint4* __restrict__ domains, const uint32_t* __restrict__ dom_idx, uint32_t i) {
  uint32_t w[8];
  ld_le(w, domains + 2 * (dom_idx ? dom_idx[i] : 0u), 2);
  return ssz_chunk(w);
}

__global__ void __launch_bounds__(256) k_ssz_digest64(const uint4* __restrict__ in, uint32_t n, uint4* __restrict__ out) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t w[16];
  ld_le(w, in + 4ull * i, 4);
  u32x16 m;
#pragma unroll
  for (int k = 0; k < 16; ++k) m[k] = __builtin_bswap32(w[k]);
  st_root(out + 2ull * i, sha256_digest64_inl(m));
}

__global__ void __launch_bounds__(256) k_ssz_signing_roots(const uint4* __restrict__ roots, uint32_t n, const uint4* __restrict__ domains,
                                                           const uint32_t* __restrict__ dom_idx, uint4* __restrict__ out) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t w[8];
  ld_le(w, roots + 2ull * i, 2);
  st_root(out + 2ull * i, sha256_digest64_inl(sha256_cat(ssz_chunk(w), domain_of(domains, dom_idx, i))));
}

__global__ void __launch_bounds__(256) k_ssz_att_signing_roots(const uint4* __restrict__ data, uint32_t n, const uint4* __restrict__ domains,
                                                               const uint32_t* __restrict__ dom_idx, uint4* __restrict__ out) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t d[32];
  ld_le(d, data + 8ull * i, 8);
  u32x8 root = ssz_attestation_data_root(d);
  st_root(out + 2ull * i, ssz_signing_root(root, domain_of(domains, dom_idx, i)));
}

static unsigned blocks_for(uint32_t n) { return (n + 255) / 256; }

void launch_ssz_digest64(hipStream_t s, const uint8_t* in64, uint32_t n, uint8_t* out32) {
  hipLaunchKernelGGL(k_ssz_digest64, dim3(blocks_for(n)), dim3(256), 0, s, (const uint4*)in64, n, (uint4*)out32);
}
void launch_ssz_signing_roots(hipStream_t s, const uint8_t* roots32, uint32_t n, const uint8_t* domains32, const uint32_t* dom_idx,
                              uint8_t* out32) {
  hipLaunchKernelGGL(k_ssz_signing_roots, dim3(blocks_for(n)), dim3(256), 0, s, (const uint4*)roots32, n, (const uint4*)domains32, dom_idx,
                     (uint4*)out32);
}
void launch_ssz_att_signing_roots(hipStream_t s, const uint8_t* data128, uint32_t n, const uint8_t* domains32, const uint32_t* dom_idx,
                                  uint8_t* out32) {
  hipLaunchKernelGGL(k_ssz_att_signing_roots, dim3(blocks_for(n)), dim3(256), 0, s, (const uint4*)data128, n, (const uint4*)domains32,
                     dom_idx, (uint4*)out32);
}
}  // namespace gbv
