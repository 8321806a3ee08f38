// index2pubkey table, aggregation and utility kernels.
#include "launch.h"
#include "kernel_common.h"

namespace gbv {

// ---- pubkey table -------------------------------------------------------------------------------
__global__ void GBV_KERNEL_ATTR k_pk_decompress(uint32_t n, const uint8_t* __restrict__ pk48, int validate,
                                                      G1A* __restrict__ table, uint8_t* __restrict__ table_ok,
                                                      uint8_t* __restrict__ status) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  G1A a;
  uint8_t st = g1_decompress(a, pk48 + 48ull * i);
  if (st == PT_OK && validate && !g1_in_subgroup(a)) st = PT_NOT_IN_GROUP;
  if (st != PT_OK) {
    a.x = fp_zero();
    a.y = fp_zero();
  }
  table[i] = a;
  table_ok[i] = st == PT_OK;
  status[i] = st;
}

__global__ void k_pk_replicate(G1A* __restrict__ table, uint8_t* __restrict__ table_ok, uint32_t src_first, uint32_t src_n,
                               uint32_t dst_first, uint32_t n) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t s = src_first + (i % src_n);
  table[dst_first + i] = table[s];
  table_ok[dst_first + i] = table_ok[s];
}

// aggregatePublicKeys over an index list (idx == nullptr: table slots 0..k-1, the serialized-key
// form): one 256-thread block, strided partial sums + LDS tree.
__global__ void __launch_bounds__(256) k_aggregate(const uint32_t* __restrict__ idx, uint32_t k, const G1A* __restrict__ table,
                                                   const uint8_t* __restrict__ table_ok, uint8_t* __restrict__ out48,
                                                   uint32_t* __restrict__ bad) {
  __shared__ G1J part[256];
  uint32_t t = threadIdx.x;
  G1J acc = jac_infinity<Fp>();
  for (uint32_t i = t; i < k; i += 256) {
    uint32_t j = idx ? idx[i] : i;
    if (!table_ok[j]) {
      if (idx) atomicOr(bad, 1u);
      if (!idx) continue;  // serialized key that decoded to infinity: contributes nothing
    }
    acc = jac_add_aff(acc, table[j]);
  }
  part[t] = acc;
  __syncthreads();
  for (uint32_t s = 128; s > 0; s >>= 1) {
    if (t < s) part[t] = jac_add(part[t], part[t + s]);
    __syncthreads();
  }
  if (t == 0) {
    G1A a;
    bool finite = jac_to_aff(a, part[0]);
    g1_compress(out48, a, !finite);
  }
}

// ---- utilities (synthetic workloads, tests) -----------------------------------------------------
__device__ inline void load_scalar_be32(uint32_t k[8], const uint8_t* b) {
  for (int i = 0; i < 8; ++i) {
    const uint8_t* q = b + 28 - 4 * i;
    k[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
}

__global__ void GBV_KERNEL_ATTR k_util_sk_to_pk(uint32_t n, const uint8_t* __restrict__ sk32, uint8_t* __restrict__ pk48) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t k[8];
  load_scalar_be32(k, sk32 + 32ull * i);
  G1A g{G1_GEN_X, G1_GEN_Y};
  G1A a;
  bool fin = jac_to_aff(a, g1_mul_u256(g, k));
  g1_compress(pk48 + 48ull * i, a, !fin);
}

__global__ void GBV_KERNEL_ATTR k_util_sign(uint32_t n, const uint8_t* __restrict__ sk32, const uint32_t* __restrict__ grp,
                                                  const G2A* __restrict__ H, uint8_t* __restrict__ sig96) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t k[8];
  load_scalar_be32(k, sk32 + 32ull * i);
  G2A a;
  bool fin = jac_to_aff(a, g2_mul_u256(H[grp[i]], k));
  g2_compress(sig96 + 96ull * i, a, !fin);
}


void launch_pk_decompress(LaunchCfg c, uint32_t n, const uint8_t* pk48, int validate, G1A* table, uint8_t* table_ok, uint8_t* status) {
  hipLaunchKernelGGL(k_pk_decompress, dim3(c.blocks), dim3(c.threads), 0, c.stream, n, pk48, validate, table, table_ok, status);
  debug_sync(c.stream, "k_pk_decompress");
}
void launch_pk_replicate(LaunchCfg c, G1A* table, uint8_t* table_ok, uint32_t src_first, uint32_t src_n, uint32_t dst_first, uint32_t n) {
  hipLaunchKernelGGL(k_pk_replicate, dim3(c.blocks), dim3(c.threads), 0, c.stream, table, table_ok, src_first, src_n, dst_first, n);
  debug_sync(c.stream, "k_pk_replicate");
}
void launch_aggregate(LaunchCfg c, const uint32_t* idx, uint32_t k, const G1A* table, const uint8_t* table_ok, uint8_t* out48,
                      uint32_t* bad) {
  hipLaunchKernelGGL(k_aggregate, dim3(c.blocks), dim3(c.threads), 0, c.stream, idx, k, table, table_ok, out48, bad);
  debug_sync(c.stream, "k_aggregate");
}
void launch_util_sk_to_pk(LaunchCfg c, uint32_t n, const uint8_t* sk32, uint8_t* pk48) {
  hipLaunchKernelGGL(k_util_sk_to_pk, dim3(c.blocks), dim3(c.threads), 0, c.stream, n, sk32, pk48);
  debug_sync(c.stream, "k_util_sk_to_pk");
}
void launch_util_sign(LaunchCfg c, uint32_t n, const uint8_t* sk32, const uint32_t* grp, const G2A* H, uint8_t* sig96) {
  hipLaunchKernelGGL(k_util_sign, dim3(c.blocks), dim3(c.threads), 0, c.stream, n, sk32, grp, H, sig96);
  debug_sync(c.stream, "k_util_sign");
}
}  // namespace gbv
