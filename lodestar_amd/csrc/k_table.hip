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

// ---- comb tables (curve.h comb_mul): built once per validator slot ----------------------------
// Pass 1, one thread per slot: the 8 bases and D = 2P (24 doublings, one shared inversion), into a
// chunk-sized scratch of 9 affine points per slot.
__global__ void GBV_KERNEL_ATTR k_comb_bases(uint32_t first, uint32_t n, const G1A* __restrict__ table, const uint8_t* __restrict__ table_ok,
                                             G1A* __restrict__ bases9) {
  uint32_t t = blockIdx.x * 64 + threadIdx.x;
  if (t >= n || !table_ok[first + t]) return;
  G1A B[8], D;
  comb_bases(table[first + t], B, D);
  for (int k = 0; k < 8; ++k) bases9[9ull * t + k] = B[k];
  bases9[9ull * t + 8] = D;
}

__device__ inline Fp comb_shfl(const Fp& a, int src) {
  Fp r;
#pragma unroll
  for (int i = 0; i < 12; ++i) r.v[i] = __shfl((unsigned)a.v[i], src, 64);
  return r;
}

// Pass 2, one wave per slot: lane l builds entries 2l (sign -B_0) and 2l + 1 = 2l + D, and the wave
// normalises its 128 Jacobian entries with ONE inversion (prefix / suffix products across lanes).
// comb_ok[slot] = 0 marks a slot without a usable table (invalid key, or a degenerate entry, which
// a subgroup point never produces): k_sm_prepare then uses the ladder for it.
__global__ void __launch_bounds__(64) k_comb_entries(uint32_t first, const G1A* __restrict__ bases9, const uint8_t* __restrict__ table_ok,
                                                     uint4* __restrict__ comb, uint8_t* __restrict__ comb_ok) {
  const uint32_t t = blockIdx.x, v = first + t;
  const int lane = (int)threadIdx.x;
  if (!table_ok[v]) {
    if (lane == 0) comb_ok[v] = 0;
    return;
  }
  G1A B[8];
  for (int k = 0; k < 8; ++k) B[k] = bases9[9ull * t + k];
  const G1A D = bases9[9ull * t + 8];
  const uint32_t e0 = 2u * (uint32_t)lane;
  G1J J0 = comb_entry_jac(B, e0);
  G1J J1 = jac_add_aff(J0, D);
  const Fp zz = fp_mul(J0.z, J1.z);
  // inclusive prefix (lanes 0..l) and suffix (lanes l..63) products of zz
  Fp pre = zz, suf = zz;
  for (int d = 1; d < 64; d <<= 1) {
    Fp po = comb_shfl(pre, lane - d >= 0 ? lane - d : lane);
    Fp so = comb_shfl(suf, lane + d < 64 ? lane + d : lane);
    if (lane - d >= 0) pre = fp_mul(pre, po);
    if (lane + d < 64) suf = fp_mul(suf, so);
  }
  const Fp total = comb_shfl(pre, 63);
  const bool ok = !fp_is_zero(total);
  const Fp inv = fp_inv(total);
  Fp ex_pre = comb_shfl(pre, lane > 0 ? lane - 1 : 0), ex_suf = comb_shfl(suf, lane < 63 ? lane + 1 : 63);
  if (lane == 0) ex_pre = FP_ONE;
  if (lane == 63) ex_suf = FP_ONE;
  const Fp izz = fp_mul(inv, fp_mul(ex_pre, ex_suf));
  uint4* out = comb + (size_t)v * (COMB_ENTRIES * COMB_U4);
  comb_entry_store(out + COMB_U4 * e0, aff_from_jac_inv(J0, fp_mul(izz, J1.z)));
  comb_entry_store(out + COMB_U4 * (e0 + 1), aff_from_jac_inv(J1, fp_mul(izz, J0.z)));
  if (lane == 0) comb_ok[v] = ok ? 1 : 0;
}

// [r] table[slot] for the batch scalar r = a - b x^2 of a digit word, through the slot's comb table
// (use_comb) or the ladder (randomize_g1): the self-check of the tables (gbv_util_g1_mul_rand).
__global__ void GBV_KERNEL_ATTR k_util_g1_mul_rand(uint32_t n, const uint32_t* __restrict__ slots, const uint64_t* __restrict__ r64,
                                                   const G1A* __restrict__ table, const uint4* __restrict__ comb, int use_comb,
                                                   uint8_t* __restrict__ out48) {
  uint32_t i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  uint32_t k = slots[i];
  uint64_t r = r64[i];
  G1J rp;
  const uint4* tab = comb + (size_t)k * (COMB_ENTRIES * COMB_U4);
  if (use_comb == 2)  // raw table entry r of the slot
    rp = jac_from_aff(comb_entry_load(tab + COMB_U4 * (r & 127u)));
  else if (use_comb)
    rp = comb_mul(comb + (size_t)k * (COMB_ENTRIES * COMB_U4), (uint32_t)r, (uint32_t)(r >> 32));
  else if (!randomize_g1(table[k], r, &rp))
    rp = jac_infinity<Fp>();
  G1A a;
  bool fin = jac_to_aff(a, rp);
  g1_compress(out48 + 48ull * i, a, !fin);
}

// slot dst_first + i <- slot src_first + i % src_n (k_pk_replicate's companion), one thread per word
__global__ void k_comb_replicate(uint4* __restrict__ comb, uint8_t* __restrict__ comb_ok, uint32_t src_first, uint32_t src_n,
                                 uint32_t dst_first, uint32_t n) {
  const size_t W = COMB_ENTRIES * COMB_U4;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)n * W) return;
  size_t slot = i / W, w = i % W;
  size_t s = src_first + slot % src_n;
  comb[(dst_first + slot) * W + w] = comb[s * W + w];
  if (w == 0) comb_ok[dst_first + slot] = comb_ok[s];
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
void launch_comb_build(hipStream_t s, uint32_t first, uint32_t n, const G1A* table, const uint8_t* table_ok, G1A* bases9, uint4* comb,
                       uint8_t* comb_ok) {
  hipLaunchKernelGGL(k_comb_bases, dim3((n + 63) / 64), dim3(64), 0, s, first, n, table, table_ok, bases9);
  debug_sync(s, "k_comb_bases");
  hipLaunchKernelGGL(k_comb_entries, dim3(n), dim3(64), 0, s, first, bases9, table_ok, comb, comb_ok);
  debug_sync(s, "k_comb_entries");
}
void launch_util_g1_mul_rand(hipStream_t s, uint32_t n, const uint32_t* slots, const uint64_t* r64, const G1A* table, const uint4* comb,
                             int use_comb, uint8_t* out48) {
  hipLaunchKernelGGL(k_util_g1_mul_rand, dim3((n + 63) / 64), dim3(64), 0, s, n, slots, r64, table, comb, use_comb, out48);
  debug_sync(s, "k_util_g1_mul_rand");
}
void launch_comb_replicate(hipStream_t s, uint4* comb, uint8_t* comb_ok, uint32_t src_first, uint32_t src_n, uint32_t dst_first, uint32_t n) {
  size_t words = (size_t)n * COMB_ENTRIES * COMB_U4;
  hipLaunchKernelGGL(k_comb_replicate, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, s, comb, comb_ok, src_first, src_n, dst_first, n);
  debug_sync(s, "k_comb_replicate");
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
