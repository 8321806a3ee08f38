// Distinct-message path kernels (verifySignatureSets).
#include "launch.h"
#include "kernel_common.h"

namespace gbv {

// ---- distinct-message path (verifySignatureSets) ------------------------------------------------
__global__ void GBV_KERNEL_ATTR k_vs_prepare(uint32_t n, const uint32_t* __restrict__ set_idx_off, const uint32_t* __restrict__ idx,
                                                   const uint8_t* __restrict__ raw_flag, const uint8_t* __restrict__ raw_pk48,
                                                   const uint8_t* __restrict__ msgs32, const uint8_t* __restrict__ sig, uint32_t sig_stride,
                                                   const uint32_t* __restrict__ sig_len, const G1A* __restrict__ table,
                                                   const uint8_t* __restrict__ table_ok, Seed seed, uint32_t nonce,
                                                   Fp12* __restrict__ f_out, G2J* __restrict__ rS_out, uint8_t* __restrict__ status) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t st = SET_OK;
  // public key: raw (validated like PublicKey.fromBytes(pk, true)) or aggregate of table entries
  G1A pk;
  bool pk_inf = false;
  if (raw_flag[i]) {
    uint8_t ds = g1_decompress(pk, raw_pk48 + 48ull * i);
    if (ds != PT_OK || !g1_in_subgroup(pk)) st = SET_BAD_PK;
  } else {
    uint32_t b = set_idx_off[i], e = set_idx_off[i + 1];
    G1J acc = jac_infinity<Fp>();
    for (uint32_t j = b; j < e; ++j) {
      uint32_t k = idx[j];
      if (!table_ok[k]) st = SET_BAD_PK;
      acc = jac_add_aff(acc, table[k]);
    }
    pk_inf = !jac_to_aff(pk, acc);
  }
  if (pk_inf) st = SET_BAD_PK;  // verify with an infinity pubkey fails in blst
  G2A s;
  uint8_t ds = g2_decode(s, sig + (size_t)sig_stride * i, sig_len[i]);
  if (ds != PT_OK || !g2_in_subgroup(s)) st = SET_BAD_SIG;
  status[i] = st;
  if (st != SET_OK) return;
  uint64_t r = prf_scalar(seed, i, nonce);
  G1J rp;
  G2J rs;
  if (!randomize_pair(pk, s, r, &rp, &rs)) {  // unreachable for subgroup points; plain 64-bit r then
    rs = g2_mul_u64(s, r);
    rp = g1_mul_u64(pk, r);
  }
  rS_out[i] = rs;
  uint32_t w[8];
  load_msg_words(w, msgs32 + 32ull * i);
  G2A h = hash_to_g2(w);
  f_out[i] = miller_loop_1j(rp, h);
}

void launch_vs_prepare(LaunchCfg c, uint32_t n, const uint32_t* set_idx_off, const uint32_t* idx, const uint8_t* raw_flag,
                       const uint8_t* raw_pk48, const uint8_t* msgs32, const uint8_t* sig, uint32_t sig_stride, const uint32_t* sig_len,
                       const G1A* table, const uint8_t* table_ok, const Seed& seed, uint32_t nonce, Fp12* f_out, G2J* rS_out,
                       uint8_t* status) {
  hipLaunchKernelGGL(k_vs_prepare, dim3(c.blocks), dim3(c.threads), 0, c.stream, n, set_idx_off, idx, raw_flag, raw_pk48, msgs32, sig,
                     sig_stride, sig_len, table, table_ok, seed, nonce, f_out, rS_out, status);
  debug_sync(c.stream, "k_vs_prepare");
}
}  // namespace gbv
