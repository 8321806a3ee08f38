// hash_to_G2 kernels.  The few-message forms are latency-bound (lane pairs, one wave per message).
#include "launch.h"
#include "kernel_common.h"
#include "quad_g2.h"

namespace gbv {

// ---- hashing ----------------------------------------------------------------------------------
__global__ void GBV_KERNEL_ATTR k_hash_msgs(const uint8_t* __restrict__ msgs32, uint32_t n, G2A* __restrict__ H) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t w[8];
  load_msg_words(w, msgs32 + 32ull * i);
  H[i] = hash_to_g2(w);
}

// Two lanes per message (hash_to_g2_lane_pair): ~25 % shorter chain, for passes with few messages.
__global__ void GBV_KERNEL_ATTR k_hash_msgs_pair(const uint8_t* __restrict__ msgs32, uint32_t n, G2A* __restrict__ H) {
  uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) >> 1;
  bool act = i < n;
  uint32_t w[8] = {};
  if (act) load_msg_words(w, msgs32 + 32ull * i);
  G2A h;
  if (hash_to_g2_lane_pair(w, act, &h)) H[i] = h;
}

// Four lanes per message (quad_g2.h): lanes q = 0, 2 map u_0 and lanes 1, 3 map u_1 (the map is two
// Fp exponentiations in a row: nothing to split), then the quad adds Q0 + Q1, clears the cofactor and
// makes the point affine with every product on its own lane -- about half the pair form's chain.
__global__ void GBV_QUAD_ATTR k_hash_msgs_quad(const uint8_t* __restrict__ msgs32, uint32_t n, G2A* __restrict__ H) {
  const uint32_t q = threadIdx.x & 3u;
  const uint32_t i = blockIdx.x * 16 + (threadIdx.x >> 2);
  const bool act = i < n;
  uint32_t w[8];
  load_msg_words(w, msgs32 + 32ull * (act ? i : 0u));  // past n: message 0 again, nothing written
  const G2J m = hash_map_iso(hash_to_field_fp2(w, (int)(q & 1u)));
  G2J p = quad::g2_add(quad::dpp<0x00>(m), quad::dpp<0x55>(m), q);
  p = quad::g2_clear_cofactor(p, q);
  G2A a;
  quad::g2_to_aff(a, p, q);
  if (act) quad::store_split<4>((Fp*)&H[i], (const Fp*)&a, q);
}

// Cofactor clearing of k_hash_msgs_pre's Q0 + Q1 on lane quads (the maps ran on lane pairs, two lanes
// per message instead of four doing each map twice), then the affine form.
__global__ void GBV_QUAD_ATTR k_hash_clear_quad(uint32_t n, const G2J* __restrict__ Qpre, G2A* __restrict__ H) {
  const uint32_t q = threadIdx.x & 3u;
  const uint32_t i = blockIdx.x * 16 + (threadIdx.x >> 2);
  const bool act = i < n;
  const G2J p = quad::g2_clear_cofactor(Qpre[act ? i : 0u], q);  // past n: message 0 again, nothing written
  G2A a;
  quad::g2_to_aff(a, p, q);
  if (act) quad::store_split<4>((Fp*)&H[i], (const Fp*)&a, q);
}

__global__ void GBV_KERNEL_ATTR k_hash_msgs_pre(const uint8_t* __restrict__ msgs32, uint32_t n, G2J* __restrict__ Qpre) {
  uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) >> 1;
  bool act = i < n;
  uint32_t w[8] = {};
  if (act) load_msg_words(w, msgs32 + 32ull * i);
  G2J q;
  if (hash_to_g2_lane_pair_pre(w, act, &q)) Qpre[i] = q;
}

__global__ void GBV_KERNEL_ATTR k_util_g2_out(uint32_t n, const G2A* __restrict__ H, uint8_t* __restrict__ out192) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t* o = out192 + 192ull * i;
  fp_store_be48(o, fp_from_mont(H[i].x.c1));
  fp_store_be48(o + 48, fp_from_mont(H[i].x.c0));
  fp_store_be48(o + 96, fp_from_mont(H[i].y.c1));
  fp_store_be48(o + 144, fp_from_mont(H[i].y.c0));
}


void launch_hash_msgs(LaunchCfg c, const uint8_t* msgs32, uint32_t n, G2A* H, G2J* Qpre) {
  if (Qpre && n <= tuning().hash_coop_max) {  // latency: lane-pair maps, then the cofactor clearing one workgroup per message
    GBV_LAUNCH("k_hash_msgs_pre", k_hash_msgs_pre, dim3((2 * n + 63) / 64), dim3(64), c.stream, n, msgs32, n, Qpre);
    launch_hash_clear_coop(c.stream, n, Qpre, H);
    return;
  }
  if (Qpre && n <= tuning().hash_quad_max) {  // latency: maps on lane pairs, the cofactor clearing on lane quads
    GBV_LAUNCH("k_hash_msgs_pre", k_hash_msgs_pre, dim3((2 * n + 63) / 64), dim3(64), c.stream, n, msgs32, n, Qpre);
    GBV_LAUNCH("k_hash_clear_quad", k_hash_clear_quad, dim3((n + 15) / 16), dim3(64), c.stream, n, n, Qpre, H);
  } else if (n <= tuning().hash_quad_max)  // lane quads, then lane pairs (grids sized here; c.blocks is for one lane per message)
    GBV_LAUNCH("k_hash_msgs_quad", k_hash_msgs_quad, dim3((n + 15) / 16), dim3(64), c.stream, n, msgs32, n, H);
  else if (n <= tuning().hash_pair_max)
    GBV_LAUNCH("k_hash_msgs_pair", k_hash_msgs_pair, dim3((2 * n + 63) / 64), dim3(64), c.stream, n, msgs32, n, H);
  else
    GBV_LAUNCH("k_hash_msgs", k_hash_msgs, dim3(c.blocks), dim3(c.threads), c.stream, n, msgs32, n, H);
}
void launch_util_g2_out(LaunchCfg c, uint32_t n, const G2A* H, uint8_t* out192) {
  hipLaunchKernelGGL(k_util_g2_out, dim3(c.blocks), dim3(c.threads), 0, c.stream, n, H, out192);
  debug_sync(c.stream, "k_util_g2_out");
}
}  // namespace gbv
