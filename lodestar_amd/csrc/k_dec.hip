// Signature.fromBytes(sig) decoding of the same-message path as a kernel of its own (the first phase
// of k_sm_prepare for large segments), in its own translation unit so that its out-of-line Fp products
// are compiled for ITS register budget.
//
// Decompression is two Fp exponentiations (the norm root and the delta power of fp2_sqrt), a chain
// of ~900 dependent products whose live state is a handful of field elements.  Inside k_sm_prepare it
// ran at that kernel's occupancy -- two waves per SIMD, set by the 63 Jacobian G2 doublings of the
// subgroup check that follow -- where the dependent v_mad_u64_u32 chains of one product leave issue
// slots empty.  Here the same chain runs at GBV_DEC_WAVES waves per SIMD, and k_sm_prepare<.., true>
// starts from the decoded point (192 B per set written and read back: ~0.05 ms of HBM per 1M sets).
#ifndef GBV_DEC_WAVES
#define GBV_DEC_WAVES 3
#endif
#include "launch.h"
#include "kernel_common.h"

namespace gbv {

// status[i] <- the GBV_PT_* code of g2_decode; S[i] <- the point (any value when the code is not
// PT_OK: k_sm_prepare reads it only for PT_OK).
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(GBV_DEC_WAVES)))
k_sig_decode(uint32_t base, uint32_t n, const uint8_t* __restrict__ sig96, G2A* __restrict__ S, uint8_t* __restrict__ status) {
  const uint32_t t = blockIdx.x * 64 + threadIdx.x;
  if (t >= n) return;
  const uint32_t i = base + t;
  G2A s;
  const uint8_t ds = g2_decode(s, sig96 + 96ull * i, 96);
  if (ds == PT_OK) S[i] = s;
  status[i] = ds;
}

// The same for verifySignatureSets passes on lane quads (k_vs_sig_pre_quad): compressed or uncompressed
// encodings (sig_len 96 / 192; 0 = a length the reference rejects), one thread per signature, so that
// the quad roles do not each run the ~900-product decompression chain on all four lanes.
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(GBV_DEC_WAVES)))
k_vs_sig_decode(uint32_t n, const uint8_t* __restrict__ sig, uint32_t sig_stride, const uint32_t* __restrict__ sig_len,
                G2A* __restrict__ S, uint8_t* __restrict__ dec_st) {
  const uint32_t i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  G2A s;
  const uint8_t ds = g2_decode(s, sig + (size_t)sig_stride * i, sig_len[i]);
  if (ds == PT_OK) S[i] = s;
  dec_st[i] = ds;
}

void launch_vs_sig_decode(hipStream_t s, uint32_t n, const uint8_t* sig, uint32_t sig_stride, const uint32_t* sig_len, G2A* S,
                          uint8_t* dec_st) {
  if (!n) return;
  GBV_LAUNCH("k_vs_sig_decode", k_vs_sig_decode, dim3((n + 63) / 64), dim3(64), s, n, n, sig, sig_stride, sig_len, S, dec_st);
}

void launch_sig_decode(hipStream_t s, uint32_t base, uint32_t n, const uint8_t* sig96, G2A* S, uint8_t* status) {
  if (!n) return;
  GBV_LAUNCH("k_sig_decode", k_sig_decode, dim3((n + 63) / 64), dim3(64), s, n, base, n, sig96, S, status);
}

}  // namespace gbv
