// Field element types shared by every kernel.  One thread holds one element in VGPRs:
// Fp = 12 x 32-bit little-endian limbs (381-bit prime, Montgomery form, R = 2^384).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define GBV_HD __host__ __device__ __forceinline__
#define GBV_NI __host__ __device__ __noinline__

namespace gbv {
struct Fp { uint32_t v[12]; };
struct Fp2 { Fp c0, c1; };
struct Fp6 { Fp2 c0, c1, c2; };
struct Fp12 { Fp6 c0, c1; };
}  // namespace gbv
