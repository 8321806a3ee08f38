// Field element types shared by every kernel.  One thread holds one element in VGPRs:
// Fp = 12 x 32-bit little-endian limbs (381-bit prime, Montgomery form, R = 2^384).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Device-only in the product build.  tests/native/hosttest.cpp defines GBV_HOST_TEST to also
// compile the same arithmetic for the CPU, where it is unit-tested against the oracle.
#if defined(GBV_HOST_TEST)
#define GBV_HD __host__ __device__ __forceinline__
#define GBV_NI __host__ __device__ __noinline__ inline
#elif defined(GBV_ALL_INLINE)
#define GBV_HD __device__ __forceinline__
#define GBV_NI __device__ __forceinline__
#else
#define GBV_HD __device__ __forceinline__
#define GBV_NI __device__ __noinline__ inline
#endif

namespace gbv {
// 12 limbs as an ext_vector so that an Fp passes to/from out-of-line functions in 12 VGPRs
// (the AMDGPU calling convention sends plain aggregates through scratch memory).
typedef uint32_t u32x12 __attribute__((ext_vector_type(12)));
struct Fp { u32x12 v; };
struct Fp2 { Fp c0, c1; };
struct Fp6 { Fp2 c0, c1, c2; };
struct Fp12 { Fp6 c0, c1; };
}  // namespace gbv
