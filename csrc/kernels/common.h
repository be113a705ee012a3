// Shared device helpers for the triton-mi355x CDNA4 (gfx950) kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tcamd {

// Datatype codes shared with triton_client_amd/ops/dtypes.py.
enum DType : int {
  kBool = 0,
  kInt8 = 1,
  kInt16 = 2,
  kInt32 = 3,
  kInt64 = 4,
  kUInt8 = 5,
  kUInt16 = 6,
  kUInt32 = 7,
  kUInt64 = 8,
  kFP16 = 9,
  kFP32 = 10,
  kFP64 = 11,
  kBF16 = 12,
  kFP8E4M3 = 13,
  kFP8E5M2 = 14,
};

__host__ __device__ inline int dtype_size(int dt) {
  switch (dt) {
    case kBool: case kInt8: case kUInt8: case kFP8E4M3: case kFP8E5M2: return 1;
    case kInt16: case kUInt16: case kFP16: case kBF16: return 2;
    case kInt32: case kUInt32: case kFP32: return 4;
    case kInt64: case kUInt64: case kFP64: return 8;
    default: return 0;
  }
}

constexpr int kBlock = 256;      // 4 waves of 64
constexpr int kMaxGrid = 2048;   // 256 CUs x 8 resident blocks: grid-stride beyond

inline int grid_for(size_t work_items, int per_block = kBlock) {
  size_t g = (work_items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > (size_t)kMaxGrid) g = kMaxGrid;
  return (int)g;
}

// ---- bf16 / fp8 scalar conversions -----------------------------------------
__device__ __forceinline__ uint16_t f32_to_bf16_trunc(float f) {
  return (uint16_t)(__float_as_uint(f) >> 16);
}

__device__ __forceinline__ uint16_t f32_to_bf16_rne(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

__device__ __forceinline__ float bf16_to_f32(uint16_t h) {
  return __uint_as_float(((uint32_t)h) << 16);
}

// OCP fp8 (gfx950 native): saturate finite values to +/-max first so the
// hardware RNE conversion never produces Inf/NaN from a finite input.
__device__ __forceinline__ float sat_e4m3(float x) {
  return (x != x) ? x : fminf(fmaxf(x, -448.0f), 448.0f);
}
__device__ __forceinline__ float sat_e5m2(float x) {
  return (x != x) ? x : fminf(fmaxf(x, -57344.0f), 57344.0f);
}

// ---- Philox4x32-10 counter-based RNG ----------------------------------------
struct u32x4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0 = __umulhi(M0, c.x), lo0 = M0 * c.x;
    uint32_t hi1 = __umulhi(M1, c.z), lo1 = M1 * c.z;
    u32x4 n;
    n.x = hi1 ^ c.y ^ k0;
    n.y = lo1;
    n.z = hi0 ^ c.w ^ k1;
    n.w = lo0;
    c = n;
    k0 += W0;
    k1 += W1;
  }
  return c;
}

__device__ __forceinline__ float u32_to_unit(uint32_t x) {
  return (float)(x >> 8) * (1.0f / 16777216.0f);  // [0,1)
}

}  // namespace tcamd
