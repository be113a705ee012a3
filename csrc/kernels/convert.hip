// K4/K5 — dtype conversion kernels for tensor pack/unpack.
//
//   FP32 -> BF16  truncation (byte-compatible with the reference's
//                 struct.pack("<f")[2:4], tritonclient/utils/__init__.py:314)
//                 or round-to-nearest-even
//   BF16 -> FP32  exact widening
//   FP32 <-> FP16 hardware cvt
//   FP32 <-> FP8  OCP e4m3fn / e5m2 via gfx950 v_cvt_pk_{fp8,bf8}_f32 with
//                 saturation of finite inputs (extension datatype)
//
// Each thread converts 8 elements per grid-stride step: two dwordx4 loads of
// fp32 (32 B) and one dwordx4 / dwordx2 store of the narrow type (and the
// reverse for widening), the vector width CDNA4 needs to reach HBM rate.

#include "kernels/common.h"

using namespace tcamd;

namespace {

struct alignas(16) F8 {
  float v[8];
};

template <int SRC>
__device__ __forceinline__ void load8(const uint8_t* __restrict__ src, uint64_t i, float* f) {
  if constexpr (SRC == kFP32) {
    const float4* p = reinterpret_cast<const float4*>(src + i * 32);
    float4 a = p[0], b = p[1];
    f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w;
    f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
  } else if constexpr (SRC == kBF16 || SRC == kFP16) {
    uint4 u = *reinterpret_cast<const uint4*>(src + i * 16);
    uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint16_t lo = (uint16_t)(w[k] & 0xffff), hi = (uint16_t)(w[k] >> 16);
      if constexpr (SRC == kBF16) {
        f[2 * k] = bf16_to_f32(lo);
        f[2 * k + 1] = bf16_to_f32(hi);
      } else {
        f[2 * k] = (float)*reinterpret_cast<const _Float16*>(&lo);
        f[2 * k + 1] = (float)*reinterpret_cast<const _Float16*>(&hi);
      }
    }
  } else {  // FP8 e4m3 / e5m2: 8 bytes
    uint2 u = *reinterpret_cast<const uint2*>(src + i * 8);
    // byte selector must be an immediate (v_cvt_f32_fp8 sdwa BYTE_k)
#define TCAMD_CVT_BYTE(K)                                        \
  if constexpr (SRC == kFP8E4M3) {                               \
    f[K] = __builtin_amdgcn_cvt_f32_fp8((int)u.x, K);            \
    f[4 + K] = __builtin_amdgcn_cvt_f32_fp8((int)u.y, K);        \
  } else {                                                       \
    f[K] = __builtin_amdgcn_cvt_f32_bf8((int)u.x, K);            \
    f[4 + K] = __builtin_amdgcn_cvt_f32_bf8((int)u.y, K);        \
  }
    TCAMD_CVT_BYTE(0)
    TCAMD_CVT_BYTE(1)
    TCAMD_CVT_BYTE(2)
    TCAMD_CVT_BYTE(3)
#undef TCAMD_CVT_BYTE
  }
}

template <int DST, bool RNE>
__device__ __forceinline__ void store8(uint8_t* __restrict__ dst, uint64_t i, const float* f) {
  if constexpr (DST == kFP32) {
    float4* p = reinterpret_cast<float4*>(dst + i * 32);
    p[0] = make_float4(f[0], f[1], f[2], f[3]);
    p[1] = make_float4(f[4], f[5], f[6], f[7]);
  } else if constexpr (DST == kBF16) {
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint16_t lo = RNE ? f32_to_bf16_rne(f[2 * k]) : f32_to_bf16_trunc(f[2 * k]);
      uint16_t hi = RNE ? f32_to_bf16_rne(f[2 * k + 1]) : f32_to_bf16_trunc(f[2 * k + 1]);
      w[k] = (uint32_t)lo | ((uint32_t)hi << 16);
    }
    *reinterpret_cast<uint4*>(dst + i * 16) = make_uint4(w[0], w[1], w[2], w[3]);
  } else if constexpr (DST == kFP16) {
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      _Float16 a = (_Float16)f[2 * k], b = (_Float16)f[2 * k + 1];
      w[k] = (uint32_t)*reinterpret_cast<uint16_t*>(&a) | ((uint32_t)*reinterpret_cast<uint16_t*>(&b) << 16);
    }
    *reinterpret_cast<uint4*>(dst + i * 16) = make_uint4(w[0], w[1], w[2], w[3]);
  } else {
    int lo = 0, hi = 0;
    if constexpr (DST == kFP8E4M3) {
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(sat_e4m3(f[0]), sat_e4m3(f[1]), lo, false);
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(sat_e4m3(f[2]), sat_e4m3(f[3]), lo, true);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(sat_e4m3(f[4]), sat_e4m3(f[5]), hi, false);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(sat_e4m3(f[6]), sat_e4m3(f[7]), hi, true);
    } else {
      lo = __builtin_amdgcn_cvt_pk_bf8_f32(sat_e5m2(f[0]), sat_e5m2(f[1]), lo, false);
      lo = __builtin_amdgcn_cvt_pk_bf8_f32(sat_e5m2(f[2]), sat_e5m2(f[3]), lo, true);
      hi = __builtin_amdgcn_cvt_pk_bf8_f32(sat_e5m2(f[4]), sat_e5m2(f[5]), hi, false);
      hi = __builtin_amdgcn_cvt_pk_bf8_f32(sat_e5m2(f[6]), sat_e5m2(f[7]), hi, true);
    }
    *reinterpret_cast<uint2*>(dst + i * 8) = make_uint2((uint32_t)lo, (uint32_t)hi);
  }
}

template <int SRC, int DST, bool RNE>
__global__ void __launch_bounds__(kBlock) cvt_kernel(const uint8_t* __restrict__ src,
                                                     uint8_t* __restrict__ dst, uint64_t n_groups) {
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n_groups; g += stride) {
    float f[8];
    load8<SRC>(src, g, f);
    store8<DST, RNE>(dst, g, f);
  }
}

// Scalar tail for the last (n % 8) elements.
template <int SRC, int DST, bool RNE>
__global__ void cvt_tail_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                uint64_t first, int count) {
  int t = threadIdx.x;
  if (t >= count) return;
  uint64_t i = first + t;
  float f;
  if constexpr (SRC == kFP32) f = reinterpret_cast<const float*>(src)[i];
  else if constexpr (SRC == kBF16) f = bf16_to_f32(reinterpret_cast<const uint16_t*>(src)[i]);
  else if constexpr (SRC == kFP16) f = (float)reinterpret_cast<const _Float16*>(src)[i];
  else if constexpr (SRC == kFP8E4M3) f = __builtin_amdgcn_cvt_f32_fp8((int)src[i], 0);
  else f = __builtin_amdgcn_cvt_f32_bf8((int)src[i], 0);
  if constexpr (DST == kFP32) reinterpret_cast<float*>(dst)[i] = f;
  else if constexpr (DST == kBF16)
    reinterpret_cast<uint16_t*>(dst)[i] = RNE ? f32_to_bf16_rne(f) : f32_to_bf16_trunc(f);
  else if constexpr (DST == kFP16) reinterpret_cast<_Float16*>(dst)[i] = (_Float16)f;
  else if constexpr (DST == kFP8E4M3)
    dst[i] = (uint8_t)__builtin_amdgcn_cvt_pk_fp8_f32(sat_e4m3(f), sat_e4m3(f), 0, false);
  else dst[i] = (uint8_t)__builtin_amdgcn_cvt_pk_bf8_f32(sat_e5m2(f), sat_e5m2(f), 0, false);
}

template <int SRC, int DST, bool RNE>
int launch(const void* src, void* dst, size_t n, hipStream_t s) {
  uint64_t groups = n / 8;
  int tail = (int)(n % 8);
  if (groups) {
    hipLaunchKernelGGL((cvt_kernel<SRC, DST, RNE>), dim3(grid_for(groups)), dim3(kBlock), 0, s,
                       (const uint8_t*)src, (uint8_t*)dst, groups);
  }
  if (tail) {
    hipLaunchKernelGGL((cvt_tail_kernel<SRC, DST, RNE>), dim3(1), dim3(64), 0, s,
                       (const uint8_t*)src, (uint8_t*)dst, groups * 8, tail);
  }
  return hipGetLastError();
}

}  // namespace

// rounding: 0 = truncate (wire-compatible BF16), 1 = round-to-nearest-even.
extern "C" int tcamd_convert(const void* src, int src_dtype, void* dst, int dst_dtype, size_t n,
                             int rounding, void* stream) {
  if ((((uintptr_t)src) | ((uintptr_t)dst)) & 15) return hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  if (n == 0) return hipSuccess;
  if (src_dtype == kFP32) {
    switch (dst_dtype) {
      case kBF16:
        return rounding ? launch<kFP32, kBF16, true>(src, dst, n, s) : launch<kFP32, kBF16, false>(src, dst, n, s);
      case kFP16: return launch<kFP32, kFP16, true>(src, dst, n, s);
      case kFP8E4M3: return launch<kFP32, kFP8E4M3, true>(src, dst, n, s);
      case kFP8E5M2: return launch<kFP32, kFP8E5M2, true>(src, dst, n, s);
      default: return hipErrorInvalidValue;
    }
  }
  if (dst_dtype == kFP32) {
    switch (src_dtype) {
      case kBF16: return launch<kBF16, kFP32, true>(src, dst, n, s);
      case kFP16: return launch<kFP16, kFP32, true>(src, dst, n, s);
      case kFP8E4M3: return launch<kFP8E4M3, kFP32, true>(src, dst, n, s);
      case kFP8E5M2: return launch<kFP8E5M2, kFP32, true>(src, dst, n, s);
      default: return hipErrorInvalidValue;
    }
  }
  if (src_dtype == kBF16 && dst_dtype == kFP8E4M3) return launch<kBF16, kFP8E4M3, true>(src, dst, n, s);
  return hipErrorInvalidValue;
}
