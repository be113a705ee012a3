// K1 synth_fill — device-side synthetic input generation (perf_analyzer
// `--input-data random|zero` equivalent).
//
// Memory-bound fill: every thread emits one 16-byte chunk per grid-stride
// step with a single 128-bit store (global_store_dwordx4), so a wave writes
// 1 KiB per instruction.  Randomness is Philox4x32-10 keyed by (seed,
// stream_id) with the chunk index as counter: output is a pure function of
// (seed, stream_id, offset) — identical on every GPU and independent of the
// launch geometry, which the multi-GPU fan-out tests rely on.

#include "kernels/common.h"

using namespace tcamd;

namespace {

enum Mode : int { kZero = 0, kConst = 1, kUniform = 2, kNormal = 3 };

struct FillParams {
  double lo, hi;
  uint32_t k0, k1, stream_lo, stream_hi;
  int mode;
};

template <typename T>
__device__ __forceinline__ T from_unit(float u, double lo, double hi) {
  return (T)(lo + (double)u * (hi - lo));
}

template <typename T>
__device__ __forceinline__ T from_bits(uint32_t x, double lo, double hi) {
  // integer range [lo, hi] inclusive
  uint64_t span = (uint64_t)(hi - lo) + 1;
  return (T)((int64_t)lo + (int64_t)(x % (span ? span : 1)));
}

__device__ __forceinline__ void gen_values(float* out4, uint64_t chunk, uint32_t sub,
                                           const FillParams& p) {
  u32x4 c{(uint32_t)chunk, (uint32_t)(chunk >> 32), sub ^ p.stream_lo, p.stream_hi};
  u32x4 r = philox4x32_10(c, p.k0, p.k1);
  if (p.mode == kNormal) {
    float u1 = fmaxf(u32_to_unit(r.x), 1e-7f), u2 = u32_to_unit(r.y);
    float u3 = fmaxf(u32_to_unit(r.z), 1e-7f), u4 = u32_to_unit(r.w);
    float m1 = sqrtf(-2.0f * logf(u1)), m2 = sqrtf(-2.0f * logf(u3));
    float s1, c1, s2, c2;
    sincosf(6.283185307f * u2, &s1, &c1);
    sincosf(6.283185307f * u4, &s2, &c2);
    out4[0] = (float)p.lo + (float)p.hi * m1 * c1;
    out4[1] = (float)p.lo + (float)p.hi * m1 * s1;
    out4[2] = (float)p.lo + (float)p.hi * m2 * c2;
    out4[3] = (float)p.lo + (float)p.hi * m2 * s2;
  } else {
    out4[0] = __uint_as_float(r.x);  // raw bits, interpreted by the caller
    out4[1] = __uint_as_float(r.y);
    out4[2] = __uint_as_float(r.z);
    out4[3] = __uint_as_float(r.w);
  }
}

template <typename T, bool kIsFloat>
__device__ __forceinline__ T make_elem(float raw, const FillParams& p) {
  if (p.mode == kZero) return (T)0;
  if (p.mode == kConst) return (T)p.lo;
  if (p.mode == kNormal) return (T)raw;
  uint32_t bits = __float_as_uint(raw);
  if constexpr (kIsFloat) return from_unit<T>(u32_to_unit(bits), p.lo, p.hi);
  return from_bits<T>(bits, p.lo, p.hi);
}

// Produce element `e` (0-based inside a 16-byte chunk) of dtype DT as raw bits.
template <int DT>
__device__ __forceinline__ void fill_chunk(uint8_t* dst_chunk, uint64_t chunk, const FillParams& p) {
  constexpr int ES = (DT == kBool || DT == kInt8 || DT == kUInt8 || DT == kFP8E4M3 || DT == kFP8E5M2)
                         ? 1
                         : (DT == kInt16 || DT == kUInt16 || DT == kFP16 || DT == kBF16) ? 2
                         : (DT == kInt64 || DT == kUInt64 || DT == kFP64) ? 8 : 4;
  constexpr int N = 16 / ES;
  union {
    uint4 v;
    uint8_t b[16];
    uint16_t h[8];
    uint32_t w[4];
    uint64_t d[2];
  } out;
  float vals[16];
#pragma unroll
  for (int s = 0; s < (N + 3) / 4; ++s) gen_values(vals + 4 * s, chunk, (uint32_t)s, p);
#pragma unroll
  for (int e = 0; e < N; ++e) {
    float r = vals[e];
    if constexpr (DT == kFP32) {
      out.w[e] = __float_as_uint(make_elem<float, true>(r, p));
    } else if constexpr (DT == kFP64) {
      double v = make_elem<double, true>(r, p);
      out.d[e] = (uint64_t)__double_as_longlong(v);
    } else if constexpr (DT == kFP16) {
      _Float16 v = (_Float16)make_elem<float, true>(r, p);
      out.h[e] = *reinterpret_cast<uint16_t*>(&v);
    } else if constexpr (DT == kBF16) {
      out.h[e] = f32_to_bf16_rne(make_elem<float, true>(r, p));
    } else if constexpr (DT == kFP8E4M3) {
      float v = sat_e4m3(make_elem<float, true>(r, p));
      out.b[e] = (uint8_t)__builtin_amdgcn_cvt_pk_fp8_f32(v, v, 0, false);
    } else if constexpr (DT == kFP8E5M2) {
      float v = sat_e5m2(make_elem<float, true>(r, p));
      out.b[e] = (uint8_t)__builtin_amdgcn_cvt_pk_bf8_f32(v, v, 0, false);
    } else if constexpr (DT == kBool) {
      out.b[e] = (p.mode == kUniform || p.mode == kNormal) ? (uint8_t)(__float_as_uint(r) & 1u)
                                                            : (uint8_t)(p.mode == kConst && p.lo != 0.0);
    } else if constexpr (DT == kInt8) {
      out.b[e] = (uint8_t)make_elem<int8_t, false>(r, p);
    } else if constexpr (DT == kUInt8) {
      out.b[e] = make_elem<uint8_t, false>(r, p);
    } else if constexpr (DT == kInt16) {
      out.h[e] = (uint16_t)make_elem<int16_t, false>(r, p);
    } else if constexpr (DT == kUInt16) {
      out.h[e] = make_elem<uint16_t, false>(r, p);
    } else if constexpr (DT == kInt32) {
      out.w[e] = (uint32_t)make_elem<int32_t, false>(r, p);
    } else if constexpr (DT == kUInt32) {
      out.w[e] = make_elem<uint32_t, false>(r, p);
    } else if constexpr (DT == kInt64) {
      out.d[e] = (uint64_t)make_elem<int64_t, false>(r, p);
    } else if constexpr (DT == kUInt64) {
      out.d[e] = make_elem<uint64_t, false>(r, p);
    }
  }
  *reinterpret_cast<uint4*>(dst_chunk) = out.v;
}

template <int DT>
__global__ void __launch_bounds__(kBlock) synth_fill_kernel(uint8_t* __restrict__ dst,
                                                            uint64_t n_chunks, FillParams p) {
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < n_chunks; c += stride) {
    fill_chunk<DT>(dst + c * 16, c, p);
  }
}

// Tail (< 16 bytes, or unaligned base): one thread builds the last chunk in
// registers and stores only the valid bytes.
template <int DT>
__global__ void synth_tail_kernel(uint8_t* __restrict__ dst, uint64_t chunk, int nbytes, FillParams p) {
  if (threadIdx.x != 0) return;
  __attribute__((aligned(16))) uint8_t tmp[16];
  fill_chunk<DT>(tmp, chunk, p);
  for (int i = 0; i < nbytes; ++i) dst[i] = tmp[i];
}

template <int DT>
int launch(void* dst, size_t nbytes, const FillParams& p, hipStream_t s) {
  uint64_t n_chunks = nbytes / 16;
  int tail = (int)(nbytes % 16);
  if (n_chunks) {
    hipLaunchKernelGGL(synth_fill_kernel<DT>, dim3(grid_for(n_chunks)), dim3(kBlock), 0, s,
                       (uint8_t*)dst, n_chunks, p);
  }
  if (tail) {
    hipLaunchKernelGGL(synth_tail_kernel<DT>, dim3(1), dim3(64), 0, s,
                       (uint8_t*)dst + n_chunks * 16, n_chunks, tail, p);
  }
  return hipGetLastError();
}

}  // namespace

extern "C" int tcamd_synth_fill(void* dst, size_t n_elems, int dtype, int mode, double lo, double hi,
                                uint64_t seed, uint64_t stream_id, void* stream) {
  if (((uintptr_t)dst & 15) != 0) return hipErrorInvalidValue;  // regions are hipMalloc-aligned
  int es = dtype_size(dtype);
  if (es == 0) return hipErrorInvalidValue;
  FillParams p;
  p.lo = lo;
  p.hi = hi;
  p.k0 = (uint32_t)seed;
  p.k1 = (uint32_t)(seed >> 32);
  p.stream_lo = (uint32_t)stream_id;
  p.stream_hi = (uint32_t)(stream_id >> 32);
  p.mode = mode;
  size_t nbytes = n_elems * (size_t)es;
  hipStream_t s = (hipStream_t)stream;
  switch (dtype) {
    case kBool: return launch<kBool>(dst, nbytes, p, s);
    case kInt8: return launch<kInt8>(dst, nbytes, p, s);
    case kInt16: return launch<kInt16>(dst, nbytes, p, s);
    case kInt32: return launch<kInt32>(dst, nbytes, p, s);
    case kInt64: return launch<kInt64>(dst, nbytes, p, s);
    case kUInt8: return launch<kUInt8>(dst, nbytes, p, s);
    case kUInt16: return launch<kUInt16>(dst, nbytes, p, s);
    case kUInt32: return launch<kUInt32>(dst, nbytes, p, s);
    case kUInt64: return launch<kUInt64>(dst, nbytes, p, s);
    case kFP16: return launch<kFP16>(dst, nbytes, p, s);
    case kFP32: return launch<kFP32>(dst, nbytes, p, s);
    case kFP64: return launch<kFP64>(dst, nbytes, p, s);
    case kBF16: return launch<kBF16>(dst, nbytes, p, s);
    case kFP8E4M3: return launch<kFP8E4M3>(dst, nbytes, p, s);
    case kFP8E5M2: return launch<kFP8E5M2>(dst, nbytes, p, s);
    default: return hipErrorInvalidValue;
  }
}
