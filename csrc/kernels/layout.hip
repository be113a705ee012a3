// K6 layout_pack — fused gather + layout transform + dtype convert + affine
// scale, for image-classification inputs (replaces the
// host preprocessing in reference src/c++/examples/image_client.cc:86-188 and
// src/python/examples/image_client.py:154-194, and the server-side batch
// assembly of shm inputs).
//
//   y[n, ...] = x_n[...] * scale[c] + bias[c],  x_n from its own pointer
//
// Layouts: NCHW <-> NHWC (or the same layout: convert + affine only).  Source dtypes: FP32 / UINT8 / BF16 / FP16; dest:
// FP32 / BF16 / FP16.  Up to 64 images per launch (pointer table passed by
// value, so there is no H2D copy of descriptors per call).
//
// Two code paths:
//  * C <= 4 (RGB images): register path, 4 pixels per thread; every lane
//    does one 16 B load per channel plane (NCHW side) and 8-24 B contiguous
//    stores (NHWC side) — fully coalesced in both directions, no LDS needed;
//  * general C: a batched 2-D transpose through a 64x64 LDS tile with a
//    +1-element row pad (bank-conflict free column reads), 256 threads, each
//    moving 16 elements per phase.

#include "kernels/common.h"

using namespace tcamd;

namespace {

constexpr int kMaxImgs = 64;
constexpr int kMaxChan = 64;

struct LayoutParams {
  const void* src[kMaxImgs];
  float scale[kMaxChan];
  float bias[kMaxChan];
  int n_imgs, C, HW;
  int affine;  // 0: no per-channel scale/bias
  int rne;     // bf16 rounding
};

template <int DT>
__device__ __forceinline__ float ld(const void* base, uint64_t i) {
  if constexpr (DT == kFP32) return reinterpret_cast<const float*>(base)[i];
  else if constexpr (DT == kUInt8) return (float)reinterpret_cast<const uint8_t*>(base)[i];
  else if constexpr (DT == kBF16) return bf16_to_f32(reinterpret_cast<const uint16_t*>(base)[i]);
  else return (float)reinterpret_cast<const _Float16*>(base)[i];
}

template <int DT>
__device__ __forceinline__ void ld4(const void* base, uint64_t i, float* f) {
  // 4 consecutive elements starting at element i (i % 4 == 0, base aligned)
  if constexpr (DT == kFP32) {
    float4 v = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(base) + i);
    f[0] = v.x; f[1] = v.y; f[2] = v.z; f[3] = v.w;
  } else if constexpr (DT == kUInt8) {
    uint32_t v = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(base) + i);
    f[0] = (float)(v & 0xff); f[1] = (float)((v >> 8) & 0xff);
    f[2] = (float)((v >> 16) & 0xff); f[3] = (float)(v >> 24);
  } else {
    uint2 v = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(base) + i);
    uint16_t h[4] = {(uint16_t)(v.x & 0xffff), (uint16_t)(v.x >> 16), (uint16_t)(v.y & 0xffff), (uint16_t)(v.y >> 16)};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if constexpr (DT == kBF16) f[k] = bf16_to_f32(h[k]);
      else f[k] = (float)*reinterpret_cast<const _Float16*>(&h[k]);
    }
  }
}

template <int DT>
__device__ __forceinline__ uint32_t bits16(float f, int rne) {
  if constexpr (DT == kBF16) return rne ? f32_to_bf16_rne(f) : f32_to_bf16_trunc(f);
  else {
    _Float16 h = (_Float16)f;
    return *reinterpret_cast<uint16_t*>(&h);
  }
}

template <int DT>
__device__ __forceinline__ void st(void* base, uint64_t i, float f, int rne) {
  if constexpr (DT == kFP32) reinterpret_cast<float*>(base)[i] = f;
  else reinterpret_cast<uint16_t*>(base)[i] = (uint16_t)bits16<DT>(f, rne);
}

// Store `count` (multiple of 4) consecutive outputs held in f[] at element i.
template <int DT, int COUNT>
__device__ __forceinline__ void st_vec(void* base, uint64_t i, const float* f, int rne) {
  if constexpr (DT == kFP32) {
    float* p = reinterpret_cast<float*>(base) + i;
    if constexpr (COUNT % 4 == 0 && true) {
#pragma unroll
      for (int k = 0; k < COUNT; k += 4)
        *reinterpret_cast<float4*>(p + k) = make_float4(f[k], f[k + 1], f[k + 2], f[k + 3]);
    }
  } else {
    uint16_t* p = reinterpret_cast<uint16_t*>(base) + i;
#pragma unroll
    for (int k = 0; k < COUNT; k += 4) {
      uint32_t a = bits16<DT>(f[k], rne) | (bits16<DT>(f[k + 1], rne) << 16);
      uint32_t b = bits16<DT>(f[k + 2], rne) | (bits16<DT>(f[k + 3], rne) << 16);
      *reinterpret_cast<uint2*>(p + k) = make_uint2(a, b);
    }
  }
}

// ---- C <= 4: NCHW -> NHWC, 4 pixels / thread ----------------------------------
template <int SRC, int DST, int C>
__global__ void __launch_bounds__(kBlock) small_c_to_nhwc(LayoutParams p, void* __restrict__ dst) {
  const uint64_t quads_per_img = (uint64_t)p.HW / 4;
  const uint64_t total = quads_per_img * p.n_imgs;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += stride) {
    const int n = (int)(q / quads_per_img);
    const uint64_t pix = (q - (uint64_t)n * quads_per_img) * 4;
    const void* src = p.src[n];
    float v[C][4];
#pragma unroll
    for (int c = 0; c < C; ++c) ld4<SRC>(src, (uint64_t)c * p.HW + pix, v[c]);
    float o[4 * C];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int c = 0; c < C; ++c)
        o[k * C + c] = p.affine ? v[c][k] * p.scale[c] + p.bias[c] : v[c][k];
    st_vec<DST, 4 * C>(dst, ((uint64_t)n * p.HW + pix) * C, o, p.rne);
  }
}

// ---- C <= 4: NHWC -> NCHW, 4 pixels / thread ----------------------------------
template <int SRC, int DST, int C>
__global__ void __launch_bounds__(kBlock) small_c_to_nchw(LayoutParams p, void* __restrict__ dst) {
  const uint64_t quads_per_img = (uint64_t)p.HW / 4;
  const uint64_t total = quads_per_img * p.n_imgs;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += stride) {
    const int n = (int)(q / quads_per_img);
    const uint64_t pix = (q - (uint64_t)n * quads_per_img) * 4;
    const void* src = p.src[n];
    float v[4 * C];
#pragma unroll
    for (int k = 0; k < 4 * C; k += 4) ld4<SRC>(src, pix * C + k, v + k);
#pragma unroll
    for (int c = 0; c < C; ++c) {
      float o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = p.affine ? v[k * C + c] * p.scale[c] + p.bias[c] : v[k * C + c];
      st_vec<DST, 4>(dst, ((uint64_t)n * C + c) * p.HW + pix, o, p.rne);
    }
  }
}

// ---- general C: LDS-tiled batched transpose -----------------------------------
// Per image the source is a [R][K] matrix and the destination is [K][R]:
//   NCHW->NHWC: R = C,  K = HW,  channel = row
//   NHWC->NCHW: R = HW, K = C,   channel = col
constexpr int kTile = 64;

template <int SRC, int DST, bool CH_IS_ROW>
__global__ void __launch_bounds__(kBlock) tiled_transpose(LayoutParams p, void* __restrict__ dst,
                                                          int R, int K) {
  __shared__ float tile[kTile][kTile + 1];
  const int tiles_k = (K + kTile - 1) / kTile;
  const int n = blockIdx.z;
  const int tr = blockIdx.y;
  for (int tk = blockIdx.x; tk < tiles_k; tk += gridDim.x) {
    const int r0 = tr * kTile, k0 = tk * kTile;
    const void* src = p.src[n];
    // load: 256 threads = 4 rows x 64 cols per pass, 16 passes
    const int lc = threadIdx.x & 63, lr = threadIdx.x >> 6;
#pragma unroll 4
    for (int rr = lr; rr < kTile; rr += 4) {
      int r = r0 + rr, k = k0 + lc;
      float v = 0.f;
      if (r < R && k < K) {
        v = ld<SRC>(src, (uint64_t)r * K + k);
        if (p.affine) {
          int c = CH_IS_ROW ? r : k;
          v = v * p.scale[c] + p.bias[c];
        }
      }
      tile[rr][lc] = v;
    }
    __syncthreads();
    // store transposed: out[k][r]
#pragma unroll 4
    for (int kk = lr; kk < kTile; kk += 4) {
      int k = k0 + kk, r = r0 + lc;
      if (k < K && r < R) st<DST>(dst, ((uint64_t)n * K + k) * R + r, tile[lc][kk], p.rne);
    }
    __syncthreads();
  }
}

// ---- same layout (NCHW -> NCHW, NHWC -> NHWC): convert + per-channel affine ----
// one element per thread-iteration over the gathered batch; the channel of a
// flat index is (i / HW) % C for NCHW and i % C for NHWC
template <int SRC, int DST, bool CHW>
__global__ void __launch_bounds__(kBlock) same_layout(LayoutParams p, void* __restrict__ dst) {
  const uint64_t per_img = (uint64_t)p.C * p.HW;
  const uint64_t total = per_img * p.n_imgs;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const uint64_t n = i / per_img, e = i - n * per_img;
    const int c = CHW ? (int)(e / p.HW) : (int)(e % p.C);
    float f = ld<SRC>(p.src[n], e);
    if (p.affine) f = f * p.scale[c] + p.bias[c];
    st<DST>(dst, i, f, p.rne);
  }
}

template <int SRC, int DST>
int dispatch_dst(const LayoutParams& p, int src_layout, int dst_layout, void* dst, hipStream_t s) {
  const int C = p.C, HW = p.HW;
  // the register path does 4-element vector accesses: every source and the
  // destination must be aligned to 4 elements of their dtype
  bool aligned = (((uintptr_t)dst) % (4 * sizeof(uint32_t) / (DST == kFP32 ? 1 : 2))) == 0;
  for (int i = 0; i < p.n_imgs; ++i)
    aligned = aligned && (((uintptr_t)p.src[i]) % (4 * (SRC == kFP32 ? 4 : SRC == kUInt8 ? 1 : 2))) == 0;
  const bool small = C <= 4 && (HW % 4) == 0 && aligned;
  const uint64_t quads = (uint64_t)(HW / 4) * p.n_imgs;
  if (src_layout == 0 && dst_layout == 1) {  // NCHW -> NHWC
    if (small) {
      dim3 g(grid_for(quads));
      switch (C) {
        case 1: hipLaunchKernelGGL((small_c_to_nhwc<SRC, DST, 1>), g, dim3(kBlock), 0, s, p, dst); break;
        case 2: hipLaunchKernelGGL((small_c_to_nhwc<SRC, DST, 2>), g, dim3(kBlock), 0, s, p, dst); break;
        case 3: hipLaunchKernelGGL((small_c_to_nhwc<SRC, DST, 3>), g, dim3(kBlock), 0, s, p, dst); break;
        case 4: hipLaunchKernelGGL((small_c_to_nhwc<SRC, DST, 4>), g, dim3(kBlock), 0, s, p, dst); break;
      }
    } else {
      int tk = (HW + kTile - 1) / kTile, tr = (C + kTile - 1) / kTile;
      dim3 g(tk < 64 ? tk : 64, tr, p.n_imgs);
      hipLaunchKernelGGL((tiled_transpose<SRC, DST, true>), g, dim3(kBlock), 0, s, p, dst, C, HW);
    }
  } else if (src_layout == 1 && dst_layout == 0) {  // NHWC -> NCHW
    if (small) {
      dim3 g(grid_for(quads));
      switch (C) {
        case 1: hipLaunchKernelGGL((small_c_to_nchw<SRC, DST, 1>), g, dim3(kBlock), 0, s, p, dst); break;
        case 2: hipLaunchKernelGGL((small_c_to_nchw<SRC, DST, 2>), g, dim3(kBlock), 0, s, p, dst); break;
        case 3: hipLaunchKernelGGL((small_c_to_nchw<SRC, DST, 3>), g, dim3(kBlock), 0, s, p, dst); break;
        case 4: hipLaunchKernelGGL((small_c_to_nchw<SRC, DST, 4>), g, dim3(kBlock), 0, s, p, dst); break;
      }
    } else {
      int tk = (C + kTile - 1) / kTile, tr = (HW + kTile - 1) / kTile;
      dim3 g(tk < 64 ? tk : 64, tr, p.n_imgs);
      hipLaunchKernelGGL((tiled_transpose<SRC, DST, false>), g, dim3(kBlock), 0, s, p, dst, HW, C);
    }
  } else if (src_layout == dst_layout) {
    dim3 g(grid_for((uint64_t)C * HW * p.n_imgs));
    if (src_layout == 0) hipLaunchKernelGGL((same_layout<SRC, DST, true>), g, dim3(kBlock), 0, s, p, dst);
    else hipLaunchKernelGGL((same_layout<SRC, DST, false>), g, dim3(kBlock), 0, s, p, dst);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <int SRC>
int dispatch_src(const LayoutParams& p, int sl, int dl, void* dst, int dst_dtype, hipStream_t s) {
  switch (dst_dtype) {
    case kFP32: return dispatch_dst<SRC, kFP32>(p, sl, dl, dst, s);
    case kBF16: return dispatch_dst<SRC, kBF16>(p, sl, dl, dst, s);
    case kFP16: return dispatch_dst<SRC, kFP16>(p, sl, dl, dst, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

// srcs: host array of n_imgs device pointers (each image C*H*W elements in
// src_layout).  dst: contiguous [n_imgs, ...] in dst_layout.  layout codes:
// 0 = NCHW, 1 = NHWC.  scale/bias: host arrays of C floats or NULL.
extern "C" int tcamd_layout_pack(const void* const* srcs, int n_imgs, int src_dtype, int src_layout,
                                 void* dst, int dst_dtype, int dst_layout, int C, int H, int W,
                                 const float* scale, const float* bias, int rounding, void* stream) {
  if (n_imgs <= 0) return hipSuccess;
  if (C <= 0 || C > kMaxChan || H <= 0 || W <= 0) return hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  const uint64_t img_out_elems = (uint64_t)C * H * W;
  const int esz = dtype_size(dst_dtype);
  for (int base = 0; base < n_imgs; base += kMaxImgs) {
    LayoutParams p;
    int cnt = n_imgs - base < kMaxImgs ? n_imgs - base : kMaxImgs;
    for (int i = 0; i < cnt; ++i) p.src[i] = srcs[base + i];
    p.n_imgs = cnt;
    p.C = C;
    p.HW = H * W;
    p.affine = (scale != nullptr || bias != nullptr) ? 1 : 0;
    for (int c = 0; c < C; ++c) {
      p.scale[c] = scale ? scale[c] : 1.0f;
      p.bias[c] = bias ? bias[c] : 0.0f;
    }
    p.rne = rounding;
    void* d = (uint8_t*)dst + (uint64_t)base * img_out_elems * esz;
    int rc;
    switch (src_dtype) {
      case kFP32: rc = dispatch_src<kFP32>(p, src_layout, dst_layout, d, dst_dtype, s); break;
      case kUInt8: rc = dispatch_src<kUInt8>(p, src_layout, dst_layout, d, dst_dtype, s); break;
      case kBF16: rc = dispatch_src<kBF16>(p, src_layout, dst_layout, d, dst_dtype, s); break;
      case kFP16: rc = dispatch_src<kFP16>(p, src_layout, dst_layout, d, dst_dtype, s); break;
      default: return hipErrorInvalidValue;
    }
    if (rc != hipSuccess) return rc;
  }
  return hipSuccess;
}
