// K11 — fused residual add + LayerNorm for the bert_large serving model (gfx950).
//
// BERT's post-LN block ends every sub-layer with LN(x + f(x)).  As two torch
// ops that is an add pass (read 2, write 1) plus a LayerNorm pass (read 1,
// write 1) over [tokens, 1024] bf16: 5 x 50 MB at bs64 x seq384, 48 times per
// forward (rocprofv3 on MI355X: add 24 us + LN 40 us per call, 23% of the
// forward with GELU).  Here one wave owns one row: each lane loads its 16
// elements of x and y (two 16-B loads each), the sum stays in registers, mean
// and variance are exact two-pass reductions over the register copy (wave
// butterfly through DPP-backed shuffles), and the normalised row leaves as
// bf16 — 3 passes over the data instead of 5, one launch instead of two.
// Reference analog: none (the reference client runs no model; this serves the
// `bert_large` perf_analyzer config of BASELINE.json).

#include "kernels/common.h"

namespace {

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pack2(float a, float b) {
  const bf16x2 v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// E = elements per lane (H = 64 * E), a multiple of 8.  Lane l owns the 16-B
// chunks l, l + 64, ... of the row (coalesced: a wave instruction covers 1 KB).
template <int E>
__global__ void __launch_bounds__(256) add_layernorm_kernel(const uint16_t* x, const uint16_t* y,  // out may alias
                                                            const uint16_t* __restrict__ gamma,
                                                            const uint16_t* __restrict__ beta, uint16_t* out,
                                                            int rows, float eps) {
  constexpr int H = 64 * E, C = E / 8;  // 16-B chunks per lane
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const size_t base = (size_t)row * H;
  float v[E];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int off = (c * 64 + lane) * 8;
    const v4u a = *reinterpret_cast<const v4u*>(x + base + off);
    const v4u b = *reinterpret_cast<const v4u*>(y + base + off);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[c * 8 + 2 * q] = __uint_as_float(a[q] << 16) + __uint_as_float(b[q] << 16);
      v[c * 8 + 2 * q + 1] = __uint_as_float(a[q] & 0xffff0000u) + __uint_as_float(b[q] & 0xffff0000u);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < E; ++e) s += v[e];
  const float mean = wave_sum(s) * (1.0f / H);
  float ss = 0.f;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const float d = v[e] - mean;
    ss += d * d;
  }
  const float rstd = rsqrtf(wave_sum(ss) * (1.0f / H) + eps);
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int off = (c * 64 + lane) * 8;
    const v4u g = *reinterpret_cast<const v4u*>(gamma + off);
    const v4u bt = *reinterpret_cast<const v4u*>(beta + off);
    v4u o;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float g0 = __uint_as_float(g[q] << 16), g1 = __uint_as_float(g[q] & 0xffff0000u);
      const float b0 = __uint_as_float(bt[q] << 16), b1 = __uint_as_float(bt[q] & 0xffff0000u);
      o[q] = pack2((v[c * 8 + 2 * q] - mean) * rstd * g0 + b0, (v[c * 8 + 2 * q + 1] - mean) * rstd * g1 + b1);
    }
    *reinterpret_cast<v4u*>(out + base + off) = o;
  }
}

}  // namespace

extern "C" {

// out = LayerNorm(x + y) * gamma + beta over rows of H bf16 elements
// (H in {512, 1024, 2048, 4096}); x, y, out, gamma, beta 16-B aligned; out may alias x or y.
int tcamd_add_layernorm(const void* x, const void* y, const void* gamma, const void* beta, void* out, int rows, int H,
                        float eps, void* stream) {
  if (rows <= 0) return hipSuccess;
  if (((uintptr_t)x | (uintptr_t)y | (uintptr_t)gamma | (uintptr_t)beta | (uintptr_t)out) % 16)
    return hipErrorInvalidValue;
  const dim3 grid((rows + 3) / 4), block(256);
  hipStream_t s = (hipStream_t)stream;
  const auto* px = (const uint16_t*)x;
  const auto* py = (const uint16_t*)y;
  const auto* pg = (const uint16_t*)gamma;
  const auto* pb = (const uint16_t*)beta;
  auto* po = (uint16_t*)out;
  switch (H) {
    case 512: hipLaunchKernelGGL(add_layernorm_kernel<8>, grid, block, 0, s, px, py, pg, pb, po, rows, eps); break;
    case 1024: hipLaunchKernelGGL(add_layernorm_kernel<16>, grid, block, 0, s, px, py, pg, pb, po, rows, eps); break;
    case 2048: hipLaunchKernelGGL(add_layernorm_kernel<32>, grid, block, 0, s, px, py, pg, pb, po, rows, eps); break;
    case 4096: hipLaunchKernelGGL(add_layernorm_kernel<64>, grid, block, 0, s, px, py, pg, pb, po, rows, eps); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // extern "C"
