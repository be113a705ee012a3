// K15: bf16 projection GEMM with fused epilogues for bert_large (gfx950).
//
//   Y[m][n] = epi( sum_k X[m][k] * W[n][k] )      X [M][K], W [N][K] (nn.Linear
//                                                  layout), Y [M][N], all bf16
//   epi: 0 plain | 1 + bias[n] | 2 GELU(. + bias[n]) (erf form) |
//        3 + bias[n] + R[m][n] (residual)
//
// The four BERT-large projections per layer (M = tokens): QKV (N 3072, K 1024,
// plain: K12 applies the bias), attention out (1024, 1024, + bias), FFN up
// (4096, 1024, bias + GELU), FFN down (1024, 4096, + bias).
//
// Block tile 256 x 256 x 64, 8 waves (2 along M x 4 along N), each wave a
// 128 (m) x 64 (n) sub-tile on 16x16x32 bf16 MFMAs with W as operand A (rows =
// output channels) and X as operand B (columns = tokens), so a lane's four
// accumulators are four consecutive output channels of one token: the
// epilogue stores 8 bytes per lane and reads bias / residual the same way.
// Operands are staged global -> LDS by LDS-DMA (global_load_lds, 16 B a lane,
// 8 per thread per K step) into two buffers: the next K step's copies are
// issued before the current step's LDS reads and MFMAs and retired at the one
// barrier per step.  The LDS image is lane-linear (the DMA writes base +
// 16 * lane); rows are 128 B and the 16-B chunk c of row r sits at physical
// chunk c ^ ((r >> 1) & 7), applied on the global SOURCE address, so the 16
// lanes of a ds_read_b128 group (16 consecutive rows, one chunk) hit 16
// distinct slots of the bank rows (conflict-free).
// Blocks are remapped so each XCD (blockIdx % 8 group) walks a contiguous
// range of tiles, N fastest: the X row-panel of consecutive tiles stays in
// that XCD's L2.

#include <atomic>
#include <type_traits>
#include <cmath>
#include <cstdlib>

#include "kernels/common.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));

constexpr int kBM = 256, kBN = 256, kBK = 64;
constexpr int kTileB = kBM * kBK * 2;        // 32 KB: one operand tile
constexpr int kBufB = 2 * kTileB;            // W tile | X tile
constexpr int kLdsG = 2 * kBufB + 8192;      // two buffers: 128 KB (+ 8 KB L2 warm-up trash)

struct GemmParams {
  const uint16_t* x;  // [M][ldx]
  const uint16_t* w;  // [N][ldw]
  const uint16_t* bias;  // [N] (epi >= 1)
  const uint16_t* r;  // [M][ldr] (epi 3)
  uint16_t* y;        // [M][ldy]
  int M, N, K, ldx, ldw, ldr, ldy;
  int mt, nt;         // tiles along M, N
};

__device__ __forceinline__ bf16x8 fr(v4u v) { return __builtin_bit_cast(bf16x8, v); }

__device__ __forceinline__ uint32_t pk(float a, float b) {
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  const bf16x2 v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}

// byte offset of 16-B chunk c of row r in a [rows][64 bf16] tile image
__device__ __forceinline__ int chunk_off(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

// GELU, erf form, with erf from Abramowitz-Stegun 7.1.26 (|error| <= 1.5e-7,
// far below the bf16 output's half ulp): one v_rcp, one v_exp and 8 FMAs
// instead of the device library's branchy erff, which took ~30% of the FFN-up
// tile time in the epilogue (PMC: MFMA busy 35% with erff against 49% with
// no epilogue, profiles/r4_gemm_k15.md)
__device__ __forceinline__ float gelu_erf(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.f));
  float q = fmaf(1.061405429f, t, -1.453152027f);
  q = fmaf(q, t, 1.421413741f);
  q = fmaf(q, t, -0.284496736f);
  q = fmaf(q, t, 0.254829592f);
  q *= t;
  const float e = __builtin_amdgcn_exp2f(-z * z * 1.4426950408889634f);
  const float erf_abs = fmaf(-q, e, 1.f);
  const float erf_x = __builtin_copysignf(erf_abs, x);
  return 0.5f * x * (1.f + erf_x);
}

// C (16x16) of a wave's 128 (m) x 64 (n) sub-tile: lane column = token m,
// rows 4 fq + e = four consecutive output channels -> 8-B stores
template <int EPI>
__device__ __forceinline__ void load_bias(const GemmParams& p, float (&bv)[4][4], int n0, int wn, int fq) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int n = n0 + 64 * wn + 16 * i + 4 * fq;
    bv[i][0] = bv[i][1] = bv[i][2] = bv[i][3] = 0.f;
    if constexpr (EPI >= 1) {
      const v2u bb = *reinterpret_cast<const v2u*>(p.bias + n);
      bv[i][0] = __uint_as_float(bb[0] << 16);
      bv[i][1] = __uint_as_float(bb[0] & 0xffff0000u);
      bv[i][2] = __uint_as_float(bb[1] << 16);
      bv[i][3] = __uint_as_float(bb[1] & 0xffff0000u);
    }
  }
}

template <int EPI, int NJ = 8>
__device__ __forceinline__ void epilogue_b(const GemmParams& p, f32x4 (&acc)[4][NJ], const float (&bv)[4][4], int m0,
                                           int n0, int wm, int wn, int fr16, int fq) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int n = n0 + 64 * wn + 16 * i + 4 * fq;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int m = m0 + NJ * 16 * wm + 16 * j + fr16;
      if (m >= p.M) continue;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e] + bv[i][e];
      if constexpr (EPI == 2) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = gelu_erf(v[e]);
      }
      if constexpr (EPI == 3) {
        const v2u rr = *reinterpret_cast<const v2u*>(p.r + (size_t)m * p.ldr + n);
        v[0] += __uint_as_float(rr[0] << 16);
        v[1] += __uint_as_float(rr[0] & 0xffff0000u);
        v[2] += __uint_as_float(rr[1] << 16);
        v[3] += __uint_as_float(rr[1] & 0xffff0000u);
      }
      *reinterpret_cast<v2u*>(p.y + (size_t)m * p.ldy + n) = v2u{pk(v[0], v[1]), pk(v[2], v[3])};
    }
  }
}

template <int EPI>
__device__ __forceinline__ void epilogue(const GemmParams& p, f32x4 (&acc)[4][8], int m0, int n0, int wm, int wn,
                                         int fr16, int fq) {
  float bv[4][4];
  load_bias<EPI>(p, bv, n0, wn, fq);
  epilogue_b<EPI>(p, acc, bv, m0, n0, wm, wn, fr16, fq);
}

// SPREAD: the next step's 8 LDS-DMA copies are issued one per 8-MFMA group
// instead of all before the step's LDS reads (an LDS-DMA piece costs ~60-185
// issue cycles; issued in a burst by every wave at once they stall the
// matrix pipe at the top of each step)
// L2PF: one more LDS-DMA per thread per step warms L2 with the operand lines
// of the step after next (one 128-B line = one tile row's 64 k; the bytes land
// in a 8 KB trash area of LDS), so the next step's real copies are L2 hits;
// the step barrier is then raw with a counted vmcnt(1) (the warm-up copy may
// stay in flight across it)
template <int EPI, bool SPREAD = false, bool L2PF = false>
__global__ void __launch_bounds__(512, 1) gemm_bf16_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // XCD-contiguous tile order (bijective for any tile count)
  const int nwg = p.mt * p.nt;
  const int b = blockIdx.x, xcd = b & 7, q = nwg >> 3, rem = nwg & 7;
  const int wg = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (b >> 3);
  const int tm = wg / p.nt, tn = wg - tm * p.nt;
  const int m0 = tm * kBM, n0 = tn * kBN;

  // LDS-DMA sources: instruction i of wave w covers tile rows 8(8i + w) ..+8;
  // lane L -> row (8i + w) * 8 + L / 8, physical chunk L % 8
  const uint16_t* srcw[4];
  const uint16_t* srcx[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (8 * i + wave) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    srcw[i] = p.w + (size_t)(n0 + row) * p.ldw + 8 * c;
    srcx[i] = p.x + (size_t)min(m0 + row, p.M - 1) * p.ldx + 8 * c;
  }
  auto stage1 = [&](int kt, int buf, int piece) {  // piece 0..7: W rows 8(8i + w).., then X
    uint8_t* dw = lds + buf * kBufB;
    const int k0 = kt * kBK, i = piece & 3;
    if (piece < 4)
      __builtin_amdgcn_global_load_lds((const void*)(srcw[i] + k0), (void*)(dw + (8 * i + wave) * 1024), 16, 0, 0);
    else
      __builtin_amdgcn_global_load_lds((const void*)(srcx[i] + k0), (void*)(dw + kTileB + (8 * i + wave) * 1024), 16,
                                       0, 0);
  };
  auto stage = [&](int kt, int buf) {
#pragma unroll
    for (int piece = 0; piece < 8; ++piece) stage1(kt, buf, piece);
  };

  const int wm = wave >> 2, wn = wave & 3;  // wave sub-tile: tokens 128 wm.., channels 64 wn..
  const int fr16 = lane & 15, fq = lane >> 4;
  f32x4 acc[4][8];  // [channel frag][token frag]
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = p.K / kBK;
  // L2 warm-up source: thread t -> W row t (t < 256) or X row t - 256
  const uint16_t* srcl2 = tid < 256 ? p.w + (size_t)(n0 + tid) * p.ldw
                                    : p.x + (size_t)min(m0 + tid - 256, p.M - 1) * p.ldx;
  auto warm = [&](int kt) {
    __builtin_amdgcn_global_load_lds((const void*)(srcl2 + (size_t)kt * kBK), (void*)(lds + 2 * kBufB + wave * 1024),
                                     16, 0, 0);
  };
  stage(0, 0);
  if constexpr (L2PF) {
    if (nk > 1) warm(1);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    const bool more = kt + 1 < nk;
    if (!SPREAD && more) stage(kt + 1, buf ^ 1);
    if constexpr (L2PF) {
      if (kt + 2 < nk) warm(kt + 2);  // issued after the copies: it may stay in flight past the barrier
    }
    const uint8_t* tw = lds + buf * kBufB;
    const uint8_t* tx = tw + kTileB;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      v4u a[4], bq[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = *reinterpret_cast<const v4u*>(tw + chunk_off(64 * wn + 16 * i + fr16, 4 * kk + fq));
#pragma unroll
      for (int j = 0; j < 8; ++j) bq[j] = *reinterpret_cast<const v4u*>(tx + chunk_off(128 * wm + 16 * j + fr16, 4 * kk + fq));
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr(a[i]), fr(bq[j]), acc[i][j], 0, 0, 0);
        if constexpr (SPREAD) {
          if (more) stage1(kt + 1, buf ^ 1, 4 * kk + i);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      __builtin_amdgcn_s_setprio(0);
    }
    if constexpr (L2PF) {
      // the next step's 8 copies landed; the warm-up issued after them may not
      __builtin_amdgcn_sched_barrier(0);
      if (kt + 2 < nk) __builtin_amdgcn_s_waitcnt(0x0071);  // vmcnt(1) lgkmcnt(0)
      else __builtin_amdgcn_s_waitcnt(0x0070);            // vmcnt(0) lgkmcnt(0)
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    } else {
      __syncthreads();  // the next step's DMA landed; this buffer's reads are done
    }
  }

  epilogue<EPI>(p, acc, m0, n0, wm, wn, fr16, fq);
}

// ---- pipelined persistent variant (TCAMD_GEMM_V=6) ----
// The one-barrier kernel reads a half step's 12 operand fragments and then
// waits for them before its first MFMA; both waves of a SIMD do so at the same
// moment (the step barrier lines them up), so every half step starts with the
// LDS latency exposed.  Here the fragments are double-buffered in registers:
// a half step's MFMAs run on fragments read during the previous half step.
//   top of step:   DMA of step + 1 -> other buffer; read kk 1 of this step
//   MFMAs kk 0;    barrier (DMA landed, kk 1 reads retired everywhere)
//   read kk 0 of step + 1 (other buffer); MFMAs kk 1
// The other buffer's last reads (kk 1 of the previous step) retired before the
// previous barrier, so its DMA may start at the top of the step.
// Persistent (one workgroup per CU walks its tiles): the next tile's first
// step is staged before this tile's epilogue, so its latency hides there.
// BMT: token rows per tile, 256 or 128 (128: twice the tiles, for N = 1024
// where 256 x 256 tiles leave the last round half empty)
// STAG (TCAMD_GEMM_V=8): waves w and w + 4 share a SIMD and both issued
// their copies at the top of the step, so the SIMD's MFMA pipe idled while
// both were issuing.  With STAG, waves 4-7 issue step kt + 2's copies right
// after step kt's middle barrier (that buffer's reads all retired there), a
// half step before waves 0-3 issue theirs at the top of step kt + 1.
// STAG 2 (TCAMD_GEMM_V=9): every wave issues step kt + 2's copies after step
// kt's middle barrier: a full step of lead for every copy (v6: half a step)
template <int EPI, int BMT = 256, int STAG = 0>
__global__ void __launch_bounds__(512, 1) gemm_bf16_pipe_kernel(GemmParams p) {
  constexpr int NJ = BMT / 32;             // token fragments per wave
  constexpr int NXP = BMT / 64;            // X copies per thread per step
  constexpr int kXB = BMT * kBK * 2;       // X tile bytes
  constexpr int kBuf = kTileB + kXB;       // W tile | X tile
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nwg = p.mt * p.nt, q = nwg >> 3, rem = nwg & 7;
  // persistent: workgroup b takes virtual tiles b, b + G, ... (G % 8 == 0
  // keeps each on the XCD of b); virtual tile -> XCD-contiguous tile order
  auto tile_of = [&](int v, int& m0, int& n0) {
    const int xcd = v & 7;
    const int wg = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (v >> 3);
    const int tm = wg / p.nt;
    m0 = tm * BMT;
    n0 = (wg - tm * p.nt) * kBN;
  };
  const uint16_t* srcw[4];
  const uint16_t* srcx[NXP];
  auto set_src = [&](int m0, int n0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = (8 * i + wave) * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      srcw[i] = p.w + (size_t)(n0 + row) * p.ldw + 8 * c;
      if (i < NXP) srcx[i] = p.x + (size_t)min(m0 + row, p.M - 1) * p.ldx + 8 * c;
    }
  };
  auto stage1 = [&](int kt, int buf, int piece) {  // piece 0-3: W rows, 4..: X rows
    uint8_t* dw = lds + buf * kBuf;
    const int k0 = kt * kBK, i = piece & 3;
    if (piece < 4)
      __builtin_amdgcn_global_load_lds((const void*)(srcw[i] + k0), (void*)(dw + (8 * i + wave) * 1024), 16, 0, 0);
    else
      __builtin_amdgcn_global_load_lds((const void*)(srcx[i] + k0), (void*)(dw + kTileB + (8 * i + wave) * 1024), 16,
                                       0, 0);
  };
  auto stage = [&](int kt, int buf) {
#pragma unroll
    for (int piece = 0; piece < 4 + NXP; ++piece) stage1(kt, buf, piece);
  };
  const int wm = wave >> 2, wn = wave & 3;
  const int fr16 = lane & 15, fq = lane >> 4;
  // per-lane byte offsets of fragment 0 of half step kk; fragment i sits
  // 16 rows (2048 B) further: the swizzle term (r >> 1) & 7 does not change
  // by 16 rows, so the other fragments are immediate offsets
  int oa[2], ob[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    oa[kk] = chunk_off(64 * wn + fr16, 4 * kk + fq);
    ob[kk] = kTileB + chunk_off(NJ * 16 * wm + fr16, 4 * kk + fq);
  }
  v4u fa[2][4], fb[2][NJ];
  auto rd = [&](int buf, int kk) {
    const uint8_t* ta = lds + buf * kBuf + oa[kk];
    const uint8_t* tb = lds + buf * kBuf + ob[kk];
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[kk][i] = *reinterpret_cast<const v4u*>(ta + 2048 * i);
#pragma unroll
    for (int j = 0; j < NJ; ++j) fb[kk][j] = *reinterpret_cast<const v4u*>(tb + 2048 * j);
  };
  f32x4 acc[4][NJ];
  auto mma = [&](int kk) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr(fa[kk][i]), fr(fb[kk][j]), acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // STAG 3: mma(1) with step kt_c's copies (clamped, unconditional: no branch
  // between the MFMA groups) into buffer bufc, one per NJ / 2 MFMAs
  auto mma_copy = [&](int kk, int kt_c, int bufc) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int j = h * NJ / 2; j < (h + 1) * NJ / 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr(fa[kk][i]), fr(fb[kk][j]), acc[i][j], 0, 0, 0);
        if (2 * i + h < 4 + NXP) stage1(kt_c, bufc, 2 * i + h);
        __builtin_amdgcn_sched_barrier(0);
      }
  };

  const int nk = p.K / kBK, G = gridDim.x;
  int vb = blockIdx.x, m0, n0;
  tile_of(vb, m0, n0);
  const bool grp_b = (STAG == 1 && wave >= 4) || STAG >= 2;
  set_src(m0, n0);
  stage(0, 0);
  if (grp_b && nk > 1) stage(1, 1);
  for (;;) {
    __syncthreads();  // this tile's step 0 landed
    rd(0, 0);
    __builtin_amdgcn_s_waitcnt(0xc07f);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < nk; ++kt) {
      const int buf = kt & 1;
      const bool more = kt + 1 < nk;
      if (more && !grp_b) stage(kt + 1, buf ^ 1);
      rd(buf, 1);
      mma(0);
      // step kt + 1's copies landed (explicit: with STAG 2 they were issued in
      // the previous iteration and the compiler does not see them here)
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
      __syncthreads();
      if (STAG != 3 && grp_b && kt + 2 < nk) stage(kt + 2, buf);
      rd(buf ^ 1, 0);  // unconditional (stale on the last step, unused)
      if constexpr (STAG == 3)
        mma_copy(1, kt + 2 < nk ? kt + 2 : nk - 1, buf);  // past the end: a re-copy nothing reads
      else
        mma(1);
      // those reads retired during mma(1); retiring them explicitly here keeps
      // the compiler from draining the kk 1 reads before mma(0) (it loses the
      // count of reads pending across the back edge)
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    }
    // the next tile's first step is in flight during this tile's epilogue;
    // the bias is loaded first (the in-order vmcnt would make its wait a wait
    // for those copies too)
    float bv[4][4];
    load_bias<EPI>(p, bv, n0, wn, fq);
    __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): the bias, before the copies queue behind it
    const int nvb = vb + G;
    int nm0 = 0, nn0 = 0;
    if (nvb < nwg) {
      tile_of(nvb, nm0, nn0);
      set_src(nm0, nn0);
      __syncthreads();  // every wave's last reads of both buffers retired (and the bias landed)
      stage(0, 0);
      if (grp_b && nk > 1) stage(1, 1);
    }
    epilogue_b<EPI, NJ>(p, acc, bv, m0, n0, wm, wn, fr16, fq);
    if (nvb >= nwg) break;
    vb = nvb;
    m0 = nm0;
    n0 = nn0;
  }
}

// ---- one wave per SIMD (TCAMD_GEMM_V=10) ----
// 4 waves of 128 x 128 (2 x 2 over the 256 x 256 tile), 64 accumulators per
// lane (256 registers, AGPR half of the 512-entry file): per 64-k step each
// wave reads 32 fragments for 128 MFMAs (v6: 24 for 64), and the step barrier
// joins 4 waves instead of 8.  With one wave per SIMD nothing hides a stall,
// so the next step's 16 copies per thread are issued one per 4 MFMAs of the
// first half step, and the fragments are double-buffered as in v6.
template <int EPI>
__global__ void __launch_bounds__(256, 1) __attribute__((amdgpu_waves_per_eu(1, 1)))
gemm_bf16_w4_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nwg = p.mt * p.nt;
  const int b = blockIdx.x, xcd = b & 7, q = nwg >> 3, rem = nwg & 7;
  const int wg = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (b >> 3);
  const int tm = wg / p.nt, tn = wg - tm * p.nt;
  const int m0 = tm * kBM, n0 = tn * kBN;
  // copy piece i (0-7) of wave w: tile rows 8 (4 i + w) ..+8 (1 KB); row
  // (4 i + w) 8 + lane / 8 = row0 + 32 i keeps the swizzle of row0, so one
  // 32-bit element offset per operand (the X row clamped per piece) instead
  // of 16 pointers
  const int row0 = wave * 8 + (lane >> 3);
  const int c0 = (lane & 7) ^ ((row0 >> 1) & 7);
  const int offw = (n0 + row0) * p.ldw + 8 * c0;
  auto stage1 = [&](int kt, int buf, int piece) {  // piece 0-7 W, 8-15 X
    uint8_t* dw = lds + buf * kBufB;
    const int k0 = kt * kBK, i = piece & 7;
    if (piece < 8) {
      const uint16_t* src = p.w + offw + (32 * i * p.ldw + k0);
      __builtin_amdgcn_global_load_lds((const void*)src, (void*)(dw + (4 * i + wave) * 1024), 16, 0, 0);
    } else {
      const uint16_t* src = p.x + (min(m0 + row0 + 32 * i, p.M - 1) * p.ldx + 8 * c0 + k0);
      __builtin_amdgcn_global_load_lds((const void*)src, (void*)(dw + kTileB + (4 * i + wave) * 1024), 16, 0, 0);
    }
  };
  const int wm = wave >> 1, wn = wave & 1;
  const int fr16 = lane & 15, fq = lane >> 4;
  int oa[2], ob[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    oa[kk] = chunk_off(128 * wn + fr16, 4 * kk + fq);
    ob[kk] = kTileB + chunk_off(128 * wm + fr16, 4 * kk + fq);
  }
  v4u fa[2][8], fb[2][8];
  auto rd = [&](int buf, int kk) {
    const uint8_t* ta = lds + buf * kBufB + oa[kk];
    const uint8_t* tb = lds + buf * kBufB + ob[kk];
#pragma unroll
    for (int i = 0; i < 8; ++i) fa[kk][i] = *reinterpret_cast<const v4u*>(ta + 2048 * i);
#pragma unroll
    for (int j = 0; j < 8; ++j) fb[kk][j] = *reinterpret_cast<const v4u*>(tb + 2048 * j);
  };
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // COPY: step kt_next's 16 copies go out one per 4 MFMAs (unconditional:
  // branches between the MFMA groups make the compiler shuffle accumulators)
  auto mma = [&](int kk, auto copy_c, int kt_next, int buf_next) {
    constexpr bool COPY = decltype(copy_c)::value;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int j = 4 * h; j < 4 * h + 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr(fa[kk][i]), fr(fb[kk][j]), acc[i][j], 0, 0, 0);
        if constexpr (COPY) {
          stage1(kt_next, buf_next, 2 * i + h);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
  };

  const int nk = p.K / kBK;
#pragma unroll
  for (int piece = 0; piece < 16; ++piece) stage1(0, 0, piece);
  __syncthreads();
  rd(0, 0);
  __builtin_amdgcn_s_waitcnt(0xc07f);
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    rd(buf, 1);
    // the last step re-copies itself into the other buffer (read by nothing)
    mma(0, std::true_type{}, kt + 1 < nk ? kt + 1 : nk - 1, buf ^ 1);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): step kt + 1 landed
    __syncthreads();
    rd(buf ^ 1, 0);  // unconditional (stale on the last step, unused)
    mma(1, std::false_type{}, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
  }
  // epilogue: lane column = token, four consecutive channels -> 8-B stores
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int n = n0 + 128 * wn + 16 * i + 4 * fq;
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if constexpr (EPI >= 1) {
      const v2u bb = *reinterpret_cast<const v2u*>(p.bias + n);
      bv[0] = __uint_as_float(bb[0] << 16);
      bv[1] = __uint_as_float(bb[0] & 0xffff0000u);
      bv[2] = __uint_as_float(bb[1] << 16);
      bv[3] = __uint_as_float(bb[1] & 0xffff0000u);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int m = m0 + 128 * wm + 16 * j + fr16;
      if (m >= p.M) continue;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e] + bv[e];
      if constexpr (EPI == 2) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = gelu_erf(v[e]);
      }
      if constexpr (EPI == 3) {
        const v2u rr = *reinterpret_cast<const v2u*>(p.r + (size_t)m * p.ldr + n);
        v[0] += __uint_as_float(rr[0] << 16);
        v[1] += __uint_as_float(rr[0] & 0xffff0000u);
        v[2] += __uint_as_float(rr[1] << 16);
        v[3] += __uint_as_float(rr[1] & 0xffff0000u);
      }
      *reinterpret_cast<v2u*>(p.y + (size_t)m * p.ldy + n) = v2u{pk(v[0], v[1]), pk(v[2], v[3])};
    }
  }
}

// ---- deep variant (TCAMD_GEMM_V=7): five 32-k stages, 3 stages of DMA lead ----
// At 2 stages of 64 k the next step's copies must land within half a step of
// their issue (v6) -- far less than an L2 miss under load.  Here a stage is
// 32 k (W 256 x 32 | X 256 x 32 bf16 = 32 KB, 2 + 2 LDS-DMA per thread) and
// five stages fill the 160 KB of LDS: the copies of stage s + 4 are issued in
// iteration s and read in iteration s + 3.  Iteration s:
//   counted vmcnt (stage s + 1 landed: stages s + 2, s + 3 may stay in
//   flight) -> raw barrier -> DMA of stage s + 4 into stage s - 1's slot ->
//   read stage s + 1's fragments -> MFMAs on stage s's (read one iteration
//   earlier) -> retire the reads.
// Past the last stage the DMA is re-issued for the last stage into the free
// slot, so every iteration issues four copies and the counts hold.
// Rows are 64 B (4 chunks); chunk c of row r sits at c ^ g((r >> 2) & 3),
// g = (0, 2, 3, 1): the 16 lanes of each ds_read_b128 group (rows 0-3 and
// 12-15 of one chunk, rows 4-11 of the next, or the mirror) hit 16 distinct
// 16-B slots of the 256-B bank row.
constexpr int kBK32 = 32;
constexpr int kStB = 2 * kBM * kBK32 * 2;  // 32 KB: W | X of one 32-k stage
constexpr int kNSt = 5;
constexpr int kLdsD = kNSt * kStB;  // 160 KB
static_assert(kLdsD <= 160 * 1024, "LDS");
__device__ __forceinline__ int g32(int r) { return (0x78 >> (2 * ((r >> 2) & 3))) & 3; }
__device__ __forceinline__ int off32(int r, int c) { return r * 64 + ((c ^ g32(r)) << 4); }
constexpr int gvm(int n) { return (((n >> 4) & 3) << 14) | (0xF << 8) | (7 << 4) | (n & 15); }

template <int EPI>
__global__ void __launch_bounds__(512, 1) gemm_bf16_deep_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nwg = p.mt * p.nt;
  const int b = blockIdx.x, xcd = b & 7, q = nwg >> 3, rem = nwg & 7;
  const int wg = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (b >> 3);
  const int tm = wg / p.nt, tn = wg - tm * p.nt;
  const int m0 = tm * kBM, n0 = tn * kBN;
  // DMA instruction i of wave w writes tile rows 16 (8 i + w) ..+16 (1 KB):
  // lane L -> row 16 (8 i + w) + L / 4, physical chunk L % 4
  const uint16_t* srcw[2];
  const uint16_t* srcx[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 16 * (8 * i + wave) + (lane >> 2);
    const int c = (lane & 3) ^ g32(row);
    srcw[i] = p.w + (size_t)(n0 + row) * p.ldw + 8 * c;
    srcx[i] = p.x + (size_t)min(m0 + row, p.M - 1) * p.ldx + 8 * c;
  }
  const int ns = p.K / kBK32;
  auto stage = [&](int st, int slot) {
    uint8_t* d = lds + slot * kStB;
    const int k0 = min(st, ns - 1) * kBK32;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(srcw[i] + k0), (void*)(d + (8 * i + wave) * 1024), 16, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(srcx[i] + k0), (void*)(d + kStB / 2 + (8 * i + wave) * 1024),
                                       16, 0, 0);
  };
  const int wm = wave >> 2, wn = wave & 3;
  const int fr16 = lane & 15, fq = lane >> 4;
  // fragment 0's offset; fragment i sits 16 rows = 1 KB further (g32 is
  // periodic in 16 rows)
  const int oa = off32(64 * wn + fr16, fq), ob = kStB / 2 + off32(128 * wm + fr16, fq);
  v4u fa[2][4], fb[2][8];
  auto rd = [&](int slot, int set) {
    const uint8_t* ta = lds + slot * kStB + oa;
    const uint8_t* tb = lds + slot * kStB + ob;
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[set][i] = *reinterpret_cast<const v4u*>(ta + 1024 * i);
#pragma unroll
    for (int j = 0; j < 8; ++j) fb[set][j] = *reinterpret_cast<const v4u*>(tb + 1024 * j);
  };
  f32x4 acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](int set) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr(fa[set][i]), fr(fb[set][j]), acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

#pragma unroll
  for (int st = 0; st < kNSt - 1; ++st) stage(st, st);
  __builtin_amdgcn_s_waitcnt(gvm(12));  // stage 0 landed (this wave's copies)
  __builtin_amdgcn_s_barrier();
  rd(0, 0);
  __builtin_amdgcn_s_waitcnt(0xc07f);
  int slot = 0;  // stage s's slot
  // the fragment set must be a compile-time index (a runtime one turns the
  // register arrays into scratch): two iterations per loop trip (ns is even)
  auto step = [&](int s, auto cur_c) {
    constexpr int C = decltype(cur_c)::value;
    const int nx = slot == kNSt - 1 ? 0 : slot + 1;   // stage s + 1
    const int fr = slot == 0 ? kNSt - 1 : slot - 1;   // stage s - 1 = s + 4
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(gvm(8));  // stage s + 1 landed
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    stage(s + kNSt - 1, fr);
    rd(nx, C ^ 1);
    mma(C);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the stage s + 1 reads retired
    slot = nx;
  };
  for (int s = 0; s < ns; s += 2) {
    step(s, std::integral_constant<int, 0>{});
    step(s + 1, std::integral_constant<int, 1>{});
  }
  __builtin_amdgcn_s_waitcnt(gvm(0));  // the trailing re-issued copies
  epilogue<EPI>(p, acc, m0, n0, wm, wn, fr16, fq);
}

// ---- phased variant: 4 phases per K step, counted vmcnt across barriers ----
// A K step's 64 MFMAs per wave run as four 16-MFMA quadrant clusters (64
// tokens x 32 channels of the wave's 128 x 64 sub-tile), ordered (qm, qn) =
// (0,0) (0,1) (1,1) (1,0) so each phase reads only the operand that changed
// (12, 4, 8, 4 ds_read_b128).  The next K step is staged by quarter-tiles in
// the order the phases need them, one per phase:
//   S0 X rows of qm 0 (tokens 0-63, 128-191), S1 W rows of qn 0 (channel rows
//   r % 64 < 32), S2 W rows of qn 1, S3 X rows of qm 1,
// each 16 KB = 2 LDS-DMA per thread.  Phase = counted vmcnt (the quarter this
// phase reads landed; the two younger quarters stay in flight) -> raw
// barrier -> stage the next step's quarter into the other buffer (every read
// of that buffer retired before this barrier) -> LDS reads -> MFMA cluster.
// One barrier per phase; no vmcnt(0) in steady state.
__device__ __forceinline__ int sub_rowbase(int s, int g) {  // 8-row group g (0..15) of quarter s
  switch (s) {
    case 0: return g < 8 ? 8 * g : 128 + 8 * (g - 8);
    case 1: return 64 * (g >> 2) + 8 * (g & 3);
    case 2: return 64 * (g >> 2) + 32 + 8 * (g & 3);
    default: return g < 8 ? 64 + 8 * g : 192 + 8 * (g - 8);
  }
}

// STAG: the two wave groups (waves 0-3 = token half 0, waves 4-7 = half 1)
// run one phase apart (waves 4-7 pass one extra barrier first, waves 0-3 one
// extra at the end), so on every SIMD one wave's MFMA cluster overlaps the
// other wave's LDS reads.  A quarter staged by the late group lands one
// barrier later, so that group retires its copies one phase earlier (the
// counts below); the buffer a group restages was last read by the late
// group in the early group's staging interval only for rows the early group
// does not write then (phase 3 reads W rows qn 0, phase 0 stages X rows qm 0).
template <int EPI, bool STAG>
__global__ void __launch_bounds__(512, 1) gemm_bf16_ph_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nwg = p.mt * p.nt;
  const int b = blockIdx.x, xcd = b & 7, q = nwg >> 3, rem = nwg & 7;
  const int wg = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (b >> 3);
  const int tm = wg / p.nt, tn = wg - tm * p.nt;
  const int m0 = tm * kBM, n0 = tn * kBN;

  // per quarter s and instruction i: the lane's source row and the group's LDS row base
  const uint16_t* src[4][2];
  int dbase[4][2];
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int rb = sub_rowbase(s, 8 * i + wave);
      const int row = rb + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      const bool isx = s == 0 || s == 3;
      src[s][i] = isx ? p.x + (size_t)min(m0 + row, p.M - 1) * p.ldx + 8 * c : p.w + (size_t)(n0 + row) * p.ldw + 8 * c;
      dbase[s][i] = (isx ? kTileB : 0) + rb * 128;
    }
  auto stage = [&](int kt, int buf, int s) {
    const int k0 = kt * kBK;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(src[s][i] + k0), (void*)(lds + buf * kBufB + dbase[s][i]), 16, 0,
                                       0);
  };

  const int wm = wave >> 2, wn = wave & 3;
  const int fr16 = lane & 15, fq = lane >> 4;
  f32x4 acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = p.K / kBK;
  const int grp = __builtin_amdgcn_readfirstlane(wave >> 2);  // scalar: a wave-uniform branch
#pragma unroll
  for (int s = 0; s < 4; ++s) stage(0, 0, s);
  __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) lgkmcnt(0): step 0 landed
  __builtin_amdgcn_s_barrier();
  if (STAG && grp) __builtin_amdgcn_s_barrier();  // the late group starts one phase behind
  v4u xa[4][2], wa[2][2];
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    const bool last = kt + 1 == nk;
    const uint8_t* tw = lds + buf * kBufB;
    const uint8_t* tx = tw + kTileB;
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) {
      const int qm = ph >> 1, qn = (ph == 1 || ph == 2) ? 1 : 0;
      // the quarter this phase reads landed (issue order: S0..S3 per step);
      // the late group retires the quarter the NEXT phase reads
      if (STAG && grp) {
        if (last) {
          if (ph == 0) __builtin_amdgcn_s_waitcnt(0x0F72);  // vmcnt(2)
          else __builtin_amdgcn_s_waitcnt(0x0F70);          // vmcnt(0)
        } else {
          if (ph == 2) __builtin_amdgcn_s_waitcnt(0x0F74);  // vmcnt(4)
          else __builtin_amdgcn_s_waitcnt(0x0F72);          // vmcnt(2)
        }
      } else if (last) {
        if (ph == 0) __builtin_amdgcn_s_waitcnt(0x0F74);       // vmcnt(4)
        else if (ph == 1) __builtin_amdgcn_s_waitcnt(0x0F72);  // vmcnt(2)
        else __builtin_amdgcn_s_waitcnt(0x0F70);               // vmcnt(0)
      } else {
        if (ph == 3) __builtin_amdgcn_s_waitcnt(0x0F76);       // vmcnt(6)
        else __builtin_amdgcn_s_waitcnt(0x0F74);               // vmcnt(4)
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (!last) stage(kt + 1, buf ^ 1, ph);
      if (ph == 0 || ph == 2) {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            xa[j][kk] = *reinterpret_cast<const v4u*>(tx + chunk_off(128 * wm + 64 * qm + 16 * j + fr16, 4 * kk + fq));
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 2; ++i)
          wa[i][kk] = *reinterpret_cast<const v4u*>(tw + chunk_off(64 * wn + 32 * qn + 16 * i + fr16, 4 * kk + fq));
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[2 * qn + i][4 * qm + j] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr(wa[i][kk]), fr(xa[j][kk]), acc[2 * qn + i][4 * qm + j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  if (STAG && !grp) __builtin_amdgcn_s_barrier();  // matches the late group's extra barrier
  epilogue<EPI>(p, acc, m0, n0, wm, wn, fr16, fq);
}

}  // namespace

extern "C" {

// Y = epi(X W^T): bf16 X [M][ldx], W [N][ldw], Y [M][ldy]; N % 256 == 0,
// K % 64 == 0, leading dimensions multiples of 8 elements, 16-B aligned bases.
int tcamd_gemm_bf16(const void* x, const void* w, const void* bias, const void* r, void* y, int M, int N, int K,
                    int ldx, int ldw, int ldr, int ldy, int epi, void* stream) {
  if (M <= 0) return hipSuccess;
  if (N <= 0 || N % kBN || K <= 0 || K % kBK || epi < 0 || epi > 3) return hipErrorInvalidValue;
  if (!x || !w || !y || ldx < K || ldw < K || ldy < N || ldx % 8 || ldw % 8 || ldy % 8) return hipErrorInvalidValue;
  if (epi >= 1 && !bias) return hipErrorInvalidValue;
  if (epi == 3 && (!r || ldr < N || ldr % 8)) return hipErrorInvalidValue;
  auto al = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
  if (!al(x) || !al(w) || !al(y) || (bias && ((uintptr_t)bias & 7)) || (r && !al(r))) return hipErrorInvalidValue;
  GemmParams p;
  p.x = (const uint16_t*)x;
  p.w = (const uint16_t*)w;
  p.bias = (const uint16_t*)bias;
  p.r = (const uint16_t*)r;
  p.y = (uint16_t*)y;
  p.M = M;
  p.N = N;
  p.K = K;
  p.ldx = ldx;
  p.ldw = ldw;
  p.ldr = ldr;
  p.ldy = ldy;
  p.mt = (M + kBM - 1) / kBM;
  p.nt = N / kBN;
  // TCAMD_GEMM_V: 1 = one barrier per K step, 2 = the phased
  // kernel, 3 = phased with the two wave groups one phase apart, 4 = one
  // barrier per step with the DMA spread over the MFMA groups, 5 = 1 with the
  // L2 warm-up of the step after next, 6 = fragments double-buffered in
  // registers, persistent (the pipelined kernel; default), 7 = five 32-k
  // stages (the deep kernel), 8 = 6 with the SIMD-partner waves' copies half a
  // step apart, 9 = 6 with every copy issued a full step ahead, 10 = one
  // wave per SIMD (4 waves of 128 x 128), 11 = 9 with the copies spread
  // over the second MFMA half
  static const int ver = getenv("TCAMD_GEMM_V") ? atoi(getenv("TCAMD_GEMM_V")) : 6;
  const void* all[11][4] = {{(const void*)gemm_bf16_kernel<0>, (const void*)gemm_bf16_kernel<1>,
                            (const void*)gemm_bf16_kernel<2>, (const void*)gemm_bf16_kernel<3>},
                           {(const void*)gemm_bf16_ph_kernel<0, false>, (const void*)gemm_bf16_ph_kernel<1, false>,
                            (const void*)gemm_bf16_ph_kernel<2, false>, (const void*)gemm_bf16_ph_kernel<3, false>},
                           {(const void*)gemm_bf16_ph_kernel<0, true>, (const void*)gemm_bf16_ph_kernel<1, true>,
                            (const void*)gemm_bf16_ph_kernel<2, true>, (const void*)gemm_bf16_ph_kernel<3, true>},
                           {(const void*)gemm_bf16_kernel<0, true>, (const void*)gemm_bf16_kernel<1, true>,
                            (const void*)gemm_bf16_kernel<2, true>, (const void*)gemm_bf16_kernel<3, true>},
                           {(const void*)gemm_bf16_kernel<0, false, true>, (const void*)gemm_bf16_kernel<1, false, true>,
                            (const void*)gemm_bf16_kernel<2, false, true>, (const void*)gemm_bf16_kernel<3, false, true>},
                           {(const void*)gemm_bf16_pipe_kernel<0>, (const void*)gemm_bf16_pipe_kernel<1>,
                            (const void*)gemm_bf16_pipe_kernel<2>, (const void*)gemm_bf16_pipe_kernel<3>},
                           {(const void*)gemm_bf16_deep_kernel<0>, (const void*)gemm_bf16_deep_kernel<1>,
                            (const void*)gemm_bf16_deep_kernel<2>, (const void*)gemm_bf16_deep_kernel<3>},
                           {(const void*)gemm_bf16_pipe_kernel<0, 256, 1>,
                            (const void*)gemm_bf16_pipe_kernel<1, 256, 1>,
                            (const void*)gemm_bf16_pipe_kernel<2, 256, 1>,
                            (const void*)gemm_bf16_pipe_kernel<3, 256, 1>},
                           {(const void*)gemm_bf16_pipe_kernel<0, 256, 2>,
                            (const void*)gemm_bf16_pipe_kernel<1, 256, 2>,
                            (const void*)gemm_bf16_pipe_kernel<2, 256, 2>,
                            (const void*)gemm_bf16_pipe_kernel<3, 256, 2>},
                           {(const void*)gemm_bf16_w4_kernel<0>, (const void*)gemm_bf16_w4_kernel<1>,
                            (const void*)gemm_bf16_w4_kernel<2>, (const void*)gemm_bf16_w4_kernel<3>},
                           {(const void*)gemm_bf16_pipe_kernel<0, 256, 3>,
                            (const void*)gemm_bf16_pipe_kernel<1, 256, 3>,
                            (const void*)gemm_bf16_pipe_kernel<2, 256, 3>,
                            (const void*)gemm_bf16_pipe_kernel<3, 256, 3>}};
  const void* half[4] = {(const void*)gemm_bf16_pipe_kernel<0, 128>, (const void*)gemm_bf16_pipe_kernel<1, 128>,
                         (const void*)gemm_bf16_pipe_kernel<2, 128>, (const void*)gemm_bf16_pipe_kernel<3, 128>};
  const void* const* fns = all[(ver >= 2 && ver <= 11) ? ver - 1 : 0];
  // v6: 128-token tiles (TCAMD_GEMM_HALF: 0 never, 1 (default) when N <= 1024
  // and 256-token tiles would fill at most half the CUs, 2 always).  Measured
  // (profiles/r4_gemm_k15.md): 3072 tokens x N 1024 +33-61%; at 24,576 tokens
  // or N >= 3072 the smaller tiles lose more per tile than the fuller last
  // round gains
  static const int half_mode = getenv("TCAMD_GEMM_HALF") ? atoi(getenv("TCAMD_GEMM_HALF")) : 1;
  const bool use_half = ver == 6 && (half_mode == 2 || (half_mode == 1 && N <= 1024 && p.mt * p.nt <= 128));
  if (use_half) {
    fns = half;
    p.mt = (M + 127) / 128;
  }
  // dynamic-LDS opt-in once per device (cached only after every call succeeded)
  static std::atomic<bool> attr_set[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (!attr_set[dev].load(std::memory_order_acquire)) {
    for (const auto& row : all)
      for (const void* f : row) {
        const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsD);
        if (e != hipSuccess) return e;
      }
    for (const void* f : half) {
      const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsD);
      if (e != hipSuccess) return e;
    }
    attr_set[dev].store(true, std::memory_order_release);
  }
  void* args[] = {&p};
  int grid = p.mt * p.nt;
  if (ver == 6 || (ver >= 8 && ver != 10)) {  // persistent: one workgroup per CU (a multiple of 8: XCD-stable)
    static std::atomic<int> ncu_cache[64];
    int ncu = ncu_cache[dev].load(std::memory_order_relaxed);
    if (ncu <= 0) {
      if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < 8) ncu = 256;
      ncu &= ~7;
      ncu_cache[dev].store(ncu, std::memory_order_relaxed);
    }
    grid = grid < ncu ? grid : ncu;
  }
  const int lds_b = ver == 7 ? kLdsD : use_half ? 2 * (kTileB + 128 * kBK * 2) : kLdsG;
  const hipError_t e =
      hipLaunchKernel(fns[epi], dim3(grid), dim3(ver == 10 ? 256 : 512), args, lds_b, (hipStream_t)stream);
  if (e != hipSuccess) return e;
  return hipGetLastError();
}

}  // extern "C"
