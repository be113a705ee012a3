// K8x/K9x/K10x — fp32-parity DenseNet-121 inference kernels for CDNA4 (gfx950).
//
// The reference's densenet_onnx contract is FP32 in, FP32 out, FP32 compute
// (reference src/python/examples/image_client.py:84-86 builds FP32 inputs for
// an fp32 ONNX graph).  gfx950 has no xf32 MFMA and its f32-input MFMA runs at
// 1/16 of the bf16 rate, so these kernels compute every conv as a
// split-precision "bf16x3" product on the bf16 MFMA:
//
//     a = a_hi + a_lo,  a_hi = bf16_rne(a),  a_lo = bf16_rne(a - a_hi)
//     a*b ~= a_hi*b_hi + a_hi*b_lo + a_lo*b_hi          (fp32 accumulate)
//
// a_hi + a_lo carries 16 significant bits (|a - a_hi - a_lo| <= 2^-17 |a|)
// and the dropped a_lo*b_lo term is <= 2^-16 of the product, so each conv is
// within ~1e-5 relative of an fp32 conv at 3/16 of the f32-MFMA cost.
//
// Layout (all activations stay fp32 in HBM — 288 GB leaves room to spare):
//  * every dense block owns ONE NHWC fp32 feature buffer [pixels][C_block];
//    a layer's 3x3 conv writes its 32 new channels into its slice (the concat
//    is free) and the next layer's 1x1 conv reads the first K channels;
//  * K8x conv1x1: the BN1+ReLU pre-activation (consumer specific) is applied
//    to the fp32 X tile while it is staged global->LDS and split into hi/lo
//    tiles there; BN2 is folded into W (pre-split on the host) and its bias +
//    ReLU run in the epilogue, which writes the 128-channel bottleneck z as
//    TWO bf16 planes z_hi/z_lo (the 3x3 conv's operands, already split:
//    same bytes as fp32).  POOL=true is the transition: BN+ReLU+2x2 avg-pool
//    in the prologue, fp32 output into the next block's buffer;
//  * K9x conv3x3 (128->32): 8 waves = 2 pixel halves x 4 input-channel
//    quarters, each wave's hi/lo weight fragments for all nine taps in
//    registers for the whole persistent kernel (loaded from a fragment-major
//    copy, x3_w3_fragments); a block walks a run of 64-pixel tiles with the
//    z_hi/z_lo band in an LDS ring fed by LDS-DMA, and the 4 partials are
//    summed through LDS in one round;
//  * K10x stem (7x7/2 conv + BN + ReLU + 3x3/2 max-pool, fp32 images read
//    through a device pointer table) and head (BN+ReLU+global avg-pool).
//
// MFMA operand orientation as in densenet.hip: WEIGHTS are operand A (rows =
// output channels), activations operand B (cols = pixels), so a lane's
// accumulators are consecutive output channels of one pixel.

#include <algorithm>
#include <atomic>
#include <climits>
#include <cstdlib>

#include "kernels/common.h"
#include "kernels/knobs.h"

// Host-side per-device caches (CU count, dynamic-LDS opt-ins): indexed by the
// current HIP device, clamped into the table.
constexpr int kMaxDevices = 64;
static int device_slot() {
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= kMaxDevices) d = 0;
  return d;
}

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));

__device__ __forceinline__ v4u ld16(const void* p) { return *reinterpret_cast<const v4u*>(p); }
__device__ __forceinline__ f32x4 ldf4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }

// two fp32 -> packed bf16, RNE (gfx950 v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint32_t pk(float a, float b) {
  const bf16x2 v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}

// hi/lo split of two fp32: a ~= hi + lo to 2^-17 relative (a - hi is exact).
// (A v_pk_fma_f32 / v_pk_add_f32 form of this and of the BN affine issues
// fewer instructions but measured 3-8% slower in K14x / K8x / K11x: round 4.)
// (hipcc turns the hi << 16 below into a second v_cvt_pk_bf16_f32 of (a, 0)
// plus a shift; a v_perm_b32 instead issued fewer instructions but measured
// 1-5% slower in K14x, round 4.)
__device__ __forceinline__ void split2(float a, float b, uint32_t& hi, uint32_t& lo) {
  hi = pk(a, b);
  lo = pk(a - __uint_as_float(hi << 16), b - __uint_as_float(hi & 0xffff0000u));
}

// relu(x * s + t), per element (as scalar v_fma_f32)
__device__ __forceinline__ f32x4 bn_relu4(f32x4 x, f32x4 s, f32x4 t) {
  f32x4 v;
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = fmaxf(__builtin_fmaf(x[e], s[e], t[e]), 0.f);
  return v;
}

__device__ __forceinline__ void split4(f32x4 v, v2u& hi, v2u& lo) {
  uint32_t h0, l0, h1, l1;
  split2(v[0], v[1], h0, l0);
  split2(v[2], v[3], h1, l1);
  hi = v2u{h0, h1};
  lo = v2u{l0, l1};
}

__device__ __forceinline__ bf16x8 fr(v4u v) { return __builtin_bit_cast(bf16x8, v); }

// bf16x3 products; the two small cross terms go in first
__device__ __forceinline__ f32x4 x3_16(v4u ah, v4u al, v4u bh, v4u bl, f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr(al), fr(bh), c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr(ah), fr(bl), c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr(ah), fr(bh), c, 0, 0, 0);
}

__device__ __forceinline__ f32x16 x3_32(v4u ah, v4u al, v4u bh, v4u bl, f32x16 c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fr(al), fr(bh), c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fr(ah), fr(bl), c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(fr(ah), fr(bh), c, 0, 0, 0);
}

// ============================================================================
// K8x: 1x1 conv, split-precision GEMM with fused pre-activation
// ============================================================================
struct X3Conv1x1Params {
  const float* x;        // [rows][ldx] fp32 (rows = M, or the pre-pool pixels)
  const float* in_scale; // [K] BN scale of the pre-activation
  const float* in_bias;  // [K]
  const uint16_t* w_hi;  // [N][K] bf16
  const uint16_t* w_lo;  // [N][K] bf16
  const float* out_bias; // [N] (SPLIT epilogue: bias + ReLU)
  uint16_t* z_hi;        // SPLIT: [M][128] bf16 planes
  uint16_t* z_lo;
  float* y;              // !SPLIT: [M][ldy] fp32, raw conv output
  float* ws;             // split-K partials [splits][M][N] (null = whole K per block)
  int ldx, M, K, N, ldy, H, W, k_per_split;
  int xcd_group;         // N > 128: sibling N-tiles of an M-tile on one XCD (see the kernel)
};

constexpr int kBN = 128, kBK = 32, kLDK = kBK + 8;  // 80-B LDS rows: conflict-free b128 reads

// Block = 4 waves as WM (pixels) x 4/WM (channels) over a BM x 128 tile:
//   BM 128, WM 2: wave tile 64 x 64 = 4 x 4 16x16x32 MFMA tiles (48 MFMAs per
//                 K step) — the big-M layers (56x56 / 28x28 at bs128);
//   BM 32,  WM 1: wave tile 32 x 32 = 2 x 2 tiles — small M (14x14 / 7x7,
//                 small batches): 4x the blocks of BM 128 so the whole K runs
//                 in one block instead of split-K partials + a reduce kernel
//                 (the partials cost more HBM traffic than the conv's input).
// The LDS tiles are double-buffered; the global loads of the next PF K steps
// are in flight in a register ring while this step's MFMAs run (one barrier
// per step).  PF 1 for BM 128 (its registers are full); PF 4 for the small
// tiles, whose per-step MFMA work is far shorter than an HBM round trip.
template <bool POOL, bool SPLIT, int BM, int WM, int PF>
__global__ void __launch_bounds__(256, 2) x3_conv1x1_kernel(X3Conv1x1Params p) {
  constexpr int NS = POOL ? 4 : 1;
  constexpr int WN = 4 / WM;
  constexpr int TI = BM / WM / 16;   // pixel tiles per wave
  constexpr int TJ = kBN / WN / 16;  // channel tiles per wave
  constexpr int XC = BM / 32;        // X 16-B chunks per thread per K step
  __shared__ __attribute__((aligned(16))) uint16_t sXh[2][BM * kLDK];
  __shared__ __attribute__((aligned(16))) uint16_t sXl[2][BM * kLDK];
  __shared__ __attribute__((aligned(16))) uint16_t sWh[2][kBN * kLDK];
  __shared__ __attribute__((aligned(16))) uint16_t sWl[2][kBN * kLDK];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  // N-tiles of one M-tile (transitions, N > 128): with p.xcd_group, grid.x =
  // m-groups x nt x 8 and block L runs (m_tile = (L/8/nt)*8 + L%8, n = L/8 %
  // nt), so the nt blocks sharing an X tile sit 8 ids apart — the same XCD,
  // back to back — and the re-reads of X hit that XCD's L2
  int mt = blockIdx.x, nt_i = blockIdx.z;
  if (p.xcd_group) {
    const int nt = p.N / kBN, r = blockIdx.x >> 3;
    mt = (r / nt) * 8 + (blockIdx.x & 7);
    nt_i = r % nt;
    if (mt * BM >= p.M) return;
  }
  const int m0 = mt * BM, n0 = nt_i * kBN;

  // X: BM rows x 8 chunks of 4 fp32 per K step, all of a thread's chunks at
  // the same K offset (tid & 7); POOL: each chunk averages 4 source rows
  const int xk = (tid & 7) * 4;
  const float* xs[XC][NS];
  bool xok[XC];
#pragma unroll
  for (int i = 0; i < XC; ++i) {
    const int r = (tid >> 3) + 32 * i;
    const int m = m0 + r;
    xok[i] = m < p.M;
    const int mm = xok[i] ? m : 0;
    if constexpr (POOL) {
      const int wo = p.W >> 1, ho = p.H >> 1;
      const int img = mm / (ho * wo), rr = mm - img * ho * wo;
      const int oh = rr / wo, ow = rr - oh * wo;
      const size_t base = ((size_t)img * p.H + 2 * oh) * p.W + 2 * ow;
      xs[i][0] = p.x + base * p.ldx + xk;
      xs[i][1] = p.x + (base + 1) * p.ldx + xk;
      xs[i][2] = p.x + (base + p.W) * p.ldx + xk;
      xs[i][3] = p.x + (base + p.W + 1) * p.ldx + xk;
    } else {
      xs[i][0] = p.x + (size_t)mm * p.ldx + xk;
    }
  }
  // W: 128 rows x 4 chunks of 8 bf16 per plane -> 2 chunks per thread per plane
  const int wk = (tid & 3) * 8;
  const uint16_t* wsh[2];
  const uint16_t* wsl[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = (tid >> 2) + 64 * i;
    wsh[i] = p.w_hi + (size_t)(n0 + r) * p.K + wk;
    wsl[i] = p.w_lo + (size_t)(n0 + r) * p.K + wk;
  }

  f32x4 rx[PF][XC][NS], rs[PF], rt[PF];
  v4u rwh[PF][2], rwl[PF][2];
  auto load_step = [&](int slot, int k0) {
    rs[slot] = ldf4(p.in_scale + k0 + xk);
    rt[slot] = ldf4(p.in_bias + k0 + xk);
#pragma unroll
    for (int i = 0; i < XC; ++i)
#pragma unroll
      for (int s = 0; s < NS; ++s) rx[slot][i][s] = xok[i] ? ldf4(xs[i][s] + k0) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      rwh[slot][i] = ld16(wsh[i] + k0);
      rwl[slot][i] = ld16(wsl[i] + k0);
    }
  };
  auto store_step = [&](int slot, int buf) {
#pragma unroll
    for (int i = 0; i < XC; ++i) {
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if constexpr (POOL) {
          float a = 0.f;
#pragma unroll
          for (int s = 0; s < NS; ++s) a += fmaxf(rx[slot][i][s][e] * rs[slot][e] + rt[slot][e], 0.f);
          v[e] = 0.25f * a;
        } else {
          v[e] = fmaxf(rx[slot][i][0][e] * rs[slot][e] + rt[slot][e], 0.f);
        }
        if (!xok[i]) v[e] = 0.f;
      }
      v2u h, l;
      split4(v, h, l);
      const int off = ((tid >> 3) + 32 * i) * kLDK + xk;
      *reinterpret_cast<v2u*>(&sXh[buf][off]) = h;
      *reinterpret_cast<v2u*>(&sXl[buf][off]) = l;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int off = ((tid >> 2) + 64 * i) * kLDK + wk;
      *reinterpret_cast<v4u*>(&sWh[buf][off]) = rwh[slot][i];
      *reinterpret_cast<v4u*>(&sWl[buf][off]) = rwl[slot][i];
    }
  };

  const int fr16 = lane & 15, fk = 8 * (lane >> 4);
  f32x4 acc[TJ][TI];
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    f32x4 b0 = f32x4{0.f, 0.f, 0.f, 0.f};
    if (SPLIT && !p.ws) b0 = ldf4(p.out_bias + n0 + wn * (kBN / WN) + j * 16 + (lane >> 4) * 4);
#pragma unroll
    for (int i = 0; i < TI; ++i) acc[j][i] = b0;
  }

  const int k_begin = p.ws ? (int)blockIdx.y * p.k_per_split : 0;
  const int k_end = p.ws ? min(p.K, k_begin + p.k_per_split) : p.K;
  // Loads are unconditional (tail steps re-load the last step) so the
  // number of loads in flight is static and the compiler's vmcnt waits can
  // leave the younger PF-1 steps outstanding; the compute is what is
  // predicated on the step being live.
  const int nsteps = (k_end - k_begin) / kBK;
  auto kstep = [&](int st) { return k_begin + min(st, nsteps - 1) * kBK; };
  // prologue: steps 0..PF-1 in flight, step 0 staged
#pragma unroll
  for (int u = 0; u < PF; ++u) load_step(u, kstep(u));
  store_step(0, 0);
  __syncthreads();
  for (int s0 = 0; s0 < nsteps; s0 += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int st = s0 + u;
      const bool live = st < nsteps;  // uniform over the block
      const int buf = (PF == 1) ? (st & 1) : (u & 1);
      if (PF == 1) load_step(0, kstep(st + 1));
      v4u ah[TJ], al[TJ], bh[TI], bl[TI];
      if (live) {
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          const int off = (wn * (kBN / WN) + j * 16 + fr16) * kLDK + fk;
          ah[j] = ld16(&sWh[buf][off]);
          al[j] = ld16(&sWl[buf][off]);
        }
#pragma unroll
        for (int i = 0; i < TI; ++i) {
          const int off = (wm * (BM / WM) + i * 16 + fr16) * kLDK + fk;
          bh[i] = ld16(&sXh[buf][off]);
          bl[i] = ld16(&sXl[buf][off]);
        }
      }
      // slot u (step st, already in LDS) refills with step st + PF
      if (PF > 1) load_step(u, kstep(st + PF));
      if (live) {
#pragma unroll
        for (int j = 0; j < TJ; ++j)
#pragma unroll
          for (int i = 0; i < TI; ++i) acc[j][i] = x3_16(ah[j], al[j], bh[i], bl[i], acc[j][i]);
      }
      if (st + 1 < nsteps) store_step((u + 1) % PF, buf ^ 1);
      __syncthreads();
    }
  }

  // lane holds output channels nb..nb+3 of pixel m
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int nb = n0 + wn * (kBN / WN) + j * 16 + (lane >> 4) * 4;
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const int m = m0 + wm * (BM / WM) + i * 16 + fr16;
      if (m >= p.M) continue;
      const f32x4 a = acc[j][i];
      if (p.ws) {
        *reinterpret_cast<f32x4*>(p.ws + ((size_t)blockIdx.y * p.M + m) * p.N + nb) = a;
      } else if constexpr (SPLIT) {
        const f32x4 r = f32x4{fmaxf(a[0], 0.f), fmaxf(a[1], 0.f), fmaxf(a[2], 0.f), fmaxf(a[3], 0.f)};
        v2u h, l;
        split4(r, h, l);
        *reinterpret_cast<v2u*>(p.z_hi + (size_t)m * kBN + nb) = h;
        *reinterpret_cast<v2u*>(p.z_lo + (size_t)m * kBN + nb) = l;
      } else {
        *reinterpret_cast<f32x4*>(p.y + (size_t)m * p.ldy + nb) = a;
      }
    }
  }
}

// split-K combine: out[m][n..n+3] = epi(sum_s ws[s][m][n..n+3] (+ bias))
template <bool SPLIT>
__global__ void __launch_bounds__(256) x3_splitk_reduce_kernel(X3Conv1x1Params p, int splits) {
  const int n4 = p.N / 4;
  const size_t total = (size_t)p.M * n4;
  for (size_t q = blockIdx.x * 256ull + threadIdx.x; q < total; q += (size_t)gridDim.x * 256) {
    const int m = (int)(q / n4), nb = (int)(q % n4) * 4;
    f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f};
    if (SPLIT) a = ldf4(p.out_bias + nb);
    for (int s = 0; s < splits; ++s) a += ldf4(p.ws + ((size_t)s * p.M + m) * p.N + nb);
    if constexpr (SPLIT) {
      const f32x4 r = f32x4{fmaxf(a[0], 0.f), fmaxf(a[1], 0.f), fmaxf(a[2], 0.f), fmaxf(a[3], 0.f)};
      v2u h, l;
      split4(r, h, l);
      *reinterpret_cast<v2u*>(p.z_hi + (size_t)m * kBN + nb) = h;
      *reinterpret_cast<v2u*>(p.z_lo + (size_t)m * kBN + nb) = l;
    } else {
      *reinterpret_cast<f32x4*>(p.y + (size_t)m * p.ldy + nb) = a;
    }
  }
}

// ---- K8x (ws): warp-specialised persistent 1x1 for the big dense layers ----
// The tiled kernel above runs every phase of a K step in lockstep (global
// loads -> BN/ReLU/split VALU -> LDS -> MFMA -> barrier), so per SIMD the MFMA
// and the conversion VALU take turns and a block's loads are exposed every
// step (MI355X, 56x56 K=256 bs128: MFMA 19% busy, ~3.1 TB/s).  Here a block
// of 8 waves (one per CU) splits the work by role:
//   * waves 0-3 (consumers) own a 64 x 64 quarter of the 128-pixel x 128-
//     channel tile: 2 x 2 blocks of 32x32x16 MFMA, 24 per K step (768 cycles),
//     operands read from the LDS stage of the step;
//   * waves 4-7 (producers) keep PF K steps of X in flight in registers,
//     apply BN1+ReLU and the hi/lo split to one step per iteration into the
//     LDS stage two steps ahead, and copy the W hi/lo slices with LDS-DMA
//     (global_load_lds) S-1 steps ahead;
// so the conversion of step q+1 runs on the same SIMDs as the MFMAs of step
// q, and the only per-step synchronisation is one raw s_barrier (counted
// vmcnt: the younger X loads and W copies stay in flight across it).
// A block walks a contiguous run of pixels (whole 16-pixel units: every
// block moves the same bytes), the K steps of its consecutive tiles form one
// flat stream, so the pipeline never drains between tiles.
// LDS stage = X hi|lo + W hi|lo, each [128 rows][32 bf16] with the 16-B
// chunks XOR-swizzled by (row >> 2) & 3 (conflict-free b128 reads by 16
// consecutive rows).
constexpr int kWsS = 4;                          // LDS stages
constexpr int kWsPlane = 128 * kBK * 2;          // 8 KB: one [128][32] bf16 plane
constexpr int kWsStage = 4 * kWsPlane;           // Xh Xl Wh Wl
constexpr int kLdsWs = kWsS * kWsStage + 4 * 8192;  // 128 KB stages + 4 x 8 KB epilogue slabs = 160 KB

struct X3WsParams {
  X3Conv1x1Params c;
  int units_per_block;  // 16-pixel units per block
  int tile_rows;        // rows per tile (<= 128): a block's run split into equal tiles
};

// s_waitcnt immediates for gfx9-family (vmcnt 6 bits split [3:0]+[15:14],
// expcnt [6:4], lgkmcnt [11:8]); as a builtin (not inline asm) the
// compiler's own wait insertion knows the wait happened
constexpr int ws_vmcnt(int n) { return (((n >> 4) & 3) << 14) | (0xF << 8) | (7 << 4) | (n & 15); }
constexpr int ws_vmcnt_lgkm0(int n) { return (((n >> 4) & 3) << 14) | (7 << 4) | (n & 15); }

// raw s_barrier (no implicit vmcnt(0)) that the compiler may not move LDS
// accesses across; the caller issues the s_waitcnt it needs first
__device__ __forceinline__ void ws_barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ int ws_chunk(int row, int c) { return row * 64 + ((c ^ ((row >> 2) & 3)) << 4); }

// kWsPF: X steps in flight in the producers' registers
template <int kWsPF>
__global__ void __launch_bounds__(512, 1) x3_conv1x1_ws_kernel(X3WsParams wp) {
  extern __shared__ __attribute__((aligned(16))) uint8_t ldsw[];
  const X3Conv1x1Params& p = wp.c;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int u0 = blockIdx.x * wp.units_per_block;
  const int mbeg = 16 * u0;
  const int mend = min(p.M, 16 * (u0 + wp.units_per_block));
  if (mbeg >= mend) return;
  const int nst = p.K / kBK;
  const int TR = wp.tile_rows;
  const int ntiles = (mend - mbeg + TR - 1) / TR;
  const int Q = ntiles * nst;  // K steps of this block
  const int Qp = (Q + kWsPF - 1) / kWsPF * kWsPF;  // both roles run Qp barrier rounds

  if (wave >= 4) {
    // ------------------------------ producer ------------------------------
    const int pt = tid - 256, pw = wave - 4;
    const int pj = pt & 7, prow = pt >> 3;  // X: rows prow + 32i, k offset 4 pj
    const ptrdiff_t lo_off = p.w_lo - p.w_hi;
    f32x4 xr[kWsPF][4], xs[kWsPF], xt[kWsPF];
    // step q -> (tile, k0); q past the end re-loads the last step (static
    // vmcnt).  BN1 scale/shift ride with the X slot: an LDS copy would be
    // read after the W DMA, and the compiler orders every LDS read after all
    // in-flight LDS-DMA (vmcnt(0)), which would drain the pipeline.
    // K steps of a tile run in a block-rotated order: at any moment the blocks
    // then read different column offsets of their X rows (all blocks on the
    // same offset would camp on a subset of the HBM channels)
    const int rot = (int)(blockIdx.x % (unsigned)nst);
    auto kofs = [&](int ks) { ks += rot; return (ks >= nst ? ks - nst : ks) * kBK; };
    auto issue_x = [&](int q, int slot) {
      q = min(q, Q - 1);
      const int tile = q / nst, k0 = kofs(q - tile * nst);
      xs[slot] = ldf4(p.in_scale + k0 + 4 * pj);
      xt[slot] = ldf4(p.in_bias + k0 + 4 * pj);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int tb = mbeg + tile * TR;
        const int m = min(tb + prow + 32 * i, min(mend, tb + TR) - 1);
        xr[slot][i] = ldf4(p.x + (size_t)m * p.ldx + k0 + 4 * pj);
      }
    };
    // W hi/lo slice of step q -> stage q % S: 16 x 1 KB DMA, 4 per producer wave
    auto issue_w = [&](int q) {
      q = min(q, Q - 1);
      const int k0 = kofs(q % nst);
      uint8_t* st = ldsw + (q % kWsS) * kWsStage + 2 * kWsPlane;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ii = 4 * pw + i, plane = ii >> 3, rb = ii & 7;
        const int row = 16 * rb + (lane >> 2), c = (lane & 3) ^ ((row >> 2) & 3);
        const uint16_t* src = p.w_hi + (plane ? lo_off : 0) + (size_t)row * p.K + k0 + 8 * c;
        __builtin_amdgcn_global_load_lds((const void*)src, (void*)(st + plane * kWsPlane + rb * 1024), 16, 0, 0);
      }
    };
    auto write_x = [&](int q, int slot) {
      const int qq = min(q, Q - 1);
      const int tile = qq / nst;
      uint8_t* st = ldsw + (q % kWsS) * kWsStage;
      const f32x4 sc = xs[slot], sb = xt[slot];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = prow + 32 * i;
        const bool ok = row < TR && mbeg + tile * TR + row < mend;
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = ok ? fmaxf(xr[slot][i][e] * sc[e] + sb[e], 0.f) : 0.f;
        v2u h, l;
        split4(v, h, l);
        const int off = ws_chunk(row, pj >> 1) + (pj & 1) * 8;
        *reinterpret_cast<v2u*>(st + off) = h;
        *reinterpret_cast<v2u*>(st + kWsPlane + off) = l;
      }
    };
    // prologue: X steps 0..PF-1, W steps 0..S-3, step 0 staged; then the
    // steady-state issue of "iteration -1" (W step S-2, X step PF)
#pragma unroll
    for (int s = 0; s < kWsPF; ++s) issue_x(s, s);
    for (int s = 0; s <= kWsS - 3; ++s) issue_w(s);
    __builtin_amdgcn_s_waitcnt(ws_vmcnt(0));
    write_x(0, 0);
    issue_w(kWsS - 2);
    __builtin_amdgcn_sched_barrier(0);
    issue_x(kWsPF, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    ws_barrier();  // B0
    // iteration q (consumers on step q): stage step q+1's X, DMA W of step
    // q+S-1, refill the X register slot with step q+1+PF, then wait for W of
    // step q+1 before the barrier.  vmcnt retires in issue order, so the W
    // copies go out BEFORE the X loads of their iteration: the W wait then
    // only drains X steps up to q+1, and PF X steps stay in flight across
    // the barrier (with X first, every W wait also drained the X loads
    // issued beside it, which held the X stream to two steps in flight
    // whatever PF was: 3.6 TB/s instead of the ~5.8 TB/s a plain persistent
    // read of the same tiles reaches, profiles/r2_read_pattern_probe.log).
    // 10 ops per iteration: 4 W copies, then 6 X-slot loads.
    // Qp steps (a multiple of PF: no early exit out of the unrolled body,
    // whose merge would make the compiler's own wait insertion drain vmcnt)
    for (int q0 = 0; q0 < Qp; q0 += kWsPF) {
#pragma unroll
      for (int u = 0; u < kWsPF; ++u) {
        const int q = q0 + u;
        const int slot = (u + 1) % kWsPF;
        // X of step q+1 closed iteration q-PF: 10 (PF-1) younger ops
        __builtin_amdgcn_s_waitcnt(ws_vmcnt(10 * (kWsPF - 1)));
        __builtin_amdgcn_sched_barrier(0);
        write_x(q + 1, slot);
        issue_w(q + kWsS - 1);
        __builtin_amdgcn_sched_barrier(0);  // keep the W copies ahead of the X loads
        issue_x(q + 1 + kWsPF, slot);
        // W of step q+1 went out S-2 = 2 iterations back, ahead of that
        // iteration's 6 X loads: 6 + 2 x 10 younger ops
        __builtin_amdgcn_s_waitcnt(ws_vmcnt_lgkm0(6 + 10 * (kWsS - 2)));
        ws_barrier();  // B(q+1)
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA into LDS after the block ends
    return;
  }

  // ------------------------------- consumer -------------------------------
  const int wm = wave & 1, wn = wave >> 1;  // 64-pixel half, 64-channel half
  const int col = lane & 31, h = lane >> 5;
  f32x16 acc[2][2];  // [channel block][pixel block]
  f32x4 ob[2][4];    // BN2 shift of this lane's 32 output channels
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int g = 0; g < 4; ++g) ob[a][g] = ldf4(p.out_bias + 64 * wn + 32 * a + 8 * g + 4 * h);
  ws_barrier();  // B0
  int tile = 0, ks = 0;
  for (int q = 0; q < Qp; ++q) {
    if (q >= Q) {  // padding rounds: keep the barrier count of the producers
      ws_barrier();
      continue;
    }
    if (ks == 0) {
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;
    }
    const uint8_t* st = ldsw + (q % kWsS) * kWsStage;
    v4u ah[2][2], al[2][2], bh[2][2], bl[2][2];  // [ksub][block]
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int xo = ws_chunk(64 * wm + 32 * b + col, 2 * kk + h);
        const int wo = ws_chunk(64 * wn + 32 * b + col, 2 * kk + h);
        bh[kk][b] = ld16(st + xo);
        bl[kk][b] = ld16(st + kWsPlane + xo);
        ah[kk][b] = ld16(st + 2 * kWsPlane + wo);
        al[kk][b] = ld16(st + 3 * kWsPlane + wo);
      }
    // pixel blocks wholly past the block's last row (the ragged last tile)
    // skip their MFMAs
    const int rv = min(TR, mend - (mbeg + tile * TR)) - 64 * wm;  // valid rows from this wave's first
    if (rv > 32) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b) acc[a][b] = x3_32(ah[kk][a], al[kk][a], bh[kk][b], bl[kk][b], acc[a][b]);
    } else if (rv > 0) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int a = 0; a < 2; ++a) acc[a][0] = x3_32(ah[kk][a], al[kk][a], bh[kk][0], bl[kk][0], acc[a][0]);
    }
    if (ks == nst - 1) {
      // epilogue through this wave's 8 KB LDS slab: per 32-pixel block, the
      // bias+ReLU+split 64-channel rows land as [32 px][64 ch] hi and lo
      // (16-B chunks XOR-swizzled by pixel), then leave as 16-B-per-lane
      // stores that cover whole 128-B lines of z (8 pixels per instruction)
      // instead of 32 scattered 16-B pieces
      uint8_t* slab = ldsw + kWsS * kWsStage + wave * 8192;
#pragma unroll
      for (int b = 0; b < 2; ++b) {
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const f32x4 bb = ob[a][g];
            const f32x4 r = f32x4{fmaxf(acc[a][b][4 * g] + bb[0], 0.f), fmaxf(acc[a][b][4 * g + 1] + bb[1], 0.f),
                                  fmaxf(acc[a][b][4 * g + 2] + bb[2], 0.f), fmaxf(acc[a][b][4 * g + 3] + bb[3], 0.f)};
            v2u hh, ll;
            split4(r, hh, ll);
            const int off = col * 128 + (((4 * a + g) ^ (col & 7)) << 4) + 8 * h;
            *reinterpret_cast<v2u*>(slab + off) = hh;
            *reinterpret_cast<v2u*>(slab + 4096 + off) = ll;
          }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int pass = 0; pass < 4; ++pass) {
          const int px = 8 * pass + (lane >> 3), c = lane & 7;
          const int off = px * 128 + ((c ^ (px & 7)) << 4);
          const v4u vh = ld16(slab + off), vl = ld16(slab + 4096 + off);
          const int m = mbeg + tile * TR + 64 * wm + 32 * b + px;
          if (32 * b + px < rv) {
            *reinterpret_cast<v4u*>(p.z_hi + (size_t)m * kBN + 64 * wn + 8 * c) = vh;
            *reinterpret_cast<v4u*>(p.z_lo + (size_t)m * kBN + 64 * wn + 8 * c) = vl;
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slab reads done before block b+1 rewrites it
      }
    }
    if (ks == nst - 1) {
      ks = 0;
      ++tile;
    } else {
      ++ks;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    ws_barrier();  // B(q+1): stage q is free
  }
}

// ============================================================================
// K9x: 3x3 conv 128 -> 32 (stride 1, pad 1) on the split bottleneck
// ============================================================================
constexpr int kC3 = 128, kTaps = 9;  // 32 output channels (growth) per conv
constexpr int kRing = 256;             // ring rows per plane (a band is 128 + 2(W+1) <= 242 rows)
constexpr int kMaxW3 = 56;

struct X3Conv3x3Params {
  const uint16_t* z_hi;  // [M][128] bf16
  const uint16_t* z_lo;
  const uint16_t* w_hi;  // bf16 MFMA fragments [tap 9][kq 4][kc 2][lane 64][8] (x3_w3_fragments)
  const uint16_t* w_lo;
  float* y;              // [M][ldy] fp32, offset to the layer's 32-channel slice
  int ldy, M, H, W;
  int tiles, tiles_per_block;
  // PART kernels: the band comes from the preceding 1x1's split-K partials
  // [splits][M][128] fp32 (z = relu(sum + bias), split hi/lo while staged)
  const float* part;
  const float* part_bias;
  int splits;
  uint32_t mag_hw, mag_w;  // ceil(2^32 / (H*W)), ceil(2^32 / W): division by multiply-high
};

// n / d and n % d for n < 2^24 via a multiply-high estimate and one correction
__device__ __forceinline__ int fast_divmod(int n, int d, uint32_t mag, int& rem) {
  int q = (int)__umulhi((uint32_t)n, mag);
  int r = n - q * d;
  if (r < 0) {
    --q;
    r += d;
  } else if (r >= d) {
    ++q;
    r -= d;
  }
  rem = r;
  return q;
}

// ---- K9x (v2): 64-pixel tiles, LDS-DMA band ring, one-round reduction ------
// 8 waves = 2 pixel halves (ph) x 4 input-channel quarters (kq): wave (ph, kq)
// computes the 32 output channels of 32 pixels over 32 input channels x 9
// taps, its hi/lo weight fragments (36 x 16 B) in registers for the whole
// persistent kernel.  A block walks a contiguous run of 64-pixel tiles:
//   * the band [m0-W-1, m0+64+W+1) lives in a 256-row LDS ring (512-B rows =
//     hi|lo planes, 16-B chunks XOR-swizzled by ring row: conflict-free
//     b128 reads by consecutive pixels); the 64 rows the NEXT tile adds are
//     written by global_load_lds (LDS-DMA, no VGPR staging, swizzle applied
//     on the source address) right after the tile starts, into ring rows the
//     current band does not use (64 + 2(W+1) + 64 <= 256), so the fetch
//     overlaps the whole MFMA phase;
//   * the 4 input-channel partials of each 32x32 output block are summed in
//     ONE balanced round: wave (ph, kq) owns output channels [8kq, 8kq+8) of
//     its 32 pixels; it writes its partials of the other three 8-channel
//     groups (3 x 1 KB) to the scratch, barrier, adds the three partials of
//     its own group and stores fp32 straight to HBM;
//   * the 4 reads of tap t+1 are issued before the 6 MFMAs of tap t.
// Two barriers per tile.
constexpr int kT2 = 64;
constexpr int kRowB = 2 * kC3 * 2;          // 512 B per ring row
constexpr int kScrSlot = 32 * 8;            // floats per (group, ph, source) slot: 32 px x 8 channels
constexpr int kLdsV2 = (kRing + 1) * kRowB + 4 * 2 * 3 * kScrSlot * 4;  // 131,584 + 24,576 B

// PART: small-M layers (bs1/bs8 at 14x14 and below, bs1 everywhere) whose
// 1x1 ran split-K: the band is summed from the fp32 partials, bias+ReLU'd
// and split while it is staged, which replaces the split-K reduce launch
// (one ~5 us launch per such layer, 28% of a bs1 forward).  Those layers have
// one or two tiles per block, so the synchronous staging costs no overlap.
template <bool PART = false>
__global__ void __launch_bounds__(512, 1) x3_conv3x3_v2_kernel(X3Conv3x3Params p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds2[];
  float* scr = reinterpret_cast<float*>(lds2 + (kRing + 1) * kRowB);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ph = wave & 1, kq = wave >> 1;
  const int W = p.W, HW = p.H * p.W;
  const int col = lane & 31, h = lane >> 5;

  // fragment-major weights: each load is the wave's 1 KB contiguous (lane
  // (h, col) = w[col][t][32kq + 16kc + 8h ..+8]).  From the plain [32][9][128]
  // layout every load touched 32 lines at 32 B each, and this prologue alone
  // took ~9 us per block (the whole bs1 kernel was ~12 us).
  v4u wh[kTaps][2], wl[kTaps][2];
#pragma unroll
  for (int t = 0; t < kTaps; ++t)
#pragma unroll
    for (int kc = 0; kc < 2; ++kc) {
      const size_t off = ((size_t)((t * 4 + kq) * 2 + kc) * 64 + lane) * 8;
      wh[t][kc] = ld16(p.w_hi + off);
      wl[t][kc] = ld16(p.w_lo + off);
    }

  const int t_begin = blockIdx.x * p.tiles_per_block;
  const int t_end = min(p.tiles, t_begin + p.tiles_per_block);
  if (t_begin >= t_end) return;

  if (tid < kRowB / 16) *reinterpret_cast<v4u*>(lds2 + kRing * kRowB + tid * 16) = v4u{0, 0, 0, 0};
  const ptrdiff_t lo_off = p.z_lo - p.z_hi;
  // rows [g0, g0+nrows) -> ring, two rows per wave-instruction (ring row of g0 even)
  auto dma_rows = [&](int g0, int nrows) {
    if constexpr (PART) {
      // (row, 8-channel chunk) items, three per thread per pass so that the
      // 6 x splits partial loads of a pass are in flight together; chunk c of
      // ring row pos lands in slot c ^ (pos & 15) of both planes, as the DMA
      // places it
      const int n = nrows * 16;
      const size_t sstride = (size_t)p.M * kC3;
      for (int i0 = tid; i0 < n; i0 += 3 * 512) {
        f32x4 a[3][2];
        const float* q[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const int it = min(i0 + 512 * j, n - 1);
          const int g = g0 + (it >> 4), c = it & 15;
          q[j] = p.part + (size_t)min(max(g, 0), p.M - 1) * kC3 + 8 * c;
          a[j][0] = ldf4(p.part_bias + 8 * c);
          a[j][1] = ldf4(p.part_bias + 8 * c + 4);
        }
#pragma unroll 4
        for (int sp = 0; sp < p.splits; ++sp) {
          f32x4 v[3][2];
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            v[j][0] = ldf4(q[j] + sp * sstride);
            v[j][1] = ldf4(q[j] + sp * sstride + 4);
          }
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            a[j][0] += v[j][0];
            a[j][1] += v[j][1];
          }
        }
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const int it = i0 + 512 * j;
          if (it >= n) break;
          const int g = g0 + (it >> 4), c = it & 15;
          const int pos = (g + W + 1) & (kRing - 1);
          uint32_t h0, l0, h1, l1, h2, l2, h3, l3;
          split2(fmaxf(a[j][0][0], 0.f), fmaxf(a[j][0][1], 0.f), h0, l0);
          split2(fmaxf(a[j][0][2], 0.f), fmaxf(a[j][0][3], 0.f), h1, l1);
          split2(fmaxf(a[j][1][0], 0.f), fmaxf(a[j][1][1], 0.f), h2, l2);
          split2(fmaxf(a[j][1][2], 0.f), fmaxf(a[j][1][3], 0.f), h3, l3);
          uint8_t* rp = lds2 + pos * kRowB + ((c ^ (pos & 15)) << 4);
          *reinterpret_cast<v4u*>(rp) = v4u{h0, h1, h2, h3};
          *reinterpret_cast<v4u*>(rp + 256) = v4u{l0, l1, l2, l3};
        }
      }
      return;
    }
    const int plane = (lane >> 4) & 1, j = lane & 15;
    for (int pr = wave; 2 * pr < nrows; pr += 8) {
      const int ga = g0 + 2 * pr;
      const int g = ga + (lane >> 5);
      const int pos = (g + W + 1) & (kRing - 1);
      const int gc = min(max(g, 0), p.M - 1);
      // plane select as an offset: a select between the two pointer fields
      // makes hipcc reload one from the kernarg segment per lane (a vector
      // load, whose vmcnt wait would drain the in-flight y stores)
      const uint16_t* src = p.z_hi + (plane ? lo_off : 0) + (size_t)gc * kC3 + ((j ^ (pos & 15)) << 3);
      const int pos0 = (ga + W + 1) & (kRing - 1);
      __builtin_amdgcn_global_load_lds((const void*)src, (void*)(lds2 + pos0 * kRowB), 16, 0, 0);
    }
  };
  dma_rows(t_begin * kT2 - W - 1, kT2 + 2 * (W + 1));

  for (int tile = t_begin; tile < t_end; ++tile) {
    const int m0 = tile * kT2;
    // B0: this band is in LDS everywhere and the scratch is free.  The vm
    // counter retires in issue order: [this band's DMA..., last tile's y
    // store], so vmcnt(1) waits for the DMA and leaves the store (an HBM
    // write round trip) in flight; the first tile has no store behind it.
    if (tile == t_begin) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(1) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (tile + 1 < t_end) dma_rows(m0 + kT2 + W + 1, kT2);

    const int m = m0 + 32 * ph + col;
    int r, xx;
    (void)fast_divmod(m, HW, p.mag_hw, r);
    const int yy = fast_divmod(r, W, p.mag_w, xx);
    const bool in = m < p.M;
    const bool up = in && yy > 0, dn = in && yy < p.H - 1, lf = xx > 0, rt = xx < W - 1;
    const int base = m + W + 1;
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    v4u bq[2][2][2];  // [tap parity][kc][plane]
    auto rd = [&](int t, int slot) {
      const int dy = t / 3 - 1, dx = t % 3 - 1;
      bool ok = dy < 0 ? up : (dy > 0 ? dn : in);
      if (dx < 0) ok = ok && lf;
      if (dx > 0) ok = ok && rt;
      const int row = ok ? ((base + dy * W + dx) & (kRing - 1)) : kRing;
      const uint8_t* rp = lds2 + row * kRowB;
      const int sw = row & 15;
#pragma unroll
      for (int kc = 0; kc < 2; ++kc) {
        const uint8_t* q = rp + (((4 * kq + 2 * kc + h) ^ sw) << 4);
        bq[slot][kc][0] = ld16(q);
        bq[slot][kc][1] = ld16(q + 256);
      }
    };
    rd(0, 0);
#pragma unroll
    for (int t = 0; t < kTaps; ++t) {
      // pin the order: tap t+1's 4 reads are issued before tap t's 6 MFMAs
      // (a scheduling fence, so the two tap buffers stay in distinct
      // registers), and each read's LDS latency hides behind a tap of MFMAs
      if (t + 1 < kTaps) rd(t + 1, (t + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int kc = 0; kc < 2; ++kc) acc = x3_32(wh[t][kc], wl[t][kc], bq[t & 1][kc][0], bq[t & 1][kc][1], acc);
    }
    // C layout (32x32): lane col = pixel, reg 4g+e -> channel 8g + 4h + e.
    // scratch slot (group g, ph, source kq != g) at index (g*2 + ph)*3 + (kq - g + 3) % 4
    auto slot = [&](int g, int src) {
      return scr + ((g * 2 + ph) * 3 + (src - g + 3) % 4) * kScrSlot + col * 8 + 4 * h;
    };
#pragma unroll
    for (int g = 0; g < 4; ++g)
      if (g != kq)
        *reinterpret_cast<f32x4*>(slot(g, kq)) = f32x4{acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]};
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // B1 (raw: the next band's DMA stays in flight)
    f32x4 o = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int g = 0; g < 4; ++g)
      if (g == kq) o = f32x4{acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]};
#pragma unroll
    for (int src = 0; src < 4; ++src)
      if (src != kq) o += *reinterpret_cast<const f32x4*>(slot(kq, src));
    if (in) *reinterpret_cast<f32x4*>(p.y + (size_t)m * p.ldy + 8 * kq + 4 * h) = o;
  }
}

// ============================================================================
// K11x: the whole dense layer in one kernel, z never leaves the CU
// ============================================================================
// K8x + K9x write the 128-channel bottleneck z (as hi/lo bf16 planes, 512 B a
// pixel) to HBM and read it back with a 2(W+1)-row halo per tile: at 56x56 x
// bs128 that is 205 MB written + 2 x 205 MB read per layer, and two launches.
// Here one persistent block (8 waves, one per CU) walks a contiguous run of
// 64-pixel tiles and produces z itself, straight into the 3x3's LDS ring:
//
//   for each tile t:  3x3 over band(t) = rows [m0-W-1, m0+64+W+1) of the ring
//                     1x1 for the 64 rows band(t+1) adds, written over the 64
//                     ring rows band(t+1) no longer needs
//
// so HBM sees only the layer's input X (read once) and its 32 output
// channels.  The ring is 192 rows (band <= 178 for W <= 56; the rows a 1x1
// chunk overwrites are always older than the next band, 2W < 127).
//
// 1x1 phase (64 pixels x 128 channels, K in 32-wide steps): wave (q1, ph) =
// output quarter x pixel half on 32x32x16 MFMAs.
//   * X: fp32 [64 px][32 k] steps by LDS-DMA (global_load_lds, one 1 KB piece
//     per wave per step) into a 4-deep stage ring, 16-B chunks XOR-swizzled
//     by pixel (conflict-free b128 reads); the first three steps of the next
//     chunk are issued before the 3x3 phase, whose MFMAs hide that HBM round
//     trip.  No VGPR staging: the waits are explicit vmcnt counts over a
//     static issue order (the compiler's own waits cannot see through
//     conditional or loop-carried register loads, and drained the prefetch
//     before every step in a register-staged first version).
//   * B operand: each lane reads its 8 fp32 of a k16 step, applies BN1+ReLU
//     (affine from LDS) and splits hi/lo in registers; 4 waves redo the
//     conversion of a fragment, which costs VALU slots the MFMAs leave idle
//     and saves a converted-tile LDS pass plus a barrier per step.
//   * A operand: BN2-folded W1 hi/lo fragments straight from L2 in a
//     fragment-major copy (1 KB per wave load), one step ahead.
//   * one barrier per step; epilogue: + bias, ReLU, hi/lo split, into the
//     ring rows (544-B row stride: each row's banks rotated two chunks from
//     the previous row's, see kRowF1).
//
// 3x3 phase: wave (kq, oh) = input-channel quarter x output half on 16x16x32
// MFMAs, so a wave's resident weights are 9 taps x 16 outputs x 32 inputs x
// hi/lo = 72 VGPRs (K9x's 32-output waves hold 144, which leaves no room for
// the 1x1 phase).  Operand reads roll two (tap, pixel-group) steps ahead.
// The 4 kq partials: lanes holding another wave's 4 channels write them to
// the owner's scratch slots (the owner its own share to a y-sum slot); the
// owners add and store y after the next 1x1 chunk's barriers.
//
// LDS: ring 197 x 544 B + scratch 24 KB + X stages 2 x 2 x 4 KB + BN1 affine
// 2 x 480 floats + y sums 8 KB = 160,160 B.
constexpr int kRingF = 192;
// physical ring row = logical + 1: [guard = logical -1 (mirrors 191)]
// [logical 0..191] [guard = logical 192 (mirrors 0)] [logical 193..195: zero]
constexpr int kZeroF = 194;             // a tap reading logical kZeroF + {-1, 0, 1} reads zeros
constexpr int kRingRowsF = kZeroF + 3;  // 197 physical rows
constexpr int kCvtF = 64 * 64;     // one plane of a converted X step: 64 px x 32 k bf16
constexpr int kPfF = 4;             // X steps in flight (registers)
constexpr int kMaxKF = 480;         // BN1 affine staged in LDS: K <= 480 (blocks 1-2)
constexpr int kScrF = 2 * 4 * 3 * 64 * 4;  // floats: [oh][owner][3 sources][px][4]
constexpr int kYsF = 2 * 4 * 4 * 64;  // floats: v1 owners' y sums [oh][owner][pg][px 16][4]
// v1 ring row stride: 512 B of z (hi | lo) + 32 B of padding, so row r's banks
// start 8 banks (two 16-B chunks) after row r-1's.  With that rotation the
// 3x3's ds_read_b128 lane groups ({0-3,12-15 | chunk c} + {20-27 | chunk c+1}
// over 16 consecutive rows) land on 16 distinct chunk slots for ANY first
// row; the XOR swizzle by (row & 15) it replaces cannot do that (a 2-way
// conflict whenever the group's first row is odd, ~10% of the 3x3's LDS time
// by SQ_LDS_BANK_CONFLICT).
constexpr int kRowF1 = kRowB + 32;
constexpr int kLdsF = kRingRowsF * kRowF1 + kScrF * 4 + 4 * kCvtF + 2 * kMaxKF * 4 + kYsF * 4;
static_assert(kLdsF <= 160 * 1024, "K11x LDS budget");
constexpr uint32_t kMagRingF = (uint32_t)((0x100000000ull + kRingF - 1) / kRingF);

struct X3FusedParams {
  const float* x;         // [M][ldx] fp32, the layer's first K channels
  const float* s1;        // [K] BN1 affine
  const float* t1;
  const uint16_t* w1_hi;  // [K/16][q1 4][lane 64][8] bf16 (x3_w1_fragments)
  const uint16_t* w1_lo;
  const float* b1;        // [128] BN2-folded bias
  const uint16_t* w2_hi;  // [tap 9][kq 4][oh 2][lane 64][8] bf16 (x3_w3f_fragments)
  const uint16_t* w2_lo;
  float* y;               // [M][ldy] fp32, offset to the layer's 32-channel slice
  int ldx, K, ldy, M, H, W;
  int tiles, tiles_per_block;
  uint32_t mag_hw, mag_w;
};

// NST = K / 32 (2..7): the k loop of a chunk is straight-line code, so the
// compiler's waits for the W1 fragments are exact (through a loop back edge
// it fell back to draining the whole counter every step).
// (A stagger of the two waves of each SIMD in the 1x1 chunk -- waves 4-7
// running a step's MFMAs before converting the next X step -- measured 5-20%
// slower at 56x56 and 28x28 in round 4 and was dropped.)
template <int NST>
__global__ void __launch_bounds__(512, 1) x3_dense_fused_kernel(X3FusedParams p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t ldsf[];
  uint8_t* const ring = ldsf;
  float* const scr = reinterpret_cast<float*>(ldsf + kRingRowsF * kRowF1);
  uint8_t* const cvt = ldsf + kRingRowsF * kRowF1 + kScrF * 4;             // [buf 2][plane 2][64 px][64 B]
  float* const bn = reinterpret_cast<float*>(cvt + 4 * kCvtF);            // s1 [kMaxKF] | t1 [kMaxKF]
  float* const ysum = bn + 2 * kMaxKF;                                     // [oh][owner][pg][16 px][4]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int W = p.W, HW = p.H * p.W;

  // 3x3 roles and resident weights: A[16oh + (lane&15)][tap t][32kq + 8(lane>>4) ..+8]
  const int kq = wave & 3, oh = wave >> 2;
  v4u w2h[kTaps], w2l[kTaps];
#pragma unroll
  for (int t = 0; t < kTaps; ++t) {
    const size_t off = ((size_t)((t * 4 + kq) * 2 + oh) * 64 + lane) * 8;
    w2h[t] = ld16(p.w2_hi + off);
    w2l[t] = ld16(p.w2_lo + off);
  }

  const int t_begin = blockIdx.x * p.tiles_per_block;
  const int t_end = min(p.tiles, t_begin + p.tiles_per_block);
  if (t_begin >= t_end) return;

  for (int i = tid; i < p.K; i += 512) {
    bn[i] = p.s1[i];
    bn[kMaxKF + i] = p.t1[i];
  }
  if (tid < 3 * kRowF1 / 16) *reinterpret_cast<v4u*>(ring + kZeroF * kRowF1 + tid * 16) = v4u{0, 0, 0, 0};
  __syncthreads();

  // ---- 1x1 phase -----------------------------------------------------------
  const int q1 = wave & 3, ph = wave >> 2;
  const int col = lane & 31, hh = lane >> 5;
  constexpr int nst = NST;
  // X: every thread loads one float4 of a step (pixel cpx, k 4cj..4cj+3) kPfF
  // steps ahead into registers, applies BN1 + ReLU, splits it and writes the
  // hi/lo halves into the step's shared bf16 stage; the conversion is done
  // once per element (a per-wave conversion of the B fragments repeated it
  // in all 4 output-quarter waves and made the kernel VALU-bound).  All
  // global loads are plain loads in a static order (fully unrolled chunk),
  // so the compiler's counted waits keep kPfF steps in flight.
  const int cpx = tid >> 3, cj = tid & 7;
  f32x4 xr[kPfF];
  const float* xrow = p.x;
  auto xload = [&](int slot, int st) { xr[slot] = ldf4(xrow + min(st, nst - 1) * 32); };
  auto prime = [&](int g0) {
    xrow = p.x + (size_t)min(max(g0 + cpx, 0), p.M - 1) * p.ldx + 4 * cj;
#pragma unroll
    for (int u = 0; u < kPfF; ++u) xload(u, u);
  };
  // stage [buf][plane][64 px][64 B]: 16-B chunk c (k 8c..8c+7) of pixel px at
  // slot c ^ ((px >> 2) & 3) (conflict-free b128 reads by 16 consecutive pixels)
  const int cw_off = cpx * 64 + (((cj >> 1) ^ ((cpx >> 2) & 3)) << 4) + 8 * (cj & 1);
  auto convert = [&](int slot, int buf, int st) {
    const f32x4 sv = *reinterpret_cast<const f32x4*>(bn + st * 32 + 4 * cj);
    const f32x4 tv = *reinterpret_cast<const f32x4*>(bn + kMaxKF + st * 32 + 4 * cj);
    const f32x4 v = bn_relu4(xr[slot], sv, tv);
    v2u h, l;
    split4(v, h, l);
    uint8_t* q = cvt + buf * 2 * kCvtF + cw_off;
    *reinterpret_cast<v2u*>(q) = h;
    *reinterpret_cast<v2u*>(q + kCvtF) = l;
  };
  v4u a1[2][2][2];  // [step parity][kc][plane]
  // buffer loads: one lane-constant VGPR offset + the step's offset in an SGPR
  const auto w1h = __builtin_amdgcn_make_buffer_rsrc((void*)p.w1_hi, (short)0, p.K * 256, 0x00020000);
  const auto w1l = __builtin_amdgcn_make_buffer_rsrc((void*)p.w1_lo, (short)0, p.K * 256, 0x00020000);
  const int w1v = (q1 * 64 + lane) * 16;
  auto wload = [&](int slot, int st) {
    st = min(st, nst - 1);
#pragma unroll
    for (int kc = 0; kc < 2; ++kc) {
      a1[slot][kc][0] = __builtin_amdgcn_raw_buffer_load_b128(w1h, w1v, (2 * st + kc) * 4096, 0);
      a1[slot][kc][1] = __builtin_amdgcn_raw_buffer_load_b128(w1l, w1v, (2 * st + kc) * 4096, 0);
    }
  };
  const int bpx = 32 * ph + col;  // this lane's B column (pixel of the chunk)
  const int bsw = (bpx >> 2) & 3;
  const int br_off[2] = {bpx * 64 + ((hh ^ bsw) << 4), bpx * 64 + (((2 + hh) ^ bsw) << 4)};  // chunks 2kc + hh
  // z rows [g0, g0 + nrows) -> ring.  The caller primed the chunk's X and
  // issued W(0).  Step st: W(st+1) and X(st+1+kPfF) go out, step st+1 is
  // converted into the other stage buffer while step st's MFMAs run on this
  // one; one barrier per step.
  auto z_chunk = [&](int g0, int nrows) {
    f32x16 acc;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 b = ldf4(p.b1 + 32 * q1 + 8 * g + 4 * hh);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[4 * g + e] = b[e];
    }
    convert(0, 0, 0);
    xload(0, kPfF);
    __syncthreads();
#pragma unroll
    for (int st = 0; st < nst; ++st) {
      wload((st + 1) & 1, st + 1);
      auto next = [&]() {
        if (st + 1 < nst) {
          convert((st + 1) % kPfF, (st + 1) & 1, st + 1);
          xload((st + 1) % kPfF, st + 1 + kPfF);
        }
      };
      auto mma = [&]() {
        const uint8_t* cb = cvt + (st & 1) * 2 * kCvtF;
#pragma unroll
        for (int kc = 0; kc < 2; ++kc) {
          const uint8_t* q = cb + br_off[kc];
          acc = x3_32(a1[st & 1][kc][0], a1[st & 1][kc][1], ld16(q), ld16(q + kCvtF), acc);
        }
      };
      next();
      mma();
      __syncthreads();
    }
    // C (32x32): lane col = pixel, reg 4g+e -> channel 32q1 + 8g + 4hh + e
    if (bpx < nrows) {
      int pos;
      (void)fast_divmod(g0 + bpx + W + 1, kRingF, kMagRingF, pos);
      // physical row pos + 1; logical rows 0 and 191 also go to the guard
      // rows 193 / 0 (same bank rotation: 192 rows x 8 banks is a multiple of 64)
      uint8_t* rp = ring + (pos + 1) * kRowF1 + 8 * hh;
      const int mirror = pos == 0 ? kRingF * kRowF1 : (pos == kRingF - 1 ? -kRingF * kRowF1 : 0);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        f32x4 r;
#pragma unroll
        for (int e = 0; e < 4; ++e) r[e] = fmaxf(acc[4 * g + e], 0.f);
        v2u h, l;
        split4(r, h, l);
        uint8_t* q = rp + ((4 * q1 + g) << 4);
        *reinterpret_cast<v2u*>(q) = h;
        *reinterpret_cast<v2u*>(q + 256) = l;
        if (mirror) {
          *reinterpret_cast<v2u*>(q + mirror) = h;
          *reinterpret_cast<v2u*>(q + mirror + 256) = l;
        }
      }
    }
  };

  // prologue: band(t_begin) in 64-row chunks
  {
    const int b0 = t_begin * kT2 - W - 1, b1 = t_begin * kT2 + kT2 + W + 1;
    for (int g0 = b0; g0 < b1; g0 += 64) {
      prime(g0);
      wload(0, 0);
      z_chunk(g0, min(64, b1 - g0));
    }
  }

  const int c4 = lane >> 4;
  for (int tile = t_begin; tile < t_end; ++tile) {
    const int m0 = tile * kT2;
    __syncthreads();  // B0: the ring holds band(tile); the scratch is free
    // this iteration's chunk: its first X steps and W(0) go out now and land
    // while the 3x3 runs (issued and consumed in one tile iteration: a load
    // carried round the loop is one the compiler's waits cannot follow)
    if (tile + 1 < t_end) {
      prime(m0 + kT2 + W + 1);
      wload(0, 0);
    }

    // ---- 3x3 phase ----
    {
    // Per pixel group pg (16 consecutive pixels; the host requires W >= 16,
    // so +16 pixels wraps an image row at most once) and tap
    // row dy: the band row R[pg][dy] (logical 0..191), or the zero rows for
    // an invalid dy; tap (dy, dx) reads logical row R + dx, which the guard
    // rows (logical -1 and 192) keep in range without a second wrap.  Per
    // (tap, pg) step that leaves: add dx, swizzle, address, and for dx != 0
    // a select of the zero row: ~4 VALU beside 3 MFMAs (the first version's
    // ~15 made the phase issue-bound, not MFMA-bound).
    int R[4][3];
    bool lfm[4], rtm[4];
    {
      const int m = m0 + (lane & 15);
      int r, xx, pm;
      (void)fast_divmod(m, HW, p.mag_hw, r);
      int yy = fast_divmod(r, W, p.mag_w, xx);
      (void)fast_divmod(m + W + 1, kRingF, kMagRingF, pm);
#pragma unroll
      for (int pg = 0; pg < 4; ++pg) {
        if (pg) {
          xx += 16;
          if (xx >= W) {
            xx -= W;
            if (++yy == p.H) yy = 0;
          }
          pm += 16;
          if (pm >= kRingF) pm -= kRingF;
        }
        const bool in = m + 16 * pg < p.M;
        const int rm = pm - W, rp = pm + W;
        R[pg][0] = (in && yy > 0) ? (rm < 0 ? rm + kRingF : rm) : kZeroF;
        R[pg][1] = in ? pm : kZeroF;
        R[pg][2] = (in && yy < p.H - 1) ? (rp >= kRingF ? rp - kRingF : rp) : kZeroF;
        lfm[pg] = xx > 0;
        rtm[pg] = xx < W - 1;
      }
    }
    f32x4 acc[4];
#pragma unroll
    for (int pg = 0; pg < 4; ++pg) acc[pg] = f32x4{0.f, 0.f, 0.f, 0.f};
    // operand reads roll over the 36 (tap, pixel group) steps kLead steps
    // ahead of the MFMAs ((kLead+1) x 8 VGPRs instead of whole taps)
    constexpr int kLead = 3;
    v4u bq[kLead + 1][2];
    const int chunk16 = (4 * kq + (lane >> 4)) << 4;
    auto rd = [&](int step) {
      const int t = step >> 2, pg = step & 3;
      const int dy = t / 3, dx = t % 3 - 1;
      const int a = R[pg][dy] + dx;  // logical row, -1 .. 192 (or a zero row)
      int off = a * kRowF1 + chunk16;
      if (dx < 0 && !lfm[pg]) off = kZeroF * kRowF1;
      if (dx > 0 && !rtm[pg]) off = kZeroF * kRowF1;
      const uint8_t* q = ring + kRowF1 + off;  // physical row = logical + 1
      bq[step % (kLead + 1)][0] = ld16(q);
      bq[step % (kLead + 1)][1] = ld16(q + 256);
    };
#pragma unroll
    for (int step = 0; step < kLead; ++step) rd(step);
#pragma unroll
    for (int step = 0; step < 4 * kTaps; ++step) {
      if (step + kLead < 4 * kTaps) rd(step + kLead);
      __builtin_amdgcn_sched_barrier(0);
      const int t = step >> 2, pg = step & 3;
      acc[pg] = x3_16(w2h[t], w2l[t], bq[step % (kLead + 1)][0], bq[step % (kLead + 1)][1], acc[pg]);
    }
    // C (16x16): lane (lane&15) = pixel of group pg, reg e -> channel 16oh + 4c + e,
    // c = lane>>4; owner of channels 16oh + 4c .. +4 is wave (kq = c, oh), whose
    // lanes 16c .. 16c+15 hold their own share and add the other three
    // C (16x16) lanes of another wave's 4 channels go to that owner's
    // scratch slots, the owner's own share to its y-sum slot: no 3x3 result
    // stays in registers through the 1x1 chunk
    if (c4 != kq) {
      float* sw = scr + ((oh * 4 + c4) * 3 + (kq - c4 + 3) % 4) * 256 + (lane & 15) * 4;
#pragma unroll
      for (int pg = 0; pg < 4; ++pg) *reinterpret_cast<f32x4*>(sw + pg * 64) = acc[pg];
    } else {
      float* yw = ysum + (oh * 4 + kq) * 256 + (lane & 15) * 4;
#pragma unroll
      for (int pg = 0; pg < 4; ++pg) *reinterpret_cast<f32x4*>(yw + pg * 64) = acc[pg];
    }
    }

    // ---- 1x1 phase: the 64 rows band(tile+1) adds; its first barrier
    // publishes the partials (no exchange barrier of its own), its last one
    // makes them readable by the owners below ----
    if (tile + 1 < t_end) {
      const int g0 = m0 + kT2 + W + 1;
      z_chunk(g0, kT2);
    } else {
      __syncthreads();
    }
    // owners: own share + the three partials -> y (the stores are issued
    // after the chunk's last W1 / X wait and long retired by the next one)
    if (c4 == kq) {
      const float* sr = scr + (oh * 4 + kq) * 3 * 256 + (lane & 15) * 4;
      const float* yr = ysum + (oh * 4 + kq) * 256 + (lane & 15) * 4;
#pragma unroll
      for (int pg = 0; pg < 4; ++pg) {
        f32x4 v = *reinterpret_cast<const f32x4*>(yr + pg * 64);
#pragma unroll
        for (int src = 0; src < 3; ++src) v += *reinterpret_cast<const f32x4*>(sr + src * 256 + pg * 64);
        const int m = m0 + 16 * pg + (lane & 15);
        if (m < p.M) *reinterpret_cast<f32x4*>(p.y + (size_t)m * p.ldy + 16 * oh + 4 * kq) = v;
      }
    }
  }
  // the last chunk's clamped tail DMAs (and, ablated, a primed chunk) must
  // land before this workgroup's LDS can be handed to the next one
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---- K11x v3: the next chunk's 1x1 interleaved into this tile's 3x3 --------
// v1 runs each tile as two serial phases: the 3x3 (MFMA + ring reads, nothing
// else in flight) and then the next chunk's 1x1, whose 32-wide K steps are
// too short to hide their own barrier, LDS round trip and conversion VALU
// (per tile at K=224: 1x1 6.7k + 3x3 5.1k + exchange 3.4k cycles against a
// 6.1k-cycle MFMA floor, profiles/r3_fused_dense_layer.md; 36% MFMA busy).
//
// Both phases read data that is stable for the whole tile: the 3x3 reads only
// band(t), which the 1x1 of chunk t+1 does not touch until its epilogue.  So
// v3 walks the chunk's K steps and deals the 36 (tap, pixel-group) steps of
// the 3x3 out over them: K step st of the chunk carries its own 6 MFMAs
// 32x32x16, the conversion of step st+1, and 36/NST 3x3 steps (3 MFMAs
// 16x16x32 each, operands rolled kLead steps ahead across the barriers).  A
// barrier interval then holds ~440 cycles of MFMA per wave at K=224 instead
// of 192, and the 3x3's MFMAs cover the step's barrier and its conversion.
// The epilogue (z -> ring rows of band(t+1)) waits for one barrier after the
// last 3x3 read (those rows overwrite band(t)'s oldest rows); the owners sum
// the 3x3 partials of tile t during the first K step of tile t+1.  Barriers
// per tile: NST + 1 (v1: NST + 2 and a serial 3x3 phase).
//
// X is loaded across chunks: once a register slot's last step of chunk t+1
// is converted it takes the first steps of chunk t+2, so the chunk's first
// conversion (before barrier B) finds its X landed.  Same LDS layout and
// roles as v1, plus the 1x1 bias (512 B) from LDS.  The first tile's band
// and a block's last tile (no next chunk) run v1's serial schedule.
constexpr int kLdsF3 = kLdsF + 128 * 4;
static_assert(kLdsF3 <= 160 * 1024, "K11x v3 LDS budget");

template <int NST>
__global__ void __launch_bounds__(512, 1) x3_dense_fused3_kernel(X3FusedParams p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t ldsf[];
  uint8_t* const ring = ldsf;
  float* const scr = reinterpret_cast<float*>(ldsf + kRingRowsF * kRowF1);
  uint8_t* const cvt = ldsf + kRingRowsF * kRowF1 + kScrF * 4;  // [buf 2][plane 2][64 px][64 B]
  float* const bn = reinterpret_cast<float*>(cvt + 4 * kCvtF);   // s1 [kMaxKF] | t1 [kMaxKF]
  float* const ysum = bn + 2 * kMaxKF;                            // [oh][owner][pg][16 px][4]
  float* const bias = ysum + kYsF;                                // b1 [128]
  auto bar = [](int) { __syncthreads(); };  // argument: the barrier's index within a tile
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int W = p.W, HW = p.H * p.W;

  // 3x3 roles and resident weights (as v1)
  const int kq = wave & 3, oh = wave >> 2;
  v4u w2h[kTaps], w2l[kTaps];
#pragma unroll
  for (int t = 0; t < kTaps; ++t) {
    const size_t off = ((size_t)((t * 4 + kq) * 2 + oh) * 64 + lane) * 8;
    w2h[t] = ld16(p.w2_hi + off);
    w2l[t] = ld16(p.w2_lo + off);
  }

  const int t_begin = blockIdx.x * p.tiles_per_block;
  const int t_end = min(p.tiles, t_begin + p.tiles_per_block);
  if (t_begin >= t_end) return;

  for (int i = tid; i < p.K; i += 512) {
    bn[i] = p.s1[i];
    bn[kMaxKF + i] = p.t1[i];
  }
  if (tid < 128) bias[tid] = p.b1[tid];
  if (tid < 3 * kRowF1 / 16) *reinterpret_cast<v4u*>(ring + kZeroF * kRowF1 + tid * 16) = v4u{0, 0, 0, 0};
  __syncthreads();

  // ---- 1x1 roles (as v1): wave (q1, ph) = output quarter x pixel half ----
  const int q1 = wave & 3, ph = wave >> 2;
  const int col = lane & 31, hh = lane >> 5;
  constexpr int nst = NST;
  constexpr int PF = NST < kPfF ? NST : kPfF;  // X register slots; step s of a chunk uses slot s % PF
  // conversion role: pixel cpx, k 4cj..4cj+3 of a step
  const int cpx = tid >> 3, cj = tid & 7;
  f32x4 xr[PF];
  auto xptr = [&](int g0) { return p.x + (size_t)min(max(g0 + cpx, 0), p.M - 1) * p.ldx + 4 * cj; };
  auto xload = [&](int slot, const float* base, int st) { xr[slot] = ldf4(base + st * 32); };
  const int cw_off = cpx * 64 + (((cj >> 1) ^ ((cpx >> 2) & 3)) << 4) + 8 * (cj & 1);
  auto convert = [&](int slot, int buf, int st) {
    const f32x4 sv = *reinterpret_cast<const f32x4*>(bn + st * 32 + 4 * cj);
    const f32x4 tv = *reinterpret_cast<const f32x4*>(bn + kMaxKF + st * 32 + 4 * cj);
    const f32x4 v = bn_relu4(xr[slot], sv, tv);
    v2u h, l;
    split4(v, h, l);
    uint8_t* q = cvt + buf * 2 * kCvtF + cw_off;
    *reinterpret_cast<v2u*>(q) = h;
    *reinterpret_cast<v2u*>(q + kCvtF) = l;
  };
  v4u a1[2][2][2];  // [step parity][kc][plane]
  const auto w1h = __builtin_amdgcn_make_buffer_rsrc((void*)p.w1_hi, (short)0, p.K * 256, 0x00020000);
  const auto w1l = __builtin_amdgcn_make_buffer_rsrc((void*)p.w1_lo, (short)0, p.K * 256, 0x00020000);
  const int w1v = (q1 * 64 + lane) * 16;
  auto wload = [&](int slot, int st) {
#pragma unroll
    for (int kc = 0; kc < 2; ++kc) {
      a1[slot][kc][0] = __builtin_amdgcn_raw_buffer_load_b128(w1h, w1v, (2 * st + kc) * 4096, 0);
      a1[slot][kc][1] = __builtin_amdgcn_raw_buffer_load_b128(w1l, w1v, (2 * st + kc) * 4096, 0);
    }
  };
  const int bpx = 32 * ph + col;  // this lane's B column (pixel of the chunk)
  const int bsw = (bpx >> 2) & 3;
  const int br_off[2] = {bpx * 64 + ((hh ^ bsw) << 4), bpx * 64 + (((2 + hh) ^ bsw) << 4)};
  auto bias_acc = [&]() {
    f32x16 acc;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 b = *reinterpret_cast<const f32x4*>(bias + 32 * q1 + 8 * g + 4 * hh);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[4 * g + e] = b[e];
    }
    return acc;
  };
  auto mma1 = [&](f32x16& acc, int st) {
    const uint8_t* cb = cvt + (st & 1) * 2 * kCvtF;
#pragma unroll
    for (int kc = 0; kc < 2; ++kc) {
      const uint8_t* q = cb + br_off[kc];
      acc = x3_32(a1[st & 1][kc][0], a1[st & 1][kc][1], ld16(q), ld16(q + kCvtF), acc);
    }
  };
  // the same with the B fragments read up front (before this interval's stage write)
  auto bread1 = [&](int st, v4u (&b)[2][2]) {
    const uint8_t* cb = cvt + (st & 1) * 2 * kCvtF;
#pragma unroll
    for (int kc = 0; kc < 2; ++kc) {
      b[kc][0] = ld16(cb + br_off[kc]);
      b[kc][1] = ld16(cb + br_off[kc] + kCvtF);
    }
  };
  auto mma1b = [&](f32x16& acc, int st, const v4u (&b)[2][2]) {
#pragma unroll
    for (int kc = 0; kc < 2; ++kc) acc = x3_32(a1[st & 1][kc][0], a1[st & 1][kc][1], b[kc][0], b[kc][1], acc);
  };
  // C (32x32) of a chunk -> ring: lane col = pixel, reg 4g+e -> channel 32q1 + 8g + 4hh + e
  auto epilogue = [&](const f32x16& acc, int g0, int nrows) {
    if (bpx < nrows) {
      int pos;
      (void)fast_divmod(g0 + bpx + W + 1, kRingF, kMagRingF, pos);
      uint8_t* rp = ring + (pos + 1) * kRowF1 + 8 * hh;
      const int mirror = pos == 0 ? kRingF * kRowF1 : (pos == kRingF - 1 ? -kRingF * kRowF1 : 0);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        f32x4 r;
#pragma unroll
        for (int e = 0; e < 4; ++e) r[e] = fmaxf(acc[4 * g + e], 0.f);
        v2u h, l;
        split4(r, h, l);
        uint8_t* q = rp + ((4 * q1 + g) << 4);
        *reinterpret_cast<v2u*>(q) = h;
        *reinterpret_cast<v2u*>(q + 256) = l;
        if (mirror) {
          *reinterpret_cast<v2u*>(q + mirror) = h;
          *reinterpret_cast<v2u*>(q + mirror + 256) = l;
        }
      }
    }
  };

  // ---- prologue: band(t_begin) in serial 64-row chunks (v1's schedule) ----
  {
    const int b0 = t_begin * kT2 - W - 1, b1 = t_begin * kT2 + kT2 + W + 1;
    for (int g0 = b0; g0 < b1; g0 += 64) {
      const float* xc = xptr(g0);
#pragma unroll
      for (int u = 0; u < PF; ++u) xload(u, xc, u);
      wload(0, 0);
      f32x16 acc = bias_acc();
      convert(0, 0, 0);
      if (PF < nst) xload(0, xc, PF);
      __syncthreads();
#pragma unroll
      for (int st = 0; st < nst; ++st) {
        if (st + 1 < nst) {
          wload((st + 1) & 1, st + 1);
          const int s = st + 1;
          convert(s % PF, s & 1, s);
          if (s + PF < nst) xload(s % PF, xc, s + PF);
        }
        mma1(acc, st);
        __syncthreads();
      }
      epilogue(acc, g0, min(64, b1 - g0));
    }
  }

  // ---- steady state: iteration t runs tile t's 3x3 and chunk g(t)'s 1x1 ----
  // entry state: stage 0 = step 0 of chunk g(t) converted, X slots hold the
  // chunk's next steps, a1[0] = W1 step 0, the ring holds band(t)
  const int c4 = lane >> 4;
  if (t_begin + 1 < t_end) {
    const int g = t_begin * kT2 + kT2 + W + 1;
    const float* xc = xptr(g);
#pragma unroll
    for (int u = 0; u < PF; ++u) xload(u, xc, u);
    wload(0, 0);
    convert(0, 0, 0);
    if (PF < nst) xload(0, xc, PF);
    else xload(0, xptr(g + 64), 0);
  }
  __syncthreads();  // B: ring = band(t_begin), stage 0 ready

  // 3x3 row bases of a tile (see v1)
  int R[4][3];
  bool lfm[4], rtm[4];
  auto rows3 = [&](int m0) {
    const int m = m0 + (lane & 15);
    int r, xx, pm;
    (void)fast_divmod(m, HW, p.mag_hw, r);
    int yy = fast_divmod(r, W, p.mag_w, xx);
    (void)fast_divmod(m + W + 1, kRingF, kMagRingF, pm);
#pragma unroll
    for (int pg = 0; pg < 4; ++pg) {
      if (pg) {
        xx += 16;
        if (xx >= W) {
          xx -= W;
          if (++yy == p.H) yy = 0;
        }
        pm += 16;
        if (pm >= kRingF) pm -= kRingF;
      }
      const bool in = m + 16 * pg < p.M;
      const int rm = pm - W, rp = pm + W;
      R[pg][0] = (in && yy > 0) ? (rm < 0 ? rm + kRingF : rm) : kZeroF;
      R[pg][1] = in ? pm : kZeroF;
      R[pg][2] = (in && yy < p.H - 1) ? (rp >= kRingF ? rp - kRingF : rp) : kZeroF;
      lfm[pg] = xx > 0;
      rtm[pg] = xx < W - 1;
    }
  };
  constexpr int kLead = 2;
  constexpr int kSteps3 = 4 * kTaps;
  v4u bq[kLead + 1][2];
  const int chunk16 = (4 * kq + (lane >> 4)) << 4;
  auto rd = [&](int step) {
    const int t = step >> 2, pg = step & 3;
    const int dy = t / 3, dx = t % 3 - 1;
    const int a = R[pg][dy] + dx;
    int off = a * kRowF1 + chunk16;
    if (dx < 0 && !lfm[pg]) off = kZeroF * kRowF1;
    if (dx > 0 && !rtm[pg]) off = kZeroF * kRowF1;
    const uint8_t* q = ring + kRowF1 + off;
    bq[step % (kLead + 1)][0] = ld16(q);
    bq[step % (kLead + 1)][1] = ld16(q + 256);
  };
  f32x4 acc3[4];
  auto mma3 = [&](int step) {
    if (step + kLead < kSteps3) rd(step + kLead);
    const int t = step >> 2, pg = step & 3;
    acc3[pg] = x3_16(w2h[t], w2l[t], bq[step % (kLead + 1)][0], bq[step % (kLead + 1)][1], acc3[pg]);
  };
  // 3x3 partials: another owner's 4 channels -> its scratch slot, own -> y-sum slot
  auto partials = [&]() {
    if (c4 != kq) {
      float* sw = scr + ((oh * 4 + c4) * 3 + (kq - c4 + 3) % 4) * 256 + (lane & 15) * 4;
#pragma unroll
      for (int pg = 0; pg < 4; ++pg) *reinterpret_cast<f32x4*>(sw + pg * 64) = acc3[pg];
    } else {
      float* yw = ysum + (oh * 4 + kq) * 256 + (lane & 15) * 4;
#pragma unroll
      for (int pg = 0; pg < 4; ++pg) *reinterpret_cast<f32x4*>(yw + pg * 64) = acc3[pg];
    }
  };
  auto owner_sums = [&](int m0) {
    if (c4 != kq) return;
    const float* sr = scr + (oh * 4 + kq) * 3 * 256 + (lane & 15) * 4;
    const float* yr = ysum + (oh * 4 + kq) * 256 + (lane & 15) * 4;
#pragma unroll
    for (int pg = 0; pg < 4; ++pg) {
      f32x4 v = *reinterpret_cast<const f32x4*>(yr + pg * 64);
#pragma unroll
      for (int src = 0; src < 3; ++src) v += *reinterpret_cast<const f32x4*>(sr + src * 256 + pg * 64);
      const int m = m0 + 16 * pg + (lane & 15);
      if (m < p.M) *reinterpret_cast<f32x4*>(p.y + (size_t)m * p.ldy + 16 * oh + 4 * kq) = v;
    }
  };

  for (int tile = t_begin; tile < t_end; ++tile) {
    const int m0 = tile * kT2;
    rows3(m0);
#pragma unroll
    for (int pg = 0; pg < 4; ++pg) acc3[pg] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (tile + 1 < t_end) {
      const int g = m0 + kT2 + W + 1;  // chunk g(t): the rows band(t+1) adds
      const float* xc = xptr(g);
      const float* xn = xptr(g + 64);
      f32x16 acc = bias_acc();
#pragma unroll
      for (int s = 0; s < kLead; ++s) rd(s);
      auto part1 = [&](int st) {  // conversion of step st+1 + the chunk's step-st MFMAs
        // step st's B fragments are read first: behind the conversion's LDS
        // write the compiler cannot hoist them (it does not see the two stage
        // buffers apart), and the MFMAs would wait for the whole conversion
        v4u b[2][2];
        bread1(st, b);
        if (st + 1 < nst) {
          const int s = st + 1, slot = s % PF;
          convert(slot, s & 1, s);
          if (s + PF < nst) xload(slot, xc, s + PF);
          else xload(slot, xn, slot);  // the slot's last step of this chunk: the next chunk's step `slot`
        }
        mma1b(acc, st, b);
        if (st + 1 == nst && nst % 2 == 1) wload(0, 0);  // a1[0] was step nst-1's
      };
      auto part3 = [&](int st) {
#pragma unroll
        for (int j = kSteps3 * st / nst; j < kSteps3 * (st + 1) / nst; ++j) mma3(j);
      };
#pragma unroll
      for (int st = 0; st < nst; ++st) {
        if (st + 1 < nst) wload((st + 1) & 1, st + 1);
        else if (nst % 2 == 0) wload(0, 0);  // the next chunk's step 0 (a1[0] is free in step nst-1)
        if (st == 0 && tile > t_begin) owner_sums(m0 - kT2);  // tile t-1's partials (barrier A behind them)
        part1(st);
        part3(st);
        if (st + 1 < nst) bar(st);
      }
      partials();
      bar(nst - 1);  // A: band(t) fully read, partials visible, the stages free
      epilogue(acc, g, kT2);
      convert(0, 0, 0);  // chunk g(t+1)'s step 0
      if (PF < nst) xload(0, xn, PF);
      else xload(0, xptr(g + 128), 0);
      bar(nst);  // B: ring = band(t+1), stage 0 ready
    } else {
      // last tile of the block: 3x3 only (v1's phase)
      if (tile > t_begin) owner_sums(m0 - kT2);
      __syncthreads();  // the owners' reads before this tile's partial writes
#pragma unroll
      for (int s = 0; s < kLead; ++s) rd(s);
#pragma unroll
      for (int j = 0; j < kSteps3; ++j) mma3(j);
      partials();
      __syncthreads();
      owner_sums(m0);
    }
  }
  // the clamped X prefetches of chunks past the block's last tile are still
  // in flight: land them before the wave ends
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---- K11w: K11x with split roles (warp-specialised) --------------------------
// v1 / v3 give every wave both jobs: convert X (BN1 + ReLU + hi/lo split, ~5
// VALU per element) and run the MFMAs, so each 32-k step is a serial chain of
// conversion, LDS write, barrier, operand read and MFMA in every wave (v1:
// ~960 cycles per step against 384 MFMA cycles per SIMD, r3/r5 cycle budgets).
// K11w is 12 waves:
//   * producers (waves 8-11, one per SIMD, no accumulators): keep kPfW K steps
//     of X in flight in registers, and stage step g+1 (BN1 from LDS, split)
//     into one of two LDS slots while the consumers multiply step g;
//   * consumers (waves 0-7, v1's roles): the 1x1 MFMAs of every step
//     (accumulators, W1 fragments by buffer loads one step ahead), the
//     epilogue z -> ring, tile t's 3x3 (weights resident) and the owner sums.
// Both roles run the same barrier sequence: Z (tables), P0 (step 0 staged),
// one R per global K step (the producer's slot g+1 is full, the consumers'
// slot g is free), and per tile T (band(t) complete in the ring) plus E after
// the last tile's 3x3.  The chunk sequence of a block: the band of its first
// tile in 64-row chunks, then the 64 rows each later tile adds.
// LDS: v1's ring, scratch, y sums, 2 stages and BN1 table (160,160 B).
// 768 threads: 168 VGPRs per wave (3 waves per SIMD).
constexpr int kLdsFW = kRingRowsF * kRowF1 + kScrF * 4 + kYsF * 4 + 4 * kCvtF + 2 * kMaxKF * 4;
static_assert(kLdsFW <= 160 * 1024, "K11w LDS budget");
constexpr int kPfW = 3;  // producer X steps in flight

template <int NST>
__global__ void __launch_bounds__(768, 1) x3_dense_ws_kernel(X3FusedParams p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t ldsfw[];
  uint8_t* const ring = ldsfw;
  float* const scr = reinterpret_cast<float*>(ldsfw + kRingRowsF * kRowF1);
  float* const ysum = scr + kScrF;                                    // [oh][owner][pg][16 px][4]
  uint8_t* const cvt = reinterpret_cast<uint8_t*>(ysum + kYsF);       // [slot 2][plane 2][64 px][64 B]
  float* const bn = reinterpret_cast<float*>(cvt + 4 * kCvtF);        // s1 [kMaxKF] | t1 [kMaxKF]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int W = p.W, HW = p.H * p.W;

  const int t_begin = blockIdx.x * p.tiles_per_block;
  const int t_end = min(p.tiles, t_begin + p.tiles_per_block);
  if (t_begin >= t_end) return;  // block-uniform, before any barrier
  const int b0 = t_begin * kT2 - W - 1, b1 = t_begin * kT2 + kT2 + W + 1;
  const int npro = (b1 - b0 + 63) >> 6;         // chunks of the first band
  const int nch = npro + (t_end - t_begin - 1);  // + one per later tile
  const int G = nch * NST;                       // K steps (R barriers) of the block
  auto chunk_g0 = [&](int c) { return c < npro ? b0 + 64 * c : (t_begin + c - npro) * kT2 + kT2 + W + 1; };

  for (int i = tid; i < p.K; i += 768) {
    bn[i] = p.s1[i];
    bn[kMaxKF + i] = p.t1[i];
  }
  if (tid < 3 * kRowF1 / 16) *reinterpret_cast<v4u*>(ring + kZeroF * kRowF1 + tid * 16) = v4u{0, 0, 0, 0};
  __syncthreads();  // Z

  if (wave >= 8) {
    // ------------------------------ producers ------------------------------
    // thread = pixel px of the step x 8-k chunk cj: two float4 of X per step,
    // one 16-B hi and one 16-B lo write (v1's stage layout: chunk c of pixel
    // px at slot c ^ ((px >> 2) & 3))
    const int pt = tid - 512;
    const int px = pt >> 2, cj = pt & 3;
    const int wo = px * 64 + ((cj ^ ((px >> 2) & 3)) << 4);
    f32x4 xr[kPfW][2];
    auto issue = [&](int s, int slot) {
      s = min(s, G - 1);  // past the end: re-load the last step (static vmcnt)
      const int c = s / NST, st = s - c * NST;
      const int m = min(max(chunk_g0(c) + px, 0), p.M - 1);
      const float* src = p.x + (size_t)m * p.ldx + st * 32 + 8 * cj;
      // inline-asm loads: hipcc's own wait before a use of a register loaded
      // across the round loop's back edge is a vmcnt(0), which drains the
      // prefetch once per kPfW rounds; the counted s_waitcnt below covers them
      asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(xr[slot][0]) : "v"(src) : "memory");
      asm volatile("global_load_dwordx4 %0, %1, off offset:16" : "=v"(xr[slot][1]) : "v"(src) : "memory");
    };
    // BN1 affine of the next step to convert, read from LDS one round ahead
    // (off the convert -> stage write -> barrier chain)
    f32x4 nb[4];
    auto ldbn = [&](int s) {
      const float* bs = bn + (s % NST) * 32 + 8 * cj;
      nb[0] = ldf4(bs);
      nb[1] = ldf4(bs + kMaxKF);
      nb[2] = ldf4(bs + 4);
      nb[3] = ldf4(bs + kMaxKF + 4);
    };
    auto convert = [&](int s, int slot) {
      v2u h0, l0, h1, l1;
      split4(bn_relu4(xr[slot][0], nb[0], nb[1]), h0, l0);
      split4(bn_relu4(xr[slot][1], nb[2], nb[3]), h1, l1);
      uint8_t* q = cvt + (s & 1) * 2 * kCvtF + wo;
      *reinterpret_cast<v4u*>(q) = v4u{h0[0], h0[1], h1[0], h1[1]};
      *reinterpret_cast<v4u*>(q + kCvtF) = v4u{l0[0], l0[1], l1[0], l1[1]};
    };
    __builtin_amdgcn_s_setprio(1);  // the producers' step is the chain every round waits on
#pragma unroll
    for (int u = 0; u < kPfW; ++u) issue(u, u);
    ldbn(0);
    __builtin_amdgcn_s_waitcnt(ws_vmcnt(2 * (kPfW - 1)));  // step 0 landed
    __builtin_amdgcn_sched_barrier(0);
    convert(0, 0);
    __builtin_amdgcn_sched_barrier(0);
    issue(kPfW, 0);
    ldbn(1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    ws_barrier();  // P0
    for (int g0 = 0; g0 < G; g0 += kPfW) {
#pragma unroll
      for (int u = 0; u < kPfW; ++u) {
        const int g = g0 + u;
        if (g >= G) break;  // block-uniform
        // unconditional (step G, past the end, converts a clamped copy into
        // a slot no consumer reads): the vmcnt below counts kPfW - 1 steps
        const int slot = (u + 1) % kPfW;
        __builtin_amdgcn_s_waitcnt(ws_vmcnt(2 * (kPfW - 1)));  // X of step g+1
        __builtin_amdgcn_sched_barrier(0);
        convert(g + 1, slot);
        __builtin_amdgcn_sched_barrier(0);
        issue(g + 1 + kPfW, slot);
        ldbn(g + 2);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        ws_barrier();  // R(g)
        if ((g + 1) % NST == 0) {
          const int c = g / NST;
          if (c >= npro - 1) {
            ws_barrier();                 // T
            if (c == nch - 1) ws_barrier();  // E
          }
        }
      }
    }
    // the clamped re-loads past the last step land before the wave ends; the
    // empty asm keeps their registers allocated until then (hipcc does not
    // know the inline-asm loads are in flight and could reuse a dead one)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < kPfW; ++u) asm volatile("" ::"v"(xr[u][0]), "v"(xr[u][1]));
    return;
  }

  // ------------------------------- consumers -------------------------------
  // 3x3 roles and resident weights: A[16oh + (lane&15)][tap t][32kq + 8(lane>>4) ..+8]
  const int kq = wave & 3, oh = wave >> 2;
  v4u w2h[kTaps], w2l[kTaps];
#pragma unroll
  for (int t = 0; t < kTaps; ++t) {
    const size_t off = ((size_t)((t * 4 + kq) * 2 + oh) * 64 + lane) * 8;
    w2h[t] = ld16(p.w2_hi + off);
    w2l[t] = ld16(p.w2_lo + off);
  }
  // 1x1 roles: output-channel quarter q1 x pixel half ph of the 64-row chunk
  const int q1 = wave & 3, ph = wave >> 2;
  const int col = lane & 31, hh = lane >> 5;
  v4u a1[2][2][2];  // [step parity][kc][plane]
  const auto w1h = __builtin_amdgcn_make_buffer_rsrc((void*)p.w1_hi, (short)0, p.K * 256, 0x00020000);
  const auto w1l = __builtin_amdgcn_make_buffer_rsrc((void*)p.w1_lo, (short)0, p.K * 256, 0x00020000);
  const int w1v = (q1 * 64 + lane) * 16;
  auto wload = [&](int slot, int st) {
    st = min(st, NST - 1);
#pragma unroll
    for (int kc = 0; kc < 2; ++kc) {
      a1[slot][kc][0] = __builtin_amdgcn_raw_buffer_load_b128(w1h, w1v, (2 * st + kc) * 4096, 0);
      a1[slot][kc][1] = __builtin_amdgcn_raw_buffer_load_b128(w1l, w1v, (2 * st + kc) * 4096, 0);
    }
  };
  const int bpx = 32 * ph + col;
  const int bsw = (bpx >> 2) & 3;
  const int br_off[2] = {bpx * 64 + ((hh ^ bsw) << 4), bpx * 64 + (((2 + hh) ^ bsw) << 4)};
  // z rows [g0, g0 + nrows) -> ring; W(0) was issued by the caller; gs = the
  // chunk's first global step (its stage slot parity)
  auto z_chunk = [&](int g0, int nrows, int gs) {
    f32x16 acc;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 b = ldf4(p.b1 + 32 * q1 + 8 * g + 4 * hh);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[4 * g + e] = b[e];
    }
#pragma unroll
    for (int st = 0; st < NST; ++st) {
      wload((st + 1) & 1, st + 1);
      const uint8_t* cb = cvt + ((gs + st) & 1) * 2 * kCvtF;
#pragma unroll
      for (int kc = 0; kc < 2; ++kc) {
        const uint8_t* q = cb + br_off[kc];
        acc = x3_32(a1[st & 1][kc][0], a1[st & 1][kc][1], ld16(q), ld16(q + kCvtF), acc);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      ws_barrier();  // R
    }
    // C (32x32): lane col = pixel, reg 4g+e -> channel 32q1 + 8g + 4hh + e
    if (bpx < nrows) {
      int pos;
      (void)fast_divmod(g0 + bpx + W + 1, kRingF, kMagRingF, pos);
      uint8_t* rp = ring + (pos + 1) * kRowF1 + 8 * hh;
      const int mirror = pos == 0 ? kRingF * kRowF1 : (pos == kRingF - 1 ? -kRingF * kRowF1 : 0);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        f32x4 r;
#pragma unroll
        for (int e = 0; e < 4; ++e) r[e] = fmaxf(acc[4 * g + e], 0.f);
        v2u h, l;
        split4(r, h, l);
        uint8_t* q = rp + ((4 * q1 + g) << 4);
        *reinterpret_cast<v2u*>(q) = h;
        *reinterpret_cast<v2u*>(q + 256) = l;
        if (mirror) {
          *reinterpret_cast<v2u*>(q + mirror) = h;
          *reinterpret_cast<v2u*>(q + mirror + 256) = l;
        }
      }
    }
  };

  ws_barrier();  // P0
  int gs = 0;
  for (int c = 0; c < npro; ++c, gs += NST) {
    wload(0, 0);
    z_chunk(chunk_g0(c), min(64, b1 - chunk_g0(c)), gs);
  }
  const int c4 = lane >> 4;
  for (int tile = t_begin; tile < t_end; ++tile) {
    const int m0 = tile * kT2;
    __syncthreads();  // T: the ring holds band(tile); the scratch is free
    // ---- 3x3 (as v1) ----
    {
      // band rows of tap rows dy 0/1/2 packed in bytes 0/1/2 (all < 256):
      // 8 VGPRs fewer than v1's table, one v_bfe per operand read
      uint32_t R[4];
      bool lfm[4], rtm[4];
      {
        const int m = m0 + (lane & 15);
        int r, xx, pm;
        (void)fast_divmod(m, HW, p.mag_hw, r);
        int yy = fast_divmod(r, W, p.mag_w, xx);
        (void)fast_divmod(m + W + 1, kRingF, kMagRingF, pm);
#pragma unroll
        for (int pg = 0; pg < 4; ++pg) {
          if (pg) {
            xx += 16;
            if (xx >= W) {
              xx -= W;
              if (++yy == p.H) yy = 0;
            }
            pm += 16;
            if (pm >= kRingF) pm -= kRingF;
          }
          const bool in = m + 16 * pg < p.M;
          const int rm = pm - W, rp = pm + W;
          const int r0 = (in && yy > 0) ? (rm < 0 ? rm + kRingF : rm) : kZeroF;
          const int r1 = in ? pm : kZeroF;
          const int r2 = (in && yy < p.H - 1) ? (rp >= kRingF ? rp - kRingF : rp) : kZeroF;
          R[pg] = (uint32_t)r0 | ((uint32_t)r1 << 8) | ((uint32_t)r2 << 16);
          lfm[pg] = xx > 0;
          rtm[pg] = xx < W - 1;
        }
      }
      f32x4 acc[4];
#pragma unroll
      for (int pg = 0; pg < 4; ++pg) acc[pg] = f32x4{0.f, 0.f, 0.f, 0.f};
      constexpr int kLead = 2;  // (3 in v1: one more operand set than 168 VGPRs hold)
      v4u bq[kLead + 1][2];
      const int chunk16 = (4 * kq + (lane >> 4)) << 4;
      auto rd = [&](int step) {
        const int t = step >> 2, pg = step & 3;
        const int dy = t / 3, dx = t % 3 - 1;
        const int a = (int)((R[pg] >> (8 * dy)) & 0xff) + dx;
        int off = a * kRowF1 + chunk16;
        if (dx < 0 && !lfm[pg]) off = kZeroF * kRowF1;
        if (dx > 0 && !rtm[pg]) off = kZeroF * kRowF1;
        const uint8_t* q = ring + kRowF1 + off;
        bq[step % (kLead + 1)][0] = ld16(q);
        bq[step % (kLead + 1)][1] = ld16(q + 256);
      };
#pragma unroll
      for (int step = 0; step < kLead; ++step) rd(step);
#pragma unroll
      for (int step = 0; step < 4 * kTaps; ++step) {
        if (step + kLead < 4 * kTaps) rd(step + kLead);
        __builtin_amdgcn_sched_barrier(0);
        const int t = step >> 2, pg = step & 3;
        acc[pg] = x3_16(w2h[t], w2l[t], bq[step % (kLead + 1)][0], bq[step % (kLead + 1)][1], acc[pg]);
      }
      // the next chunk's W(0): issued after the operand reads (168 VGPRs do
      // not hold it beside them), in flight during the partial stores
      if (tile + 1 < t_end) wload(0, 0);
      if (c4 != kq) {
        float* sw = scr + ((oh * 4 + c4) * 3 + (kq - c4 + 3) % 4) * 256 + (lane & 15) * 4;
#pragma unroll
        for (int pg = 0; pg < 4; ++pg) *reinterpret_cast<f32x4*>(sw + pg * 64) = acc[pg];
      } else {
        float* yw = ysum + (oh * 4 + kq) * 256 + (lane & 15) * 4;
#pragma unroll
        for (int pg = 0; pg < 4; ++pg) *reinterpret_cast<f32x4*>(yw + pg * 64) = acc[pg];
      }
    }
    if (tile + 1 < t_end) {
      z_chunk(m0 + kT2 + W + 1, kT2, gs);
      gs += NST;
    } else {
      __syncthreads();  // E
    }
    if (c4 == kq) {
      const float* sr = scr + (oh * 4 + kq) * 3 * 256 + (lane & 15) * 4;
      const float* yr = ysum + (oh * 4 + kq) * 256 + (lane & 15) * 4;
#pragma unroll
      for (int pg = 0; pg < 4; ++pg) {
        f32x4 v = *reinterpret_cast<const f32x4*>(yr + pg * 64);
#pragma unroll
        for (int src = 0; src < 3; ++src) v += *reinterpret_cast<const f32x4*>(sr + src * 256 + pg * 64);
        const int m = m0 + 16 * pg + (lane & 15);
        if (m < p.M) *reinterpret_cast<f32x4*>(p.y + (size_t)m * p.ldy + 16 * oh + 4 * kq) = v;
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ============================================================================
// K14x: the whole dense layer in one kernel for the 14x14 and 7x7 blocks
// ============================================================================
// K11x's ring needs W >= 16; at 14x14 / 7x7 the K8x + K9x pair ran every
// layer as two launches with z (hi|lo, 512 B a pixel) written to HBM and read
// back (40 of the 58 dense layers, 36% of a bs128 forward).  Here one block
// owns one TILE of whole image rows and keeps z on chip:
//
//   14x14: tile = half an image (output rows 0-6 or 7-13) plus the one halo
//          row the 3x3 needs from the other half: z over 8 rows = 112 pixels,
//          98 outputs.  Both halves of an image go to blocks b and b+8, which
//          the dispatcher places on one XCD (blockIdx % 8 labels the XCD), so
//          the halo rows' second read is an L2 hit.
//    7x7:  tile = one whole image (49 pixels; no halo).
//
//   1x1 (K -> 128, BN1+ReLU prologue, BN2-folded bias+ReLU epilogue): the K8x
//   ws pipeline on ONE tile of <= 128 rows: producer waves 4-7 keep PF K steps
//   of X in flight in registers and stage each step split hi/lo into LDS, W
//   slices go by LDS-DMA (or the consumers load their own W1 fragments: WR),
//   consumer waves 0-3 run the 32x32x16 MFMAs (wave = 32-channel quarter x
//   every 32-pixel block of the tile); one raw s_barrier per K step.
//   The epilogue writes z into a zero-PADDED image of the tile in LDS
//   ([rows+2][W+2] pixels x 512 B, 16-B chunks XOR-swizzled by pixel) that
//   aliases the drained K-step stages, so every 3x3 tap is one constant
//   offset from the output pixel: no bounds tests in the tap loop.
//   3x3 (128 -> 32): all 8 waves as K11x v1 (input-channel quarter x output
//   half, 16x16x32 MFMAs, weights resident: x3_w3f_fragments), the 4 partials
//   summed through an LDS scratch, fp32 stores of the layer's 32 channels.
//
// HBM per layer: the input X once (+ the halo rows through L2) and 32 output
// channels; one launch.  LDS: 4 K-step stages (128 KB); z and the 3x3
// scratch alias them once the 1x1 drained.

struct X3SmallParams {
  const float* x;  // block buffer rows of ldx (the layer's first K channels)
  const float* s1;  // [K] BN1 affine
  const float* t1;
  const uint16_t* w1f_hi;  // [K/16][q 4][lane 64][8] bf16 (x3_w1_fragments, BN2 folded)
  const uint16_t* w1f_lo;
  const float* b1;        // [128] BN2 shift
  const uint16_t* w2_hi;  // [tap 9][kq 4][oh 2][lane 64][8] bf16 (x3_w3f_fragments)
  const uint16_t* w2_lo;
  float* y;               // [pixels][ldy] fp32, offset to the layer's 32-channel slice
  int ldx, K, ldy, imgs;
};

// Tile geometry of T tiles per W x W image: tile t owns output rows
// [tW/T, (t+1)W/T) and computes z over those rows plus one halo row on each
// side that exists (the halo's 1x1 is recomputed by the neighbour tile).
constexpr int x3s_zrows_max(int W, int T) {
  int m = 0;
  for (int t = 0; t < T; ++t) {
    const int r0 = t * W / T, r1 = (t + 1) * W / T;
    const int z0 = r0 > 0 ? r0 - 1 : 0, z1 = r1 < W ? r1 + 1 : W;
    m = z1 - z0 > m ? z1 - z0 : m;
  }
  return m;
}

// W = image side (14 or 7); T = tiles per image.  More tiles per image give a
// small batch more workgroups (bs64 at 14x14: 128 half-image tiles on 256
// CUs) for the price of the recomputed halo rows.  PF = 3 X K-steps in the
// producers' registers, 4 K-step stages, W1 loaded by the consumers.
template <int W, int T>
__device__ __forceinline__ void x3_small_body(const X3SmallParams& p) {
  // (6 X steps in flight measured the same as 3 at 16..128 images: the step
  // is bound by the producers' conversion, not by X latency; round 5)
  constexpr int PF = 3, kSmS = 4;
  constexpr int kLdsSm = kSmS * kWsStage;
  constexpr int kRowsOut = (W + T - 1) / T;          // most output rows of a tile
  constexpr int kPW = W + 2, kPR = kRowsOut + 2;     // padded tile image
  constexpr int kNPad = kPR * kPW;
  constexpr int kPOut = kRowsOut * W;                // most outputs of a tile
  constexpr int kNPG = (kPOut + 15) / 16;            // 16-pixel groups of the 3x3
  constexpr int kTRMax = x3s_zrows_max(W, T) * W;    // most z pixels of a tile
  constexpr int kNRI = (kTRMax + 31) / 32;           // producer row passes (32 rows each)
  constexpr int kOps = kNRI;                         // vm ops per producer iteration
  constexpr int kNB = (kTRMax + 31) / 32;            // 32-pixel blocks of the 1x1 tile
  static_assert(kTRMax <= 128, "one 1x1 tile");
  static_assert(kNPad * kRowB + 2 * 4 * 3 * kNPG * 64 * 4 <= kLdsSm, "K14x LDS budget");
  extern __shared__ __attribute__((aligned(16))) uint8_t ldss[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  // tile t of image 8g+j is block 8Tg + 8t + j: an image's tiles share
  // blockIdx % 8, which the dispatcher maps to one XCD, so the halo rows'
  // second read is an L2 hit (speed only, never correctness)
  const int g8 = blockIdx.x / (8 * T), rr = blockIdx.x % (8 * T);
  const int tile = rr >> 3, img = 8 * g8 + (rr & 7);
  if (img >= p.imgs) return;  // block-uniform, before any barrier
  const int r0 = tile * W / T, r1 = (tile + 1) * W / T;
  const int zr0 = max(r0 - 1, 0), zr1 = min(r1 + 1, W);
  const int TR = (zr1 - zr0) * W;  // z rows of the tile
  const int mz0 = img * W * W + zr0 * W;
  const int nst = p.K / kBK;
  const int Q = nst;  // K steps = barrier rounds of both roles (no padding to a multiple of PF)
  // consumer wave = 32-channel quarter of the 1x1 output x every 32-pixel
  // block: each W1 fragment is loaded by one wave only, for twice the X
  // operand reads, which go to LDS (256 B/clk) instead of the vector-memory path
  f32x16 acc[kNB];
  const int col = lane & 31, h = lane >> 5;
  const int rot = (int)(blockIdx.x % (unsigned)nst);  // blocks read different K offsets at a time
  auto kofs = [&](int ks) { ks += rot; return (ks >= nst ? ks - nst : ks) * kBK; };
  // BN1 affine s1 | t1 (2 x K floats) in stage 0's W planes (no W copies there)
  float* const bnl = reinterpret_cast<float*>(ldss + 2 * kWsPlane);

  if (wave >= 4) {
    // ------------------------------ producer (K8x ws) ------------------------------
    const int pt = tid - 256;
    const int pj = pt & 7, prow = pt >> 3;
    f32x4 xr[PF][kNRI], xs, xt;
    // the BN1 affine of step 0 from global memory, of every later step from the
    // LDS copy the consumers make before B0
    auto issue_x = [&](int q, int slot) {
      q = min(q, Q - 1);
      const int k0 = kofs(q);
#pragma unroll
      for (int i = 0; i < kNRI; ++i) {
        const int m = mz0 + min(prow + 32 * i, TR - 1);
        xr[slot][i] = ldf4(p.x + (size_t)m * p.ldx + k0 + 4 * pj);
      }
    };
    auto write_x = [&](int q, int slot) {
      uint8_t* st = ldss + (q % kSmS) * kWsStage;
      f32x4 sc = xs, sb = xt;
      if (q > 0) {
        const int k0 = kofs(min(q, Q - 1)) + 4 * pj;
        sc = *reinterpret_cast<const f32x4*>(bnl + k0);
        sb = *reinterpret_cast<const f32x4*>(bnl + p.K + k0);
      }
#pragma unroll
      for (int i = 0; i < kNRI; ++i) {
        // rows >= TR hold row TR-1's data (clamped loads): their z columns
        // are never written to the tile image, so they need no zeroing
        const int row = prow + 32 * i;
        const f32x4 v = bn_relu4(xr[slot][i], sc, sb);
        v2u hh, ll;
        split4(v, hh, ll);
        const int off = ws_chunk(row, pj >> 1) + (pj & 1) * 8;
        *reinterpret_cast<v2u*>(st + off) = hh;
        *reinterpret_cast<v2u*>(st + kWsPlane + off) = ll;
      }
    };
    xs = ldf4(p.s1 + kofs(0) + 4 * pj);
    xt = ldf4(p.t1 + kofs(0) + 4 * pj);
#pragma unroll
    for (int s = 0; s < PF; ++s) issue_x(s, s);
    __builtin_amdgcn_s_waitcnt(ws_vmcnt(0));
    write_x(0, 0);
    __builtin_amdgcn_sched_barrier(0);
    issue_x(PF, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    ws_barrier();  // B0
    for (int q0 = 0; q0 < Q; q0 += PF) {
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        const int q = q0 + u;
        if (q >= Q) break;  // block-uniform: both roles run Q barrier rounds
        const int slot = (u + 1) % PF;
        __builtin_amdgcn_s_waitcnt(ws_vmcnt(kOps * (PF - 1)));  // X of step q+1
        __builtin_amdgcn_sched_barrier(0);
        write_x(q + 1, slot);
        __builtin_amdgcn_sched_barrier(0);
        issue_x(q + 1 + PF, slot);
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this step's stage writes
        ws_barrier();  // B(q+1)
      }
    }
  } else {
    // ------------------------------- consumer -------------------------------
#pragma unroll
    for (int b = 0; b < kNB; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[b][e] = 0.f;
    // one K step's operands: W hi/lo [kk] of this wave's channel quarter, X hi/lo [kk][pixel block]
    struct AOps {
      v4u h[2], l[2];
    };
    struct BOps {
      v4u h[2][kNB], l[2][kNB];
    };
    auto rd_b = [&](int q, BOps& o) {
      const uint8_t* st = ldss + (q % kSmS) * kWsStage;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int b = 0; b < kNB; ++b) {
          const int xo = ws_chunk(32 * b + col, 2 * kk + h);
          o.h[kk][b] = ld16(st + xo);
          o.l[kk][b] = ld16(st + kWsPlane + xo);
        }
    };
    // this wave's W1 fragments from L2 (1 KB per wave load) as buffer loads: a
    // lane-constant VGPR offset and the step's offset in an SGPR
    const auto w1h = __builtin_amdgcn_make_buffer_rsrc((void*)p.w1f_hi, (short)0, p.K * 256, 0x00020000);
    const auto w1l = __builtin_amdgcn_make_buffer_rsrc((void*)p.w1f_lo, (short)0, p.K * 256, 0x00020000);
    auto ld_a = [&](int q, AOps& o) {
      const int k16 = kofs(min(q, Q - 1)) / 16;
      const int vo = (wave * 64 + lane) * 16;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        o.h[kk] = __builtin_amdgcn_raw_buffer_load_b128(w1h, vo, (k16 + kk) * 4096, 0);
        o.l[kk] = __builtin_amdgcn_raw_buffer_load_b128(w1l, vo, (k16 + kk) * 4096, 0);
      }
    };
    auto mma = [&](const AOps& A, const BOps& B) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int b = 0; b < kNB; ++b)
          if (32 * b < TR) acc[b] = x3_32(A.h[kk], A.l[kk], B.h[kk][b], B.l[kk][b], acc[b]);
    };
    // W of step q is loaded during step q-1 (two register sets, the loop
    // unrolled by 2 so each has a fixed name); the step's counted wait leaves
    // the next step's 4 fragment loads in flight.  The prefetch is
    // unconditional (past the last step it reloads that step's fragments):
    // with a conditional one the compiler's own waits before the MFMAs assume
    // the no-prefetch path and drain it.
    constexpr int kAOps = 4;
    // the producers' BN1 affine for steps >= 1 (published by B0)
    for (int i = tid; i < p.K / 4; i += 256) {
      *reinterpret_cast<f32x4*>(bnl + 4 * i) = ldf4(p.s1 + 4 * i);
      *reinterpret_cast<f32x4*>(bnl + p.K + 4 * i) = ldf4(p.t1 + 4 * i);
    }
    AOps fa, fb;
    ld_a(0, fa);  // lands during the producers' prologue
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the copy is in LDS
    ws_barrier();  // B0
    auto step = [&](int q, const AOps& cur, AOps& nxt) {
      ld_a(q + 1, nxt);
      if (q < Q) {
        BOps B;
        rd_b(q, B);
        __builtin_amdgcn_s_waitcnt(ws_vmcnt(kAOps));  // this step's fragments
        mma(cur, B);
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
      ws_barrier();  // B(q+1)
    };
    for (int q = 0; q < Q; q += 2) {
      step(q, fa, fb);
      if (q + 1 >= Q) break;
      step(q + 1, fb, fa);
    }
  }
  // BN2 bias of this consumer lane's channels, loaded BEFORE the 3x3
  // weights: a later load would make its wait drain the weight loads too
  f32x4 ob[4];
  if (wave < 4) {
#pragma unroll
    for (int g = 0; g < 4; ++g) ob[g] = ldf4(p.b1 + 32 * wave + 8 * g + 4 * h);
  }
  // 3x3 weights: in flight while the LDS changes hands and z is written
  const int kq = wave & 3, oh = wave >> 2;
  v4u w2h[kTaps], w2l[kTaps];
#pragma unroll
  for (int t = 0; t < kTaps; ++t) {
    const size_t off = ((size_t)((t * 4 + kq) * 2 + oh) * 64 + lane) * 8;
    w2h[t] = ld16(p.w2_hi + off);
    w2l[t] = ld16(p.w2_lo + off);
  }
  // Bz: every stage read retired, the LDS holds z from here; raw barrier, so
  // the weight loads stay in flight across it (a __syncthreads would drain them)
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_waitcnt(ws_vmcnt_lgkm0(2 * kTaps));
  ws_barrier();
  // zero the padding of the tile image (columns 0 and W+1, rows outside the image)
  for (int i = tid; i < kNPad * 32; i += 512) {
    const int pos = i >> 5, piece = i & 31;
    const int prr = pos / kPW, pc = pos - prr * kPW;
    const int ir = r0 - 1 + prr;
    if (pc == 0 || pc == kPW - 1 || ir < zr0 || ir >= zr1)
      *reinterpret_cast<v4u*>(ldss + pos * kRowB + piece * 16) = v4u{0, 0, 0, 0};
  }
  if (wave < 4) {
    // 1x1 epilogue: + bias, ReLU, hi/lo split into the padded tile image.
    // C (32x32): lane col = pixel, reg 4g+e -> channel 32wave + 8g + 4h + e
#pragma unroll
    for (int b = 0; b < kNB; ++b) {
      const int pz = 32 * b + col;  // z pixel of the tile
      if (pz < TR) {
        const int zy = pz / W, zx = pz - zy * W;
        const int pos = (zr0 + zy - r0 + 1) * kPW + zx + 1;
        uint8_t* rp = ldss + pos * kRowB + 8 * h;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          f32x4 r;
#pragma unroll
          for (int e = 0; e < 4; ++e) r[e] = fmaxf(acc[b][4 * g + e] + ob[g][e], 0.f);
          v2u hh, ll;
          split4(r, hh, ll);
          uint8_t* q = rp + ((((4 * wave) + g) ^ (pos & 15)) << 4);
          *reinterpret_cast<v2u*>(q) = hh;
          *reinterpret_cast<v2u*>(q + 256) = ll;
        }
      }
    }
  }

  // ---- 3x3 phase: 8 waves = input-channel quarter kq x output half oh ----
  __syncthreads();  // z and its padding complete
  const int nout = (r1 - r0) * W;  // this tile's outputs (the last tile may have fewer rows)
  int base[kNPG];
#pragma unroll
  for (int pg = 0; pg < kNPG; ++pg) {
    const int o = 16 * pg + (lane & 15);
    const int yy = o / W, xx = o - (o / W) * W;
    // padded (yy, xx) is tap (0, 0) of output (yy, xx); lanes past the tile
    // read from pixel 0 (in bounds; their columns are never stored)
    base[pg] = o < nout ? yy * kPW + xx : 0;
  }
  f32x4 acc3[kNPG];
#pragma unroll
  for (int pg = 0; pg < kNPG; ++pg) acc3[pg] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int chunk16 = 4 * kq + (lane >> 4);
  constexpr int kSteps = kTaps * kNPG;
  constexpr int kLead = 3;
  v4u bq[kLead + 1][2];
  auto rd = [&](int step) {
    const int t = step / kNPG, pg = step - (step / kNPG) * kNPG;
    const int pos = base[pg] + (t / 3) * kPW + (t % 3);
    const uint8_t* q = ldss + pos * kRowB + (((chunk16 ^ (pos & 15))) << 4);
    bq[step % (kLead + 1)][0] = ld16(q);
    bq[step % (kLead + 1)][1] = ld16(q + 256);
  };
#pragma unroll
  for (int step = 0; step < kLead; ++step) rd(step);
#pragma unroll
  for (int step = 0; step < kSteps; ++step) {
    if (step + kLead < kSteps) rd(step + kLead);
    __builtin_amdgcn_sched_barrier(0);
    const int t = step / kNPG, pg = step - (step / kNPG) * kNPG;
    acc3[pg] = x3_16(w2h[t], w2l[t], bq[step % (kLead + 1)][0], bq[step % (kLead + 1)][1], acc3[pg]);
  }
  // C (16x16): lane (lane&15) = pixel of group pg, reg e -> channel 16oh + 4c + e
  // (c = lane>>4); wave (kq = c, oh) owns those 4 channels and adds the other
  // three waves' partials
  float* scr = reinterpret_cast<float*>(ldss + kNPad * kRowB);
  const int c4 = lane >> 4;
  constexpr int kSlot = kNPG * 64;
  if (c4 != kq) {
    float* sw = scr + ((oh * 4 + c4) * 3 + (kq - c4 + 3) % 4) * kSlot + (lane & 15) * 4;
#pragma unroll
    for (int pg = 0; pg < kNPG; ++pg) *reinterpret_cast<f32x4*>(sw + pg * 64) = acc3[pg];
  }
  __syncthreads();
  if (c4 == kq) {
    const float* sr = scr + (oh * 4 + kq) * 3 * kSlot + (lane & 15) * 4;
    const int m0 = img * W * W + r0 * W;
#pragma unroll
    for (int pg = 0; pg < kNPG; ++pg) {
      f32x4 v = acc3[pg];
#pragma unroll
      for (int src = 0; src < 3; ++src) v += *reinterpret_cast<const f32x4*>(sr + src * kSlot + pg * 64);
      const int o = 16 * pg + (lane & 15);
      if (o < nout) *reinterpret_cast<f32x4*>(p.y + (size_t)(m0 + o) * p.ldy + 16 * oh + 4 * kq) = v;
    }
  }
}

template <int W, int T>
__global__ void __launch_bounds__(512, 1) x3_dense_small_kernel(X3SmallParams p) {
  x3_small_body<W, T>(p);
}

// ============================================================================
// K10x stem: y = relu(maxpool3x3/2(conv7x7/2(x)) + b), 3 -> 64 channels, fp32
// ============================================================================
// As K10s in densenet.hip (patch staged once per block, conv as an implicit
// GEMM on v_mfma_f32_32x32x16 with weights [64][kh 7][kw 8][ch 4] as operand
// A), with the patch split into hi/lo planes and the weights' hi/lo fragments
// in registers; the 3x3/2 max-pool runs on the conv rows in registers.
// (A conv tile in LDS and a one-block-per-tile grid were the v1 / v2 of
// round 2: both slower than the persistent kernel below, removed in round 5.)
constexpr int kSPR = 4, kSPC = 14;       // pooled outputs per block
constexpr int kSCR = 2 * kSPR + 1;       // 9 conv rows
constexpr int kSIR = 2 * kSCR + 5;       // 23 input rows
constexpr int kSIC = 72;                 // input cols
constexpr int kSK = 7 * 32;              // (kh, kw[8], ch[4])
constexpr int kSHin = 224, kSHo = 56;

struct X3StemParams {
  const float* const* srcs;  // per-image fp32 NCHW [3][224][224] (device pointer table)
  const uint16_t* w_hi;      // [64][kSK] bf16 (BN0 scale folded), fragment-major (x3_stem_fragments)
  const uint16_t* w_lo;
  const float* bias;         // [64] BN0 shift
  float* y;                  // [imgs][56][56] pixels, rows of ldy fp32
  int ldy;
};

constexpr int kStage = (kSIR * kSIC + 255) / 256;

// The 23x72 input patch (3 channels) of the tile whose pooled origin is
// (pr0, pc0) into registers, zero outside the image.  Branch-free (clamped
// addresses, then a select) through a global-address-space pointer: the
// pointer comes from the srcs table, and as a generic pointer the loads were
// flat loads under per-element branches, each waited for (vmcnt(0)) before
// the next was issued, and counted against lgkmcnt too.
typedef const __attribute__((address_space(1))) float* x3_gptr;
__device__ __forceinline__ void x3_stem_load(const float* src, int pr0, int pc0, int tid, float (&v)[kStage][3]) {
  const x3_gptr g = (x3_gptr)src;
  const int ir0 = 4 * pr0 - 5, ic0 = 4 * pc0 - 5;
#pragma unroll
  for (int i = 0; i < kStage; ++i) {
    const int e = tid + i * 256;
    const int ec = min(e, kSIR * kSIC - 1);
    const int r = ec / kSIC, c = ec - r * kSIC;
    const int ih = ir0 + r, iw = ic0 + c;
    const bool in = e < kSIR * kSIC && ih >= 0 && ih < kSHin && iw >= 0 && iw < kSHin;
    const int o = min(max(ih, 0), kSHin - 1) * kSHin + min(max(iw, 0), kSHin - 1);
    const float a0 = __builtin_nontemporal_load(g + o);
    const float a1 = __builtin_nontemporal_load(g + o + kSHin * kSHin);
    const float a2 = __builtin_nontemporal_load(g + o + 2 * kSHin * kSHin);
    v[i][0] = in ? a0 : 0.f;
    v[i][1] = in ? a1 : 0.f;
    v[i][2] = in ? a2 : 0.f;
  }
}

// The patch, split into hi/lo bf16 planes: pixel e = 4 channels (the 4th 0).
__device__ __forceinline__ void x3_stem_stage(uint16_t* Ih, uint16_t* Il, int tid, const float (&v)[kStage][3]) {
#pragma unroll
  for (int i = 0; i < kStage; ++i) {
    const int e = tid + i * 256;
    if (e < kSIR * kSIC) {
      uint32_t h0, l0, h1, l1;
      split2(v[i][0], v[i][1], h0, l0);
      split2(v[i][2], 0.f, h1, l1);
      *reinterpret_cast<v2u*>(&Ih[e * 4]) = v2u{h0, h1};
      *reinterpret_cast<v2u*>(&Il[e * 4]) = v2u{l0, l1};
    }
  }
}

// Wave (nh = channel half, mg = conv-row group)'s weight fragments, from the
// fragment-major copy (x3_stem_fragments: one load = the wave's 1 KB).
__device__ __forceinline__ void x3_stem_weights(const X3StemParams& p, int lane, int nh, v4u (&wh)[kSK / 16],
                                                v4u (&wl)[kSK / 16]) {
#pragma unroll
  for (int s = 0; s < kSK / 16; ++s) {
    const size_t off = ((size_t)(nh * (kSK / 16) + s) * 64 + lane) * 8;
    wh[s] = ld16(p.w_hi + off);
    wl[s] = ld16(p.w_lo + off);
  }
}

// One conv row (32 conv cols x this wave's 32 channels) on MFMA.  The next
// k-step's patch fragments are read from LDS while this step's 3 MFMAs run
// (reading them just before use left every step waiting on LDS latency).
__device__ __forceinline__ f32x16 x3_stem_conv_row(const uint16_t* Ih, const uint16_t* Il, const v4u (&wh)[kSK / 16],
                                                   const v4u (&wl)[kSK / 16], int cr, int lane) {
  const int jj = lane & 31, hh = lane >> 5;
  auto off = [&](int s) { return ((2 * cr + (s >> 1)) * kSIC + 2 * jj + 2 * ((s & 1) * 2 + hh)) * 4; };
  f32x16 acc;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.f;
  v4u bh = ld16(&Ih[off(0)]), bl = ld16(&Il[off(0)]);
#pragma unroll
  for (int s = 0; s < kSK / 16; ++s) {
    v4u nh = bh, nl = bl;
    if (s + 1 < kSK / 16) {
      nh = ld16(&Ih[off(s + 1)]);
      nl = ld16(&Il[off(s + 1)]);
    }
    __builtin_amdgcn_sched_barrier(0);  // keep the reads ahead of the MFMAs
    acc = x3_32(wh[s], wl[s], bh, bl, acc);
    bh = nh;
    bl = nl;
  }
  return acc;
}

// lane i <- lane i + 1 (DPP wave_shl:1; lanes past the end keep their own value)
__device__ __forceinline__ float x3_lane_next(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(x), __float_as_int(x), 0x130, 0xf, 0xf, false));
}

// v2 pooling: no conv tile in LDS (bias from LDS copy sb: a global load here
// would make the compiler wait for the next tile's prefetch, vmcnt(0)).  Waves mg = 0/1 own conv rows 0-4 / 4-8
// (row 4 twice: 5 rows each) = pooled rows 2mg, 2mg+1; the 3-wide column max
// runs across lanes (shuffles within each 32-lane half), the 3-tall row max
// in registers.  C layout: lane col jj = conv col, reg 4g+e -> channel
// 8g + 4h + e of this wave's 32.
__device__ __forceinline__ void x3_stem_pool_tile(const X3StemParams& p, const uint16_t* Ih, const uint16_t* Il,
                                                  const float* sb,
                                                  const v4u (&wh)[kSK / 16], const v4u (&wl)[kSK / 16], int img,
                                                  int pr0, int pc0, int lane, int wave) {
  const int nh = wave & 1, mg = wave >> 1;
  const int jj = lane & 31, hh = lane >> 5;
  const float ninf = -3.0e38f;
  f32x16 pm[2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) pm[i][e] = ninf;
  const bool left_pad = pc0 == 0 && jj == 0;  // conv col -1
#pragma unroll 1
  for (int r = 0; r < 5; ++r) {
    const int cr = 4 * mg + r;
    f32x16 acc = x3_stem_conv_row(Ih, Il, wh, wl, cr, lane);
    if (left_pad) {
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = ninf;
    }
    // column max over conv cols jj, jj+1, jj+2 (read by even lanes jj = 2b <
    // 28, so the shift never needs a lane of the other 32-lane half)
    f32x16 cm;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const float a1 = x3_lane_next(acc[e]), a2 = x3_lane_next(a1);
      cm[e] = fmaxf(acc[e], fmaxf(a1, a2));
    }
    if (pr0 == 0 && cr == 0) continue;  // conv row -1 (top padding)
    if (r <= 2) {
#pragma unroll
      for (int e = 0; e < 16; ++e) pm[0][e] = fmaxf(pm[0][e], cm[e]);
    }
    if (r >= 2) {
#pragma unroll
      for (int e = 0; e < 16; ++e) pm[1][e] = fmaxf(pm[1][e], cm[e]);
    }
  }
  if ((jj & 1) == 0 && jj < 2 * kSPC) {
    const int pc = pc0 + (jj >> 1);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int pr = pr0 + 2 * mg + i;
      float* o = p.y + (((size_t)img * kSHo + pr) * kSHo + pc) * p.ldy + nh * 32 + 4 * hh;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 bb = *reinterpret_cast<const f32x4*>(sb + nh * 32 + 8 * g + 4 * hh);
        *reinterpret_cast<f32x4*>(o + 8 * g) =
            f32x4{fmaxf(pm[i][4 * g] + bb[0], 0.f), fmaxf(pm[i][4 * g + 1] + bb[1], 0.f),
                  fmaxf(pm[i][4 * g + 2] + bb[2], 0.f), fmaxf(pm[i][4 * g + 3] + bb[3], 0.f)};
      }
    }
  }
}

// K10x stem v3: persistent.  A block loads its waves' weight fragments once
// and walks tiles t = blockIdx.x, +gridDim.x, ...; the next tile's input
// patch is loaded into registers while the current tile's conv rows run on
// MFMA, so neither the weight prologue nor the patch load sits on the
// critical path of every tile (v2 pays both per 4x14 tile).
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) x3_stem_p_kernel(X3StemParams p, int ntiles) {
  __shared__ __attribute__((aligned(16))) uint16_t Ih[kSIR * kSIC * 4];
  __shared__ __attribute__((aligned(16))) uint16_t Il[kSIR * kSIC * 4];
  __shared__ __attribute__((aligned(16))) float sb[64];
  constexpr int kTX = kSHo / kSPC, kTY = kSHo / kSPR;  // 4 x 14 tiles per image
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid < 16) *reinterpret_cast<f32x4*>(sb + 4 * tid) = ldf4(p.bias + 4 * tid);
  v4u wh[kSK / 16], wl[kSK / 16];
  x3_stem_weights(p, lane, wave & 1, wh, wl);
  float v[kStage][3];
  int t = blockIdx.x;
  if (t < ntiles) {
    const int img = t / (kTX * kTY), r = t - img * kTX * kTY;
    x3_stem_load(p.srcs[img], (r / kTX) * kSPR, (r % kTX) * kSPC, tid, v);
  }
  for (; t < ntiles; t += gridDim.x) {
    const int img = t / (kTX * kTY), r = t - img * kTX * kTY;
    const int pr0 = (r / kTX) * kSPR, pc0 = (r % kTX) * kSPC;
    __syncthreads();  // the previous tile's conv rows are done with Ih/Il
    x3_stem_stage(Ih, Il, tid, v);
    __syncthreads();
    const int tn = t + gridDim.x;
    if (tn < ntiles) {
      const int imn = tn / (kTX * kTY), rn = tn - imn * kTX * kTY;
      x3_stem_load(p.srcs[imn], (rn / kTX) * kSPR, (rn % kTX) * kSPC, tid, v);
    }
    x3_stem_pool_tile(p, Ih, Il, sb, wh, wl, img, pr0, pc0, lane, wave);
  }
}

// ============================================================================
// K10x head: out[img][c] = mean_p relu(x[img][p][c]*s[c] + b[c])   (fp32)
// ============================================================================
// Head: relu(x * s + b) averaged over the HW pixels of each image.  Block =
// (image, 256-channel group); the 4 waves take every 4th pixel (4 pixel loads
// per lane in flight) and sum through LDS.  The first version (one block per
// image, each thread a serial pixel loop) paid an L2 round trip per pixel:
// 14 us at bs1, 1.4% of that forward.
__global__ void __launch_bounds__(256) x3_head_pool_kernel(const float* __restrict__ x, const float* __restrict__ s,
                                                           const float* __restrict__ b, float* __restrict__ out, int HW,
                                                           int C) {
  __shared__ f32x4 part[4][64];
  const int img = blockIdx.x, lane = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int c4 = blockIdx.y * 64 + lane;
  const bool live = c4 < C / 4;
  const int cc = live ? c4 : 0;
  const f32x4 sc = ldf4(s + cc * 4), bi = ldf4(b + cc * 4);
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  const float* xi = x + (size_t)img * HW * C + cc * 4;
  int q = ph;
  for (; q + 12 < HW; q += 16) {
    f32x4 f[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) f[u] = ldf4(xi + (size_t)(q + 4 * u) * C);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] += fmaxf(f[u][e] * sc[e] + bi[e], 0.f);
  }
  for (; q < HW; q += 4) {
    const f32x4 f = ldf4(xi + (size_t)q * C);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[e] += fmaxf(f[e] * sc[e] + bi[e], 0.f);
  }
  part[ph][lane] = acc;
  __syncthreads();
  if (ph == 0 && live) {
    const f32x4 t = part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane];
    *reinterpret_cast<f32x4*>(out + (size_t)img * C + c4 * 4) = t * (1.0f / (float)HW);
  }
}

__global__ void x3_split_kernel(const float* __restrict__ w, uint16_t* __restrict__ hi, uint16_t* __restrict__ lo,
                                size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    uint32_t h, l;
    split2(w[i], 0.f, h, l);
    hi[i] = (uint16_t)h;
    lo[i] = (uint16_t)l;
  }
}

bool aligned16(const void* q) { return ((uintptr_t)q & 15) == 0; }

}  // namespace

namespace {
// Tile plan of one 1x1 conv: BM 128 while that fills the chip, else BM 32
// with the whole K per block; split-K (partials + reduce) only when even
// 32-row tiles leave most CUs idle (7x7 layers, small batches).
struct X3Plan {
  int bm, tiles, splits, k_per_split;
};

X3Plan x3_plan(int M, int K, int N) {
  X3Plan pl;
  const int nt = std::max(1, N / kBN);
  const int big = ((M + 127) / 128) * nt;
  const int mid = ((M + 63) / 64) * nt;
  pl.bm = big >= 384 ? 128 : (mid >= 256 ? 64 : 32);
  const int force_bm = (int)tcamd::knob(tcamd::Knob::X3Bm);  // A/B knob for tools/x3_kbench.py
  if (force_bm == 32 || force_bm == 64 || force_bm == 128) pl.bm = force_bm;
  pl.tiles = ((M + pl.bm - 1) / pl.bm) * nt;
  pl.splits = 1;
  pl.k_per_split = K;
  // split-K when fewer tiles than TCAMD_X3_SPLITK_BELOW (192).  The cap: the
  // 3x3 that follows re-reads every split's partials of its band, so more
  // splits trade 1x1 parallelism for 3x3 staging.  4 measured best (bs1
  // 1.005 -> 0.975 ms, bs8 1.166 -> 1.082 ms vs uncapped, 8-16 splits;
  // profiles/r3_splitk_cap.log); TCAMD_X3_MAX_SPLITS overrides
  const int splitk_below = (int)tcamd::knob(tcamd::Knob::X3SplitkBelow);
  const int max_splits = std::max(1, (int)tcamd::knob(tcamd::Knob::X3MaxSplits));
  if (pl.tiles < splitk_below && K >= 4 * kBK) {
    const int steps = K / kBK;
    int want = std::min(std::min(steps / 2, (384 + pl.tiles - 1) / pl.tiles), max_splits);
    if (want > 1) {
      pl.k_per_split = ((steps + want - 1) / want) * kBK;
      pl.splits = (K + pl.k_per_split - 1) / pl.k_per_split;
    }
  }
  return pl;
}

template <bool POOL, bool SPLIT>
void launch_x3_1x1(const X3Plan& pl, const dim3& g, hipStream_t s, const X3Conv1x1Params& p) {
  if (pl.bm == 128) hipLaunchKernelGGL((x3_conv1x1_kernel<POOL, SPLIT, 128, 2, 1>), g, dim3(256), 0, s, p);
  // the pooled prologue holds 4 source rows per chunk: a shallower ring
  else if (pl.bm == 64) hipLaunchKernelGGL((x3_conv1x1_kernel<POOL, SPLIT, 64, 1, POOL ? 2 : 4>), g, dim3(256), 0, s, p);
  else hipLaunchKernelGGL((x3_conv1x1_kernel<POOL, SPLIT, 32, 1, POOL ? 2 : 4>), g, dim3(256), 0, s, p);
}
}  // namespace

static int x3_conv1x1_impl(const float* x, int ldx, int M, int K, int N, const float* in_scale, const float* in_bias,
                           const void* w_hi, const void* w_lo, const float* out_bias, void* z_hi, void* z_lo,
                           float* y, int ldy, int pool, int H, int W, float* ws, size_t ws_bytes, void* stream,
                           int* defer_splits);

// part != null: the band comes from `splits` fp32 split-K partials [splits][M][128]
// plus part_bias (z_hi/z_lo unused)
static int x3_conv3x3_launch(const void* z_hi, const void* z_lo, const float* part, const float* part_bias, int splits,
                             int imgs, int H, int W, const void* w_hi, const void* w_lo, float* y, int ldy,
                             void* stream) {
  if (imgs <= 0) return hipSuccess;
  if (W > kMaxW3 || W < 1 || H < 1 || ldy % 4 || !w_hi || !w_lo || !y) return hipErrorInvalidValue;
  if (part ? (!part_bias || splits < 1 || !aligned16(part) || !aligned16(part_bias))
           : (!z_hi || !z_lo || !aligned16(z_hi) || !aligned16(z_lo)))
    return hipErrorInvalidValue;
  if (!aligned16(w_hi) || !aligned16(w_lo) || !aligned16(y)) return hipErrorInvalidValue;
  X3Conv3x3Params p;
  p.z_hi = (const uint16_t*)z_hi;
  p.z_lo = (const uint16_t*)z_lo;
  p.w_hi = (const uint16_t*)w_hi;
  p.w_lo = (const uint16_t*)w_lo;
  p.part = part;
  p.part_bias = part_bias;
  p.splits = splits;
  p.y = y;
  p.ldy = ldy;
  p.M = imgs * H * W;
  p.H = H;
  p.W = W;
  p.mag_hw = (uint32_t)((0x100000000ull + H * W - 1) / (uint64_t)(H * W));
  p.mag_w = (uint32_t)((0x100000000ull + W - 1) / (uint64_t)W);
  if (p.M >= (1 << 24)) return hipErrorInvalidValue;  // fast_divmod range
  // one block (8 waves) per CU; each walks a contiguous run of tiles so the
  // halo rows its neighbour tile re-reads are still in this XCD's L2
  // the dynamic-LDS opt-in is per device; it is cached only once every call succeeded
  static std::atomic<bool> attr_set[kMaxDevices];
  const int dev_slot = device_slot();
  if (!attr_set[dev_slot].load(std::memory_order_acquire)) {
    hipError_t e = hipFuncSetAttribute((const void*)x3_conv3x3_v2_kernel<false>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, kLdsV2);
    if (e == hipSuccess)
      e = hipFuncSetAttribute((const void*)x3_conv3x3_v2_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              kLdsV2);
    if (e != hipSuccess) return e;
    attr_set[dev_slot].store(true, std::memory_order_release);
  }
  p.tiles = (p.M + kT2 - 1) / kT2;
  const int grid = std::min(p.tiles, 256);
  p.tiles_per_block = (p.tiles + grid - 1) / grid;
  const int blocks = (p.tiles + p.tiles_per_block - 1) / p.tiles_per_block;
  if (part)
    hipLaunchKernelGGL((x3_conv3x3_v2_kernel<true>), dim3(blocks), dim3(512), kLdsV2, (hipStream_t)stream, p);
  else hipLaunchKernelGGL((x3_conv3x3_v2_kernel<false>), dim3(blocks), dim3(512), kLdsV2, (hipStream_t)stream, p);
  return hipGetLastError();
}

extern "C" {

// Split-K workspace bytes the 1x1 conv wants for an M x K -> N problem (0 = none).
size_t tcamd_x3_conv1x1_ws_bytes(int M, int K, int N) {
  const X3Plan pl = x3_plan(M, K, N);
  return pl.splits > 1 ? (size_t)pl.splits * M * N * sizeof(float) : 0;
}

// 1x1 conv, N output channels (a multiple of 128).  split_out: z_hi/z_lo
// [M][128] bf16 with bias+ReLU (N = 128); else y fp32 [M][ldy] raw.  pool: x
// holds the pre-pool H x W pixels, M = imgs * H/2 * W/2.  ws: split-K
// workspace (may be null: then the whole K runs in each block).
int tcamd_x3_conv1x1(const float* x, int ldx, int M, int K, int N, const float* in_scale, const float* in_bias,
                     const void* w_hi, const void* w_lo, const float* out_bias, void* z_hi, void* z_lo, float* y,
                     int ldy, int pool, int H, int W, float* ws, size_t ws_bytes, void* stream) {
  return x3_conv1x1_impl(x, ldx, M, K, N, in_scale, in_bias, w_hi, w_lo, out_bias, z_hi, z_lo, y, ldy, pool, H, W,
                         ws, ws_bytes, stream, nullptr);
}

}  // extern "C"

// The 1x1 of the host entry points.  defer_splits != null: a split-K plan
// leaves its fp32 partials in ws WITHOUT the reduce launch and reports the
// split count there (1 = no split: z was written as usual).
static int x3_conv1x1_impl(const float* x, int ldx, int M, int K, int N, const float* in_scale, const float* in_bias,
                           const void* w_hi, const void* w_lo, const float* out_bias, void* z_hi, void* z_lo,
                           float* y, int ldy, int pool, int H, int W, float* ws, size_t ws_bytes, void* stream,
                           int* defer_splits) {
  if (defer_splits) *defer_splits = 1;
  if (M <= 0) return hipSuccess;
  const bool split_out = z_hi != nullptr;
  if (K % kBK || K <= 0 || ldx % 4 || ldx < K || !x || !in_scale || !in_bias || !w_hi || !w_lo)
    return hipErrorInvalidValue;
  if (N <= 0 || N % kBN) return hipErrorInvalidValue;
  if (split_out ? (N != kBN || !z_lo || !out_bias || !aligned16(z_hi) || !aligned16(z_lo))
                : (!y || ldy % 4 || ldy < N || !aligned16(y)))
    return hipErrorInvalidValue;
  if (!aligned16(x) || !aligned16(w_hi) || !aligned16(w_lo) || !aligned16(in_scale) || !aligned16(in_bias))
    return hipErrorInvalidValue;
  if (pool && (H % 2 || W % 2 || (size_t)M % ((size_t)(H / 2) * (W / 2)))) return hipErrorInvalidValue;
  X3Conv1x1Params p;
  p.x = x;
  p.in_scale = in_scale;
  p.in_bias = in_bias;
  p.w_hi = (const uint16_t*)w_hi;
  p.w_lo = (const uint16_t*)w_lo;
  p.out_bias = out_bias;
  p.z_hi = (uint16_t*)z_hi;
  p.z_lo = (uint16_t*)z_lo;
  p.y = y;
  p.ws = nullptr;
  p.ldx = ldx;
  p.M = M;
  p.K = K;
  p.N = N;
  p.ldy = ldy;
  p.H = H;
  p.W = W;
  X3Plan pl = x3_plan(M, K, N);
  if (pl.splits > 1 && ws && ws_bytes >= (size_t)pl.splits * M * N * sizeof(float) && aligned16(ws)) {
    p.ws = ws;
    p.k_per_split = pl.k_per_split;
  } else {
    pl.splits = 1;
    p.k_per_split = K;
  }
  hipStream_t s = (hipStream_t)stream;
  // warp-specialised persistent kernel for the big dense-layer 1x1s
  // (TCAMD_X3_WS=0 turns it off, TCAMD_X3_WS_MIN moves its M floor: A/B runs)
  if (tcamd::knob(tcamd::Knob::X3Ws) && !pool && split_out && N == kBN && M >= tcamd::knob(tcamd::Knob::X3WsMin)) {
    // per device: the CU count and the dynamic-LDS opt-in, cached only after
    // every attribute call succeeded (a failed setup is retried, never launched)
    static std::atomic<int> ncu_dev[kMaxDevices];
    const int dev_slot = device_slot();
    int ncu = ncu_dev[dev_slot].load(std::memory_order_acquire);
    if (!ncu) {
      int dev = 0, n = 0;
      hipError_t e = hipGetDevice(&dev);
      if (e == hipSuccess) e = hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
      if (e == hipSuccess && n <= 0) e = hipErrorInvalidDevice;
      if (e == hipSuccess)
        e = hipFuncSetAttribute((const void*)x3_conv1x1_ws_kernel<3>, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsWs);
      if (e != hipSuccess) return e;
      ncu = n;
      ncu_dev[dev_slot].store(ncu, std::memory_order_release);
    }
    X3WsParams wp;
    wp.c = p;
    const int units = (M + 15) / 16;
    wp.units_per_block = (units + ncu - 1) / ncu;
    // equal tiles: 392 rows -> 4 x 98 instead of 3 x 128 + 8 (every tile
    // costs nst barrier rounds whatever its row count)
    const int rpb = 16 * wp.units_per_block;
    const int nt = (rpb + 127) / 128;
    wp.tile_rows = (rpb + nt - 1) / nt;
    const int blocks = (units + wp.units_per_block - 1) / wp.units_per_block;
    hipLaunchKernelGGL((x3_conv1x1_ws_kernel<3>), dim3(blocks), dim3(512), kLdsWs, s, wp);
    return hipGetLastError();
  }
  const int mb = (M + pl.bm - 1) / pl.bm, ntl = N / kBN;
  p.xcd_group = (ntl > 1 && pl.splits == 1) ? 1 : 0;
  const dim3 g = p.xcd_group ? dim3((mb + 7) / 8 * 8 * ntl, 1, 1) : dim3(mb, pl.splits, ntl);
  if (pool) {
    if (split_out) launch_x3_1x1<true, true>(pl, g, s, p);
    else launch_x3_1x1<true, false>(pl, g, s, p);
  } else {
    if (split_out) launch_x3_1x1<false, true>(pl, g, s, p);
    else launch_x3_1x1<false, false>(pl, g, s, p);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !p.ws) return e;
  if (defer_splits && split_out) {
    *defer_splits = pl.splits;  // the 3x3 sums the partials while staging its band
    return hipSuccess;
  }
  const int rg = tcamd::grid_for((size_t)M * (N / 4));
  if (split_out) hipLaunchKernelGGL(x3_splitk_reduce_kernel<true>, dim3(rg), dim3(256), 0, s, p, pl.splits);
  else hipLaunchKernelGGL(x3_splitk_reduce_kernel<false>, dim3(rg), dim3(256), 0, s, p, pl.splits);
  return hipGetLastError();
}

extern "C" {

// 3x3 conv 128 -> 32 over imgs x H x W pixels (W <= 56); z_hi/z_lo [M][128]
// bf16, w_hi/w_lo [32][9][128] bf16, y fp32 rows of ldy (offset to the slice).
int tcamd_x3_conv3x3(const void* z_hi, const void* z_lo, int imgs, int H, int W, const void* w_hi, const void* w_lo,
                     float* y, int ldy, void* stream) {
  return x3_conv3x3_launch(z_hi, z_lo, nullptr, nullptr, 0, imgs, H, W, w_hi, w_lo, y, ldy, stream);
}

// One dense layer: BN1+ReLU+1x1 (K -> 128) then the 3x3 (128 -> 32) into the
// layer's slice of the block buffer.  When the 1x1 plans split-K (small M)
// its partials go straight to the 3x3, which reduces them while staging its
// band (no reduce launch, z never written).
int tcamd_x3_dense_layer(const float* x, int ldx, int imgs, int H, int W, int K, const float* s1, const float* t1,
                         const void* w1_hi, const void* w1_lo, const float* b1, void* z_hi, void* z_lo,
                         const void* w2_hi, const void* w2_lo, float* y, int ldy, float* ws, size_t ws_bytes,
                         void* stream) {
  int splits = 1;
  int e = x3_conv1x1_impl(x, ldx, imgs * H * W, K, kBN, s1, t1, w1_hi, w1_lo, b1, z_hi, z_lo, nullptr, 0, 0, 0, 0,
                          ws, ws_bytes, stream, &splits);
  if (e != hipSuccess) return e;
  if (splits > 1) return x3_conv3x3_launch(nullptr, nullptr, ws, b1, splits, imgs, H, W, w2_hi, w2_lo, y, ldy, stream);
  return x3_conv3x3_launch(z_hi, z_lo, nullptr, nullptr, 0, imgs, H, W, w2_hi, w2_lo, y, ldy, stream);
}

static int cu_count();

// K11x: the whole dense layer in one kernel (z stays in LDS).  v 1: the
// 8-wave kernel; v 3: v1 with the next chunk's 1x1 interleaved into each
// tile's 3x3.  w1 in x3_w1_fragments, w2 in x3_w3f_fragments; 16 <= W <= 56,
// K in 64..480.
static int x3_dense_fused_impl(int v, const float* x, int ldx, int imgs, int H, int W, int K, const float* s1,
                               const float* t1, const void* w1_hi, const void* w1_lo, const float* b1,
                               const void* w2_hi, const void* w2_lo, float* y, int ldy, void* stream) {
  if (imgs <= 0) return hipSuccess;
  if (W > kMaxW3 || W < 16 || H < 1 || K <= 0 || K % 32 || K > kMaxKF || ldx < K || ldx % 4 || ldy % 4)
    return hipErrorInvalidValue;
  if (!x || !s1 || !t1 || !w1_hi || !w1_lo || !b1 || !w2_hi || !w2_lo || !y) return hipErrorInvalidValue;
  if (!aligned16(x) || !aligned16(s1) || !aligned16(t1) || !aligned16(w1_hi) || !aligned16(w1_lo) ||
      !aligned16(b1) || !aligned16(w2_hi) || !aligned16(w2_lo) || !aligned16(y))
    return hipErrorInvalidValue;
  X3FusedParams p;
  p.x = x;
  p.s1 = s1;
  p.t1 = t1;
  p.w1_hi = (const uint16_t*)w1_hi;
  p.w1_lo = (const uint16_t*)w1_lo;
  p.b1 = b1;
  p.w2_hi = (const uint16_t*)w2_hi;
  p.w2_lo = (const uint16_t*)w2_lo;
  p.y = y;
  p.ldx = ldx;
  p.K = K;
  p.ldy = ldy;
  p.M = imgs * H * W;
  p.H = H;
  p.W = W;
  if (p.M >= (1 << 24) - 2 * kRingF) return hipErrorInvalidValue;  // fast_divmod range
  p.mag_hw = (uint32_t)((0x100000000ull + H * W - 1) / (uint64_t)(H * W));
  p.mag_w = (uint32_t)((0x100000000ull + W - 1) / (uint64_t)W);
  // NST 2..15 (K 64..480; the BN1 affine table in LDS holds K <= 480).  v1
  // at NST 15 spills 12 B per lane; measured per K before the engine uses it
#define X3F_ROW(KERN)                                                                                  \
  {(const void*)KERN<2>,  (const void*)KERN<3>,  (const void*)KERN<4>,  (const void*)KERN<5>,  (const void*)KERN<6>, \
   (const void*)KERN<7>,  (const void*)KERN<8>,  (const void*)KERN<9>,  (const void*)KERN<10>, (const void*)KERN<11>, \
   (const void*)KERN<12>, (const void*)KERN<13>, (const void*)KERN<14>, (const void*)KERN<15>}
  // [version 1 / 3 / 5 (K11w)][NST - 2]
  static const void* const kFns[3][14] = {X3F_ROW(x3_dense_fused_kernel), X3F_ROW(x3_dense_fused3_kernel),
                                          X3F_ROW(x3_dense_ws_kernel)};
#undef X3F_ROW
  const int nst = K / 32;
  if (nst < 2 || nst > 15 || (v != 1 && v != 3 && v != 5)) return hipErrorInvalidValue;
  static std::atomic<bool> attr_set[kMaxDevices];
  const int dev_slot = device_slot();
  if (!attr_set[dev_slot].load(std::memory_order_acquire)) {
    for (const auto& fs : kFns)
      for (const void* f : fs) {
        const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsF3);
        if (e != hipSuccess) return e;
      }
    attr_set[dev_slot].store(true, std::memory_order_release);
  }
  p.tiles = (p.M + kT2 - 1) / kT2;
  const int grid = std::min(p.tiles, cu_count());
  p.tiles_per_block = (p.tiles + grid - 1) / grid;
  const int blocks = (p.tiles + p.tiles_per_block - 1) / p.tiles_per_block;
  void* args[] = {&p};
  const int vi = v == 1 ? 0 : (v == 3 ? 1 : 2);
  const hipError_t e = hipLaunchKernel(kFns[vi][nst - 2], dim3(blocks), dim3(v == 5 ? 768 : 512), args,
                                       v == 1 ? kLdsF : (v == 3 ? kLdsF3 : kLdsFW), (hipStream_t)stream);
  if (e != hipSuccess) return e;
  return hipGetLastError();
}

int tcamd_x3_dense_fused(const float* x, int ldx, int imgs, int H, int W, int K, const float* s1, const float* t1,
                         const void* w1_hi, const void* w1_lo, const float* b1, const void* w2_hi, const void* w2_lo,
                         float* y, int ldy, void* stream) {
  return x3_dense_fused_impl(1, x, ldx, imgs, H, W, K, s1, t1, w1_hi, w1_lo, b1, w2_hi, w2_lo, y, ldy, stream);
}

// K11x v3: v1's roles and weight layouts (x3_w3f_fragments), the next chunk's
// 1x1 interleaved into each tile's 3x3
int tcamd_x3_dense_fused3(const float* x, int ldx, int imgs, int H, int W, int K, const float* s1, const float* t1,
                          const void* w1_hi, const void* w1_lo, const float* b1, const void* w2_hi,
                          const void* w2_lo, float* y, int ldy, void* stream) {
  return x3_dense_fused_impl(3, x, ldx, imgs, H, W, K, s1, t1, w1_hi, w1_lo, b1, w2_hi, w2_lo, y, ldy, stream);
}

// K11w: v1's layer with producer / consumer waves (768 threads); same inputs.
int tcamd_x3_dense_fused_ws(const float* x, int ldx, int imgs, int H, int W, int K, const float* s1, const float* t1,
                            const void* w1_hi, const void* w1_lo, const float* b1, const void* w2_hi,
                            const void* w2_lo, float* y, int ldy, void* stream) {
  return x3_dense_fused_impl(5, x, ldx, imgs, H, W, K, s1, t1, w1_hi, w1_lo, b1, w2_hi, w2_lo, y, ldy, stream);
}


static int cu_count();

// Tiles per image K14x uses for imgs images of side W when the caller passes
// tiles <= 0: the fewest (least halo recompute) that give every CU a
// workgroup; 14x14: 2 (half images) or 4, 7x7: 1 (whole images), 2 or 4.
int tcamd_x3_small_tiles(int imgs, int W) {
  const int ncu = cu_count();
  const int opts14[2] = {2, 4}, opts7[3] = {1, 2, 4};
  const int* o = W == 14 ? opts14 : opts7;
  const int n = W == 14 ? 2 : 3;
  const int padded = (imgs + 7) / 8 * 8;
  for (int i = 0; i < n; ++i)
    if (padded * o[i] >= ncu) return o[i];
  // 14x14 images too few to fill the CUs with quarters: 2-row tiles (7 per
  // image) while they still fit one round (bs8-32: -20..23 % per layer; at 7x7
  // a 7-way split gains nothing; profiles/r5_k14x_tiles.md)
  if (W == 14 && padded * 7 <= ncu) return 7;
  return o[n - 1];
}

// K14x: one dense layer of the 14x14 or 7x7 block in one kernel, `tiles`
// tiles per image (14x14: 2, 4 or 7, 7x7: 1, 2, 4 or 7; <= 0: the chip-filling
// default above); w1 in x3_w1_fragments, w2 in x3_w3f_fragments.  K a
// multiple of 32 in 64..2048.
int tcamd_x3_dense_small(const float* x, int ldx, int imgs, int H, int W, int K, const float* s1, const float* t1,
                         const void* w1f_hi, const void* w1f_lo, const float* b1, const void* w2_hi,
                         const void* w2_lo, float* y, int ldy, int tiles, void* stream) {
  if (imgs <= 0) return hipSuccess;
  if ((W != 14 && W != 7) || H != W || K < 64 || K > 2048 || K % 32 || ldx < K || ldx % 4 || ldy % 4)
    return hipErrorInvalidValue;
  if (!x || !s1 || !t1 || !w1f_hi || !w1f_lo || !b1 || !w2_hi || !w2_lo || !y) return hipErrorInvalidValue;
  if (!aligned16(x) || !aligned16(s1) || !aligned16(t1) || !aligned16(w1f_hi) || !aligned16(w1f_lo) ||
      !aligned16(b1) || !aligned16(w2_hi) || !aligned16(w2_lo) || !aligned16(y))
    return hipErrorInvalidValue;
  if ((size_t)imgs * H * W >= (1u << 30) / 4) return hipErrorInvalidValue;
  if (tiles <= 0) tiles = tcamd_x3_small_tiles(imgs, W);
  const int ti = tiles == 1 ? 0 : tiles == 2 ? 1 : tiles == 4 ? 2 : tiles == 7 ? 3 : -1;
  if (ti < 0 || (W == 14 && ti == 0)) return hipErrorInvalidValue;
  X3SmallParams p;
  p.x = x;
  p.s1 = s1;
  p.t1 = t1;
  p.w1f_hi = (const uint16_t*)w1f_hi;
  p.w1f_lo = (const uint16_t*)w1f_lo;
  p.b1 = b1;
  p.w2_hi = (const uint16_t*)w2_hi;
  p.w2_lo = (const uint16_t*)w2_lo;
  p.y = y;
  p.ldx = ldx;
  p.K = K;
  p.ldy = ldy;
  p.imgs = imgs;
  // [14x14 / 7x7][1 / 2 / 4 / 7 tiles per image]
  const void* const fns[2][4] = {
      {nullptr, (const void*)x3_dense_small_kernel<14, 2>, (const void*)x3_dense_small_kernel<14, 4>,
       (const void*)x3_dense_small_kernel<14, 7>},
      {(const void*)x3_dense_small_kernel<7, 1>, (const void*)x3_dense_small_kernel<7, 2>,
       (const void*)x3_dense_small_kernel<7, 4>, (const void*)x3_dense_small_kernel<7, 7>}};
  constexpr int kLds = 4 * kWsStage;  // 4 K-step stages
  static std::atomic<bool> attr_set[kMaxDevices];
  const int dev_slot = device_slot();
  if (!attr_set[dev_slot].load(std::memory_order_acquire)) {
    for (const auto& row : fns)
      for (const void* f : row) {
        if (!f) continue;
        const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kLds);
        if (e != hipSuccess) return e;
      }
    attr_set[dev_slot].store(true, std::memory_order_release);
  }
  const int blocks = (imgs + 7) / 8 * 8 * tiles;
  void* args[] = {&p};
  const hipError_t e = hipLaunchKernel(fns[W == 14 ? 0 : 1][ti], dim3(blocks), dim3(512), args, kLds,
                                       (hipStream_t)stream);
  if (e != hipSuccess) return e;
  return hipGetLastError();
}


static int cu_count() {
  static std::atomic<int> ncu_dev[kMaxDevices];
  const int dev_slot = device_slot();
  int ncu = ncu_dev[dev_slot].load(std::memory_order_acquire);
  if (!ncu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
      ncu = 256;
    ncu_dev[dev_slot].store(ncu, std::memory_order_release);
  }
  return ncu;
}

// fp32 stem over fp32 NCHW 224x224x3 images (device pointer table srcs)
// -> y fp32 [imgs][56][56] rows of ldy (channels 0..63).
int tcamd_x3_stem(const void* srcs, const void* w_hi, const void* w_lo, const float* bias, float* y, int imgs, int ldy,
                  void* stream) {
  if (imgs <= 0) return hipSuccess;
  if (ldy % 4 || ldy < 64 || !srcs || !w_hi || !w_lo || !bias || !y) return hipErrorInvalidValue;
  if (!aligned16(w_hi) || !aligned16(w_lo) || !aligned16(y) || !aligned16(bias) || (uintptr_t)srcs % 8)
    return hipErrorInvalidValue;
  X3StemParams p;
  p.srcs = (const float* const*)srcs;
  p.w_hi = (const uint16_t*)w_hi;
  p.w_lo = (const uint16_t*)w_lo;
  p.bias = bias;
  p.y = y;
  p.ldy = ldy;
  // persistent: TCAMD_X3_STEM_BPC workgroups per CU walk the 4 x 14 tiles of every image
  const int bpc = std::max(1, (int)tcamd::knob(tcamd::Knob::X3StemBpc));
  const int ntiles = (kSHo / kSPC) * (kSHo / kSPR) * imgs;
  const int grid = std::min(ntiles, bpc * cu_count());
  hipLaunchKernelGGL(x3_stem_p_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, p, ntiles);
  return hipGetLastError();
}

int tcamd_x3_head_pool(const float* x, const float* s, const float* b, float* out, int imgs, int HW, int C,
                       void* stream) {
  if (imgs <= 0) return hipSuccess;
  if (C % 4 || !aligned16(x) || !aligned16(s) || !aligned16(b) || !aligned16(out)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(x3_head_pool_kernel, dim3(imgs, (C / 4 + 63) / 64), dim3(256), 0, (hipStream_t)stream, x, s, b,
                     out, HW, C);
  return hipGetLastError();
}

int tcamd_x3_split(const float* w, void* hi, void* lo, size_t n, void* stream) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(x3_split_kernel, dim3(tcamd::grid_for(n)), dim3(256), 0, (hipStream_t)stream, w, (uint16_t*)hi,
                     (uint16_t*)lo, n);
  return hipGetLastError();
}

}  // extern "C"
