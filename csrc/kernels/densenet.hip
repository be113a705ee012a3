// K8/K9/K10 — fused DenseNet-121 inference kernels for CDNA4 (gfx950).
//
// The reference serves `densenet_onnx` through onnxruntime in the server
// (reference src/python/examples/image_client.py:86-152 and
// src/c++/perf_analyzer docs name it as the headline model); here the model
// runs on hand-written MFMA kernels whose layout is chosen for the hardware
// instead of per-op library calls:
//
//  * every dense block owns ONE NHWC bf16 feature buffer [pixels][C_block];
//    each layer's 3x3 conv writes its 32 new channels straight into its slice
//    (no torch.cat: the concat is free), and the next layer's 1x1 conv reads
//    the first K channels of the same rows;
//  * K8 conv1x1: Y = epi( relu(X*s+b) @ W^T ) — the pre-activation BN+ReLU
//    of DenseNet (different per consumer layer, so it cannot be folded into
//    a producer) is applied while staging the X tile global->LDS, the
//    following BN (norm2) is folded into W/bias and applied with ReLU in the
//    epilogue.  POOL=true is the transition layer: BN+ReLU+2x2 avg-pool in
//    the prologue, 4x fewer GEMM rows;
//  * K9 conv3x3 (128->32, pad 1): implicit GEMM, the whole 73 KB weight
//    tensor resident in LDS for a persistent block, activations fetched
//    with bounds-checked buffer loads (out-of-image taps read as 0); the
//    default for M > 8192 is K9w2: the activation band lives in a 256-row
//    LDS ring sliding over a contiguous run of tiles (128 new rows per
//    tile) and 8 waves, two per SIMD, split the nine taps;
//  * K10 stem epilogue (bias+ReLU+3x3/2 max-pool) and head (BN+ReLU+global
//    avg-pool).
//
// MFMA: v_mfma_f32_16x16x32_bf16 with the WEIGHT tile as operand A (rows =
// output channels) and the activation tile as operand B (cols = pixels), so
// each lane's 4 accumulators are 4 consecutive output channels of one pixel
// and the epilogue stores 8 contiguous bytes per lane with no LDS transpose.

#include <algorithm>

#include "kernels/common.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));

constexpr int kMaxK = 1024;      // prologue scale/bias table
constexpr int kC3 = 128;         // 3x3 conv input channels (bn_size * growth)
constexpr int kN3 = 32;          // 3x3 conv output channels (growth)
constexpr int kK3 = 9 * kC3;     // 1152
constexpr int kWsK = kK3 + 8;    // LDS row stride of the resident 3x3 weights

__device__ __forceinline__ v4u ldg16(const uint16_t* p) { return *reinterpret_cast<const v4u*>(p); }

__device__ __forceinline__ void unpack8(v4u v, float* f) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f[2 * q] = __uint_as_float(v[q] << 16);
    f[2 * q + 1] = __uint_as_float(v[q] & 0xffff0000u);
  }
}

// two fp32 -> packed bf16 (RNE) in ONE instruction: gfx950's v_cvt_pk_bf16_f32
// (the software RNE costs ~6 VALU per element; this runs in every prologue
// and epilogue of the engine)
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  const bf16x2 v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}

// ReLU on two packed bf16 values as ONE v_pk_max_i16: a bf16 with the sign
// bit set is a negative int16, so max(x, 0) in int16 zeroes exactly the
// negative (and -0 / negative-NaN) halves.  relu(bf16(x)) == bf16(relu(x)).
typedef short s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t relu_pk(uint32_t v) {
  const s16x2 z = {0, 0};
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s16x2, v), z));
}

__device__ __forceinline__ v4u pack8(const float* f) {
  v4u v;
#pragma unroll
  for (int q = 0; q < 4; ++q) v[q] = pack2(f[2 * q], f[2 * q + 1]);
  return v;
}

__device__ __forceinline__ bf16x8 as_frag(v4u v) { return __builtin_bit_cast(bf16x8, v); }

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// ============================================================================
// K8: 1x1 conv as GEMM with fused pre-activation (and optional 2x2 avg-pool)
// ============================================================================
struct Conv1x1Params {
  const uint16_t* x;        // [rows][ldx] bf16 (rows = M, or the pre-pool pixels)
  const float* in_scale;    // [K] prologue BN scale (PRO)
  const float* in_bias;     // [K]
  const uint16_t* w;        // [N][K] bf16
  const float* out_bias;    // [N] or null
  uint16_t* y;              // [M][ldy] bf16, already offset to the first output channel
  int ldx, M, K, N, ldy;
  int relu_out;
  int H, W;                 // POOL: pre-pool spatial dims (M = imgs * H/2 * W/2)
  float* ws;                // split-K: fp32 partials [splits][M][N] (null = no split)
  int k_per_split;          // K range per blockIdx.z (multiple of BK)
};

// Block = 4 waves as 2 (pixels) x 2 (channels); block tile (32*TM) x 128,
// wave tile (16*TM pixels) x 64 channels, K tile BK (32 or 64), LDS
// double-buffered with register prefetch (global loads of tile k+1 are in
// flight during the MFMAs on tile k).  K need not be a multiple of BK: the
// tail chunk is zero-filled (K % 32 == 0 always holds).
template <int TM, int BK, bool PRO, bool POOL, int BN = 128>
__global__ void __launch_bounds__(256) conv1x1_kernel(Conv1x1Params p) {
  constexpr int BM = 32 * TM, NJ = BN / 32, WN = BN / 2;  // wave: 16*TM pixels x BN/2 channels
  constexpr int CPR = BK / 8;                 // 16-B chunks per row of a K tile
  constexpr int LDK = BK + 8;                 // LDS row stride (elements): conflict-free b128 reads
  constexpr int A_CHUNKS = BM * CPR, AI = (A_CHUNKS + 255) / 256;
  constexpr int BI = (BN * CPR + 255) / 256;
  static_assert(BN * CPR % 256 == 0, "B chunks per thread");
  constexpr int NS = POOL ? 4 : 1;
  __shared__ __attribute__((aligned(16))) uint16_t sA[2][BM * LDK];
  __shared__ __attribute__((aligned(16))) uint16_t sB[2][BN * LDK];
  __shared__ float sS[PRO ? kMaxK : 1], sT[PRO ? kMaxK : 1];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  if constexpr (PRO) {
    for (int k = tid; k < p.K; k += 256) {
      sS[k] = p.in_scale[k];
      sT[k] = p.in_bias[k];
    }
  }

  // per-thread A chunk sources (row pointers; POOL: the 2x2 window's 4 rows)
  const uint16_t* a_src[AI][NS];
  bool a_ok[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int c = tid + i * 256;
    const int m = m0 + c / CPR;
    a_ok[i] = (c < A_CHUNKS) && (m < p.M);
    const int mm = a_ok[i] ? m : 0;
    const int kc = (c % CPR) * 8;
    if constexpr (POOL) {
      const int wo = p.W >> 1, ho = p.H >> 1;
      const int img = mm / (ho * wo), r = mm - img * ho * wo;
      const int oh = r / wo, ow = r - oh * wo;
      const size_t base = ((size_t)img * p.H + 2 * oh) * p.W + 2 * ow;
      a_src[i][0] = p.x + base * p.ldx + kc;
      a_src[i][1] = p.x + (base + 1) * p.ldx + kc;
      a_src[i][2] = p.x + (base + p.W) * p.ldx + kc;
      a_src[i][3] = p.x + (base + p.W + 1) * p.ldx + kc;
    } else {
      a_src[i][0] = p.x + (size_t)mm * p.ldx + kc;
    }
  }
  const uint16_t* b_src[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int c = tid + i * 256;
    b_src[i] = p.w + (size_t)(n0 + c / CPR) * p.K + (c % CPR) * 8;
  }

  v4u ra[AI][NS], rb[BI];
  auto load_tile = [&](int kt) {
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int kc = ((tid + i * 256) % CPR) * 8;
      const bool kin = BK == 32 || k0 + kc < p.K;
#pragma unroll
      for (int s = 0; s < NS; ++s) ra[i][s] = kin ? ldg16(a_src[i][s] + k0) : v4u{0, 0, 0, 0};
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int kc = ((tid + i * 256) % CPR) * 8;
      rb[i] = (BK == 32 || k0 + kc < p.K) ? ldg16(b_src[i] + k0) : v4u{0, 0, 0, 0};
    }
  };
  auto store_tile = [&](int kt, int buf) {
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int c = tid + i * 256;
      if (c < A_CHUNKS) {
        const int kc = (c % CPR) * 8;
        const bool kin = BK == 32 || k0 + kc < p.K;
        v4u v;
        if constexpr (PRO) {
          float o[8];
          if (kin) {
#pragma unroll
            for (int s = 0; s < NS; ++s) {
              float f[8];
              unpack8(ra[i][s], f);
#pragma unroll
              for (int e = 0; e < 8; ++e) {
                const float t = f[e] * sS[k0 + kc + e] + sT[k0 + kc + e];
                // pool: average of ReLUs (fp32); plain: ReLU after the pack, packed
                // (no "0 + t" either: IEEE forbids folding it away)
                if constexpr (POOL) o[e] = s ? o[e] + 0.25f * fmaxf(t, 0.f) : 0.25f * fmaxf(t, 0.f);
                else o[e] = t;
              }
            }
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = 0.f;
          }
          v = pack8(o);
          if constexpr (!POOL) {
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = relu_pk(v[q]);
          }
        } else {
          v = ra[i][0];
        }
        if (!a_ok[i] || !kin) v = v4u{0, 0, 0, 0};
        *reinterpret_cast<v4u*>(&sA[buf][(c / CPR) * LDK + kc]) = v;
      }
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int c = tid + i * 256;
      *reinterpret_cast<v4u*>(&sB[buf][(c / CPR) * LDK + (c % CPR) * 8]) = rb[i];
    }
  };

  // the output bias starts the accumulators (split-K adds it in the reduce)
  f32x4 acc[NJ][TM];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    f32x4 b0 = f32x4{0.f, 0.f, 0.f, 0.f};
    if (p.out_bias && !p.ws) {
      const int nb = n0 + wn * WN + j * 16 + (lane >> 4) * 4;
      b0 = f32x4{p.out_bias[nb], p.out_bias[nb + 1], p.out_bias[nb + 2], p.out_bias[nb + 3]};
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[j][i] = b0;
  }

  // K tiles of this block: all of K, or one split's range
  const int kt0 = p.ws ? (int)blockIdx.z * (p.k_per_split / BK) : 0;
  const int KT = p.ws ? min((p.K + BK - 1) / BK, kt0 + p.k_per_split / BK) : (p.K + BK - 1) / BK;
  load_tile(kt0);
  __syncthreads();  // prologue tables
  store_tile(kt0, 0);
  __syncthreads();
  const int fr = lane & 15, fk = 8 * (lane >> 4);
  for (int kt = kt0; kt < KT; ++kt) {
    const int buf = (kt - kt0) & 1;
    if (kt + 1 < KT) load_tile(kt + 1);
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8 fa[NJ], fb[TM];
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        fa[j] = *reinterpret_cast<const bf16x8*>(&sB[buf][(wn * WN + j * 16 + fr) * LDK + ks * 32 + fk]);
#pragma unroll
      for (int i = 0; i < TM; ++i)
        fb[i] = *reinterpret_cast<const bf16x8*>(&sA[buf][(wm * 16 * TM + i * 16 + fr) * LDK + ks * 32 + fk]);
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[j][i] = mfma16(fa[j], fb[i], acc[j][i]);
    }
    if (kt + 1 < KT) store_tile(kt + 1, buf ^ 1);
    __syncthreads();
  }

  if (p.ws) {  // split-K: raw fp32 partials, epilogue in dn_splitk_reduce
    float* ws = p.ws + (size_t)blockIdx.z * p.M * p.N;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int nb = n0 + wn * WN + j * 16 + (lane >> 4) * 4;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = m0 + wm * 16 * TM + i * 16 + fr;
        if (m < p.M) *reinterpret_cast<f32x4*>(ws + (size_t)m * p.N + nb) = acc[j][i];
      }
    }
    return;
  }
  // epilogue: lane holds out channels nb..nb+3 of pixel m (bias already in acc)
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int nb = n0 + wn * WN + j * 16 + (lane >> 4) * 4;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wm * 16 * TM + i * 16 + fr;
      if (m < p.M) {
        v2u o = v2u{pack2(acc[j][i][0], acc[j][i][1]), pack2(acc[j][i][2], acc[j][i][3])};
        if (p.relu_out) o = v2u{relu_pk(o[0]), relu_pk(o[1])};
        *reinterpret_cast<v2u*>(p.y + (size_t)m * p.ldy + nb) = o;
      }
    }
  }
}

// ============================================================================
// K8w: weight-resident, whole-K 1x1 conv for the dense layers with K <= 256
// (all of block 1, the first layers of block 2: M up to 401k rows at bs128).
// K8 walks K in 32-wide steps with a barrier per step — 2-8 steps of 8 MFMAs
// per 64-pixel tile — and re-fetches the weight tile for every pixel tile.
// Here a persistent block (one per CU: 137 KB LDS at K = 256) stages ALL of
// W [128][K] once, then walks 64-pixel tiles with the whole K of the next
// tile's activations in flight in registers (KS x 16 B per thread) while the
// current tile runs its 8*KS MFMAs from LDS: one barrier per tile.  BN1+ReLU
// prologue on the way into LDS, BN2-folded bias + ReLU epilogue (as K8).
// ============================================================================
constexpr int kOStride = 128 + 8;  // K8w output staging row (272 B: conflict-free b64 writes / b128 reads)

template <int KS>  // K / 32
__global__ void __launch_bounds__(256) conv1x1_wres_kernel(Conv1x1Params p) {
  constexpr int K = KS * 32, LDK = K + 8, CPR = K / 8;
  constexpr int BM = 64, BN = 128, NJ = 4, TM = 2, WN = 64;
  constexpr int AI = BM * CPR / 256;  // = KS: A chunks per thread per tile
  constexpr int BI = BN * CPR / 256;  // = 2 * KS
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* sB = smem;                       // [BN][LDK]
  uint16_t* sA = smem + BN * LDK;            // [2][BM][LDK]
  uint16_t* sO = sA + 2 * BM * LDK;         // [BM][kOStride] output staging
  float* sS = reinterpret_cast<float*>(sO + BM * kOStride);
  float* sT = sS + K;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int n0 = blockIdx.y * BN;
  const int tiles = (p.M + BM - 1) / BM;
  for (int k = tid; k < K; k += 256) {
    sS[k] = p.in_scale[k];
    sT[k] = p.in_bias[k];
  }
  {
    v4u r[BI];
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int c = tid + i * 256;
      r[i] = ldg16(p.w + (size_t)(n0 + c / CPR) * p.K + (c % CPR) * 8);
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int c = tid + i * 256;
      *reinterpret_cast<v4u*>(&sB[(c / CPR) * LDK + (c % CPR) * 8]) = r[i];
    }
  }
  v4u ra[AI];
  auto load_a = [&](int tile) {
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int c = tid + i * 256;
      const int m = tile * BM + c / CPR;
      ra[i] = m < p.M ? ldg16(p.x + (size_t)m * p.ldx + (c % CPR) * 8) : v4u{0, 0, 0, 0};
    }
  };
  auto store_a = [&](int buf) {  // BN1 + ReLU prologue (rows past M only feed unstored outputs)
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int c = tid + i * 256;
      const int kc = (c % CPR) * 8;
      float f[8], o[8];
      unpack8(ra[i], f);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = f[e] * sS[kc + e] + sT[kc + e];
      v4u v = pack8(o);
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = relu_pk(v[q]);
      *reinterpret_cast<v4u*>(&sA[buf * BM * LDK + (c / CPR) * LDK + kc]) = v;
    }
  };
  f32x4 bias0[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int nb = n0 + wn * WN + j * 16 + (lane >> 4) * 4;
    bias0[j] = p.out_bias ? f32x4{p.out_bias[nb], p.out_bias[nb + 1], p.out_bias[nb + 2], p.out_bias[nb + 3]}
                          : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  int tile = blockIdx.x;
  if (tile < tiles) load_a(tile);
  __syncthreads();  // sS / sT / sB staged
  if (tile < tiles) store_a(0);
  __syncthreads();
  const int fr = lane & 15, fk = 8 * (lane >> 4);
  int buf = 0;
  for (; tile < tiles; tile += gridDim.x) {
    const int nxt = tile + (int)gridDim.x;
    if (nxt < tiles) load_a(nxt);
    f32x4 acc[NJ][TM];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int i = 0; i < TM; ++i) acc[j][i] = bias0[j];
    const uint16_t* a_base = sA + buf * BM * LDK;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 fa[NJ], fb[TM];
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        fa[j] = *reinterpret_cast<const bf16x8*>(&sB[(wn * WN + j * 16 + fr) * LDK + ks * 32 + fk]);
#pragma unroll
      for (int i = 0; i < TM; ++i)
        fb[i] = *reinterpret_cast<const bf16x8*>(&a_base[(wm * 16 * TM + i * 16 + fr) * LDK + ks * 32 + fk]);
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[j][i] = mfma16(fa[j], fb[i], acc[j][i]);
    }
    // epilogue through LDS: a lane's accumulators are 4 channels of one pixel
    // (8 B pieces, 32 B per row per store instruction); staged as the 64 x 128
    // tile, every output row leaves as one 256-B run (16 lanes x 16 B)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int nb = wn * WN + j * 16 + (lane >> 4) * 4;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        v2u o = v2u{pack2(acc[j][i][0], acc[j][i][1]), pack2(acc[j][i][2], acc[j][i][3])};
        if (p.relu_out) o = v2u{relu_pk(o[0]), relu_pk(o[1])};
        *reinterpret_cast<v2u*>(&sO[(wm * 16 * TM + i * 16 + fr) * kOStride + nb]) = o;
      }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < BM * 16 / 256; ++q) {
      const int c = tid + q * 256, r = c >> 4, m = tile * BM + r;
      if (m < p.M)
        *reinterpret_cast<v4u*>(p.y + (size_t)m * p.ldy + n0 + (c & 15) * 8) =
            *reinterpret_cast<const v4u*>(&sO[r * kOStride + (c & 15) * 8]);
    }
    if (nxt < tiles) store_a(buf ^ 1);  // that buffer's last reads were before the previous barrier
    __syncthreads();
    buf ^= 1;
  }
}

template <int KS>
int launch_1x1_wres(const Conv1x1Params& p, hipStream_t s) {
  constexpr int LDK = KS * 32 + 8;
  const int lds = ((128 + 2 * 64) * LDK + 64 * kOStride) * 2 + 2 * KS * 32 * 4;  // sB, 2 x sA, sO, sS/sT
  static int attr = 0;
  if (attr < lds) {
    int rc = hipFuncSetAttribute((const void*)conv1x1_wres_kernel<KS>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (rc != hipSuccess) return rc;
    attr = lds;
  }
  const int tiles = (p.M + 63) / 64;
  hipLaunchKernelGGL(conv1x1_wres_kernel<KS>, dim3(tiles < 256 ? tiles : 256, p.N / 128), dim3(256), lds, s, p);
  return hipGetLastError();
}

int launch_1x1_wres_k(const Conv1x1Params& p, hipStream_t s) {
  switch (p.K / 32) {
    case 1: return launch_1x1_wres<1>(p, s);
    case 2: return launch_1x1_wres<2>(p, s);
    case 3: return launch_1x1_wres<3>(p, s);
    case 4: return launch_1x1_wres<4>(p, s);
    case 5: return launch_1x1_wres<5>(p, s);
    case 6: return launch_1x1_wres<6>(p, s);
    case 7: return launch_1x1_wres<7>(p, s);
    case 8: return launch_1x1_wres<8>(p, s);
    default: return hipErrorInvalidValue;
  }
}

// ============================================================================
// K8p: persistent, software-pipelined 1x1 conv.  Profiling K8 showed every
// dense-layer 1x1 latency-bound: each block walks K in 32-wide steps with one
// tile of loads in flight, so a 14x14 layer (K up to 992) waits ~31 global
// round trips, and the 56x56 layers (2-7 steps per tile) pay the pipeline
// fill per 64-pixel tile.  Here a block (grid = resident capacity) owns tiles
// t = blockIdx.x + j * gridDim.x and walks ONE flattened stream of (tile,
// k-step) steps with D steps of loads in flight in registers — across tile
// boundaries too — while the MFMAs consume the LDS double buffer; the
// epilogue of a tile is just a step with a store.  Same block tile, BN
// prologue and epilogue as K8 (BK = 32, 4 waves as 2 x 2, 16x16x32 MFMA).
// ============================================================================
template <int TM, int D, bool PRO>
__global__ void __launch_bounds__(256) conv1x1_pipe_kernel(Conv1x1Params p) {
  constexpr int BK = 32, BM = 32 * TM, BN = 128;
  constexpr int CPR = BK / 8, LDK = BK + 8;
  constexpr int A_CHUNKS = BM * CPR, AI = (A_CHUNKS + 255) / 256;
  constexpr int BI = BN * CPR / 256;
  __shared__ __attribute__((aligned(16))) uint16_t sA[2][BM * LDK];
  __shared__ __attribute__((aligned(16))) uint16_t sB[2][BN * LDK];
  __shared__ float sS[PRO ? kMaxK : 1], sT[PRO ? kMaxK : 1], sBias[kMaxK];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  if constexpr (PRO) {
    for (int k = tid; k < p.K; k += 256) {
      sS[k] = p.in_scale[k];
      sT[k] = p.in_bias[k];
    }
  }
  // epilogue bias from LDS: a global load in the epilogue would make the
  // in-order vmcnt wait drain every prefetched tile behind it
  for (int n = tid; n < p.N; n += 256) sBias[n] = p.out_bias ? p.out_bias[n] : 0.f;
  const int nt = p.N / BN, tiles = ((p.M + BM - 1) / BM) * nt;
  const int KT = p.K / BK;
  const int mine = (int)blockIdx.x < tiles ? (tiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  const int G = mine * KT;
  if (G == 0) return;  // whole block

  // step g -> tile origin (m0, n0) and k offset
  auto decode = [&](int g, int& m0, int& n0, int& k0) {
    const int j = g / KT, kt = g - j * KT;
    const int t = (int)blockIdx.x + j * (int)gridDim.x;
    const int tm = t / nt;
    m0 = tm * BM;
    n0 = (t - tm * nt) * BN;
    k0 = kt * BK;
  };
  v4u ra[D][AI], rb[D][BI];
  auto load = [&](int g, v4u(&a)[AI], v4u(&b)[BI]) {
    int m0, n0, k0;
    decode(g, m0, n0, k0);
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int c = tid + i * 256;
      const int m = m0 + c / CPR;
      a[i] = (c < A_CHUNKS && m < p.M) ? ldg16(p.x + (size_t)m * p.ldx + k0 + (c % CPR) * 8) : v4u{0, 0, 0, 0};
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int c = tid + i * 256;
      b[i] = ldg16(p.w + (size_t)(n0 + c / CPR) * p.K + k0 + (c % CPR) * 8);
    }
  };
  auto store = [&](int g, int buf, const v4u(&a)[AI], const v4u(&b)[BI]) {
    int m0, n0, k0;
    decode(g, m0, n0, k0);
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int c = tid + i * 256;
      if (c < A_CHUNKS) {
        const int kc = (c % CPR) * 8;
        v4u v = a[i];
        if constexpr (PRO) {
          float f[8];
          unpack8(v, f);
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] = fmaxf(f[e] * sS[k0 + kc + e] + sT[k0 + kc + e], 0.f);
          v = pack8(f);
        }
        if (m0 + c / CPR >= p.M) v = v4u{0, 0, 0, 0};
        *reinterpret_cast<v4u*>(&sA[buf][(c / CPR) * LDK + kc]) = v;
      }
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int c = tid + i * 256;
      *reinterpret_cast<v4u*>(&sB[buf][(c / CPR) * LDK + (c % CPR) * 8]) = b[i];
    }
  };

  // loads are issued unconditionally (past the end: the last step again), so
  // the waitcnt pass sees a straight-line stream of D in-flight steps
#pragma unroll
  for (int s = 0; s < D; ++s) load(min(s, G - 1), ra[s], rb[s]);
  __syncthreads();  // prologue tables
  store(0, 0, ra[0], rb[0]);
  __syncthreads();

  f32x4 acc[4][TM];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fk = 8 * (lane >> 4);
  for (int g0 = 0; g0 < G; g0 += D) {
#pragma unroll
    for (int s = 0; s < D; ++s) {
      const int g = g0 + s;
      if (g < G) {  // block-uniform
        const int buf = g & 1;
        // stage s held step g (already in LDS): refill it with step g + D
        load(min(g + D, G - 1), ra[s], rb[s]);
        bf16x8 fa[4], fb[TM];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          fa[j] = *reinterpret_cast<const bf16x8*>(&sB[buf][(wn * 64 + j * 16 + fr) * LDK + fk]);
#pragma unroll
        for (int i = 0; i < TM; ++i)
          fb[i] = *reinterpret_cast<const bf16x8*>(&sA[buf][(wm * 16 * TM + i * 16 + fr) * LDK + fk]);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int i = 0; i < TM; ++i) acc[j][i] = mfma16(fa[j], fb[i], acc[j][i]);
        if (g % KT == KT - 1) {  // tile done: epilogue, restart the accumulators
          int m0, n0, k0;
          decode(g, m0, n0, k0);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int nb = n0 + wn * 64 + j * 16 + (lane >> 4) * 4;
            float bias[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) bias[r] = sBias[nb + r];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
              const int m = m0 + wm * 16 * TM + i * 16 + fr;
              if (m < p.M) {
                float v[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                  v[r] = acc[j][i][r] + bias[r];
                  if (p.relu_out) v[r] = fmaxf(v[r], 0.f);
                }
                *reinterpret_cast<v2u*>(p.y + (size_t)m * p.ldy + nb) = v2u{pack2(v[0], v[1]), pack2(v[2], v[3])};
              }
              acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
          }
        }
        if (g + 1 < G) store(g + 1, buf ^ 1, ra[(s + 1) % D], rb[(s + 1) % D]);
        __syncthreads();
      }
    }
  }
}

// split-K combine: y[m][n..n+3] = epi(sum_z ws[z][m][n..n+3] + bias)
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const float* __restrict__ ws, int splits, int M, int N,
                                                            const float* __restrict__ bias, int relu,
                                                            uint16_t* __restrict__ y, int ldy) {
  const int q = N / 4;
  const size_t total = (size_t)M * q;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (size_t)gridDim.x * blockDim.x) {
    const int m = (int)(t / q), n = (int)(t - (size_t)m * q) * 4;
    f32x4 a = *reinterpret_cast<const f32x4*>(ws + (size_t)m * N + n);
    for (int z = 1; z < splits; ++z) a += *reinterpret_cast<const f32x4*>(ws + ((size_t)z * M + m) * N + n);
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      v[r] = a[r] + (bias ? bias[n + r] : 0.f);
      if (relu) v[r] = fmaxf(v[r], 0.f);
    }
    *reinterpret_cast<v2u*>(y + (size_t)m * ldy + n) = v2u{pack2(v[0], v[1]), pack2(v[2], v[3])};
  }
}


// ============================================================================
// K8s: small-M 1x1 conv.  Block = 32 pixels x 128 output channels; the four
// waves split K (wave w takes the 32-wide K chunks w, w+4, ...), so the
// serial load -> MFMA chain per wave is 4x shorter than in K8, where the
// waves split the tile and each walks all of K.  The partial tiles are summed
// through LDS in two rounds (waves 2,3 -> 0,1, then 1 -> 0) and wave 0 runs
// the epilogue.  Operands come straight from global memory (L2-resident
// weights, one pass over the activations), so no LDS staging is needed.
// ============================================================================
template <bool POOL>
__global__ void __launch_bounds__(256) conv1x1_sk_kernel(Conv1x1Params p) {
  constexpr int NS = POOL ? 4 : 1;
  __shared__ __attribute__((aligned(16))) f32x4 red[2][16][64];  // [slot][frag][lane], 32 KB
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m0 = blockIdx.x * 32, n0 = blockIdx.y * 128;
  const int fr = lane & 15, fk = 8 * (lane >> 4);
  const int KC = p.K / 32;

  // this lane's two activation rows (POOL: the 2x2 windows' 4 rows each)
  const uint16_t* a_src[2][NS];
  bool a_ok[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + 16 * i + fr;
    a_ok[i] = m < p.M;
    const int mm = a_ok[i] ? m : 0;
    if constexpr (POOL) {
      const int wo = p.W >> 1, ho = p.H >> 1;
      const int img = mm / (ho * wo), r = mm - img * ho * wo;
      const int oh = r / wo, ow = r - oh * wo;
      const size_t base = ((size_t)img * p.H + 2 * oh) * p.W + 2 * ow;
      a_src[i][0] = p.x + base * p.ldx + fk;
      a_src[i][1] = p.x + (base + 1) * p.ldx + fk;
      a_src[i][2] = p.x + (base + p.W) * p.ldx + fk;
      a_src[i][3] = p.x + (base + p.W + 1) * p.ldx + fk;
    } else {
      a_src[i][0] = p.x + (size_t)mm * p.ldx + fk;
    }
  }
  const uint16_t* w_src = p.w + (size_t)(n0 + fr) * p.K + fk;

  struct Raw {
    v4u w[8];
    v4u a[2][NS];
    f32x4 s0, s1, t0, t1;
  };
  auto load = [&](int c, Raw& r) {
    const int k0 = 32 * c;
#pragma unroll
    for (int j = 0; j < 8; ++j) r.w[j] = ldg16(w_src + (size_t)16 * j * p.K + k0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int q = 0; q < NS; ++q) r.a[i][q] = a_ok[i] ? ldg16(a_src[i][q] + k0) : v4u{0, 0, 0, 0};
    r.s0 = *reinterpret_cast<const f32x4*>(p.in_scale + k0 + fk);
    r.s1 = *reinterpret_cast<const f32x4*>(p.in_scale + k0 + fk + 4);
    r.t0 = *reinterpret_cast<const f32x4*>(p.in_bias + k0 + fk);
    r.t1 = *reinterpret_cast<const f32x4*>(p.in_bias + k0 + fk + 4);
  };

  f32x4 acc[8][2];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int i = 0; i < 2; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](const Raw& r) {
    const float sc[8] = {r.s0[0], r.s0[1], r.s0[2], r.s0[3], r.s1[0], r.s1[1], r.s1[2], r.s1[3]};
    const float sh[8] = {r.t0[0], r.t0[1], r.t0[2], r.t0[3], r.t1[0], r.t1[1], r.t1[2], r.t1[3]};
    bf16x8 af[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = 0.f;
#pragma unroll
      for (int q = 0; q < NS; ++q) {
        float f[8];
        unpack8(r.a[i][q], f);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float t = fmaxf(f[e] * sc[e] + sh[e], 0.f);
          o[e] += POOL ? 0.25f * t : t;
        }
      }
      af[i] = as_frag(pack8(o));
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int i = 0; i < 2; ++i) acc[j][i] = mfma16(as_frag(r.w[j]), af[i], acc[j][i]);
  };

  Raw cur, nxt;
  int c = wave;
  if (c < KC) load(c, cur);
  for (; c < KC; c += 4) {
    if (c + 4 < KC) load(c + 4, nxt);
    compute(cur);
    cur = nxt;
  }

  // cross-wave reduction: 2,3 -> 0,1 ; 1 -> 0
  if (wave >= 2) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int i = 0; i < 2; ++i) red[wave - 2][j * 2 + i][lane] = acc[j][i];
  }
  __syncthreads();
  if (wave < 2) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int i = 0; i < 2; ++i) acc[j][i] += red[wave][j * 2 + i][lane];
  }
  __syncthreads();
  if (wave == 1) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int i = 0; i < 2; ++i) red[0][j * 2 + i][lane] = acc[j][i];
  }
  __syncthreads();
  if (wave != 0) return;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int nb = n0 + j * 16 + (lane >> 4) * 4;
    float bias[4] = {0.f, 0.f, 0.f, 0.f};
    if (p.out_bias) {
#pragma unroll
      for (int r = 0; r < 4; ++r) bias[r] = p.out_bias[nb + r];
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const f32x4 a = acc[j][i] + red[0][j * 2 + i][lane];
      const int m = m0 + 16 * i + fr;
      if (m < p.M) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = a[r] + bias[r];
          if (p.relu_out) v[r] = fmaxf(v[r], 0.f);
        }
        *reinterpret_cast<v2u*>(p.y + (size_t)m * p.ldy + nb) = v2u{pack2(v[0], v[1]), pack2(v[2], v[3])};
      }
    }
  }
}

// ============================================================================
// K9: 3x3 conv, 128 -> 32 channels, stride 1, pad 1 (implicit GEMM)
// ============================================================================
struct Conv3x3Params {
  const uint16_t* z;   // [M][128] bf16 NHWC (contiguous rows)
  const uint16_t* w;   // [32][3][3][128] bf16
  uint16_t* y;         // [M][ldy], already offset to the first output channel
  int M, H, W, ldy;
  int tiles;           // ceil(M / (64*TM))
  int ablate;          // diagnostics only (tools/kbench_densenet.py): bit0 drop activation loads, bit1 drop stores
};

// Persistent blocks: weights loaded to LDS once, then the block walks pixel
// tiles of 4 waves x 16*TM pixels.  Each tap's 16 B activation fragments are
// prefetched one tap ahead (register double-buffer across the unrolled taps).
template <int TM, int G>
__global__ void __launch_bounds__(256) conv3x3_kernel(Conv3x3Params p) {
  extern __shared__ __attribute__((aligned(16))) uint16_t Ws[];  // [32][kWsK]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int c = tid; c < kN3 * (kK3 / 8); c += 256) {
    const int n = c / (kK3 / 8), kc = (c - n * (kK3 / 8)) * 8;
    *reinterpret_cast<v4u*>(&Ws[n * kWsK + kc]) = ldg16(p.w + (size_t)n * kK3 + kc);
  }
  __syncthreads();

  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)p.z, (short)0,
                                                      (p.ablate & 1) ? 0 : (int)((size_t)p.M * kC3 * 2),
                                                      0x00020000);
  const int HW = p.H * p.W;
  const int fr = lane & 15, fk = 8 * (lane >> 4);
  for (int tile = blockIdx.x; tile < p.tiles; tile += gridDim.x) {
    const int mb = tile * (64 * TM) + wave * 16 * TM;
    int pm[TM], ph[TM], pw[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = mb + i * 16 + fr;
      pm[i] = m < p.M ? m : -1;
      const int mm = m < p.M ? m : 0;
      const int img = mm / HW, r = mm - img * HW;
      ph[i] = r / p.W;
      pw[i] = r - ph[i] * p.W;
    }
    f32x4 acc[2][TM];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto load_tap = [&](int tap, v4u (&dst)[TM][4]) {
      const int dy = tap / 3 - 1, dx = tap % 3 - 1;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int hh = ph[i] + dy, ww = pw[i] + dx;
        const bool ok = pm[i] >= 0 && hh >= 0 && hh < p.H && ww >= 0 && ww < p.W;
        // out-of-image taps: an offset past num_records makes the buffer load return 0
        const int off = ok ? ((pm[i] + dy * p.W + dx) * kC3 + fk) * 2 : 0x40000000;
#pragma unroll
        for (int c = 0; c < 4; ++c) dst[i][c] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off + c * 64, 0, 0);
      }
    };
    auto mma_tap = [&](int tap, const v4u (&src)[TM][4]) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        bf16x8 fa[2];
#pragma unroll
        for (int j = 0; j < 2; ++j)
          fa[j] = *reinterpret_cast<const bf16x8*>(&Ws[(j * 16 + fr) * kWsK + tap * kC3 + c * 32 + fk]);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int i = 0; i < TM; ++i) acc[j][i] = mfma16(fa[j], as_frag(src[i][c]), acc[j][i]);
      }
    };
    if constexpr (G >= 4) {
      // tap-major steps of 32 channels with a G-deep load ring: G * TM 16-B
      // loads in flight per lane to cover L2 latency at 2 waves / SIMD
      auto load_step = [&](int st, v4u (&dst)[TM]) {
        const int tap = st >> 2, c = st & 3;
        const int dy = tap / 3 - 1, dx = tap % 3 - 1;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int hh = ph[i] + dy, ww = pw[i] + dx;
          const bool ok = pm[i] >= 0 && hh >= 0 && hh < p.H && ww >= 0 && ww < p.W;
          const int off = ok ? ((pm[i] + dy * p.W + dx) * kC3 + fk) * 2 : 0x40000000;
          dst[i] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off + c * 64, 0, 0);
        }
      };
      v4u ring[G][TM];
#pragma unroll
      for (int st = 0; st < G; ++st) load_step(st, ring[st]);
#pragma unroll 1
      for (int s0 = 0; s0 < 36; s0 += G) {
#pragma unroll
        for (int u = 0; u < G; ++u) {
          const int st = s0 + u;
          const int tap = st >> 2, c = st & 3;
          bf16x8 fa[2];
#pragma unroll
          for (int j = 0; j < 2; ++j)
            fa[j] = *reinterpret_cast<const bf16x8*>(&Ws[(j * 16 + fr) * kWsK + tap * kC3 + c * 32 + fk]);
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int i = 0; i < TM; ++i) acc[j][i] = mfma16(fa[j], as_frag(ring[u][i]), acc[j][i]);
          if (st + G < 36) load_step(st + G, ring[u]);
        }
      }
    } else if constexpr (G == 0) {
      // channel-major order: for each 32-channel chunk walk all 9 taps, so the
      // 3 input rows touched by a tile stay L1-resident across the taps
      // (working set (64 + 2W + 2) x 64 B instead of x 256 B); 4 steps in flight.
      auto load_step = [&](int st, v4u (&dst)[TM]) {
        const int c = st / 9, tap = st - c * 9;
        const int dy = tap / 3 - 1, dx = tap % 3 - 1;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int hh = ph[i] + dy, ww = pw[i] + dx;
          const bool ok = pm[i] >= 0 && hh >= 0 && hh < p.H && ww >= 0 && ww < p.W;
          const int off = ok ? ((pm[i] + dy * p.W + dx) * kC3 + fk) * 2 : 0x40000000;
          dst[i] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off + c * 64, 0, 0);
        }
      };
      v4u ring[4][TM];
#pragma unroll
      for (int st = 0; st < 4; ++st) load_step(st, ring[st]);
#pragma unroll 1
      for (int s0 = 0; s0 < 36; s0 += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int st = s0 + u;
          const int c = st / 9, tap = st - c * 9;
          bf16x8 fa[2];
#pragma unroll
          for (int j = 0; j < 2; ++j)
            fa[j] = *reinterpret_cast<const bf16x8*>(&Ws[(j * 16 + fr) * kWsK + tap * kC3 + c * 32 + fk]);
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int i = 0; i < TM; ++i) acc[j][i] = mfma16(fa[j], as_frag(ring[u][i]), acc[j][i]);
          if (st + 4 < 36) load_step(st + 4, ring[u]);
        }
      }
    } else if constexpr (G == 1) {
      // taps in ping-pong pairs: tap t+1's fragments load while tap t multiplies
      v4u xa[TM][4], xb[TM][4];
      load_tap(0, xa);
#pragma unroll 1
      for (int tap = 0; tap < 8; tap += 2) {
        load_tap(tap + 1, xb);
        mma_tap(tap, xa);
        load_tap(tap + 2, xa);
        mma_tap(tap + 1, xb);
      }
      mma_tap(8, xa);
    } else {
      // groups of 3 taps (one filter row): 12*TM loads in flight per lane
      v4u ga[3][TM][4], gb[3][TM][4];
#pragma unroll
      for (int t = 0; t < 3; ++t) load_tap(t, ga[t]);
#pragma unroll
      for (int t = 0; t < 3; ++t) load_tap(3 + t, gb[t]);
#pragma unroll
      for (int t = 0; t < 3; ++t) mma_tap(t, ga[t]);
#pragma unroll
      for (int t = 0; t < 3; ++t) load_tap(6 + t, ga[t]);
#pragma unroll
      for (int t = 0; t < 3; ++t) mma_tap(3 + t, gb[t]);
#pragma unroll
      for (int t = 0; t < 3; ++t) mma_tap(6 + t, ga[t]);
    }
    if (p.ablate & 2) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i) asm volatile("" ::"v"(acc[j][i]));
      continue;
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int nb = j * 16 + (lane >> 4) * 4;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if (pm[i] >= 0) {
          const f32x4 v = acc[j][i];
          *reinterpret_cast<v2u*>(p.y + (size_t)pm[i] * p.ldy + nb) = v2u{pack2(v[0], v[1]), pack2(v[2], v[3])};
        }
      }
    }
  }
}

// K9b: the same conv on v_mfma_f32_32x32x16_bf16 with the weights as operand A.
// One 32x16 weight slab (all 32 output channels) is ONE ds_read_b128 per
// lane and is reused by the wave's TM 32-pixel subtiles, so LDS traffic per
// MFMA drops 4-8x against the 16x16x32 form (which needs 2 weight fragments
// per 2 MFMAs).  Wave tile: 32*TM pixels x 32 channels; block: 4 waves.
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

template <int TM>
__global__ void __launch_bounds__(256) conv3x3_m32_kernel(Conv3x3Params p) {
  extern __shared__ __attribute__((aligned(16))) uint16_t Ws[];  // [32][kWsK]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int c = tid; c < kN3 * (kK3 / 8); c += 256) {
    const int n = c / (kK3 / 8), kc = (c - n * (kK3 / 8)) * 8;
    *reinterpret_cast<v4u*>(&Ws[n * kWsK + kc]) = ldg16(p.w + (size_t)n * kK3 + kc);
  }
  __syncthreads();
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)p.z, (short)0,
                                                      (int)((size_t)p.M * kC3 * 2), 0x00020000);
  const int HW = p.H * p.W;
  const int col = lane & 31, kh = 8 * (lane >> 5);
  for (int tile = blockIdx.x; tile < p.tiles; tile += gridDim.x) {
    const int mb = tile * (128 * TM) + wave * 32 * TM;
    int pm[TM], ph[TM], pw[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = mb + i * 32 + col;
      pm[i] = m < p.M ? m : -1;
      const int mm = m < p.M ? m : 0;
      const int img = mm / HW, r = mm - img * HW;
      ph[i] = r / p.W;
      pw[i] = r - ph[i] * p.W;
    }
    f32x16 acc[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;

    // per tap: 8 k-steps of 16 channels; lane fetches 16 B = 8 channels of its pixel
    auto load_tap = [&](int tap, v4u (&dst)[TM][8]) {
      const int dy = tap / 3 - 1, dx = tap % 3 - 1;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int hh = ph[i] + dy, ww = pw[i] + dx;
        const bool ok = pm[i] >= 0 && hh >= 0 && hh < p.H && ww >= 0 && ww < p.W;
        const int off = ok ? ((pm[i] + dy * p.W + dx) * kC3 + kh) * 2 : 0x40000000;
#pragma unroll
        for (int c = 0; c < 8; ++c) dst[i][c] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off + c * 32, 0, 0);
      }
    };
    auto mma_tap = [&](int tap, const v4u (&src)[TM][8]) {
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(&Ws[col * kWsK + tap * kC3 + c * 16 + kh]);
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[i] = mfma32(a, as_frag(src[i][c]), acc[i]);
      }
    };
    v4u xa[TM][8], xb[TM][8];
    load_tap(0, xa);
#pragma unroll 1
    for (int tap = 0; tap < 8; tap += 2) {
      load_tap(tap + 1, xb);
      mma_tap(tap, xa);
      load_tap(tap + 2, xa);
      mma_tap(tap + 1, xb);
    }
    mma_tap(8, xa);
    // C/D: col = pixel (lane & 31); reg r -> channel (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      if (pm[i] < 0) continue;
      uint16_t* yp = p.y + (size_t)pm[i] * p.ldy + 4 * (lane >> 5);
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<v2u*>(yp + 8 * g) =
            v2u{pack2(acc[i][4 * g], acc[i][4 * g + 1]), pack2(acc[i][4 * g + 2], acc[i][4 * g + 3])};
    }
  }
}

// K9c: LDS-staged activations.  Profiling (ablation in tools/kbench_densenet.py)
// showed K9's time is 60% fragment-shaped activation fetches: every input
// pixel is pulled through L1 9x (once per tap) in 64-B pieces.  Here a block
// stages the contiguous pixel band its 128 output pixels need ([m0-W-1,
// m0+128+W+1), 272-B padded rows: conflict-free b128 reads) into LDS once,
// with full-row coalesced loads that are issued for the NEXT tile while the
// current one computes; all 9 taps then read LDS.  Weights stay LDS-resident
// (74 KB) and feed v_mfma_f32_32x32x16_bf16 as operand A; one 32-pixel
// subtile per wave.  Out-of-image taps are zeroed by a per-tap mask.
// 74 KB of weights global -> LDS with all 18 loads per thread in flight at
// once (a rolled load->store loop serialises 18 L2 round trips: ~10 us per
// launch, most of a 14x14 layer's time when each block walks one tile)
__device__ __forceinline__ void stage_weights(const uint16_t* __restrict__ w, uint16_t* Ws, int tid) {
  constexpr int kChunks = kN3 * (kK3 / 8), kPer = kChunks / 256;  // 4608 / 256 = 18
  static_assert(kChunks % 256 == 0, "weight chunks per thread");
  v4u r[kPer];
#pragma unroll
  for (int i = 0; i < kPer; ++i) r[i] = ldg16(w + (size_t)(tid + i * 256) * 8);
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int c = tid + i * 256;
    const int n = c / (kK3 / 8), kc = (c - n * (kK3 / 8)) * 8;
    *reinterpret_cast<v4u*>(&Ws[n * kWsK + kc]) = r[i];
  }
}

constexpr int kActStride = kC3 + 8;  // 272-B rows
constexpr int kTileP = 128;          // output pixels per tile (4 waves x 32)
// An all-zero activation row after the largest band: out-of-image taps read
// it (one address select per tap) instead of masking every fragment (four
// v_cndmask per MFMA).
constexpr int kZeroRow = kTileP + 2 * 57;

__global__ void __launch_bounds__(256) conv3x3_lds_kernel(Conv3x3Params p) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* Ws = smem;                   // [32][kWsK]
  uint16_t* As = smem + kN3 * kWsK;      // [rows][kActStride], row kZeroRow = 0
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  stage_weights(p.w, Ws, tid);
  if (tid < kActStride / 8) *reinterpret_cast<v4u*>(&As[kZeroRow * kActStride + tid * 8]) = v4u{0, 0, 0, 0};
  const int W = p.W, HW = p.H * p.W;
  const int halo = W + 1, rows = kTileP + 2 * halo, chunks = rows * 16;
  constexpr int kMaxChunks = (kTileP + 2 * 57) * 16;       // W <= 56
  constexpr int CPT = (kMaxChunks + 255) / 256;           // 16-B chunks per thread
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)p.z, (short)0,
                                                      (int)((size_t)p.M * kC3 * 2), 0x00020000);
  v4u st[CPT];
  auto load_tile = [&](int tile) {
    const int base = tile * kTileP - halo;
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int c = tid + i * 256;
      const int r = c >> 4, q = c & 15;
      const int pix = base + r;
      const bool ok = c < chunks && pix >= 0 && pix < p.M;
      st[i] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, ok ? (pix * kC3 + q * 8) * 2 : 0x40000000, 0, 0);
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int c = tid + i * 256;
      if (c < chunks) *reinterpret_cast<v4u*>(&As[(c >> 4) * kActStride + (c & 15) * 8]) = st[i];
    }
  };
  const int col = lane & 31, kh = 8 * (lane >> 5);
  int tile = blockIdx.x;
  if (tile < p.tiles) load_tile(tile);
  for (; tile < p.tiles; tile += gridDim.x) {
    __syncthreads();  // previous tile's LDS reads done (and, first time, weights staged)
    store_tile();
    __syncthreads();
    if (tile + (int)gridDim.x < p.tiles) load_tile(tile + gridDim.x);
    const int tp = wave * 32 + col;  // tile-relative output pixel of this lane
    const int m = tile * kTileP + tp;
    const int mm = m < p.M ? m : 0;
    const int img = mm / HW, rr = mm - img * HW;
    const int h = rr / W, w = rr - h * W;
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    const bool up = h > 0, down = h + 1 < p.H, left = w > 0, right = w + 1 < W, in = m < p.M;
#pragma unroll 1
    for (int tap = 0; tap < 9; ++tap) {
      const int dy = tap / 3 - 1, dx = tap % 3 - 1;
      const bool ok = in && (dy < 0 ? up : dy > 0 ? down : true) && (dx < 0 ? left : dx > 0 ? right : true);
      const uint16_t* arow = &As[(ok ? tp + halo + dy * W + dx : kZeroRow) * kActStride + kh];
      const uint16_t* wrow = &Ws[col * kWsK + tap * kC3 + kh];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const v4u b = *reinterpret_cast<const v4u*>(arow + c * 16);
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(wrow + c * 16);
        acc = mfma32(a, as_frag(b), acc);
      }
    }
    if (m < p.M) {
      uint16_t* yp = p.y + (size_t)m * p.ldy + 4 * (lane >> 5);
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<v2u*>(yp + 8 * g) =
            v2u{pack2(acc[4 * g], acc[4 * g + 1]), pack2(acc[4 * g + 2], acc[4 * g + 3])};
    }
  }
}

// K9r: the K9c tile walk with the weights in REGISTERS instead of LDS.  K9c
// keeps 74 KB of weights + a 66 KB activation band in LDS, so one block (4
// waves, one per SIMD) fills a CU and nothing else co-resides.  Here wave w
// owns input channels [32w, 32w+32) of all 9 taps: its 18 weight fragments
// (32 out-ch x 16 k each) live in 72 VGPRs for the whole kernel, it runs all
// four 32-pixel subtiles of the tile over its K quarter, and the four partial
// tiles are summed through LDS (aliasing the activation band once the taps
// are done).  LDS per block = the activation band -> two blocks per CU, and
// per MFMA only the activation fragment is read from LDS.
constexpr int kRedFloats = 4 * 3 * 64 * 16;  // [subtile][3 other waves][lane][16]

__global__ void __launch_bounds__(256, 2) conv3x3_kr_kernel(Conv3x3Params p) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* As = smem;                                  // [rows][kActStride] bf16, row kZeroRow = 0
  float* red = reinterpret_cast<float*>(smem);          // aliases As after the taps (below kZeroRow)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  static_assert(kRedFloats * 4 <= kZeroRow * kActStride * 2, "reduction scratch must not reach the zero row");
  if (tid < kActStride / 8) *reinterpret_cast<v4u*>(&As[kZeroRow * kActStride + tid * 8]) = v4u{0, 0, 0, 0};
  const int col = lane & 31, kh = 8 * (lane >> 5);
  v4u wr[18];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int h = 0; h < 2; ++h) wr[t * 2 + h] = ldg16(p.w + (size_t)col * kK3 + t * kC3 + 32 * wave + 16 * h + kh);
  const int W = p.W, HW = p.H * p.W;
  const int halo = W + 1, rows = kTileP + 2 * halo, chunks = rows * 16;
  constexpr int kMaxChunks = (kTileP + 2 * 57) * 16;
  constexpr int CPT = (kMaxChunks + 255) / 256;
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)p.z, (short)0,
                                                      (int)((size_t)p.M * kC3 * 2), 0x00020000);
  v4u st[CPT];
  auto load_tile = [&](int tile) {
    const int base = tile * kTileP - halo;
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int c = tid + i * 256;
      const int r = c >> 4, q = c & 15;
      const int pix = base + r;
      const bool ok = c < chunks && pix >= 0 && pix < p.M;
      st[i] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, ok ? (pix * kC3 + q * 8) * 2 : 0x40000000, 0, 0);
    }
  };
  // no cross-tile register prefetch (it would not fit next to the resident
  // weights): the other block on the CU computes while this one loads
  for (int tile = blockIdx.x; tile < p.tiles; tile += gridDim.x) {
    load_tile(tile);
    __syncthreads();  // previous tile's reduction reads done
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int c = tid + i * 256;
      if (c < chunks) *reinterpret_cast<v4u*>(&As[(c >> 4) * kActStride + (c & 15) * 8]) = st[i];
    }
    __syncthreads();
    bool pv[4], up[4], down[4], left[4], right[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = tile * kTileP + i * 32 + col;
      pv[i] = m < p.M;
      const int r = (pv[i] ? m : 0) % HW;
      const int ph = r / W, pw = r - ph * W;
      up[i] = ph > 0;
      down[i] = ph + 1 < p.H;
      left[i] = pw > 0;
      right[i] = pw + 1 < W;
    }
    f32x16 acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int dy = t / 3 - 1, dx = t % 3 - 1;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool ok = pv[i] && (dy < 0 ? up[i] : dy > 0 ? down[i] : true) &&
                        (dx < 0 ? left[i] : dx > 0 ? right[i] : true);
        const uint16_t* arow = &As[(ok ? i * 32 + col + halo + dy * W + dx : kZeroRow) * kActStride + 32 * wave + kh];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const v4u b = *reinterpret_cast<const v4u*>(arow + 16 * h);
          acc[i] = mfma32(as_frag(wr[t * 2 + h]), as_frag(b), acc[i]);
        }
      }
    }
    __syncthreads();  // every wave is done reading the activation band
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (i == wave) continue;
      const int slot = wave < i ? wave : wave - 1;
      f32x4* dst = reinterpret_cast<f32x4*>(red + ((i * 3 + slot) * 64 + lane) * 16);
#pragma unroll
      for (int q = 0; q < 4; ++q) dst[q] = f32x4{acc[i][4 * q], acc[i][4 * q + 1], acc[i][4 * q + 2], acc[i][4 * q + 3]};
    }
    __syncthreads();
    f32x16 sum = acc[0];
#pragma unroll
    for (int i = 1; i < 4; ++i)
      if (i == wave) sum = acc[i];  // static register selection (no dynamic indexing)
#pragma unroll
    for (int sl = 0; sl < 3; ++sl) {
      const f32x4* src = reinterpret_cast<const f32x4*>(red + ((wave * 3 + sl) * 64 + lane) * 16);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 v = src[q];
#pragma unroll
        for (int e = 0; e < 4; ++e) sum[4 * q + e] += v[e];
      }
    }
    const int m = tile * kTileP + wave * 32 + col;
    if (m < p.M) {
      uint16_t* yp = p.y + (size_t)m * p.ldy + 4 * (lane >> 5);
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<v2u*>(yp + 8 * g) =
            v2u{pack2(sum[4 * g], sum[4 * g + 1]), pack2(sum[4 * g + 2], sum[4 * g + 3])};
    }
  }
}

// K9w: K9c with a SLIDING activation band.  K9c re-stages the whole band
// [m0-W-1, m0+128+W+1) of every 128-pixel tile: 242 rows per 128 output
// pixels at 56x56 (1.9x the activation bytes through L2 and LDS, and the
// per-tile load is what bounds it).  Here each block owns a CONTIGUOUS run of
// tiles and keeps the band in a 256-row LDS ring (pixel q lives in ring row
// q & 255): after the first tile of its run a block fetches only the 128 rows
// the next tile adds — issued into registers while the current tile computes,
// written after the barrier over ring rows no later tile of the run reads
// (valid while 2 * (W + 1) <= 128).  Weights LDS-resident as in K9c.
constexpr int kRing = 256;

template <int TU>  // tap-loop unroll (1: as K9c; 9: LDS reads of tap t+1 can overlap tap t's MFMAs)
__global__ void __launch_bounds__(256) conv3x3_ring_kernel(Conv3x3Params p) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* Ws = smem;                   // [32][kWsK]
  uint16_t* As = smem + kN3 * kWsK;      // [kRing + 1][kActStride], row kRing = 0
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  stage_weights(p.w, Ws, tid);
  if (tid < kActStride / 8) *reinterpret_cast<v4u*>(&As[kRing * kActStride + tid * 8]) = v4u{0, 0, 0, 0};
  const int W = p.W, HW = p.H * p.W;
  const int halo = W + 1;
  const int per = p.tiles / (int)gridDim.x, extra = p.tiles % (int)gridDim.x;
  const int t0 = (int)blockIdx.x * per + min((int)blockIdx.x, extra);
  const int t1 = t0 + per + ((int)blockIdx.x < extra ? 1 : 0);
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)p.z, (short)0,
                                                      (int)((size_t)p.M * kC3 * 2), 0x00020000);
  // chunk c (16 B) of pixel rows [first, first + nrows); out-of-range pixels read as 0
  auto fetch = [&](int first, int nrows, int c) -> v4u {
    const int pix = first + (c >> 4);
    const bool ok = c < nrows * 16 && pix >= 0 && pix < p.M;
    return __builtin_amdgcn_raw_buffer_load_b128(rsrc, ok ? (pix * kC3 + (c & 15) * 8) * 2 : 0x40000000, 0, 0);
  };
  auto put = [&](int first, int nrows, int c, v4u v) {
    if (c < nrows * 16)
      *reinterpret_cast<v4u*>(&As[((first + (c >> 4)) & (kRing - 1)) * kActStride + (c & 15) * 8]) = v;
  };
  constexpr int CPT0 = ((kTileP + 2 * 57) * 16 + 255) / 256;  // first band (W <= 56): 16 chunks per thread
  constexpr int CPT = kTileP * 16 / 256;                       // a step's new rows: 8
  if (t0 < t1) {
    const int first = t0 * kTileP - halo, n = kTileP + 2 * halo;
    v4u st0[CPT0];
#pragma unroll
    for (int i = 0; i < CPT0; ++i) st0[i] = fetch(first, n, tid + i * 256);
#pragma unroll
    for (int i = 0; i < CPT0; ++i) put(first, n, tid + i * 256, st0[i]);
  }
  v4u st[CPT];
  const int col = lane & 31, kh = 8 * (lane >> 5);
  for (int tile = t0; tile < t1; ++tile) {
    __syncthreads();  // previous tile's LDS reads done (first time: weights + first band staged)
    if (tile > t0) {
#pragma unroll
      for (int i = 0; i < CPT; ++i) put(tile * kTileP + halo, kTileP, tid + i * 256, st[i]);
    }
    __syncthreads();
    if (tile + 1 < t1) {
#pragma unroll
      for (int i = 0; i < CPT; ++i) st[i] = fetch((tile + 1) * kTileP + halo, kTileP, tid + i * 256);
    }
    const int m = tile * kTileP + wave * 32 + col;
    const int mm = m < p.M ? m : 0;
    const int img = mm / HW, rr = mm - img * HW;
    const int h = rr / W, w = rr - h * W;
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    const bool up = h > 0, down = h + 1 < p.H, left = w > 0, right = w + 1 < W, in = m < p.M;
#pragma unroll TU
    for (int tap = 0; tap < 9; ++tap) {
      const int dy = tap / 3 - 1, dx = tap % 3 - 1;
      const bool ok = in && (dy < 0 ? up : dy > 0 ? down : true) && (dx < 0 ? left : dx > 0 ? right : true);
      const uint16_t* arow = &As[(ok ? ((m + dy * W + dx) & (kRing - 1)) : kRing) * kActStride + kh];
      const uint16_t* wrow = &Ws[col * kWsK + tap * kC3 + kh];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const v4u b = *reinterpret_cast<const v4u*>(arow + c * 16);
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(wrow + c * 16);
        acc = mfma32(a, as_frag(b), acc);
      }
    }
    if (m < p.M) {
      uint16_t* yp = p.y + (size_t)m * p.ldy + 4 * (lane >> 5);
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<v2u*>(yp + 8 * g) =
            v2u{pack2(acc[4 * g], acc[4 * g + 1]), pack2(acc[4 * g + 2], acc[4 * g + 3])};
    }
  }
}

// ============================================================================
// K9w2: K9w with 8 waves (2 per SIMD) instead of 4.  K9w keeps one wave per
// SIMD, so every LDS read an MFMA waits on and every barrier is exposed.
// Here the two waves of a SIMD share one 32-pixel subtile and split its nine
// taps (0-4 / 5-8); the second half's accumulators are added through a 16 KB
// LDS scratch (weights 74 KB + ring 70 KB + scratch 16 KB = 157 KB).
// ============================================================================
constexpr int kRed2Floats = 4 * 64 * 16;  // [subtile][lane][16]

__global__ void __launch_bounds__(512) conv3x3_ring2_kernel(Conv3x3Params p) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* Ws = smem;                                                 // [32][kWsK]
  uint16_t* As = smem + kN3 * kWsK;                                    // [kRing + 1][kActStride]
  float* red = reinterpret_cast<float*>(As + (kRing + 1) * kActStride);  // [4][64][16]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int sub = wave & 3, half = wave >> 2;
  if (tid < 256) stage_weights(p.w, Ws, tid);
  if (tid < kActStride / 8) *reinterpret_cast<v4u*>(&As[kRing * kActStride + tid * 8]) = v4u{0, 0, 0, 0};
  const int W = p.W, HW = p.H * p.W;
  const int halo = W + 1;
  const int per = p.tiles / (int)gridDim.x, extra = p.tiles % (int)gridDim.x;
  const int t0 = (int)blockIdx.x * per + min((int)blockIdx.x, extra);
  const int t1 = t0 + per + ((int)blockIdx.x < extra ? 1 : 0);
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)p.z, (short)0,
                                                      (int)((size_t)p.M * kC3 * 2), 0x00020000);
  auto fetch = [&](int first, int nrows, int c) -> v4u {
    const int pix = first + (c >> 4);
    const bool ok = c < nrows * 16 && pix >= 0 && pix < p.M;
    return __builtin_amdgcn_raw_buffer_load_b128(rsrc, ok ? (pix * kC3 + (c & 15) * 8) * 2 : 0x40000000, 0, 0);
  };
  auto put = [&](int first, int nrows, int c, v4u v) {
    if (c < nrows * 16)
      *reinterpret_cast<v4u*>(&As[((first + (c >> 4)) & (kRing - 1)) * kActStride + (c & 15) * 8]) = v;
  };
  constexpr int CPT0 = ((kTileP + 2 * 57) * 16 + 511) / 512;  // first band: 8 chunks per thread
  constexpr int CPT = kTileP * 16 / 512;                       // a step's new rows: 4
  if (t0 < t1) {
    const int first = t0 * kTileP - halo, n = kTileP + 2 * halo;
    v4u st0[CPT0];
#pragma unroll
    for (int i = 0; i < CPT0; ++i) st0[i] = fetch(first, n, tid + i * 512);
#pragma unroll
    for (int i = 0; i < CPT0; ++i) put(first, n, tid + i * 512, st0[i]);
  }
  v4u st[CPT];
  const int col = lane & 31, kh = 8 * (lane >> 5);
  for (int tile = t0; tile < t1; ++tile) {
    __syncthreads();  // previous tile's LDS reads (ring and scratch) done
    if (tile > t0) {
#pragma unroll
      for (int i = 0; i < CPT; ++i) put(tile * kTileP + halo, kTileP, tid + i * 512, st[i]);
    }
    __syncthreads();
    if (tile + 1 < t1) {
#pragma unroll
      for (int i = 0; i < CPT; ++i) st[i] = fetch((tile + 1) * kTileP + halo, kTileP, tid + i * 512);
    }
    const int m = tile * kTileP + sub * 32 + col;
    const int mm = m < p.M ? m : 0;
    const int img = mm / HW, rr = mm - img * HW;
    const int h = rr / W, w = rr - h * W;
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    const bool up = h > 0, down = h + 1 < p.H, left = w > 0, right = w + 1 < W, in = m < p.M;
#pragma unroll
    for (int t = 0; t < 5; ++t) {
      const int tap = half * 5 + t;  // wave-uniform
      if (tap < 9) {
        const int dy = tap / 3 - 1, dx = tap % 3 - 1;
        const bool ok = in && (dy < 0 ? up : dy > 0 ? down : true) && (dx < 0 ? left : dx > 0 ? right : true);
        const uint16_t* arow = &As[(ok ? ((m + dy * W + dx) & (kRing - 1)) : kRing) * kActStride + kh];
        const uint16_t* wrow = &Ws[col * kWsK + tap * kC3 + kh];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          const v4u b = *reinterpret_cast<const v4u*>(arow + c * 16);
          const bf16x8 a = *reinterpret_cast<const bf16x8*>(wrow + c * 16);
          acc = mfma32(a, as_frag(b), acc);
        }
      }
    }
    f32x4* rp = reinterpret_cast<f32x4*>(red + (sub * 64 + lane) * 16);
    if (half) {
#pragma unroll
      for (int q = 0; q < 4; ++q) rp[q] = f32x4{acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]};
    }
    __syncthreads();
    if (!half && m < p.M) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 o = rp[q];
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[4 * q + e] += o[e];
      }
      uint16_t* yp = p.y + (size_t)m * p.ldy + 4 * (lane >> 5);
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<v2u*>(yp + 8 * g) =
            v2u{pack2(acc[4 * g], acc[4 * g + 1]), pack2(acc[4 * g + 2], acc[4 * g + 3])};
    }
  }
}

// ============================================================================
// K10a: stem epilogue  y = relu(maxpool3x3/2(x) + b)  (bias+ReLU commute with max)
// ============================================================================
// x: [imgs][H][W][C] bf16 (conv0 output without bias), y: [imgs][Ho][Wo] rows of ldy.
// One thread per (output pixel, 8-channel chunk).
__global__ void __launch_bounds__(256) stem_pool_kernel(const uint16_t* __restrict__ x, const float* __restrict__ bias,
                                                        uint16_t* __restrict__ y, int imgs, int H, int W, int C,
                                                        int ldy) {
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2, CC = C / 8;
  const size_t total = (size_t)imgs * Ho * Wo * CC;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (size_t)gridDim.x * blockDim.x) {
    const int cc = (int)(t % CC);
    const size_t pix = t / CC;
    const int ow = (int)(pix % Wo);
    const int oh = (int)((pix / Wo) % Ho);
    const int img = (int)(pix / ((size_t)Wo * Ho));
    float mx[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) mx[e] = -3.0e38f;
    for (int dy = -1; dy <= 1; ++dy) {
      const int h = 2 * oh + dy;
      if (h < 0 || h >= H) continue;
      for (int dx = -1; dx <= 1; ++dx) {
        const int w = 2 * ow + dx;
        if (w < 0 || w >= W) continue;
        float f[8];
        unpack8(ldg16(x + (((size_t)img * H + h) * W + w) * C + cc * 8), f);
#pragma unroll
        for (int e = 0; e < 8; ++e) mx[e] = fmaxf(mx[e], f[e]);
      }
    }
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = fmaxf(mx[e] + bias[cc * 8 + e], 0.f);
    *reinterpret_cast<v4u*>(y + pix * ldy + cc * 8) = pack8(o);
  }
}

// ============================================================================
// K10s: fused stem  y = relu(maxpool3x3/2(conv7x7/2(x)) + b), 3 -> 64 channels
// ============================================================================
// Replaces four passes of the unfused path (K6 fp32 NCHW -> bf16 NHWC batch
// assembly, the library 7x7 conv, its bias op, K10a) with one: a block stages
// the input patch its 4x14 pooled outputs need ([23 rows][72 cols][4 ch] bf16,
// read straight from each request's fp32 NCHW image through a device pointer
// table, so the batch is never assembled), runs the conv for the 9x32 conv
// pixels under the pooling windows as an implicit GEMM on
// v_mfma_f32_32x32x16_bf16 (weights = operand A, 64 x K=7*8*4 with the 8th kw
// and 4th channel zero; one conv row = one 32-pixel MFMA column tile), keeps
// the conv tile in LDS, and max-pools it from there.  For output (r, c) and
// kernel row kh, the K values (kw, ch) are 8 contiguous bf16 per lane in the
// staged patch (stride-2 conv: input col = 2*conv col + kw), so each B
// fragment is one aligned ds_read_b128.  Conv pixels outside the image (row
// or col -1) are excluded from the max, as in max-pool padding.
constexpr int kStemPR = 4, kStemPC = 14;   // pooled outputs per block
constexpr int kStemCR = 2 * kStemPR + 1;   // 9 conv rows
constexpr int kStemCC = 32;                // conv cols computed (2*PC+1 = 29 used)
constexpr int kStemIR = 2 * kStemCR + 5;   // 23 input rows
constexpr int kStemIC = 72;                // input cols (2*31 + 2*3 + 2 = 70 read, padded)
constexpr int kStemK = 7 * 32;             // (kh, kw[8], ch[4])
constexpr int kStemOS = 64 + 4;            // conv-tile pixel stride (bf16): 34 dwords, conflict-free, 3 blocks/CU
constexpr int kStemHin = 224, kStemHo = 56;

struct StemParams {
  const float* const* srcs;  // F32: per-image fp32 NCHW [3][224][224] (device pointer table)
  const uint16_t* x;         // !F32: bf16 NHWC [imgs][224][224][3]
  const uint16_t* w;         // [64][kStemK] packed bf16 (BN0 scale folded)
  const float* bias;         // [64] BN0 shift
  uint16_t* y;               // [imgs][56][56] pixels, rows of ldy
  int ldy;
};

template <bool F32>
__global__ void __launch_bounds__(256) stem_fused_kernel(StemParams p) {
  __shared__ __attribute__((aligned(16))) uint16_t In[kStemIR * kStemIC * 4];        // 13.2 KB
  __shared__ __attribute__((aligned(16))) uint16_t Cv[kStemCR * kStemCC * kStemOS];  // 39 KB
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int img = blockIdx.z, pr0 = blockIdx.y * kStemPR, pc0 = blockIdx.x * kStemPC;
  const int ir0 = 4 * pr0 - 5, ic0 = 4 * pc0 - 5;
  const float* src = F32 ? p.srcs[img] : nullptr;
  // all loads of the patch in flight at once (7 per thread per channel), then the LDS stores
  constexpr int kStage = (kStemIR * kStemIC + 255) / 256;
  float v[kStage][3];
#pragma unroll
  for (int i = 0; i < kStage; ++i) {
    const int e = tid + i * 256;
    const int r = e / kStemIC, c = e - r * kStemIC;
    const int ih = ir0 + r, iw = ic0 + c;
    v[i][0] = v[i][1] = v[i][2] = 0.f;
    if (e < kStemIR * kStemIC && ih >= 0 && ih < kStemHin && iw >= 0 && iw < kStemHin) {
      if (F32) {
        const float* s = src + ih * kStemHin + iw;
        v[i][0] = __builtin_nontemporal_load(s);
        v[i][1] = __builtin_nontemporal_load(s + kStemHin * kStemHin);
        v[i][2] = __builtin_nontemporal_load(s + 2 * kStemHin * kStemHin);
      } else {
        const uint16_t* s = p.x + (((size_t)img * kStemHin + ih) * kStemHin + iw) * 3;
        v[i][0] = tcamd::bf16_to_f32(s[0]);
        v[i][1] = tcamd::bf16_to_f32(s[1]);
        v[i][2] = tcamd::bf16_to_f32(s[2]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < kStage; ++i) {
    const int e = tid + i * 256;
    if (e < kStemIR * kStemIC)
      *reinterpret_cast<v2u*>(&In[e * 4]) = v2u{pack2(v[i][0], v[i][1]), pack2(v[i][2], 0.f)};
  }
  // wave = (channel half nh) x (conv-row group mg: rows 0-4 / 5-8); its 14
  // weight fragments stay in registers for all of its rows
  const int nh = wave & 1, mg = wave >> 1;
  v4u wa[kStemK / 16];
  const uint16_t* wp = p.w + (size_t)(nh * 32 + (lane & 31)) * kStemK + 8 * (lane >> 5);
#pragma unroll
  for (int s = 0; s < kStemK / 16; ++s) wa[s] = ldg16(wp + s * 16);
  __syncthreads();
  const int jj = lane & 31;
  const int r_lo = mg ? 5 : 0, r_hi = mg ? kStemCR : 5;
  for (int cr = r_lo; cr < r_hi; ++cr) {
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
    for (int s = 0; s < kStemK / 16; ++s) {
      const int kh = s >> 1, q = (s & 1) * 2 + (lane >> 5);
      const v4u b = *reinterpret_cast<const v4u*>(&In[((2 * cr + kh) * kStemIC + 2 * jj + 2 * q) * 4]);
      acc = mfma32(as_frag(wa[s]), as_frag(b), acc);
    }
    uint16_t* cp = &Cv[(cr * kStemCC + jj) * kStemOS + nh * 32 + 4 * (lane >> 5)];
#pragma unroll
    for (int g = 0; g < 4; ++g)
      *reinterpret_cast<v2u*>(cp + 8 * g) =
          v2u{pack2(acc[4 * g], acc[4 * g + 1]), pack2(acc[4 * g + 2], acc[4 * g + 3])};
  }
  __syncthreads();
  for (int t = tid; t < kStemPR * kStemPC * 8; t += 256) {
    const int cc = t & 7, px = t >> 3;
    const int a = px / kStemPC, b = px - a * kStemPC;
    const int pr = pr0 + a, pc = pc0 + b;
    float mx[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) mx[e] = -3.0e38f;
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
      if (2 * pr - 1 + dy < 0) continue;
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        if (2 * pc - 1 + dx < 0) continue;
        float f[8];
        const uint16_t* cp = &Cv[((2 * a + dy) * kStemCC + 2 * b + dx) * kStemOS + cc * 8];  // 8-B aligned
        const v2u lo = *reinterpret_cast<const v2u*>(cp), hi = *reinterpret_cast<const v2u*>(cp + 4);
        unpack8(v4u{lo[0], lo[1], hi[0], hi[1]}, f);
#pragma unroll
        for (int e = 0; e < 8; ++e) mx[e] = fmaxf(mx[e], f[e]);
      }
    }
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = fmaxf(mx[e] + p.bias[cc * 8 + e], 0.f);
    *reinterpret_cast<v4u*>(p.y + (((size_t)img * kStemHo + pr) * kStemHo + pc) * p.ldy + cc * 8) = pack8(o);
  }
}

// ============================================================================
// K10b: head  out[img][c] = mean_p relu(x[img][p][c]*s[c] + b[c])   (bf16 out)
// ============================================================================
// One block per image; each thread owns 8-channel chunks and walks the pixels.
__global__ void __launch_bounds__(256) head_pool_kernel(const uint16_t* __restrict__ x, const float* __restrict__ s,
                                                        const float* __restrict__ b, uint16_t* __restrict__ out,
                                                        int HW, int C) {
  const int img = blockIdx.x;
  for (int cc = threadIdx.x; cc < C / 8; cc += blockDim.x) {
    float sc[8], bi[8], acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      sc[e] = s[cc * 8 + e];
      bi[e] = b[cc * 8 + e];
      acc[e] = 0.f;
    }
    for (int p = 0; p < HW; ++p) {
      float f[8];
      unpack8(ldg16(x + ((size_t)img * HW + p) * C + cc * 8), f);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += fmaxf(f[e] * sc[e] + bi[e], 0.f);
    }
    const float inv = 1.0f / (float)HW;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] *= inv;
    *reinterpret_cast<v4u*>(out + (size_t)img * C + cc * 8) = pack8(acc);
  }
}


// ============================================================================
// K9s: small-M 3x3 conv.  Block = 32 pixels x 32 output channels; wave w owns
// input channels [32w, 32w+32) of all 9 taps (9 K chunks), issues all of its
// activation and weight fragment loads up front (one memory round trip
// instead of a tap-by-tap chain), and the 4 partial tiles are summed through
// LDS.  For the 7x7 / 14x14 blocks where K9's persistent 64-pixel tiles leave
// most CUs idle and every block pays for a 73 KB weight preload.
// ============================================================================
__global__ void __launch_bounds__(256) conv3x3_sk_kernel(Conv3x3Params p) {
  __shared__ __attribute__((aligned(16))) f32x4 red[2][4][64];  // [slot][frag][lane], 8 KB
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m0 = blockIdx.x * 32;
  const int fr = lane & 15, fk = 8 * (lane >> 4);
  const int ch0 = wave * 32 + fk;
  const int HW = p.H * p.W;
  int pm[2], ph[2], pw[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + 16 * i + fr;
    pm[i] = m < p.M ? m : -1;
    const int mm = m < p.M ? m : 0;
    const int r = mm % HW;
    ph[i] = r / p.W;
    pw[i] = r - ph[i] * p.W;
  }
  v4u act[9][2], wt[9][2];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int dh = t / 3 - 1, dw = t % 3 - 1;
#pragma unroll
    for (int j = 0; j < 2; ++j) wt[t][j] = ldg16(p.w + (size_t)(16 * j + fr) * kK3 + t * kC3 + ch0);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int h = ph[i] + dh, w = pw[i] + dw;
      const bool ok = pm[i] >= 0 && h >= 0 && h < p.H && w >= 0 && w < p.W;
      act[t][i] = ok ? ldg16(p.z + (size_t)(pm[i] + dh * p.W + dw) * kC3 + ch0) : v4u{0, 0, 0, 0};
    }
  }
  f32x4 acc[2][2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int i = 0; i < 2; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 2; ++i) acc[j][i] = mfma16(as_frag(wt[t][j]), as_frag(act[t][i]), acc[j][i]);

  if (wave >= 2) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 2; ++i) red[wave - 2][j * 2 + i][lane] = acc[j][i];
  }
  __syncthreads();
  if (wave < 2) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 2; ++i) acc[j][i] += red[wave][j * 2 + i][lane];
  }
  __syncthreads();
  if (wave == 1) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 2; ++i) red[0][j * 2 + i][lane] = acc[j][i];
  }
  __syncthreads();
  if (wave != 0) return;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int nb = j * 16 + (lane >> 4) * 4;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (pm[i] < 0) continue;
      const f32x4 a = acc[j][i] + red[0][j * 2 + i][lane];
      *reinterpret_cast<v2u*>(p.y + (size_t)pm[i] * p.ldy + nb) = v2u{pack2(a[0], a[1]), pack2(a[2], a[3])};
    }
  }
}

template <int TM, int BK, bool PRO, bool POOL, int BN = 128>
int launch_1x1(Conv1x1Params p, int splits, hipStream_t s) {
  const int mb = (p.M + 32 * TM - 1) / (32 * TM), nb = p.N / BN;
  if (splits > 1) {
    const int kts = (p.K + BK - 1) / BK;
    const int per = (kts + splits - 1) / splits;
    splits = (kts + per - 1) / per;
    p.k_per_split = per * BK;
  } else {
    p.ws = nullptr;
  }
  dim3 g(mb, nb, splits > 1 ? splits : 1);
  hipLaunchKernelGGL((conv1x1_kernel<TM, BK, PRO, POOL, BN>), g, dim3(256), 0, s, p);
  if (splits > 1) {
    const size_t total = (size_t)p.M * (p.N / 4);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(tcamd::grid_for(total)), dim3(256), 0, s, p.ws, splits, p.M, p.N,
                       p.out_bias, p.relu_out, p.y, p.ldy);
  }
  return hipGetLastError();
}

// K8p launch: one persistent block per resident slot (occupancy x CUs), or
// one per tile when there are fewer tiles.
template <int TM, int D, bool PRO>
int launch_1x1_pipe(const Conv1x1Params& p, hipStream_t s) {
  static int slots = 0;
  if (!slots) {
    int dev = 0, cus = 0, occ = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, conv1x1_pipe_kernel<TM, D, PRO>, 256, 0) != hipSuccess)
      return hipErrorInvalidValue;
    slots = std::max(1, cus * occ);
  }
  const int tiles = ((p.M + 32 * TM - 1) / (32 * TM)) * (p.N / 128);
  hipLaunchKernelGGL((conv1x1_pipe_kernel<TM, D, PRO>), dim3(std::min(tiles, slots)), dim3(256), 0, s, p);
  return hipGetLastError();
}

// variant: 0 = heuristic, else 10*TM + BK/32 (e.g. 42 = TM 4, BK 64)
// variant: 0 = heuristic, else 10*TM + BK/32.  splits: 0 = heuristic (needs a
// workspace), 1 = no split-K.  Heuristic from tools/kbench_densenet.py on
// MI355X: TM 2 / BK 32 once M >= 32K rows, TM 1 below; BK 64 for small M,
// where the launch is latency-bound over K; small grids split K until ~256
// blocks run (the reduce launch costs ~2 us, so only when it pays).
template <bool PRO, bool POOL>
int pick_1x1(const Conv1x1Params& p, int variant, int splits, size_t ws_bytes, hipStream_t s) {
  // measured (tools/kbench_densenet.py, bs128): the 56x56 layers (M >= 196k) run
  // 10-15% faster on 128-pixel tiles (TM=4) than on 64 (K=224: 80 vs 95 us);
  // the 14x14 layers (M = 25k) ~12% faster on 64-pixel tiles than on 32
  // (K=992: 23.6 vs 27.7 us)
  if (variant == 0)
    variant = p.M >= 196608 ? 41 : p.M >= 16384 ? 21 : p.M >= 8192 ? 11 : (p.M > 4096 && !POOL) ? 212 : 12;
  if (variant == 300) {  // K8w: weight-resident whole-K (K <= 256, BN prologue, no pool / split)
    if (!PRO || POOL || p.K % 32 || p.K > 256 || p.N % 128) return hipErrorInvalidValue;
    if (p.ldy % 8 || ((uintptr_t)p.y) % 16) return hipErrorInvalidValue;  // 16-B output rows
    return launch_1x1_wres_k(p, s);
  }
  if (variant == 70) {  // K8s: waves split K (needs the BN prologue)
    if (!PRO || p.K % 32) return hipErrorInvalidValue;
    hipLaunchKernelGGL((conv1x1_sk_kernel<POOL>), dim3((p.M + 31) / 32, p.N / 128), dim3(256), 0, s, p);
    return hipGetLastError();
  }
  if (variant > 200) {  // K8 with 64-channel block tiles: 200 + 10*TM + BK/32 (2x the blocks for small M)
    if (p.N % 64) return hipErrorInvalidValue;
    const int tm = (variant - 200) / 10, bk = (variant % 10) * 32;
    const long blocks = (long)((p.M + 32 * tm - 1) / (32 * tm)) * (p.N / 64);
    const int kts = (p.K + bk - 1) / bk;
    if (splits == 0) {
      splits = 1;
      if (p.ws && blocks < 128 && kts >= 4) {
        splits = (int)((256 + blocks - 1) / blocks);
        if (splits > kts / 2) splits = kts / 2;
        if (splits > 16) splits = 16;
      }
    }
    if (splits > 1 && (!p.ws || ws_bytes < (size_t)splits * p.M * p.N * sizeof(float))) splits = 1;
    switch (variant) {
      case 211: return launch_1x1<1, 32, PRO, POOL, 64>(p, splits, s);
      case 212: return launch_1x1<1, 64, PRO, POOL, 64>(p, splits, s);
      case 221: return launch_1x1<2, 32, PRO, POOL, 64>(p, splits, s);
      case 222: return launch_1x1<2, 64, PRO, POOL, 64>(p, splits, s);
      default: return hipErrorInvalidValue;
    }
  }
  if (variant > 100) {  // K8p: 100 + 10*TM + pipeline depth (no split-K, no pool)
    if (POOL || p.K % 32 || p.N > kMaxK) return hipErrorInvalidValue;
    switch (variant) {
      case 112: return launch_1x1_pipe<1, 2, PRO>(p, s);
      case 113: return launch_1x1_pipe<1, 3, PRO>(p, s);
      case 114: return launch_1x1_pipe<1, 4, PRO>(p, s);
      case 122: return launch_1x1_pipe<2, 2, PRO>(p, s);
      case 123: return launch_1x1_pipe<2, 3, PRO>(p, s);
      case 124: return launch_1x1_pipe<2, 4, PRO>(p, s);
      case 142: return launch_1x1_pipe<4, 2, PRO>(p, s);
      case 143: return launch_1x1_pipe<4, 3, PRO>(p, s);
      default: return hipErrorInvalidValue;
    }
  }
  const int tm = variant / 10, bk = (variant % 10) * 32;
  const long blocks = (long)((p.M + 32 * tm - 1) / (32 * tm)) * (p.N / 128);
  const int kts = (p.K + bk - 1) / bk;
  if (splits == 0) {
    splits = 1;
    if (p.ws && blocks < 128 && kts >= 4) {
      splits = (int)((256 + blocks - 1) / blocks);
      if (splits > kts / 2) splits = kts / 2;
      if (splits > 16) splits = 16;
    }
  }
  if (splits > 1 && (!p.ws || ws_bytes < (size_t)splits * p.M * p.N * sizeof(float))) splits = 1;
  switch (variant) {
    case 11: return launch_1x1<1, 32, PRO, POOL>(p, splits, s);
    case 12: return launch_1x1<1, 64, PRO, POOL>(p, splits, s);
    case 21: return launch_1x1<2, 32, PRO, POOL>(p, splits, s);
    case 22: return launch_1x1<2, 64, PRO, POOL>(p, splits, s);
    case 41: return launch_1x1<4, 32, PRO, POOL>(p, splits, s);
    case 42: return launch_1x1<4, 64, PRO, POOL>(p, splits, s);
    default: return hipErrorInvalidValue;
  }
}

template <int TM, int G>
int launch_3x3(Conv3x3Params p, hipStream_t s) {
  static bool attr = false;
  const int lds = kN3 * kWsK * 2;
  if (!attr) {
    int rc = hipFuncSetAttribute((const void*)conv3x3_kernel<TM, G>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (rc != hipSuccess) return rc;
    attr = true;
  }
  p.tiles = (p.M + 64 * TM - 1) / (64 * TM);
  const int grid = p.tiles < 512 ? p.tiles : 512;  // 2 resident blocks per CU (LDS-limited)
  hipLaunchKernelGGL((conv3x3_kernel<TM, G>), dim3(grid), dim3(256), lds, s, p);
  return hipGetLastError();
}

template <int TM>
int launch_3x3_m32(Conv3x3Params p, hipStream_t s) {
  static bool attr = false;
  const int lds = kN3 * kWsK * 2;
  if (!attr) {
    int rc = hipFuncSetAttribute((const void*)conv3x3_m32_kernel<TM>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (rc != hipSuccess) return rc;
    attr = true;
  }
  p.tiles = (p.M + 128 * TM - 1) / (128 * TM);
  const int grid = p.tiles < 512 ? p.tiles : 512;
  hipLaunchKernelGGL((conv3x3_m32_kernel<TM>), dim3(grid), dim3(256), lds, s, p);
  return hipGetLastError();
}

int launch_3x3_kr(Conv3x3Params p, hipStream_t s) {
  if (p.W > 56) return hipErrorInvalidValue;
  const int lds = (kZeroRow + 1) * kActStride * 2;  // band + zero row (the reduction aliases the band)
  static int attr = 0;
  const int lmax = lds;
  if (attr < lmax) {
    int rc = hipFuncSetAttribute((const void*)conv3x3_kr_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lmax);
    if (rc != hipSuccess) return rc;
    attr = lmax;
  }
  p.tiles = (p.M + kTileP - 1) / kTileP;
  const int grid = p.tiles < 512 ? p.tiles : 512;  // two resident blocks per CU
  hipLaunchKernelGGL(conv3x3_kr_kernel, dim3(grid), dim3(256), lds, s, p);
  return hipGetLastError();
}

int launch_3x3_ring2(Conv3x3Params p, hipStream_t s) {
  if (p.W > 56) return hipErrorInvalidValue;
  const int lds = (kN3 * kWsK + (kRing + 1) * kActStride) * 2 + kRed2Floats * 4;
  static int attr = 0;
  if (attr < lds) {
    int rc = hipFuncSetAttribute((const void*)conv3x3_ring2_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (rc != hipSuccess) return rc;
    attr = lds;
  }
  p.tiles = (p.M + kTileP - 1) / kTileP;
  const int grid = p.tiles < 256 ? p.tiles : 256;
  hipLaunchKernelGGL(conv3x3_ring2_kernel, dim3(grid), dim3(512), lds, s, p);
  return hipGetLastError();
}

template <int TU>
int launch_3x3_ring(Conv3x3Params p, hipStream_t s) {
  if (p.W > 56) return hipErrorInvalidValue;  // ring reuse needs 2 * (W + 1) <= kTileP
  const int lds = (kN3 * kWsK + (kRing + 1) * kActStride) * 2;
  static int attr = 0;
  if (attr < lds) {
    int rc = hipFuncSetAttribute((const void*)conv3x3_ring_kernel<TU>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (rc != hipSuccess) return rc;
    attr = lds;
  }
  p.tiles = (p.M + kTileP - 1) / kTileP;
  const int grid = p.tiles < 256 ? p.tiles : 256;  // one resident block per CU (LDS-limited)
  hipLaunchKernelGGL(conv3x3_ring_kernel<TU>, dim3(grid), dim3(256), lds, s, p);
  return hipGetLastError();
}

int launch_3x3_lds(Conv3x3Params p, hipStream_t s) {
  if (p.W > 56) return hipErrorInvalidValue;
  const int lds = (kN3 * kWsK + (kZeroRow + 1) * kActStride) * 2;
  static int attr = 0;
  if (attr < lds) {
    int rc = hipFuncSetAttribute((const void*)conv3x3_lds_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (kN3 * kWsK + (kZeroRow + 1) * kActStride) * 2);
    if (rc != hipSuccess) return rc;
    attr = (kN3 * kWsK + (kZeroRow + 1) * kActStride) * 2;
  }
  p.tiles = (p.M + kTileP - 1) / kTileP;
  const int grid = p.tiles < 256 ? p.tiles : 256;  // one resident block per CU (LDS-limited)
  hipLaunchKernelGGL(conv3x3_lds_kernel, dim3(grid), dim3(256), lds, s, p);
  return hipGetLastError();
}

}  // namespace

extern "C" {

// 1x1 conv (GEMM) with optional fused pre-activation BN+ReLU (in_scale/in_bias
// non-null) and 2x2 average pool (pool != 0; H, W = pre-pool dims, M = pooled
// rows).  Requires K % 32 == 0, K <= 1024 when fused, N % 128 == 0,
// ldx/ldy/y offsets multiples of 8 elements and 16-B aligned x/w.
int tcamd_dn_conv1x1_ex(const void* x, int ldx, int M, int K, const float* in_scale, const float* in_bias,
                        const void* w, int N, const float* out_bias, int relu_out, void* y, int ldy, int pool, int H,
                        int W, int variant, int splits, void* ws, size_t ws_bytes, void* stream) {
  if (M <= 0) return hipSuccess;
  if (K % 32 || N % 128 || ldx % 8 || ldy % 4 || K > ldx) return hipErrorInvalidValue;
  const bool pro = in_scale != nullptr && in_bias != nullptr;
  if (pro && K > kMaxK) return hipErrorInvalidValue;
  if (pool && (!pro || H % 2 || W % 2)) return hipErrorInvalidValue;
  if (((uintptr_t)x | (uintptr_t)w) % 16 || ((uintptr_t)y) % 8) return hipErrorInvalidValue;
  Conv1x1Params p;
  p.x = (const uint16_t*)x;
  p.in_scale = in_scale;
  p.in_bias = in_bias;
  p.w = (const uint16_t*)w;
  p.out_bias = out_bias;
  p.y = (uint16_t*)y;
  p.ldx = ldx;
  p.M = M;
  p.K = K;
  p.N = N;
  p.ldy = ldy;
  p.relu_out = relu_out;
  p.H = H;
  p.W = W;
  p.ws = (float*)ws;
  p.k_per_split = 0;
  if (ws && ((uintptr_t)ws) % 16) return hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  if (pool) return pick_1x1<true, true>(p, variant, splits, ws_bytes, s);
  if (pro) return pick_1x1<true, false>(p, variant, splits, ws_bytes, s);
  return pick_1x1<false, false>(p, variant, splits, ws_bytes, s);
}

int tcamd_dn_conv1x1_v(const void* x, int ldx, int M, int K, const float* in_scale, const float* in_bias,
                       const void* w, int N, const float* out_bias, int relu_out, void* y, int ldy, int pool, int H,
                       int W, int variant, void* stream) {
  return tcamd_dn_conv1x1_ex(x, ldx, M, K, in_scale, in_bias, w, N, out_bias, relu_out, y, ldy, pool, H, W,
                             variant, 1, nullptr, 0, stream);
}

int tcamd_dn_conv1x1(const void* x, int ldx, int M, int K, const float* in_scale, const float* in_bias,
                     const void* w, int N, const float* out_bias, int relu_out, void* y, int ldy, int pool, int H,
                     int W, void* stream) {
  return tcamd_dn_conv1x1_v(x, ldx, M, K, in_scale, in_bias, w, N, out_bias, relu_out, y, ldy, pool, H, W, 0, stream);
}

// 3x3 conv 128->32, pad 1, over z [imgs*H*W][128]; w [32][3][3][128];
// writes 32 channels per pixel at y + pixel*ldy.
int tcamd_dn_conv3x3_v(const void* z, int imgs, int H, int W, const void* w, void* y, int ldy, int variant,
                       void* stream) {
  const long M = (long)imgs * H * W;
  if (M <= 0) return hipSuccess;
  if (M * kC3 * 2 >= 0x3ffff000L || ldy % 4) return hipErrorInvalidValue;
  if (((uintptr_t)z | (uintptr_t)w) % 16 || ((uintptr_t)y) % 8) return hipErrorInvalidValue;
  Conv3x3Params p;
  p.ablate = variant / 1000;
  variant %= 1000;
  p.z = (const uint16_t*)z;
  p.w = (const uint16_t*)w;
  p.y = (uint16_t*)y;
  p.M = (int)M;
  p.H = H;
  p.W = W;
  p.ldy = ldy;
  hipStream_t s = (hipStream_t)stream;
  // heuristic from tools/kbench_densenet.py on MI355X: tiny problems
  // (M <= 8192: the 7x7 / 14x14 layers of small batches) take the wave-split
  // K9s, and above that the sliding-band K9w2 (8 waves, taps split between
  // SIMD-mates; bs128 on MI355X: 56x56 43 us vs 45 K9w / 55 K9r / 60 K9c,
  // 28x28 15.8 vs 16.7 / 20.3 / 21.9, 14x14 6.3 vs 6.6 / 8.2 / 7.3;
  // profiles/r1_kbench_3x3_ring.log)
  if (variant == 0)
    variant = M <= 8192 ? 70 : W <= 56 ? 92 : 11;
  switch (variant) {
    case 10: return launch_3x3<1, 0>(p, s);  // channel-major tap walk
    case 16: return launch_3x3<1, 6>(p, s);   // 6-deep load ring
    case 19: return launch_3x3<1, 12>(p, s);  // 12-deep load ring
    case 29: return launch_3x3<2, 12>(p, s);
    case 26: return launch_3x3<2, 6>(p, s);
    case 20: return launch_3x3<2, 0>(p, s);
    case 11: return launch_3x3<1, 1>(p, s);
    case 13: return launch_3x3<1, 3>(p, s);
    case 21: return launch_3x3<2, 1>(p, s);
    case 23: return launch_3x3<2, 3>(p, s);
    case 41: return launch_3x3<4, 1>(p, s);
    case 60: return launch_3x3_lds(p, s);     // LDS-staged activations, 32x32x16 MFMA
    case 80: return launch_3x3_kr(p, s);      // K9r: weights in registers, K split over waves
    case 90: return launch_3x3_ring<1>(p, s); // K9w: K9c with a sliding band (contiguous tile runs)
    case 91: return launch_3x3_ring<9>(p, s); // K9w, taps fully unrolled
    case 93: return launch_3x3_ring<3>(p, s); // K9w, taps unrolled by 3
    case 92: return launch_3x3_ring2(p, s);   // K9w2: 8 waves, taps split between SIMD-mates
    case 70:                                  // K9s: waves split the input channels
      hipLaunchKernelGGL(conv3x3_sk_kernel, dim3((p.M + 31) / 32), dim3(256), 0, s, p);
      return hipGetLastError();
    case 51: return launch_3x3_m32<1>(p, s);  // 32x32x16 MFMA, 32 px / wave
    case 52: return launch_3x3_m32<2>(p, s);  // 32x32x16 MFMA, 64 px / wave
    default: return hipErrorInvalidValue;
  }
}

int tcamd_dn_conv3x3(const void* z, int imgs, int H, int W, const void* w, void* y, int ldy, void* stream) {
  return tcamd_dn_conv3x3_v(z, imgs, H, W, w, y, ldy, 0, stream);
}

int tcamd_dn_stem_pool(const void* x, const float* bias, void* y, int imgs, int H, int W, int C, int ldy,
                       void* stream) {
  if (imgs <= 0) return hipSuccess;
  if (C % 8 || ldy % 8) return hipErrorInvalidValue;
  const size_t total = (size_t)imgs * ((H + 1) / 2) * ((W + 1) / 2) * (C / 8);
  hipLaunchKernelGGL(stem_pool_kernel, dim3(tcamd::grid_for(total)), dim3(256), 0, (hipStream_t)stream,
                     (const uint16_t*)x, bias, (uint16_t*)y, imgs, H, W, C, ldy);
  return hipGetLastError();
}

// Fused stem over 224x224x3 images -> 56x56x64 (conv 7x7/2 pad 3, bias, ReLU,
// max-pool 3x3/2 pad 1).  srcs (device array of imgs fp32 NCHW image
// pointers) if non-null, else x = bf16 NHWC [imgs][224][224][3].
// w = [64][7][8][4] bf16 (zero at kw 7 / ch 3); y rows of ldy elements.
int tcamd_dn_stem_fused(const void* srcs, const void* x, const void* w, const float* bias, void* y, int imgs,
                        int ldy, void* stream) {
  if (imgs <= 0) return hipSuccess;
  if (ldy % 8 || ldy < 64 || (!srcs && !x) || !w || !bias || !y) return hipErrorInvalidValue;
  if (((uintptr_t)w | (uintptr_t)y) % 16 || (srcs && (uintptr_t)srcs % 8)) return hipErrorInvalidValue;
  StemParams p;
  p.srcs = (const float* const*)srcs;
  p.x = (const uint16_t*)x;
  p.w = (const uint16_t*)w;
  p.bias = bias;
  p.y = (uint16_t*)y;
  p.ldy = ldy;
  const dim3 g(kStemHo / kStemPC, kStemHo / kStemPR, imgs);
  if (srcs)
    hipLaunchKernelGGL(stem_fused_kernel<true>, g, dim3(256), 0, (hipStream_t)stream, p);
  else
    hipLaunchKernelGGL(stem_fused_kernel<false>, g, dim3(256), 0, (hipStream_t)stream, p);
  return hipGetLastError();
}

int tcamd_dn_head_pool(const void* x, const float* s, const float* b, void* out, int imgs, int HW, int C,
                       void* stream) {
  if (imgs <= 0) return hipSuccess;
  if (C % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(head_pool_kernel, dim3(imgs), dim3(128), 0, (hipStream_t)stream, (const uint16_t*)x, s, b,
                     (uint16_t*)out, HW, C);
  return hipGetLastError();
}

}  // extern "C"
