// K13x — the small-M fp32-parity dense layers (bs1-4 at every block width,
// bs8-16 at 14x14 / 7x7; the engine's default limit is 3,136 pixels).
//
// At small M the K8x/K9x pair is latency-bound, not byte- or MFMA-bound: a
// bs1 14x14 layer is 196 pixels, and its 3x3 (K9x with the split-K partials
// summed while staging) ran on 4 CUs, each pulling the whole 147 KB of 3x3
// weights plus 4 x 94 rows of fp32 partials before its first MFMA — 11 us per
// layer for ~1 us of matrix work (profiles/r3_x3_forward_b1.md: the 48
// small-M 3x3s were 52% of a 1.02 ms bs1 forward).  Two designs live here,
// both spreading their operand bytes over many workgroups with short, fully
// in-flight load lists (profiles/r3_x3s_small_m.md):
//
// The chain (default, x3c_* below): one launch per layer.  A layer's 1x1 is
// linear in its per-channel activated inputs, so each layer's 32 new
// channels are folded into every later layer's fp32 accumulator as soon as
// they exist; a layer's launch adds the previous layer's chunk for its tile
// and halo, runs its 3x3 (tiles x 4 input quarters) and fans that chunk out
// to the later layers.  bs1 forward 0.978 -> 0.457 ms.
//
// Two launches per layer (x3s_*; TCAMD_X3_CHAIN=0, and the fallback):
//   S1 (1x1, K -> 128): grid = 32-pixel tiles x 4 output quarters x K chunks;
//      the 4 waves of a block take interleaved k16 steps of the block's chunk
//      straight from global memory (A = BN2-folded W1 hi/lo in the K11x
//      fragment-major copy, one 1 KB wave load per step; B = X with BN1+ReLU
//      and the hi/lo split applied in registers), sum through LDS, and add
//      the 32 x 32 fp32 tile into zacc with global float atomics (two whole
//      128-B row segments per wave instruction).  zacc is zero on entry.
//   S2 (3x3, 128 -> 32): grid = 32-pixel tiles x 4 input quarters (or all
//      quarters per block), each wave loading its taps' weight fragments (K9x
//      layout) and its pixels' zacc rows directly (bias + ReLU + split in
//      registers, zero for taps outside the image), summed through LDS and
//      added into (or stored as) the layer's 32 new fp32 channels.  The same
//      blocks zero the NEXT layer's zacc (a ping-pong pair): no memset launch.
//
// Precision: the same bf16x3 products as K8x/K9x.  The float atomics sum in
// arrival order (last-bit run-to-run differences, ~6e-6 rel-L2 on the
// logits; see tcamd_x3s_steps_per_block for the reproducible setting of the
// two-launch path).  Float atomics run at memory side at ~1.3 TB/s chip-wide
// (MI355X_MICROARCH.md, Global float atomics); every launch here adds at
// most a few hundred KB.

#include <algorithm>
#include <cstdlib>

#include "kernels/common.h"
#include "kernels/knobs.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ v4u ld16(const void* p) { return *reinterpret_cast<const v4u*>(p); }
__device__ __forceinline__ f32x4 ldf4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }

__device__ __forceinline__ uint32_t pk(float a, float b) {
  const bf16x2 v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}

// 8 fp32 -> hi/lo bf16x8 fragments (a ~= hi + lo to 2^-17 relative)
__device__ __forceinline__ void split8(f32x4 a, f32x4 b, v4u& hi, v4u& lo) {
  const float v[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t h = pk(v[2 * i], v[2 * i + 1]);
    hi[i] = h;
    lo[i] = pk(v[2 * i] - __uint_as_float(h << 16), v[2 * i + 1] - __uint_as_float(h & 0xffff0000u));
  }
}

__device__ __forceinline__ bf16x8 fr(v4u v) { return __builtin_bit_cast(bf16x8, v); }

__device__ __forceinline__ f32x16 x3_32(v4u ah, v4u al, v4u bh, v4u bl, f32x16 c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fr(al), fr(bh), c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fr(ah), fr(bl), c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(fr(ah), fr(bh), c, 0, 0, 0);
}

constexpr int kZ = 128;        // bottleneck channels
constexpr int kTile = 32;      // pixels per block
constexpr int kRedPitch = 36;  // floats per pixel row of an LDS reduction slab (16-B aligned rows)

// one wave's 32x32 accumulator tile (C[out][px]: lane (h, col) holds outputs
// 8g + 4h + e of pixel col) -> slab[px][out]
__device__ __forceinline__ void put_tile(float* slab, const f32x16& acc, int col, int h) {
#pragma unroll
  for (int g = 0; g < 4; ++g)
    *reinterpret_cast<f32x4*>(slab + col * kRedPitch + 8 * g + 4 * h) =
        f32x4{acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]};
}

struct X3sConv1x1Params {
  const float* x;  // [M][ldx] fp32, the layer's first K channels
  const float* s1;  // [K] BN1 affine
  const float* t1;
  const uint16_t* w1_hi;  // x3_w1_fragments: [K/16][q 4][lane 64][8]
  const uint16_t* w1_lo;
  float* zacc;  // [M][128] fp32, zero on entry, += this conv
  float* y_zero;  // split 3x3 (atomic y): the layer's 32-channel y slice, zeroed here (else null)
  int ldy;
  int ldx, M, K;
  int steps_per_block;  // k16 steps per K chunk (blockIdx.z)
};

// U k16 steps per wave in flight: their 8 loads a step are issued together
constexpr int kU1 = 4;

__global__ void __launch_bounds__(256) x3s_conv1x1_kernel(X3sConv1x1Params p) {
  __shared__ __attribute__((aligned(16))) float red[4][kTile * kRedPitch];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = lane & 31, h = lane >> 5;
  const int m0 = blockIdx.x * kTile, q = blockIdx.y;
  const int nst = p.K / 16;
  const int sb = blockIdx.z * p.steps_per_block, se = min(nst, sb + p.steps_per_block);
  const int m = m0 + col;
  const bool in = m < p.M;
  const float* xr = p.x + (size_t)(in ? m : 0) * p.ldx + 8 * h;
  const float* sr = p.s1 + 8 * h;
  const float* tr = p.t1 + 8 * h;
  if (p.y_zero && q == 0 && blockIdx.z == 0) {
    // the split 3x3 adds its input-quarter partials into y: zero the tile's slice
    const int px = threadIdx.x >> 3;
    if (m0 + px < p.M) *reinterpret_cast<f32x4*>(p.y_zero + (size_t)(m0 + px) * p.ldy + 4 * (threadIdx.x & 7)) = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  f32x16 acc;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.f;
  for (int s0 = sb + wave; s0 < se; s0 += 4 * kU1) {
    v4u ah[kU1], al[kU1];
    f32x4 xa[kU1], xb[kU1], sa[kU1], sc[kU1], ta[kU1], tc[kU1];
#pragma unroll
    for (int u = 0; u < kU1; ++u) {
      const int s = min(s0 + 4 * u, se - 1);  // dead steps re-load a live one and multiply zeros
      const size_t wo = ((size_t)(s * 4 + q) * 64 + lane) * 8;
      ah[u] = ld16(p.w1_hi + wo);
      al[u] = ld16(p.w1_lo + wo);
      const int k = 16 * s;
      xa[u] = ldf4(xr + k);
      xb[u] = ldf4(xr + k + 4);
      sa[u] = ldf4(sr + k);
      sc[u] = ldf4(sr + k + 4);
      ta[u] = ldf4(tr + k);
      tc[u] = ldf4(tr + k + 4);
    }
    // straight-line: a dead step multiplies zeros (a branch here made the
    // compiler sink each step's loads to its use, one HBM round trip a step)
#pragma unroll
    for (int u = 0; u < kU1; ++u) {
      const bool live = in && s0 + 4 * u < se;
      f32x4 va, vb;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        va[e] = live ? fmaxf(xa[u][e] * sa[u][e] + ta[u][e], 0.f) : 0.f;
        vb[e] = live ? fmaxf(xb[u][e] * sc[u][e] + tc[u][e], 0.f) : 0.f;
      }
      v4u bh, bl;
      split8(va, vb, bh, bl);
      acc = x3_32(ah[u], al[u], bh, bl, acc);
    }
  }
  put_tile(red[wave], acc, col, h);
  __syncthreads();
  // 2 pixels x 32 outputs per wave instruction: two whole 128-B segments of zacc
  const int oc = threadIdx.x & 31;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int px = (threadIdx.x >> 5) + 8 * j;
    const float v = red[0][px * kRedPitch + oc] + red[1][px * kRedPitch + oc] + red[2][px * kRedPitch + oc] +
                    red[3][px * kRedPitch + oc];
    if (m0 + px < p.M) atomicAdd(p.zacc + (size_t)(m0 + px) * kZ + 32 * q + oc, v);
  }
}

struct X3sConv3x3Params {
  const float* zacc;  // [M][128] fp32 1x1 sums (bias not yet added)
  const float* b1;    // [128] BN2-folded bias
  const uint16_t* w_hi;  // x3_w3_fragments: [tap 9][kq 4][kc 2][lane 64][8]
  const uint16_t* w_lo;
  float* y;  // [M][ldy], offset to the layer's 32-channel slice
  float* zero_next;  // the next layer's zacc: rows [0, zero_rows) zeroed here (may be null)
  int ldy, M, H, W, zero_rows;
};

// NKQ input-channel quarters per block x TG tap groups = the block's waves;
// a wave takes taps tg, tg + TG, ... .  NKQ 4: all of K in the block, y
// stored; NKQ 1: one quarter per block (grid.y = 4), a quarter of the weight
// bytes per block, y accumulated with float atomics (zeroed by S1)
template <int NKQ, int TG>
__global__ void __launch_bounds__(64 * NKQ * TG) x3s_conv3x3_kernel(X3sConv3x3Params p) {
  constexpr int NW = NKQ * TG, NT = (9 + TG - 1) / TG;
  __shared__ __attribute__((aligned(16))) float red[NW][kTile * kRedPitch];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 31, h = lane >> 5;
  const int kq = NKQ == 4 ? (wave & 3) : (int)blockIdx.y, tg = NKQ == 4 ? (wave >> 2) : wave;
  const int m0 = blockIdx.x * kTile;

  if (p.zero_next && (NKQ == 4 || blockIdx.y == 0)) {
    // rows [m0, m0 + 32) of the next layer's accumulator: 1024 float4
#pragma unroll
    for (int j = 0; j < 1024 / (64 * NW); ++j) {
      const int i = tid + 64 * NW * j;
      const int r = m0 + (i >> 5);
      if (r < p.zero_rows) *reinterpret_cast<f32x4*>(p.zero_next + (size_t)r * kZ + 4 * (i & 31)) = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }

  const int m = m0 + col;
  const bool in = m < p.M;
  const int HW = p.H * p.W;
  const int r = in ? m % HW : 0;
  const int yy = r / p.W, xx = r - yy * p.W;

  f32x4 ba[2], bb[2];
#pragma unroll
  for (int kc = 0; kc < 2; ++kc) {
    const int c = 32 * kq + 16 * kc + 8 * h;
    ba[kc] = ldf4(p.b1 + c);
    bb[kc] = ldf4(p.b1 + c + 4);
  }
  v4u wh[NT][2], wl[NT][2];
  f32x4 za[NT][2], zb[NT][2];
  bool ok[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    const int t = min(tg + TG * i, 8);
    const int dy = t / 3 - 1, dx = t % 3 - 1;
    const int y2 = yy + dy, x2 = xx + dx;
    ok[i] = in && tg + TG * i < 9 && y2 >= 0 && y2 < p.H && x2 >= 0 && x2 < p.W;
    const int mm = ok[i] ? m + dy * p.W + dx : 0;
#pragma unroll
    for (int kc = 0; kc < 2; ++kc) {
      const size_t wo = ((size_t)((t * 4 + kq) * 2 + kc) * 64 + lane) * 8;
      wh[i][kc] = ld16(p.w_hi + wo);
      wl[i][kc] = ld16(p.w_lo + wo);
      const float* zr = p.zacc + (size_t)mm * kZ + 32 * kq + 16 * kc + 8 * h;
      za[i][kc] = ldf4(zr);
      zb[i][kc] = ldf4(zr + 4);
    }
  }
  f32x16 acc;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
  for (int i = 0; i < NT; ++i) {  // a wave's dead last tap (ok = false) multiplies zeros
#pragma unroll
    for (int kc = 0; kc < 2; ++kc) {
      f32x4 va, vb;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        // ReLU(z + b) of a pixel outside the image is padding: zero, not ReLU(b)
        va[e] = ok[i] ? fmaxf(za[i][kc][e] + ba[kc][e], 0.f) : 0.f;
        vb[e] = ok[i] ? fmaxf(zb[i][kc][e] + bb[kc][e], 0.f) : 0.f;
      }
      v4u bh, bl;
      split8(va, vb, bh, bl);
      acc = x3_32(wh[i][kc], wl[i][kc], bh, bl, acc);
    }
  }
  put_tile(red[wave], acc, col, h);
  __syncthreads();
  const int oc = tid & 31;
#pragma unroll
  for (int j = 0; j < 1024 / (64 * NW); ++j) {
    const int px = (tid >> 5) + 2 * NW * j;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += red[w][px * kRedPitch + oc];
    if (m0 + px < p.M) {
      if (NKQ == 4) p.y[(size_t)(m0 + px) * p.ldy + oc] = v;
      else atomicAdd(p.y + (size_t)(m0 + px) * p.ldy + oc, v);
    }
  }
}


// ============================================================================
// K13x chain: one launch per small-M dense layer
// ============================================================================
// A layer's 1x1 is linear in its per-channel activated inputs, so the
// contribution of each 32-channel chunk (one earlier layer's output) to each
// later layer's bottleneck accumulator can be added as soon as that chunk
// exists.  Over a run of small-M layers f..L-1 of one dense block:
//   base launch: zacc_l = W1_l[:, 0:K_f] . act_l(x[:, 0:K_f]) for every l
//                (plain stores), and the y slices of every layer zeroed;
//   layer l:     part A (tiles x 4 input quarters): the 3x3 of layer l from
//                zacc_l + the chunk of layer l-1 (computed here for the tile
//                and its halo rows: 2 k16 steps), bias + ReLU + split into an
//                LDS band, 9 taps, float atomics into y_l;
//                part B (tiles x later layers, l > f): the chunk of layer l-1
//                fanned out into zacc_l' for every l' > l (read-add-write: in
//                one launch each element has exactly one writer).
// So zacc_l = base + the chunks of layers f..l-2 (parts B of launches
// f+1..l-1, in layer order: deterministic) + chunk l-1 (part A) when its 3x3
// runs: one launch per layer instead of two, one more per run.
struct X3cLayer {  // device table entry, one per layer of the run (72 B)
  const uint16_t* w1_hi;  // x3_w1_fragments [K/16][q 4][lane 64][8]
  const uint16_t* w1_lo;
  const float* s1;  // [K] BN1 affine
  const float* t1;
  const float* b1;  // [128] BN2-folded bias
  const uint16_t* w2_hi;  // x3_w3_fragments
  const uint16_t* w2_lo;
  float* zacc;  // [>= M][128] fp32
  long long K;  // input channels of the layer
};

struct X3cParams {
  const X3cLayer* layers;  // [L - f]: entry i = layer f + i
  float* x;                // [M][ldx] the block's feature buffer (layer l's y = x + K_l)
  int ldx, M, H, W;
  int l, n;                // this layer (index into layers), layers in the run
  int nA;                  // part-A blocks (tiles x 4)
};

constexpr int kBandPitch = 144;  // B per LDS band row: 64 B hi + 64 B lo + 16 B pad (b128 reads spread over banks)
constexpr int kBandRows = 160;   // 32 + 2(W + 1) <= 160: W <= 63 (5 row tiles over 4 waves)

// acc += W1_l[32q.., 16 s.. +16] . act(x[row][16 s..]) over k16 steps [s0, s1)
__device__ __forceinline__ f32x16 chunk_1x1(const X3cLayer& L, const float* xr, bool live, int q, int lane, int h,
                                            int s0, int s1, f32x16 acc) {
  for (int s = s0; s < s1; ++s) {
    const size_t wo = ((size_t)(s * 4 + q) * 64 + lane) * 8;
    const v4u ah = ld16(L.w1_hi + wo), al = ld16(L.w1_lo + wo);
    const int k = 16 * s + 8 * h;
    const f32x4 xa = ldf4(xr + 16 * s), xb = ldf4(xr + 16 * s + 4);
    const f32x4 sa = ldf4(L.s1 + k), sb = ldf4(L.s1 + k + 4), ta = ldf4(L.t1 + k), tb = ldf4(L.t1 + k + 4);
    f32x4 va, vb;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      va[e] = live ? fmaxf(xa[e] * sa[e] + ta[e], 0.f) : 0.f;
      vb[e] = live ? fmaxf(xb[e] * sb[e] + tb[e], 0.f) : 0.f;
    }
    v4u bh, bl;
    split8(va, vb, bh, bl);
    acc = x3_32(ah, al, bh, bl, acc);
  }
  return acc;
}

// the chain's per-chunk 1x1: exactly the 2 k16 steps of one 32-channel chunk,
// every load issued before the first use (one memory round trip, not two)
__device__ __forceinline__ f32x16 chunk2_1x1(const X3cLayer& L, const float* xr, bool live, int q, int lane, int h,
                                             int s0, f32x16 acc) {
  v4u ah[2], al[2];
  f32x4 xa[2], xb[2], sa[2], sb[2], ta[2], tb[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int s = s0 + i;
    const size_t wo = ((size_t)(s * 4 + q) * 64 + lane) * 8;
    ah[i] = ld16(L.w1_hi + wo);
    al[i] = ld16(L.w1_lo + wo);
    const int k = 16 * s + 8 * h;
    xa[i] = ldf4(xr + 16 * s);
    xb[i] = ldf4(xr + 16 * s + 4);
    sa[i] = ldf4(L.s1 + k);
    sb[i] = ldf4(L.s1 + k + 4);
    ta[i] = ldf4(L.t1 + k);
    tb[i] = ldf4(L.t1 + k + 4);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    f32x4 va, vb;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      va[e] = live ? fmaxf(xa[i][e] * sa[i][e] + ta[i][e], 0.f) : 0.f;
      vb[e] = live ? fmaxf(xb[i][e] * sb[i][e] + tb[i][e], 0.f) : 0.f;
    }
    v4u bh, bl;
    split8(va, vb, bh, bl);
    acc = x3_32(ah[i], al[i], bh, bl, acc);
  }
  return acc;
}

// base: grid (tiles, n layers, 4 quarters); 4 waves split the k16 steps of
// [0, K_f), sum through LDS, plain-store zacc_l[tile][quarter]; quarter 0
// also zeroes the tile's rows of y_l
__global__ void __launch_bounds__(256) x3c_base_kernel(X3cParams p) {
  __shared__ __attribute__((aligned(16))) float red[4][kTile * kRedPitch];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = lane & 31, h = lane >> 5;
  const int m0 = blockIdx.x * kTile, q = blockIdx.z;
  const X3cLayer L = p.layers[blockIdx.y];
  const int kf = (int)p.layers[0].K;
  if (q == 0) {
    const int px = threadIdx.x >> 3;
    if (m0 + px < p.M)
      *reinterpret_cast<f32x4*>(p.x + (size_t)(m0 + px) * p.ldx + L.K + 4 * (threadIdx.x & 7)) = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int m = m0 + col;
  const bool in = m < p.M;
  const float* xr = p.x + (size_t)(in ? m : 0) * p.ldx + 8 * h;
  const int nst = kf / 16, per = (nst + 3) / 4;
  f32x16 acc;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.f;
  acc = chunk_1x1(L, xr, in, q, lane, h, wave * per, min(nst, wave * per + per), acc);
  put_tile(red[wave], acc, col, h);
  __syncthreads();
  const int oc = threadIdx.x & 31;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int px = (threadIdx.x >> 5) + 8 * j;
    const float v = red[0][px * kRedPitch + oc] + red[1][px * kRedPitch + oc] + red[2][px * kRedPitch + oc] +
                    red[3][px * kRedPitch + oc];
    if (m0 + px < p.M) L.zacc[(size_t)(m0 + px) * kZ + 32 * q + oc] = v;
  }
}

// NW waves per block (4 launched; 8 measured slower).  Part A: wave w takes taps w, w + NW, ... and
// band row tiles w, w + NW, ...; part B: each group of 4 waves (one per
// output quarter) takes one later layer, NW / 4 layers per block
template <int NW>
__global__ void __launch_bounds__(64 * NW) x3c_layer_kernel(X3cParams p) {
  constexpr int NL = NW / 4, NT = (9 + NW - 1) / NW;
  __shared__ __attribute__((aligned(16))) uint8_t band[kBandRows * kBandPitch];
  __shared__ __attribute__((aligned(16))) float red[NW][kTile * kRedPitch];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = lane & 31, h = lane >> 5;
  const X3cLayer L = p.layers[p.l];
  const int c0 = (int)L.K - 32;  // the previous layer's chunk
  if ((int)blockIdx.x >= p.nA) {
    // ---- part B: chunk l-1 into zacc of layer l + 1 + j, quarter = wave ----
    const int b = blockIdx.x - p.nA, ntl = p.n - p.l - 1, nbp = (ntl + NL - 1) / NL;
    const int m0 = (b / nbp) * kTile, j = (b % nbp) * NL + (wave >> 2), q = wave & 3;
    if (j >= ntl) return;  // wave-uniform
    const X3cLayer T = p.layers[p.l + 1 + j];
    const int m = m0 + col;
    const bool in = m < p.M;
    const float* xr = p.x + (size_t)(in ? m : 0) * p.ldx + 8 * h;
    // the accumulator rows go out with the chunk's loads (one round trip)
    f32x4* zp = reinterpret_cast<f32x4*>(T.zacc + (size_t)(in ? m : 0) * kZ + 32 * q + 4 * h);
    f32x4 zv[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) zv[g] = zp[2 * g];
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    acc = chunk2_1x1(T, xr, in, q, lane, h, c0 / 16, acc);
    if (in) {
#pragma unroll
      for (int g = 0; g < 4; ++g) zp[2 * g] = zv[g] + f32x4{acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]};
    }
    return;
  }
  // ---- part A: the 3x3 of layer l over one tile and one input quarter ----
  const int kq = blockIdx.x & 3, m0 = (blockIdx.x >> 2) * kTile;
  const int W = p.W, band0 = m0 - W - 1, R = kTile + 2 * W + 2;
  // this wave's taps: weight fragments in flight first
  v4u wh[NT][2], wl[NT][2];
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    const int t = min(wave + NW * i, 8);
#pragma unroll
    for (int kc = 0; kc < 2; ++kc) {
      const size_t wo = ((size_t)((t * 4 + kq) * 2 + kc) * 64 + lane) * 8;
      wh[i][kc] = ld16(L.w2_hi + wo);
      wl[i][kc] = ld16(L.w2_lo + wo);
    }
  }
  // band rows [band0, band0 + R): z = zacc + chunk(l-1) + bias -> ReLU -> split
  for (int rt = wave; rt * kTile < R; rt += NW) {  // wave-uniform: the 56x56 band has 5 row tiles
    const int row = band0 + rt * kTile + col;
    const bool rin = row >= 0 && row < p.M;
    const int rc = rin ? row : 0;
    // the accumulator rows and bias go out with the chunk's loads
    f32x4 zsv[4], bbv[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      zsv[g] = ldf4(L.zacc + (size_t)rc * kZ + 32 * kq + 8 * g + 4 * h);
      bbv[g] = ldf4(L.b1 + 32 * kq + 8 * g + 4 * h);
    }
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    if (p.l > 0) {
      const float* xr = p.x + (size_t)rc * p.ldx + 8 * h;
      acc = chunk2_1x1(L, xr, rin, kq, lane, h, c0 / 16, acc);
    }
    uint8_t* br = band + (rt * kTile + col) * kBandPitch;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int c = 8 * g + 4 * h;
      const f32x4 zs = zsv[g];
      const f32x4 bb = bbv[g];
      const float v0 = fmaxf(acc[4 * g] + zs[0] + bb[0], 0.f), v1 = fmaxf(acc[4 * g + 1] + zs[1] + bb[1], 0.f);
      const float v2 = fmaxf(acc[4 * g + 2] + zs[2] + bb[2], 0.f), v3 = fmaxf(acc[4 * g + 3] + zs[3] + bb[3], 0.f);
      const uint32_t h0 = pk(v0, v1), h1 = pk(v2, v3);
      const uint32_t l0 = pk(v0 - __uint_as_float(h0 << 16), v1 - __uint_as_float(h0 & 0xffff0000u));
      const uint32_t l1 = pk(v2 - __uint_as_float(h1 << 16), v3 - __uint_as_float(h1 & 0xffff0000u));
      typedef uint32_t v2u __attribute__((ext_vector_type(2)));
      *reinterpret_cast<v2u*>(br + 2 * c) = v2u{h0, h1};
      *reinterpret_cast<v2u*>(br + 64 + 2 * c) = v2u{l0, l1};
    }
  }
  __syncthreads();
  const int m = m0 + col;
  const bool in = m < p.M;
  const int HW = p.H * W;
  const int r = in ? m % HW : 0;
  const int yy = r / W, xx = r - yy * W;
  f32x16 acc;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    const int t = wave + NW * i;
    const int dy = t / 3 - 1, dx = t % 3 - 1;
    const int y2 = yy + dy, x2 = xx + dx;
    const bool ok = in && t < 9 && y2 >= 0 && y2 < p.H && x2 >= 0 && x2 < W;
    const uint8_t* br = band + (ok ? col + (dy + 1) * W + dx + 1 : 0) * kBandPitch;
#pragma unroll
    for (int kc = 0; kc < 2; ++kc) {
      v4u bh = ld16(br + (2 * kc + h) * 16), bl = ld16(br + 64 + (2 * kc + h) * 16);
      if (!ok) bh = bl = v4u{0u, 0u, 0u, 0u};
      acc = x3_32(wh[i][kc], wl[i][kc], bh, bl, acc);
    }
  }
  put_tile(red[wave], acc, col, h);
  __syncthreads();
  const int oc = threadIdx.x & 31;
  float* y = p.x + L.K;
#pragma unroll
  for (int j = 0; j < 16 / NW; ++j) {
    const int px = (threadIdx.x >> 5) + 2 * NW * j;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += red[w][px * kRedPitch + oc];
    if (m0 + px < p.M) atomicAdd(y + (size_t)(m0 + px) * p.ldx + oc, v);
  }
}

bool a16(const void* q) { return ((uintptr_t)q & 15) == 0; }

}  // namespace

extern "C" {

// K chunking of the small-M 1x1: k16 steps per block (blockIdx.z chunks).
// Up to TCAMD_X3S_MAX_CHUNKS (default 8) chunks, aiming for about
// TCAMD_X3S_BLOCKS workgroups (default 384) with a step per wave.  Float
// atomics sum in arrival order, so results can differ in the last bits from
// run to run; with at most 2 chunks and TCAMD_X3S_SPLIT3=0 the layer is
// bitwise reproducible (two adds onto a zero are order-free).
int tcamd_x3s_steps_per_block(int M, int K) {
  const int target = std::max(1, (int)tcamd::knob(tcamd::Knob::X3sBlocks));
  const int max_chunks = std::max(1, (int)tcamd::knob(tcamd::Knob::X3sMaxChunks));
  const int tiles = (M + kTile - 1) / kTile * 4;
  const int nst = K / 16;
  const int chunks = std::max(1, std::min(std::min(target / std::max(tiles, 1), nst / 4), max_chunks));
  return (nst + chunks - 1) / chunks;
}

// One small-M dense layer: BN1+ReLU+1x1 (K -> 128, w1 in x3_w1_fragments,
// BN2 folded, bias b1) summed into zacc (ZERO on entry, [M][128] fp32), then
// the 3x3 (128 -> 32, w2 in x3_w3_fragments) into y rows of ldy.  zacc_next
// (may be null): rows [0, M) are zeroed for the next layer.
int tcamd_x3s_dense_layer(const float* x, int ldx, int imgs, int H, int W, int K, const float* s1, const float* t1,
                          const void* w1_hi, const void* w1_lo, const float* b1, float* zacc, float* zacc_next,
                          const void* w2_hi, const void* w2_lo, float* y, int ldy, void* stream) {
  if (imgs <= 0) return hipSuccess;
  if (H < 1 || W < 1 || K <= 0 || K % 16 || ldx < K || ldx % 4 || ldy % 4 || ldy < 32) return hipErrorInvalidValue;
  if (!x || !s1 || !t1 || !w1_hi || !w1_lo || !b1 || !zacc || !w2_hi || !w2_lo || !y) return hipErrorInvalidValue;
  for (const void* q : {(const void*)x, (const void*)s1, (const void*)t1, w1_hi, w1_lo, (const void*)b1,
                        (const void*)zacc, w2_hi, w2_lo, (const void*)y})
    if (!a16(q)) return hipErrorInvalidValue;
  if (zacc_next && (!a16(zacc_next) || zacc_next == zacc)) return hipErrorInvalidValue;
  const long long Ml = (long long)imgs * H * W;
  if (Ml >= (1 << 24)) return hipErrorInvalidValue;
  const int M = (int)Ml;
  hipStream_t s = (hipStream_t)stream;
  const int tiles = (M + kTile - 1) / kTile;

  X3sConv1x1Params a;
  a.x = x;
  a.s1 = s1;
  a.t1 = t1;
  a.w1_hi = (const uint16_t*)w1_hi;
  a.w1_lo = (const uint16_t*)w1_lo;
  a.zacc = zacc;
  a.ldx = ldx;
  a.M = M;
  a.K = K;
  a.steps_per_block = tcamd_x3s_steps_per_block(M, K);
  // the 3x3 spreads over the 4 input quarters (grid.y = 4): a quarter of the
  // weight bytes per block, y accumulated by float atomics (zeroed by S1).
  // bs1 forward 0.862 -> 0.682 ms (profiles/r3_x3s_small_m.md);
  // TCAMD_X3S_SPLIT3=0: all quarters in one block, y stored (bitwise reproducible)
  const bool split3 = tcamd::knob(tcamd::Knob::X3sSplit3) != 0;
  a.y_zero = split3 ? y : nullptr;
  a.ldy = ldy;
  const int chunks = (K / 16 + a.steps_per_block - 1) / a.steps_per_block;
  hipLaunchKernelGGL(x3s_conv1x1_kernel, dim3(tiles, 4, chunks), dim3(256), 0, s, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;

  X3sConv3x3Params c;
  c.zacc = zacc;
  c.b1 = b1;
  c.w_hi = (const uint16_t*)w2_hi;
  c.w_lo = (const uint16_t*)w2_lo;
  c.y = y;
  c.zero_next = zacc_next;
  c.ldy = ldy;
  c.M = M;
  c.H = H;
  c.W = W;
  c.zero_rows = M;
  if (split3) hipLaunchKernelGGL((x3s_conv3x3_kernel<1, 4>), dim3(tiles, 4), dim3(256), 0, s, c);
  else hipLaunchKernelGGL((x3s_conv3x3_kernel<4, 2>), dim3(tiles), dim3(512), 0, s, c);
  return hipGetLastError();
}

// K13x chain over the small-M layers f..f+n-1 of one dense block (W <= 63):
// `layers` is a device table of n X3cLayer entries (layer f first; every
// zacc has >= M rows); x the block's feature buffer [M][ldx] (layer l's y =
// x + K_l).  Call tcamd_x3c_base once, then tcamd_x3c_layer for l = 0..n-1 in
// order on the same stream.
static int x3c_check(const void* layers, const float* x, int ldx, int imgs, int H, int W, int l, int n, X3cParams& p) {
  if (!layers || !x || !a16(layers) || !a16(x) || ldx % 4 || n < 1 || l < 0 || l >= n) return hipErrorInvalidValue;
  if (H < 1 || W < 1 || W > (kBandRows - kTile - 2) / 2) return hipErrorInvalidValue;
  const long long Ml = (long long)imgs * H * W;
  if (Ml >= (1 << 24)) return hipErrorInvalidValue;
  p.layers = (const X3cLayer*)layers;
  p.x = (float*)x;
  p.ldx = ldx;
  p.M = (int)Ml;
  p.H = H;
  p.W = W;
  p.l = l;
  p.n = n;
  p.nA = (p.M + kTile - 1) / kTile * 4;
  return hipSuccess;
}

int tcamd_x3c_base(const void* layers, int n, float* x, int ldx, int imgs, int H, int W, void* stream) {
  if (imgs <= 0) return hipSuccess;
  X3cParams p;
  int e = x3c_check(layers, x, ldx, imgs, H, W, 0, n, p);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(x3c_base_kernel, dim3((p.M + kTile - 1) / kTile, n, 4), dim3(256), 0, (hipStream_t)stream, p);
  return hipGetLastError();
}

int tcamd_x3c_layer(const void* layers, int l, int n, float* x, int ldx, int imgs, int H, int W, void* stream) {
  if (imgs <= 0) return hipSuccess;
  X3cParams p;
  int e = x3c_check(layers, x, ldx, imgs, H, W, l, n, p);
  if (e != hipSuccess) return e;
  // 4 waves per block, one later layer per part-B block (8 waves, taps and
  // band tiles over 8 and two later layers per block, measured slower in
  // round 3: bs1 0.430 -> 0.455 ms; removed in round 5)
  const int nB = l > 0 ? (p.M + kTile - 1) / kTile * (n - l - 1) : 0;
  hipLaunchKernelGGL(x3c_layer_kernel<4>, dim3(p.nA + nB), dim3(256), 0, (hipStream_t)stream, p);
  return hipGetLastError();
}

}  // extern "C"
