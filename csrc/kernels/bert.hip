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

#include <algorithm>
#include <atomic>
#include <type_traits>

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

// LayerNorm of one row held as v[E] per lane (lane l owns the 16-B chunks
// l, l + 64, ...) -> bf16 out row: exact two-pass mean / variance over the
// register copy, wave butterflies through DPP-backed shuffles
template <int E>
__device__ __forceinline__ void ln_store_row(const float (&v)[E], const uint16_t* __restrict__ gamma,
                                             const uint16_t* __restrict__ beta, uint16_t* orow, int lane, float eps) {
  constexpr int H = 64 * E, C = E / 8;
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
    *reinterpret_cast<v4u*>(orow + off) = o;
  }
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
  ln_store_row<E>(v, gamma, beta, out + base, lane, eps);
}

// ---- K11p: LN(x + bias + sum_z parts[z]) -----------------------------------
// The consumer of a split-K projection (K18, csrc/kernels/gemm_tiles.hip):
// the attention-out / FFN-down GEMM leaves fp32 partial slabs instead of a
// bf16 y, and this pass -- which BERT needs anyway for the residual add +
// LayerNorm -- sums them with the bias on the way in, so the split costs no
// reduce launch and y never exists as its own tensor.  T = uint16_t (bf16
// x / gamma / beta / out: the bf16 model) or float (the fp32-parity model).
__device__ __forceinline__ void load8(const uint16_t* p, float* v) {
  const v4u a = *reinterpret_cast<const v4u*>(p);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    v[2 * q] = __uint_as_float(a[q] << 16);
    v[2 * q + 1] = __uint_as_float(a[q] & 0xffff0000u);
  }
}
__device__ __forceinline__ void load8(const float* p, float* v) {
  const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
  v[0] = a.x, v[1] = a.y, v[2] = a.z, v[3] = a.w, v[4] = b.x, v[5] = b.y, v[6] = b.z, v[7] = b.w;
}
__device__ __forceinline__ void add8(const float* p, float* v) {
  const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
  v[0] += a.x, v[1] += a.y, v[2] += a.z, v[3] += a.w, v[4] += b.x, v[5] += b.y, v[6] += b.z, v[7] += b.w;
}
__device__ __forceinline__ void store8(uint16_t* p, const float* v) {
  *reinterpret_cast<v4u*>(p) = v4u{pack2(v[0], v[1]), pack2(v[2], v[3]), pack2(v[4], v[5]), pack2(v[6], v[7])};
}
__device__ __forceinline__ void store8(float* p, const float* v) {
  reinterpret_cast<float4*>(p)[0] = make_float4(v[0], v[1], v[2], v[3]);
  reinterpret_cast<float4*>(p)[1] = make_float4(v[4], v[5], v[6], v[7]);
}

// out3 (fp32 model, or null): the row also as the next bf16x3 GEMM's operand,
// bf16 [rows][3H] = [hi | hi | lo] (x3_cat's layout), so that GEMM needs no
// x3_cat pass over the LayerNorm output.
template <int E, typename T>
__global__ void __launch_bounds__(256) add_ln_parts_kernel(const T* x, const float* parts, int nparts, long long pstride,
                                                           const float* __restrict__ bias, const T* __restrict__ gamma,
                                                           const T* __restrict__ beta, T* out, uint16_t* __restrict__ out3,
                                                           int rows, float eps) {
  constexpr int H = 64 * E, C = E / 8;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const size_t base = (size_t)row * H;
  float v[E];
#pragma unroll
  for (int c = 0; c < C; ++c) load8(x + base + (c * 64 + lane) * 8, v + 8 * c);
  if (bias)
#pragma unroll
    for (int c = 0; c < C; ++c) add8(bias + (c * 64 + lane) * 8, v + 8 * c);
  for (int zz = 0; zz < nparts; ++zz) {
    const float* pz = parts + zz * pstride + base;
#pragma unroll
    for (int c = 0; c < C; ++c) add8(pz + (c * 64 + lane) * 8, v + 8 * c);
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
    float g[8], bt[8], o[8];
    load8(gamma + off, g);
    load8(beta + off, bt);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (v[8 * c + e] - mean) * rstd * g[e] + bt[e];
    store8(out + base + off, o);
    if (out3) {
      v4u hi, lo;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        hi[q] = pack2(o[2 * q], o[2 * q + 1]);
        lo[q] = pack2(o[2 * q] - __uint_as_float(hi[q] << 16), o[2 * q + 1] - __uint_as_float(hi[q] & 0xffff0000u));
      }
      uint16_t* r3 = out3 + 3 * base + off;
      *reinterpret_cast<v4u*>(r3) = hi;
      *reinterpret_cast<v4u*>(r3 + H) = hi;
      *reinterpret_cast<v4u*>(r3 + 2 * H) = lo;
    }
  }
}

// ---- QA head: (start, end)[r] = x[r] . w[0 / 1] + b[0 / 1] -----------------
// BERT's span head is a [2 x H] Linear over every token: as a library GEMM an
// N = 2 launch plus a cast and two strided copies.  One wave per row: each
// lane dots its 8-element chunks with both weight rows, a butterfly sums the
// wave, lane 0 writes the two fp32 logits into their separate [rows] planes.
template <int E, typename T>
__global__ void __launch_bounds__(256) qa_head_kernel(const T* __restrict__ x, const T* __restrict__ w,
                                                      const float* __restrict__ b, float* __restrict__ start,
                                                      float* __restrict__ end, int rows) {
  constexpr int H = 64 * E, C = E / 8;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float s0 = 0.f, s1 = 0.f;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int off = (c * 64 + lane) * 8;
    float xv[8], w0[8], w1[8];
    load8(x + (size_t)row * H + off, xv);
    load8(w + off, w0);
    load8(w + H + off, w1);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      s0 += xv[e] * w0[e];
      s1 += xv[e] * w1[e];
    }
  }
  s0 = wave_sum(s0);
  s1 = wave_sum(s1);
  if (lane == 0) {
    start[row] = s0 + b[0];
    end[row] = s1 + b[1];
  }
}

// Embedding sum + LayerNorm: out[r] = LN(word[ids[r]] + pos[r % S] +
// type[types[r]]) in one pass (torch: three gathers, two adds and a LayerNorm,
// six launches and ~5 passes over [tokens, H]).  Ids outside the tables are
// clamped (torch would raise).
template <int E>
__global__ void __launch_bounds__(256) embed_layernorm_kernel(const int64_t* __restrict__ ids,
                                                              const int64_t* __restrict__ types,
                                                              const uint16_t* __restrict__ word,
                                                              const uint16_t* __restrict__ pos,
                                                              const uint16_t* __restrict__ tok,
                                                              const uint16_t* __restrict__ gamma,
                                                              const uint16_t* __restrict__ beta, uint16_t* __restrict__ out,
                                                              int rows, int S, int vocab, int ntypes, float eps) {
  constexpr int H = 64 * E, C = E / 8;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const long long id = min(max(ids[row], (int64_t)0), (int64_t)vocab - 1);
  const long long ty = min(max(types[row], (int64_t)0), (int64_t)ntypes - 1);
  const uint16_t* rw = word + (size_t)id * H;
  const uint16_t* rp = pos + (size_t)(row % S) * H;
  const uint16_t* rt = tok + (size_t)ty * H;
  float v[E];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int off = (c * 64 + lane) * 8;
    const v4u a = *reinterpret_cast<const v4u*>(rw + off);
    const v4u b = *reinterpret_cast<const v4u*>(rp + off);
    const v4u t = *reinterpret_cast<const v4u*>(rt + off);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[c * 8 + 2 * q] = __uint_as_float(a[q] << 16) + __uint_as_float(b[q] << 16) + __uint_as_float(t[q] << 16);
      v[c * 8 + 2 * q + 1] = __uint_as_float(a[q] & 0xffff0000u) + __uint_as_float(b[q] & 0xffff0000u) +
                             __uint_as_float(t[q] & 0xffff0000u);
    }
  }
  ln_store_row<E>(v, gamma, beta, out + (size_t)row * H, lane, eps);
}

}  // namespace


namespace {
// ============================================================================
// K12 — fused multi-head attention for bert_large (non-causal, head dim 64,
// additive key-padding mask), straight from the fused QKV GEMM's output.
// ============================================================================
// torch-ROCm's SDPA with a key-padding bias costs 216 us per layer at bs64 x
// seq384 (120 us unmasked) plus a transpose copy of its output; here one block
// owns one (sequence, head):
//   * K [S][64] and V^T [64][S] (bf16) of the head go to LDS once (96 KB at
//     S = 384): K rows 128 B with 16-B chunks XOR-swizzled by (row >> 1) & 7
//     (conflict-free b128 reads by 16 consecutive keys), V transposed while it
//     is staged (pairs of keys -> 32-bit writes), rows padded to S + 4 so the
//     dim-major b64 reads of 32 lanes hit 32 distinct bank pairs;
//   * wave w owns queries [32w, 32w + 32) (S/32 waves, 3 per SIMD at S = 384):
//     its Q^T fragments stay in registers; per 64-key chunk S^T = K Q^T on
//     v_mfma_f32_32x32x16_bf16 (8 MFMAs), an online softmax in the exp2
//     domain (per-lane partial row sums, one cross-half max shuffle per
//     chunk), then O^T += V^T P^T (8 MFMAs) with P^T taken straight from the
//     S^T accumulators: the MFMA k index is permuted so a lane's 8 keys are
//     exactly the 8 scores it already holds, and V^T is read in that order;
//   * exponentials are raw v_exp_f32 (flushed denormals are exactly what a
//     softmax wants; exp2f adds a range fix-up of ~4 VALU per score);
//   * O / l leaves as bf16 in [tokens][heads * 64] — the layout the output
//     projection GEMM reads, so no transpose kernel follows.
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));
typedef short v4s __attribute__((ext_vector_type(4)));

constexpr int kAD = 64;           // head dim
constexpr int kAMaxS = 384;       // keys / queries per sequence (multiple of 64)

__device__ __forceinline__ bf16x8 as_bf8(v4u v) { return __builtin_bit_cast(bf16x8, v); }

// qkv_bias (may be null): the QKV projection's bias [3 * heads * 64], applied
// here so the projection runs as a plain GEMM (hipBLASLt's bias epilogue cost
// ~20 us per layer at bs64 x 384): q + b_q feeds the scores; the key bias
// adds (q + b_q) . b_k to every score of a query, a constant that softmax
// removes, so it is dropped; the value bias passes through the normalised
// weights unchanged and is added to the output.
template <bool MASKED>
__global__ void __launch_bounds__(768, 1) attention_kernel(const uint16_t* __restrict__ qkv, const int* __restrict__ mask,
                                                           uint16_t* __restrict__ out, int S, int heads, float scale,
                                                           const uint16_t* __restrict__ qkv_bias) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_a[];
  uint16_t* Ks = reinterpret_cast<uint16_t*>(lds_a);
  uint16_t* Vs = Ks + S * kAD;
  float* kb = reinterpret_cast<float*>(Vs + S * kAD);  // per-key log2-domain bias
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nthr = blockDim.x;
  const int seq = blockIdx.x / heads, head = blockIdx.x % heads;
  const int HD = heads * kAD, ld = 3 * HD;
  const uint16_t* base = qkv + (size_t)seq * S * ld + head * kAD;
  constexpr float kLog2e = 1.4426950408889634f;

  // ---- stage K and V rows (128 B each) by LDS-DMA (round 6) ----
  // Both row-major, 16-B chunks XOR-swizzled on the SOURCE address (the DMA
  // writes lane-linear: one wave instruction = 8 rows), every instruction of
  // the block in flight at once and one wait.  K chunk c of key k sits at
  // c ^ ((k >> 1) & 7) (conflict-free b128 reads by 16 consecutive keys);
  // V chunk c at c ^ (((k >> 1) & 1) << 2), which makes the transposing
  // ds_read_b64_tr_b16 reads of the PV operand conflict-free.  (Round 5
  // staged with per-thread 16-B loads and transposed V by 4-byte LDS writes:
  // ~25 of 83 us at bs64 and half of bs1's 11 us went to that staging,
  // profiles/r6_k12/.)
  {
    const int nw = nthr >> 6, nrb = S >> 3;  // waves, 8-row blocks per operand
    const int r8 = lane >> 3, cs = lane & 7;
    for (int j = wave; j < 2 * nrb; j += nw) {
      const bool isv = j >= nrb;
      const int row = 8 * (isv ? j - nrb : j) + r8;
      const int c = isv ? cs ^ (((row >> 1) & 1) << 2) : cs ^ ((row >> 1) & 7);
      const uint16_t* src = base + (size_t)row * ld + (isv ? 2 * HD : HD) + 8 * c;
      uint8_t* dst = lds_a + (isv ? S * 128 : 0) + (j - (isv ? nrb : 0)) * 1024;
      __builtin_amdgcn_global_load_lds((const void*)src, (void*)dst, 16, 0, 0);
    }
  }
  if (MASKED)
    for (int k = tid; k < S; k += nthr) kb[k] = mask[(size_t)seq * S + k] == 0 ? -10000.0f * kLog2e : 0.0f;

  // ---- this wave's queries: Q^T fragments (B operand: lane col = query) ----
  const int col = lane & 31, h = lane >> 5;
  const int q = 32 * (blockIdx.y * (nthr >> 6) + wave) + col;
  v4u qf[4];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) qf[kk] = *reinterpret_cast<const v4u*>(base + (size_t)q * ld + 16 * kk + 8 * h);
  if (qkv_bias) {
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const v4u bq = *reinterpret_cast<const v4u*>(qkv_bias + head * kAD + 16 * kk + 8 * h);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float a0 = __uint_as_float(qf[kk][j] << 16) + __uint_as_float(bq[j] << 16);
        const float a1 = __uint_as_float(qf[kk][j] & 0xffff0000u) + __uint_as_float(bq[j] & 0xffff0000u);
        qf[kk][j] = pack2(a0, a1);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's K / V DMAs landed
  __syncthreads();                                   // ... and every other wave's

  const float sl2 = scale * kLog2e;
  float m_run = -1.0e30f, l_part = 0.f;
  f32x16 o[2];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int e = 0; e < 16; ++e) o[r][e] = 0.f;

  // Chunk classes (round 6).  A key-padding mask is a run of valid keys, so
  // most 64-key chunks are all valid or all padded: an all-valid chunk takes
  // the unmasked math (no bias add, one FMA per score into the exponent), an
  // all-padded chunk is skipped -- exactly: behind any valid key its scores
  // are exp2(<= -14000) = 0 in fp32, and if it comes first the first valid
  // chunk's rescale zeroes it.  Only a sequence with no valid key at all runs
  // every chunk masked (softmax over the padded scores, as torch does).
  const int nch = S / 64;
  uint32_t todo = (1u << nch) - 1u, full = todo;
  if constexpr (MASKED) {
    full = 0u;
    uint32_t empty = 0u;
    for (int c = 0; c < nch; ++c) {
      const uint64_t v = __ballot(kb[64 * c + lane] == 0.0f);
      if (v == ~0ull) full |= 1u << c;
      if (v == 0ull) empty |= 1u << c;
    }
    if (empty != todo) todo &= ~empty;
  }

  // transposed V reads: lane 4 q4 + p4 of 16-lane group g supplies row (key)
  // 4 h + q4 of the 16-key step, dims 32 rd + 16 (g & 1) + 4 p4 .. + 3 (8 B of
  // chunk 4 rd + 2 (g & 1) + p4 / 2, swizzled by its key -- bit 1 of the key
  // is bit 1 of q4, the other terms are multiples of 4)
  const int q4 = (lane >> 2) & 3, p4 = lane & 3, g1 = (lane >> 4) & 1;
  const int vch = 2 * g1 + (p4 >> 1);
  const uint8_t* vbase = lds_a + S * 128 + (4 * h + q4) * 128 + ((vch ^ (((q4 >> 1) & 1) << 2)) << 4) + 8 * (p4 & 1);
  const int vrd = ((4 ^ (((q4 >> 1) & 1) << 2)) - (((q4 >> 1) & 1) << 2)) << 4;  // rd = 1: chunk + 4, swizzled
  // S^T for keys [c0, c0 + 64): two 32-key row blocks; lane (query, h) holds
  // keys 32 rb + 8 g + 4 h + e
  auto qk = [&](f32x16 (&st)[2], int c0) {
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
#pragma unroll
      for (int e = 0; e < 16; ++e) st[rb][e] = 0.f;
      const int key = c0 + 32 * rb + col;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const v4u kf = *reinterpret_cast<const v4u*>(Ks + key * kAD + 8 * ((2 * kk + h) ^ ((key >> 1) & 7)));
        st[rb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf8(kf), as_bf8(qf[kk]), st[rb], 0, 0, 0);
      }
    }
  };
  // online softmax of one chunk's scores and O^T += V^T P^T.  masked: x = s
  // scale log2e + bias, max and exp2(x - m) on x; unmasked (or an all-valid
  // chunk): max on the raw scores (scale > 0 commutes with max) and p =
  // exp2(s c - m c) as one FMA per score
  auto soft_pv = [&](f32x16 (&st)[2], int c0, auto bias_tag) {
    constexpr bool bias_chunk = decltype(bias_tag)::value;
    float mx = -1.0e30f;
    if constexpr (bias_chunk) {
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 bb = *reinterpret_cast<const f32x4*>(kb + c0 + 32 * rb + 8 * g + 4 * h);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float x = st[rb][4 * g + e] * sl2 + bb[e];
            st[rb][4 * g + e] = x;
            mx = fmaxf(mx, x);
          }
        }
    } else {
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int e = 0; e < 16; ++e) mx = fmaxf(mx, st[rb][e]);
      mx *= sl2;
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m_run, mx);
    const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
    m_run = m_new;
    f32x2 ls2 = f32x2{0.f, 0.f};
    v4u pf[4];  // P^T fragments per 16-key step: keys 16 kk2 + {4h..4h+3, 8+4h..8+4h+3}
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float pv[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          pv[e] = bias_chunk ? __builtin_amdgcn_exp2f(st[rb][4 * g + e] - m_new)
                             : __builtin_amdgcn_exp2f(__builtin_fmaf(st[rb][4 * g + e], sl2, -m_new));
        ls2 += f32x2{pv[0], pv[1]} + f32x2{pv[2], pv[3]};
        const int kk2 = 2 * rb + (g >> 1), half = g & 1;
        pf[kk2][2 * half] = pack2(pv[0], pv[1]);
        pf[kk2][2 * half + 1] = pack2(pv[2], pv[3]);
      }
    const float ls = ls2[0] + ls2[1];
    l_part = l_part * alpha + ls;
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int e = 0; e < 16; ++e) o[r][e] *= alpha;
    // O^T += V^T P^T: A = V^T rows (dims 32 rd + col), keys in the permuted
    // order, read TRANSPOSED from the row-major V image: ds_read_b64_tr_b16
    // gives lane i of a 16-lane group column i (= its dim) of 4 key rows
#pragma unroll
    for (int kk2 = 0; kk2 < 4; ++kk2)
#pragma unroll
      for (int rd = 0; rd < 2; ++rd) {
        const uint8_t* vr = vbase + (c0 + 16 * kk2) * 128 + rd * vrd;
        const v2u a0 = __builtin_bit_cast(v2u, __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                                                   (__attribute__((address_space(3))) v4s*)(vr)));
        const v2u a1 = __builtin_bit_cast(v2u, __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                                                   (__attribute__((address_space(3))) v4s*)(vr + 8 * 128)));
        const v4u af = v4u{a0[0], a0[1], a1[0], a1[1]};
        o[rd] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf8(af), as_bf8(pf[kk2]), o[rd], 0, 0, 0);
      }
  };
  // all-valid chunks first (unmasked math), then the partial ones (masked
  // math): the online softmax does not depend on the chunk order, and each
  // loop keeps one compile-time path (a per-chunk branch inside the softmax
  // cost registers and 10 % on the masked kernel, profiles/r6_k12.md)
  f32x16 st[2];
  for (uint32_t f = todo & full; f; f &= f - 1u) {
    const int c0 = 64 * __builtin_ctz(f);
    qk(st, c0);
    soft_pv(st, c0, std::false_type{});
  }
  if constexpr (MASKED)
    for (uint32_t m = todo & ~full; m; m &= m - 1u) {
      const int c0 = 64 * __builtin_ctz(m);
      qk(st, c0);
      soft_pv(st, c0, std::true_type{});
    }
  const float inv = 1.0f / (l_part + __shfl_xor(l_part, 32, 64));
  uint16_t* orow = out + ((size_t)seq * S + q) * HD + head * kAD;
#pragma unroll
  for (int rd = 0; rd < 2; ++rd)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = 32 * rd + 8 * g + 4 * h;
      float bv[4] = {0.f, 0.f, 0.f, 0.f};
      if (qkv_bias) {
        const v2u b2 = *reinterpret_cast<const v2u*>(qkv_bias + 2 * HD + head * kAD + d);
        bv[0] = __uint_as_float(b2[0] << 16);
        bv[1] = __uint_as_float(b2[0] & 0xffff0000u);
        bv[2] = __uint_as_float(b2[1] << 16);
        bv[3] = __uint_as_float(b2[1] & 0xffff0000u);
      }
      *reinterpret_cast<v2u*>(orow + d) = v2u{pack2(o[rd][4 * g] * inv + bv[0], o[rd][4 * g + 1] * inv + bv[1]),
                                             pack2(o[rd][4 * g + 2] * inv + bv[2], o[rd][4 * g + 3] * inv + bv[3])};
    }
}

// bf16x3 operand of the fp32-parity bert mode: x fp32 [rows][K] -> out bf16
// [rows][3K] = [hi | hi | lo] (hi = bf16_rne(x), lo = bf16_rne(x - hi)), so
// ONE bf16 GEMM against W' = [W_hi | W_lo | W_hi] (K' = 3K) accumulates
// x_hi W_hi + x_hi W_lo + x_lo W_hi in fp32: ~1e-5 of an fp32 GEMM at 3x the
// bf16 MFMA work (gfx950 has no xf32, and its f32-input MFMA runs at 1/16 of
// the bf16 rate).  One thread per 4 elements: a 16-B load, three 8-B stores.
__global__ void __launch_bounds__(256) x3_cat_kernel(const float* __restrict__ x, uint16_t* __restrict__ out,
                                                     long n4, int k4) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    const long r = i / k4, c = i - r * k4;
    const float4 v = reinterpret_cast<const float4*>(x)[i];
    const uint32_t h0 = pack2(v.x, v.y), h1 = pack2(v.z, v.w);
    const uint32_t l0 = pack2(v.x - __uint_as_float(h0 << 16), v.y - __uint_as_float(h0 & 0xffff0000u));
    const uint32_t l1 = pack2(v.z - __uint_as_float(h1 << 16), v.w - __uint_as_float(h1 & 0xffff0000u));
    uint2* row = reinterpret_cast<uint2*>(out) + r * 3 * k4;  // 3 segments of k4 x 8 B
    row[c] = make_uint2(h0, h1);
    row[k4 + c] = make_uint2(h0, h1);
    row[2 * k4 + c] = make_uint2(l0, l1);
  }
}


// ---- K12x: fp32-parity attention (bf16x3 products, fp32 softmax) -----------
// The fp32-parity bert's attention (it ran torch SDPA in fp32, 25 % of that
// forward).  Block = (sequence, head, 16 NW queries), NW waves x 16 queries; keys
// in 64-key chunks staged into LDS split hi / lo (K row-major, V transposed);
// every product is bf16x3 (hi*hi + hi*lo + lo*hi, fp32 accumulate), the
// online softmax is fp32 with exp; masked keys get the reference's additive
// -10000 (so a fully masked row averages like torch's).
//   S^T = K Q^T on 16x16x32 MFMAs: lane (l & 15) = query, reg e -> key 4g + e
//   (g = l >> 4), so the softmax state of a query is lane-local after two
//   xor-shuffles over the lane groups, and the same registers are the B
//   operand of O^T = V^T P^T: k position 8g + i <-> key 4g + i of the chunk's
//   16-key tile 2ks (i < 4) or 2ks + 1 (i >= 4), read from V^T in LDS as two
//   8-B runs.  O^T's C layout: lane = query, reg e -> head dim 16 dt + 4g + e.
constexpr int kXR = 64 * 2 + 16;  // LDS row: 64 bf16 + 16 B (16 rows' b128 reads spread over all banks)
constexpr int kBufAX = 4 * 64 * kXR + 64 * 4;  // one chunk: K hi | K lo | V^T hi | V^T lo | key bias
constexpr int kLdsAX = 2 * kBufAX;             // double-buffered: chunk c + 1 is staged during chunk c

__device__ __forceinline__ void split_pk(float a, float b, uint32_t& hi, uint32_t& lo) {
  hi = pack2(a, b);
  lo = pack2(a - __uint_as_float(hi << 16), b - __uint_as_float(hi & 0xffff0000u));
}

__device__ __forceinline__ f32x4 mma_x3(v4u ah, v4u al, v4u bh, v4u bl, f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf8(al), as_bf8(bh), c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf8(ah), as_bf8(bl), c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf8(ah), as_bf8(bh), c, 0, 0, 0);
}

// out3 (or null): write the output as the out-projection's bf16x3 operand,
// bf16 [tokens][3H] = [hi | hi | lo], instead of fp32 into out
template <int NW>
__global__ void __launch_bounds__(64 * NW) attention_x3_kernel(const float* __restrict__ qkv,
                                                               const int* __restrict__ mask, float* __restrict__ out,
                                                               uint16_t* __restrict__ out3, int S, int heads,
                                                               float scale) {
  extern __shared__ __attribute__((aligned(16))) uint8_t ldsa[];
  // per buffer: K hi [64 keys][kXR] | K lo | V^T hi [64 d][kXR] | V^T lo | key bias [64]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int seq = blockIdx.x / heads, h = blockIdx.x - seq * heads;
  const int H = heads * 64, ld = 3 * H;
  const float* const base = qkv + (size_t)seq * S * ld + h * 64;
  const int g = lane >> 4, c = lane & 15;
  const int q = blockIdx.y * (16 * NW) + wave * 16 + c;  // this lane's query

  // Q^T operand, pre-scaled (1/8: exact), d = 32 ks + 8 g .. +8
  v4u qh[2], ql[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const float4 a = *reinterpret_cast<const float4*>(base + (size_t)q * ld + 32 * ks + 8 * g);
    const float4 b = *reinterpret_cast<const float4*>(base + (size_t)q * ld + 32 * ks + 8 * g + 4);
    uint32_t hh[4], ll[4];
    split_pk(a.x * scale, a.y * scale, hh[0], ll[0]);
    split_pk(a.z * scale, a.w * scale, hh[1], ll[1]);
    split_pk(b.x * scale, b.y * scale, hh[2], ll[2]);
    split_pk(b.z * scale, b.w * scale, hh[3], ll[3]);
    qh[ks] = v4u{hh[0], hh[1], hh[2], hh[3]};
    ql[ks] = v4u{ll[0], ll[1], ll[2], ll[3]};
  }
  f32x4 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;

  // staging of one 64-key chunk, split so that its global loads are in
  // flight during the previous chunk's math: K row-major (thread -> key, 4
  // head dims), V transposed (thread -> key pair, 4 head dims: 4-B words of
  // two keys, a wave's 32 key pairs one contiguous 128-B run per V^T row)
  constexpr int KIT = 1024 / (64 * NW), VIT = 512 / (64 * NW);
  float4 kr[KIT], va[VIT], vb[VIT];
  float mkb = 0.f;
  auto stage_load = [&](int c0) {
#pragma unroll
    for (int it = 0; it < KIT; ++it) {
      const int i = it * 64 * NW + tid, key = i >> 4, d4 = (i & 15) * 4;
      kr[it] = *reinterpret_cast<const float4*>(base + (size_t)(c0 + key) * ld + H + d4);
    }
#pragma unroll
    for (int it = 0; it < VIT; ++it) {
      const int u = it * 64 * NW + tid, kp = u & 31, d4 = (u >> 5) * 4;
      const float* r0 = base + (size_t)(c0 + 2 * kp) * ld + 2 * H + d4;
      va[it] = *reinterpret_cast<const float4*>(r0);
      vb[it] = *reinterpret_cast<const float4*>(r0 + ld);
    }
    if (tid < 64) mkb = (mask && mask[seq * S + c0 + tid] == 0) ? -10000.f : 0.f;
  };
  auto stage_store = [&](uint8_t* buf) {
#pragma unroll
    for (int it = 0; it < KIT; ++it) {
      const int i = it * 64 * NW + tid, key = i >> 4, d4 = (i & 15) * 4;
      uint32_t h0, l0, h1, l1;
      split_pk(kr[it].x, kr[it].y, h0, l0);
      split_pk(kr[it].z, kr[it].w, h1, l1);
      *reinterpret_cast<uint2*>(buf + key * kXR + d4 * 2) = make_uint2(h0, h1);
      *reinterpret_cast<uint2*>(buf + 64 * kXR + key * kXR + d4 * 2) = make_uint2(l0, l1);
    }
#pragma unroll
    for (int it = 0; it < VIT; ++it) {
      const int u = it * 64 * NW + tid, kp = u & 31, d4 = (u >> 5) * 4;
      const float a[4] = {va[it].x, va[it].y, va[it].z, va[it].w}, b[4] = {vb[it].x, vb[it].y, vb[it].z, vb[it].w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint32_t hh, ll;
        split_pk(a[j], b[j], hh, ll);
        *reinterpret_cast<uint32_t*>(buf + 128 * kXR + (d4 + j) * kXR + 4 * kp) = hh;
        *reinterpret_cast<uint32_t*>(buf + 192 * kXR + (d4 + j) * kXR + 4 * kp) = ll;
      }
    }
    if (tid < 64) reinterpret_cast<float*>(buf + 256 * kXR)[tid] = mkb;
  };
  stage_load(0);
  stage_store(ldsa);
  __syncthreads();
  const int nch = S / 64;
  for (int ci = 0; ci < nch; ++ci) {
    uint8_t* const kh = ldsa + (ci & 1) * kBufAX;
    uint8_t* const kl = kh + 64 * kXR;
    uint8_t* const vth = kh + 128 * kXR;
    uint8_t* const vtl = kh + 192 * kXR;
    const float* const kb = reinterpret_cast<const float*>(kh + 256 * kXR);
    if (ci + 1 < nch) stage_load(64 * (ci + 1));

    // S^T tiles [16 keys][16 queries]
    f32x4 st[4];
    float mx = m;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      st[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const uint8_t* ar = kh + (kt * 16 + c) * kXR + (32 * ks + 8 * g) * 2;
        st[kt] = mma_x3(*reinterpret_cast<const v4u*>(ar), *reinterpret_cast<const v4u*>(ar + 64 * kXR), qh[ks],
                        ql[ks], st[kt]);
      }
      const f32x4 kbv = *reinterpret_cast<const f32x4*>(kb + kt * 16 + 4 * g);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        st[kt][e] += kbv[e];
        mx = fmaxf(mx, st[kt][e]);
      }
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16));
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    const float corr = __expf(m - mx);
    float sum = 0.f;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        st[kt][e] = __expf(st[kt][e] - mx);
        sum += st[kt][e];
      }
    sum += __shfl_xor(sum, 16);
    sum += __shfl_xor(sum, 32);
    l = l * corr + sum;
    m = mx;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] *= corr;
    // O^T += V^T P^T over the chunk's two 32-key steps
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      uint32_t ph[4], pl[4];
      split_pk(st[2 * ks][0], st[2 * ks][1], ph[0], pl[0]);
      split_pk(st[2 * ks][2], st[2 * ks][3], ph[1], pl[1]);
      split_pk(st[2 * ks + 1][0], st[2 * ks + 1][1], ph[2], pl[2]);
      split_pk(st[2 * ks + 1][2], st[2 * ks + 1][3], ph[3], pl[3]);
      const v4u pbh = v4u{ph[0], ph[1], ph[2], ph[3]}, pbl = v4u{pl[0], pl[1], pl[2], pl[3]};
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int off = (dt * 16 + c) * kXR + (ks * 32 + 4 * g) * 2;
        const uint2 a0 = *reinterpret_cast<const uint2*>(vth + off), a1 = *reinterpret_cast<const uint2*>(vth + off + 32);
        const uint2 b0 = *reinterpret_cast<const uint2*>(vtl + off), b1 = *reinterpret_cast<const uint2*>(vtl + off + 32);
        o[dt] = mma_x3(v4u{a0.x, a0.y, a1.x, a1.y}, v4u{b0.x, b0.y, b1.x, b1.y}, pbh, pbl, o[dt]);
      }
    }
    // chunk ci + 1 into the other buffer (read last in iteration ci - 1, which
    // every wave left behind the previous barrier)
    if (ci + 1 < nch) stage_store(ldsa + ((ci + 1) & 1) * kBufAX);
    __syncthreads();
  }
  const float inv = 1.f / l;
  if (out3) {
    uint16_t* const op = out3 + ((size_t)seq * S + q) * 3 * H + h * 64 + 4 * g;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      f32x4 r = o[dt] * inv;
      // the rounded product (hipcc would contract r - hi into fma(o, inv, -hi)):
      // the operand is then bitwise x3_cat of the fp32 output
      asm volatile("" : "+v"(r));
      uint32_t h0, l0, h1, l1;
      split_pk(r[0], r[1], h0, l0);
      split_pk(r[2], r[3], h1, l1);
      *reinterpret_cast<uint2*>(op + dt * 16) = make_uint2(h0, h1);
      *reinterpret_cast<uint2*>(op + H + dt * 16) = make_uint2(h0, h1);
      *reinterpret_cast<uint2*>(op + 2 * H + dt * 16) = make_uint2(l0, l1);
    }
    return;
  }
  float* const op = out + ((size_t)seq * S + q) * H + h * 64 + 4 * g;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) *reinterpret_cast<f32x4*>(op + dt * 16) = o[dt] * inv;
}

}  // namespace

extern "C" {

// fp32-parity bert: out bf16 [rows][3K] = [hi | hi | lo] of x fp32 [rows][K]
// (K % 4 == 0, 16-B aligned x, 8-B aligned out)
int tcamd_x3_cat(const float* x, void* out, int rows, int K, void* stream) {
  if (rows <= 0) return hipSuccess;
  if (!x || !out || K <= 0 || K % 4 || (uintptr_t)x % 16 || (uintptr_t)out % 8) return hipErrorInvalidValue;
  const long n4 = (long)rows * (K / 4);
  const int grid = (int)std::min<long>((n4 + 255) / 256, 256L * 16);
  hipLaunchKernelGGL(x3_cat_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, x, (uint16_t*)out, n4, K / 4);
  return hipGetLastError();
}

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

// K11p: out = LayerNorm(x + bias + sum_{z < nparts} parts[z]) * gamma + beta
// over rows of H elements (H in {512, 1024, 2048, 4096}); parts fp32, slab z
// at parts + z * pstride (elements, [rows][H] each); bias fp32 [H] or null;
// f32 = 0: x / gamma / beta / out bf16, 1: fp32.  16-B aligned pointers;
// out may alias x.
int tcamd_add_layernorm_parts3(const void* x, const float* parts, int nparts, long long pstride, const float* bias,
                               const void* gamma, const void* beta, void* out, void* out3, int rows, int H, float eps,
                               int f32, void* stream) {
  if (rows <= 0) return hipSuccess;
  if (nparts < 0 || (nparts > 0 && (!parts || pstride < (long long)rows * H)) || (out3 && !f32) ||
      ((uintptr_t)x | (uintptr_t)parts | (uintptr_t)bias | (uintptr_t)gamma | (uintptr_t)beta | (uintptr_t)out |
       (uintptr_t)out3) % 16)
    return hipErrorInvalidValue;
  const dim3 grid((rows + 3) / 4), block(256);
  hipStream_t s = (hipStream_t)stream;
#define TC_K11P(E, T)                                                                                            \
  hipLaunchKernelGGL((add_ln_parts_kernel<E, T>), grid, block, 0, s, (const T*)x, parts, nparts, pstride, bias, \
                     (const T*)gamma, (const T*)beta, (T*)out, (uint16_t*)out3, rows, eps)
  switch (H * 2 + (f32 ? 1 : 0)) {
    case 1024: TC_K11P(8, uint16_t); break;
    case 1025: TC_K11P(8, float); break;
    case 2048: TC_K11P(16, uint16_t); break;
    case 2049: TC_K11P(16, float); break;
    case 4096: TC_K11P(32, uint16_t); break;
    case 4097: TC_K11P(32, float); break;
    case 8192: TC_K11P(64, uint16_t); break;
    case 8193: TC_K11P(64, float); break;
    default: return hipErrorInvalidValue;
  }
#undef TC_K11P
  return hipGetLastError();
}

int tcamd_add_layernorm_parts(const void* x, const float* parts, int nparts, long long pstride, const float* bias,
                              const void* gamma, const void* beta, void* out, int rows, int H, float eps, int f32,
                              void* stream) {
  return tcamd_add_layernorm_parts3(x, parts, nparts, pstride, bias, gamma, beta, out, nullptr, rows, H, eps, f32,
                                    stream);
}

// QA head: start[r] = x[r] . w[0] + b[0], end[r] = x[r] . w[1] + b[1] (fp32
// out) over rows of H (512 / 1024 / 2048 / 4096) elements; x / w bf16 (f32 =
// 0) or fp32, b fp32 [2]; 16-B aligned x / w.
int tcamd_qa_head(const void* x, const void* w, const float* b, float* start, float* end, int rows, int H, int f32,
                  void* stream) {
  if (rows <= 0) return hipSuccess;
  if (!x || !w || !b || !start || !end || ((uintptr_t)x | (uintptr_t)w) % 16) return hipErrorInvalidValue;
  const dim3 grid((rows + 3) / 4), block(256);
  hipStream_t s = (hipStream_t)stream;
#define TC_QA(E, T) \
  hipLaunchKernelGGL((qa_head_kernel<E, T>), grid, block, 0, s, (const T*)x, (const T*)w, b, start, end, rows)
  switch (H * 2 + (f32 ? 1 : 0)) {
    case 1024: TC_QA(8, uint16_t); break;
    case 1025: TC_QA(8, float); break;
    case 2048: TC_QA(16, uint16_t); break;
    case 2049: TC_QA(16, float); break;
    case 4096: TC_QA(32, uint16_t); break;
    case 4097: TC_QA(32, float); break;
    case 8192: TC_QA(64, uint16_t); break;
    case 8193: TC_QA(64, float); break;
    default: return hipErrorInvalidValue;
  }
#undef TC_QA
  return hipGetLastError();
}

// Embedding sum + LayerNorm (H in {512, 1024, 2048, 4096}): out [rows][H] bf16
// = LN(word[ids] + pos[row % S] + type[types]); ids / types int64 [rows].
int tcamd_embed_layernorm(const int64_t* ids, const int64_t* types, const void* word, const void* pos,
                          const void* type, const void* gamma, const void* beta, void* out, int rows, int S, int H,
                          int vocab, int ntypes, float eps, void* stream) {
  if (rows <= 0) return hipSuccess;
  if (!ids || !types || S <= 0 || vocab <= 0 || ntypes <= 0 ||
      ((uintptr_t)word | (uintptr_t)pos | (uintptr_t)type | (uintptr_t)gamma | (uintptr_t)beta | (uintptr_t)out) % 16)
    return hipErrorInvalidValue;
  const dim3 grid((rows + 3) / 4), block(256);
  hipStream_t st = (hipStream_t)stream;
  const auto *w = (const uint16_t*)word, *p = (const uint16_t*)pos, *t = (const uint16_t*)type;
  const auto *g = (const uint16_t*)gamma, *b = (const uint16_t*)beta;
  auto* o = (uint16_t*)out;
  switch (H) {
    case 512: hipLaunchKernelGGL(embed_layernorm_kernel<8>, grid, block, 0, st, ids, types, w, p, t, g, b, o, rows, S, vocab, ntypes, eps); break;
    case 1024: hipLaunchKernelGGL(embed_layernorm_kernel<16>, grid, block, 0, st, ids, types, w, p, t, g, b, o, rows, S, vocab, ntypes, eps); break;
    case 2048: hipLaunchKernelGGL(embed_layernorm_kernel<32>, grid, block, 0, st, ids, types, w, p, t, g, b, o, rows, S, vocab, ntypes, eps); break;
    case 4096: hipLaunchKernelGGL(embed_layernorm_kernel<64>, grid, block, 0, st, ids, types, w, p, t, g, b, o, rows, S, vocab, ntypes, eps); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// K12: multi-head attention over qkv [seqs * S][3 * heads * 64] bf16 (the fused
// QKV projection's output: q | k | v, each [heads][64]) -> out [seqs * S][heads *
// 64] bf16.  mask: int32 [seqs][S] key-padding mask (0 = padded) or null.
// S % 64 == 0 and S <= 384; pointers 16-B aligned.
int tcamd_attention_bias(const void* qkv, const void* qkv_bias, const int* mask, void* out, int seqs, int S, int heads,
                         float scale, void* stream) {
  if (seqs <= 0) return hipSuccess;
  if (S <= 0 || S % 64 || S > kAMaxS || heads <= 0 || ((uintptr_t)qkv | (uintptr_t)out | (uintptr_t)qkv_bias) % 16 ||
      (uintptr_t)mask % 16)
    return hipErrorInvalidValue;
  const size_t lds = (size_t)S * kAD * 2 * 2 + (size_t)S * 4;  // K rows | V rows | key bias
  static bool attr = false;
  if (!attr) {
    hipError_t e =
        hipFuncSetAttribute((const void*)attention_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e == hipSuccess)
      e = hipFuncSetAttribute((const void*)attention_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    if (e != hipSuccess) return e;
    attr = true;
  }
  // (a streamed variant — 4-wave blocks, K/V in double-buffered 64-key chunks,
  // 35 KB of LDS — measured slower: 98-105 us vs 93 us at bs64 x 384; the
  // kernel is bound by the softmax VALU work, not by staging)
  // one block per (sequence, head) with a wave per 32 queries; small batches
  // split a head's queries over 3 or 2 blocks (each staging the head's K/V)
  // as long as that still fits one block per CU (bs1/4/8 x 384: 13/14/~16 us
  // vs torch SDPA 17/17/22 unmasked)
  const int nw = S / 32;
  int splits = 1;
  for (int sp : {3, 2})
    if (splits == 1 && nw % sp == 0 && nw / sp >= 2 && seqs * heads * sp <= 256) splits = sp;
  const int qw = nw / splits;
  const dim3 grid(seqs * heads, S / (32 * qw)), block(64 * qw);
  if (mask)
    hipLaunchKernelGGL(attention_kernel<true>, grid, block, lds, (hipStream_t)stream, (const uint16_t*)qkv, mask,
                       (uint16_t*)out, S, heads, scale, (const uint16_t*)qkv_bias);
  else
    hipLaunchKernelGGL(attention_kernel<false>, grid, block, lds, (hipStream_t)stream, (const uint16_t*)qkv, mask,
                       (uint16_t*)out, S, heads, scale, (const uint16_t*)qkv_bias);
  return hipGetLastError();
}

// K12x: fp32-parity attention over qkv [seqs * S][3 * heads * 64] fp32 (bias
// included) -> out [seqs * S][heads * 64] fp32; mask int32 [seqs][S] (0 =
// padded: additive -10000) or null.  S % 64 == 0; pointers 16-B aligned.
// x3: out is the out-projection's bf16x3 operand, bf16 [seqs * S][3 * heads * 64].
int tcamd_attention_f32(const float* qkv, const int* mask, void* out, int seqs, int S, int heads, float scale, int x3,
                        void* stream) {
  if (seqs <= 0) return hipSuccess;
  if (S <= 0 || S % 64 || heads <= 0 || ((uintptr_t)qkv | (uintptr_t)out | (uintptr_t)mask) % 16)
    return hipErrorInvalidValue;
  float* const o32 = x3 ? nullptr : (float*)out;
  uint16_t* const o3 = x3 ? (uint16_t*)out : nullptr;
  static std::atomic<bool> attr{false};  // 72.5 KB of dynamic LDS: past the 64 KB default
  if (!attr.load(std::memory_order_acquire)) {
    for (const void* fn : {(const void*)attention_x3_kernel<4>, (const void*)attention_x3_kernel<8>}) {
      const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsAX);
      if (e != hipSuccess) return e;
    }
    attr.store(true, std::memory_order_release);
  }
  // 128 queries per block (half the K / V staging per query; bs64 x 384: 331
  // -> 248 us) once that still gives every CU a block (bs1 keeps 64: 20.5 vs
  // 21.2 us; profiles/r6_bert_fp32/k12x_ab*.log)
  if (S % 128 == 0 && seqs * heads * (S / 128) >= 256)
    hipLaunchKernelGGL(attention_x3_kernel<8>, dim3(seqs * heads, S / 128), dim3(512), kLdsAX, (hipStream_t)stream,
                       qkv, mask, o32, o3, S, heads, scale);
  else
    hipLaunchKernelGGL(attention_x3_kernel<4>, dim3(seqs * heads, S / 64), dim3(256), kLdsAX, (hipStream_t)stream,
                       qkv, mask, o32, o3, S, heads, scale);
  return hipGetLastError();
}

// K12 without a bias (the projection's output already holds it)
int tcamd_attention(const void* qkv, const int* mask, void* out, int seqs, int S, int heads, float scale,
                    void* stream) {
  return tcamd_attention_bias(qkv, nullptr, mask, out, seqs, S, heads, scale, stream);
}

}  // extern "C"
