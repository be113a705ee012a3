// K18 — tiled bf16 GEMM for the bert_large projections at small and mid M
// (gfx950), with an optional split-K into fp32 partial slabs.
//
//   C[M, N] = A[M, K] . B[N, K]^T (+ bias[N]) (GELU), fp32 accumulate,
//   bf16 or fp32 out; or, split over K, fp32 partials C_z = A[:, Kz] . B[:, Kz]^T
//   that the consumer sums (K11p, csrc/kernels/bert.hip: residual + bias +
//   sum of partials + LayerNorm in one pass, so the split costs no extra
//   launch).
//
// Why a second GEMM next to K17 (csrc/kernels/gemm.hip): K17's 256x256
// persistent tile is built for 12k+ tokens.  At bert's small batches (384 -
// 6,144 tokens) a projection is 36 - 200 such tiles -- too few for 256 CUs --
// and one tile walks all of K serially (a block's latency ~ K, not N:
// cdna_hip_programming.md "Projection GEMM at M = 256").  Here:
//   * small tiles (64x64 .. 128x128) on 4- or 8-wave workgroups, several
//     resident per CU (48 - 96 KB of LDS each), so the CUs fill and blocks
//     hide each other's staging latency;
//   * K split over workgroups where the tiles are still too few (the N = 1024
//     projections: attention-out, FFN-down), each split writing an fp32 slab;
//   * K in 64-deep stages (one 128-B row per operand row) staged by LDS-DMA
//     (global_load_lds_dwordx4, no VGPR staging) into a ring of NS stages,
//     NS - 1 in flight; one raw barrier per stage, counted vmcnt (never 0
//     inside the loop).  At small M a block is bound by the latency of its
//     K walk, not by its MFMAs: the small tiles take deep rings (up to 8
//     stages, 7 in flight) to keep enough bytes in flight per CU;
//   * rows' 16-B chunks XOR-swizzled on the source address by (row >> 1) & 7:
//     every ds_read_b128 lane group of a 16x16x32 fragment read covers 16
//     distinct bank slots (MI355X_MICROARCH.md LDS table);
//   * v_mfma_f32_16x16x32_bf16, the C/D map col = lane % 16, row =
//     4 (lane / 16) + e; bias / tanh-GELU epilogue as K17's;
//   * XCD-aware block order: the blocks of one XCD walk the M tiles of a
//     weight panel together, so the panel is fetched into that XCD's L2 once.
//
// Reference analog: none (the reference client runs no model; this serves
// the bert_large perf_analyzer config of BASELINE.json).

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>

#include "kernels/common.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

constexpr int kBK = 64;         // k per stage
constexpr int kRow = kBK * 2;   // bytes of one staged operand row

// kEpiBiasGeluErf: the erf form of GELU (the fp32-parity bert, whose
// reference module uses it; the bf16 model keeps the tanh form)
enum : int { kEpiNone = 0, kEpiBias = 1, kEpiBiasGelu = 2, kEpiBiasGeluErf = 3 };

struct K18Params {
  const uint16_t* A;  // [M][lda] bf16
  const uint16_t* B;  // [N][ldb] bf16
  const float* bias;  // [N] fp32 (epi >= 1)
  void* C;            // [M][ldc] bf16 / fp32, or splits x [M][ldc] fp32
  int M, N, lda, ldb, ldc;
  int tiles_m, tiles_n, kchunk;
  long long split_stride;  // elements between the splits' slabs
};

__device__ __forceinline__ v4u lds16(const uint8_t* p) { return *reinterpret_cast<const v4u*>(p); }

__device__ __forceinline__ f32x4 mma(v4u a, v4u b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}

// 16-B chunk c of staged row r sits at chunk c ^ swz(r) (r % 16 decides)
__device__ __forceinline__ int swz(int r) { return (r >> 1) & 7; }

__device__ __forceinline__ void bar() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// vmcnt(L * n) for a runtime n <= NMAX stages left in flight (L LDS-DMAs
// per stage): the counted wait must be an immediate
template <int L, int NMAX>
__device__ __forceinline__ void wait_stages(int n) {
  if constexpr (NMAX <= 0) {
    vm_wait<0>();
  } else {
    if (n >= NMAX) vm_wait<L * NMAX>();
    else wait_stages<L, NMAX - 1>(n);
  }
}

__device__ __forceinline__ uint32_t pk2(float lo, float hi) {
  const bf16x2 v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(uint32_t, v);
}

// tanh-form GELU on column pairs (the form K17 and hipBLASLt's epilogue use)
__device__ __forceinline__ f32x2 gelu2(f32x2 x) {
  constexpr float kC1 = -2.3022081983f;  // -2 sqrt(2/pi) log2(e)
  constexpr float kC3 = kC1 * 0.044715f;
  const f32x2 w = x * __builtin_elementwise_fma(x * x, f32x2{kC3, kC3}, f32x2{kC1, kC1});
  const f32x2 d = f32x2{__builtin_amdgcn_exp2f(w.x), __builtin_amdgcn_exp2f(w.y)} + 1.0f;
  return x * f32x2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
}

__device__ __forceinline__ f32x2 gelu_erf2(f32x2 x) {
  return f32x2{0.5f * x.x * (1.0f + erff(x.x * 0.70710678118654752f)),
               0.5f * x.y * (1.0f + erff(x.y * 0.70710678118654752f))};
}

// TM x TN output tile per workgroup of WM x WN waves, an NS-stage ring; EPI;
// F32 output (a split-K launch writes slab z at C + z * split_stride).
template <int TM, int TN, int WM, int WN, int NS, int EPI, bool F32>
__global__ void __launch_bounds__(64 * WM * WN) k18_gemm_kernel(K18Params p) {
  constexpr int NW = WM * WN;
  constexpr int RM = TM / WM, RN = TN / WN;  // a wave's output rows / columns
  constexpr int FM = RM / 16, FN = RN / 16;  // its 16x16 fragments
  constexpr int SB = (TM + TN) * kRow;       // one stage: A rows | B rows
  constexpr int L = (TM + TN) / (8 * NW);    // 1-KB LDS-DMAs per wave per stage
  static_assert((TM + TN) % (8 * NW) == 0 && RM % 16 == 0 && RN % 16 == 0, "tile / wave split");
  static_assert(TM % 16 == 0, "A rows keep the swizzle phase of the B rows");
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WN, wc = wave % WN;

  // XCD-aware order (bijective): blocks with equal b % 8 share an XCD; each
  // XCD gets a contiguous run of ids, M tiles fastest (one weight panel)
  const int G = (int)gridDim.x, b = (int)blockIdx.x;
  const int q8 = G >> 3, r8 = G & 7, x8 = b & 7;
  const int id = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + (b >> 3);
  const int mt = id % p.tiles_m, rest = id / p.tiles_m;
  const int nt = rest % p.tiles_n, z = rest / p.tiles_n;
  const int m0 = mt * TM, n0 = nt * TN;
  const int nk = p.kchunk / kBK;

  // LDS-DMA: wave w's instruction i fills staged rows 8 (L w + i) .. + 7
  // (rows < TM: A, else B), lane-linear (row + lane / 8, chunk' lane % 8)
  // from global chunk (lane % 8) ^ swz(row) of that row
  const uint16_t* src[L];
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const int row = 8 * (L * wave + i) + (lane >> 3);
    const int ch = (lane & 7) ^ swz(row);
    src[i] = row < TM ? p.A + (size_t)min(m0 + row, p.M - 1) * p.lda + (size_t)z * p.kchunk + 8 * ch
                      : p.B + (size_t)(n0 + row - TM) * p.ldb + (size_t)z * p.kchunk + 8 * ch;
  }
  auto stage = [&](int t, int buf) {
    uint8_t* dst = lds + buf * SB + L * wave * 1024;
#pragma unroll
    for (int i = 0; i < L; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(src[i] + t * kBK), (void*)(dst + i * 1024), 16, 0, 0);
  };
  // fragment reads: lane (row r = lane % 16 of a 16-row block, k chunk
  // 4 ks + lane / 16) -> swizzled chunk
  int lofs[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
    lofs[ks] = (lane & 15) * kRow + (((4 * ks + (lane >> 4)) ^ swz(lane & 15)) << 4);
  const int a_off = wr * RM * kRow, b_off = (TM + wc * RN) * kRow;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: stages 0 .. NS - 2 in flight (past nk: nothing)
#pragma unroll
  for (int i = 0; i < NS - 1; ++i)
    if (i < nk) stage(i, i);
  int buf = 0;
  for (int t = 0; t < nk; ++t) {
    // stage t landed (this wave's DMAs; the barrier makes every wave's
    // visible), the later ones stay in flight; every wave is past its reads
    // of stage t - 1, whose buffer stage t + NS - 1 now refills.  The wait
    // count: min(NS - 2, nk - 1 - t) stages may stay in flight
    wait_stages<L, NS - 2>(min(NS - 2, nk - 1 - t));
    bar();
    if (t + NS - 1 < nk) stage(t + NS - 1, buf == 0 ? NS - 1 : buf - 1);
    const uint8_t* sb = lds + buf * SB;
    // both 32-deep k steps' fragments first, then the MFMAs
    v4u a[2][FM], bb[2][FN];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int j = 0; j < FN; ++j) bb[ks][j] = lds16(sb + b_off + j * 16 * kRow + lofs[ks]);
#pragma unroll
      for (int i = 0; i < FM; ++i) a[ks][i] = lds16(sb + a_off + i * 16 * kRow + lofs[ks]);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mma(a[ks][i], bb[ks][j], acc[i][j]);
    buf = buf == NS - 1 ? 0 : buf + 1;
  }

  // ---- epilogue: C/D map col = lane % 16, row = 4 (lane / 16) + e ----
  const int col_l = lane & 15, row_l = (lane >> 4) * 4, par = lane & 1;
  const bool full = m0 + TM <= p.M;  // block-uniform
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int col = n0 + wc * RN + j * 16 + col_l;
    const float bj = EPI >= kEpiBias ? p.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int row0 = m0 + wr * RM + i * 16 + row_l;
      f32x2 v01 = f32x2{acc[i][j][0], acc[i][j][1]} + bj, v23 = f32x2{acc[i][j][2], acc[i][j][3]} + bj;
      if (EPI == kEpiBiasGelu) {
        v01 = gelu2(v01);
        v23 = gelu2(v23);
      } else if (EPI == kEpiBiasGeluErf) {
        v01 = gelu_erf2(v01);
        v23 = gelu_erf2(v23);
      }
      const float v[4] = {v01.x, v01.y, v23.x, v23.y};
      if constexpr (F32) {
        float* out = reinterpret_cast<float*>(p.C) + (size_t)z * p.split_stride;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (full || row0 + e < p.M) out[(size_t)(row0 + e) * p.ldc + col] = v[e];
      } else {
        // lanes 2c / 2c + 1 swap halves (DPP quad_perm [1, 0, 3, 2]) so each
        // stores two rows of a column pair as 4-byte words
        const uint32_t send = par ? pk2(v[0], v[1]) : pk2(v[2], v[3]);
        const uint32_t recv = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)send, 0xB1, 0xf, 0xf, false);
        const float r0 = __uint_as_float(recv << 16), r1 = __uint_as_float(recv & 0xffff0000u);
        const uint32_t w0 = par ? pk2(r0, v[2]) : pk2(v[0], r0);
        const uint32_t w1 = par ? pk2(r1, v[3]) : pk2(v[1], r1);
        const int r = row0 + 2 * par, c = col - par;
        uint32_t* out = reinterpret_cast<uint32_t*>(reinterpret_cast<uint16_t*>(p.C) + (size_t)r * p.ldc + c);
        if (full || r < p.M) out[0] = w0;
        if (full || r + 1 < p.M) out[p.ldc / 2] = w1;
      }
    }
  }
}

struct Cfg {
  int tm, tn, threads, stages;
};
// the tile configurations (index = the cfg argument of tcamd_k18_gemm)
constexpr Cfg kCfgs[] = {
    {64, 64, 256, 3},    // 0: 48 KB LDS, 3 blocks per CU
    {128, 64, 256, 3},   // 1: 72 KB, 2 per CU
    {64, 128, 256, 3},   // 2: 72 KB, 2 per CU
    {128, 128, 512, 3},  // 3: 96 KB, 1 per CU, 8 waves
    {128, 128, 256, 3},  // 4: 96 KB, 1 per CU, 4 waves of 64 x 64
    {64, 64, 256, 8},    // 5: 128 KB, 1 per CU, 7 stages in flight
    {64, 64, 256, 5},    // 6: 80 KB, 2 per CU, 4 in flight
    {64, 128, 256, 6},   // 7: 144 KB, 1 per CU, 5 in flight
    {128, 64, 256, 6},   // 8: 144 KB, 1 per CU, 5 in flight
    {32, 64, 256, 8},    // 9: 96 KB, 1 per CU, 7 in flight (4 waves of 16 x 32)
    {128, 128, 512, 4},  // 10: 128 KB, 1 per CU, 3 in flight, 8 waves
    {128, 64, 256, 5},   // 11: 120 KB, 1 per CU, 4 in flight
    {256, 128, 512, 3},  // 12: 144 KB, 1 per CU, 8 waves of 128 x 32
};
constexpr int kNumCfgs = sizeof(kCfgs) / sizeof(kCfgs[0]);

template <int TM, int TN, int WM, int WN, int NS, int EPI, bool F32>
hipError_t launch_k(const K18Params& prm, int grid, hipStream_t s) {
  constexpr int lds = NS * (TM + TN) * kRow;
  static std::atomic<uint32_t> attr_done{0};  // one bit per device (<= 32)
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  const uint32_t bit = 1u << (dev & 31);
  if (!(attr_done.load(std::memory_order_acquire) & bit)) {
    e = hipFuncSetAttribute((const void*)k18_gemm_kernel<TM, TN, WM, WN, NS, EPI, F32>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    attr_done.fetch_or(bit, std::memory_order_acq_rel);
  }
  hipLaunchKernelGGL((k18_gemm_kernel<TM, TN, WM, WN, NS, EPI, F32>), dim3(grid), dim3(64 * WM * WN), lds, s, prm);
  return hipGetLastError();
}

template <int TM, int TN, int WM, int WN, int NS>
hipError_t launch_cfg(const K18Params& prm, int grid, hipStream_t s, int epi, bool f32) {
  if (f32) {
    if (epi == kEpiNone) return launch_k<TM, TN, WM, WN, NS, kEpiNone, true>(prm, grid, s);
    if (epi == kEpiBias) return launch_k<TM, TN, WM, WN, NS, kEpiBias, true>(prm, grid, s);
    if (epi == kEpiBiasGeluErf) return launch_k<TM, TN, WM, WN, NS, kEpiBiasGeluErf, true>(prm, grid, s);
    return launch_k<TM, TN, WM, WN, NS, kEpiBiasGelu, true>(prm, grid, s);
  }
  if (epi == kEpiNone) return launch_k<TM, TN, WM, WN, NS, kEpiNone, false>(prm, grid, s);
  if (epi == kEpiBias) return launch_k<TM, TN, WM, WN, NS, kEpiBias, false>(prm, grid, s);
  return launch_k<TM, TN, WM, WN, NS, kEpiBiasGelu, false>(prm, grid, s);
}

std::atomic<long long> g_k18_calls{0};

}  // namespace

extern "C" {

// K18: C = A . B^T (+ bias) (GELU) with bf16 A [M][lda], B [N][ldb] (K
// contiguous), fp32 bias [N], C bf16 (out_f32 = 0) or fp32 [M][ldc]; cfg
// indexes the tile table above.  splits > 1 splits K over
// workgroups: C is then fp32 (out_f32 = 1, epi = 0); epi 3 (bias + erf
// GELU) with fp32 C only and split z writes its
// partial A[:, Kz] . B[:, Kz]^T at C + z * split_stride (elements, >= M * ldc).
// N a multiple of the tile width, K of 64 x splits; lda / ldb / ldc multiples
// of 8 (2 for fp32 C), 16-B aligned A / B / C; any M >= 1.
int tcamd_k18_gemm(const void* A, const void* B, const float* bias, void* C, int M, int N, int K, int lda, int ldb,
                   int ldc, int epi, int out_f32, int cfg, int splits, long long split_stride, void* stream) {
  if (M <= 0) return hipSuccess;
  if (cfg < 0 || cfg >= kNumCfgs || splits < 1 || splits > 64) return hipErrorInvalidValue;
  const Cfg c = kCfgs[cfg];
  if (!A || !B || !C || N <= 0 || N % c.tn || K <= 0 || K % (kBK * splits) || epi < 0 || epi > 3)
    return hipErrorInvalidValue;
  if (epi == kEpiBiasGeluErf && !out_f32) return hipErrorInvalidValue;  // the fp32-parity form only
  if (lda < K || ldb < K || ldc < N || lda % 8 || ldb % 8 || ldc % (out_f32 ? 2 : 8)) return hipErrorInvalidValue;
  if (((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) % 16 || (epi && (!bias || (uintptr_t)bias % 4)))
    return hipErrorInvalidValue;
  if (splits > 1 && (!out_f32 || epi != kEpiNone || split_stride < (long long)M * ldc)) return hipErrorInvalidValue;
  K18Params prm;
  prm.A = (const uint16_t*)A;
  prm.B = (const uint16_t*)B;
  prm.bias = bias;
  prm.C = C;
  prm.M = M;
  prm.N = N;
  prm.lda = lda;
  prm.ldb = ldb;
  prm.ldc = ldc;
  prm.tiles_m = (M + c.tm - 1) / c.tm;
  prm.tiles_n = N / c.tn;
  prm.kchunk = K / splits;
  prm.split_stride = split_stride;
  const long long grid = (long long)prm.tiles_m * prm.tiles_n * splits;
  if (grid > (1ll << 30)) return hipErrorInvalidValue;
  g_k18_calls.fetch_add(1, std::memory_order_relaxed);
  hipStream_t s = (hipStream_t)stream;
  const bool f32 = out_f32 != 0;
  switch (cfg) {
    case 0: return launch_cfg<64, 64, 2, 2, 3>(prm, (int)grid, s, epi, f32);
    case 1: return launch_cfg<128, 64, 2, 2, 3>(prm, (int)grid, s, epi, f32);
    case 2: return launch_cfg<64, 128, 2, 2, 3>(prm, (int)grid, s, epi, f32);
    case 3: return launch_cfg<128, 128, 2, 4, 3>(prm, (int)grid, s, epi, f32);
    case 4: return launch_cfg<128, 128, 2, 2, 3>(prm, (int)grid, s, epi, f32);
    case 5: return launch_cfg<64, 64, 2, 2, 8>(prm, (int)grid, s, epi, f32);
    case 6: return launch_cfg<64, 64, 2, 2, 5>(prm, (int)grid, s, epi, f32);
    case 7: return launch_cfg<64, 128, 2, 2, 6>(prm, (int)grid, s, epi, f32);
    case 8: return launch_cfg<128, 64, 2, 2, 6>(prm, (int)grid, s, epi, f32);
    case 9: return launch_cfg<32, 64, 2, 2, 8>(prm, (int)grid, s, epi, f32);
    case 10: return launch_cfg<128, 128, 2, 4, 4>(prm, (int)grid, s, epi, f32);
    case 11: return launch_cfg<128, 64, 2, 2, 5>(prm, (int)grid, s, epi, f32);
    default: return launch_cfg<256, 128, 2, 4, 3>(prm, (int)grid, s, epi, f32);
  }
}

// the tile table: cfg i -> tile rows, columns, threads and ring stages (tools, tests)
int tcamd_k18_cfg(int cfg, int* tm, int* tn, int* threads, int* stages) {
  if (cfg < 0 || cfg >= kNumCfgs) return -1;
  if (tm) *tm = kCfgs[cfg].tm;
  if (tn) *tn = kCfgs[cfg].tn;
  if (threads) *threads = kCfgs[cfg].threads;
  if (stages) *stages = kCfgs[cfg].stages;
  return 0;
}

// launches so far (tests: which projections a model routed through K18)
long long tcamd_k18_calls() { return g_k18_calls.load(std::memory_order_relaxed); }

}  // extern "C"
