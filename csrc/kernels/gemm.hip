// K17 — bf16 GEMM for the bert_large projections (gfx950).
//
//   C[M, N] = A[M, K] . B[N, K]^T (+ bias[N]) (GELU), fp32 accumulate,
//   bf16 or fp32 out.  A = activations (tokens x hidden), B = a torch Linear
//   weight [out, in]: both operands K-contiguous.
//
// Structure (the 256x256 ping-pong schedule of the CDNA4 playbook, built
// for these operands):
//   * one 256x256 output tile per 512-thread workgroup, 8 waves as 2 (M) x
//     4 (N), each wave 128 x 64 outputs = 8 x 4 accumulators of
//     v_mfma_f32_16x16x32_bf16 (128 VGPRs);
//   * K in slabs of 32: A and B slabs [256 rows][32 k] bf16 (16 KB each)
//     staged by LDS-DMA (global_load_lds_dwordx4, no VGPR staging) into a
//     ring of 4 slab buffers (128 KB), 3 slabs ahead, swizzled on the source
//     address (16-B chunk c of row r lands at chunk c ^ swz(r)) so every
//     ds_read_b128 of a fragment is bank-conflict free;
//   * per slab an R interval (the slab's fragments from LDS, the LDS-DMAs of
//     slab s+3, the counted vmcnt that retires slab s+1, lgkmcnt(0),
//     barrier) and an M interval (32 MFMAs, barrier);
//     waves 4-7 run one barrier behind waves 0-3, so on every SIMD one wave
//     reads while the other multiplies;
//   * the counted vmcnt never drains the ring inside the loop (loads past the
//     last slab re-read it into a free buffer, so the counts stay constant);
//   * persistent: one workgroup per CU walks its tiles, and their K slabs are
//     one continuous stream through the ring (no per-tile prologue wait);
//     the bf16 epilogue stores 4-byte column pairs (a lane-pair swap);
//   * XCD-aware tile order: the tiles of one M panel run on one XCD (its L2
//     keeps the A panel);
//   * dynamic tile scheduling (round 6): a workgroup's first tile is its own
//     id, every later one is claimed from a device counter (one returning
//     atomic per tile, issued at the start of the tile before it, so its
//     round trip hides behind a slab interval).  A workgroup that starts late --
//     its CU still running the previous kernel's tail -- simply claims fewer
//     tiles, instead of finishing a fixed tile list late (the in-graph loss of
//     the fixed list: profiles/r5_k17_gemm.md).  The last workgroup to finish
//     resets the counter, so a HIP graph replays the launch with no memset
//     node; one counter per stream (kernels of one stream never overlap).
//
// Reference analog: none (the reference client runs no model; this serves
// the bert_large perf_analyzer config of BASELINE.json).

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <mutex>

#include "kernels/common.h"
#include "kernels/knobs.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

constexpr int kTile = 256;   // N per tile; M per tile: TM = 256 or 128
constexpr int kSlabK = 32;   // k per slab
constexpr int kBBytes = kTile * kSlabK * 2;  // B's slab: 16 KB
constexpr int kRing = 4;
constexpr int kMaxBiasN = 8188;  // bias copy behind the ring and the tile queue (<= 32 KB - 16 B)
constexpr int kTq = 16;          // LDS tile queue of the dynamic scheduler (4 ints)
constexpr int slab_bytes(int tm) { return tm * kSlabK * 2 + kBBytes; }  // A | B
constexpr int ring_bytes(int tm) { return kRing * slab_bytes(tm); }     // 128 / 96 KB

// kEpiBiasGeluErf: the erf form of GELU (the fp32-parity bert, whose
// reference module uses it; the bf16 model keeps the tanh form).
// kEpiBiasGeluErfX3: the same, written as the next bf16x3 GEMM's operand:
// bf16 C [M][ldc >= 3N] = [hi | hi | lo] of each fp32 result (the FFN-down
// input of the fp32-parity bert, which then needs no x3_cat pass)
enum : int { kEpiNone = 0, kEpiBias = 1, kEpiBiasGelu = 2, kEpiBiasGeluErf = 3, kEpiBiasGeluErfX3 = 4 };

struct K17Params {
  const uint16_t* A;  // [M][lda] bf16
  const uint16_t* B;  // [N][ldb] bf16
  const float* bias;  // [N] fp32 (epi >= 1)
  void* C;            // [M][ldc] bf16 or fp32
  int M, N, K, lda, ldb, ldc;
  int tiles_m, tiles_n;
  int* sched;  // {next, done} claim counters (dynamic scheduling) or null (static tile list)
};

__device__ __forceinline__ v4u lds16(const uint8_t* p) { return *reinterpret_cast<const v4u*>(p); }

__device__ __forceinline__ f32x4 mma(v4u a, v4u b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}

// GELU in its tanh form, x sigmoid(2 sqrt(2/pi) (x + 0.044715 x^3)) (the
// form hipBLASLt's GELU epilogue -- bert's library path -- computes; within
// 5e-4 of the erf form, far below bf16's rounding), on column pairs: the
// multiplies/FMAs as packed f32 (v_pk_*: two columns per issue), exp2 and the
// reciprocal on the transcendental unit.  The epilogue runs between barriers,
// so every instruction of it stalls the other wave group: ~14 issue cycles
// per element (the erf form with scalar f32 took ~34; FFN-up at 24,576
// tokens 219.8 -> 200.3 us, profiles/r5_k17_gemm.md)
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 gelu2(f32x2 x) {
  constexpr float kC1 = -2.3022081983f;            // -2 sqrt(2/pi) log2(e)
  constexpr float kC3 = kC1 * 0.044715f;
  const f32x2 w = x * __builtin_elementwise_fma(x * x, f32x2{kC3, kC3}, f32x2{kC1, kC1});
  const f32x2 d = f32x2{__builtin_amdgcn_exp2f(w.x), __builtin_amdgcn_exp2f(w.y)} + 1.0f;
  return x * f32x2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};  // x -> -inf: x * 0
}

// The dynamic scheduler's claim: a returning atomic add of 1 to *ctr, as
// inline asm so hipcc does not wait for it -- its own waits would be a
// vmcnt(0) at the use (the claim is loop-carried across the slab loop), which
// drains the LDS-DMA ring.  The kernel's counted ring wait one slab later
// retires it instead (VMEM ops return in issue order).  The destination VGPR
// must stay untouched until then: tests/test_gemm_isa.py checks the built code
// object for that (the register is read only by the consumer).
__device__ __forceinline__ int claim_tile(int* ctr) {
  int old;
  asm volatile("global_atomic_add %0, %1, %2, off sc0" : "=v"(old) : "v"(ctr), "v"(1) : "memory");
  return old;
}

// raw barrier (no vmcnt(0): the ring's LDS-DMAs stay in flight across it);
// the empty asm keeps LDS reads from moving across
__device__ __forceinline__ void bar() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// A-operand LDS-DMAs per slab of a wave in group 0 (waves 0-3) / group 1
// (waves 4-7): TM / 16 instructions of 16 rows, split 2 / 2 (256), 2 / 1
// (192), 1 / 1 (128)
constexpr int ai0(int tm) { return tm == 128 ? 1 : 2; }
constexpr int ai1(int tm) { return tm == 256 ? 2 : 1; }

// the counted wait that retires slab g + 1 (slabs g + 2 and g + 3 in
// flight: 2 x this wave's LDS-DMAs per slab), and the deeper one before a
// tile's epilogue (slabs g + 1 AND g + 2 landed, only g + 3 in flight) so the
// next tile's first R interval needs no wait and the epilogue's stores (which
// vmcnt counts in issue order with the LDS-DMAs) get two intervals to retire
__device__ __forceinline__ void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <int TM>
__device__ __forceinline__ void wait_ring(bool grp1) {
  if (grp1) vm_wait<2 * (ai1(TM) + 2)>();
  else vm_wait<2 * (ai0(TM) + 2)>();
}
template <int TM>
__device__ __forceinline__ void wait_ring_deep(bool grp1) {
  if (grp1) vm_wait<ai1(TM) + 2>();
  else vm_wait<ai0(TM) + 2>();
}

// 16-B chunk swizzle of a 64-B slab row: chunk c of row r sits at c ^ swz(r).
// A fragment read (lane l: row l % 16, chunk l / 16) is then conflict-free
// in each of ds_read_b128's four lane groups ({0-3, 12-15, 20-27}, ...:
// MI355X_MICROARCH.md LDS table): within a group the rows that share a
// bank-row quarter (equal r % 4) land on four different chunks.  (The
// (r >> 2) & 3 swizzle of a contiguous-16-lane model is 2-way there.)
__device__ __forceinline__ int swz(int r) { return ((r >> 3) & 1) << 1; }

__device__ __forceinline__ uint32_t pk2(float lo, float hi) {
  const bf16x2 v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(uint32_t, v);
}

template <int TM, int EPI, bool OUTF32>
__global__ void __launch_bounds__(512, 1) k17_gemm_kernel(K17Params p) {
  constexpr int kAI = ai0(TM);  // the most A LDS-DMAs per slab of a wave
  constexpr int kMT = TM / 32;  // 16-row MFMA tiles per wave (TM / 2 rows)
  constexpr int kSlab = slab_bytes(TM), kLds = ring_bytes(TM);
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const bool grp1 = __builtin_amdgcn_readfirstlane(wave) >= 4;  // wave-uniform
  const int nai = grp1 ? ai1(TM) : ai0(TM);                     // this wave's A LDS-DMAs per slab
  const int arow0 = grp1 ? 64 * ai0(TM) + 16 * ai1(TM) * (wave - 4) : 16 * ai0(TM) * wave;
  // persistent: workgroup b takes tiles seq[0], seq[1], ... and the K slabs
  // of all of them form ONE stream through the LDS ring (the next tile's
  // first slabs load during this tile's last ones and its epilogue).
  // Static: seq[k] = b + k G.  Dynamic (p.sched): seq[0] = b, seq[k + 1] = G +
  // a claimed counter value, claimed by thread 0 in the R interval of tile
  // k's slab 0 and written to an LDS ring of 4 (tq) in slab 1's, which every
  // wave reads behind at least one barrier (staging reaches tile k + 1 at
  // slab nsl - 3; the host asks for nsl >= 6).
  const int G = (int)gridDim.x, wg = (int)blockIdx.x;
  const int ntiles = p.tiles_m * p.tiles_n;
  const int nsl = p.K / kSlabK;
  const bool dyn = p.sched != nullptr;  // launch-uniform
  int* const tq = reinterpret_cast<int*>(lds + kLds);
  const bool claimer = dyn && tid == 0;
  auto seq = [&](int k) -> int {
    if (!dyn) return wg + k * G;
    return k == 0 ? wg : __builtin_amdgcn_readfirstlane(tq[k & 3]);
  };

  // XCD-aware tile order (bijective): tiles with equal t % 8 run on one XCD
  // (G is a multiple of 8 or the whole grid); give each XCD a contiguous
  // M-panel-major run of tile ids, so the tiles an XCD runs together share
  // their A panel in its L2 (dynamic claims keep the claim order, which
  // interleaves the XCDs the same way)
  auto origin = [&](int t, int& m0, int& n0) {
    const int x = t & 7, q8 = ntiles >> 3, r8 = ntiles & 7;
    const int id = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + (t >> 3);
    const int tm = id / p.tiles_n;
    m0 = tm * TM;
    n0 = (id - tm * p.tiles_n) * kTile;
  };

  // ---- LDS-DMA: wave w's instruction i of an operand fills slab rows
  // 16 (n w + i) .. + 15 (n = that operand's instructions per wave; 1 KB,
  // lane-linear: row 16 (n w + i) + lane/4, chunk' lane%4) from global
  // chunk c = chunk' ^ swz(row) of that row
  int arow[kAI], acol[kAI], brow[2], bcol[2];
#pragma unroll
  for (int i = 0; i < kAI; ++i) {
    arow[i] = arow0 + 16 * i + (lane >> 2);
    acol[i] = 8 * ((lane & 3) ^ swz(arow[i]));
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    brow[i] = 16 * (2 * wave + i) + (lane >> 2);
    bcol[i] = 8 * ((lane & 3) ^ swz(brow[i]));
  }
  // staging cursor: the slab stream position gs (its ring buffer gs % 4),
  // the tile and slab it loads (past the end: the last slab again, into a
  // buffer nobody reads, so every vmcnt count stays constant) and that
  // tile's per-lane source rows
  int gs = 0, st_tl = 0, st_s = 0;
  const uint16_t* sa[kAI];
  const uint16_t* sbp[2];
  auto set_tile = [&](int t) {
    int m0, n0;
    origin(t, m0, n0);
#pragma unroll
    for (int i = 0; i < kAI; ++i) sa[i] = p.A + (size_t)min(m0 + arow[i], p.M - 1) * p.lda + acol[i];
#pragma unroll
    for (int i = 0; i < 2; ++i) sbp[i] = p.B + (size_t)(n0 + brow[i]) * p.ldb + bcol[i];
  };
  set_tile(wg);
  auto stage = [&]() {
    uint8_t* dst = lds + (gs & (kRing - 1)) * kSlab;
    const int k0 = st_s * kSlabK;
#pragma unroll
    for (int i = 0; i < kAI; ++i)
      if (i < nai)
        __builtin_amdgcn_global_load_lds((const void*)(sa[i] + k0), (void*)(dst + (arow0 / 16 + i) * 1024), 16, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(sbp[i] + k0), (void*)(dst + TM * 64 + (2 * wave + i) * 1024), 16,
                                       0, 0);
    ++gs;
    if (++st_s == nsl) {
      const int nxt = seq(st_tl + 1);
      if (nxt < ntiles) {
        st_s = 0;
        ++st_tl;
        set_tile(nxt);
      } else {
        st_s = nsl - 1;
      }
    }
  };
  // fragment reads: 16-row tile at row R0 (a multiple of 16), lane row R0 +
  // lane%16, k chunk lane/16 -> swizzled chunk (lane/16) ^ swz(lane % 16)
  const int lane_off = (lane & 15) * 64 + (((lane >> 4) ^ swz(lane & 15)) << 4);
  const int a_off = (wr * (TM / 2)) * 64 + lane_off;
  const int b_off = TM * 64 + (wc * 64) * 64 + lane_off;

  // the bias in LDS behind the ring: an ordinary global load used in the
  // epilogue would make hipcc wait vmcnt(0) there, draining the ring's
  // in-flight LDS-DMAs of the next tile
  float* const bias_l = reinterpret_cast<float*>(lds + kLds + kTq);
  if (EPI >= kEpiBias) {
    for (int c = tid; c < p.N; c += 512) bias_l[c] = p.bias[c];
    __syncthreads();
  }
  // prologue: slabs 0..2 in flight, slab 0 landed
  for (int i = 0; i < 3; ++i) stage();
  wait_ring<TM>(grp1);
  bar();
  // waves 4-7 run one barrier behind
  if (grp1) bar();

  const int col_l = lane & 15, row_l = (lane >> 4) * 4, par = lane & 1;
  f32x4 acc[kMT][4];
  v4u a[kMT], b[4];
  int g = 0;
  int cn;  // the claimed counter value (dynamic), in flight from slab 0 to slab 1
  for (int tl = 0;; ++tl) {
    const int tile = seq(tl);
    if (tile >= ntiles) break;
#pragma unroll
    for (int i = 0; i < kMT; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < nsl; ++s, ++g) {
      const uint8_t* sb = lds + (g & (kRing - 1)) * kSlab;
      // ---- R interval: this slab's fragments (the wave's TM / 2 rows x 64
      // columns), the LDS-DMAs of slab g + 3, slab g + 1 landed ----
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = lds16(sb + b_off + j * 16 * 64);
#pragma unroll
      for (int i = 0; i < kMT; ++i) a[i] = lds16(sb + a_off + i * 16 * 64);
      // dynamic: claim seq[tl + 1] ahead of this slab's LDS-DMAs (claim_tile)
      if (claimer && s == 0) cn = claim_tile(p.sched);
      stage();
      // this wave's LDS-DMAs of slab g + 1 landed (g + 2, g + 3 in flight);
      // a tile's first slab: waited for before the last epilogue
      if (s != 0 || tl == 0) wait_ring<TM>(grp1);
      // slab 1: that wait retired every VMEM op issued before slab 0's
      // LDS-DMAs, the claim's return among them
      if (claimer && s == 1) tq[(tl + 1) & 3] = G + cn;
      wait_lgkm0();
      bar();
      // ---- M interval: 4 kMT MFMAs ----
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < kMT; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mma(a[i], b[j], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
      bar();
    }

    wait_ring_deep<TM>(grp1);
    // ---- epilogue of tile tl (no barriers: the other wave group's interval
    // just runs longer).  C/D map of 16x16x32: col = lane % 16, row =
    // 4 (lane / 16) + e.  bf16: lanes 2c and 2c + 1 swap halves so each
    // stores two rows of a column pair as 4-byte words ----
    int m0, n0;
    origin(tile, m0, n0);
    float bj[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bj[j] = EPI >= kEpiBias ? bias_l[n0 + wc * 64 + j * 16 + col_l] : 0.f;
    const bool full = m0 + TM <= p.M;  // block-uniform
#pragma unroll
    for (int i = 0; i < kMT; ++i) {
      const int row0 = m0 + wr * (TM / 2) + i * 16 + row_l;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = n0 + wc * 64 + j * 16 + col_l;
        f32x2 v01 = f32x2{acc[i][j][0], acc[i][j][1]}, v23 = f32x2{acc[i][j][2], acc[i][j][3]};
        if (EPI >= kEpiBias) {
          v01 += bj[j];
          v23 += bj[j];
        }
        if (EPI == kEpiBiasGelu) {
          v01 = gelu2(v01);
          v23 = gelu2(v23);
        } else if (EPI == kEpiBiasGeluErf || EPI == kEpiBiasGeluErfX3) {
          v01 = f32x2{0.5f * v01.x * (1.0f + erff(v01.x * 0.70710678118654752f)),
                      0.5f * v01.y * (1.0f + erff(v01.y * 0.70710678118654752f))};
          v23 = f32x2{0.5f * v23.x * (1.0f + erff(v23.x * 0.70710678118654752f)),
                      0.5f * v23.y * (1.0f + erff(v23.y * 0.70710678118654752f))};
        }
        float v[4] = {v01.x, v01.y, v23.x, v23.y};
        // bf16 stores of 4 rows of this column at column offset co
        auto store_bf16 = [&](const float (&w)[4], int co) {
          const uint32_t send = par ? pk2(w[0], w[1]) : pk2(w[2], w[3]);
          // lane ^ 1 by DPP quad_perm [1, 0, 3, 2] (a VALU move, no LDS round trip)
          const uint32_t recv = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)send, 0xB1, 0xf, 0xf, false);
          const float r0 = __uint_as_float(recv << 16), r1 = __uint_as_float(recv & 0xffff0000u);
          // even lane: rows 0, 1 of columns (c, c + 1); odd lane: rows 2, 3 of (c - 1, c)
          const uint32_t w0 = par ? pk2(r0, w[2]) : pk2(w[0], r0);
          const uint32_t w1 = par ? pk2(r1, w[3]) : pk2(w[1], r1);
          const int r = row0 + 2 * par, c = col - par + co;
          uint32_t* out = reinterpret_cast<uint32_t*>(reinterpret_cast<uint16_t*>(p.C) + (size_t)r * p.ldc + c);
          if (full || r < p.M) out[0] = w0;
          if (full || r + 1 < p.M) out[p.ldc / 2] = w1;
        };
        if constexpr (OUTF32) {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (full || row0 + e < p.M) reinterpret_cast<float*>(p.C)[(size_t)(row0 + e) * p.ldc + col] = v[e];
        } else if constexpr (EPI == kEpiBiasGeluErfX3) {
          // hi = bf16(v) (exact in the bf16 stores), lo = v - hi (rounded by
          // them); the asm keeps v the rounded GELU value (no contraction of
          // v - hi into its product), as x3_cat would see it
          asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]));
          float hv[4], lv[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            hv[e] = __uint_as_float(pk2(v[e], 0.f) << 16);
            lv[e] = v[e] - hv[e];
          }
          store_bf16(hv, 0);
          store_bf16(hv, p.N);
          store_bf16(lv, 2 * p.N);
        } else {
          store_bf16(v, 0);
        }
      }
    }
  }
  if (!grp1) bar();  // the same barrier count for all waves
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the re-reads past the last slab
  // dynamic: the last workgroup out (all claims of all workgroups returned
  // before their done adds) resets the counters for the next launch
  if (claimer && atomicAdd(p.sched + 1, 1) == G - 1) {
    atomicExch(p.sched, 0);
    atomicExch(p.sched + 1, 0);
  }
}

bool a16(const void* q) { return ((uintptr_t)q & 15) == 0; }

int cu_count() {
  static std::atomic<int> n{0};
  int v = n.load(std::memory_order_relaxed);
  if (!v) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    n.store(v, std::memory_order_relaxed);
  }
  return v;
}

template <int TM, int EPI, bool F32>
hipError_t launch_tm(const K17Params& prm, int grid, hipStream_t s) {
  constexpr int kLds = ring_bytes(TM);
  const int lds_bytes = kLds + kTq + (EPI >= kEpiBias ? 4 * prm.N : 0);
  static std::atomic<uint32_t> attr_done{0};  // one bit per device (<= 32)
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  const uint32_t bit = 1u << (dev & 31);
  if (!(attr_done.load(std::memory_order_acquire) & bit)) {
    e = hipFuncSetAttribute((const void*)k17_gemm_kernel<TM, EPI, F32>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            kLds + kTq + 4 * kMaxBiasN);
    if (e != hipSuccess) return e;
    attr_done.fetch_or(bit, std::memory_order_acq_rel);
  }
  hipLaunchKernelGGL((k17_gemm_kernel<TM, EPI, F32>), dim3(grid), dim3(512), lds_bytes, s, prm);
  return hipGetLastError();
}

template <int TM>
hipError_t launch(const K17Params& prm, int grid, hipStream_t s, int epi, int out_f32) {
  if (out_f32) {
    if (epi == kEpiNone) return launch_tm<TM, kEpiNone, true>(prm, grid, s);
    if (epi == kEpiBias) return launch_tm<TM, kEpiBias, true>(prm, grid, s);
    if (epi == kEpiBiasGeluErf) return launch_tm<TM, kEpiBiasGeluErf, true>(prm, grid, s);
    return launch_tm<TM, kEpiBiasGelu, true>(prm, grid, s);
  }
  if (epi == kEpiNone) return launch_tm<TM, kEpiNone, false>(prm, grid, s);
  if (epi == kEpiBias) return launch_tm<TM, kEpiBias, false>(prm, grid, s);
  if (epi == kEpiBiasGeluErfX3) return launch_tm<TM, kEpiBiasGeluErfX3, false>(prm, grid, s);
  return launch_tm<TM, kEpiBiasGelu, false>(prm, grid, s);
}

std::atomic<int> g_k17_last_tm{0};
std::atomic<long long> g_k17_calls{0};

// the dynamic scheduler's claim counters: one {next, done} pair per stream on
// a 128-B line of its own, in the code object's device memory (zero at load;
// every launch leaves them zero again)
constexpr int kSchedSlots = 64;
__device__ int g_k17_sched[kSchedSlots * 32];

struct SchedMap {
  std::mutex mu;
  int* base[32] = {};            // g_k17_sched's address per device
  uintptr_t key[32][kSchedSlots];  // stream handle + 1 per slot (0 = free)
  SchedMap() { std::memset(key, 0, sizeof(key)); }
};
SchedMap& sched_map() {
  static SchedMap m;
  return m;
}

// the counter pair of (device, stream), or null when the slots are used up
// (the launch then runs the static tile list)
int* sched_for(hipStream_t s) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 32) return nullptr;
  SchedMap& m = sched_map();
  std::lock_guard<std::mutex> g(m.mu);
  if (!m.base[dev]) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_k17_sched)) != hipSuccess || !p) return nullptr;
    m.base[dev] = (int*)p;
  }
  const uintptr_t k = (uintptr_t)s + 1;
  for (int i = 0; i < kSchedSlots; ++i)
    if (m.key[dev][i] == k) return m.base[dev] + 32 * i;
  for (int i = 0; i < kSchedSlots; ++i)
    if (!m.key[dev][i]) {
      m.key[dev][i] = k;
      return m.base[dev] + 32 * i;
    }
  return nullptr;
}

}  // namespace

extern "C" {

// K17: C = A . B^T (+ bias) (GELU) with bf16 A [M][lda], B [N][ldb] (K
// contiguous), fp32 bias [N], C bf16 (out_f32 = 0) or fp32 [M][ldc].
// epi: 0 none, 1 bias, 2 bias + GELU (tanh form), 3 bias + GELU (erf form,
// fp32 C only), 4 the erf form as a bf16x3 operand (bf16 C, ldc >= 3N:
// [hi | hi | lo]) (N <= 8188).  N a multiple of 256, K of 32, lda /
// ldb / ldc multiples of 8, 16-B aligned pointers; any M >= 1.
int tcamd_k17_gemm(const void* A, const void* B, const float* bias, void* C, int M, int N, int K, int lda, int ldb,
                   int ldc, int epi, int out_f32, void* stream) {
  if (M <= 0) return hipSuccess;
  if (!A || !B || !C || N <= 0 || N % kTile || K <= 0 || K % kSlabK || epi < 0 || epi > 4) return hipErrorInvalidValue;
  if (epi == 3 && !out_f32) return hipErrorInvalidValue;  // erf GELU: the fp32-parity form only
  if (epi == 4 && (out_f32 || ldc < 3 * N)) return hipErrorInvalidValue;
  if (lda < K || ldb < K || ldc < N || lda % 8 || ldb % 8 || ldc % 8) return hipErrorInvalidValue;
  if (!a16(A) || !a16(B) || !a16(C) || (epi && (!bias || ((uintptr_t)bias & 3) || N > kMaxBiasN)))
    return hipErrorInvalidValue;
  if ((size_t)M * lda >= (1ull << 31) || (size_t)N * ldb >= (1ull << 31) || (size_t)M * ldc >= (1ull << 31))
    return hipErrorInvalidValue;  // 32-bit element offsets in the slab sources
  K17Params prm;
  prm.A = (const uint16_t*)A;
  prm.B = (const uint16_t*)B;
  prm.bias = bias;
  prm.C = C;
  prm.M = M;
  prm.N = N;
  prm.K = K;
  prm.lda = lda;
  prm.ldb = ldb;
  prm.ldc = ldc;
  // tile height: the one whose persistent grid finishes first -- rounds of
  // tiles per CU x tile time (a 192- / 128-row tile costs ~0.9 / ~0.72 of a
  // 256-row one, measured: profiles/r5_k17_gemm.md); TCAMD_K17_TM forces one
  const int ncu = cu_count();
  auto makespan = [&](int tm) {
    const long t = (long)((M + tm - 1) / tm) * (N / kTile);
    return (double)((t + ncu - 1) / ncu) * (tm == 256 ? 1.0 : tm == 192 ? 0.9 : 0.72);
  };
  int tm = (int)tcamd::knob(tcamd::Knob::K17Tm);
  if (tm != 128 && tm != 192 && tm != 256) {
    tm = 256;
    for (int c : {192, 128})
      if (makespan(c) < makespan(tm) * 0.97) tm = c;
  }
  prm.tiles_m = (M + tm - 1) / tm;
  prm.tiles_n = N / kTile;
  const int ntiles = prm.tiles_m * prm.tiles_n;
  const int grid = ntiles <= ncu ? ntiles : ncu / 8 * 8;  // persistent: one workgroup per CU
  g_k17_last_tm = tm;
  g_k17_calls.fetch_add(1, std::memory_order_relaxed);
  hipStream_t s = (hipStream_t)stream;
  // dynamic scheduling when some workgroup runs more than one tile and a
  // tile has the >= 6 slabs the claim-ahead needs (TCAMD_K17_DYN=0: static)
  prm.sched = nullptr;
  if (ntiles > grid && K / kSlabK >= 6 && tcamd::knob(tcamd::Knob::K17Dyn) != 0) prm.sched = sched_for(s);
  if (tm == 128) return launch<128>(prm, grid, s, epi, out_f32);
  if (tm == 192) return launch<192>(prm, grid, s, epi, out_f32);
  return launch<256>(prm, grid, s, epi, out_f32);
}

// tile height of the last tcamd_k17_gemm call (tests, tools)
int tcamd_k17_last_tm() { return g_k17_last_tm; }

// launches so far (tests: which projections a model routed through K17)
long long tcamd_k17_calls() { return g_k17_calls.load(std::memory_order_relaxed); }

}  // extern "C"
