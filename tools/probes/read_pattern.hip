// HBM read-pattern probe for the fp32 DenseNet 1x1 (K8x ws) X stream.
// Same bytes, same per-block tile shape (128 pixel rows x K channels, 32-channel
// K steps, 3 steps of loads in flight per thread), three layouts of X:
//   A  NHWC rows [M][ldx] fp32: a step reads 128 B from each of 128 rows
//      (what x3_conv1x1_ws_kernel does today);
//   B  channel-blocked [ldx/32][M][32] fp32: a step reads one contiguous 16 KB chunk;
//   C  NHWC rows, one block sweeps its tile's rows whole (K = ldx only).
// Build: hipcc --offload-arch=gfx950 -O3 -o read_pattern read_pattern.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

constexpr int PF = 3;

// one block = 256 threads = one 128-row tile, all K steps
template <int MODE>
__global__ void __launch_bounds__(256) probe(const float* __restrict__ x, float* __restrict__ out, int M, int ldx,
                                             int K, int tiles_per_block) {
  const int t = threadIdx.x;
  f32x4 acc = {0, 0, 0, 0};
  const int nst = K / 32;
  for (int tb = 0; tb < tiles_per_block; ++tb) {
    const int tile = blockIdx.x * tiles_per_block + tb;
    const int m0 = tile * 128;
    if (m0 >= M) break;
    const int rot = blockIdx.x % nst;
    for (int s0 = 0; s0 < nst; s0 += PF) {
      f32x4 v[PF][4];
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        int s = s0 + u;
        if (s >= nst) s = nst - 1;
        s += rot;
        if (s >= nst) s -= nst;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float* src;
          if (MODE == 0) {
            const int row = m0 + (t >> 3) + 32 * i;
            src = x + (size_t)row * ldx + 32 * s + 4 * (t & 7);
          } else {
            // [ldx/32][M][32]: rows m0..m0+127 of channel block s are contiguous
            src = x + ((size_t)s * M + m0) * 32 + 4 * t + 1024 * i;
          }
          v[u][i] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src));
        }
      }
#pragma unroll
      for (int u = 0; u < PF; ++u)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc += v[u][i];
    }
  }
  if (acc[0] == 1234.5f) out[blockIdx.x * 256 + t] = acc[1] + acc[2] + acc[3];
}

// D/E: 256 persistent blocks (one per CU, like x3_conv1x1_ws_kernel's producers):
//   D  each block walks a contiguous run of tiles (the ws kernel's assignment);
//   E  tiles dealt round-robin (tile = block + i * grid).
template <int MODE>
__global__ void __launch_bounds__(256) probe_persist(const float* __restrict__ x, float* __restrict__ out, int M,
                                                     int ldx, int K, int tiles) {
  const int t = threadIdx.x;
  f32x4 acc = {0, 0, 0, 0};
  const int nst = K / 32;
  const int per = (tiles + gridDim.x - 1) / gridDim.x;
  const int rot = blockIdx.x % nst;
  for (int i = 0; i < per; ++i) {
    const int tile = MODE == 0 ? blockIdx.x * per + i : blockIdx.x + i * gridDim.x;
    if (tile >= tiles) break;
    const int m0 = tile * 128;
    for (int s0 = 0; s0 < nst; s0 += PF) {
      f32x4 v[PF][4];
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        int s = min(s0 + u, nst - 1) + rot;
        if (s >= nst) s -= nst;
#pragma unroll
        for (int i2 = 0; i2 < 4; ++i2)
          v[u][i2] = __builtin_nontemporal_load(
              reinterpret_cast<const f32x4*>(x + (size_t)(m0 + (t >> 3) + 32 * i2) * ldx + 32 * s + 4 * (t & 7)));
      }
#pragma unroll
      for (int u = 0; u < PF; ++u)
#pragma unroll
        for (int i2 = 0; i2 < 4; ++i2) acc += v[u][i2];
    }
  }
  if (acc[0] == 1234.5f) out[blockIdx.x * 256 + t] = acc[1] + acc[2] + acc[3];
}

// C: whole rows, contiguous sweep of the tile (K == ldx)
__global__ void __launch_bounds__(256) probe_sweep(const float* __restrict__ x, float* __restrict__ out, int M,
                                                   int ldx, int K, int tiles_per_block) {
  const int t = threadIdx.x;
  f32x4 acc = {0, 0, 0, 0};
  const size_t per_tile = (size_t)128 * ldx;  // floats
  const int nst = K / 32;
  for (int tb = 0; tb < tiles_per_block; ++tb) {
    const int tile = blockIdx.x * tiles_per_block + tb;
    if (tile * 128 >= M) break;
    const float* base = x + tile * per_tile;
    for (int s0 = 0; s0 < nst; s0 += PF) {
      f32x4 v[PF][4];
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        int s = min(s0 + u, nst - 1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
          v[u][i] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(base + (size_t)s * 4096 + 4 * t + 1024 * i));
      }
#pragma unroll
      for (int u = 0; u < PF; ++u)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc += v[u][i];
    }
  }
  if (acc[0] == 1234.5f) out[blockIdx.x * 256 + t] = acc[1] + acc[2] + acc[3];
}

int main(int argc, char** argv) {
  const int M = 128 * 56 * 56;
  const int ldx = 256;
  const size_t bytes = (size_t)M * ldx * 4;
  float* x;
  float* out;
  CK(hipMalloc(&x, bytes));
  CK(hipMemset(x, 0, bytes));
  const int tiles = M / 128;
  CK(hipMalloc(&out, (size_t)tiles * 256 * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int Ks[] = {256};
  const int tpbs[] = {1, 6};
  for (int K : Ks)
    for (int tpb : tpbs)
      for (int mode = 0; mode < 3; ++mode) {
        if (mode == 2 && K != ldx) continue;
        const int grid = (tiles + tpb - 1) / tpb;
        auto launch = [&]() {
          if (mode == 0) probe<0><<<grid, 256>>>(x, out, M, ldx, K, tpb);
          else if (mode == 1) probe<1><<<grid, 256>>>(x, out, M, ldx, K, tpb);
          else probe_sweep<<<grid, 256>>>(x, out, M, ldx, K, tpb);
        };
        for (int w = 0; w < 3; ++w) launch();
        CK(hipDeviceSynchronize());
        const int reps = 20;
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = 1000.0 * ms / reps;
        const double rd = (double)M * K * 4;
        printf("mode %c K %3d tiles/block %d grid %5d: %7.1f us  %.2f TB/s\n", "ABC"[mode], K, tpb, grid, us,
               rd / us / 1e6);
        fflush(stdout);
      }
  for (int K : {128, 224, 256})
    for (int grid : {256, 512, 1024})
      for (int mode = 0; mode < 2; ++mode) {
        auto launch = [&]() {
          if (mode == 0) probe_persist<0><<<grid, 256>>>(x, out, M, ldx, K, tiles);
          else probe_persist<1><<<grid, 256>>>(x, out, M, ldx, K, tiles);
        };
        for (int w = 0; w < 3; ++w) launch();
        CK(hipDeviceSynchronize());
        const int reps = 20;
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = 1000.0 * ms / reps;
        printf("persistent %s K %3d grid %4d: %7.1f us  %.2f TB/s\n", mode ? "round-robin" : "contiguous ", K, grid,
               us, (double)M * K * 4 / us / 1e6);
        fflush(stdout);
      }
  CK(hipFree(x));
  CK(hipFree(out));
  return 0;
}
