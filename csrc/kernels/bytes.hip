// K2 pack_bytes / K3 unpack_bytes — BYTES tensor (de)serialisation on device
// (SURVEY.md §2.9 K2/K3).  Wire format (reference tritonclient/utils/
// __init__.py:193-276, src/c++/library/common.cc:168-183): each element is a
// little-endian u32 length followed by that many bytes, row-major.
//
// pack: 3 launches
//   1. per-block exclusive scan of the u32 lengths in LDS (1024 per block:
//      256 threads x 4, Hillis-Steele over wave partials)
//   2. single-block scan of the block totals
//   3. scatter: element i goes to out + in_off[i] + 4*i (prefix + payload)
// unpack (index): one workgroup walks the length chain; the buffer is staged
//   through a 32 KiB LDS window loaded cooperatively with 16-B loads, so each
//   hop costs an LDS read instead of a dependent HBM round trip.  The walk is
//   inherently sequential — the index lets every later consumer run in
//   parallel.

#include "kernels/common.h"

using namespace tcamd;

namespace {

constexpr int kPer = 4;                  // lengths per thread
constexpr int kSpan = kBlock * kPer;     // lengths per block

__device__ __forceinline__ uint64_t block_exclusive_scan(uint64_t v, uint64_t* lds_warp, uint64_t* total) {
  // wave-level inclusive scan (64 lanes)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint64_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint64_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) lds_warp[wid] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t run = 0;
    for (int w = 0; w < kBlock / 64; ++w) {
      uint64_t t = lds_warp[w];
      lds_warp[w] = run;
      run += t;
    }
    lds_warp[kBlock / 64] = run;
  }
  __syncthreads();
  uint64_t excl = x - v + lds_warp[wid];
  *total = lds_warp[kBlock / 64];
  return excl;
}

__global__ void __launch_bounds__(kBlock) scan_lengths(const uint32_t* __restrict__ lens, uint64_t n,
                                                       uint64_t* __restrict__ offs,
                                                       uint64_t* __restrict__ block_sums) {
  __shared__ uint64_t lds_warp[kBlock / 64 + 1];
  const uint64_t base = (uint64_t)blockIdx.x * kSpan + (uint64_t)threadIdx.x * kPer;
  uint64_t local[kPer];
  uint64_t sum = 0;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    uint64_t i = base + k;
    local[k] = (i < n) ? lens[i] : 0;
    sum += local[k];
  }
  uint64_t total;
  uint64_t excl = block_exclusive_scan(sum, lds_warp, &total);
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    uint64_t i = base + k;
    if (i < n) offs[i] = excl;
    excl += local[k];
  }
  if (threadIdx.x == 0) block_sums[blockIdx.x] = total;
}

__global__ void __launch_bounds__(kBlock) scan_block_sums(uint64_t* __restrict__ block_sums, uint64_t nb) {
  __shared__ uint64_t lds_warp[kBlock / 64 + 1];
  uint64_t carry = 0;
  for (uint64_t base = 0; base < nb; base += kBlock) {
    uint64_t i = base + threadIdx.x;
    uint64_t v = i < nb ? block_sums[i] : 0;
    uint64_t total;
    uint64_t excl = block_exclusive_scan(v, lds_warp, &total);
    if (i < nb) block_sums[i] = excl + carry;
    carry += total;
    __syncthreads();
  }
}

__global__ void __launch_bounds__(kBlock) scatter_elements(const uint8_t* __restrict__ data,
                                                           const uint32_t* __restrict__ lens,
                                                           const uint64_t* __restrict__ offs,
                                                           const uint64_t* __restrict__ block_sums,
                                                           uint64_t n, uint8_t* __restrict__ out) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t in_off = offs[i] + block_sums[i / kSpan];
    const uint64_t out_off = in_off + 4 * i;
    const uint32_t L = lens[i];
    out[out_off + 0] = (uint8_t)(L);
    out[out_off + 1] = (uint8_t)(L >> 8);
    out[out_off + 2] = (uint8_t)(L >> 16);
    out[out_off + 3] = (uint8_t)(L >> 24);
    const uint8_t* s = data + in_off;
    uint8_t* d = out + out_off + 4;
    for (uint32_t j = 0; j < L; ++j) d[j] = s[j];
  }
}

constexpr int kWin = 32768;  // LDS window (bytes)

__global__ void __launch_bounds__(kBlock) index_bytes(const uint8_t* __restrict__ buf, uint64_t nbytes,
                                                      uint64_t n_expected, uint64_t* __restrict__ offs,
                                                      uint32_t* __restrict__ lens, int* __restrict__ status) {
  __shared__ __attribute__((aligned(16))) uint8_t win[kWin + 16];
  __shared__ uint64_t s_pos, s_count;
  __shared__ int s_err;
  if (threadIdx.x == 0) {
    s_pos = 0;
    s_count = 0;
    s_err = 0;
  }
  __syncthreads();
  while (true) {
    const uint64_t pos = s_pos;
    if (s_err || s_count >= n_expected || pos >= nbytes) break;
    // window aligned down to 16 B; cooperative dwordx4 loads
    const uint64_t wbase = pos & ~(uint64_t)15;
    const uint64_t wlen = (nbytes - wbase) < (uint64_t)kWin ? (nbytes - wbase) : (uint64_t)kWin;
    const uint64_t nvec = wlen / 16;
    const bool aligned = (((uintptr_t)buf) & 15) == 0;
    if (aligned) {
      for (uint64_t v = threadIdx.x; v < nvec; v += blockDim.x)
        reinterpret_cast<uint4*>(win)[v] = reinterpret_cast<const uint4*>(buf + wbase)[v];
      for (uint64_t b = nvec * 16 + threadIdx.x; b < wlen; b += blockDim.x) win[b] = buf[wbase + b];
    } else {
      for (uint64_t b = threadIdx.x; b < wlen; b += blockDim.x) win[b] = buf[wbase + b];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint64_t p = pos, cnt = s_count;
      const uint64_t wend = wbase + wlen;
      while (cnt < n_expected && p < nbytes) {
        if (p + 4 > wend) {
          if (wend >= nbytes) s_err = 1;  // truncated length prefix
          break;                          // else: reload window at p
        }
        const uint8_t* q = win + (p - wbase);
        const uint32_t L = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) |
                           ((uint32_t)q[3] << 24);
        if (p + 4 + (uint64_t)L > nbytes) {
          s_err = 1;
          break;
        }
        offs[cnt] = p + 4;
        lens[cnt] = L;
        ++cnt;
        p += 4 + (uint64_t)L;
      }
      s_pos = p;
      s_count = cnt;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    status[0] = s_err ? -1 : (int)(s_count == n_expected ? 0 : 1);
    reinterpret_cast<uint64_t*>(status + 2)[0] = s_count;
  }
}

}  // namespace

// workspace must hold n*8 + ceil(n/1024)*8 bytes (see tcamd_pack_bytes_workspace).
extern "C" uint64_t tcamd_pack_bytes_workspace(uint64_t n) {
  return n * 8 + ((n + kSpan - 1) / kSpan) * 8 + 16;
}

extern "C" int tcamd_pack_bytes(const void* data, const uint32_t* lens, uint64_t n, void* out,
                                void* workspace, void* stream) {
  if (n == 0) return hipSuccess;
  hipStream_t s = (hipStream_t)stream;
  uint64_t* offs = (uint64_t*)workspace;
  uint64_t nb = (n + kSpan - 1) / kSpan;
  uint64_t* bsum = offs + n;
  hipLaunchKernelGGL(scan_lengths, dim3((unsigned)nb), dim3(kBlock), 0, s, lens, n, offs, bsum);
  hipLaunchKernelGGL(scan_block_sums, dim3(1), dim3(kBlock), 0, s, bsum, nb);
  hipLaunchKernelGGL(scatter_elements, dim3(grid_for(n)), dim3(kBlock), 0, s, (const uint8_t*)data, lens,
                     offs, bsum, n, (uint8_t*)out);
  return hipGetLastError();
}

// status: device int[4]: [0] = 0 ok / 1 fewer elements than expected / -1
// malformed; [2..3] = u64 element count found.
extern "C" int tcamd_index_bytes(const void* buf, uint64_t nbytes, uint64_t n_expected, uint64_t* offs,
                                 uint32_t* lens, int* status, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(index_bytes, dim3(1), dim3(kBlock), 0, s, (const uint8_t*)buf, nbytes, n_expected, offs,
                     lens, status);
  return hipGetLastError();
}
