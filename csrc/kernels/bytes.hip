// K2 pack_bytes / K3 unpack_bytes — BYTES tensor (de)serialisation on device
// (SURVEY.md §2.9 K2/K3).  Wire format (reference tritonclient/utils/
// __init__.py:193-276, src/c++/library/common.cc:168-183): each element is a
// little-endian u32 length followed by that many bytes, row-major.
//
// pack: 3 launches
//   1. per-block exclusive scan of the u32 lengths in LDS (1024 per block:
//      256 threads x 4, Hillis-Steele over wave partials)
//   2. single-block scan of the block totals (+ the grand total)
//   3. OUTPUT-centric emit: every thread builds one 16-B chunk of the packed
//      stream and writes it with one dwordx4 store (fully coalesced whatever
//      the length distribution: one long string is spread over all lanes,
//      many short ones are packed by one lane).  The owner element of a chunk
//      is found by a two-level binary search over the element start offsets
//      (block level, then inside the 1024-element block; neighbouring lanes
//      search the same lines), then the chunk walks forward across element
//      boundaries (length prefix bytes, then payload bytes).
// unpack (index), by size:
//   * <= 64 KiB: one workgroup walks the length chain through a 32 KiB LDS
//     window (each hop an LDS read, not a dependent HBM round trip);
//   * larger: a parallel 3-phase walk over 8 KiB blocks —
//     1. every byte position p of a block is a candidate element start:
//        next(p) = p + 4 + len(p); pointer DOUBLING in LDS (11 rounds) gives,
//        for every p, the first chain position at or past the block end and
//        the number of elements started on the way (exit/count tables);
//     2. chaining the blocks: entry(b+1) = exit(entry(b)), element base
//        index += count.  Fast path (every element the chain meets is at most
//        kR - 4 bytes): compose 32-block superblocks over the first kR entry
//        offsets in parallel, one lane hops superblocks, one lane per
//        superblock expands its blocks.  Otherwise one lane hops blocks
//        through the full exit table (one dependent HBM hop per 8 KiB);
//     3. every block re-walks from its entry in LDS and writes its elements'
//        offsets/lengths at base(b) + k.

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
  if (threadIdx.x == 0) block_sums[nb] = carry;  // total payload bytes
}

// Packed-stream start of element i: payload bytes before it + 4 per prefix.
__device__ __forceinline__ uint64_t in_start(const uint64_t* offs, const uint64_t* bsum, uint64_t i) {
  return offs[i] + bsum[i / kSpan];
}

__global__ void __launch_bounds__(kBlock) emit_packed(const uint8_t* __restrict__ data,
                                                      const uint32_t* __restrict__ lens,
                                                      const uint64_t* __restrict__ offs,
                                                      const uint64_t* __restrict__ bsum, uint64_t n, uint64_t nb,
                                                      uint8_t* __restrict__ out) {
  const uint64_t total = bsum[nb] + 4 * n;
  const uint64_t nchunks = (total + 15) / 16;
  const bool out_aligned = (((uintptr_t)out) & 15) == 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nchunks; c += stride) {
    const uint64_t pos0 = c * 16;
    // block level: last block whose first element starts at or before pos0
    uint64_t lo = 0, hi = nb;  // invariant: ostart(first of lo) <= pos0
    while (hi - lo > 1) {
      const uint64_t mid = (lo + hi) >> 1;
      if (bsum[mid] + 4 * mid * (uint64_t)kSpan <= pos0) lo = mid;
      else hi = mid;
    }
    uint64_t elo = lo * kSpan, ehi = (lo + 1) * (uint64_t)kSpan < n ? (lo + 1) * (uint64_t)kSpan : n;
    while (ehi - elo > 1) {
      const uint64_t mid = (elo + ehi) >> 1;
      if (in_start(offs, bsum, mid) + 4 * mid <= pos0) elo = mid;
      else ehi = mid;
    }
    uint64_t e = elo;
    uint64_t es = in_start(offs, bsum, e);        // payload start of e in `data`
    uint64_t os = es + 4 * e;                     // packed start of e
    uint32_t L = lens[e];
    uint64_t oe = os + 4 + L;                     // packed end of e
    union {
      uint4 v;
      uint8_t b[16];
    } chunk;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint64_t pos = pos0 + k;
      while (pos >= oe && e + 1 < n) {  // cross into the next element(s)
        ++e;
        es = in_start(offs, bsum, e);
        os = es + 4 * e;
        L = lens[e];
        oe = os + 4 + L;
      }
      const uint64_t local = pos - os;
      uint8_t byte = 0;
      if (pos < total) byte = local < 4 ? (uint8_t)(L >> (8 * local)) : data[es + (local - 4)];
      chunk.b[k] = byte;
    }
    if (out_aligned && pos0 + 16 <= total) {
      *reinterpret_cast<uint4*>(out + pos0) = chunk.v;
    } else {
      for (int k = 0; k < 16 && pos0 + k < total; ++k) out[pos0 + k] = chunk.b[k];
    }
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

// ---- K3 large inputs: parallel 3-phase walk over 8 KiB blocks --------------
constexpr int kIdxB = 8192;                 // bytes per block
constexpr int kIdxPer = kIdxB / kBlock;     // positions per thread (32)
constexpr uint64_t kBad = ~(uint64_t)0;     // malformed element on the chain
constexpr uint64_t kNone = ~(uint64_t)0 - 1;  // block not entered / past n_expected
constexpr int kR = kBlock;                    // compact-table entry offsets per block
constexpr int kS = 32;                        // blocks per superblock (fast chain)
constexpr uint32_t kTBad = 0xFFFFFFFFu;       // compact-table sentinels: malformed element,
constexpr uint32_t kTEnd = 0xFFFFFFFEu;       //   chain ended (past the data),
constexpr uint32_t kTFar = 0xFFFFFFFDu;       //   exit beyond the next block's first kR bytes

__device__ __forceinline__ void stage_block(const uint8_t* __restrict__ buf, uint64_t nbytes, uint64_t b0,
                                            uint8_t* win) {
  // kIdxB + 16 bytes (a length prefix may straddle the block end); zero past nbytes
  const bool aligned = ((((uintptr_t)buf) + b0) & 15) == 0;
  for (int v = threadIdx.x; v < (kIdxB + 16) / 16; v += blockDim.x) {
    const uint64_t g = b0 + 16 * (uint64_t)v;
    if (aligned && g + 16 <= nbytes) {
      reinterpret_cast<uint4*>(win)[v] = *reinterpret_cast<const uint4*>(buf + g);
    } else {
      for (int k = 0; k < 16; ++k) win[16 * v + k] = (g + k < nbytes) ? buf[g + k] : 0;
    }
  }
}

__device__ __forceinline__ uint32_t le32(const uint8_t* q) {
  return (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
}

// Phase 1: exit/count of every candidate start position of one block.
// FULL = false: the compact tables of the fast chain (exit/count of the first
// kR positions, one sequential walk per position through the LDS window).
// FULL = true (run only when the fast chain gave up, *fast == 0): pointer
// doubling over every position and the whole exit/count tables for
// idx_chain — 10 bytes written per input byte, which the fast path skips.
template <bool FULL>
__global__ void __launch_bounds__(kBlock) idx_blocks(const uint8_t* __restrict__ buf, uint64_t nbytes,
                                                     uint64_t* __restrict__ exit_pos,
                                                     uint16_t* __restrict__ count, uint32_t* __restrict__ tab,
                                                     uint16_t* __restrict__ tcnt, const int* __restrict__ fast) {
  if (FULL && *fast) return;  // uniform per launch
  __shared__ __attribute__((aligned(16))) uint8_t win[kIdxB + 16];
  const uint64_t b0 = (uint64_t)blockIdx.x * kIdxB;
  const uint64_t bend = b0 + kIdxB;
  stage_block(buf, nbytes, b0, win);
  __syncthreads();
  if constexpr (!FULL) {
    // the fast chain needs the exits of the first kR positions only: thread e
    // walks the chain from b0 + e through the LDS window (no doubling tables)
    const int e = threadIdx.x;
    uint64_t p = b0 + e;
    uint32_t c = 0, v;
    if (p >= nbytes) {
      v = kTEnd;
    } else {
      for (;;) {
        if (p + 4 > nbytes) {
          v = kTBad;
          break;
        }
        const uint64_t x = p + 4 + (uint64_t)le32(win + (p - b0));
        if (x > nbytes) {
          v = kTBad;
          break;
        }
        ++c;
        p = x;
        if (p >= bend) {
          v = p - bend < (uint64_t)kR ? (uint32_t)(p - bend) : kTFar;
          break;
        }
        if (p >= nbytes) {
          v = kTEnd;
          break;
        }
      }
    }
    tab[(uint64_t)blockIdx.x * kR + e] = v;
    tcnt[(uint64_t)blockIdx.x * kR + e] = (uint16_t)c;
    return;
  }
  __shared__ uint64_t nxt[kIdxB];
  __shared__ uint16_t cnt[kIdxB];
  // interleaved ownership (q = threadIdx.x + k*256): conflict-free LDS rows
#pragma unroll 4
  for (int k = 0; k < kIdxPer; ++k) {
    const int q = threadIdx.x + k * kBlock;
    const uint64_t p = b0 + q;
    uint64_t x = kBad;
    if (p + 4 <= nbytes) {
      const uint64_t e = p + 4 + (uint64_t)le32(win + q);
      if (e <= nbytes) x = e;
    }
    nxt[q] = (p < nbytes) ? x : kNone;
    cnt[q] = (x == kBad || p >= nbytes) ? 0 : 1;
  }
  __syncthreads();
  // pointer doubling: 2^11 = 2048 >= kIdxB/4 hops per block
  for (int round = 0; round < 11; ++round) {
    uint64_t nx[kIdxPer];
    uint16_t nc[kIdxPer];
#pragma unroll
    for (int k = 0; k < kIdxPer; ++k) {
      const int q = threadIdx.x + k * kBlock;
      uint64_t x = nxt[q];
      uint16_t c = cnt[q];
      if (x != kBad && x != kNone && x < bend) {
        const int j = (int)(x - b0);
        c = (uint16_t)(c + cnt[j]);
        x = nxt[j];
      }
      nx[k] = x;
      nc[k] = c;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kIdxPer; ++k) {
      const int q = threadIdx.x + k * kBlock;
      nxt[q] = nx[k];
      cnt[q] = nc[k];
    }
    __syncthreads();
  }
#pragma unroll 4
  for (int k = 0; k < kIdxPer; ++k) {
    const int q = threadIdx.x + k * kBlock;
    if (b0 + q < nbytes) {
      exit_pos[b0 + q] = nxt[q];
      count[b0 + q] = cnt[q];
    }
  }
}

// Phase 2 (fast path), in three short steps instead of one dependent HBM hop
// per 8 KiB block:
//   a. compose: workgroup sb follows all kR entry offsets through its kS
//      blocks' compact tables in LDS -> superblock exit offset + count;
//   b. chain: one lane hops superblocks (kS blocks per hop);
//   c. expand: one lane per superblock re-walks its kS blocks from the
//      superblock entry and writes every block's entry / base.
// A chain that meets an element longer than the compact tables cover (kTFar
// while elements are still wanted) clears *fast and idx_chain runs instead.
__global__ void __launch_bounds__(kBlock) idx_sb_compose(const uint32_t* __restrict__ tab,
                                                         const uint16_t* __restrict__ tcnt, uint64_t nblk,
                                                         uint32_t* __restrict__ g, uint32_t* __restrict__ gc) {
  __shared__ uint32_t st[kS][kR];
  __shared__ uint16_t sc[kS][kR];
  const uint64_t blk0 = (uint64_t)blockIdx.x * kS;
  const int nb = (int)min((uint64_t)kS, nblk - blk0);
  for (int i = threadIdx.x; i < nb * kR; i += kBlock) {
    st[i / kR][i % kR] = tab[blk0 * kR + i];
    sc[i / kR][i % kR] = tcnt[blk0 * kR + i];
  }
  __syncthreads();
  uint32_t v = threadIdx.x, c = 0;
  for (int k = 0; k < nb && v < (uint32_t)kR; ++k) {
    c += sc[k][v];
    v = st[k][v];
  }
  g[(uint64_t)blockIdx.x * kR + threadIdx.x] = v;
  gc[(uint64_t)blockIdx.x * kR + threadIdx.x] = c;
}

__global__ void idx_sb_chain(const uint32_t* __restrict__ g, const uint32_t* __restrict__ gc, uint64_t nsb,
                             uint64_t n_expected, uint32_t* __restrict__ sb_entry, uint64_t* __restrict__ sb_base,
                             int* __restrict__ fast, int* __restrict__ status) {
  if (threadIdx.x != 0) return;
  uint32_t v = 0;
  uint64_t idx = 0;
  for (uint64_t sb = 0; sb < nsb; ++sb) {
    sb_entry[sb] = v;
    sb_base[sb] = idx;
    if (v < (uint32_t)kR && idx < n_expected) {
      idx += gc[sb * kR + v];
      v = g[sb * kR + v];
    }
  }
  if (v == kTFar && idx < n_expected) {  // an element longer than the tables cover is still wanted
    *fast = 0;
    return;
  }
  *fast = 1;
  const bool err = v == kTBad && idx < n_expected;
  status[0] = err ? -1 : (idx >= n_expected ? 0 : 1);
  reinterpret_cast<uint64_t*>(status + 2)[0] = idx < n_expected ? idx : n_expected;
}

__global__ void idx_sb_expand(const uint32_t* __restrict__ tab, const uint16_t* __restrict__ tcnt, uint64_t nbytes,
                              uint64_t nblk, uint64_t n_expected, const uint32_t* __restrict__ sb_entry,
                              const uint64_t* __restrict__ sb_base, const int* __restrict__ fast,
                              uint64_t* __restrict__ entry, uint64_t* __restrict__ base) {
  if (threadIdx.x != 0 || !*fast) return;
  const uint64_t blk0 = (uint64_t)blockIdx.x * kS;
  const uint64_t bl_end = min(blk0 + kS, nblk);
  uint32_t v = sb_entry[blockIdx.x];
  uint64_t idx = sb_base[blockIdx.x];
  for (uint64_t b = blk0; b < bl_end; ++b) {
    const uint64_t p = b * (uint64_t)kIdxB + v;
    if (v >= (uint32_t)kR || idx >= n_expected || p >= nbytes) {
      entry[b] = kNone;
      continue;
    }
    entry[b] = p;
    base[b] = idx;
    idx += tcnt[b * kR + v];
    v = tab[b * kR + v];
  }
}

// Phase 2: one lane chains the blocks.  entry[b] = first chain position in
// block b (kNone if the chain skips it or is done), base[b] = its element index.
__global__ void idx_chain(const uint64_t* __restrict__ exit_pos, const uint16_t* __restrict__ count,
                          uint64_t nbytes, uint64_t nblk, uint64_t n_expected, uint64_t* __restrict__ entry,
                          uint64_t* __restrict__ base, int* __restrict__ status, const int* __restrict__ fast) {
  if (threadIdx.x != 0 || *fast) return;  // the superblock chain already did it
  uint64_t p = 0, idx = 0;
  int err = 0;
  for (uint64_t b = 0; b < nblk; ++b) {
    const uint64_t bend = (b + 1) * (uint64_t)kIdxB;
    if (err || idx >= n_expected || p >= nbytes || p >= bend) {
      entry[b] = kNone;
      continue;
    }
    entry[b] = p;
    base[b] = idx;
    const uint64_t x = exit_pos[p];
    idx += count[p];
    if (x == kBad) {
      if (idx < n_expected) err = 1;  // the malformed element is one the caller asked for
      p = nbytes;
    } else {
      p = x;
    }
  }
  status[0] = err ? -1 : (idx >= n_expected ? 0 : 1);
  reinterpret_cast<uint64_t*>(status + 2)[0] = idx < n_expected ? idx : n_expected;
}

// Phase 3: each entered block re-walks its elements from the entry in LDS.
__global__ void __launch_bounds__(kBlock) idx_emit(const uint8_t* __restrict__ buf, uint64_t nbytes,
                                                   const uint64_t* __restrict__ entry,
                                                   const uint64_t* __restrict__ base, uint64_t n_expected,
                                                   uint64_t* __restrict__ offs, uint32_t* __restrict__ lens) {
  __shared__ __attribute__((aligned(16))) uint8_t win[kIdxB + 16];
  const uint64_t p0 = entry[blockIdx.x];
  if (p0 == kNone) return;  // uniform per block
  const uint64_t b0 = (uint64_t)blockIdx.x * kIdxB, bend = b0 + kIdxB;
  stage_block(buf, nbytes, b0, win);
  __syncthreads();
  if (threadIdx.x != 0) return;
  uint64_t p = p0, idx = base[blockIdx.x];
  while (p < bend && p + 4 <= nbytes && idx < n_expected) {
    const uint32_t L = le32(win + (p - b0));
    if (p + 4 + (uint64_t)L > nbytes) break;  // reported by phase 2
    offs[idx] = p + 4;
    lens[idx] = L;
    ++idx;
    p += 4 + (uint64_t)L;
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
  hipLaunchKernelGGL(emit_packed, dim3(grid_for(n < 4096 ? 4096 : n)), dim3(kBlock), 0, s,
                     (const uint8_t*)data, lens, offs, bsum, n, nb, (uint8_t*)out);
  return hipGetLastError();
}

// status: device int[4]: [0] = 0 ok / 1 fewer elements than expected / -1
// malformed; [2..3] = u64 element count found.
extern "C" int tcamd_index_bytes(const void* buf, uint64_t nbytes, uint64_t n_expected, uint64_t* offs,
                                 uint32_t* lens, int* status, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (nbytes <= 65536 || n_expected < 2048) {
    hipLaunchKernelGGL(index_bytes, dim3(1), dim3(kBlock), 0, s, (const uint8_t*)buf, nbytes, n_expected, offs,
                       lens, status);
    return hipGetLastError();
  }
  // parallel path: stream-ordered scratch (exit u64 + count u16 per byte, entry/base per block)
  const uint64_t nblk = (nbytes + kIdxB - 1) / kIdxB;
  const uint64_t nsb = (nblk + kS - 1) / kS;
  void* ws = nullptr;
  const size_t wsb = nbytes * 8 + nbytes * 2 + 16 + nblk * 16 + nblk * kR * 6 + nsb * kR * 8 + nsb * 12 + 64;
  hipError_t e = hipMallocAsync(&ws, wsb, s);
  if (e != hipSuccess) return e;
  uint64_t* exit_pos = (uint64_t*)ws;
  uint16_t* count = (uint16_t*)(exit_pos + nbytes);
  uint64_t* entry = (uint64_t*)(((uintptr_t)(count + nbytes) + 15) & ~(uintptr_t)15);
  uint64_t* base = entry + nblk;
  uint64_t* sb_base = base + nblk;
  uint32_t* tab = (uint32_t*)(sb_base + nsb);
  uint32_t* g = tab + nblk * kR;
  uint32_t* gc = g + nsb * kR;
  uint32_t* sb_entry = gc + nsb * kR;
  int* fast = (int*)(sb_entry + nsb);
  uint16_t* tcnt = (uint16_t*)(fast + 4);
  hipLaunchKernelGGL(idx_blocks<false>, dim3((unsigned)nblk), dim3(kBlock), 0, s, (const uint8_t*)buf, nbytes,
                     exit_pos, count, tab, tcnt, fast);
  hipLaunchKernelGGL(idx_sb_compose, dim3((unsigned)nsb), dim3(kBlock), 0, s, tab, tcnt, nblk, g, gc);
  hipLaunchKernelGGL(idx_sb_chain, dim3(1), dim3(64), 0, s, g, gc, nsb, n_expected, sb_entry, sb_base, fast, status);
  hipLaunchKernelGGL(idx_sb_expand, dim3((unsigned)nsb), dim3(64), 0, s, tab, tcnt, nbytes, nblk, n_expected, sb_entry,
                     sb_base, fast, entry, base);
  hipLaunchKernelGGL(idx_blocks<true>, dim3((unsigned)nblk), dim3(kBlock), 0, s, (const uint8_t*)buf, nbytes,
                     exit_pos, count, tab, tcnt, fast);
  hipLaunchKernelGGL(idx_chain, dim3(1), dim3(64), 0, s, exit_pos, count, nbytes, nblk, n_expected, entry, base,
                     status, fast);
  hipLaunchKernelGGL(idx_emit, dim3((unsigned)nblk), dim3(kBlock), 0, s, (const uint8_t*)buf, nbytes, entry, base,
                     n_expected, offs, lens);
  e = hipGetLastError();
  hipError_t f = hipFreeAsync(ws, s);
  return e != hipSuccess ? e : f;
}
