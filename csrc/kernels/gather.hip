// K7 gather_concat / scatter — one launch for a batch of byte-range copies
// (SURVEY.md §2.9 K7).  Replaces the reference's k x cudaMemcpyAsync + sync
// in set_shared_memory_region (tritonclient/utils/cuda_shared_memory/
// __init__.py:199-231) and drives the server's output scatter into per-request
// device shm regions.
//
// Up to 32 {src, dst, bytes} descriptors travel by value in the kernel
// arguments (no descriptor upload).  blockIdx.y selects the descriptor;
// blocks of a descriptor stride over it in 16-byte (dwordx4) units when src,
// dst and size are 16-B aligned, else in bytes.

#include "kernels/common.h"

using namespace tcamd;

namespace {

constexpr int kMaxDesc = 32;

struct CopyBatch {
  const uint8_t* src[kMaxDesc];
  uint8_t* dst[kMaxDesc];
  uint64_t bytes[kMaxDesc];
};

__global__ void __launch_bounds__(kBlock) batched_copy(CopyBatch b) {
  const int d = blockIdx.y;
  const uint8_t* __restrict__ src = b.src[d];
  uint8_t* __restrict__ dst = b.dst[d];
  const uint64_t n = b.bytes[d];
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  if ((((uintptr_t)src | (uintptr_t)dst) & 15) == 0) {
    const uint64_t nv = n / 16;
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    uint4* d4 = reinterpret_cast<uint4*>(dst);
    uint64_t i = tid;
    // two independent 16-B loads in flight per lane
    for (; i + stride < nv; i += 2 * stride) {
      uint4 a = s4[i], c = s4[i + stride];
      d4[i] = a;
      d4[i + stride] = c;
    }
    for (; i < nv; i += stride) d4[i] = s4[i];
    for (uint64_t j = nv * 16 + tid; j < n; j += stride) dst[j] = src[j];
  } else {
    for (uint64_t j = tid; j < n; j += stride) dst[j] = src[j];
  }
}

}  // namespace

// srcs/dsts/bytes: host arrays of `count` entries (device or host-mapped
// pointers).  Any count is accepted; launches are chunked by 32.
extern "C" int tcamd_batched_copy(const void* const* srcs, void* const* dsts, const uint64_t* bytes,
                                  int count, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  for (int base = 0; base < count; base += kMaxDesc) {
    CopyBatch b;
    int cnt = count - base < kMaxDesc ? count - base : kMaxDesc;
    uint64_t maxb = 0;
    for (int i = 0; i < cnt; ++i) {
      b.src[i] = (const uint8_t*)srcs[base + i];
      b.dst[i] = (uint8_t*)dsts[base + i];
      b.bytes[i] = bytes[base + i];
      if (b.bytes[i] > maxb) maxb = b.bytes[i];
    }
    if (maxb == 0) continue;
    // enough blocks per descriptor to cover it once in 32-B-per-lane steps,
    // capped so the whole launch stays around 2K blocks
    uint64_t per = (maxb + (uint64_t)kBlock * 32 - 1) / ((uint64_t)kBlock * 32);
    uint64_t cap = (uint64_t)kMaxGrid / cnt;
    if (cap < 1) cap = 1;
    if (per > cap) per = cap;
    if (per < 1) per = 1;
    hipLaunchKernelGGL(batched_copy, dim3((unsigned)per, cnt), dim3(kBlock), 0, s, b);
    int rc = hipGetLastError();
    if (rc != hipSuccess) return rc;
  }
  return hipSuccess;
}
