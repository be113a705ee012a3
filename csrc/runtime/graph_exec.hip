// Native batch executor for pointer-table graph models (the served
// densenet_onnx engines): the per-batch dispatch of tcserve runs here, in
// C++, with no Python and no GIL on the request path.
//
// A pointer-table model reads each image straight from its request's buffer
// through a device table of per-row pointers (models/densenet_fp32.py
// forward_ptrs), so one batch is:
//
//   host: build the row-pointer table (device shm rows point into the
//         client's region; in-band / system-shm rows are staged through
//         pinned memory and one H2D)
//   stream: H2D table -> hipGraphLaunch(bucket) -> K7 batched_copy of each
//           request's logits into its device-shm output region, one D2H for
//           host outputs -> event; the worker thread waits on that event and
//           copies host outputs into the request buffers.
//
// tcserve (csrc/cpp/server) calls tcamd_pgx_execute as the model's
// tcserve_exec_fn with `user` = the executor; worker thread i always passes
// instance i, and each instance owns its stream, graphs and staging buffers.
// A per-instance mutex also admits the Python scheduler's requests for the
// same model (triton_client_amd/server/gpu_models.py), which call the same
// function through ctypes.
//
// Host-side timing (CLOCK_MONOTONIC) is accumulated per phase so the server
// can account for every microsecond between "batch leaves the queue" and
// "responses encoded": tcamd_pgx_stats.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <time.h>

#include <atomic>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "cpp/server/tcserve.h"

extern "C" int tcamd_batched_copy(const void* const* srcs, void* const* dsts, const uint64_t* bytes, int count,
                                  void* stream);

namespace {

uint64_t MonoNs()
{
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<uint64_t>(ts.tv_sec) * 1000000000ull + static_cast<uint64_t>(ts.tv_nsec);
}

struct Instance {
  std::mutex mu;
  bool ready = false;
  hipStream_t stream = nullptr;
  std::vector<hipGraphExec_t> execs;  // one per bucket
  uint64_t* tbl_host = nullptr;       // pinned [max_rows]
  uint64_t tbl_dev = 0;               // device [max_rows] (the engine's ptrs buffer)
  uint8_t* stage_host = nullptr;      // pinned [max_rows * in_row]
  uint64_t stage_dev = 0;             // device [max_rows * in_row]
  uint64_t out_dev = 0;               // device [max_rows * out_row] (graph output)
  uint8_t* out_host = nullptr;        // pinned [max_rows * out_row]
  std::vector<uint64_t> pad;          // [max_rows] finite padding sources
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
};

// phase accumulators (ns) + counters
enum { kBatches, kPrepNs, kEnqueueNs, kWaitNs, kPostNs, kTotalNs, kRows, kStatCount };

struct Executor {
  int device = 0;
  uint64_t in_row = 0, out_row = 0;
  int max_rows = 0;
  std::vector<int> buckets;
  std::vector<std::unique_ptr<Instance>> inst;
  std::atomic<uint64_t> stat[kStatCount];
};

void SetErr(char* err, int32_t errlen, const std::string& m)
{
  if (err && errlen > 0) {
    strncpy(err, m.c_str(), errlen - 1);
    err[errlen - 1] = 0;
  }
}

int Fail(char* err, int32_t errlen, const char* what, hipError_t rc)
{
  SetErr(err, errlen, std::string(what) + ": " + hipGetErrorString(rc));
  return 1;
}

#define PGX_CHECK(call, what)                      \
  do {                                             \
    hipError_t rc_ = (call);                       \
    if (rc_ != hipSuccess) return Fail(err, errlen, what, rc_); \
  } while (0)

void FreeInstance(Instance* in)
{
  if (in->tbl_host) (void)hipHostFree(in->tbl_host);
  if (in->stage_host) (void)hipHostFree(in->stage_host);
  if (in->out_host) (void)hipHostFree(in->out_host);
  for (auto& e : in->ev)
    if (e) (void)hipEventDestroy(e);
  in->tbl_host = nullptr;
  in->stage_host = in->out_host = nullptr;
  in->ready = false;
}

}  // namespace

extern "C" {

/// Executor for `n_instances` model instances on `device`.  Rows are
/// in_row_bytes in / out_row_bytes out; buckets ascending (graph batch sizes).
void* tcamd_pgx_create(int32_t device, int32_t n_instances, uint64_t in_row_bytes, uint64_t out_row_bytes,
                       int32_t n_buckets, const int32_t* buckets, char* err, int32_t errlen)
{
  if (n_instances < 1 || n_buckets < 1 || in_row_bytes == 0 || out_row_bytes == 0) {
    SetErr(err, errlen, "tcamd_pgx_create: bad arguments");
    return nullptr;
  }
  auto* x = new Executor();
  x->device = device;
  x->in_row = in_row_bytes;
  x->out_row = out_row_bytes;
  for (int i = 0; i < n_buckets; ++i) {
    if (buckets[i] < 1 || (i && buckets[i] <= buckets[i - 1])) {
      SetErr(err, errlen, "tcamd_pgx_create: buckets must be positive and ascending");
      delete x;
      return nullptr;
    }
    x->buckets.push_back(buckets[i]);
  }
  x->max_rows = x->buckets.back();
  for (int i = 0; i < n_instances; ++i) x->inst.emplace_back(new Instance());
  for (auto& s : x->stat) s.store(0);
  return x;
}

/// Bind instance `i`: its HIP stream, one graph exec per bucket, the engine's
/// device pointer table, a device staging area for host rows, the graph's
/// output buffer and per-row padding pointers ([max_rows]).
int32_t tcamd_pgx_set_instance(void* xp, int32_t i, void* stream, const uint64_t* graph_execs, uint64_t tbl_dev,
                               uint64_t stage_dev, uint64_t out_dev, const uint64_t* pad_ptrs, char* err,
                               int32_t errlen)
{
  auto* x = static_cast<Executor*>(xp);
  if (!x || i < 0 || i >= static_cast<int>(x->inst.size())) {
    SetErr(err, errlen, "tcamd_pgx_set_instance: bad instance");
    return 1;
  }
  Instance* in = x->inst[i].get();
  std::lock_guard<std::mutex> lk(in->mu);
  FreeInstance(in);
  PGX_CHECK(hipSetDevice(x->device), "hipSetDevice");
  in->stream = static_cast<hipStream_t>(stream);
  in->execs.assign(x->buckets.size(), nullptr);
  for (size_t b = 0; b < x->buckets.size(); ++b) {
    in->execs[b] = reinterpret_cast<hipGraphExec_t>(graph_execs[b]);
    if (!in->execs[b]) {
      SetErr(err, errlen, "tcamd_pgx_set_instance: null graph exec");
      return 1;
    }
  }
  const size_t rows = static_cast<size_t>(x->max_rows);
  in->tbl_dev = tbl_dev;
  in->stage_dev = stage_dev;
  in->out_dev = out_dev;
  in->pad.assign(pad_ptrs, pad_ptrs + rows);
  PGX_CHECK(hipHostMalloc(reinterpret_cast<void**>(&in->tbl_host), rows * 8, hipHostMallocDefault), "hipHostMalloc");
  PGX_CHECK(hipHostMalloc(reinterpret_cast<void**>(&in->stage_host), rows * x->in_row, hipHostMallocDefault),
            "hipHostMalloc");
  PGX_CHECK(hipHostMalloc(reinterpret_cast<void**>(&in->out_host), rows * x->out_row, hipHostMallocDefault),
            "hipHostMalloc");
  for (auto& e : in->ev) PGX_CHECK(hipEventCreate(&e), "hipEventCreate");
  in->ready = true;
  return 0;
}

/// tcserve_exec_fn: run one batch on instance `instance`.
int tcamd_pgx_execute(void* user, int32_t instance, const tcserve_batch* b, char* err, int32_t errlen)
{
  const uint64_t t0 = MonoNs();
  auto* x = static_cast<Executor*>(user);
  if (!x || instance < 0 || instance >= static_cast<int>(x->inst.size())) {
    SetErr(err, errlen, "pgx: bad instance");
    return 1;
  }
  Instance* in = x->inst[instance].get();
  std::lock_guard<std::mutex> lk(in->mu);
  if (!in->ready) {
    SetErr(err, errlen, "pgx: instance not bound");
    return 1;
  }
  const int total = b->total_rows;
  if (total < 1 || total > x->max_rows) {
    SetErr(err, errlen, "batch of " + std::to_string(total) + " rows exceeds the largest bucket");
    return 1;
  }
  if (b->n_inputs < 1 || b->n_outputs < 1) {
    SetErr(err, errlen, "pgx: model needs one input and one output");
    return 1;
  }
  size_t bi = 0;
  while (x->buckets[bi] < total) ++bi;
  const int bucket = x->buckets[bi];
  PGX_CHECK(hipSetDevice(x->device), "hipSetDevice");

  // ---- host: row-pointer table, host rows staged into pinned memory
  const uint64_t in_row = x->in_row, out_row = x->out_row;
  int row = 0, host_rows = 0;
  for (int r = 0; r < b->n_requests; ++r) {
    const int n = b->rows[r];
    const tcserve_ref& ref = b->inputs[r * b->n_inputs];
    if (ref.bytes < static_cast<uint64_t>(n) * in_row) {
      SetErr(err, errlen, "input buffer too small for the batch rows");
      return 1;
    }
    if (ref.kind == 1) {
      for (int k = 0; k < n; ++k) in->tbl_host[row + k] = ref.ptr + static_cast<uint64_t>(k) * in_row;
    } else {
      memcpy(in->stage_host + static_cast<size_t>(host_rows) * in_row, reinterpret_cast<const void*>(ref.ptr),
             static_cast<size_t>(n) * in_row);
      for (int k = 0; k < n; ++k)
        in->tbl_host[row + k] = in->stage_dev + static_cast<uint64_t>(host_rows + k) * in_row;
      host_rows += n;
    }
    row += n;
  }
  for (int k = total; k < bucket; ++k) in->tbl_host[k] = in->pad[k];
  const uint64_t t1 = MonoNs();

  // ---- stream: inputs, graph, outputs
  hipStream_t s = in->stream;
  PGX_CHECK(hipEventRecord(in->ev[0], s), "hipEventRecord");
  if (host_rows)
    PGX_CHECK(hipMemcpyAsync(reinterpret_cast<void*>(in->stage_dev), in->stage_host,
                             static_cast<size_t>(host_rows) * in_row, hipMemcpyHostToDevice, s),
              "hipMemcpyAsync(stage)");
  PGX_CHECK(hipMemcpyAsync(reinterpret_cast<void*>(in->tbl_dev), in->tbl_host, static_cast<size_t>(bucket) * 8,
                           hipMemcpyHostToDevice, s),
            "hipMemcpyAsync(table)");
  PGX_CHECK(hipEventRecord(in->ev[1], s), "hipEventRecord");
  PGX_CHECK(hipGraphLaunch(in->execs[bi], s), "hipGraphLaunch");
  PGX_CHECK(hipEventRecord(in->ev[2], s), "hipEventRecord");
  std::vector<const void*> c_src;
  std::vector<void*> c_dst;
  std::vector<uint64_t> c_n;
  bool host_out = false;
  row = 0;
  for (int r = 0; r < b->n_requests; ++r) {
    const int n = b->rows[r];
    const tcserve_ref& ref = b->outputs[r * b->n_outputs];
    if (ref.ptr) {
      if (ref.bytes < static_cast<uint64_t>(n) * out_row) {
        SetErr(err, errlen, "output buffer too small for the batch rows");
        (void)hipStreamSynchronize(s);
        return 1;
      }
      if (ref.kind == 1) {
        c_src.push_back(reinterpret_cast<const void*>(in->out_dev + static_cast<uint64_t>(row) * out_row));
        c_dst.push_back(reinterpret_cast<void*>(ref.ptr));
        c_n.push_back(static_cast<uint64_t>(n) * out_row);
      } else {
        host_out = true;
      }
    }
    row += n;
  }
  if (!c_src.empty()) {
    int rc = tcamd_batched_copy(c_src.data(), c_dst.data(), c_n.data(), static_cast<int>(c_src.size()), s);
    if (rc != 0) return Fail(err, errlen, "batched_copy", static_cast<hipError_t>(rc));
  }
  if (host_out)
    PGX_CHECK(hipMemcpyAsync(in->out_host, reinterpret_cast<void*>(in->out_dev), static_cast<size_t>(total) * out_row,
                             hipMemcpyDeviceToHost, s),
              "hipMemcpyAsync(out)");
  PGX_CHECK(hipEventRecord(in->ev[3], s), "hipEventRecord");
  const uint64_t t2 = MonoNs();
  PGX_CHECK(hipEventSynchronize(in->ev[3]), "hipEventSynchronize");
  const uint64_t t3 = MonoNs();

  // ---- host outputs, GPU phase times
  if (host_out) {
    row = 0;
    for (int r = 0; r < b->n_requests; ++r) {
      const int n = b->rows[r];
      const tcserve_ref& ref = b->outputs[r * b->n_outputs];
      if (ref.ptr && ref.kind != 1)
        memcpy(reinterpret_cast<void*>(ref.ptr), in->out_host + static_cast<size_t>(row) * out_row,
               static_cast<size_t>(n) * out_row);
      row += n;
    }
  }
  float ms[3] = {0, 0, 0};
  for (int k = 0; k < 3; ++k) PGX_CHECK(hipEventElapsedTime(&ms[k], in->ev[k], in->ev[k + 1]), "hipEventElapsedTime");
  for (int k = 0; k < 3; ++k) b->timing_ns[k] = static_cast<uint64_t>(static_cast<double>(ms[k]) * 1e6);
  const uint64_t t4 = MonoNs();
  x->stat[kBatches] += 1;
  x->stat[kRows] += static_cast<uint64_t>(total);
  x->stat[kPrepNs] += t1 - t0;
  x->stat[kEnqueueNs] += t2 - t1;
  x->stat[kWaitNs] += t3 - t2;
  x->stat[kPostNs] += t4 - t3;
  x->stat[kTotalNs] += t4 - t0;
  return 0;
}

/// out[0..6]: batches, prep_ns, enqueue_ns, wait_ns, post_ns, total_ns, rows.
int32_t tcamd_pgx_stats(void* xp, uint64_t* out)
{
  auto* x = static_cast<Executor*>(xp);
  if (!x) return 1;
  for (int k = 0; k < kStatCount; ++k) out[k] = x->stat[k].load();
  return 0;
}

void tcamd_pgx_destroy(void* xp)
{
  auto* x = static_cast<Executor*>(xp);
  if (!x) return;
  for (auto& in : x->inst) {
    std::lock_guard<std::mutex> lk(in->mu);
    FreeInstance(in.get());
  }
  delete x;
}

}  // extern "C"
