// tcserve — native gRPC front end of the bench/test server.
//
// The Python server (triton_client_amd/server) implements every KServe-v2
// endpoint; its grpc.aio front end tops out at a few thousand requests/s on
// one core, which caps perf_analyzer at small batch sizes.  tcserve puts a
// C++ HTTP/2 server on the public gRPC port:
//
//   * ModelInfer for models registered as *native* is handled entirely here:
//     protobuf decode (generated classes, csrc/cpp/proto), shared-memory
//     resolution against a mirror of the Python registries, a C++ dynamic
//     batcher with one worker per model instance, and ONE call per batch into
//     the model's executor (a Python callback that launches HIP work and
//     drops the GIL while the GPU runs), then response encode and send;
//   * every other RPC (control plane, streaming, non-native models, requests
//     using features the fast path does not cover) is proxied verbatim over
//     HTTP/2 to the Python grpc.aio server on an internal loopback port.
//
// Threading: N event loops (epoll + nghttp2 server sessions, one connection
// belongs to one loop); other threads post closures to a loop via eventfd.
#pragma once

#include <cstdint>

extern "C" {

/// One tensor reference of a batch: kind 0 = host memory, 1 = device memory.
struct tcserve_ref {
  int32_t kind;
  int32_t device;
  uint64_t ptr;
  uint64_t bytes;
};

/// A batch handed to a native model's executor.
struct tcserve_batch {
  int32_t n_requests;
  int32_t total_rows;
  const int32_t* rows;              // [n_requests]
  int32_t n_inputs;
  const tcserve_ref* inputs;        // [n_requests][n_inputs]
  int32_t n_outputs;
  const tcserve_ref* outputs;       // [n_requests][n_outputs]; ptr 0 = output not requested
  uint64_t* timing_ns;              // out: compute_input, compute_infer, compute_output
};

/// Executor: return 0 on success, else write a message into err.
typedef int (*tcserve_exec_fn)(void* user, int32_t instance, const tcserve_batch* batch, char* err, int32_t errlen);

void* tcserve_create(const char* host, int32_t port, const char* upstream_host, int32_t upstream_port,
                     int32_t io_threads, char* err, int32_t errlen);
int32_t tcserve_port(void* server);
/// Also serve KServe REST on host:port (native infer fast path; everything else is
/// relayed to the HTTP server at upstream_host:upstream_port).  Returns the bound port or -1.
int32_t tcserve_listen_http(void* server, const char* host, int32_t port, const char* upstream_host,
                            int32_t upstream_port, char* err, int32_t errlen);
/// dims are per-sample (without the batch dimension), flattened; ndims[i] gives each tensor's rank.
int32_t tcserve_add_model(void* server, const char* name, const char* version, int32_t max_batch,
                          int32_t max_queue_delay_us, int32_t instances, int32_t n_inputs, const char** in_names,
                          const char** in_dtypes, const int32_t* in_ndims, const int64_t* in_dims, int32_t n_outputs,
                          const char** out_names, const char** out_dtypes, const int32_t* out_ndims,
                          const int64_t* out_dims, tcserve_exec_fn fn, void* user, char* err, int32_t errlen);
int32_t tcserve_remove_model(void* server, const char* name);
/// Idle-aware batching (default on): skip the queue delay while no instance is executing.
int32_t tcserve_set_idle_dispatch(void* server, const char* name, int32_t on);
/// dynamic_batching.preferred_batch_size for a registered model (n = 0 clears).
int32_t tcserve_set_preferred(void* server, const char* name, const int32_t* sizes, int32_t n);
/// Discrete-event simulation of the native batcher's dispatch policy
/// (batch_policy.h, the functions Server::Worker runs) over scripted
/// arrivals: request i arrives at arrive_ns[i] (non-decreasing) with rows[i]
/// rows; a batch of r rows executes for exec_base_ns + r * exec_per_row_ns on
/// one of `instances` instances.  flags: bit 0 idle-aware, bit 1 pipelined,
/// bit 2 staggered.  Writes per batch its start time, rows, first request and
/// instance; returns the batch count (-1 on bad arguments, -2 if max_batches
/// was too small).
int32_t tcserve_batch_policy_sim(int32_t max_batch, uint64_t delay_ns, const int32_t* preferred, int32_t n_pref,
                                 int32_t instances, int32_t flags, const uint64_t* arrive_ns, const int32_t* rows,
                                 int32_t n, uint64_t exec_base_ns, uint64_t exec_per_row_ns, uint64_t* out_start_ns,
                                 int32_t* out_rows, int32_t* out_first, int32_t* out_instance, int32_t max_batches);
/// Closed-loop variant: `clients` clients each keep one request of rows_per_req rows in flight (client k
/// first arrives at k * spread_ns; a finished batch's clients come back turnaround_ns after its end, the
/// j-th of them j * resp_spacing_ns later).  Reports the batches started before horizon_ns; returns their
/// count (-1 on bad arguments, -2 if max_batches was too small).
int32_t tcserve_batch_policy_sim_closed(int32_t max_batch, uint64_t delay_ns, const int32_t* preferred,
                                        int32_t n_pref, int32_t instances, int32_t flags, int32_t clients,
                                        int32_t rows_per_req, uint64_t spread_ns, uint64_t turnaround_ns,
                                        uint64_t resp_spacing_ns, uint64_t exec_base_ns, uint64_t exec_per_row_ns,
                                        uint64_t horizon_ns, uint64_t* out_start_ns, int32_t* out_rows,
                                        int32_t* out_instance, int32_t max_batches);
/// Mirror of the Python shared-memory registries; kind 0 = system (ptr = host mapping), 1 = device.
int32_t tcserve_shm_add(void* server, const char* name, int32_t kind, uint64_t ptr, uint64_t bytes, int32_t device);
/// Unregister (name "" = all of kind).  Never blocks: returns how many of the removed regions
/// are still pinned by queued/executing requests (-1 on a bad kind); poll tcserve_shm_busy
/// before unmapping / closing such a region.
int32_t tcserve_shm_remove(void* server, int32_t kind, const char* name);
/// 1 while a removed region at `ptr` is still referenced by a queued or executing request.
int32_t tcserve_shm_busy(void* server, int32_t kind, uint64_t ptr);
/// out[0..9]: inference_count, execution_count, success_count, success_ns, fail_count, fail_ns,
/// queue_ns, compute_input_ns, compute_infer_ns, compute_output_ns; last_inference_ms at out[10].
int32_t tcserve_model_stats(void* server, const char* name, uint64_t* out);
/// Per batch size rows of 7: batch_size, count, in_ns, infer_ns, out_ns, (reserved x2). Returns row count.
int32_t tcserve_batch_stats(void* server, const char* name, uint64_t* out, int32_t max_rows);
/// Counters: [0] native requests, [1] proxied calls, [2] connections accepted, [3] REST requests
/// with a gzip/deflate body + gRPC infer messages that arrived compressed, [4] native REST
/// responses sent compressed.
int32_t tcserve_counters(void* server, uint64_t* out);
void tcserve_destroy(void* server);

}  // extern "C"
