// perf_analyzer for MI355X hosts — native load generator for KServe-v2 servers.
//
// The reference snapshot ships only relocation stubs for perf_analyzer
// (reference src/c++/perf_analyzer/README.md:29-30); this is the functional
// equivalent specified in SURVEY.md Appendix D, built on our C++ clients
// (src/http_client.cc, src/grpc_client.cc) with no Python on the hot path:
//
//   Options      perf_analyzer-compatible CLI (-m -x -u -i -b -a --sync
//                --streaming --shape -H --concurrency-range
//                --request-rate-range --request-distribution
//                --request-intervals --sequence-length --sequence-id-range
//                --input-data --string-length --string-data
//                --shared-memory none|system|cuda|hip
//                --output-shared-memory-size --measurement-interval/-p
//                --measurement-mode --measurement-request-count
//                --stability-percentage/-s --max-trials/-r --percentile
//                --latency-threshold/-l -f --warmup-request-count ...)
//   Backend      one protocol client (HTTP/1.1 or gRPC/h2) + control plane
//   DataSet      request tensors: host bytes, or system / HIP shared-memory
//                regions filled once (HIP: K1 Philox fill on the device)
//   LoadEngine   closed-loop concurrency slots or open-loop request-rate
//                schedule; completions are handed to a worker thread that
//                records timestamps and re-issues (never inside the
//                transport's callback thread)
//   Profiler     measurement windows, 3-window stability, percentiles,
//                server-side breakdown from ModelInferenceStatistics deltas
//   Reporter     perf_analyzer-style stdout, CSV (-f) and JSON reports
//   MultiSession (multigpu.cc) --gpus N / --devices: one Session (client,
//                regions, LoadEngine worker thread, HIP stream) per GPU; the
//                synthetic batch is made ONCE (K1 on the first GPU) and
//                replicated into every GPU's regions by a Fanout (RCCL
//                broadcast, xGMI peer-copy star, or host copies); the
//                Profiler measures all lanes over common windows and reports
//                per-GPU rows plus the aggregate row.
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "common.h"
#include "grpc_client.h"
#include "http_client.h"

namespace tcperf {

using triton::client::Error;
using triton::client::InferInput;
using triton::client::InferOptions;
using triton::client::InferRequestedOutput;
using triton::client::InferResult;

uint64_t NowNs();
struct Session;

struct SslFlags {
  bool grpc_use_ssl = false;
  std::string grpc_root_certs, grpc_private_key, grpc_cert_chain;
  bool https = false;  // any --ssl-https-* flag given
  long https_verify_peer = 1, https_verify_host = 2;
  std::string https_ca, https_cert, https_key;
  bool https_cert_der = false, https_key_der = false;
};

struct Options {
  std::string model;
  std::string version;
  std::string url;
  std::string protocol = "http";
  bool async = true;
  bool streaming = false;
  int batch = 1;
  std::map<std::string, std::vector<int64_t>> shapes;
  std::map<std::string, std::string> headers;
  SslFlags ssl;
  bool verbose = false;
  // load
  bool rate_mode = false;
  uint64_t conc_start = 1, conc_end = 1, conc_step = 1;
  double rate_start = 0, rate_end = 0, rate_step = 1;
  std::string distribution = "constant";
  std::string request_intervals_file;
  int sequence_length = 20;
  uint64_t seq_id_start = 1, seq_id_end = UINT32_MAX;
  int num_clients = 0;  // 0: auto
  // data
  std::string input_data = "random";
  int string_length = 128;
  std::string string_data;
  std::string shared_memory = "none";
  size_t output_shm_size = 102400;
  std::map<std::string, std::string> preregistered_inputs;  // input -> registered region name
  // [ext] NAME=R0,R1,..: several caller regions per input / output.  Request
  // slot s (a concurrency slot) always uses entry s % n, so after a run the
  // caller can check every output region against its own input region (the
  // served batch mixes rows of distinct requests: a row mix-up is visible)
  std::map<std::string, std::vector<std::string>> preregistered_input_lists;
  std::map<std::string, std::vector<std::string>> preregistered_outputs;
  int device = 0;
  uint64_t seed = 0;
  // multi-GPU: one lane per device
  std::vector<int> devices;        // --gpus N -> 0..N-1, --devices a,b,c; empty -> {device}
  std::vector<std::string> urls;   // -u a,b,...: lane i talks to urls[i % n]
  std::string fanout = "auto";     // rccl | p2p | host | auto (rccl for hip shm, host otherwise)
  bool load_per_gpu = false;       // --load-per-gpu: each lane gets the full load (weak scaling)
  // measurement
  std::string measurement_mode = "time_windows";
  uint64_t measurement_interval_ms = 5000;
  uint64_t measurement_request_count = 50;
  double stability_pct = 10.0;
  int max_trials = 10;
  int percentile = -1;
  uint64_t latency_threshold_ms = 0;
  uint64_t warmup_requests = 0;
  std::string csv_file;
  std::string json_file;
  bool collect_metrics = false;     // --collect-metrics: GPU busy %, power, VRAM (amdgpu sysfs)
  uint64_t metrics_interval_ms = 1000;
  std::string metrics_sysfs_root;   // default /sys/class/drm (tests point it at a fake tree)
  bool resume = false;  // --resume: continue a sweep checkpointed in json_file
  bool verbose_csv = false;
  bool collect_server_stats = true;
  std::string input_tensor_format = "binary";   // HTTP: binary | json (inline "data")
  std::string output_tensor_format = "binary";
  std::string compression = "none";              // none | gzip | deflate (gRPC messages / HTTP bodies)
  std::map<std::string, triton::client::RequestParameter> request_parameters;
};

/// Parse perf_analyzer flags.  Returns an error for unknown/invalid flags;
/// *help is set when -h/--help was given.
Error ParseOptions(int argc, char** argv, Options* opts, bool* help);
std::string Usage();

struct TensorSpec {
  std::string name;
  std::string datatype;
  std::vector<int64_t> shape;  // without the batch dim
};

struct ModelInfo {
  std::vector<TensorSpec> inputs, outputs;
  int max_batch_size = 0;
  bool sequential = false;
  bool decoupled = false;
};

// GPU metrics sampler (metrics.cc): amdgpu sysfs counters of GPU `device`.
class GpuMetrics {
 public:
  GpuMetrics(int device, uint64_t interval_ms, const std::string& sysfs_root);
  ~GpuMetrics();
  bool Available() const;
  void Start();
  void Stop();
  /// Averages over the samples since Start (false if none).
  bool Summary(double* util_pct, double* power_w, double* mem_mib) const;

 private:
  std::string dev_, power_file_;
  uint64_t interval_ms_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::thread th_;
  bool running_ = false, stop_ = false;
  uint64_t samples_ = 0, mem_max_ = 0;
  double busy_sum_ = 0, power_sum_ = 0;
};

struct ServerStats {
  uint64_t inference_count = 0, execution_count = 0;
  uint64_t success_count = 0, success_ns = 0;
  uint64_t queue_ns = 0, compute_input_ns = 0, compute_infer_ns = 0, compute_output_ns = 0;
};

// ---------------------------------------------------------------------------
class Backend {
 public:
  static Error Create(const Options& o, std::unique_ptr<Backend>* out);
  ~Backend();
  Error ModelMeta(ModelInfo* info);
  Error Stats(ServerStats* st);
  Error RegisterSystem(const std::string& name, const std::string& key, size_t bytes);
  Error UnregisterSystem(const std::string& name);
  Error RegisterDevice(const std::string& name, const cudaIpcMemHandle_t& h, int dev, size_t bytes);
  Error UnregisterDevice(const std::string& name);
  Error AsyncInfer(std::function<void(InferResult*)> cb, const InferOptions& opt,
                   const std::vector<InferInput*>& in, const std::vector<const InferRequestedOutput*>& out);
  Error SyncInfer(InferResult** r, const InferOptions& opt, const std::vector<InferInput*>& in,
                  const std::vector<const InferRequestedOutput*>& out);
  Error StartStream(std::function<void(InferResult*)> cb);
  Error StreamInfer(const InferOptions& opt, const std::vector<InferInput*>& in,
                    const std::vector<const InferRequestedOutput*>& out);
  Error StopStream();
  Error ClientStat(triton::client::InferStat* st);
  bool IsGrpc() const { return grpc_ != nullptr; }

 private:
  Options o_;
  triton::client::Headers headers_;
  std::unique_ptr<triton::client::InferenceServerHttpClient> http_;
  std::unique_ptr<triton::client::InferenceServerGrpcClient> grpc_;
};

// ---------------------------------------------------------------------------
/// Request tensors shared by every request of a run.
class DataSet {
 public:
  ~DataSet();
  /// `fill_inputs` false: input regions are allocated and registered but
  /// left for a Fanout to fill (the replicas of a multi-GPU run).
  Error Init(const Options& o, const ModelInfo& info, Backend* be, size_t max_slots, bool fill_inputs = true);
  /// Inputs of request number `seq` (JSON data with several entries cycles
  /// through them; synthetic data has one entry).
  const std::vector<InferInput*>& Inputs(uint64_t seq = 0) const { return inputs_[seq % inputs_.size()]; }
  /// Inputs of request `seq` issued on concurrency slot `slot`: slot-pinned
  /// entries (caller region lists) use entry slot % n, otherwise as Inputs(seq).
  const std::vector<InferInput*>& Inputs(uint64_t seq, size_t slot) const
  {
    return inputs_[(slot_entries_ ? slot : seq) % inputs_.size()];
  }
  size_t Entries() const { return inputs_.size(); }
  /// Shared-memory input regions in creation order (what a Fanout replicates).
  struct RegionView {
    void* ptr;     // device pointer (HIP) or host mapping (system)
    size_t bytes;
    bool device;
    int dev;
  };
  std::vector<RegionView> InputRegions() const;
  /// The lane's HIP stream (K1 fill, fan-out copies), null when not HIP.
  void* Stream() const { return stream_; }
  const std::vector<const InferRequestedOutput*>& Outputs(size_t slot) const;
  std::string Describe() const { return describe_; }
  void Release(Backend* be);

 private:
  struct Region {
    std::string name;
    std::string key;   // system shm key
    int fd = -1;
    void* host = nullptr;
    void* dev = nullptr;
    size_t bytes = 0;
    bool device = false;
    bool owned = true;
  };
  Error MakeRegion(Backend* be, const std::string& name, size_t bytes, bool device, Region* r);
  Error FillHost(const TensorSpec& t, const std::vector<int64_t>& shape, std::vector<uint8_t>* bytes,
                 std::vector<std::string>* strs);
  Options o_;
  std::string prefix_;  // region names: unique per DataSet (several sessions may share one server)
  std::vector<std::vector<InferInput*>> inputs_;              // [entry][input]
  std::vector<std::vector<InferRequestedOutput*>> outputs_;  // [slot][output]
  std::vector<std::vector<const InferRequestedOutput*>> outputs_c_;
  std::vector<std::vector<uint8_t>> host_data_;
  std::vector<Region> regions_;
  std::vector<size_t> input_regions_;  // indices into regions_
  void* stream_ = nullptr;             // hipStream_t on o_.device
  bool slot_entries_ = false;          // entries pinned to slots (caller region lists)
  std::string describe_;
};

// ---------------------------------------------------------------------------
struct Record {
  uint64_t start_ns, end_ns;
  bool ok;
};

/// Issues requests and records completions.  Closed loop (concurrency) or
/// open loop (request rate).  Thread-safe accessors for the profiler.
class LoadEngine {
 public:
  LoadEngine(const Options& o, Backend* be, DataSet* data, size_t max_slots);
  ~LoadEngine();
  /// Closed loop with `n` requests in flight (0 stops issuing).
  Error SetConcurrency(size_t n);
  /// Open loop at `rate` requests/sec (distribution from options).
  Error SetRequestRate(double rate);
  /// Closed loop that issues exactly `total` requests and waits for all of
  /// them; latencies (ns) are returned in completion order, and with
  /// `end_ns` each one's completion time (ns after the run started).
  Error RunFixed(size_t concurrency, uint64_t total, std::vector<uint64_t>* lat_ns, double* elapsed_s,
                 std::vector<uint64_t>* end_ns = nullptr);
  void Stop();
  /// Continuous closed loop for steady-state measurement: quiesces any
  /// previous load, then keeps `concurrency` requests in flight until
  /// SetConcurrency(0) (or StopLoop).  Callers mark record indices with
  /// CompletedCount and read the records with Snapshot.
  Error StartLoop(size_t concurrency);
  /// Stops issuing and waits (<= 30 s) until nothing is in flight.
  Error StopLoop();
  /// Waits until `target` records exist (all time, CompletedCount's index),
  /// at most `timeout_s`; fails on a request error or the timeout.
  Error WaitCompleted(size_t target, double timeout_s);
  /// Records completed since `since_index`; returns the new end index.
  size_t Snapshot(size_t since_index, std::vector<Record>* out);
  size_t CompletedCount();
  std::string FirstError();
  size_t InFlight() const { return in_flight_.load(); }

  struct Slot {
    InferOptions opt{""};
    uint64_t seq_id = 0;
    int seq_pos = 0;
    uint64_t sent_ns = 0;
    bool busy = false;
  };
  void SetSequenceModel(bool v) { seq_model_ = v; }

 private:
  void Worker();
  void SyncLoop(size_t slot);
  Error Issue(size_t slot);
  Error EnsureStream();
  void PrepareSequence(Slot* s);
  void RateLoop(double rate, uint64_t gen);
  void OnComplete(size_t slot, uint64_t start_ns, InferResult* r);

  Options o_;
  Backend* be_;
  std::vector<Backend*> clients_;                // async issue targets (clients_[0] == be_)
  std::vector<std::unique_ptr<Backend>> owned_;  // clients_[1..]
  DataSet* data_;
  std::vector<Slot> slots_;
  std::mutex mu_;
  std::condition_variable cv_;        // worker wake-up
  std::condition_variable fixed_cv_;  // completion progress
  std::deque<std::pair<size_t, Record>> done_;
  std::vector<size_t> pending_start_;
  std::vector<Record> records_;
  std::mutex rec_mu_;
  size_t target_conc_ = 0;
  uint64_t fixed_left_ = 0;  // fixed-count mode: requests still to issue
  bool fixed_mode_ = false;
  std::vector<uint64_t>* fixed_lat_ = nullptr;
  std::vector<uint64_t>* fixed_end_ = nullptr;
  std::atomic<size_t> in_flight_{0};
  std::atomic<bool> stop_{false};
  bool exiting_ = false;
  bool seq_model_ = false;
  std::atomic<bool> rate_active_{false};
  bool streaming_ = false;
  std::thread worker_;
  std::thread rate_thread_;
  std::vector<std::thread> sync_threads_;
  std::atomic<uint64_t> rate_gen_{0};
  std::atomic<uint64_t> delayed_{0};  // rate mode: schedule slips that dropped the backlog
  uint64_t next_seq_ = 0;
  std::atomic<uint64_t> issued_{0};  // request counter (selects the JSON data entry)
  std::string first_error_;
  std::vector<uint64_t> intervals_ns_;
  // streaming: request id -> (slot, send time)
  std::mutex stream_mu_;
  std::map<std::string, std::pair<size_t, uint64_t>> stream_ids_;
  uint64_t stream_counter_ = 0;
};

// ---------------------------------------------------------------------------
struct PointResult {
  double load = 0;  // concurrency or rate
  bool rate_mode = false;
  bool stable = false;
  uint64_t request_count = 0;
  double window_s = 0;
  double throughput = 0;  // infer/sec (requests * batch / s)
  double avg_us = 0, std_us = 0, p50_us = 0, p90_us = 0, p95_us = 0, p99_us = 0;
  double client_send_us = 0, client_recv_us = 0;
  uint64_t errors = 0;
  ServerStats server;  // delta over the windows
  bool has_server = false;
  bool has_gpu = false;  // --collect-metrics
  double gpu_util_pct = 0, gpu_power_w = 0, gpu_mem_mib = 0;
  int gpu = -1;                      // lane device (per-GPU rows), -1 = aggregate / single
  std::vector<PointResult> per_gpu;  // multi-GPU: one row per lane
};

/// Measures one or more lanes (one per GPU) over COMMON windows: every lane's
/// records, client and server stats are cut at the same t0/t1, stability is
/// judged on the aggregate, and a multi-lane point carries per-GPU rows.
class Profiler {
 public:
  Profiler(const Options& o, Backend* be, LoadEngine* eng) : o_(o) { AddLane(be, eng, o.device, o.url); }
  Profiler(const Options& o, const std::vector<Session*>& lanes);
  Error Profile(double load, PointResult* out);
  /// Share of `load` lane i runs (the full load with --load-per-gpu).
  double LaneLoad(double load, size_t i) const;

 private:
  struct Lane {
    Backend* be;
    LoadEngine* eng;
    int device;
    bool first_of_url;  // lanes sharing a server count its statistics once in the aggregate
    size_t rec_index = 0;
    std::unique_ptr<GpuMetrics> gpu;
  };
  void AddLane(Backend* be, LoadEngine* eng, int device, const std::string& url);
  std::vector<std::string> urls_;
  Error Window(std::vector<PointResult>* w, std::vector<std::vector<uint64_t>>* lat);
  Options o_;
  std::vector<Lane> lanes_;
};

void PrintSettings(const Options& o, const ModelInfo& info, const std::string& data_desc);
void PrintPoint(const Options& o, const PointResult& p);
void PrintSummary(const Options& o, const std::vector<PointResult>& pts);
Error WriteCsv(const Options& o, const std::vector<PointResult>& pts);
Error WriteJson(const Options& o, const std::vector<PointResult>& pts, const std::string& data_desc);
/// --resume: sweep points already completed in o.json_file (empty if none / other config).
Error LoadCheckpoint(const Options& o, std::vector<PointResult>* pts);
double Percentile(std::vector<uint64_t>& v, double p);

/// Everything one perf run needs; used by main() and the C API.
struct Session {
  Options opts;
  std::unique_ptr<Backend> backend;
  ModelInfo info;
  std::unique_ptr<DataSet> data;
  std::unique_ptr<LoadEngine> engine;
  size_t max_slots = 0;
  static Error Create(const Options& o, std::unique_ptr<Session>* out, bool fill_inputs = true);
  ~Session();
};

/// Replicates device (or host) buffers from the first lane to the others.
class Fanout {
 public:
  /// mode: rccl | p2p | host.  `devices[0]` is the root.
  static Error Create(const std::string& mode, const std::vector<int>& devices, std::unique_ptr<Fanout>* out);
  ~Fanout();
  /// dst[i] (on devices[i], i >= 1) <- src (on devices[0]); `device` false:
  /// host buffers (system shm).  Blocks until every copy has landed.
  Error Broadcast(const void* src, const std::vector<void*>& dst, size_t bytes, bool device);
  const std::string& Mode() const { return mode_; }
  double LastUs() const { return last_us_; }
  double TotalBytes() const { return total_bytes_; }

 private:
  std::string mode_;
  std::vector<int> devices_;
  std::vector<void*> streams_;  // hipStream_t per device
  std::vector<void*> comms_;    // ncclComm_t per device (rccl)
  double last_us_ = 0, total_bytes_ = 0;
};

/// --gpus N: one Session per GPU plus the fan-out of the synthetic batch.
struct MultiSession {
  Options opts;
  std::vector<std::unique_ptr<Session>> lanes;
  std::unique_ptr<Fanout> fanout;
  double fanout_us = 0;        // replication wall time (all input regions)
  bool replicas_verified = false;
  static Error Create(const Options& o, std::unique_ptr<MultiSession>* out);
  std::vector<Session*> LanePtrs() const;
  std::string Describe() const;
  ~MultiSession();
};

}  // namespace tcperf
