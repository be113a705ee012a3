// perf_analyzer Profiler (measurement windows + stability) and Reporter
// (stdout in perf_analyzer's layout, CSV, JSON), and Session setup.
#include <time.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <fstream>
#include <iterator>
#include <numeric>
#include <sstream>

#include "json.h"
#include "perf.h"
#include "trace.h"

namespace tcperf {

double Percentile(std::vector<uint64_t>& v, double p)
{
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  size_t idx = static_cast<size_t>(std::ceil(p / 100.0 * v.size()));
  idx = idx == 0 ? 0 : idx - 1;
  return static_cast<double>(v[std::min(idx, v.size() - 1)]);
}

static void SleepMs(uint64_t ms)
{
  struct timespec ts = {static_cast<time_t>(ms / 1000), static_cast<long>((ms % 1000) * 1000000)};
  nanosleep(&ts, nullptr);
}

static ServerStats Delta(const ServerStats& a, const ServerStats& b)
{
  ServerStats d;
  d.inference_count = b.inference_count - a.inference_count;
  d.execution_count = b.execution_count - a.execution_count;
  d.success_count = b.success_count - a.success_count;
  d.success_ns = b.success_ns - a.success_ns;
  d.queue_ns = b.queue_ns - a.queue_ns;
  d.compute_input_ns = b.compute_input_ns - a.compute_input_ns;
  d.compute_infer_ns = b.compute_infer_ns - a.compute_infer_ns;
  d.compute_output_ns = b.compute_output_ns - a.compute_output_ns;
  return d;
}

static void Accumulate(ServerStats* a, const ServerStats& b)
{
  a->inference_count += b.inference_count;
  a->execution_count += b.execution_count;
  a->success_count += b.success_count;
  a->success_ns += b.success_ns;
  a->queue_ns += b.queue_ns;
  a->compute_input_ns += b.compute_input_ns;
  a->compute_infer_ns += b.compute_infer_ns;
  a->compute_output_ns += b.compute_output_ns;
}

static void FillLatency(PointResult* r, std::vector<uint64_t>& lat)
{
  if (lat.empty()) return;
  double sum = 0, sq = 0;
  for (auto x : lat) {
    sum += x;
    sq += static_cast<double>(x) * x;
  }
  const double n = static_cast<double>(lat.size());
  const double mean = sum / n;
  r->avg_us = mean / 1000.0;
  r->std_us = std::sqrt(std::max(0.0, sq / n - mean * mean)) / 1000.0;
  r->p50_us = Percentile(lat, 50) / 1000.0;
  r->p90_us = Percentile(lat, 90) / 1000.0;
  r->p95_us = Percentile(lat, 95) / 1000.0;
  r->p99_us = Percentile(lat, 99) / 1000.0;
}

static double StabilityLatency(const Options& o, const PointResult& r)
{
  switch (o.percentile) {
    case 50: return r.p50_us;
    case 90: return r.p90_us;
    case 95: return r.p95_us;
    case 99: return r.p99_us;
    default: return r.avg_us;
  }
}

Profiler::Profiler(const Options& o, const std::vector<Session*>& lanes) : o_(o)
{
  for (Session* s : lanes) AddLane(s->backend.get(), s->engine.get(), s->opts.device, s->opts.url);
}

void Profiler::AddLane(Backend* be, LoadEngine* eng, int device, const std::string& url)
{
  Lane l;
  l.be = be;
  l.eng = eng;
  l.device = device;
  l.first_of_url = std::find(urls_.begin(), urls_.end(), url) == urls_.end();
  urls_.push_back(url);
  if (o_.collect_metrics) l.gpu.reset(new GpuMetrics(device, o_.metrics_interval_ms, o_.metrics_sysfs_root));
  lanes_.push_back(std::move(l));
}

double Profiler::LaneLoad(double load, size_t i) const
{
  const size_t n = lanes_.size();
  if (n <= 1 || o_.load_per_gpu) return load;
  if (o_.rate_mode) return load / n;
  // concurrency: integral split, the remainder on the first lanes
  const uint64_t c = static_cast<uint64_t>(load);
  return static_cast<double>(c / n + (i < c % n ? 1 : 0));
}

// One window over every lane, cut at common t0/t1.  w[i] / lat[i] per lane.
Error Profiler::Window(std::vector<PointResult>* w, std::vector<std::vector<uint64_t>>* lat)
{
  char tag[96];
  snprintf(tag, sizeof(tag), "perf.window %s=%g", o_.rate_mode ? "rate" : "concurrency", (*w)[0].load);
  triton::client::trace::Range range(tag);
  const size_t n = lanes_.size();
  std::vector<ServerStats> s0(n), s1(n);
  std::vector<triton::client::InferStat> c0(n), c1(n);
  std::vector<size_t> start_count(n);
  for (size_t i = 0; i < n; ++i) {
    if (o_.collect_server_stats) {
      Error e = lanes_[i].be->Stats(&s0[i]);
      if (!e.IsOk()) return e;
    }
    lanes_[i].be->ClientStat(&c0[i]);
  }
  const uint64_t t0 = NowNs();
  for (size_t i = 0; i < n; ++i) start_count[i] = lanes_[i].eng->CompletedCount();
  if (o_.measurement_mode == "count_windows") {
    const uint64_t limit = t0 + 600ull * 1000000000ull;
    while (NowNs() < limit) {
      size_t done = 0;
      bool err = false;
      for (size_t i = 0; i < n; ++i) {
        done += lanes_[i].eng->CompletedCount() - start_count[i];
        err = err || !lanes_[i].eng->FirstError().empty();
      }
      if (err || done >= o_.measurement_request_count) break;
      SleepMs(1);
    }
  } else {
    SleepMs(o_.measurement_interval_ms);
  }
  const uint64_t t1 = NowNs();
  for (size_t i = 0; i < n; ++i) {
    Lane& L = lanes_[i];
    PointResult& r = (*w)[i];
    L.be->ClientStat(&c1[i]);
    if (o_.collect_server_stats) {
      Error e = L.be->Stats(&s1[i]);
      if (!e.IsOk()) return e;
      r.server = Delta(s0[i], s1[i]);
      r.has_server = true;
    }
    std::vector<Record> recs;
    L.rec_index = L.eng->Snapshot(L.rec_index, &recs);
    (*lat)[i].clear();
    for (const auto& rc : recs) {
      if (rc.ok) (*lat)[i].push_back(rc.end_ns - rc.start_ns);
      else r.errors++;
    }
    r.request_count = (*lat)[i].size();
    r.window_s = (t1 - t0) * 1e-9;
    r.throughput = r.window_s > 0 ? r.request_count * static_cast<double>(o_.batch) / r.window_s : 0;
    const uint64_t dn = c1[i].completed_request_count - c0[i].completed_request_count;
    if (dn) {
      r.client_send_us = (c1[i].cumulative_send_time_ns - c0[i].cumulative_send_time_ns) / 1000.0 / dn;
      r.client_recv_us = (c1[i].cumulative_receive_time_ns - c0[i].cumulative_receive_time_ns) / 1000.0 / dn;
    }
    std::vector<uint64_t> tmp = (*lat)[i];
    FillLatency(&r, tmp);
  }
  return Error::Success;
}

// Sum lane rows (same window) into one aggregate row.
static PointResult Aggregate(const std::vector<PointResult>& rows, const std::vector<bool>& count_server,
                             std::vector<uint64_t>* all_lat)
{
  PointResult a;
  a.load = rows[0].load;
  a.window_s = rows[0].window_s;
  double sends = 0, recvs = 0;
  for (size_t k = 0; k < rows.size(); ++k) {
    const PointResult& r = rows[k];
    a.request_count += r.request_count;
    a.throughput += r.throughput;
    a.errors += r.errors;
    sends += r.client_send_us * r.request_count;
    recvs += r.client_recv_us * r.request_count;
    if (r.has_server && count_server[k]) {
      Accumulate(&a.server, r.server);
      a.has_server = true;
    }
  }
  if (a.request_count) {
    a.client_send_us = sends / a.request_count;
    a.client_recv_us = recvs / a.request_count;
  }
  std::vector<uint64_t> tmp = *all_lat;
  FillLatency(&a, tmp);
  return a;
}

Error Profiler::Profile(double load, PointResult* out)
{
  *out = PointResult();
  out->load = load;
  out->rate_mode = o_.rate_mode;
  const size_t n = lanes_.size();
  for (size_t i = 0; i < n; ++i) {
    const double l = LaneLoad(load, i);
    Error e = o_.rate_mode ? lanes_[i].eng->SetRequestRate(l) : lanes_[i].eng->SetConcurrency(static_cast<size_t>(l));
    if (!e.IsOk()) return e;
  }
  if (o_.warmup_requests) {
    for (auto& L : lanes_) {
      const size_t c0 = L.eng->CompletedCount();
      while (L.eng->CompletedCount() - c0 < o_.warmup_requests && L.eng->FirstError().empty()) SleepMs(1);
    }
  }
  for (auto& L : lanes_) {
    L.rec_index = L.eng->CompletedCount();
    if (L.gpu) L.gpu->Start();  // samples over this point's windows
  }
  std::vector<PointResult> wins;                      // aggregate per window
  std::vector<std::vector<PointResult>> lane_wins;    // [window][lane]
  std::vector<std::vector<std::vector<uint64_t>>> lats;  // [window][lane]
  for (int trial = 0; trial < o_.max_trials; ++trial) {
    std::vector<PointResult> w(n);
    for (size_t i = 0; i < n; ++i) {
      w[i].load = LaneLoad(load, i);
      w[i].rate_mode = o_.rate_mode;
      w[i].gpu = lanes_[i].device;
    }
    std::vector<std::vector<uint64_t>> lat(n);
    Error e = Window(&w, &lat);
    if (!e.IsOk()) return e;
    for (auto& L : lanes_) {
      const std::string err = L.eng->FirstError();
      if (!err.empty()) return Error("request failed: " + err);
    }
    std::vector<uint64_t> all;
    for (const auto& l : lat) all.insert(all.end(), l.begin(), l.end());
    std::vector<bool> count_server;
    for (const auto& L : lanes_) count_server.push_back(L.first_of_url);
    PointResult agg = n == 1 ? w[0] : Aggregate(w, count_server, &all);
    agg.load = load;
    if (o_.verbose)
      fprintf(stderr, "  window %d: %lu requests, %.1f infer/sec, latency %.0f usec\n", trial,
              static_cast<unsigned long>(agg.request_count), agg.throughput, StabilityLatency(o_, agg));
    wins.push_back(agg);
    lane_wins.push_back(std::move(w));
    lats.push_back(std::move(lat));
    if (wins.size() >= 3) {
      const size_t m = wins.size();
      double tsum = 0, lsum = 0;
      for (size_t i = m - 3; i < m; ++i) {
        tsum += wins[i].throughput;
        lsum += StabilityLatency(o_, wins[i]);
      }
      const double tmean = tsum / 3, lmean = lsum / 3, pct = o_.stability_pct / 100.0;
      bool stable = tmean > 0;
      for (size_t i = m - 3; i < m && stable; ++i) {
        if (std::fabs(wins[i].throughput - tmean) > pct * tmean) stable = false;
        if (std::fabs(StabilityLatency(o_, wins[i]) - lmean) > pct * lmean) stable = false;
      }
      if (stable) {
        out->stable = true;
        break;
      }
    }
  }
  // merge the last (up to) 3 windows, per lane and in aggregate
  const size_t m = wins.size();
  const size_t from = m >= 3 ? m - 3 : 0;
  auto merge = [&](PointResult* dst, auto get_row, auto get_lat) {
    std::vector<uint64_t> all;
    for (size_t i = from; i < m; ++i) {
      const PointResult& r = get_row(i);
      dst->request_count += r.request_count;
      dst->window_s += r.window_s;
      dst->errors += r.errors;
      dst->client_send_us += r.client_send_us / (m - from);
      dst->client_recv_us += r.client_recv_us / (m - from);
      if (r.has_server) {
        Accumulate(&dst->server, r.server);
        dst->has_server = true;
      }
      get_lat(i, &all);
    }
    dst->throughput = dst->window_s > 0 ? dst->request_count * static_cast<double>(o_.batch) / dst->window_s : 0;
    FillLatency(dst, all);
  };
  merge(out, [&](size_t i) -> const PointResult& { return wins[i]; },
        [&](size_t i, std::vector<uint64_t>* all) {
          for (const auto& l : lats[i]) all->insert(all->end(), l.begin(), l.end());
        });
  if (n > 1) {
    for (size_t k = 0; k < n; ++k) {
      PointResult r;
      r.load = LaneLoad(load, k);
      r.rate_mode = o_.rate_mode;
      r.gpu = lanes_[k].device;
      r.stable = out->stable;
      merge(&r, [&](size_t i) -> const PointResult& { return lane_wins[i][k]; },
            [&](size_t i, std::vector<uint64_t>* all) { all->insert(all->end(), lats[i][k].begin(), lats[i][k].end()); });
      out->per_gpu.push_back(r);
    }
  }
  for (size_t k = 0; k < n; ++k) {
    Lane& L = lanes_[k];
    if (!L.gpu) continue;
    L.gpu->Stop();
    PointResult& dst = n > 1 ? out->per_gpu[k] : *out;
    dst.has_gpu = L.gpu->Summary(&dst.gpu_util_pct, &dst.gpu_power_w, &dst.gpu_mem_mib);
    if (n > 1 && dst.has_gpu) {  // aggregate: mean utilisation, summed power / memory
      out->has_gpu = true;
      out->gpu_util_pct += dst.gpu_util_pct / n;
      out->gpu_power_w += dst.gpu_power_w;
      out->gpu_mem_mib += dst.gpu_mem_mib;
    }
  }
  return Error::Success;
}

// ============================================================================
// Reporter
// ============================================================================
void PrintSettings(const Options& o, const ModelInfo& info, const std::string& data_desc)
{
  printf("*** Measurement Settings ***\n");
  printf("  Batch size: %d\n", o.batch);
  printf("  Service Kind: Triton (%s)\n", o.protocol == "grpc" ? "gRPC" : "HTTP");
  if (o.measurement_mode == "count_windows")
    printf("  Using \"count_windows\" mode for stabilization\n  Minimum number of samples in each window: %lu\n",
           static_cast<unsigned long>(o.measurement_request_count));
  else
    printf("  Using \"time_windows\" mode for stabilization\n  Measurement window: %lu msec\n",
           static_cast<unsigned long>(o.measurement_interval_ms));
  if (o.latency_threshold_ms) printf("  Latency limit: %lu msec\n", static_cast<unsigned long>(o.latency_threshold_ms));
  if (o.rate_mode) {
    if (!o.request_intervals_file.empty())
      printf("  Using request intervals from %s\n", o.request_intervals_file.c_str());
    else
      printf("  Request Rate limit: %g - %g requests per second (%s distribution)\n", o.rate_start, o.rate_end,
             o.distribution.c_str());
  } else {
    printf("  Concurrency limit: %lu concurrent requests\n", static_cast<unsigned long>(o.conc_end));
  }
  printf("  Using %s calls for inference\n",
         o.streaming ? "streaming" : (o.async ? "asynchronous" : "synchronous"));
  if (info.sequential) printf("  Sequence model: %d requests per sequence\n", o.sequence_length);
  printf("  Data: %s\n", data_desc.c_str());
  if (o.percentile > 0) printf("  Stabilizing using p%d latency\n", o.percentile);
  else printf("  Stabilizing using average latency\n");
  printf("\n");
  fflush(stdout);
}

void PrintPoint(const Options& o, const PointResult& p)
{
  if (p.rate_mode) printf("Request Rate: %g inference requests per seconds\n", p.load);
  else printf("Request concurrency: %g\n", p.load);
  printf("  Client: \n");
  printf("    Request count: %lu\n", static_cast<unsigned long>(p.request_count));
  printf("    Throughput: %.2f infer/sec\n", p.throughput);
  if (o.percentile > 0) {
    printf("    p50 latency: %.0f usec\n    p90 latency: %.0f usec\n    p95 latency: %.0f usec\n"
           "    p99 latency: %.0f usec\n", p.p50_us, p.p90_us, p.p95_us, p.p99_us);
  } else {
    printf("    Avg latency: %.0f usec (standard deviation %.0f usec)\n", p.avg_us, p.std_us);
    printf("    p50 latency: %.0f usec\n    p90 latency: %.0f usec\n    p95 latency: %.0f usec\n"
           "    p99 latency: %.0f usec\n", p.p50_us, p.p90_us, p.p95_us, p.p99_us);
  }
  printf("    Avg %s time: %.0f usec (marshal request %.0f usec + response wait/unmarshal %.0f usec)\n",
         o.protocol == "grpc" ? "gRPC" : "HTTP", p.client_send_us + p.client_recv_us, p.client_send_us,
         p.client_recv_us);
  if (p.errors) printf("    Failed requests: %lu\n", static_cast<unsigned long>(p.errors));
  if (p.has_server) {
    const ServerStats& s = p.server;
    const double n = s.success_count ? static_cast<double>(s.success_count) : 1.0;
    const double req = s.success_ns / n / 1000.0, q = s.queue_ns / n / 1000.0;
    const double ci = s.compute_input_ns / n / 1000.0, cf = s.compute_infer_ns / n / 1000.0,
                 co = s.compute_output_ns / n / 1000.0;
    printf("  Server: \n");
    printf("    Inference count: %lu\n", static_cast<unsigned long>(s.inference_count));
    printf("    Execution count: %lu\n", static_cast<unsigned long>(s.execution_count));
    printf("    Successful request count: %lu\n", static_cast<unsigned long>(s.success_count));
    printf("    Avg request latency: %.0f usec (overhead %.0f usec + queue %.0f usec + compute input %.0f usec + "
           "compute infer %.0f usec + compute output %.0f usec)\n",
           req, std::max(0.0, req - q - ci - cf - co), q, ci, cf, co);
  }
  if (!p.stable) printf("  [WARNING] measurement did not stabilise within %d windows\n", o.max_trials);
  if (p.has_gpu)
    printf("    GPU: utilization %.1f%%, power %.1f W, max memory used %.0f MiB\n", p.gpu_util_pct, p.gpu_power_w,
           p.gpu_mem_mib);
  if (!p.per_gpu.empty()) {
    printf("  Per-GPU (%zu lanes, common windows):\n", p.per_gpu.size());
    for (const auto& g : p.per_gpu) {
      printf("    GPU %d: %s %g, requests %lu, throughput %.2f infer/sec, p50 %.0f / p90 %.0f / p99 %.0f usec",
             g.gpu, g.rate_mode ? "rate" : "concurrency", g.load, static_cast<unsigned long>(g.request_count),
             g.throughput, g.p50_us, g.p90_us, g.p99_us);
      if (g.has_server && g.server.execution_count)
        printf(", server batches %lu (avg %.1f rows)", static_cast<unsigned long>(g.server.execution_count),
               static_cast<double>(g.server.inference_count) / g.server.execution_count);
      if (g.has_gpu) printf(", GPU util %.1f%%", g.gpu_util_pct);
      printf("\n");
    }
  }
  printf("\n");
  fflush(stdout);
}

void PrintSummary(const Options& o, const std::vector<PointResult>& pts)
{
  printf("Inferences/Second vs. Client %s Batch Latency\n", o.percentile > 0 ? ("p" + std::to_string(o.percentile)).c_str() : "Average");
  for (const auto& p : pts)
    printf("%s: %g, throughput: %.2f infer/sec, latency %.0f usec\n", p.rate_mode ? "Request Rate" : "Concurrency",
           p.load, p.throughput, StabilityLatency(o, p));
  fflush(stdout);
}

Error WriteCsv(const Options& o, const std::vector<PointResult>& pts)
{
  if (o.csv_file.empty()) return Error::Success;
  std::ofstream f(o.csv_file);
  if (!f) return Error("cannot write " + o.csv_file);
  // multi-GPU: a leading GPU column, the aggregate row ("all") then one row per GPU
  const bool multi = o.devices.size() > 1;
  if (multi) f << "GPU,";
  f << (o.rate_mode ? "Request Rate" : "Concurrency")
    << ",Inferences/Second,Client Send,Network+Server Send/Recv,Server Queue,Server Compute Input,"
       "Server Compute Infer,Server Compute Output,Client Recv,p50 latency,p90 latency,p95 latency,p99 latency,"
       "Avg latency,request/response,response wait";
  if (o.collect_metrics) f << ",Avg GPU Utilization,Avg GPU Power Usage,Max GPU Memory Usage";
  if (o.verbose_csv) f << ",Failed requests,Stable";
  f << "\n";
  auto row = [&](const PointResult& p, const std::string& gpu) {
    const ServerStats& s = p.server;
    const double n = s.success_count ? static_cast<double>(s.success_count) : 1.0;
    const double q = s.queue_ns / n / 1000.0, ci = s.compute_input_ns / n / 1000.0,
                 cf = s.compute_infer_ns / n / 1000.0, co = s.compute_output_ns / n / 1000.0;
    const double net = std::max(0.0, p.avg_us - p.client_send_us - p.client_recv_us - q - ci - cf - co);
    char line[1024];
    snprintf(line, sizeof(line), "%g,%.2f,%.0f,%.0f,%.0f,%.0f,%.0f,%.0f,%.0f,%.0f,%.0f,%.0f,%.0f,%.0f,%.0f,%.0f",
             p.load, p.throughput, p.client_send_us, net, q, ci, cf, co, p.client_recv_us, p.p50_us, p.p90_us,
             p.p95_us, p.p99_us, p.avg_us, p.client_send_us, p.client_recv_us);
    if (multi) f << gpu << ",";
    f << line;
    if (o.collect_metrics) {
      // perf_analyzer's units: utilization as a fraction, power in W, memory in bytes
      char g[160];
      snprintf(g, sizeof(g), ",%.4f,%.1f,%.0f", p.gpu_util_pct / 100.0, p.gpu_power_w, p.gpu_mem_mib * 1048576.0);
      f << g;
    }
    if (o.verbose_csv) f << "," << p.errors << "," << (p.stable ? 1 : 0);
    f << "\n";
  };
  for (const auto& p : pts) {
    row(p, "all");
    for (const auto& g : p.per_gpu) row(g, std::to_string(g.gpu));
  }
  return Error::Success;
}

Error WriteJson(const Options& o, const std::vector<PointResult>& pts, const std::string& data_desc)
{
  if (o.json_file.empty()) return Error::Success;
  std::ofstream f(o.json_file);
  if (!f) return Error("cannot write " + o.json_file);
  f << "{\"model\":\"" << o.model << "\",\"gpus\":" << std::max<size_t>(1, o.devices.size())
    << ",\"batch_size\":" << o.batch << ",\"protocol\":\"" << o.protocol
    << "\",\"shared_memory\":\"" << o.shared_memory << "\",\"mode\":\"" << (o.rate_mode ? "request_rate" : "concurrency")
    << "\",\"data\":\"" << data_desc << "\",\"points\":[";
  for (size_t i = 0; i < pts.size(); ++i) {
    const auto& p = pts[i];
    const auto& s = p.server;
    char buf[1024];
    snprintf(buf, sizeof(buf),
             "%s{\"load\":%g,\"stable\":%s,\"request_count\":%lu,\"window_s\":%.6f,\"throughput\":%.3f,"
             "\"avg_us\":%.1f,\"std_us\":%.1f,\"p50_us\":%.1f,\"p90_us\":%.1f,\"p95_us\":%.1f,\"p99_us\":%.1f,"
             "\"client_send_us\":%.1f,\"client_recv_us\":%.1f,\"errors\":%lu,\"server\":{\"inference_count\":%lu,"
             "\"execution_count\":%lu,\"success_count\":%lu,\"queue_ns\":%lu,\"compute_input_ns\":%lu,"
             "\"compute_infer_ns\":%lu,\"compute_output_ns\":%lu}}",
             i ? "," : "", p.load, p.stable ? "true" : "false", static_cast<unsigned long>(p.request_count),
             p.window_s, p.throughput, p.avg_us, p.std_us, p.p50_us, p.p90_us, p.p95_us, p.p99_us, p.client_send_us,
             p.client_recv_us, static_cast<unsigned long>(p.errors), static_cast<unsigned long>(s.inference_count),
             static_cast<unsigned long>(s.execution_count), static_cast<unsigned long>(s.success_count),
             static_cast<unsigned long>(s.queue_ns), static_cast<unsigned long>(s.compute_input_ns),
             static_cast<unsigned long>(s.compute_infer_ns), static_cast<unsigned long>(s.compute_output_ns));
    std::string pt(buf);
    if (p.has_gpu) {
      char g[200];
      snprintf(g, sizeof(g), ",\"gpu\":{\"util_pct\":%.2f,\"power_w\":%.2f,\"mem_mib\":%.1f}}", p.gpu_util_pct,
               p.gpu_power_w, p.gpu_mem_mib);
      pt.pop_back();  // reopen the point object
      pt += g;
    }
    if (!p.per_gpu.empty()) {
      std::string rows = ",\"per_gpu\":[";
      for (size_t k = 0; k < p.per_gpu.size(); ++k) {
        const auto& g = p.per_gpu[k];
        char r[512];
        snprintf(r, sizeof(r),
                 "%s{\"gpu\":%d,\"load\":%g,\"request_count\":%lu,\"throughput\":%.3f,\"avg_us\":%.1f,"
                 "\"p50_us\":%.1f,\"p90_us\":%.1f,\"p95_us\":%.1f,\"p99_us\":%.1f,\"errors\":%lu,"
                 "\"server_inference_count\":%lu,\"server_execution_count\":%lu%s}",
                 k ? "," : "", g.gpu, g.load, static_cast<unsigned long>(g.request_count), g.throughput, g.avg_us,
                 g.p50_us, g.p90_us, g.p95_us, g.p99_us, static_cast<unsigned long>(g.errors),
                 static_cast<unsigned long>(g.server.inference_count),
                 static_cast<unsigned long>(g.server.execution_count), "");
        rows += r;
      }
      rows += "]}";
      pt.pop_back();
      pt += rows;
    }
    f << pt;
  }
  f << "]}\n";
  return Error::Success;
}

Error LoadCheckpoint(const Options& o, std::vector<PointResult>* pts)
{
  pts->clear();
  if (!o.resume || o.json_file.empty()) return Error::Success;
  std::ifstream f(o.json_file);
  if (!f) return Error::Success;  // nothing to resume yet
  std::string text((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  namespace js = triton::client::json;
  js::Value root;
  std::string err;
  if (!js::Parse(text, &root, &err)) return Error("--resume: cannot parse " + o.json_file + ": " + err);
  auto str = [&](const char* k) {
    const js::Value* v = root.Find(k);
    return v && v->IsString() ? v->AsString() : std::string();
  };
  const js::Value* b = root.Find("batch_size");
  if (str("model") != o.model || !b || b->AsInt() != static_cast<int64_t>(o.batch) || str("protocol") != o.protocol ||
      str("shared_memory") != o.shared_memory || str("mode") != (o.rate_mode ? "request_rate" : "concurrency"))
    return Error("--resume: " + o.json_file + " holds a different sweep (model/batch/protocol/shm/mode)");
  const js::Value* arr = root.Find("points");
  if (!arr || !arr->IsArray()) return Error::Success;
  auto num = [](const js::Value& o, const char* k) {
    const js::Value* v = o.Find(k);
    return v ? v->AsDouble() : 0.0;
  };
  for (const js::Value& e : arr->Elements()) {
    PointResult p;
    p.load = num(e, "load");
    p.rate_mode = o.rate_mode;
    const js::Value* st = e.Find("stable");
    p.stable = st && st->AsBool();
    p.request_count = static_cast<uint64_t>(num(e, "request_count"));
    p.window_s = num(e, "window_s");
    p.throughput = num(e, "throughput");
    p.avg_us = num(e, "avg_us");
    p.std_us = num(e, "std_us");
    p.p50_us = num(e, "p50_us");
    p.p90_us = num(e, "p90_us");
    p.p95_us = num(e, "p95_us");
    p.p99_us = num(e, "p99_us");
    p.client_send_us = num(e, "client_send_us");
    p.client_recv_us = num(e, "client_recv_us");
    p.errors = static_cast<uint64_t>(num(e, "errors"));
    if (const js::Value* sv = e.Find("server")) {
      p.has_server = true;
      p.server.inference_count = static_cast<uint64_t>(num(*sv, "inference_count"));
      p.server.execution_count = static_cast<uint64_t>(num(*sv, "execution_count"));
      p.server.success_count = static_cast<uint64_t>(num(*sv, "success_count"));
      p.server.queue_ns = static_cast<uint64_t>(num(*sv, "queue_ns"));
      p.server.compute_input_ns = static_cast<uint64_t>(num(*sv, "compute_input_ns"));
      p.server.compute_infer_ns = static_cast<uint64_t>(num(*sv, "compute_infer_ns"));
      p.server.compute_output_ns = static_cast<uint64_t>(num(*sv, "compute_output_ns"));
    }
    if (const js::Value* g = e.Find("gpu")) {
      p.has_gpu = true;
      p.gpu_util_pct = num(*g, "util_pct");
      p.gpu_power_w = num(*g, "power_w");
      p.gpu_mem_mib = num(*g, "mem_mib");
    }
    pts->push_back(p);
  }
  return Error::Success;
}

// ============================================================================
// Session
// ============================================================================
Error Session::Create(const Options& o, std::unique_ptr<Session>* out, bool fill_inputs)
{
  std::unique_ptr<Session> s(new Session());
  s->opts = o;
  Error e = Backend::Create(o, &s->backend);
  if (!e.IsOk()) return e;
  e = s->backend->ModelMeta(&s->info);
  if (!e.IsOk()) return Error("failed to get metadata of model '" + o.model + "': " + e.Message());
  if (s->info.decoupled && !o.streaming) return Error("model is decoupled; use --streaming with -i grpc");
  s->max_slots = o.rate_mode ? 64 : static_cast<size_t>(std::max<uint64_t>(1, o.conc_end));
  s->data.reset(new DataSet());
  e = s->data->Init(o, s->info, s->backend.get(), s->max_slots, fill_inputs);
  if (!e.IsOk()) {
    s->data->Release(s->backend.get());
    return e;
  }
  s->engine.reset(new LoadEngine(o, s->backend.get(), s->data.get(), s->max_slots));
  s->engine->SetSequenceModel(s->info.sequential);
  *out = std::move(s);
  return Error::Success;
}

Session::~Session()
{
  engine.reset();
  if (data) data->Release(backend.get());
}

}  // namespace tcperf
