// C ABI of the perf engine for in-process use from Python (bench.py drives
// the native load generator through ctypes; ctypes drops the GIL for the
// duration of each call, so no Python runs on the request path).
#include <algorithm>
#include <cstring>

#include "perf.h"

namespace {

void SetErr(char* err, int errlen, const std::string& msg)
{
  if (err && errlen > 0) {
    strncpy(err, msg.c_str(), errlen - 1);
    err[errlen - 1] = '\0';
  }
}

}  // namespace

extern "C" {

void* tcperf_session_create(int argc, const char** argv, char* err, int errlen)
{
  tcperf::Options o;
  bool help = false;
  std::vector<char*> args;
  args.push_back(const_cast<char*>("perf_analyzer"));
  for (int i = 0; i < argc; ++i) args.push_back(const_cast<char*>(argv[i]));
  tcperf::Error e = tcperf::ParseOptions(static_cast<int>(args.size()), args.data(), &o, &help);
  if (!e.IsOk() || help) {
    SetErr(err, errlen, help ? "help requested" : e.Message());
    return nullptr;
  }
  std::unique_ptr<tcperf::Session> s;
  e = tcperf::Session::Create(o, &s);
  if (!e.IsOk()) {
    SetErr(err, errlen, e.Message());
    return nullptr;
  }
  return s.release();
}

int tcperf_run_fixed(void* h, int concurrency, uint64_t total, uint64_t* lat_ns, double* elapsed_s, char* err,
                     int errlen)
{
  auto* s = static_cast<tcperf::Session*>(h);
  std::vector<uint64_t> lat;
  tcperf::Error e = s->engine->RunFixed(static_cast<size_t>(concurrency), total, &lat, elapsed_s);
  if (lat_ns) memcpy(lat_ns, lat.data(), std::min<size_t>(lat.size(), total) * sizeof(uint64_t));
  if (!e.IsOk()) {
    SetErr(err, errlen, e.Message());
    return 1;
  }
  return 0;
}

// As tcperf_run_fixed, plus each request's completion time (ns after the
// start) in end_ns, in completion order: lets a caller cut one continuous
// closed-loop run into back-to-back measurement windows with no drain between.
int tcperf_run_fixed_timed(void* h, int concurrency, uint64_t total, uint64_t* lat_ns, uint64_t* end_ns,
                           double* elapsed_s, char* err, int errlen)
{
  auto* s = static_cast<tcperf::Session*>(h);
  std::vector<uint64_t> lat, end;
  tcperf::Error e = s->engine->RunFixed(static_cast<size_t>(concurrency), total, &lat, elapsed_s, &end);
  if (lat_ns) memcpy(lat_ns, lat.data(), std::min<size_t>(lat.size(), total) * sizeof(uint64_t));
  if (end_ns) memcpy(end_ns, end.data(), std::min<size_t>(end.size(), total) * sizeof(uint64_t));
  if (!e.IsOk()) {
    SetErr(err, errlen, e.Message());
    return 1;
  }
  return 0;
}

// Continuous closed loop (steady-state measurement without a restart between
// the warm-up and the timed windows): start, mark indices with
// tcperf_loop_count, wait for a completion count, read records, stop.
int tcperf_loop_start(void* h, int concurrency, char* err, int errlen)
{
  auto* s = static_cast<tcperf::Session*>(h);
  tcperf::Error e = s->engine->StartLoop(static_cast<size_t>(concurrency));
  if (!e.IsOk()) {
    SetErr(err, errlen, e.Message());
    return 1;
  }
  return 0;
}

// completions so far (a record index) and the engine clock (ns)
uint64_t tcperf_loop_count(void* h, uint64_t* now_ns)
{
  auto* s = static_cast<tcperf::Session*>(h);
  if (now_ns) *now_ns = tcperf::NowNs();
  return s->engine->CompletedCount();
}

int tcperf_loop_wait(void* h, uint64_t target, double timeout_s, char* err, int errlen)
{
  auto* s = static_cast<tcperf::Session*>(h);
  tcperf::Error e = s->engine->WaitCompleted(static_cast<size_t>(target), timeout_s);
  if (!e.IsOk()) {
    SetErr(err, errlen, e.Message());
    return 1;
  }
  return 0;
}

// records [from, from + n) (n clipped to what exists): start / end ns on the
// engine clock and an ok flag; returns the number copied
uint64_t tcperf_loop_records(void* h, uint64_t from, uint64_t n, uint64_t* start_ns, uint64_t* end_ns, uint8_t* ok)
{
  auto* s = static_cast<tcperf::Session*>(h);
  std::vector<tcperf::Record> recs;
  s->engine->Snapshot(static_cast<size_t>(from), &recs);
  const uint64_t m = std::min<uint64_t>(n, recs.size());
  for (uint64_t i = 0; i < m; ++i) {
    if (start_ns) start_ns[i] = recs[i].start_ns;
    if (end_ns) end_ns[i] = recs[i].end_ns;
    if (ok) ok[i] = recs[i].ok ? 1 : 0;
  }
  return m;
}

int tcperf_loop_stop(void* h, char* err, int errlen)
{
  auto* s = static_cast<tcperf::Session*>(h);
  tcperf::Error e = s->engine->StopLoop();
  if (!e.IsOk()) {
    SetErr(err, errlen, e.Message());
    return 1;
  }
  return 0;
}

// out[0..7]: inference_count, execution_count, success_count, success_ns,
// queue_ns, compute_input_ns, compute_infer_ns, compute_output_ns
int tcperf_server_stats(void* h, uint64_t* out, char* err, int errlen)
{
  auto* s = static_cast<tcperf::Session*>(h);
  tcperf::ServerStats st;
  tcperf::Error e = s->backend->Stats(&st);
  if (!e.IsOk()) {
    SetErr(err, errlen, e.Message());
    return 1;
  }
  const uint64_t v[8] = {st.inference_count, st.execution_count, st.success_count, st.success_ns,
                         st.queue_ns, st.compute_input_ns, st.compute_infer_ns, st.compute_output_ns};
  memcpy(out, v, sizeof(v));
  return 0;
}

// One profiled load point; out[0..11]: load, stable, request_count, window_s,
// throughput, avg_us, p50_us, p90_us, p95_us, p99_us, client_send_us, client_recv_us
int tcperf_profile(void* h, double load, double* out, char* err, int errlen)
{
  auto* s = static_cast<tcperf::Session*>(h);
  tcperf::Profiler prof(s->opts, s->backend.get(), s->engine.get());
  tcperf::PointResult p;
  tcperf::Error e = prof.Profile(load, &p);
  s->engine->SetConcurrency(0);
  if (!e.IsOk()) {
    SetErr(err, errlen, e.Message());
    return 1;
  }
  const double v[12] = {p.load, p.stable ? 1.0 : 0.0, static_cast<double>(p.request_count), p.window_s,
                        p.throughput, p.avg_us, p.p50_us, p.p90_us, p.p95_us, p.p99_us, p.client_send_us,
                        p.client_recv_us};
  memcpy(out, v, sizeof(v));
  return 0;
}

int tcperf_describe(void* h, char* out, int outlen)
{
  auto* s = static_cast<tcperf::Session*>(h);
  SetErr(out, outlen, s->data->Describe());
  return 0;
}

void tcperf_session_destroy(void* h)
{
  delete static_cast<tcperf::Session*>(h);
}

}  // extern "C"
