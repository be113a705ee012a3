// C ABI of the perf engine for in-process use from Python (bench.py drives
// the native load generator through ctypes; ctypes drops the GIL for the
// duration of each call, so no Python runs on the request path).
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
