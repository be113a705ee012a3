// perf_analyzer CLI entry point (see perf.h for the architecture).
#include <algorithm>
#include <cmath>
#include <cstdio>

#include "perf.h"

int main(int argc, char** argv)
{
  tcperf::Options o;
  bool help = false;
  tcperf::Error e = tcperf::ParseOptions(argc, argv, &o, &help);
  if (help) {
    printf("%s", tcperf::Usage().c_str());
    return 0;
  }
  if (!e.IsOk()) {
    fprintf(stderr, "error: %s\n\n%s", e.Message().c_str(), tcperf::Usage().c_str());
    return 1;
  }
  // one lane per GPU (a single lane without --gpus/--devices)
  std::unique_ptr<tcperf::MultiSession> s;
  e = tcperf::MultiSession::Create(o, &s);
  if (!e.IsOk()) {
    fprintf(stderr, "error: %s\n", e.Message().c_str());
    return 1;
  }
  const std::string desc = s->Describe();
  tcperf::PrintSettings(o, s->lanes[0]->info, desc);
  std::vector<double> loads;
  if (o.rate_mode && o.request_intervals_file.empty()) {
    for (double r = o.rate_start; r <= o.rate_end + 1e-9; r += o.rate_step) loads.push_back(r);
  } else if (o.rate_mode) {
    loads.push_back(1.0);  // schedule comes from the intervals file
  } else {
    for (uint64_t c = o.conc_start; c <= o.conc_end; c += o.conc_step) loads.push_back(static_cast<double>(c));
  }
  std::vector<tcperf::PointResult> pts;
  e = tcperf::LoadCheckpoint(o, &pts);
  if (!e.IsOk()) {
    fprintf(stderr, "error: %s\n", e.Message().c_str());
    return 1;
  }
  for (const auto& p : pts) {
    printf("Resumed from %s: %s %g (already measured)\n", o.json_file.c_str(),
           o.rate_mode ? "request rate" : "concurrency", p.load);
    tcperf::PrintPoint(o, p);
  }
  tcperf::Profiler prof(o, s->LanePtrs());
  int rc = 0;
  for (double load : loads) {
    bool done = false;
    for (const auto& q : pts) done = done || std::fabs(q.load - load) < 1e-9;
    if (done) continue;
    tcperf::PointResult p;
    e = prof.Profile(load, &p);
    if (!e.IsOk()) {
      fprintf(stderr, "error: %s\n", e.Message().c_str());
      rc = 1;
      break;
    }
    tcperf::PrintPoint(o, p);
    pts.push_back(p);
    // checkpoint after every point: a killed sweep resumes with --resume
    tcperf::Error ce = tcperf::WriteJson(o, pts, desc);
    if (!ce.IsOk()) fprintf(stderr, "error: %s\n", ce.Message().c_str());
    const double lat = o.percentile > 0 ? p.p99_us : p.avg_us;
    if (o.latency_threshold_ms && lat > o.latency_threshold_ms * 1000.0) {
      printf("Measured latency went over the set limit of %lu msec.\n",
             static_cast<unsigned long>(o.latency_threshold_ms));
      break;
    }
  }
  for (auto& l : s->lanes) l->engine->Stop();
  std::sort(pts.begin(), pts.end(),
            [](const tcperf::PointResult& a, const tcperf::PointResult& b) { return a.load < b.load; });
  if (!pts.empty()) tcperf::PrintSummary(o, pts);
  e = tcperf::WriteCsv(o, pts);
  if (!e.IsOk()) fprintf(stderr, "error: %s\n", e.Message().c_str());
  e = tcperf::WriteJson(o, pts, desc);
  if (!e.IsOk()) fprintf(stderr, "error: %s\n", e.Message().c_str());
  s.reset();
  return rc;
}
