// perf_analyzer LoadEngine: closed-loop concurrency, open-loop request rate,
// fixed-count runs; sync, async and gRPC-streaming issue paths.
#include <time.h>

#include <algorithm>
#include <cmath>
#include <fstream>
#include <random>

#include "perf.h"

namespace tcperf {

LoadEngine::LoadEngine(const Options& o, Backend* be, DataSet* data, size_t max_slots)
    : o_(o), be_(be), data_(data), slots_(std::max<size_t>(1, max_slots))
{
  for (auto& s : slots_) {
    s.opt = InferOptions(o.model);
    s.opt.model_version_ = o.version;
    for (const auto& kv : o.request_parameters) s.opt.request_parameters[kv.first] = kv.second;  // --request-parameter
  }
  if (!o.request_intervals_file.empty()) {
    std::ifstream f(o.request_intervals_file);
    uint64_t us;
    while (f >> us) intervals_ns_.push_back(us * 1000);
  }
  // async requests spread over several protocol clients (one connection and
  // one I/O thread each), so neither side funnels every tensor through one
  // socket: slot i uses client i % n (--num-clients; auto = min(slots, 4))
  if (o.async && !o.streaming) {
    size_t n = o.num_clients > 0 ? static_cast<size_t>(o.num_clients) : std::min<size_t>(slots_.size(), 4);
    n = std::max<size_t>(1, std::min(n, slots_.size()));
    clients_.push_back(be_);
    for (size_t i = 1; i < n; ++i) {
      std::unique_ptr<Backend> b;
      if (!Backend::Create(o_, &b).IsOk()) break;
      clients_.push_back(b.get());
      owned_.push_back(std::move(b));
    }
  }
  if (o.async || o.streaming) worker_ = std::thread(&LoadEngine::Worker, this);
}

LoadEngine::~LoadEngine()
{
  Stop();
  {
    std::lock_guard<std::mutex> lk(mu_);
    exiting_ = true;
  }
  cv_.notify_all();
  if (worker_.joinable()) worker_.join();
  clients_.clear();
  owned_.clear();  // after the worker: completions may still reference them
}

void LoadEngine::Stop()
{
  {
    std::lock_guard<std::mutex> lk(mu_);
    target_conc_ = 0;
    fixed_left_ = 0;
  }
  rate_gen_++;
  if (rate_thread_.joinable()) rate_thread_.join();
  // wait for in-flight requests to drain (bounded)
  const uint64_t t0 = NowNs();
  while (in_flight_.load() > 0 && NowNs() - t0 < 30ull * 1000000000ull) {
    struct timespec ts = {0, 1000000};
    nanosleep(&ts, nullptr);
  }
  stop_ = true;
  cv_.notify_all();
  for (auto& t : sync_threads_)
    if (t.joinable()) t.join();
  sync_threads_.clear();
  stop_ = false;
  if (streaming_) {
    be_->StopStream();
    streaming_ = false;
  }
}

void LoadEngine::PrepareSequence(Slot* s)
{
  if (!seq_model_) return;
  if (s->seq_pos == 0) {
    const uint64_t span = o_.seq_id_end - o_.seq_id_start;
    s->seq_id = o_.seq_id_start + (next_seq_++ % span);
  }
  s->opt.sequence_id_ = s->seq_id;
  s->opt.sequence_start_ = s->seq_pos == 0;
  s->opt.sequence_end_ = s->seq_pos == o_.sequence_length - 1;
  s->seq_pos = (s->seq_pos + 1) % o_.sequence_length;
}

void LoadEngine::OnComplete(size_t slot, uint64_t start_ns, InferResult* r)
{
  Record rec{start_ns, NowNs(), true};
  if (r) {
    Error e = r->RequestStatus();
    if (!e.IsOk()) {
      rec.ok = false;
      std::lock_guard<std::mutex> lk(rec_mu_);
      if (first_error_.empty()) first_error_ = e.Message();
    }
    delete r;
  } else {
    rec.ok = false;
  }
  // runs on a client's io thread: notify under the lock, since the engine
  // (and cv_) may be destroyed as soon as the worker has drained done_
  std::lock_guard<std::mutex> lk(mu_);
  done_.emplace_back(slot, rec);
  cv_.notify_one();
}

Error LoadEngine::Issue(size_t slot)
{
  Slot& s = slots_[slot];
  PrepareSequence(&s);
  const uint64_t t = NowNs();
  in_flight_++;
  Error e;
  if (streaming_) {
    std::string id;
    {
      std::lock_guard<std::mutex> lk(stream_mu_);
      id = std::to_string(++stream_counter_);
      stream_ids_[id] = {slot, t};
    }
    s.opt.request_id_ = id;
    e = be_->StreamInfer(s.opt, data_->Inputs(issued_++, slot), data_->Outputs(slot));
    if (!e.IsOk()) {
      std::lock_guard<std::mutex> lk(stream_mu_);
      stream_ids_.erase(id);
    }
  } else {
    Backend* be = clients_.empty() ? be_ : clients_[slot % clients_.size()];
    e = be->AsyncInfer([this, slot, t](InferResult* r) { OnComplete(slot, t, r); }, s.opt, data_->Inputs(issued_++, slot),
                       data_->Outputs(slot));
  }
  if (!e.IsOk()) {
    {
      std::lock_guard<std::mutex> lk(rec_mu_);
      if (first_error_.empty()) first_error_ = e.Message();
    }
    OnComplete(slot, t, nullptr);  // counts as a failed request; keeps the accounting whole
  }
  return e;
}

Error LoadEngine::EnsureStream()
{
  if (!o_.streaming || streaming_) return Error::Success;
  Error e = be_->StartStream([this](InferResult* r) {
    std::string id;
    if (r) r->Id(&id);
    size_t slot = 0;
    uint64_t t = 0;
    bool found = false;
    {
      std::lock_guard<std::mutex> lk(stream_mu_);
      auto it = stream_ids_.find(id);
      if (it != stream_ids_.end()) {
        slot = it->second.first;
        t = it->second.second;
        stream_ids_.erase(it);
        found = true;
      }
    }
    if (found) {
      OnComplete(slot, t, r);
    } else {
      delete r;  // extra responses of a decoupled model
    }
  });
  if (e.IsOk()) streaming_ = true;
  return e;
}

void LoadEngine::Worker()
{
  std::unique_lock<std::mutex> lk(mu_);
  while (true) {
    cv_.wait(lk, [&] { return exiting_ || !done_.empty() || !pending_start_.empty(); });
    if (exiting_ && done_.empty() && pending_start_.empty()) return;
    std::vector<size_t> to_issue;
    to_issue.swap(pending_start_);
    while (!done_.empty()) {
      auto d = done_.front();
      done_.pop_front();
      in_flight_--;
      {
        std::lock_guard<std::mutex> rl(rec_mu_);
        records_.push_back(d.second);
        if (fixed_lat_) fixed_lat_->push_back(d.second.end_ns - d.second.start_ns);
        if (fixed_end_) fixed_end_->push_back(d.second.end_ns);
      }
      const size_t slot = d.first;
      slots_[slot].busy = false;
      if (rate_active_) continue;  // open loop: the rate thread issues
      const bool again = fixed_mode_ ? (fixed_left_ > 0) : (slot < target_conc_);
      if (again) {
        if (fixed_mode_) fixed_left_--;
        to_issue.push_back(slot);
      }
    }
    if (to_issue.empty()) {
      fixed_cv_.notify_all();
      continue;
    }
    for (size_t s : to_issue) slots_[s].busy = true;
    lk.unlock();
    for (size_t s : to_issue) Issue(s);
    lk.lock();
    fixed_cv_.notify_all();
  }
}

void LoadEngine::SyncLoop(size_t slot)
{
  std::unique_ptr<Backend> be;
  Error e = Backend::Create(o_, &be);
  if (!e.IsOk()) {
    std::lock_guard<std::mutex> lk(rec_mu_);
    if (first_error_.empty()) first_error_ = e.Message();
    return;
  }
  while (!stop_) {
    {
      std::unique_lock<std::mutex> lk(mu_);
      if (fixed_mode_) {
        if (fixed_left_ == 0) break;
        fixed_left_--;
      } else if (slot >= target_conc_) {
        break;
      }
    }
    Slot& s = slots_[slot];
    PrepareSequence(&s);
    InferResult* r = nullptr;
    const uint64_t t = NowNs();
    in_flight_++;
    e = be->SyncInfer(&r, s.opt, data_->Inputs(issued_++, slot), data_->Outputs(slot));
    Record rec{t, NowNs(), e.IsOk()};
    if (r) {
      if (!r->RequestStatus().IsOk()) rec.ok = false;
      delete r;
    }
    in_flight_--;
    {
      std::lock_guard<std::mutex> lk(rec_mu_);
      if (!rec.ok && first_error_.empty()) first_error_ = e.IsOk() ? "request failed" : e.Message();
      records_.push_back(rec);
      if (fixed_lat_) fixed_lat_->push_back(rec.end_ns - rec.start_ns);
      if (fixed_end_) fixed_end_->push_back(rec.end_ns);
    }
    fixed_cv_.notify_all();
  }
  std::lock_guard<std::mutex> lk(mu_);
  slots_[slot].busy = false;
  fixed_cv_.notify_all();
}

Error LoadEngine::SetConcurrency(size_t n)
{
  rate_gen_++;
  if (rate_thread_.joinable()) rate_thread_.join();
  rate_active_ = false;
  if (n > slots_.size()) return Error("concurrency exceeds the prepared slot count");
  Error e = EnsureStream();
  if (!e.IsOk()) return e;
  std::unique_lock<std::mutex> lk(mu_);
  fixed_mode_ = false;
  target_conc_ = n;
  if (!o_.async && !o_.streaming) {
    for (size_t i = 0; i < n; ++i)
      if (!slots_[i].busy) {
        slots_[i].busy = true;
        sync_threads_.emplace_back(&LoadEngine::SyncLoop, this, i);
      }
    return Error::Success;
  }
  for (size_t i = 0; i < n; ++i)
    if (!slots_[i].busy) {
      slots_[i].busy = true;
      pending_start_.push_back(i);
    }
  lk.unlock();
  cv_.notify_one();
  return Error::Success;
}

Error LoadEngine::RunFixed(size_t concurrency, uint64_t total, std::vector<uint64_t>* lat_ns, double* elapsed_s,
                          std::vector<uint64_t>* end_ns)
{
  if (concurrency == 0 || concurrency > slots_.size()) return Error("bad concurrency for the prepared slots");
  // quiesce any previous load
  SetConcurrency(0);
  {
    std::unique_lock<std::mutex> lk(mu_);
    fixed_cv_.wait(lk, [&] { return in_flight_.load() == 0 && done_.empty(); });
  }
  for (auto& t : sync_threads_)
    if (t.joinable()) t.join();
  sync_threads_.clear();
  Error e = EnsureStream();
  if (!e.IsOk()) return e;
  lat_ns->clear();
  lat_ns->reserve(total);
  if (end_ns) {
    end_ns->clear();
    end_ns->reserve(total);
  }
  const size_t first = std::min<uint64_t>(concurrency, total);
  std::unique_lock<std::mutex> lk(mu_);
  fixed_mode_ = true;
  fixed_left_ = total - first;
  {
    std::lock_guard<std::mutex> rl(rec_mu_);
    fixed_lat_ = lat_ns;
    fixed_end_ = end_ns;
  }
  const uint64_t t0 = NowNs();
  if (!o_.async && !o_.streaming) {
    fixed_left_ = total;
    for (size_t i = 0; i < first; ++i) {
      slots_[i].busy = true;
      sync_threads_.emplace_back(&LoadEngine::SyncLoop, this, i);
    }
  } else {
    for (size_t i = 0; i < first; ++i) {
      slots_[i].busy = true;
      pending_start_.push_back(i);
    }
    cv_.notify_one();
  }
  fixed_cv_.wait(lk, [&] {
    std::lock_guard<std::mutex> rl(rec_mu_);
    return lat_ns->size() >= total || (!first_error_.empty() && in_flight_.load() == 0 && fixed_left_ == 0);
  });
  const uint64_t t1 = NowNs();
  fixed_mode_ = false;
  fixed_left_ = 0;
  {
    std::lock_guard<std::mutex> rl(rec_mu_);
    fixed_lat_ = nullptr;
    fixed_end_ = nullptr;
  }
  if (end_ns)
    for (auto& t : *end_ns) t = t > t0 ? t - t0 : 0;
  lk.unlock();
  for (auto& t : sync_threads_)
    if (t.joinable()) t.join();
  sync_threads_.clear();
  *elapsed_s = (t1 - t0) * 1e-9;
  std::string err = FirstError();
  if (lat_ns->size() < total) return Error("fixed run ended early: " + err);
  return Error::Success;
}

void LoadEngine::RateLoop(double rate, uint64_t gen)
{
  std::mt19937_64 rng(o_.seed + 17);
  std::exponential_distribution<double> expo(rate);
  size_t idx = 0, slot = 0;
  uint64_t next = NowNs();
  while (rate_gen_.load() == gen) {
    uint64_t gap;
    if (!intervals_ns_.empty()) gap = intervals_ns_[idx++ % intervals_ns_.size()];
    else if (o_.distribution == "poisson") gap = static_cast<uint64_t>(expo(rng) * 1e9);
    else gap = static_cast<uint64_t>(1e9 / rate);
    next += gap;
    // Open loop: send times do not wait for responses.  If the scheduler itself
    // fell behind (descheduled, CPU-starved host) by more than a bounded lag,
    // drop the backlog instead of bursting it into the next window, which
    // would report a rate the schedule never asked for.
    {
      const uint64_t now = NowNs();
      const uint64_t max_lag = std::max<uint64_t>(20ull * 1000000ull, 4 * gap);
      if (now > next + max_lag) {
        delayed_.fetch_add(1);
        next = now;
      }
    }
    // sleep until the scheduled send time (not blocked by responses)
    while (true) {
      const uint64_t now = NowNs();
      if (now >= next || rate_gen_.load() != gen) break;
      const uint64_t d = next - now;
      struct timespec ts = {static_cast<time_t>(d / 1000000000ull), static_cast<long>(d % 1000000000ull)};
      nanosleep(&ts, nullptr);
    }
    if (rate_gen_.load() != gen) break;
    Issue(slot);
    slot = (slot + 1) % slots_.size();
  }
}

Error LoadEngine::SetRequestRate(double rate)
{
  SetConcurrency(0);
  if (!o_.async && !o_.streaming) return Error("request-rate mode needs async or streaming requests");
  Error e = EnsureStream();
  if (!e.IsOk()) return e;
  rate_active_ = true;
  const uint64_t gen = ++rate_gen_;
  rate_thread_ = std::thread(&LoadEngine::RateLoop, this, rate, gen);
  return Error::Success;
}

Error LoadEngine::StartLoop(size_t concurrency)
{
  if (concurrency == 0 || concurrency > slots_.size()) return Error("bad concurrency for the prepared slots");
  Error e = StopLoop();
  if (!e.IsOk()) return e;
  return SetConcurrency(concurrency);
}

Error LoadEngine::StopLoop()
{
  Error e = SetConcurrency(0);
  if (!e.IsOk()) return e;
  std::unique_lock<std::mutex> lk(mu_);
  const bool drained = fixed_cv_.wait_for(lk, std::chrono::seconds(30),
                                          [&] { return in_flight_.load() == 0 && done_.empty(); });
  lk.unlock();
  for (auto& t : sync_threads_)
    if (t.joinable()) t.join();
  sync_threads_.clear();
  return drained ? Error::Success : Error("requests still in flight 30 s after the loop stopped");
}

Error LoadEngine::WaitCompleted(size_t target, double timeout_s)
{
  std::unique_lock<std::mutex> lk(mu_);
  bool failed = false;
  const bool ok = fixed_cv_.wait_for(lk, std::chrono::duration<double>(timeout_s), [&] {
    std::lock_guard<std::mutex> rl(rec_mu_);
    failed = !first_error_.empty();
    return failed || records_.size() >= target;
  });
  lk.unlock();
  if (failed) return Error("request failed during the loop: " + FirstError());
  return ok ? Error::Success : Error("loop timed out waiting for completions");
}

size_t LoadEngine::Snapshot(size_t since, std::vector<Record>* out)
{
  std::lock_guard<std::mutex> lk(rec_mu_);
  if (since < records_.size()) out->insert(out->end(), records_.begin() + since, records_.end());
  return records_.size();
}

size_t LoadEngine::CompletedCount()
{
  std::lock_guard<std::mutex> lk(rec_mu_);
  return records_.size();
}

std::string LoadEngine::FirstError()
{
  std::lock_guard<std::mutex> lk(rec_mu_);
  return first_error_;
}

}  // namespace tcperf
