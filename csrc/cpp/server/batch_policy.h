// Dynamic-batcher dispatch policy of tcserve's native batcher, as pure
// functions of a snapshot of the model's queue state (taken under the model
// lock).  Server::Worker re-evaluates WaitUntil() after every wake-up and
// takes TakeLimit() rows once it returns 0; tcserve_batch_policy_sim() (C
// API) runs the same two functions in a discrete-event simulation of scripted
// arrivals, which is how the rules are unit-tested without threads or clocks.
//
// Rules (Triton dynamic-batcher semantics plus three of ours):
//   * a batch of the largest preferred size (or max_batch) dispatches at once;
//     otherwise a worker waits up to the queue delay, measured from the oldest
//     queued request's arrival, for one;
//   * idle-aware: with every instance idle the queue goes out now (a lone
//     request never waits out the delay on an idle GPU);
//   * pipelined (per model, opt-in): an instance is free and the queue holds
//     as many rows as the last batch carried -> go now (in a closed loop the
//     delay cannot build a bigger batch);
//   * staggered (full batches only): with another instance busy, a batch
//     starts no sooner than ema(exec) / instances after the previous start,
//     so closed-loop load settles into instances offset by a fraction of a
//     batch instead of starting together.
#pragma once

#include <algorithm>
#include <cstdint>
#include <vector>

namespace tcserve {

struct BatchPolicyConfig {
  int max_batch = 0;           // 0: no batching (one request per execution)
  uint64_t delay_ns = 0;       // max_queue_delay
  std::vector<int> preferred;  // ascending
  bool idle_dispatch = true;
  bool pipelined = false;
  bool stagger = true;
  int instances = 1;

  int Cap() const { return max_batch > 0 ? max_batch : 1; }
  int PrefMax() const { return preferred.empty() ? Cap() : std::min(Cap(), preferred.back()); }
};

struct BatchPolicyState {
  uint64_t now_ns = 0;
  uint64_t front_arrive_ns = 0;  // the oldest queued request
  int q_rows = 0;                // > 0
  int busy = 0;                  // instances executing
  int last_rows = 0;             // rows of the last dispatched batch
  double ema_exec_ns = 0;        // EMA of a batch's execution wall time
  uint64_t last_start_ns = 0;    // the last batch's start
};

// 0: dispatch now; otherwise the time to re-evaluate at (or on any change of
// the queue or of the busy count, whichever comes first).
inline uint64_t WaitUntil(const BatchPolicyConfig& c, const BatchPolicyState& s)
{
  const int pref_max = c.PrefMax();
  if (c.max_batch > 0 && c.delay_ns > 0 && s.q_rows < pref_max) {
    const bool idle_go = c.idle_dispatch && s.busy == 0;
    const bool pipe_go = c.pipelined && s.busy < c.instances && s.last_rows > 0 && s.q_rows >= s.last_rows;
    const uint64_t deadline = s.front_arrive_ns + c.delay_ns;
    if (!idle_go && !pipe_go && s.now_ns < deadline) return deadline;
  }
  if (c.stagger && c.instances > 1 && s.busy > 0 && s.ema_exec_ns > 0 && s.q_rows >= pref_max) {
    const uint64_t earliest = s.last_start_ns + static_cast<uint64_t>(s.ema_exec_ns / c.instances);
    if (s.now_ns < earliest) return earliest;
  }
  return 0;
}

// Rows the dispatched batch may carry: the largest preferred size the queue
// fills (so pipelined instances keep alternating), else the cap.  The worker
// then takes whole requests in arrival order while they fit (at least one).
inline int TakeLimit(const BatchPolicyConfig& c, int q_rows)
{
  const int cap = c.Cap();
  for (auto it = c.preferred.rbegin(); it != c.preferred.rend(); ++it)
    if (*it <= q_rows && *it <= cap) return *it;
  return cap;
}

}  // namespace tcserve
