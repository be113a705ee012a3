// perf_analyzer multi-GPU lanes.
//
// `--gpus N` builds one Session per GPU: its own protocol clients (one
// connection + I/O thread each), LoadEngine worker thread, HIP stream and
// shared-memory regions registered with that GPU's server (-u url0,url1,...).
// The synthetic request batch is generated ONCE, by K1 on the first GPU's
// stream, and replicated into the other lanes' input regions by a Fanout:
//
//   rccl  X1: one single-process RCCL communicator over the N devices
//         (ncclCommInitAll) and a grouped ncclBroadcast from device 0, one
//         HIP stream per device.  Over xGMI this is RCCL's ring/tree.
//   p2p   X2: a peer-copy star — N-1 hipMemcpyPeerAsync on N-1 streams (each
//         destination pulls over its own xGMI link from the root).
//   host  copies through host memory (system shared memory lanes, or GPUs
//         without peer access).
//
// Every replica is compared byte for byte against the root after the
// fan-out.  The Profiler then measures all lanes over common windows.
#include <algorithm>
#include <cstring>
#include <sstream>

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include "perf.h"

namespace tcperf {

namespace {

Error HipErr(const char* what, hipError_t e)
{
  return Error(std::string(what) + ": " + hipGetErrorString(e));
}

Error NcclErr(const char* what, ncclResult_t r)
{
  return Error(std::string(what) + ": " + ncclGetErrorString(r));
}

}  // namespace

Error Fanout::Create(const std::string& mode, const std::vector<int>& devices, std::unique_ptr<Fanout>* out)
{
  std::unique_ptr<Fanout> f(new Fanout());
  f->mode_ = mode;
  f->devices_ = devices;
  const int n = static_cast<int>(devices.size());
  if (mode == "host" || n <= 1) {
    *out = std::move(f);
    return Error::Success;
  }
  for (int i = 0; i < n; ++i) {
    hipError_t he = hipSetDevice(devices[i]);
    hipStream_t s = nullptr;
    if (he == hipSuccess) he = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (he != hipSuccess) return HipErr("fanout stream", he);
    f->streams_.push_back(s);
  }
  if (mode == "rccl") {
    std::vector<ncclComm_t> comms(n);
    ncclResult_t r = ncclCommInitAll(comms.data(), n, devices.data());
    if (r != ncclSuccess) return NcclErr("ncclCommInitAll", r);
    for (auto c : comms) f->comms_.push_back(c);
  } else if (mode == "p2p") {
    for (int i = 1; i < n; ++i) {
      if (devices[i] == devices[0]) continue;  // same device: a plain D2D copy
      int can = 0;
      hipError_t he = hipDeviceCanAccessPeer(&can, devices[i], devices[0]);
      if (he != hipSuccess) return HipErr("hipDeviceCanAccessPeer", he);
      if (!can)
        return Error("GPU " + std::to_string(devices[i]) + " has no peer access to GPU " + std::to_string(devices[0]) +
                     "; use --fanout rccl|host");
      (void)hipSetDevice(devices[i]);
      he = hipDeviceEnablePeerAccess(devices[0], 0);
      if (he != hipSuccess && he != hipErrorPeerAccessAlreadyEnabled) return HipErr("hipDeviceEnablePeerAccess", he);
      (void)hipGetLastError();  // clear a sticky "already enabled"
    }
  } else {
    return Error("unknown fan-out mode " + mode);
  }
  *out = std::move(f);
  return Error::Success;
}

Fanout::~Fanout()
{
  for (void* c : comms_) (void)ncclCommDestroy(static_cast<ncclComm_t>(c));
  for (void* s : streams_) (void)hipStreamDestroy(static_cast<hipStream_t>(s));
}

Error Fanout::Broadcast(const void* src, const std::vector<void*>& dst, size_t bytes, bool device)
{
  const size_t n = devices_.size();
  const uint64_t t0 = NowNs();
  if (!device) {
    for (size_t i = 1; i < n; ++i) memcpy(dst[i], src, bytes);
  } else if (mode_ == "rccl") {
    // X1: grouped broadcast, root = lane 0 (in place on the root's region)
    ncclResult_t r = ncclGroupStart();
    for (size_t i = 0; i < n && r == ncclSuccess; ++i) {
      void* buf = i == 0 ? const_cast<void*>(src) : dst[i];
      r = ncclBroadcast(buf, buf, bytes, ncclUint8, 0, static_cast<ncclComm_t>(comms_[i]),
                        static_cast<hipStream_t>(streams_[i]));
    }
    ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess) return NcclErr("ncclBroadcast", r);
    if (r2 != ncclSuccess) return NcclErr("ncclGroupEnd", r2);
  } else if (mode_ == "p2p") {
    // X2: star — every destination stream pulls its copy concurrently
    for (size_t i = 1; i < n; ++i) {
      (void)hipSetDevice(devices_[i]);
      hipError_t he = hipMemcpyPeerAsync(dst[i], devices_[i], src, devices_[0], bytes,
                                         static_cast<hipStream_t>(streams_[i]));
      if (he != hipSuccess) return HipErr("hipMemcpyPeerAsync", he);
    }
  } else {
    // host staging: one D2H, N-1 H2D
    std::vector<uint8_t> tmp(bytes);
    (void)hipSetDevice(devices_[0]);
    hipError_t he = hipMemcpy(tmp.data(), src, bytes, hipMemcpyDeviceToHost);
    for (size_t i = 1; i < n && he == hipSuccess; ++i) {
      (void)hipSetDevice(devices_[i]);
      he = hipMemcpy(dst[i], tmp.data(), bytes, hipMemcpyHostToDevice);
    }
    if (he != hipSuccess) return HipErr("host fan-out copy", he);
  }
  for (size_t i = 0; i < streams_.size(); ++i) {
    (void)hipSetDevice(devices_[i]);
    hipError_t he = hipStreamSynchronize(static_cast<hipStream_t>(streams_[i]));
    if (he != hipSuccess) return HipErr("fan-out sync", he);
  }
  last_us_ = (NowNs() - t0) / 1000.0;
  total_bytes_ += static_cast<double>(bytes) * (n - 1);
  return Error::Success;
}

// ============================================================================
// MultiSession
// ============================================================================
static Error SameBytes(const DataSet::RegionView& a, const DataSet::RegionView& b)
{
  if (a.bytes != b.bytes) return Error("replica size mismatch");
  std::vector<uint8_t> x(a.bytes), y(b.bytes);
  if (a.device) {
    (void)hipSetDevice(a.dev);
    hipError_t he = hipMemcpy(x.data(), a.ptr, a.bytes, hipMemcpyDeviceToHost);
    if (he == hipSuccess) {
      (void)hipSetDevice(b.dev);
      he = hipMemcpy(y.data(), b.ptr, b.bytes, hipMemcpyDeviceToHost);
    }
    if (he != hipSuccess) return HipErr("replica read-back", he);
  } else {
    memcpy(x.data(), a.ptr, a.bytes);
    memcpy(y.data(), b.ptr, b.bytes);
  }
  if (x != y) return Error("replica differs from the root region");
  return Error::Success;
}

Error MultiSession::Create(const Options& o, std::unique_ptr<MultiSession>* out)
{
  std::unique_ptr<MultiSession> ms(new MultiSession());
  ms->opts = o;
  const std::vector<int> devs = o.devices.empty() ? std::vector<int>{o.device} : o.devices;
  const size_t n = devs.size();
  const bool shm = o.shared_memory != "none";
  // per-lane slot capacity: the largest share any lane gets
  uint64_t lane_conc = o.conc_end;
  if (n > 1 && !o.load_per_gpu && !o.rate_mode) lane_conc = (o.conc_end + n - 1) / n;
  for (size_t i = 0; i < n; ++i) {
    Options lo = o;
    lo.device = devs[i];
    lo.url = o.urls.empty() ? o.url : o.urls[i % o.urls.size()];
    lo.conc_end = std::max<uint64_t>(1, lane_conc);
    lo.collect_metrics = false;  // the Profiler samples per lane
    std::unique_ptr<Session> s;
    // replicas: regions are created and registered, the fan-out fills them
    Error e = Session::Create(lo, &s, /*fill_inputs=*/i == 0 || !shm);
    if (!e.IsOk()) return Error("GPU " + std::to_string(devs[i]) + " (" + lo.url + "): " + e.Message());
    ms->lanes.push_back(std::move(s));
  }
  if (n > 1 && shm) {
    std::string mode = o.fanout;
    if (mode == "auto") mode = o.shared_memory == "hip" ? "rccl" : "host";
    if (o.shared_memory != "hip") mode = "host";
    Error e = Fanout::Create(mode, devs, &ms->fanout);
    if (!e.IsOk()) return e;
    const auto root = ms->lanes[0]->data->InputRegions();
    uint64_t t0 = NowNs();
    for (size_t r = 0; r < root.size(); ++r) {
      std::vector<void*> dst(n, nullptr);
      for (size_t i = 1; i < n; ++i) {
        const auto reg = ms->lanes[i]->data->InputRegions();
        if (reg.size() != root.size() || reg[r].bytes != root[r].bytes)
          return Error("lane " + std::to_string(i) + " input regions do not match the root's");
        dst[i] = reg[r].ptr;
      }
      e = ms->fanout->Broadcast(root[r].ptr, dst, root[r].bytes, root[r].device);
      if (!e.IsOk()) return e;
    }
    ms->fanout_us = (NowNs() - t0) / 1000.0;
    for (size_t i = 1; i < n; ++i) {
      const auto reg = ms->lanes[i]->data->InputRegions();
      for (size_t r = 0; r < root.size(); ++r) {
        e = SameBytes(root[r], reg[r]);
        if (!e.IsOk()) return Error("fan-out to GPU " + std::to_string(devs[i]) + ": " + e.Message());
      }
    }
    ms->replicas_verified = true;
  }
  *out = std::move(ms);
  return Error::Success;
}

std::vector<Session*> MultiSession::LanePtrs() const
{
  std::vector<Session*> v;
  for (const auto& l : lanes) v.push_back(l.get());
  return v;
}

std::string MultiSession::Describe() const
{
  std::ostringstream d;
  d << lanes[0]->data->Describe();
  if (lanes.size() > 1) {
    d << "; " << lanes.size() << " GPUs [";
    for (size_t i = 0; i < lanes.size(); ++i) d << (i ? "," : "") << lanes[i]->opts.device;
    d << "]";
    if (fanout) {
      char b[160];
      snprintf(b, sizeof(b), ", inputs fanned out by %s in %.0f us (%.2f MB to each replica), replicas %s",
               fanout->Mode().c_str(), fanout_us, fanout->TotalBytes() / (lanes.size() - 1) / 1e6,
               replicas_verified ? "verified" : "unverified");
      d << b;
    }
    d << (opts.load_per_gpu ? ", full load per GPU" : ", load split over GPUs");
  }
  return d.str();
}

MultiSession::~MultiSession()
{
  for (auto& l : lanes)
    if (l && l->engine) l->engine->Stop();
  lanes.clear();
  fanout.reset();
}

}  // namespace tcperf
