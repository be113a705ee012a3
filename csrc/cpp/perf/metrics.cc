// GPU metrics for perf_analyzer --collect-metrics ("optional
// GPU metrics"): the amdgpu driver's sysfs counters of the MI355X under test
// — busy percent, board power, VRAM in use — sampled every
// --metrics-interval ms on a background thread while a sweep point is
// measured.  No ROCm library or server endpoint is needed, so the sampler
// also works against a remote server when the tool runs on the GPU host.
#include <dirent.h>
#include <limits.h>
#include <stdlib.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <fstream>
#include <string>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "perf.h"

namespace tcperf {

namespace {

bool ReadU64(const std::string& path, uint64_t* v)
{
  std::ifstream f(path);
  if (!f) return false;
  unsigned long long x = 0;
  f >> x;
  if (!f) return false;
  *v = x;
  return true;
}

std::string ReadStr(const std::string& path)
{
  std::ifstream f(path);
  std::string s;
  if (f) std::getline(f, s);
  return s;
}

// amdgpu PCI device directories (vendor 0x1002 with gpu_busy_percent), in PCI
// address order — the order HIP enumerates devices in.
std::vector<std::string> AmdGpus(const std::string& root)
{
  std::vector<std::string> out;
  DIR* d = opendir(root.c_str());
  if (!d) return out;
  while (dirent* e = readdir(d)) {
    const std::string name = e->d_name;
    if (name.rfind("card", 0) != 0 || name.find('-') != std::string::npos) continue;
    const std::string dev = root + "/" + name + "/device";
    if (ReadStr(dev + "/vendor") != "0x1002") continue;
    uint64_t busy;
    if (!ReadU64(dev + "/gpu_busy_percent", &busy)) continue;
    out.push_back(dev);
  }
  closedir(d);
  std::sort(out.begin(), out.end(), [](const std::string& a, const std::string& b) {
    char ra[4096] = {0}, rb[4096] = {0};
    if (!realpath(a.c_str(), ra) || !realpath(b.c_str(), rb)) return a < b;
    return std::string(ra) < std::string(rb);
  });
  return out;
}

std::string PowerFile(const std::string& dev)
{
  DIR* d = opendir((dev + "/hwmon").c_str());
  if (!d) return std::string();
  std::string found;
  while (dirent* e = readdir(d)) {
    const std::string h = e->d_name;
    if (h.rfind("hwmon", 0) != 0) continue;
    for (const char* f : {"power1_average", "power1_input"}) {
      uint64_t v;
      const std::string p = dev + "/hwmon/" + h + "/" + f;
      if (ReadU64(p, &v)) {
        found = p;
        break;
      }
    }
    if (!found.empty()) break;
  }
  closedir(d);
  return found;
}

std::string Lower(std::string s)
{
  for (auto& c : s) c = static_cast<char>(tolower(static_cast<unsigned char>(c)));
  return s;
}

// PCI address ("0000:75:00.0", lower case) of HIP device `device`, or "".
std::string HipPciAddress(int device)
{
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) != hipSuccess) return std::string();
  return Lower(bus);
}

}  // namespace

GpuMetrics::GpuMetrics(int device, uint64_t interval_ms, const std::string& sysfs_root)
    : interval_ms_(std::max<uint64_t>(10, interval_ms))
{
  const auto gpus = AmdGpus(sysfs_root.empty() ? "/sys/class/drm" : sysfs_root);
  if (sysfs_root.empty()) {
    // a container or HIP_VISIBLE_DEVICES can hide cards, so HIP device N is
    // not necessarily the N-th amdgpu card in sysfs: match it by PCI address
    const std::string pci = HipPciAddress(device);
    for (const auto& g : gpus) {
      char rp[4096] = {0};
      if (pci.empty() || !realpath(g.c_str(), rp)) continue;
      const std::string r = Lower(rp);
      if (r.size() >= pci.size() && r.compare(r.size() - pci.size(), pci.size(), pci) == 0) {
        dev_ = g;
        break;
      }
    }
  }
  if (dev_.empty()) {
    if (device < 0 || device >= static_cast<int>(gpus.size())) return;
    dev_ = gpus[device];
  }
  power_file_ = PowerFile(dev_);
}

GpuMetrics::~GpuMetrics() { Stop(); }

bool GpuMetrics::Available() const { return !dev_.empty(); }

void GpuMetrics::Start()
{
  if (!Available() || running_) return;
  {
    std::lock_guard<std::mutex> lk(mu_);
    samples_ = 0;
    busy_sum_ = power_sum_ = 0;
    mem_max_ = 0;
    stop_ = false;
  }
  running_ = true;
  th_ = std::thread([this] {
    std::unique_lock<std::mutex> lk(mu_);
    while (!stop_) {
      lk.unlock();
      uint64_t busy = 0, power = 0, mem = 0;
      const bool ok = ReadU64(dev_ + "/gpu_busy_percent", &busy);
      if (!power_file_.empty()) ReadU64(power_file_, &power);
      ReadU64(dev_ + "/mem_info_vram_used", &mem);
      lk.lock();
      if (ok) {
        samples_++;
        busy_sum_ += static_cast<double>(busy);
        power_sum_ += static_cast<double>(power) * 1e-6;  // uW -> W
        mem_max_ = std::max(mem_max_, mem);
      }
      cv_.wait_for(lk, std::chrono::milliseconds(interval_ms_), [this] { return stop_; });
    }
  });
}

void GpuMetrics::Stop()
{
  if (!running_) return;
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
    cv_.notify_all();
  }
  th_.join();
  running_ = false;
}

bool GpuMetrics::Summary(double* util_pct, double* power_w, double* mem_mib) const
{
  std::lock_guard<std::mutex> lk(mu_);
  if (!samples_) return false;
  *util_pct = busy_sum_ / samples_;
  *power_w = power_sum_ / samples_;
  *mem_mib = static_cast<double>(mem_max_) / (1024.0 * 1024.0);
  return true;
}

}  // namespace tcperf
