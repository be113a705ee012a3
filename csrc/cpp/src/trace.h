// roctx ranges for rocprofv3 --marker-trace (the reference's
// 6-point RequestTimers plus markers around transport, batching and load
// windows).  The roctx library is dlopen'ed on first use and only when
// TC_ROCTX=1, so the clients keep no ROCm link dependency and pay one
// static-pointer check per call otherwise.
#pragma once

#include <dlfcn.h>

#include <cstdlib>
#include <cstring>

namespace triton { namespace client { namespace trace {

struct Roctx {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
  void (*mark)(const char*) = nullptr;
};

inline const Roctx* Lib()
{
  static const Roctx* lib = []() -> const Roctx* {
    const char* e = std::getenv("TC_ROCTX");
    if (!e || std::strcmp(e, "1") != 0) return nullptr;
    static Roctx r;
    for (const char* name : {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4",
                             "libroctx64.so"}) {
      void* h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
      if (!h) continue;
      r.push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
      r.pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
      r.mark = reinterpret_cast<void (*)(const char*)>(dlsym(h, "roctxMarkA"));
      if (r.push && r.pop) return &r;
    }
    return nullptr;
  }();
  return lib;
}

inline void Mark(const char* msg)
{
  if (const Roctx* r = Lib())
    if (r->mark) r->mark(msg);
}

/// RAII roctx range (a no-op unless TC_ROCTX=1 and roctx is loadable).
class Range {
 public:
  explicit Range(const char* msg) : lib_(Lib())
  {
    if (lib_) lib_->push(msg);
  }
  ~Range()
  {
    if (lib_) lib_->pop();
  }
  Range(const Range&) = delete;
  Range& operator=(const Range&) = delete;

 private:
  const Roctx* lib_;
};

}}}  // namespace triton::client::trace
