// The knob registry of libtcamd_hip.so (csrc/kernels/knobs.h).
//
// One table instead of a getenv per launch site: each knob is seeded from
// its environment variable once, then read with a relaxed atomic load at
// every launch, so a test or a tuning tool can switch a path in-process
// (tcamd_knob_set) and put it back.  Names are the environment variable
// names.
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "kernels/knobs.h"

namespace {

struct KnobDef {
  const char* name;
  long long def;
  const char* doc;
};

// order = tcamd::Knob
constexpr KnobDef kDefs[] = {
    {"TCAMD_X3_BM", 0, "K8x 1x1: force the tile rows (32, 64 or 128); 0 picks by problem size"},
    {"TCAMD_X3_SPLITK_BELOW", 192, "K8x 1x1: split K across workgroups when the tiles are fewer than this"},
    {"TCAMD_X3_MAX_SPLITS", 4, "K8x 1x1: most K splits (bs1 0.975 ms at 4 vs 1.005 uncapped)"},
    {"TCAMD_X3_WS", 1, "K8x 1x1: warp-specialised persistent kernel for the dense-layer 1x1s (0: tiled only)"},
    {"TCAMD_X3_WS_MIN", 16384, "K8x 1x1: pixels from which the warp-specialised kernel runs"},
    {"TCAMD_X3_STEM_BPC", 2, "K10x stem: persistent workgroups per CU"},
    {"TCAMD_X3S_BLOCKS", 384, "K13x small-M 1x1: target workgroups (sets the K chunking)"},
    {"TCAMD_X3S_MAX_CHUNKS", 8, "K13x small-M 1x1: most K chunks (float atomics sum them)"},
    {"TCAMD_X3S_SPLIT3", 1, "K13x 3x3 over the 4 input quarters; 0: one block, bitwise reproducible"},
    {"TCAMD_PK_BIG_LIM", (1ll << 31) - (1ll << 20), "K2 BYTES pack: output offset from which blocks take the 64-bit path"},
    {"TCAMD_K3_MODE", 0, "K3 BYTES index: 1 = general walk only (no windowed v3 walk)"},
    {"TCAMD_K17_TM", 0, "K17 GEMM: tile height 128, 192 or 256; 0 picks the one whose persistent grid finishes first"},
    {"TCAMD_K17_DYN", 1, "K17 GEMM: claim tiles from a device counter (1) or walk a fixed tile list per workgroup (0)"},
};
static_assert(sizeof(kDefs) / sizeof(kDefs[0]) == (size_t)tcamd::Knob::kCount, "knob table != enum");

constexpr int kN = (int)tcamd::Knob::kCount;
std::atomic<long long> g_val[kN];
std::once_flag g_once;

void seed() {
  std::call_once(g_once, [] {
    for (int i = 0; i < kN; ++i) {
      long long v = kDefs[i].def;
      if (const char* e = std::getenv(kDefs[i].name)) {
        char* end = nullptr;
        const long long x = std::strtoll(e, &end, 10);
        if (end != e) v = x;
      }
      g_val[i].store(v, std::memory_order_relaxed);
    }
  });
}

int find(const char* name) {
  if (!name) return -1;
  for (int i = 0; i < kN; ++i)
    if (!std::strcmp(kDefs[i].name, name)) return i;
  return -1;
}

}  // namespace

namespace tcamd {
long long knob(Knob k) {
  seed();
  return g_val[(int)k].load(std::memory_order_relaxed);
}
}  // namespace tcamd

extern "C" {

int tcamd_knob_count() { return kN; }

// Knob i: name, default, current value and a one-line description.
int tcamd_knob_info(int i, const char** name, long long* def, long long* value, const char** doc) {
  if (i < 0 || i >= kN) return -1;
  seed();
  if (name) *name = kDefs[i].name;
  if (def) *def = kDefs[i].def;
  if (value) *value = g_val[i].load(std::memory_order_relaxed);
  if (doc) *doc = kDefs[i].doc;
  return 0;
}

// Sets a knob by name; returns 0 (prev = the old value) or -1 for an unknown name.
int tcamd_knob_set(const char* name, long long value, long long* prev) {
  const int i = find(name);
  if (i < 0) return -1;
  seed();
  const long long old = g_val[i].exchange(value, std::memory_order_relaxed);
  if (prev) *prev = old;
  return 0;
}

}  // extern "C"
