// common.cpp — error string and the grow-only device workspace cache.
#include "common.hpp"

#include <cstdarg>
#include <cstdio>
#include <map>
#include <mutex>
#include <utility>
#include <vector>

namespace acoss {

static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

void clear_error() { g_err[0] = '\0'; }

const char* last_error() { return g_err; }

namespace {
std::mutex g_mu;
struct Buf {
  void* ptr = nullptr;
  size_t bytes = 0;
};
std::map<std::pair<int, int>, Buf> g_ws;  // (device, slot) -> buffer
}  // namespace

void* workspace(int slot, size_t bytes) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    set_error("workspace: hipGetDevice failed");
    return nullptr;
  }
  std::lock_guard<std::mutex> lk(g_mu);
  Buf& b = g_ws[{dev, slot}];
  if (b.bytes >= bytes && b.ptr) return b.ptr;
  if (b.ptr) {
    // Growth: the old buffer may still be read by queued work on some stream.
    if (hipDeviceSynchronize() != hipSuccess || hipFree(b.ptr) != hipSuccess) {
      set_error("workspace: failed to release slot %d", slot);
      return nullptr;
    }
    b.ptr = nullptr;
    b.bytes = 0;
  }
  const size_t want = align_up(bytes < 256 ? 256 : bytes, 1 << 20);
  if (hipMalloc(&b.ptr, want) != hipSuccess) {
    b.ptr = nullptr;
    set_error("workspace: hipMalloc(%zu) failed for slot %d", want, slot);
    return nullptr;
  }
  b.bytes = want;
  return b.ptr;
}

// One extra stream and a few timing-free events per device, for overlapping independent
// sub-batches inside one ABI call (the caller's stream stays the ordering point).
hipStream_t side_stream(int idx) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  static std::map<std::pair<int, int>, hipStream_t> streams;
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = streams.find({dev, idx});
  if (it != streams.end()) return it->second;
  hipStream_t st = nullptr;
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return nullptr;
  streams[{dev, idx}] = st;
  return st;
}

hipEvent_t sync_event(int idx) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  static std::map<std::pair<int, int>, hipEvent_t> evs;
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = evs.find({dev, idx});
  if (it != evs.end()) return it->second;
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
  evs[{dev, idx}] = e;
  return e;
}

int release_all_workspaces() {
  std::lock_guard<std::mutex> lk(g_mu);
  if (hipDeviceSynchronize() != hipSuccess) return ACOSS_E_HIP;
  for (auto& kv : g_ws)
    if (kv.second.ptr) (void)hipFree(kv.second.ptr);
  g_ws.clear();
  return ACOSS_OK;
}

namespace {
struct PhaseRec {
  int phase;
  hipEvent_t a, b;
};
bool g_prof = false;
std::vector<PhaseRec> g_recs;
std::vector<hipEvent_t> g_pool;
PhaseRec g_open[PH_COUNT];
const char* kPhaseNames[PH_COUNT] = {"prep",      "oti",     "select_rows", "select_cols", "crp_mask", "dp_qmax",
                                     "dp_dmax",   "sw",      "csm",         "binarize",    "wcsm",     "simple_mp",
                                     "sweep"};
hipEvent_t get_event() {
  if (!g_pool.empty()) {
    hipEvent_t e = g_pool.back();
    g_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}
}  // namespace

bool profiling() { return g_prof; }

void prof_begin(int phase, hipStream_t s) {
  if (!g_prof) return;
  std::lock_guard<std::mutex> lk(g_mu);
  g_open[phase].phase = phase;
  g_open[phase].a = get_event();
  (void)hipEventRecord(g_open[phase].a, s);
}

void prof_end(int phase, hipStream_t s) {
  if (!g_prof) return;
  std::lock_guard<std::mutex> lk(g_mu);
  PhaseRec r = g_open[phase];
  r.b = get_event();
  (void)hipEventRecord(r.b, s);
  g_recs.push_back(r);
}

}  // namespace acoss

using namespace acoss;

// Enable (1) / disable (0) phase timing; enabling clears what was recorded.
extern "C" int acoss_profile_enable(int on) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_prof = on != 0;
  for (auto& r : g_recs) {
    g_pool.push_back(r.a);
    g_pool.push_back(r.b);
  }
  g_recs.clear();
  return ACOSS_OK;
}

// Synchronises the recorded events and writes, per phase, the total milliseconds and the
// number of launches recorded. Returns the number of phases (PH_COUNT).
extern "C" int acoss_profile_read(double* total_ms, int64_t* count, int n) {
  std::lock_guard<std::mutex> lk(g_mu);
  for (int i = 0; i < n && i < PH_COUNT; ++i) {
    total_ms[i] = 0.0;
    count[i] = 0;
  }
  for (auto& r : g_recs) {
    if (hipEventSynchronize(r.b) != hipSuccess) return ACOSS_E_HIP;
    float ms = 0.0f;
    if (hipEventElapsedTime(&ms, r.a, r.b) != hipSuccess) return ACOSS_E_HIP;
    if (r.phase < n) {
      total_ms[r.phase] += ms;
      count[r.phase] += 1;
    }
  }
  return PH_COUNT;
}

extern "C" const char* acoss_profile_phase_name(int i) { return (i >= 0 && i < PH_COUNT) ? kPhaseNames[i] : ""; }

extern "C" const char* acoss_last_error(void) { return acoss::last_error(); }
extern "C" int acoss_release_workspace(void) { return acoss::release_all_workspaces(); }
extern "C" const char* acoss_version(void) { return "acoss-mi355x 0.1.0 (gfx950)"; }
