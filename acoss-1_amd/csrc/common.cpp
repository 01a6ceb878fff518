// common.cpp — error string and the grow-only device workspace cache.
#include "common.hpp"

#include <cstdarg>
#include <cstdio>
#include <map>
#include <mutex>
#include <utility>

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
struct Buf {
  void* ptr = nullptr;
  size_t bytes = 0;
};
std::mutex g_mu;
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

int release_all_workspaces() {
  std::lock_guard<std::mutex> lk(g_mu);
  if (hipDeviceSynchronize() != hipSuccess) return ACOSS_E_HIP;
  for (auto& kv : g_ws)
    if (kv.second.ptr) (void)hipFree(kv.second.ptr);
  g_ws.clear();
  return ACOSS_OK;
}

}  // namespace acoss

extern "C" const char* acoss_last_error(void) { return acoss::last_error(); }
extern "C" int acoss_release_workspace(void) { return acoss::release_all_workspaces(); }
extern "C" const char* acoss_version(void) { return "acoss-mi355x 0.1.0 (gfx950)"; }
