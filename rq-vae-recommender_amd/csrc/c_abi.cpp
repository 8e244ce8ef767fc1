// C-ABI support: thread-local last-error text and library identification.
// Every entry point in include/rqvae_hip.h returns 0 on success, a hipError_t (>0) for a
// runtime/launch failure, or a negative argument-check code; rq_last_error() explains it.
#include <stdarg.h>
#include <stdio.h>

#include <mutex>

#include "common.h"

namespace rqhip {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace rqhip

extern "C" {

const char* rq_last_error(void) { return rqhip::g_err; }

int rq_abi_version(void) { return 3; }

// Dropout epoch (common.h): the three translation units' device copies, resolved once per device
// (the symbol addresses differ per device) and cached; resolving costs three runtime lookups, and the
// epoch is advanced on every step, inside captured graphs too.
static int epoch_addrs(void** p) {
  constexpr int kMaxDev = 64;
  static std::mutex mu;
  static void* cache[kMaxDev][3];
  static bool have[kMaxDev];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) {
    rqhip::set_error("rq_seed_epoch: hipGetDevice failed");
    return rqhip::kBadArg;
  }
  std::lock_guard<std::mutex> lk(mu);
  if (dev < kMaxDev && have[dev]) {
    for (int i = 0; i < 3; ++i) p[i] = cache[dev][i];
    return 0;
  }
  if (rqhip::seed_epoch_addr_dropout(&p[0]) || rqhip::seed_epoch_addr_rowwise(&p[1]) ||
      rqhip::seed_epoch_addr_linear(&p[2])) {
    rqhip::set_error("rq_seed_epoch: hipGetSymbolAddress failed");
    return rqhip::kBadArg;
  }
  if (dev < kMaxDev) {
    for (int i = 0; i < 3; ++i) cache[dev][i] = p[i];
    have[dev] = true;
  }
  return 0;
}

int rq_seed_epoch_advance(void* stream) {
  void* p[3];
  int rc = epoch_addrs(p);
  return rc ? rc : rqhip::seed_epoch_update(p[0], p[1], p[2], 0, 1, stream);
}

int rq_seed_epoch_set(uint64_t value, void* stream) {
  void* p[3];
  int rc = epoch_addrs(p);
  return rc ? rc : rqhip::seed_epoch_update(p[0], p[1], p[2], value, 0, stream);
}

}  // extern "C"
