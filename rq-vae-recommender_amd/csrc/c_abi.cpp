// C-ABI support: thread-local last-error text and library identification.
// Every entry point in include/rqvae_hip.h returns 0 on success, a hipError_t (>0) for a
// runtime/launch failure, or a negative argument-check code; rq_last_error() explains it.
#include <stdarg.h>
#include <stdio.h>

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

int rq_abi_version(void) { return 2; }

int rq_seed_epoch_addr_dropout(void** out);
int rq_seed_epoch_addr_rowwise(void** out);
int rq_seed_epoch_addr_linear(void** out);
int rq_seed_epoch_update(void* a, void* b, void* c, uint64_t value, int add, void* stream);

// Dropout epoch (common.h): the three translation units' device copies, resolved once.
static int epoch_addrs(void** p) {
  static void* cache[3] = {nullptr, nullptr, nullptr};
  if (!cache[0]) {
    void* t[3];
    if (rq_seed_epoch_addr_dropout(&t[0]) || rq_seed_epoch_addr_rowwise(&t[1]) || rq_seed_epoch_addr_linear(&t[2])) {
      rqhip::set_error("rq_seed_epoch: hipGetSymbolAddress failed");
      return rqhip::kBadArg;
    }
    cache[1] = t[1];
    cache[2] = t[2];
    cache[0] = t[0];
  }
  for (int i = 0; i < 3; ++i) p[i] = cache[i];
  return 0;
}

int rq_seed_epoch_advance(void* stream) {
  void* p[3];
  int rc = epoch_addrs(p);
  return rc ? rc : rq_seed_epoch_update(p[0], p[1], p[2], 0, 1, stream);
}

int rq_seed_epoch_set(uint64_t value, void* stream) {
  void* p[3];
  int rc = epoch_addrs(p);
  return rc ? rc : rq_seed_epoch_update(p[0], p[1], p[2], value, 0, stream);
}

}  // extern "C"
