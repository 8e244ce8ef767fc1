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

int rq_abi_version(void) { return 1; }

}  // extern "C"
