// Shared helpers for the MI355X (gfx950, CDNA4) kernels of the RQ-VAE training path.
// Wave64 everywhere; no CUDA-compat shims, no dual backend.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4v __attribute__((ext_vector_type(4)));

namespace rqhip {

// Thread-local last error text; surfaced by rq_last_error() (c_abi.cpp).
void set_error(const char* fmt, ...);

// Argument-check failure code (negative; distinct from hipError_t values).
constexpr int kBadArg = -22;

#define RQ_CHECK_ARG(cond, ...)                                   \
  do {                                                            \
    if (!(cond)) {                                                \
      ::rqhip::set_error(__VA_ARGS__);                            \
      return ::rqhip::kBadArg;                                    \
    }                                                             \
  } while (0)

#define RQ_LAUNCH_CHECK(what)                                     \
  do {                                                            \
    hipError_t e_ = hipGetLastError();                            \
    if (e_ != hipSuccess) {                                       \
      ::rqhip::set_error("%s: %s", what, hipGetErrorString(e_));  \
      return (int)e_;                                             \
    }                                                             \
  } while (0)

#define RQ_HIP(call)                                                      \
  do {                                                                    \
    hipError_t e_ = (call);                                               \
    if (e_ != hipSuccess) {                                               \
      ::rqhip::set_error("%s: %s", #call, hipGetErrorString(e_));         \
      return (int)e_;                                                     \
    }                                                                     \
  } while (0)

// Butterfly sum over an aligned group of G lanes (G power of two <= 64). Every lane of
// the group ends with the identical value (pairwise adds are commutative).
template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = G / 2; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ int ceil_div(int a, int b) { return (a + b - 1) / b; }

}  // namespace rqhip
