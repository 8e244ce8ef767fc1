// Shared helpers for the MI355X (gfx950, CDNA4) kernels of the RQ-VAE training path.
// Wave64 everywhere; no CUDA-compat shims, no dual backend.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include <math.h>
#include <algorithm>

#include "../../include/rqvae_hip.h"   // every extern "C" definition is checked against its declaration

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

// Zero `bytes` of device memory on `stream` with a kernel (16-B stores, byte tail). Used instead of
// hipMemsetAsync on every path a train step may record into a hipGraph: on this stack (ROCm 7.0 runtime
// under torch) a captured memset node was seen to miss replays (stale workspaces in p_unique_ids under
// the graphed trainer), while kernels replay in stream order.
template <int U>
__global__ void __launch_bounds__(256) rq_zero_kernel(uint4* __restrict__ p, int64_t n16, unsigned char* __restrict__ tail,
                                                      int ntail) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) p[i] = make_uint4(0u, 0u, 0u, 0u);
  if (blockIdx.x == 0 && (int)threadIdx.x < ntail) tail[threadIdx.x] = 0;
}

static inline hipError_t zero_async(void* p, size_t bytes, hipStream_t s) {
  if (bytes == 0) return hipSuccess;
  const uintptr_t a = (uintptr_t)p;
  if (a % 16 != 0) return hipMemsetAsync(p, 0, bytes, s);   // unaligned: never the case for torch allocations
  const int64_t n16 = (int64_t)(bytes / 16);
  const int ntail = (int)(bytes % 16);
  int64_t blocks = (n16 + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(rq_zero_kernel<0>, dim3((unsigned)blocks), dim3(256), 0, s, reinterpret_cast<uint4*>(p), n16,
                     reinterpret_cast<unsigned char*>(p) + n16 * 16, ntail);
  return hipGetLastError();
}

// Butterfly sum over an aligned group of G lanes (G power of two <= 64). Every lane of
// the group ends with the identical value (pairwise adds are commutative).
template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = G / 2; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ int ceil_div(int a, int b) { return (a + b - 1) / b; }

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));

// Split-bf16 operand form of the 'high' matmul path (linear.hip): (a, b) -> packed bf16 (hi) and
// packed bf16 of the exact remainders (lo), round-to-nearest-even.
__device__ __forceinline__ void split_bf16x2(float a, float b, uint32_t& hi, uint32_t& lo) {
  const f32x2_t v = {a, b};
  const uint32_t hb = __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
  const f32x2_t hf = {__builtin_bit_cast(float, hb << 16), __builtin_bit_cast(float, hb & 0xffff0000u)};
  const f32x2_t r = v - hf;
  hi = hb;
  lo = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, bf16x2_t));
}

// 4 consecutive fp32 values -> their hi / lo bf16 planes (8-B stores each).
__device__ __forceinline__ void split_store4(const float4 o, uint16_t* hi, uint16_t* lo) {
  uint2 h, l;
  split_bf16x2(o.x, o.y, h.x, l.x);
  split_bf16x2(o.z, o.w, h.y, l.y);
  *reinterpret_cast<uint2*>(hi) = h;
  *reinterpret_cast<uint2*>(lo) = l;
}

// 0 + P[s0] + P[s0 + stride] + P[s0 + 2 stride] + ... (s ascending) over the (n)-float partials P[s][..] at
// float4 column j: the order every split-K / partial reduction here is defined by. Eight partial loads are in
// flight per round whatever S is — indices past the end re-read partial S - 1 (a cache hit) and are not
// added — so a lane with 5..8 partials waits for one round trip instead of up to five dependent ones.
__device__ __forceinline__ float4 strided_slab_sum(const float* __restrict__ P, int S, int64_t n, int64_t j, int s0,
                                                   int stride) {
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int s = s0; s < S; s += 8 * stride) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      v[u] = *reinterpret_cast<const float4*>(P + (int64_t)min(s + stride * u, S - 1) * n + j);
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (s + stride * u < S) { a.x += v[u].x; a.y += v[u].y; a.z += v[u].z; a.w += v[u].w; }
  }
  return a;
}

// The four-way slab sum of the split-K reductions by ONE thread: p_w = 0 + P[w] + P[w + 4] + ... (ascending s,
// w = s mod 4), returned as ((p0 + p1) + p2) + p3 — bitwise strided_slab_sum(.., w, 4) per wave combined in
// wave order (the layout-0 order), without the LDS exchange and its barrier, 16 partial loads in flight per
// round (past-the-end indices re-read partial S - 1 and are not added).
__device__ __forceinline__ float4 slab_sum_w4(const float* __restrict__ P, int S, int64_t n, int64_t j) {
  float4 p[4];
#pragma unroll
  for (int w = 0; w < 4; ++w) p[w] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int s = 0; s < S; s += 16) {
    float4 v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = *reinterpret_cast<const float4*>(P + (int64_t)min(s + u, S - 1) * n + j);
#pragma unroll
    for (int u = 0; u < 16; ++u)
      if (s + u < S) { p[u & 3].x += v[u].x; p[u & 3].y += v[u].y; p[u & 3].z += v[u].z; p[u & 3].w += v[u].w; }
  }
  float4 r = p[0];
#pragma unroll
  for (int w = 1; w < 4; ++w) { r.x += p[w].x; r.y += p[w].y; r.z += p[w].z; r.w += p[w].w; }
  return r;
}

// Correctly rounded a / b (bitwise the IEEE quotient) for a divisor shared by many numerators:
// y = 1.0f / b is computed once with the IEEE division, then q0 = RN(a*y) is within an ulp of
// a/b and one fma correction returns RN(a/b) (Markstein's theorem) whenever the residual
// a - b*q0 is exact, i.e. away from under/overflow: |a| in [2^-90, 2^90] and b in [2^-60, 2^60].
// Callers check that range once per row (div_rn_ok; a row holding an exact zero also takes the
// slow path, which keeps the sign of a zero quotient) and use the IEEE division otherwise.
// 3 VALU ops instead of ~10.
__device__ __forceinline__ float div_rn(float a, float b, float y) {
  const float q0 = a * y;
  const float r = __builtin_fmaf(-b, q0, a);
  return __builtin_fmaf(r, y, q0);
}
// min_abs / max_abs = min / max |a| over the numerators of the row.
__device__ __forceinline__ bool div_rn_ok(float min_abs, float max_abs, float b) {
  return min_abs >= 0x1p-90f && max_abs <= 0x1p90f && b >= 0x1p-60f && b <= 0x1p60f;
}

// Counter-based dropout mask (stateless, so a backward kernel regenerates the forward's mask from
// (seed, element index) instead of storing it). SplitMix64 output for counter c under key seed;
// element e = 4q + j of a tensor draws 32-bit word j of (mix(2q), mix(2q + 1)) and is kept iff
// word >= thr, thr = round(p * 2^32), i.e. with probability 1 - p (nn.Dropout semantics, kept
// values scaled by 1 / (1 - p)). thr == 0 means no dropout.
__device__ __forceinline__ uint64_t splitmix64(uint64_t seed, uint64_t c) {
  uint64_t z = seed + (c + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// Dropout epoch: a device word mixed into every mask key. Eager callers leave it at 0 (keys =
// the host seeds); a captured (hipGraph) train step advances it once per replay
// (rq_seed_epoch_advance, captured at the end of the step), so each replay draws fresh masks while
// the forward and backward of one step see the same epoch. One copy per translation unit (no
// relocatable device code): dropout.hip / rowwise.hip / linear.hip each export its address and
// rq_seed_epoch_advance / rq_seed_epoch_set update all of them.
static __device__ uint64_t rq_seed_epoch = 0;
__device__ __forceinline__ uint64_t epoch_seed(uint64_t seed) {
  return seed + rq_seed_epoch * 0xD6E8FEB86659FD93ull;
}
// the three copies' device addresses (current device) and their update launch (c_abi.cpp's callers)
int seed_epoch_addr_dropout(void** out);
int seed_epoch_addr_rowwise(void** out);
int seed_epoch_addr_linear(void** out);
int seed_epoch_update(void* a, void* b, void* c, uint64_t value, int add, void* stream);
// thr / scale of nn.Dropout(p) for the kernels below (dropout.hip).
void dropout_params(float p, uint32_t* thr, float* scale);
struct Keep4 {
  bool k[4];
};
__device__ __forceinline__ Keep4 keep4(uint64_t seed, uint64_t q, uint32_t thr) {
  const uint64_t a = splitmix64(seed, 2 * q), b = splitmix64(seed, 2 * q + 1);
  Keep4 r;
  r.k[0] = (uint32_t)a >= thr;
  r.k[1] = (uint32_t)(a >> 32) >= thr;
  r.k[2] = (uint32_t)b >= thr;
  r.k[3] = (uint32_t)(b >> 32) >= thr;
  return r;
}
// Element e of a tensor under the same mask: word (e & 1) of mix(e >> 1) (= keep4(seed, e / 4).k[e % 4]).
__device__ __forceinline__ bool keep1(uint64_t seed, uint64_t e, uint32_t thr) {
  return (uint32_t)(splitmix64(seed, e >> 1) >> (32 * (e & 1))) >= thr;
}
// SiLU and its gradient, ATen's formulas: silu(z) = z / (1 + exp(-z)),
// silu'(z) g = g * s * (1 + z * (1 - s)), s = 1 / (1 + exp(-z)).
__device__ __forceinline__ float silu_f(float z) { return z / (1.0f + expf(-z)); }
__device__ __forceinline__ float silu_grad_f(float g, float z) {
  const float s = 1.0f / (1.0f + expf(-z));
  return g * s * (1.0f + z * (1.0f - s));
}
__device__ __forceinline__ float4 drop4(float4 v, uint64_t seed, uint64_t q, uint32_t thr, float scale) {
  if (thr == 0) return v;
  const Keep4 m = keep4(seed, q, thr);
  return make_float4(m.k[0] ? v.x * scale : 0.f, m.k[1] ? v.y * scale : 0.f, m.k[2] ? v.z * scale : 0.f,
                     m.k[3] ? v.w * scale : 0.f);
}

}  // namespace rqhip
