// Padded <-> jagged conversion for variable-length user sequences (HBM-bound byte movers).
//
// Reference: ops/triton/jagged.py
//   forward  :11-66 + Triton kernel :92-125 — values[offsets[b] + t] = x[b, t] for t < len_b,
//            offsets = [0, cumsum(lengths)], followed by `target + 1 - 1` (:65), which rounds
//            every value through (v + 1) in the tensor dtype; reproduced bit-exactly when
//            add_one_sub_one != 0 (no fp contraction: compiled with -ffp-contract=off).
//   backward :69-77 — grad_x = zeros(B, N, D); grad_x[mask] = grad_values.
//
// Layout: x (B, N, D) contiguous; values (T, D) with T = offsets[B]; offsets int64 (B+1).
// One launch streams each valid row once (16-B per lane); the backward writes every padded
// element exactly once (copy or zero), so no separate memset pass is spent.
#include "common.h"

#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>

namespace rqhip {

enum DType { kF32 = 0, kBF16 = 1, kF16 = 2 };

// offsets[0] = 0, offsets[b+1] = offsets[b] + lengths[b]; lengths clamped to [0, N].
__global__ void __launch_bounds__(1024) jagged_offsets_kernel(const int64_t* __restrict__ lengths, int64_t B, int64_t N,
                                                               int64_t* __restrict__ offsets) {
  __shared__ int64_t part[1024];
  const int t = threadIdx.x;
  const int64_t per = (B + 1023) / 1024;
  const int64_t a = t * per, e = a + per < B ? a + per : B;
  int64_t s = 0;
  for (int64_t i = a; i < e; ++i) {
    int64_t v = lengths[i];
    v = v < 0 ? 0 : (v > N ? N : v);
    s += v;
  }
  part[t] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const int64_t v = t >= o ? part[t - o] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int64_t run = part[t] - s;
  if (t == 0) offsets[0] = 0;
  for (int64_t i = a; i < e; ++i) {
    int64_t v = lengths[i];
    v = v < 0 ? 0 : (v > N ? N : v);
    run += v;
    offsets[i + 1] = run;
  }
}

__device__ __forceinline__ float p1m1(float v) {
  const float t = v + 1.0f;   // separate statements: -ffp-contract=off keeps two roundings
  return t - 1.0f;
}

// Grid: (ceil(N*D/VEC / 256), B [+1]). Each thread moves VEC contiguous elements of one row. With
// alloc_rows >= 0 the extra grid row y == B zero-fills the values rows [offsets[B], alloc_rows) (a
// row-bucketed buffer's tail, so callers never need the valid row count on the host).
template <typename T, int VEC>
__global__ void __launch_bounds__(256) jagged_gather_kernel(const T* __restrict__ x, const int64_t* __restrict__ off,
                                                             int64_t N, int64_t D, T* __restrict__ values, int p1m1_on,
                                                             int64_t nseq, int64_t alloc_rows) {
  const int64_t b = blockIdx.y;
  if (b == nseq) {   // tail rows of the allocation
    const int64_t e0 = off[nseq] * D, e1 = alloc_rows * D;
    for (int64_t e = e0 + ((int64_t)blockIdx.x * 256 + threadIdx.x) * VEC; e < e1; e += (int64_t)gridDim.x * 256 * VEC) {
#pragma unroll
      for (int k = 0; k < VEC; ++k) values[e + k] = T(0.0f);
    }
    return;
  }
  const int64_t o0 = off[b], len = off[b + 1] - o0;
  const int64_t idx = ((int64_t)blockIdx.x * 256 + threadIdx.x) * VEC;
  if (idx >= len * D) return;   // rows past len_b are never read (ragged tail)
  const T* src = x + b * N * D + idx;
  T* dst = values + o0 * D + idx;
  if constexpr (sizeof(T) == 4 && VEC == 4) {
    float4 v = *reinterpret_cast<const float4*>(src);
    if (p1m1_on) { v.x = p1m1(v.x); v.y = p1m1(v.y); v.z = p1m1(v.z); v.w = p1m1(v.w); }
    *reinterpret_cast<float4*>(dst) = v;
  } else {
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      T v = src[k];
      if (p1m1_on) {
        if constexpr (sizeof(T) == 4) {
          v = p1m1(v);
        } else {
          // (v + 1) and (t - 1) each rounded to T, as torch does for bf16/fp16 tensors.
          const T t = T(float(v) + 1.0f);
          v = T(float(t) - 1.0f);
        }
      }
      dst[k] = v;
    }
  }
}

template <typename T, int VEC>
__global__ void __launch_bounds__(256) jagged_scatter_kernel(const T* __restrict__ values, const int64_t* __restrict__ off,
                                                              int64_t N, int64_t D, T* __restrict__ x) {
  const int64_t b = blockIdx.y;
  const int64_t o0 = off[b], len = off[b + 1] - o0;
  const int64_t idx = ((int64_t)blockIdx.x * 256 + threadIdx.x) * VEC;
  if (idx >= N * D) return;
  T* dst = x + b * N * D + idx;
  const bool in = idx < len * D;   // D % VEC == 0 so a vector never straddles the boundary
  if constexpr (sizeof(T) == 4 && VEC == 4) {
    float4 v = in ? *reinterpret_cast<const float4*>(values + o0 * D + idx) : make_float4(0.f, 0.f, 0.f, 0.f);
    *reinterpret_cast<float4*>(dst) = v;
  } else {
#pragma unroll
    for (int k = 0; k < VEC; ++k) dst[k] = in ? values[o0 * D + idx + k] : T(0.0f);
  }
}

template <typename T>
static int launch_gather(const void* x, const int64_t* off, int64_t B, int64_t N, int64_t D, void* values, int p1,
                         int64_t alloc_rows, hipStream_t s) {
  const unsigned gy = (unsigned)(alloc_rows >= 0 ? B + 1 : B);
  if (sizeof(T) == 4 && D % 4 == 0) {
    dim3 g((unsigned)((N * D / 4 + 255) / 256), gy);
    hipLaunchKernelGGL((jagged_gather_kernel<T, 4>), g, dim3(256), 0, s, (const T*)x, off, N, D, (T*)values, p1, B,
                       alloc_rows);
  } else {
    dim3 g((unsigned)((N * D + 255) / 256), gy);
    hipLaunchKernelGGL((jagged_gather_kernel<T, 1>), g, dim3(256), 0, s, (const T*)x, off, N, D, (T*)values, p1, B,
                       alloc_rows);
  }
  return 0;
}

template <typename T>
static int launch_scatter(const void* values, const int64_t* off, int64_t B, int64_t N, int64_t D, void* x,
                          hipStream_t s) {
  if (sizeof(T) == 4 && D % 4 == 0) {
    dim3 g((unsigned)((N * D / 4 + 255) / 256), (unsigned)B);
    hipLaunchKernelGGL((jagged_scatter_kernel<T, 4>), g, dim3(256), 0, s, (const T*)values, off, N, D, (T*)x);
  } else {
    dim3 g((unsigned)((N * D + 255) / 256), (unsigned)B);
    hipLaunchKernelGGL((jagged_scatter_kernel<T, 1>), g, dim3(256), 0, s, (const T*)values, off, N, D, (T*)x);
  }
  return 0;
}

}  // namespace rqhip

using namespace rqhip;

extern "C" {

int jagged_offsets(const int64_t* lengths, int64_t B, int64_t N, int64_t* offsets, void* stream) {
  RQ_CHECK_ARG(lengths && offsets && B >= 0 && N >= 0, "jagged_offsets: bad arguments");
  hipLaunchKernelGGL(jagged_offsets_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, lengths, B, N, offsets);
  RQ_LAUNCH_CHECK("jagged_offsets");
  return 0;
}

int jagged_from_padded_rows(const void* x, int64_t B, int64_t N, int64_t D, const int64_t* offsets, void* values,
                            int64_t alloc_rows, int dtype, int add_one_sub_one, void* stream) {
  RQ_CHECK_ARG(x && offsets && values, "jagged_from_padded: null pointer");
  RQ_CHECK_ARG(B >= 0 && B < 65535 && N >= 0 && D > 0, "jagged_from_padded: bad shape (B < 65535 per call)");
  if (B == 0 || (N == 0 && alloc_rows < 0)) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int64_t n = N > 0 ? N : 1;   // N == 0 with a tail: one grid column zero-fills it
  switch (dtype) {
    case kF32: launch_gather<float>(x, offsets, B, n, D, values, add_one_sub_one, alloc_rows, s); break;
    case kBF16: launch_gather<__hip_bfloat16>(x, offsets, B, n, D, values, add_one_sub_one, alloc_rows, s); break;
    case kF16: launch_gather<__half>(x, offsets, B, n, D, values, add_one_sub_one, alloc_rows, s); break;
    default: RQ_CHECK_ARG(false, "jagged_from_padded: dtype %d unsupported", dtype);
  }
  RQ_LAUNCH_CHECK("jagged_from_padded");
  return 0;
}

int jagged_from_padded(const void* x, int64_t B, int64_t N, int64_t D, const int64_t* offsets, void* values, int dtype,
                       int add_one_sub_one, void* stream) {
  if (N == 0) return (x && offsets && values) ? 0 : jagged_from_padded_rows(x, B, N, D, offsets, values, -1, dtype, 0, stream);
  return jagged_from_padded_rows(x, B, N, D, offsets, values, -1, dtype, add_one_sub_one, stream);
}

int jagged_to_padded(const void* values, const int64_t* offsets, int64_t B, int64_t N, int64_t D, void* x, int dtype,
                     void* stream) {
  RQ_CHECK_ARG(values && offsets && x, "jagged_to_padded: null pointer");
  RQ_CHECK_ARG(B >= 0 && B <= 65535 && N >= 0 && D > 0, "jagged_to_padded: bad shape (B <= 65535 per call)");
  if (B == 0 || N == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  switch (dtype) {
    case kF32: launch_scatter<float>(values, offsets, B, N, D, x, s); break;
    case kBF16: launch_scatter<__hip_bfloat16>(values, offsets, B, N, D, x, s); break;
    case kF16: launch_scatter<__half>(values, offsets, B, N, D, x, s); break;
    default: RQ_CHECK_ARG(false, "jagged_to_padded: dtype %d unsupported", dtype);
  }
  RQ_LAUNCH_CHECK("jagged_to_padded");
  return 0;
}

}  // extern "C"
