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

// ------------------------------------------------------------------ decoder prologue (forward)
// The generative-retrieval decoder's input embeddings straight into its two jagged batches
// (reference modules/model.py:101-129 _predict with modules/embedding/id_embedder.py:28-53):
//   context row 0      user_w[uid mod nb]
//   context row 1 + j  sem_w[mask ? type * K + sem : pad] + wpe_w[j]            (j < sum(mask[b]))
//   future  row 0      bos
//   future  row 1 + t  sem_w[type_fut * K + sem_fut] + tte_w[type_fut]
// every value through padded_to_jagged's (v + 1) - 1 (ops/triton/jagged.py:65), the context at
// offsets [0, cumsum(sum(mask[b]) + 1)] with the allocation's tail rows zero, the future at b * nf:
// bitwise the composition (gathers, one fp32 add, the +1-1), in two launches instead of ~24.
// Also writes the table rows the backward's segmented sums key on: keys (B, N + L) = the context's
// sem-table rows (pad where masked) then the future's, and uid mod nb (B).
// 1 in each byte of w that is nonzero, 0 elsewhere (bit 0 of byte k = OR of its bits 0..7)
__device__ __forceinline__ uint32_t nz_bytes(uint32_t w) {
  w |= w >> 4;
  w |= w >> 2;
  w |= w >> 1;
  return w & 0x01010101u;
}
constexpr int kDecLensLds = 4096;   // sequences whose lengths the offsets kernel keeps in LDS
constexpr int kDecMaskLds = 24576;  // mask bytes (B x N) the offsets kernel stages in LDS
__global__ void __launch_bounds__(1024) dec_prologue_offsets_kernel(const unsigned char* __restrict__ mask, int64_t B, int64_t N,
                                                                    int64_t nf, int64_t alloc_rows,
                                                                    int64_t* __restrict__ off_ctx,
                                                                    int64_t* __restrict__ off_fut, int* __restrict__ order) {
  __shared__ int64_t part[1024];
  __shared__ int64_t lens[kDecLensLds];
  __shared__ __attribute__((aligned(16))) unsigned char mask_s[kDecMaskLds];
  __shared__ __attribute__((aligned(16))) int lens32[kDecLensLds];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  // lengths sum(mask[b]) + 1: one wave per sequence, a wave reduction; a mask that fits LDS is staged
  // first in one pass of 16-byte loads by the whole workgroup (one memory round trip instead of a
  // dependent global read per sequence and wave: B = 256 short sequences took 24 us, 16 per wave)
  const bool in_lds = B <= kDecLensLds;
  const int64_t nbytes = B * N;
  const bool staged = in_lds && nbytes <= kDecMaskLds && ((uintptr_t)mask & 15) == 0;
  if (staged) {
    const int64_t n16 = nbytes >> 4;
    for (int64_t i = t; i < n16; i += 1024) {   // bytes normalised to 0 / 1 (a bool tensor viewed from uint8 may
      uint4 v = reinterpret_cast<const uint4*>(mask)[i];   // hold any nonzero byte; the byte sums below need 0 / 1)
      v.x = nz_bytes(v.x), v.y = nz_bytes(v.y), v.z = nz_bytes(v.z), v.w = nz_bytes(v.w);
      *reinterpret_cast<uint4*>(mask_s + 16 * i) = v;
    }
    for (int64_t i = 16 * n16 + t; i < nbytes; i += 1024) mask_s[i] = mask[i] ? 1 : 0;
    __syncthreads();
  }
  if (in_lds && staged && N % 16 == 0 && B >= 64) {   // one thread per sequence, 16 mask bytes per LDS read
    // (many short sequences: Amazon's 256 x 80; a few long ones keep a wave each, below)
    const int n16r = (int)(N >> 4);
    for (int64_t b = t; b < B; b += 1024) {
      const uint4* row = reinterpret_cast<const uint4*>(mask_s + b * N);
      uint32_t c = 0;
      for (int q = 0; q < n16r; ++q) {
        const uint4 v = row[q];   // byte sums of each word: 4 bytes <= 1 each, by a multiply
        c += ((v.x * 0x01010101u) >> 24) + ((v.y * 0x01010101u) >> 24) + ((v.z * 0x01010101u) >> 24) +
             ((v.w * 0x01010101u) >> 24);
      }
      lens[b] = (int64_t)c + 1;
    }
    __syncthreads();
  } else if (in_lds) {
    for (int64_t b = wave; b < B; b += 16) {
      int c = 0;
      if (staged)
        for (int64_t j = lane; j < N; j += 64) c += mask_s[b * N + j] ? 1 : 0;
      else
        for (int64_t j = lane; j < N; j += 64) c += mask[b * N + j] ? 1 : 0;
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o, 64);
      if (lane == 0) lens[b] = c + 1;
    }
    __syncthreads();
  }
  auto len_of = [&](int64_t i) -> int64_t {
    if (in_lds) return lens[i];
    int64_t c = 1;   // the user token
    for (int64_t j = 0; j < N; ++j) c += mask[i * N + j] ? 1 : 0;
    return c;
  };
  const int64_t per = (B + 1023) / 1024;
  const int64_t a = t * per, e = a + per < B ? a + per : B;
  int64_t s = 0;
  for (int64_t i = a; i < e; ++i) s += len_of(i);
  part[t] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const int64_t v = t >= o ? part[t - o] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int64_t run = part[t] - s;
  if (t == 0) off_ctx[0] = 0;
  for (int64_t i = a; i < e; ++i) {   // clamped to the allocation: host row counts that undercount the mask
    run += len_of(i);                   // (stale registration) shorten the last sequences instead of sending
    off_ctx[i + 1] = run < alloc_rows ? run : alloc_rows;   // every consumer past the values
  }
  for (int64_t i = t; i <= B; i += 1024) off_fut[i] = i * nf;
  // longest-first order of the contexts (attention.hip attn_order_kernel's ranking: length descending,
  // ties by index), for the attention launches over these offsets (RQ_ATTN_ORDER_GIVEN)
  // The O(B^2) ranking reads an int32 copy of the lengths 4 at a time (independent compares, 16-byte LDS
  // reads; B = 256 sequences: the int64 one-at-a-time loop was most of the kernel's 21 us); the copy is padded
  // to a multiple of 4 with -1, which never ranks ahead of or ties a length >= 1.
#ifndef RQ_PRO_DIAG
#define RQ_PRO_DIAG 0   // diagnostic builds only: 1 = no LPT ranking (the order is left unwritten)
#endif
  if (order != nullptr && in_lds && RQ_PRO_DIAG != 1) {
    const int B4 = (int)((B + 3) >> 2);
    for (int64_t b = t; b < 4 * (int64_t)B4; b += 1024) lens32[b] = b < B ? (int)lens[b] : -1;
    __syncthreads();
    const int4* __restrict__ l4 = reinterpret_cast<const int4*>(lens32);
    // 64 <= B <= 256: four threads per sequence, each over a quarter of the j range (integer partial ranks summed
    // by LDS atomics: exact); otherwise one thread per sequence over all of j
    const int parts = (B >= 64 && B <= 256) ? 4 : 1;
    const int per_q = (B4 + parts - 1) / parts;
    int* rank_s = reinterpret_cast<int*>(part);   // the scan's buffer is free again
    for (int64_t b = t; b < B; b += 1024) rank_s[b] = 0;
    __syncthreads();
    for (int64_t i = t; i < (int64_t)B * parts; i += 1024) {
      const int bi = (int)(i % B), qp = (int)(i / B);
      const int lb = lens32[bi];
      int rank = 0;
      const int q1 = min(B4, (qp + 1) * per_q);
#pragma unroll 4
      for (int q = qp * per_q; q < q1; ++q) {
        const int4 v = l4[q];
        const int j0 = 4 * q;
        rank += (v.x > lb) | ((v.x == lb) & (j0 < bi));
        rank += (v.y > lb) | ((v.y == lb) & (j0 + 1 < bi));
        rank += (v.z > lb) | ((v.z == lb) & (j0 + 2 < bi));
        rank += (v.w > lb) | ((v.w == lb) & (j0 + 3 < bi));
      }
      if (parts == 1) order[rank] = bi;
      else atomicAdd(&rank_s[bi], rank);
    }
    if (parts > 1) {
      __syncthreads();
      for (int64_t b = t; b < B; b += 1024) order[rank_s[b]] = (int)b;
    }
  }
}

struct DecPrologueArgs {
  const int64_t *uid, *sem, *typ, *sem_fut, *typ_fut;
  const unsigned char* mask;   // the bool mask's bytes: any nonzero byte is true
  const float *w_user, *w_sem, *w_wpe, *w_tte, *bos;
  int64_t n_buckets, K, pad, n_sem_rows, n_wpe_rows, n_tte_rows;
  int64_t B, N, L, E;
  const int64_t* off_ctx;
  float *ctx, *fut;
  int64_t alloc_rows;
  int64_t *keys, *uid_mod;
};

__device__ __forceinline__ int64_t clamp_row(int64_t r, int64_t n) { return r < 0 ? 0 : (r >= n ? n - 1 : r); }

// Grid (ceil((1 + max(N, L)) * E / 4 / 256), 2 B + 1): y < B the context rows of sequence y, y == B the
// context allocation's tail, y > B the future rows of sequence y - B - 1. Block x == 0 also writes the keys.
__global__ void __launch_bounds__(256) dec_prologue_fwd_kernel(DecPrologueArgs a) {
  const int64_t y = blockIdx.y, E = a.E;
  if (y == a.B) {   // zero the context tail rows [off_ctx[B], alloc_rows)
    const int64_t e0 = a.off_ctx[a.B] * E, e1 = a.alloc_rows * E;
    for (int64_t e = e0 + ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4; e < e1; e += (int64_t)gridDim.x * 256 * 4)
      *reinterpret_cast<float4*>(a.ctx + e) = make_float4(0.f, 0.f, 0.f, 0.f);
    return;
  }
  const bool ctx = y < a.B;
  const int64_t b = ctx ? y : y - a.B - 1;
  if (blockIdx.x == 0) {   // keys of the backward's segmented sums (context then future), uid mod nb
    if (ctx) {
      for (int64_t j = threadIdx.x; j < a.N; j += 256) {
        const int64_t o = b * a.N + j;
        a.keys[b * (a.N + a.L) + j] = a.mask[o] ? a.typ[o] * a.K + a.sem[o] : a.pad;
      }
      if (threadIdx.x == 0) {
        const int64_t u = a.uid[b] % a.n_buckets;
        a.uid_mod[b] = u < 0 ? u + a.n_buckets : u;   // torch's remainder: the divisor's sign
      }
    } else {
      for (int64_t t = threadIdx.x; t < a.L; t += 256) {
        const int64_t o = b * a.L + t;
        a.keys[b * (a.N + a.L) + a.N + t] = a.typ_fut[o] * a.K + a.sem_fut[o];
      }
    }
  }
  const int64_t idx = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  const int64_t r = idx / E, d = idx - r * E;   // E % 4 == 0: a float4 never crosses a row
  float4 v;
  float* dst;
  if (ctx) {
    const int64_t o0 = a.off_ctx[b], len = a.off_ctx[b + 1] - o0;
    if (r >= len || o0 + r >= a.alloc_rows) return;   // (an allocation below the valid total drops rows, never faults)
    if (r == 0) {
      int64_t u = a.uid[b] % a.n_buckets;
      u = u < 0 ? u + a.n_buckets : u;
      v = *reinterpret_cast<const float4*>(a.w_user + u * E + d);
    } else {
      const int64_t j = r - 1, o = b * a.N + j;
      const int64_t row = clamp_row(a.mask[o] ? a.typ[o] * a.K + a.sem[o] : a.pad, a.n_sem_rows);
      const float4 se = *reinterpret_cast<const float4*>(a.w_sem + row * E + d);
      const float4 pe = *reinterpret_cast<const float4*>(a.w_wpe + clamp_row(j, a.n_wpe_rows) * E + d);
      v = make_float4(pe.x + se.x, pe.y + se.y, pe.z + se.z, pe.w + se.w);
    }
    dst = a.ctx + (o0 + r) * E + d;
  } else {
    if (r > a.L) return;
    if (r == 0) {
      v = *reinterpret_cast<const float4*>(a.bos + d);
    } else {
      const int64_t o = b * a.L + r - 1;
      const int64_t row = clamp_row(a.typ_fut[o] * a.K + a.sem_fut[o], a.n_sem_rows);
      const float4 se = *reinterpret_cast<const float4*>(a.w_sem + row * E + d);
      const float4 te = *reinterpret_cast<const float4*>(a.w_tte + clamp_row(a.typ_fut[o], a.n_tte_rows) * E + d);
      v = make_float4(se.x + te.x, se.y + te.y, se.z + te.z, se.w + te.w);
    }
    dst = a.fut + (b * (a.L + 1) + r) * E + d;
  }
  *reinterpret_cast<float4*>(dst) = make_float4(p1m1(v.x), p1m1(v.y), p1m1(v.z), p1m1(v.w));
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

int rq_dec_prologue_fwd(const int64_t* user_ids, const int64_t* sem_ids, const int64_t* type_ids, const bool* seq_mask,
                        const int64_t* sem_ids_fut, const int64_t* type_ids_fut, int64_t B, int64_t N, int64_t L,
                        int64_t E, const float* user_w, int64_t n_buckets, const float* sem_w, int64_t n_sem_rows,
                        int64_t K, int64_t pad, const float* wpe_w, int64_t n_wpe_rows, const float* tte_w,
                        int64_t n_tte_rows, const float* bos, float* ctx_values, int64_t ctx_alloc_rows,
                        int64_t* ctx_offsets, float* fut_values, int64_t* fut_offsets, int64_t* keys, int64_t* uid_mod,
                        int* lpt_order, void* stream) {
  RQ_CHECK_ARG(lpt_order == nullptr || B <= kDecLensLds, "rq_dec_prologue_fwd: lpt_order needs B <= %d", kDecLensLds);
  RQ_CHECK_ARG(user_ids && sem_ids && type_ids && seq_mask && sem_ids_fut && type_ids_fut && user_w && sem_w && wpe_w &&
                   tte_w && bos && ctx_values && ctx_offsets && fut_values && fut_offsets && keys && uid_mod,
               "rq_dec_prologue_fwd: null pointer");
  RQ_CHECK_ARG(B >= 0 && 2 * B + 1 < 65535 && N >= 0 && L >= 0 && E > 0 && E % 4 == 0 && n_buckets > 0 && K > 0 &&
                   n_sem_rows > 0 && n_wpe_rows >= N && n_tte_rows > 0 && ctx_alloc_rows >= B,
               "rq_dec_prologue_fwd: bad shape (E %% 4 == 0, wpe rows >= N, 2 B + 1 < 65535)");
  if (B == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(dec_prologue_offsets_kernel, dim3(1), dim3(1024), 0, s,
                     reinterpret_cast<const unsigned char*>(seq_mask), B, N, L + 1, ctx_alloc_rows, ctx_offsets,
                     fut_offsets, lpt_order);
  DecPrologueArgs a{user_ids, sem_ids, type_ids, sem_ids_fut, type_ids_fut,
                    reinterpret_cast<const unsigned char*>(seq_mask), user_w, sem_w, wpe_w, tte_w, bos,
                    n_buckets, K, pad, n_sem_rows, n_wpe_rows, n_tte_rows, B, N, L, E, ctx_offsets, ctx_values,
                    fut_values, ctx_alloc_rows, keys, uid_mod};
  const int64_t rows = 1 + (N > L ? N : L);
  const dim3 g((unsigned)((rows * E / 4 + 255) / 256), (unsigned)(2 * B + 1));
  hipLaunchKernelGGL(dec_prologue_fwd_kernel, g, dim3(256), 0, s, a);
  RQ_LAUNCH_CHECK("rq_dec_prologue_fwd");
  return 0;
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
