// Varlen (jagged) multi-head attention, forward + backward, fp32 on v_mfma_f32_32x32x2_f32.
//
// Reference: modules/transformer/attention.py:113-124 (Attend.jagged_forward) —
// F.scaled_dot_product_attention on NJT q/k/v (B, H, j, hd), dropout 0 (:177), scale
// 1/sqrt(hd), is_causal = top-left aligned tril mask. Three call shapes in the model:
// encoder self-attention (non-causal), decoder self-attention (causal) and cross-attention
// (decoder queries x encoder keys, non-causal) — all served by this one kernel family.
//
// Layout: packed token-major rows. q[t][h][d] at q + t*sq + h*HD + d (sq = row stride, so the
// (T, 3A) qkv projection is consumed in place); cu_q / cu_k int64 (B+1) NJT offsets;
// out (Tq, H*HD) rows with stride so; lse (H, Tq) = m + log(l) per query (saved for bwd).
//
// Orientation trick: every score tile is computed TRANSPOSED (keys on the MFMA row axis,
// queries on lanes) in the forward and dQ passes, so a query's running max / sum / output
// live in ONE lane pair (lane j and j+32) — the online softmax needs a single lane swap per
// tile, no LDS round trip. The dK/dV pass puts keys on lanes the same way. P / dS feed the
// next MFMA straight from the accumulator registers (register t of the 32x32 tile is the
// k-slice of MFMA step t with key index (t&3)+8(t>>2)+4*(lane>>5)).
// Backward = two launches (dQ per query block, which also stores delta = rowsum(dO*O); then
// dK,dV per key block) with recomputed P: no atomics, bitwise deterministic.
#include "common.h"

#include <math.h>

#ifndef RQ_ATTN_ONE_WAVE_MAX
#define RQ_ATTN_ONE_WAVE_MAX 96   // longest sequence served by one-wave workgroups
#endif

namespace rqhip {

__device__ __forceinline__ int crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// Head dims below 32 use 32-wide LDS rows / output tiles whose extra columns stay zero.
template <int HD>
struct Pad {
  static constexpr int P = HD < 32 ? 32 : HD;   // padded width
  static constexpr int LD = P + 4;              // LDS row stride (floats)
};

// Zero the padding columns [HD, P) of a [32][LD] LDS image once per kernel.
template <int HD, int NT>
__device__ __forceinline__ void zero_pad32(float* dst, int tid) {
  constexpr int P = Pad<HD>::P, LD = Pad<HD>::LD;
  if constexpr (P > HD) {
    for (int f = tid; f < 32 * (P - HD); f += NT) dst[(f / (P - HD)) * LD + HD + f % (P - HD)] = 0.f;
  }
}

template <int HD>
__device__ __forceinline__ void load_half_row(const float* p, bool valid, float (&f)[HD / 2]) {
#pragma unroll
  for (int s = 0; s < HD / 2; s += 4) {
    float4 v = valid ? *reinterpret_cast<const float4*>(p + s) : make_float4(0.f, 0.f, 0.f, 0.f);
    f[s] = v.x; f[s + 1] = v.y; f[s + 2] = v.z; f[s + 3] = v.w;
  }
}

// Stage 32 rows x HD of a strided row source into LDS [32][HD+4]; rows >= n are zero.
template <int HD, int NT>
__device__ __forceinline__ void stage32(float* dst, const float* src, int64_t stride, int row0, int n, int tid) {
  constexpr int F4 = HD / 4, LD = Pad<HD>::LD;
  for (int f = tid; f < 32 * F4; f += NT) {
    const int r = f / F4, c = (f % F4) * 4;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (row0 + r < n) v = *reinterpret_cast<const float4*>(src + (int64_t)(row0 + r) * stride + c);
    *reinterpret_cast<float4*>(dst + r * LD + c) = v;
  }
}

// acc += Mat[rows i][HD] (LDS, A operand, row = lane&31) x frag (B operand, registers)
template <int HD>
__device__ __forceinline__ floatx16 mfma_rows_x_frag(const float* Ms, const float (&frag)[HD / 2], int lane, floatx16 acc) {
  const float* ap = Ms + (lane & 31) * Pad<HD>::LD + (lane >> 5) * (HD / 2);
#pragma unroll
  for (int s = 0; s < HD / 2; s += 4) {
    const float4 a = *reinterpret_cast<const float4*>(ap + s);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, frag[s], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, frag[s + 1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, frag[s + 2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, frag[s + 3], acc, 0, 0, 0);
  }
  return acc;
}

// acc[tile] (rows d, cols lane) += Ms^T[d][t-row] * w[t] over the 32 rows of Ms (LDS [32][LD]).
template <int HD>
__device__ __forceinline__ void mfma_colsT_x_regs(const float* Ms, const floatx16& w, int lane,
                                                  floatx16 (&acc)[Pad<HD>::P / 32]) {
  const int h = lane >> 5, c = lane & 31;
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    const float* row = Ms + crow(t, h) * Pad<HD>::LD + c;
#pragma unroll
    for (int tl = 0; tl < Pad<HD>::P / 32; ++tl)
      acc[tl] = __builtin_amdgcn_mfma_f32_32x32x2f32(row[tl * 32], w[t], acc[tl], 0, 0, 0);
  }
}

// Write rows-d accumulators for one row (lane) as float4 runs: d = 32 tl + 8 g + 4 h + 0..3.
template <int HD>
__device__ __forceinline__ void store_dT(float* rowp, const floatx16 (&acc)[Pad<HD>::P / 32], float mul, int h) {
#pragma unroll
  for (int tl = 0; tl < Pad<HD>::P / 32; ++tl)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = tl * 32 + 8 * g + 4 * h;
      if (d < HD)
        *reinterpret_cast<float4*>(rowp + d) =
            make_float4(acc[tl][4 * g] * mul, acc[tl][4 * g + 1] * mul, acc[tl][4 * g + 2] * mul, acc[tl][4 * g + 3] * mul);
    }
}

// ---------------------------------------------------------------------------------------- fwd
template <int HD, int NW>
__global__ void __launch_bounds__(64 * NW) attn_fwd_kernel(const float* __restrict__ q, int64_t sq, const float* __restrict__ k,
                                                        int64_t sk, const float* __restrict__ v, int64_t sv,
                                                        const int64_t* __restrict__ cu_q, const int64_t* __restrict__ cu_k,
                                                        int causal, float scale, float* __restrict__ out, int64_t so,
                                                        float* __restrict__ lse, int64_t Tq) {
  constexpr int LD = Pad<HD>::LD, NTL = Pad<HD>::P / 32;
  __shared__ __attribute__((aligned(16))) float smem[2 * 32 * LD];
  float* K_s = smem;
  float* V_s = smem + 32 * LD;
  const int b = blockIdx.z, hh = blockIdx.y, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, h = lane >> 5;
  zero_pad32<HD, 64 * NW>(K_s, tid);
  zero_pad32<HD, 64 * NW>(V_s, tid);
  const int64_t q0 = cu_q[b], k0 = cu_k[b];
  const int lq = (int)(cu_q[b + 1] - q0), lk = (int)(cu_k[b + 1] - k0);
  const int qbase = blockIdx.x * 32 * NW;
  if (qbase >= lq) return;
  const int qi = qbase + wave * 32 + (lane & 31);
  const bool qv = qi < lq;
  float qf[HD / 2];
  load_half_row<HD>(q + (q0 + (qv ? qi : 0)) * sq + hh * HD + h * (HD / 2), qv, qf);
  floatx16 o[NTL];
#pragma unroll
  for (int tl = 0; tl < NTL; ++tl)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[tl][r] = 0.f;
  float m = -INFINITY, l = 0.f;
  const int kend = causal ? min(lk, qbase + 32 * NW) : lk;
  for (int kt = 0; kt < kend; kt += 32) {
    __syncthreads();
    stage32<HD, 64 * NW>(K_s, k + k0 * sk + hh * HD, sk, kt, lk, tid);
    stage32<HD, 64 * NW>(V_s, v + k0 * sv + hh * HD, sv, kt, lk, tid);
    __syncthreads();
    floatx16 s;
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = 0.f;
    s = mfma_rows_x_frag<HD>(K_s, qf, lane, s);   // S^T: rows = keys, cols = queries
    float mt = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = kt + crow(r, h);
      const bool ok = key < lk && (!causal || key <= qi);
      s[r] = ok ? s[r] * scale : -INFINITY;
      mt = fmaxf(mt, s[r]);
    }
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    const float mn = fmaxf(m, mt);
    const float alpha = (mn == -INFINITY) ? 1.f : expf(m - mn);
    float ls = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      s[r] = (s[r] == -INFINITY) ? 0.f : expf(s[r] - mn);
      ls += s[r];
    }
    ls += __shfl_xor(ls, 32, 64);
    l = l * alpha + ls;
    m = mn;
#pragma unroll
    for (int tl = 0; tl < NTL; ++tl)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[tl][r] *= alpha;
    mfma_colsT_x_regs<HD>(V_s, s, lane, o);        // O^T += V^T P^T
  }
  if (!qv) return;
  const float inv = l > 0.f ? 1.f / l : 0.f;
  store_dT<HD>(out + (q0 + qi) * so + hh * HD, o, inv, h);
  if (h == 0) lse[(int64_t)hh * Tq + q0 + qi] = l > 0.f ? m + logf(l) : 0.f;
}

// ------------------------------------------------------------------------------- bwd: dK, dV
template <int HD, int NW>
__global__ void __launch_bounds__(64 * NW) attn_bwd_dkdv_kernel(
    const float* __restrict__ q, int64_t sq, const float* __restrict__ k, int64_t sk, const float* __restrict__ v,
    int64_t sv, const float* __restrict__ out, int64_t so, const float* __restrict__ dout, int64_t sdo,
    const float* __restrict__ lse, const float* __restrict__ delta, int64_t Tq, const int64_t* __restrict__ cu_q,
    const int64_t* __restrict__ cu_k, int causal, float scale, float* __restrict__ dk, int64_t sdk,
    float* __restrict__ dv, int64_t sdv) {
  constexpr int LD = Pad<HD>::LD, NTL = Pad<HD>::P / 32;
  __shared__ __attribute__((aligned(16))) float smem[2 * 32 * LD + 64];
  float* Q_s = smem;
  float* O_s = smem + 32 * LD;   // dO tile
  float* lse_s = O_s + 32 * LD;
  float* dl_s = lse_s + 32;
  const int b = blockIdx.z, hh = blockIdx.y, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, h = lane >> 5;
  zero_pad32<HD, 64 * NW>(Q_s, tid);
  zero_pad32<HD, 64 * NW>(O_s, tid);
  const int64_t q0 = cu_q[b], k0 = cu_k[b];
  const int lq = (int)(cu_q[b + 1] - q0), lk = (int)(cu_k[b + 1] - k0);
  const int kbase = blockIdx.x * 32 * NW;
  if (kbase >= lk) return;
  const int kj = kbase + wave * 32 + (lane & 31);
  const bool kv = kj < lk;
  float kf[HD / 2], vf[HD / 2];
  load_half_row<HD>(k + (k0 + (kv ? kj : 0)) * sk + hh * HD + h * (HD / 2), kv, kf);
  load_half_row<HD>(v + (k0 + (kv ? kj : 0)) * sv + hh * HD + h * (HD / 2), kv, vf);
  floatx16 dka[NTL], dva[NTL];
#pragma unroll
  for (int tl = 0; tl < NTL; ++tl)
#pragma unroll
    for (int r = 0; r < 16; ++r) { dka[tl][r] = 0.f; dva[tl][r] = 0.f; }
  const int qstart = causal ? (kbase / 32) * 32 : 0;
  for (int qt = qstart; qt < lq; qt += 32) {
    __syncthreads();
    stage32<HD, 64 * NW>(Q_s, q + q0 * sq + hh * HD, sq, qt, lq, tid);
    stage32<HD, 64 * NW>(O_s, dout + q0 * sdo + hh * HD, sdo, qt, lq, tid);
    if (tid < 32) {   // delta_q = sum_d dO*O (written by the dQ pass) and lse for the 32 queries
      const int qq = qt + tid;
      const bool ok = qq < lq;
      dl_s[tid] = ok ? delta[(int64_t)hh * Tq + q0 + qq] : 0.f;
      lse_s[tid] = ok ? lse[(int64_t)hh * Tq + q0 + qq] : 0.f;
    }
    __syncthreads();
    floatx16 s, dp;
#pragma unroll
    for (int r = 0; r < 16; ++r) { s[r] = 0.f; dp[r] = 0.f; }
    s = mfma_rows_x_frag<HD>(Q_s, kf, lane, s);    // S: rows = queries, cols = keys
    dp = mfma_rows_x_frag<HD>(O_s, vf, lane, dp);  // dP = dO V^T
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qr = crow(r, h), qq = qt + qr;
      const bool ok = kv && qq < lq && (!causal || kj <= qq);
      const float p = ok ? expf(s[r] * scale - lse_s[qr]) : 0.f;
      s[r] = p;
      dp[r] = p * (dp[r] - dl_s[qr]);
    }
    mfma_colsT_x_regs<HD>(O_s, s, lane, dva);   // dV^T += dO^T P
    mfma_colsT_x_regs<HD>(Q_s, dp, lane, dka);  // dK^T += Q^T dS
  }
  if (!kv) return;
  store_dT<HD>(dk + (k0 + kj) * sdk + hh * HD, dka, scale, h);
  store_dT<HD>(dv + (k0 + kj) * sdv + hh * HD, dva, 1.f, h);
}

// ------------------------------------------------------------------------------------ bwd: dQ
template <int HD, int NW>
__global__ void __launch_bounds__(64 * NW) attn_bwd_dq_kernel(
    const float* __restrict__ q, int64_t sq, const float* __restrict__ k, int64_t sk, const float* __restrict__ v,
    int64_t sv, const float* __restrict__ out, int64_t so, const float* __restrict__ dout, int64_t sdo,
    const float* __restrict__ lse, int64_t Tq, const int64_t* __restrict__ cu_q, const int64_t* __restrict__ cu_k,
    int causal, float scale, float* __restrict__ dq, int64_t sdq, float* __restrict__ delta_out) {
  constexpr int LD = Pad<HD>::LD, NTL = Pad<HD>::P / 32;
  __shared__ __attribute__((aligned(16))) float smem[2 * 32 * LD];
  float* K_s = smem;
  float* V_s = smem + 32 * LD;
  const int b = blockIdx.z, hh = blockIdx.y, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, h = lane >> 5;
  zero_pad32<HD, 64 * NW>(K_s, tid);
  zero_pad32<HD, 64 * NW>(V_s, tid);
  const int64_t q0 = cu_q[b], k0 = cu_k[b];
  const int lq = (int)(cu_q[b + 1] - q0), lk = (int)(cu_k[b + 1] - k0);
  const int qbase = blockIdx.x * 32 * NW;
  if (qbase >= lq) return;
  const int qi = qbase + wave * 32 + (lane & 31);
  const bool qv = qi < lq;
  const int64_t qrow = q0 + (qv ? qi : 0);
  float qf[HD / 2], dof[HD / 2];
  load_half_row<HD>(q + qrow * sq + hh * HD + h * (HD / 2), qv, qf);
  load_half_row<HD>(dout + qrow * sdo + hh * HD + h * (HD / 2), qv, dof);
  float delta = 0.f;
  {
    const float* orow = out + qrow * so + hh * HD + h * (HD / 2);
    if (qv)
      for (int d = 0; d < HD / 2; ++d) delta += dof[d] * orow[d];
    delta += __shfl_xor(delta, 32, 64);
    if (qv && h == 0) delta_out[(int64_t)hh * Tq + qrow] = delta;   // reused by the dK/dV pass
  }
  const float lq_lse = qv ? lse[(int64_t)hh * Tq + qrow] : 0.f;
  floatx16 dqa[NTL];
#pragma unroll
  for (int tl = 0; tl < NTL; ++tl)
#pragma unroll
    for (int r = 0; r < 16; ++r) dqa[tl][r] = 0.f;
  const int kend = causal ? min(lk, qbase + 32 * NW) : lk;
  for (int kt = 0; kt < kend; kt += 32) {
    __syncthreads();
    stage32<HD, 64 * NW>(K_s, k + k0 * sk + hh * HD, sk, kt, lk, tid);
    stage32<HD, 64 * NW>(V_s, v + k0 * sv + hh * HD, sv, kt, lk, tid);
    __syncthreads();
    floatx16 s, dp;
#pragma unroll
    for (int r = 0; r < 16; ++r) { s[r] = 0.f; dp[r] = 0.f; }
    s = mfma_rows_x_frag<HD>(K_s, qf, lane, s);    // S^T
    dp = mfma_rows_x_frag<HD>(V_s, dof, lane, dp); // dP^T = V dO^T
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = kt + crow(r, h);
      const bool ok = qv && key < lk && (!causal || key <= qi);
      const float p = ok ? expf(s[r] * scale - lq_lse) : 0.f;
      s[r] = p * (dp[r] - delta);   // dS^T
    }
    mfma_colsT_x_regs<HD>(K_s, s, lane, dqa);     // dQ^T += K^T dS^T
  }
  if (!qv) return;
  store_dT<HD>(dq + (q0 + qi) * sdq + hh * HD, dqa, scale, h);
}

// Short sequences (<= 96 rows, e.g. Amazon contexts of <= 81 tokens) run one wave (32 rows) per
// workgroup so no wave idles on a padded 32-row half; longer ones share each staged K/V (Q/dO)
// tile between two waves.
template <int HD>
static void launch_fwd(int64_t B, int64_t H, int64_t max_q, hipStream_t st, const float* q, int64_t sq, const float* k,
                       int64_t sk, const float* v, int64_t sv, const int64_t* cq, const int64_t* ck, int causal,
                       float scale, float* out, int64_t so, float* lse, int64_t Tq) {
  if (max_q <= RQ_ATTN_ONE_WAVE_MAX) {
    dim3 g((unsigned)((max_q + 31) / 32), (unsigned)H, (unsigned)B);
    hipLaunchKernelGGL((attn_fwd_kernel<HD, 1>), g, dim3(64), 0, st, q, sq, k, sk, v, sv, cq, ck, causal, scale, out,
                       so, lse, Tq);
  } else {
    dim3 g((unsigned)((max_q + 63) / 64), (unsigned)H, (unsigned)B);
    hipLaunchKernelGGL((attn_fwd_kernel<HD, 2>), g, dim3(128), 0, st, q, sq, k, sk, v, sv, cq, ck, causal, scale, out,
                       so, lse, Tq);
  }
}

template <int HD>
static void launch_bwd(int64_t B, int64_t H, int64_t max_q, int64_t max_k, hipStream_t st, const float* q, int64_t sq,
                       const float* k, int64_t sk, const float* v, int64_t sv, const float* out, int64_t so,
                       const float* dout, int64_t sdo, const float* lse, int64_t Tq, const int64_t* cq, const int64_t* ck,
                       int causal, float scale, float* dq, int64_t sdq, float* dk, int64_t sdk, float* dv, int64_t sdv,
                       float* delta) {
  // dQ pass first: it also writes delta_q = dO.O, which the dK/dV pass reads per query tile
  if (max_q <= RQ_ATTN_ONE_WAVE_MAX) {
    dim3 gq((unsigned)((max_q + 31) / 32), (unsigned)H, (unsigned)B);
    hipLaunchKernelGGL((attn_bwd_dq_kernel<HD, 1>), gq, dim3(64), 0, st, q, sq, k, sk, v, sv, out, so, dout, sdo, lse,
                       Tq, cq, ck, causal, scale, dq, sdq, delta);
  } else {
    dim3 gq((unsigned)((max_q + 63) / 64), (unsigned)H, (unsigned)B);
    hipLaunchKernelGGL((attn_bwd_dq_kernel<HD, 2>), gq, dim3(128), 0, st, q, sq, k, sk, v, sv, out, so, dout, sdo, lse,
                       Tq, cq, ck, causal, scale, dq, sdq, delta);
  }
  if (max_k <= RQ_ATTN_ONE_WAVE_MAX) {
    dim3 gk((unsigned)((max_k + 31) / 32), (unsigned)H, (unsigned)B);
    hipLaunchKernelGGL((attn_bwd_dkdv_kernel<HD, 1>), gk, dim3(64), 0, st, q, sq, k, sk, v, sv, out, so, dout, sdo,
                       lse, delta, Tq, cq, ck, causal, scale, dk, sdk, dv, sdv);
  } else {
    dim3 gk((unsigned)((max_k + 63) / 64), (unsigned)H, (unsigned)B);
    hipLaunchKernelGGL((attn_bwd_dkdv_kernel<HD, 2>), gk, dim3(128), 0, st, q, sq, k, sk, v, sv, out, so, dout, sdo,
                       lse, delta, Tq, cq, ck, causal, scale, dk, sdk, dv, sdv);
  }
}

static bool attn_args_ok(int64_t B, int64_t H, int64_t hd, int64_t max_q, int64_t max_k) {
  // max_q / max_k bound the grid's x extent and every in-kernel int index (row * stride fits int64)
  return B >= 0 && B <= 65535 && H >= 1 && H <= 65535 && (hd == 16 || hd == 32 || hd == 64 || hd == 128) && max_q >= 0 &&
         max_k >= 0 && max_q <= (1 << 24) && max_k <= (1 << 24);
}

}  // namespace rqhip

using namespace rqhip;

extern "C" {

int varlen_attn_fwd(const float* q, int64_t sq, const float* k, int64_t sk, const float* v, int64_t sv,
                    const int64_t* cu_q, const int64_t* cu_k, int64_t B, int64_t H, int64_t hd, int64_t max_q,
                    int64_t max_k, int causal, float scale, float* out, int64_t so, float* lse, int64_t Tq, void* stream) {
  RQ_CHECK_ARG(q && k && v && cu_q && cu_k && out && lse, "varlen_attn_fwd: null pointer");
  RQ_CHECK_ARG(attn_args_ok(B, H, hd, max_q, max_k), "varlen_attn_fwd: bad shape (hd must be 16/32/64/128, B<=65535)");
  RQ_CHECK_ARG(sq % 4 == 0 && sk % 4 == 0 && sv % 4 == 0 && so % 4 == 0, "varlen_attn_fwd: row strides must be x4");
  if (B == 0 || max_q == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  switch (hd) {
    case 16: launch_fwd<16>(B, H, max_q, st, q, sq, k, sk, v, sv, cu_q, cu_k, causal, scale, out, so, lse, Tq); break;
    case 32: launch_fwd<32>(B, H, max_q, st, q, sq, k, sk, v, sv, cu_q, cu_k, causal, scale, out, so, lse, Tq); break;
    case 64: launch_fwd<64>(B, H, max_q, st, q, sq, k, sk, v, sv, cu_q, cu_k, causal, scale, out, so, lse, Tq); break;
    case 128: launch_fwd<128>(B, H, max_q, st, q, sq, k, sk, v, sv, cu_q, cu_k, causal, scale, out, so, lse, Tq); break;
  }
  RQ_LAUNCH_CHECK("varlen_attn_fwd");
  return 0;
}

int varlen_attn_bwd(const float* q, int64_t sq, const float* k, int64_t sk, const float* v, int64_t sv, const float* out,
                    int64_t so, const float* dout, int64_t sdo, const float* lse, int64_t Tq, const int64_t* cu_q,
                    const int64_t* cu_k, int64_t B, int64_t H, int64_t hd, int64_t max_q, int64_t max_k, int causal,
                    float scale, float* dq, int64_t sdq, float* dk, int64_t sdk, float* dv, int64_t sdv, float* delta,
                    void* stream) {
  RQ_CHECK_ARG(q && k && v && out && dout && lse && cu_q && cu_k && dq && dk && dv && delta,
               "varlen_attn_bwd: null pointer");
  RQ_CHECK_ARG(attn_args_ok(B, H, hd, max_q, max_k), "varlen_attn_bwd: bad shape (hd must be 16/32/64/128, B<=65535)");
  RQ_CHECK_ARG(sq % 4 == 0 && sk % 4 == 0 && sv % 4 == 0 && so % 4 == 0 && sdo % 4 == 0 && sdq % 4 == 0 &&
                   sdk % 4 == 0 && sdv % 4 == 0,
               "varlen_attn_bwd: row strides must be x4");
  if (B == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  switch (hd) {
    case 16: launch_bwd<16>(B, H, max_q, max_k, st, q, sq, k, sk, v, sv, out, so, dout, sdo, lse, Tq, cu_q, cu_k, causal, scale, dq, sdq, dk, sdk, dv, sdv, delta); break;
    case 32: launch_bwd<32>(B, H, max_q, max_k, st, q, sq, k, sk, v, sv, out, so, dout, sdo, lse, Tq, cu_q, cu_k, causal, scale, dq, sdq, dk, sdk, dv, sdv, delta); break;
    case 64: launch_bwd<64>(B, H, max_q, max_k, st, q, sq, k, sk, v, sv, out, so, dout, sdo, lse, Tq, cu_q, cu_k, causal, scale, dq, sdq, dk, sdk, dv, sdv, delta); break;
    case 128: launch_bwd<128>(B, H, max_q, max_k, st, q, sq, k, sk, v, sv, out, so, dout, sdo, lse, Tq, cu_q, cu_k, causal, scale, dq, sdq, dk, sdk, dv, sdv, delta); break;
  }
  RQ_LAUNCH_CHECK("varlen_attn_bwd");
  return 0;
}

}  // extern "C"
