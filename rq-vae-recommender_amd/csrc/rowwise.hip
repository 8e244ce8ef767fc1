// Row-wise fused kernels around the RQ-VAE decoder head (HBM-bound, one wave per row).
//
// Reference: modules/rqvae.py:145-150 — x_hat = decoder(sum_l emb_l) where the decoder MLP ends
// in l2norm (modules/encoder.py:34 with modules/normalize.py:7-8, F.normalize eps 1e-12), then
// ReconstructionLoss: recon_b = sum_c (x_hat_bc - x_bc)^2 (modules/loss.py:5-10).
// In eager torch that is ~10 separate B x C passes forward+backward; fused here into one read
// of (pre, x) forward and one read + one write backward:
//   fwd: n_b = max(|pre_b|, 1e-12); y = pre_b / n_b; recon_b = sum (y - x_b)^2; saves n_b
//   bwd: g_y = 2 g_b (y - x_b); g_pre = (g_y - y (g_y . y)) / n_b   (|pre_b| > eps)
//                                g_pre = g_y / eps                  (clamped rows)
//        written fp32, or (rq_l2norm_recon_bwd_split) as the split-bf16 planes the next data-grad /
//        weight-grad GEMMs of the 'high' path consume directly (same bytes as fp32).
#include "common.h"

#include <algorithm>
#include <stdlib.h>

namespace rqhip {

// The gradient of one row from its values in registers (pre: av, x: bv, zero past C), its norm
// |pre_r| (raw) and g_recon[r] (gr): shared by the backward kernel and the forward's speculative
// gradient, so the two write the same bits for the same gr.
template <int VPL, bool SPLIT>
__device__ __forceinline__ void l2r_grad_row(const float4 (&av)[VPL], const float4 (&bv)[VPL], float raw, float gr,
                                             int64_t r, int C, int lane, float* __restrict__ g_pre,
                                             uint16_t* __restrict__ g_hi, uint16_t* __restrict__ g_lo) {
  const float n = fmaxf(raw, 1e-12f);
  const float g2 = 2.f * gr;
  float4 yv[VPL], gy[VPL];
  float dot = 0.f;
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    const float4 a = av[v], b = bv[v];
    yv[v] = make_float4(a.x / n, a.y / n, a.z / n, a.w / n);
    gy[v] = make_float4(g2 * (yv[v].x - b.x), g2 * (yv[v].y - b.y), g2 * (yv[v].z - b.z), g2 * (yv[v].w - b.w));
    dot += gy[v].x * yv[v].x + gy[v].y * yv[v].y + gy[v].z * yv[v].z + gy[v].w * yv[v].w;
  }
  dot = group_sum<64>(dot);
  const bool clamped = !(raw > 1e-12f);
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    const int c = (v * 64 + lane) * 4;
    if (c >= C) continue;
    float4 o;
    if (clamped) {
      o = make_float4(gy[v].x / n, gy[v].y / n, gy[v].z / n, gy[v].w / n);
    } else {
      o = make_float4((gy[v].x - yv[v].x * dot) / n, (gy[v].y - yv[v].y * dot) / n, (gy[v].z - yv[v].z * dot) / n,
                      (gy[v].w - yv[v].w * dot) / n);
    }
    if constexpr (SPLIT)
      split_store4(o, g_hi + r * C + c, g_lo + r * C + c);
    else
      *reinterpret_cast<float4*>(g_pre + r * C + c) = o;
  }
}

template <int VPL>
__device__ __forceinline__ void l2r_load_row(const float* __restrict__ pre, const float* __restrict__ x, int64_t r,
                                             int C, int lane, float4 (&pv)[VPL], float4 (&xv)[VPL]) {
  const float* p = pre + r * C;
  const float* q = x + r * C;
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    const int c = (v * 64 + lane) * 4;
    const bool ok = c < C;
    pv[v] = ok ? *reinterpret_cast<const float4*>(p + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    xv[v] = ok ? *reinterpret_cast<const float4*>(q + c) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// Forward, one row per wave (C = 256 VPL at most). GRAD: also the split gradient the backward would
// write for g_recon[r] = gs (the batch-mean loss's uniform 1 / B): the backward then only checks g_recon
// (l2norm_recon_fix_kernel) instead of reading pre and x again.
template <int VPL, bool GRAD>
__global__ void __launch_bounds__(256) l2norm_recon_fwd_kernel(const float* __restrict__ pre, const float* __restrict__ x,
                                                                int64_t B, int C, float* __restrict__ recon,
                                                                float* __restrict__ nrm, float gs,
                                                                uint16_t* __restrict__ g_hi, uint16_t* __restrict__ g_lo) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= B) return;
  float4 pv[VPL], xv[VPL];
  l2r_load_row<VPL>(pre, x, r, C, lane, pv, xv);
  float s = 0.f;
#pragma unroll
  for (int v = 0; v < VPL; ++v) s += pv[v].x * pv[v].x + pv[v].y * pv[v].y + pv[v].z * pv[v].z + pv[v].w * pv[v].w;
  s = group_sum<64>(s);
  const float n = fmaxf(sqrtf(s), 1e-12f);
  float acc = 0.f;
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    if ((v * 64 + lane) * 4 >= C) continue;
    const float d0 = pv[v].x / n - xv[v].x, d1 = pv[v].y / n - xv[v].y;
    const float d2 = pv[v].z / n - xv[v].z, d3 = pv[v].w / n - xv[v].w;
    acc += d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
  }
  acc = group_sum<64>(acc);
  if (lane == 0) {
    recon[r] = acc;
    nrm[r] = sqrtf(s);
  }
  if constexpr (GRAD) l2r_grad_row<VPL, true>(pv, xv, sqrtf(s), gs, r, C, lane, nullptr, g_hi, g_lo);
}

// Backward, one row per wave.
template <int VPL, bool SPLIT>
__global__ void __launch_bounds__(256) l2norm_recon_bwd_kernel(const float* __restrict__ pre, const float* __restrict__ x,
                                                                const float* __restrict__ nrm,
                                                                const float* __restrict__ g_recon, int64_t B, int C,
                                                                float* __restrict__ g_pre, uint16_t* __restrict__ g_hi,
                                                                uint16_t* __restrict__ g_lo) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= B) return;
  float4 av[VPL], bv[VPL];
  const float raw = nrm[r], gr = g_recon[r];
  l2r_load_row<VPL>(pre, x, r, C, lane, av, bv);
  l2r_grad_row<VPL, SPLIT>(av, bv, raw, gr, r, C, lane, g_pre, g_hi, g_lo);
}

// Backward after a GRAD forward: rows whose g_recon[r g_stride] is bitwise gs already hold their split
// gradient; any other row (a weighted or scaled loss) is recomputed from pre and x. Waves stride over
// the rows (at most 2,048 workgroups, not one per row: the common case reads one scalar per wave).
template <int VPL>
__global__ void __launch_bounds__(256) l2norm_recon_fix_kernel(const float* __restrict__ pre, const float* __restrict__ x,
                                                                const float* __restrict__ nrm,
                                                                const float* __restrict__ g_recon, int64_t g_stride,
                                                                int64_t B, int C, uint32_t gs_bits,
                                                                uint16_t* __restrict__ g_hi, uint16_t* __restrict__ g_lo) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < B; r += nw) {
    const float gr = g_recon[r * g_stride];
    if (__float_as_uint(gr) == gs_bits) {
      if (g_stride == 0) return;   // one value for every row: all done
      continue;
    }
    float4 av[VPL], bv[VPL];
    l2r_load_row<VPL>(pre, x, r, C, lane, av, bv);
    l2r_grad_row<VPL, true>(av, bv, nrm[r], gr, r, C, lane, nullptr, g_hi, g_lo);
  }
}

// One row per wave: 2 or 4 rows per wave were no faster at 65,536 x 768 (profiles/r02/l2r_rpw_ab.txt).

// ---------------------------------------------------------------------------------------
// RMSNorm (modules/normalize.py:22-32): t = x * rsqrt(mean(x^2) + eps), y = t * w.
// fwd: one wave per row, saves rstd. bwd: gx = r (w gy) - x (r^3 / D) sum_j (w gy x)_j per row;
// gw = sum_b gy_b t_b reduced deterministically: each 4-wave workgroup owns kRmsRows rows and writes
// a [D] partial (waves combined in order through LDS), rms_reduce_kernel sums partials in order.
constexpr int kRmsRows = 16;   // rows per workgroup: T=11.6k decoder rows -> 725 workgroups
// Fewer rows per workgroup (8, 4: one row per wave) while 16-row workgroups would leave the chip half
// empty (ML-32M at 8 sequences per GPU: ~3.2k rows -> 200 workgroups, each wave walking 4 dependent
// rows); the partials (one [D] row per workgroup) stay small either way.
static int rms_rows_per_blk(int64_t B) {
  int r = kRmsRows;
  while (r > 4 && (B + r - 1) / r < 512) r /= 2;
  return r;
}

template <int VPL>
__global__ void __launch_bounds__(256) rmsnorm_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                          int64_t B, int D, float eps, uint32_t thr, float dscale,
                                                          uint64_t seed, float* __restrict__ y,
                                                          float* __restrict__ rstd) {
  seed = epoch_seed(seed);
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= B) return;
  const float* p = x + r * D;
  float4 xv[VPL];
  float s = 0.f;
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    const int c = (v * 64 + lane) * 4;
    xv[v] = c < D ? *reinterpret_cast<const float4*>(p + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    s = __builtin_fmaf(xv[v].x, xv[v].x, s);
    s = __builtin_fmaf(xv[v].y, xv[v].y, s);
    s = __builtin_fmaf(xv[v].z, xv[v].z, s);
    s = __builtin_fmaf(xv[v].w, xv[v].w, s);
  }
  s = group_sum<64>(s);
  const float rs = rsqrtf(s / (float)D + eps);
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    const int c = (v * 64 + lane) * 4;
    if (c >= D) continue;
    const float4 wv = *reinterpret_cast<const float4*>(w + c);
    *reinterpret_cast<float4*>(y + r * D + c) =
        drop4(make_float4((xv[v].x * rs) * wv.x, (xv[v].y * rs) * wv.y, (xv[v].z * rs) * wv.z, (xv[v].w * rs) * wv.w),
              seed, (uint64_t)(r * D + c) / 4, thr, dscale);
  }
  if (lane == 0) rstd[r] = rs;
}

template <int VPL>
__global__ void __launch_bounds__(256) rmsnorm_bwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                          const float* __restrict__ rstd, const float* __restrict__ gy,
                                                          int64_t B, int D, uint32_t thr, float dscale, uint64_t seed,
                                                          const float* __restrict__ gres, float* __restrict__ gx,
                                                          float* __restrict__ gw_part, int rows) {
  seed = epoch_seed(seed);
  __shared__ float4 part[4][VPL * 64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float4 wv[VPL], gwa[VPL];
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    const int c = (v * 64 + lane) * 4;
    wv[v] = c < D ? *reinterpret_cast<const float4*>(w + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    gwa[v] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const float invD = 1.f / (float)D;
  for (int i = wave; i < rows; i += 4) {
    const int64_t r = (int64_t)blockIdx.x * rows + i;
    if (r >= B) break;
    const float rs = rstd[r];
    float4 xv[VPL], gt[VPL];
    float dot = 0.f;
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      const int c = (v * 64 + lane) * 4;
      const bool ok = c < D;
      xv[v] = ok ? *reinterpret_cast<const float4*>(x + r * D + c) : make_float4(0.f, 0.f, 0.f, 0.f);
      const float4 g = ok ? drop4(*reinterpret_cast<const float4*>(gy + r * D + c), seed, (uint64_t)(r * D + c) / 4, thr,
                                  dscale)
                          : make_float4(0.f, 0.f, 0.f, 0.f);
      gt[v] = make_float4(wv[v].x * g.x, wv[v].y * g.y, wv[v].z * g.z, wv[v].w * g.w);
      dot = __builtin_fmaf(gt[v].x, xv[v].x, dot);
      dot = __builtin_fmaf(gt[v].y, xv[v].y, dot);
      dot = __builtin_fmaf(gt[v].z, xv[v].z, dot);
      dot = __builtin_fmaf(gt[v].w, xv[v].w, dot);
      gwa[v].x = __builtin_fmaf(g.x, xv[v].x * rs, gwa[v].x);
      gwa[v].y = __builtin_fmaf(g.y, xv[v].y * rs, gwa[v].y);
      gwa[v].z = __builtin_fmaf(g.z, xv[v].z * rs, gwa[v].z);
      gwa[v].w = __builtin_fmaf(g.w, xv[v].w * rs, gwa[v].w);
    }
    dot = group_sum<64>(dot);
    const float k = rs * rs * rs * invD * dot;
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      const int c = (v * 64 + lane) * 4;
      if (c >= D) continue;
      float4 o = make_float4(rs * gt[v].x - xv[v].x * k, rs * gt[v].y - xv[v].y * k, rs * gt[v].z - xv[v].z * k,
                             rs * gt[v].w - xv[v].w * k);
      if (gres) {   // + the gradient reaching x along other paths (the residual stream): one pass
        const float4 e = *reinterpret_cast<const float4*>(gres + r * D + c);
        o = make_float4(o.x + e.x, o.y + e.y, o.z + e.z, o.w + e.w);
      }
      *reinterpret_cast<float4*>(gx + r * D + c) = o;
    }
  }
#pragma unroll
  for (int v = 0; v < VPL; ++v) part[wave][v * 64 + lane] = gwa[v];
  __syncthreads();
  if (wave == 0) {
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      const int c = (v * 64 + lane) * 4;
      if (c >= D) continue;
      float4 a = part[0][v * 64 + lane];
#pragma unroll
      for (int q = 1; q < 4; ++q) {
        const float4 b = part[q][v * 64 + lane];
        a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
      }
      *reinterpret_cast<float4*>(gw_part + (int64_t)blockIdx.x * D + c) = a;
    }
  }
}

// Two RMSNorms of the same rows (the decoder block's attn_norm and cross_attn_norm of x,
// modules/transformer/model.py:75-82): rstd once, y1 = Dropout_1(t w1), y2 = Dropout_2(t w2) — bitwise the two
// single-norm launches, in one. The backward gives gx = norm2'(g2) + (norm1'(g1) + gres) in that order (the
// chained single-norm launches' roundings) and both weight-gradient partials.
template <int VPL>
__global__ void __launch_bounds__(256) rmsnorm2_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w1,
                                                           const float* __restrict__ w2, int64_t B, int D, float eps,
                                                           uint32_t thr1, float ds1, uint64_t seed1, uint32_t thr2,
                                                           float ds2, uint64_t seed2, float* __restrict__ y1,
                                                           float* __restrict__ y2, float* __restrict__ rstd) {
  seed1 = epoch_seed(seed1);
  seed2 = epoch_seed(seed2);
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= B) return;
  const float* p = x + r * D;
  float4 xv[VPL];
  float s = 0.f;
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    const int c = (v * 64 + lane) * 4;
    xv[v] = c < D ? *reinterpret_cast<const float4*>(p + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    s = __builtin_fmaf(xv[v].x, xv[v].x, s);
    s = __builtin_fmaf(xv[v].y, xv[v].y, s);
    s = __builtin_fmaf(xv[v].z, xv[v].z, s);
    s = __builtin_fmaf(xv[v].w, xv[v].w, s);
  }
  s = group_sum<64>(s);
  const float rs = rsqrtf(s / (float)D + eps);
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    const int c = (v * 64 + lane) * 4;
    if (c >= D) continue;
    const float4 t = make_float4(xv[v].x * rs, xv[v].y * rs, xv[v].z * rs, xv[v].w * rs);
    const float4 a = *reinterpret_cast<const float4*>(w1 + c);
    const float4 b = *reinterpret_cast<const float4*>(w2 + c);
    const uint64_t e = (uint64_t)(r * D + c) / 4;
    *reinterpret_cast<float4*>(y1 + r * D + c) =
        drop4(make_float4(t.x * a.x, t.y * a.y, t.z * a.z, t.w * a.w), seed1, e, thr1, ds1);
    *reinterpret_cast<float4*>(y2 + r * D + c) =
        drop4(make_float4(t.x * b.x, t.y * b.y, t.z * b.z, t.w * b.w), seed2, e, thr2, ds2);
  }
  if (lane == 0) rstd[r] = rs;
}

template <int VPL>
__device__ __forceinline__ void rms_part_store(float4 (&part)[4][VPL * 64], const float4 (&gwa)[VPL], int wave, int lane,
                                               int D, float* __restrict__ gw_part) {
#pragma unroll
  for (int v = 0; v < VPL; ++v) part[wave][v * 64 + lane] = gwa[v];
  __syncthreads();
  if (wave == 0) {
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      const int c = (v * 64 + lane) * 4;
      if (c >= D) continue;
      float4 a = part[0][v * 64 + lane];
#pragma unroll
      for (int q = 1; q < 4; ++q) {
        const float4 b = part[q][v * 64 + lane];
        a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
      }
      *reinterpret_cast<float4*>(gw_part + (int64_t)blockIdx.x * D + c) = a;
    }
  }
  __syncthreads();   // part is reused by the next call
}

template <int VPL>
__global__ void __launch_bounds__(256) rmsnorm2_bwd_kernel(const float* __restrict__ x, const float* __restrict__ w1,
                                                           const float* __restrict__ w2, const float* __restrict__ rstd,
                                                           const float* __restrict__ gy1, const float* __restrict__ gy2,
                                                           int64_t B, int D, uint32_t thr1, float ds1, uint64_t seed1,
                                                           uint32_t thr2, float ds2, uint64_t seed2,
                                                           const float* __restrict__ gres, float* __restrict__ gx,
                                                           float* __restrict__ gw1_part, float* __restrict__ gw2_part,
                                                           int rows) {
  seed1 = epoch_seed(seed1);
  seed2 = epoch_seed(seed2);
  __shared__ float4 part[4][VPL * 64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float4 wa[VPL], wb[VPL], ga[VPL], gb[VPL];
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    const int c = (v * 64 + lane) * 4;
    wa[v] = c < D ? *reinterpret_cast<const float4*>(w1 + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    wb[v] = c < D ? *reinterpret_cast<const float4*>(w2 + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    ga[v] = gb[v] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const float invD = 1.f / (float)D;
  for (int i = wave; i < rows; i += 4) {
    const int64_t r = (int64_t)blockIdx.x * rows + i;
    if (r >= B) break;
    const float rs = rstd[r];
    float4 xv[VPL], t1[VPL], t2[VPL];
    float d1 = 0.f, d2 = 0.f;
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      const int c = (v * 64 + lane) * 4;
      const bool ok = c < D;
      const uint64_t e = (uint64_t)(r * D + c) / 4;
      xv[v] = ok ? *reinterpret_cast<const float4*>(x + r * D + c) : make_float4(0.f, 0.f, 0.f, 0.f);
      const float4 g1 = ok ? drop4(*reinterpret_cast<const float4*>(gy1 + r * D + c), seed1, e, thr1, ds1)
                           : make_float4(0.f, 0.f, 0.f, 0.f);
      const float4 g2 = ok ? drop4(*reinterpret_cast<const float4*>(gy2 + r * D + c), seed2, e, thr2, ds2)
                           : make_float4(0.f, 0.f, 0.f, 0.f);
      t1[v] = make_float4(wa[v].x * g1.x, wa[v].y * g1.y, wa[v].z * g1.z, wa[v].w * g1.w);
      t2[v] = make_float4(wb[v].x * g2.x, wb[v].y * g2.y, wb[v].z * g2.z, wb[v].w * g2.w);
      d1 = __builtin_fmaf(t1[v].x, xv[v].x, d1);
      d1 = __builtin_fmaf(t1[v].y, xv[v].y, d1);
      d1 = __builtin_fmaf(t1[v].z, xv[v].z, d1);
      d1 = __builtin_fmaf(t1[v].w, xv[v].w, d1);
      d2 = __builtin_fmaf(t2[v].x, xv[v].x, d2);
      d2 = __builtin_fmaf(t2[v].y, xv[v].y, d2);
      d2 = __builtin_fmaf(t2[v].z, xv[v].z, d2);
      d2 = __builtin_fmaf(t2[v].w, xv[v].w, d2);
      ga[v].x = __builtin_fmaf(g1.x, xv[v].x * rs, ga[v].x);
      ga[v].y = __builtin_fmaf(g1.y, xv[v].y * rs, ga[v].y);
      ga[v].z = __builtin_fmaf(g1.z, xv[v].z * rs, ga[v].z);
      ga[v].w = __builtin_fmaf(g1.w, xv[v].w * rs, ga[v].w);
      gb[v].x = __builtin_fmaf(g2.x, xv[v].x * rs, gb[v].x);
      gb[v].y = __builtin_fmaf(g2.y, xv[v].y * rs, gb[v].y);
      gb[v].z = __builtin_fmaf(g2.z, xv[v].z * rs, gb[v].z);
      gb[v].w = __builtin_fmaf(g2.w, xv[v].w * rs, gb[v].w);
    }
    d1 = group_sum<64>(d1);
    d2 = group_sum<64>(d2);
    const float k1 = rs * rs * rs * invD * d1, k2 = rs * rs * rs * invD * d2;
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      const int c = (v * 64 + lane) * 4;
      if (c >= D) continue;
      float4 o = make_float4(rs * t1[v].x - xv[v].x * k1, rs * t1[v].y - xv[v].y * k1, rs * t1[v].z - xv[v].z * k1,
                             rs * t1[v].w - xv[v].w * k1);
      if (gres) {
        const float4 e = *reinterpret_cast<const float4*>(gres + r * D + c);
        o = make_float4(o.x + e.x, o.y + e.y, o.z + e.z, o.w + e.w);
      }
      const float4 q = make_float4(rs * t2[v].x - xv[v].x * k2, rs * t2[v].y - xv[v].y * k2,
                                   rs * t2[v].z - xv[v].z * k2, rs * t2[v].w - xv[v].w * k2);
      *reinterpret_cast<float4*>(gx + r * D + c) = make_float4(q.x + o.x, q.y + o.y, q.z + o.z, q.w + o.w);
    }
  }
  rms_part_store<VPL>(part, ga, wave, lane, D, gw1_part);
  rms_part_store<VPL>(part, gb, wave, lane, D, gw2_part);
}

// out[j] = sum_{s < S} P[s*n + j] in a fixed order (n % 4 == 0): a workgroup owns kRedCols float4
// columns; its 256 / kRedCols row lanes q sum s = q, q + 64, ... (strided_slab_sum), then the 64
// partials are combined by a fixed-shape tree through LDS. Deterministic, no atomics. Few columns per
// workgroup: at D = 512 and ~700 partials the sum is latency-bound, so more workgroups with shorter
// chains (32 x 11 loads per lane, not 8 x 44).
constexpr int kRedCols = 4;
__global__ void __launch_bounds__(256) rms_reduce_kernel(const float* __restrict__ P, int S, int64_t n,
                                                         float* __restrict__ out, int accumulate) {
  constexpr int kQ = 256 / kRedCols;
  __shared__ float4 red[kQ][kRedCols];
  const int c = threadIdx.x % kRedCols, q = threadIdx.x / kRedCols;
  const int64_t j = ((int64_t)blockIdx.x * kRedCols + c) * 4;
  const bool ok = j < n;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (ok) a = strided_slab_sum(P, S, n, j, q, kQ);
  red[q][c] = a;
  __syncthreads();
#pragma unroll
  for (int h = kQ / 2; h >= 1; h >>= 1) {
    if (q < h) {
      const float4 u = red[q][c], v = red[q + h][c];
      red[q][c] = make_float4(u.x + v.x, u.y + v.y, u.z + v.z, u.w + v.w);
    }
    __syncthreads();
  }
  if (q == 0 && ok) {
    float4 r = red[0][c];
    if (accumulate) {   // out += sum: a parameter gradient accumulated in place (flat DP bucket)
      const float4 o = *reinterpret_cast<const float4*>(out + j);
      r = make_float4(o.x + r.x, o.y + r.y, o.z + r.z, o.w + r.w);
    }
    *reinterpret_cast<float4*>(out + j) = r;
  }
}

// Row L2 norms: out[r] = sqrt(sum_d x[r][d]^2), one wave per row (the RqVae embs_norm statistic,
// modules/rqvae.py:155: emb.norm(dim=-1) over (L, B, D) embeddings in one pass).
// One row per group of G lanes (G = D / 4 rounded up to a power of two, <= 64): at D = 64 a wave
// covers 4 rows with every lane loading a float4 (one row per wave left 3/4 of the lanes idle).
template <int G>
__global__ void __launch_bounds__(256) row_norm_kernel(const float* __restrict__ x, int64_t rows, int D,
                                                       float* __restrict__ out) {
  const int lane = threadIdx.x & (G - 1);
  const int64_t r = (int64_t)blockIdx.x * (256 / G) + (threadIdx.x / G);
  const bool ok = r < rows;
  const float* p = x + (ok ? r : 0) * D;
  float s = 0.f;
  if (ok) {
    for (int c = lane * 4; c < D; c += 4 * G) {
      const float4 v = *reinterpret_cast<const float4*>(p + c);
      s = __builtin_fmaf(v.x, v.x, s);
      s = __builtin_fmaf(v.y, v.y, s);
      s = __builtin_fmaf(v.z, v.z, s);
      s = __builtin_fmaf(v.w, v.w, s);
    }
  }
  s = group_sum<G>(s);
  if (ok && lane == 0) out[r] = sqrtf(s);
}

// Their backward when only the total has a gradient (the train step): s = g * (1 / B) — torch's true_divide of
// a 0-dim tensor by the scalar B — once as a scalar (the reconstruction rows read it with stride 0) and as the
// (B,) per-row qloss gradient the quantize backward reads, in one launch (was a scalar op + an expand copy).
__global__ void __launch_bounds__(256) loss_means_bwd_kernel(const float* __restrict__ g, int64_t B, float inv_b,
                                                             float* __restrict__ out_scalar, float* __restrict__ out_vec) {
  const float v = g[0] * inv_b;
  const int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i0 == 0) *out_scalar = v;
  for (int64_t i = i0; i < B; i += (int64_t)gridDim.x * 256) out_vec[i] = v;
}

// The three scalar losses of RqVae.forward (modules/rqvae.py:151-162) in one pass over (B,) vectors:
// out = {mean(recon + qloss), mean(recon), mean(qloss)}; one 1024-thread workgroup, each thread a
// strided slice, then a fixed-order tree in LDS (deterministic).
__global__ void __launch_bounds__(1024) loss_means_kernel(const float* __restrict__ recon,
                                                          const float* __restrict__ ql, int64_t B,
                                                          float* __restrict__ out) {
  __shared__ float red[3][1024];
  const int t = threadIdx.x;
  float a = 0.f, b = 0.f, c = 0.f;
  // fixed order: thread t sums float4 groups t, t + 1024, ... (8 loads of each vector in flight: one
  // round trip per 8 groups, the same additions in the same order as 4 or 1 at a time), then the tail
  const int64_t n4 = B / 4;
  int64_t i = t;
  for (; i + 7 * 1024 < n4; i += 8 * 1024) {
    float4 r[8], q[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      r[u] = reinterpret_cast<const float4*>(recon)[i + u * 1024];
      q[u] = reinterpret_cast<const float4*>(ql)[i + u * 1024];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      a += (r[u].x + q[u].x) + (r[u].y + q[u].y) + (r[u].z + q[u].z) + (r[u].w + q[u].w);
      b += r[u].x + r[u].y + r[u].z + r[u].w;
      c += q[u].x + q[u].y + q[u].z + q[u].w;
    }
  }
  for (; i + 3 * 1024 < n4; i += 4 * 1024) {
    float4 r[4], q[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      r[u] = reinterpret_cast<const float4*>(recon)[i + u * 1024];
      q[u] = reinterpret_cast<const float4*>(ql)[i + u * 1024];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a += (r[u].x + q[u].x) + (r[u].y + q[u].y) + (r[u].z + q[u].z) + (r[u].w + q[u].w);
      b += r[u].x + r[u].y + r[u].z + r[u].w;
      c += q[u].x + q[u].y + q[u].z + q[u].w;
    }
  }
  for (; i < n4; i += 1024) {
    const float4 r = reinterpret_cast<const float4*>(recon)[i], q = reinterpret_cast<const float4*>(ql)[i];
    a += (r.x + q.x) + (r.y + q.y) + (r.z + q.z) + (r.w + q.w);
    b += r.x + r.y + r.z + r.w;
    c += q.x + q.y + q.z + q.w;
  }
  if (t < B - n4 * 4) {
    const float r = recon[n4 * 4 + t], q = ql[n4 * 4 + t];
    a += r + q;
    b += r;
    c += q;
  }
  red[0][t] = a; red[1][t] = b; red[2][t] = c;
  __syncthreads();
  for (int o = 512; o >= 64; o >>= 1) {   // pairwise tree: the cross-wave levels through LDS
    if (t < o) {
      red[0][t] += red[0][t + o]; red[1][t] += red[1][t + o]; red[2][t] += red[2][t + o];
    }
    __syncthreads();
  }
  if (t < 64) {   // the last six levels inside wave 0 (lane t < o adds lane t + o: the same tree, no barriers)
    float x0 = red[0][t], x1 = red[1][t], x2 = red[2][t];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      x0 += __shfl_down(x0, o, 64);
      x1 += __shfl_down(x1, o, 64);
      x2 += __shfl_down(x2, o, 64);
    }
    if (t == 0) {
      out[0] = x0 / (float)B;
      out[1] = x1 / (float)B;
      out[2] = x2 / (float)B;
    }
  }
}

// ------------------------------------------------------------- decoder output loss (cross-entropy)
// EncoderDecoderRetrievalModel.forward's loss head (reference modules/model.py:137-143):
//   logits = out_proj(..).view(B, L + 2, K)[:, :-1, :].flatten(0, 1)       (B * (L + 1), K)
//   unred  = cross_entropy(logits, sem_ids_fut.flatten(), reduction="none", ignore_index=-1).view(B, -1)
//   loss   = unred.sum(1).mean();   loss_d = unred.mean(0)
// as two forward launches (per-row log-sum-exp / loss / the contiguous logits copy; then the two means in
// one workgroup, fixed-order sums) and one backward launch (every row of the (B * npos_x, K) input
// gradient, zeros for the dropped last position and ignored targets) instead of ~13 torch kernels.
// Row r = b * npos + j of the logits is input row b * npos_x + j. One wave per row, K <= 1024.
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ void __launch_bounds__(256) ce_rows_kernel(const float* __restrict__ X, int64_t ldx, int K,
                                                      const int64_t* __restrict__ tgt, int rows, int npos,
                                                      int npos_x, float* __restrict__ u, float* __restrict__ lse,
                                                      float* __restrict__ logits) {
  const int lane = threadIdx.x & 63, r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int b = r / npos, j = r - b * npos;
  const float* x = X + ((int64_t)b * npos_x + j) * ldx;
  float* lg = logits + (int64_t)r * K;
  float m = -INFINITY;
  for (int k = lane; k < K; k += 64) {
    const float v = x[k];
    lg[k] = v;
    m = fmaxf(m, v);
  }
  m = wave_max(m);
  float s = 0.f;
  for (int k = lane; k < K; k += 64) s += expf(x[k] - m);
  s = wave_sum(s);
  if (lane == 0) {
    const float L = m + logf(s);
    const int64_t t = tgt[r];
    lse[r] = L;
    u[r] = t < 0 ? 0.f : (t < K ? L - x[t] : __builtin_nanf(""));   // out-of-range target: NaN, loudly
  }
}

// loss = (sum_b sum_j u[b][j]) / B, loss_d[j] = (sum_b u[b][j]) / B: one 256-thread workgroup; per-b row
// sums in order, then a fixed LDS tree; per-position sums sequential over b (deterministic).
constexpr int kCeStage = 8192;   // u values (B x npos) staged in LDS by the means kernel
__global__ void __launch_bounds__(256) ce_means_kernel(const float* __restrict__ u, int B, int npos,
                                                       float* __restrict__ loss, float* __restrict__ loss_d) {
  __shared__ float red[256];
  __shared__ float us[kCeStage];
  const int t = threadIdx.x;
  // the per-position means walk b serially (fixed order); with u in LDS (one coalesced pass by the whole
  // workgroup) those walks read LDS instead of issuing B dependent-order global loads per position (Amazon's
  // 256 x 4 values: 16.5 -> a few us). Same order, same bits.
  const int64_t nu = (int64_t)B * npos;
  const bool staged = nu <= kCeStage;
  if (staged) {
    for (int64_t i = t; i < nu; i += 256) us[i] = u[i];
    __syncthreads();
  }
  const float* __restrict__ src = staged ? us : u;
  float a = 0.f;
  for (int b = t; b < B; b += 256) {
    float sb = 0.f;
    for (int j = 0; j < npos; ++j) sb += src[(int64_t)b * npos + j];
    a += sb;
  }
  red[t] = a;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) red[t] += red[t + o];
    __syncthreads();
  }
  if (t == 0) loss[0] = red[0] / (float)B;
  for (int j = t; j < npos; j += 256) {
    float c = 0.f;
    for (int b = 0; b < B; ++b) c += src[(int64_t)b * npos + j];
    loss_d[j] = c / (float)B;
  }
}

// dX row R = b * npos_x + j: (g_loss + g_loss_d[j]) / B * (softmax(x) - onehot(t)) (+ g_logits row) for
// j < npos and t >= 0; g_logits only for j < npos and t < 0; zeros otherwise.
__global__ void __launch_bounds__(256) ce_bwd_kernel(const float* __restrict__ X, int64_t ldx, int K,
                                                     const int64_t* __restrict__ tgt, const float* __restrict__ lse,
                                                     int B, int npos, int npos_x, const float* __restrict__ g_loss,
                                                     const float* __restrict__ g_loss_d,
                                                     const float* __restrict__ g_logits, float* __restrict__ dX) {
  const int lane = threadIdx.x & 63, R = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (R >= B * npos_x) return;
  const int b = R / npos_x, j = R - b * npos_x;
  float* dx = dX + (int64_t)R * K;
  if (j >= npos) {
    for (int k = lane; k < K; k += 64) dx[k] = 0.f;
    return;
  }
  const int r = b * npos + j;
  const int64_t t = tgt[r];
  const float* gl = g_logits ? g_logits + (int64_t)r * K : nullptr;
  if (t < 0) {
    for (int k = lane; k < K; k += 64) dx[k] = gl ? gl[k] : 0.f;
    return;
  }
  const float g = ((g_loss ? g_loss[0] : 0.f) + (g_loss_d ? g_loss_d[j] : 0.f)) / (float)B;
  const float L = lse[r];
  const float* x = X + ((int64_t)b * npos_x + j) * ldx;
  for (int k = lane; k < K; k += 64) {
    const float p = expf(x[k] - L);
    const float v = g * (p - (k == t ? 1.f : 0.f));
    dx[k] = gl ? v + gl[k] : v;
  }
}


// ------------------------------------------------------------------------ Gumbel-softmax quantize
// Reference: modules/quantize.py:107-112,121,124-129 (training, GUMBEL_SOFTMAX, L2 distance) with
// distributions/gumbel.py:8-18: dist_k = |x|^2 + |c_k|^2 - 2 x.c_k; ids = argmin_k dist (lowest index on
// ties); w = softmax((-dist + g) / T) over the K codes (g: the Gumbel noise the caller sampled, as the
// reference's sample_gumbel does); emb = w @ codebook. One wave per row: lanes over codes for the
// distances / softmax (y and w staged in the wave's LDS slice), lanes over dims for the w @ codebook sum.
// Backward (rows independent): dw_k = g_emb . c_k; dy = w (dw - sum_j w_j dw_j) / T; ddist = -dy;
// dx = 2 x sum_k ddist_k - 2 sum_k ddist_k c_k. The codebook gradient (a K x B x D contraction:
// w^T g_emb + 2 colsum(ddist) c - 2 ddist^T x) is left to the caller's GEMMs, so ddist is written out.
constexpr int kGsMaxK = 4096, kGsMaxD = 256, kGsWaves = 4;

__device__ __forceinline__ float gs_wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ void __launch_bounds__(64 * kGsWaves) gumbel_softmax_fwd_kernel(
    const float* __restrict__ x, int64_t B, int D, const float* __restrict__ cb, int K, const float* __restrict__ noise,
    float inv_t, float* __restrict__ w_out, float* __restrict__ emb, int64_t* __restrict__ ids) {
  __shared__ float ys[kGsWaves][kGsMaxK];
  __shared__ float xs[kGsWaves][kGsMaxD];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * kGsWaves + wave;
  if (b >= B) return;   // uniform per wave; no workgroup barrier below
  const float* xr = x + b * D;
  float xx = 0.f;
  for (int d = lane; d < D; d += 64) {
    const float v = xr[d];
    xs[wave][d] = v;
    xx += v * v;
  }
  xx = gs_wave_sum(xx);
  __builtin_amdgcn_wave_barrier();   // xs of every lane visible to the wave
  float best = INFINITY, ymax = -INFINITY;
  int bi = 0x7fffffff;
  for (int k = lane; k < K; k += 64) {
    const float* c = cb + (int64_t)k * D;
    float dot = 0.f, cc = 0.f;
    for (int d = 0; d < D; ++d) {
      const float cv = c[d];
      dot += xs[wave][d] * cv;
      cc += cv * cv;
    }
    const float dist = xx + cc - 2.f * dot;
    if (dist < best) { best = dist; bi = k; }   // k ascending per lane: first minimum kept
    const float y = (noise[b * K + k] - dist) * inv_t;
    ys[wave][k] = y;
    ymax = fmaxf(ymax, y);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ob < best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    ymax = fmaxf(ymax, __shfl_xor(ymax, o, 64));
  }
  float se = 0.f;
  for (int k = lane; k < K; k += 64) {
    const float e = expf(ys[wave][k] - ymax);
    ys[wave][k] = e;
    se += e;
  }
  se = gs_wave_sum(se);
  const float inv = 1.f / se;
  for (int k = lane; k < K; k += 64) {
    const float wk = ys[wave][k] * inv;
    ys[wave][k] = wk;
    w_out[b * K + k] = wk;
  }
  if (lane == 0) ids[b] = bi;
  __builtin_amdgcn_wave_barrier();   // ys of every lane visible to the wave (LDS, same wave)
  for (int d = lane; d < D; d += 64) {
    float a = 0.f;
    for (int k = 0; k < K; ++k) a += ys[wave][k] * cb[(int64_t)k * D + d];
    emb[b * D + d] = a;
  }
}

__global__ void __launch_bounds__(64 * kGsWaves) gumbel_softmax_bwd_kernel(
    const float* __restrict__ x, const float* __restrict__ cb, const float* __restrict__ w, const float* __restrict__ g,
    int64_t B, int D, int K, float inv_t, float* __restrict__ dx, float* __restrict__ ddist) {
  __shared__ float ds[kGsWaves][kGsMaxK];
  __shared__ float gs[kGsWaves][kGsMaxD];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * kGsWaves + wave;
  if (b >= B) return;
  for (int d = lane; d < D; d += 64) gs[wave][d] = g[b * D + d];
  __builtin_amdgcn_wave_barrier();
  float swd = 0.f;
  for (int k = lane; k < K; k += 64) {
    const float* c = cb + (int64_t)k * D;
    float dw = 0.f;
    for (int d = 0; d < D; ++d) dw += gs[wave][d] * c[d];
    ds[wave][k] = dw;
    swd += w[b * K + k] * dw;
  }
  swd = gs_wave_sum(swd);
  float s1 = 0.f;
  for (int k = lane; k < K; k += 64) {
    const float dd = -w[b * K + k] * (ds[wave][k] - swd) * inv_t;
    ds[wave][k] = dd;
    ddist[b * K + k] = dd;
    s1 += dd;
  }
  s1 = gs_wave_sum(s1);
  __builtin_amdgcn_wave_barrier();
  for (int d = lane; d < D; d += 64) {
    float a = 0.f;
    for (int k = 0; k < K; ++k) a += ds[wave][k] * cb[(int64_t)k * D + d];
    dx[b * D + d] = 2.f * x[b * D + d] * s1 - 2.f * a;
  }
}

}  // namespace rqhip

using namespace rqhip;

extern "C" {

int rq_ce_loss_fwd(const float* X, int64_t ldx, int64_t K, const int64_t* tgt, int64_t B, int64_t npos, int64_t npos_x,
                   float* u, float* lse, float* logits, float* loss, float* loss_d, void* stream) {
  RQ_CHECK_ARG(B > 0 && K > 0 && K <= 1024 && npos > 0 && npos_x >= npos && ldx >= K && B * npos_x < (1LL << 31),
               "rq_ce_loss_fwd: bad shape");
  RQ_CHECK_ARG(X && tgt && u && lse && logits && loss && loss_d, "rq_ce_loss_fwd: null pointer");
  hipStream_t s = (hipStream_t)stream;
  const int rows = (int)(B * npos);
  hipLaunchKernelGGL(ce_rows_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, X, ldx, (int)K, tgt, rows,
                     (int)npos, (int)npos_x, u, lse, logits);
  hipLaunchKernelGGL(ce_means_kernel, dim3(1), dim3(256), 0, s, u, (int)B, (int)npos, loss, loss_d);
  RQ_LAUNCH_CHECK("rq_ce_loss_fwd");
  return 0;
}

int rq_ce_loss_bwd(const float* X, int64_t ldx, int64_t K, const int64_t* tgt, const float* lse, int64_t B, int64_t npos,
                   int64_t npos_x, const float* g_loss, const float* g_loss_d, const float* g_logits, float* dX,
                   void* stream) {
  RQ_CHECK_ARG(B > 0 && K > 0 && K <= 1024 && npos > 0 && npos_x >= npos && ldx >= K && B * npos_x < (1LL << 31),
               "rq_ce_loss_bwd: bad shape");
  RQ_CHECK_ARG(X && tgt && lse && dX, "rq_ce_loss_bwd: null pointer");
  const int rows = (int)(B * npos_x);
  hipLaunchKernelGGL(ce_bwd_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream, X, ldx, (int)K,
                     tgt, lse, (int)B, (int)npos, (int)npos_x, g_loss, g_loss_d, g_logits, dX);
  RQ_LAUNCH_CHECK("rq_ce_loss_bwd");
  return 0;
}

int rq_col_sum(const float* P, int64_t S, int64_t n, float* out, int accumulate, void* stream) {
  RQ_CHECK_ARG((P || S == 0) && out, "rq_col_sum: null pointer");
  RQ_CHECK_ARG(S >= 0 && S < (1ll << 31) && n > 0 && n % 4 == 0 && ((uintptr_t)P | (uintptr_t)out) % 16 == 0,
               "rq_col_sum: need n %% 4 == 0 and 16-byte aligned P / out");
  hipStream_t s = (hipStream_t)stream;
  if (S == 0) {
    if (!accumulate) RQ_HIP(zero_async(out, (size_t)n * sizeof(float), s));
    return 0;
  }
  hipLaunchKernelGGL(rms_reduce_kernel, dim3((unsigned)((n / 4 + kRedCols - 1) / kRedCols)), dim3(256), 0, s, P,
                     (int)S, n, out, accumulate);
  RQ_LAUNCH_CHECK("rq_col_sum");
  return 0;
}

#define L2R_VPL_SWITCH(CASE)                                                                      \
  switch (vpl) {                                                                                  \
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8) CASE(9) CASE(10) CASE(11) CASE(12) \
    CASE(13) CASE(14) CASE(15) CASE(16)                                                           \
  }

static int l2norm_recon_fwd_launch(const float* pre, const float* x, int64_t B, int64_t C, float* recon, float* norms,
                                   float gs, uint16_t* g_hi, uint16_t* g_lo, void* stream) {
  RQ_CHECK_ARG(B >= 0 && C > 0 && C % 4 == 0 && C <= 4096, "rq_l2norm_recon_fwd: need C %% 4 == 0, C <= 4096");
  if (B == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int vpl = (int)((C + 255) / 256);
  const dim3 g((unsigned)((B + 3) / 4));
  const bool grad = g_hi != nullptr;
#define L2R_CASE(V)                                                                                              \
  case V:                                                                                                        \
    if (grad)                                                                                                    \
      hipLaunchKernelGGL((l2norm_recon_fwd_kernel<V, true>), g, dim3(256), 0, s, pre, x, B, (int)C, recon, norms, \
                         gs, g_hi, g_lo);                                                                        \
    else                                                                                                         \
      hipLaunchKernelGGL((l2norm_recon_fwd_kernel<V, false>), g, dim3(256), 0, s, pre, x, B, (int)C, recon,      \
                         norms, gs, g_hi, g_lo);                                                                 \
    break;
  L2R_VPL_SWITCH(L2R_CASE)
#undef L2R_CASE
  RQ_LAUNCH_CHECK("rq_l2norm_recon_fwd");
  return 0;
}

int rq_l2norm_recon_fwd(const float* pre, const float* x, int64_t B, int64_t C, float* recon, float* norms,
                        void* stream) {
  RQ_CHECK_ARG(pre && x && recon && norms, "rq_l2norm_recon_fwd: null pointer");
  return l2norm_recon_fwd_launch(pre, x, B, C, recon, norms, 0.f, nullptr, nullptr, stream);
}

int rq_l2norm_recon_fwd_grad(const float* pre, const float* x, int64_t B, int64_t C, float* recon, float* norms,
                             float gs, uint16_t* g_hi, uint16_t* g_lo, void* stream) {
  RQ_CHECK_ARG(pre && x && recon && norms && g_hi && g_lo, "rq_l2norm_recon_fwd_grad: null pointer");
  RQ_CHECK_ARG(((uintptr_t)g_hi | (uintptr_t)g_lo) % 8 == 0, "rq_l2norm_recon_fwd_grad: planes must be 8-byte aligned");
  return l2norm_recon_fwd_launch(pre, x, B, C, recon, norms, gs, g_hi, g_lo, stream);
}

int rq_l2norm_recon_bwd_fix(const float* pre, const float* x, const float* norms, const float* g_recon,
                            int64_t g_stride, int64_t B, int64_t C, float gs, uint16_t* g_hi, uint16_t* g_lo,
                            void* stream) {
  RQ_CHECK_ARG(pre && x && norms && g_recon && g_hi && g_lo && (g_stride == 0 || g_stride == 1),
               "rq_l2norm_recon_bwd_fix: bad arguments");
  RQ_CHECK_ARG(B >= 0 && C > 0 && C % 4 == 0 && C <= 4096, "rq_l2norm_recon_bwd_fix: need C %% 4 == 0, C <= 4096");
  if (B == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int vpl = (int)((C + 255) / 256);
  const dim3 g((unsigned)std::min<int64_t>((B + 3) / 4, 2048));
  const uint32_t bits = __builtin_bit_cast(uint32_t, gs);
#define L2R_CASE(V)                                                                                                  \
  case V:                                                                                                            \
    hipLaunchKernelGGL((l2norm_recon_fix_kernel<V>), g, dim3(256), 0, s, pre, x, norms, g_recon, g_stride, B, (int)C, \
                       bits, g_hi, g_lo);                                                                            \
    break;
  L2R_VPL_SWITCH(L2R_CASE)
#undef L2R_CASE
  RQ_LAUNCH_CHECK("rq_l2norm_recon_bwd_fix");
  return 0;
}

static int l2norm_recon_bwd_launch(const float* pre, const float* x, const float* norms, const float* g_recon,
                                   int64_t B, int64_t C, float* g_pre, uint16_t* g_hi, uint16_t* g_lo, void* stream) {
  RQ_CHECK_ARG(B >= 0 && C > 0 && C % 4 == 0 && C <= 4096, "rq_l2norm_recon_bwd: need C %% 4 == 0, C <= 4096");
  if (B == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int vpl = (int)((C + 255) / 256);
  const dim3 g((unsigned)((B + 3) / 4));
  const bool sp = g_hi != nullptr;
#define L2R_LAUNCH(V, SP)                                                                                     \
  hipLaunchKernelGGL((l2norm_recon_bwd_kernel<V, SP>), g, dim3(256), 0, s, pre, x, norms, g_recon, B, (int)C, \
                     g_pre, g_hi, g_lo)
#define L2R_CASE1(V) case V: if (sp) L2R_LAUNCH(V, true); else L2R_LAUNCH(V, false); break;
  L2R_VPL_SWITCH(L2R_CASE1)
#undef L2R_CASE1
#undef L2R_LAUNCH
  RQ_LAUNCH_CHECK("rq_l2norm_recon_bwd");
  return 0;
}

int rq_l2norm_recon_bwd(const float* pre, const float* x, const float* norms, const float* g_recon, int64_t B,
                        int64_t C, float* g_pre, void* stream) {
  RQ_CHECK_ARG(pre && x && norms && g_recon && g_pre, "rq_l2norm_recon_bwd: null pointer");
  return l2norm_recon_bwd_launch(pre, x, norms, g_recon, B, C, g_pre, nullptr, nullptr, stream);
}

int rq_l2norm_recon_bwd_split(const float* pre, const float* x, const float* norms, const float* g_recon, int64_t B,
                              int64_t C, uint16_t* g_hi, uint16_t* g_lo, void* stream) {
  RQ_CHECK_ARG(pre && x && norms && g_recon && g_hi && g_lo, "rq_l2norm_recon_bwd_split: null pointer");
  RQ_CHECK_ARG(((uintptr_t)g_hi | (uintptr_t)g_lo) % 8 == 0, "rq_l2norm_recon_bwd_split: planes must be 8-byte aligned");
  return l2norm_recon_bwd_launch(pre, x, norms, g_recon, B, C, nullptr, g_hi, g_lo, stream);
}

int rq_row_norms(const float* x, int64_t rows, int64_t D, float* out, void* stream) {
  RQ_CHECK_ARG(rows >= 0 && D > 0 && D % 4 == 0, "rq_row_norms: need D %% 4 == 0");
  if (rows == 0) return 0;
  RQ_CHECK_ARG(x && out, "rq_row_norms: null pointer");
  int g = 1;
  while (g < 64 && 4 * g < D) g <<= 1;
  const dim3 grid((unsigned)((rows + 256 / g - 1) / (256 / g)));
  hipStream_t st = (hipStream_t)stream;
  switch (g) {
#define RN_CASE(G) case G: hipLaunchKernelGGL((row_norm_kernel<G>), grid, dim3(256), 0, st, x, rows, (int)D, out); break;
    RN_CASE(1) RN_CASE(2) RN_CASE(4) RN_CASE(8) RN_CASE(16) RN_CASE(32) RN_CASE(64)
#undef RN_CASE
  }
  RQ_LAUNCH_CHECK("rq_row_norms");
  return 0;
}

int rq_loss_means(const float* recon, const float* qloss, int64_t B, float* out, void* stream) {
  RQ_CHECK_ARG(B > 0 && recon && qloss && out, "rq_loss_means: bad arguments");
  RQ_CHECK_ARG(((uintptr_t)recon | (uintptr_t)qloss) % 16 == 0, "rq_loss_means: inputs must be 16-byte aligned");
  hipLaunchKernelGGL(loss_means_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, recon, qloss, B, out);
  RQ_LAUNCH_CHECK("rq_loss_means");
  return 0;
}

int rq_loss_means_bwd(const float* g, int64_t B, float* out_scalar, float* out_vec, void* stream) {
  RQ_CHECK_ARG(B > 0 && g && out_scalar && out_vec, "rq_loss_means_bwd: bad arguments");
  const float inv_b = 1.0f / (float)B;
  const int64_t blocks = std::min<int64_t>(256, (B + 255) / 256);
  hipLaunchKernelGGL(loss_means_bwd_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, g, B, inv_b,
                     out_scalar, out_vec);
  RQ_LAUNCH_CHECK("rq_loss_means_bwd");
  return 0;
}

size_t rq_rmsnorm_bwd_workspace(int64_t B, int64_t D) {
  if (B <= 0 || D <= 0) return 0;
  const int rows = rms_rows_per_blk(B);
  return (size_t)((B + rows - 1) / rows) * (size_t)D * sizeof(float);
}

#define RMS_SWITCH(VPL_EXPR, LAUNCH)                                                                      \
  switch (VPL_EXPR) {                                                                                     \
    case 1: LAUNCH(1) break; case 2: LAUNCH(2) break; case 3: LAUNCH(3) break; case 4: LAUNCH(4) break;  \
    case 5: LAUNCH(5) break; case 6: LAUNCH(6) break; case 7: LAUNCH(7) break; case 8: LAUNCH(8) break;  \
    case 9: LAUNCH(9) break; case 10: LAUNCH(10) break; case 11: LAUNCH(11) break;                       \
    case 12: LAUNCH(12) break; case 13: LAUNCH(13) break; case 14: LAUNCH(14) break;                     \
    case 15: LAUNCH(15) break; case 16: LAUNCH(16) break;                                                 \
  }

int rq_rmsnorm_dropout_fwd(const float* x, const float* w, int64_t B, int64_t D, float eps, float p, uint64_t seed,
                           float* y, float* rstd, void* stream) {
  RQ_CHECK_ARG(B >= 0 && D > 0 && D % 4 == 0 && D <= 4096, "rq_rmsnorm_fwd: need D %% 4 == 0, D <= 4096");
  if (B == 0) return 0;
  RQ_CHECK_ARG(x && w && y && rstd, "rq_rmsnorm_fwd: null pointer");
  uint32_t thr;
  float dscale;
  dropout_params(p, &thr, &dscale);
  dim3 g((unsigned)((B + 3) / 4));
  hipStream_t s = (hipStream_t)stream;
#define RMS_F(V) hipLaunchKernelGGL((rmsnorm_fwd_kernel<V>), g, dim3(256), 0, s, x, w, B, (int)D, eps, thr, dscale, seed, y, rstd);
  RMS_SWITCH((int)((D + 255) / 256), RMS_F)
#undef RMS_F
  RQ_LAUNCH_CHECK("rq_rmsnorm_fwd");
  return 0;
}

int rq_rmsnorm_fwd(const float* x, const float* w, int64_t B, int64_t D, float eps, float* y, float* rstd,
                   void* stream) {
  return rq_rmsnorm_dropout_fwd(x, w, B, D, eps, 0.f, 0, y, rstd, stream);
}

int rq_rmsnorm_dropout_bwd(const float* x, const float* w, const float* rstd, const float* gy, const float* gres,
                           int64_t B, int64_t D, float p, uint64_t seed, float* gx, float* gw, int accumulate_gw,
                           int defer, int* parts, void* workspace, size_t ws_bytes, void* stream) {
  if (parts) *parts = 0;
  RQ_CHECK_ARG(B >= 0 && D > 0 && D % 4 == 0 && D <= 4096, "rq_rmsnorm_bwd: need D %% 4 == 0, D <= 4096");
  RQ_CHECK_ARG(gw && (B == 0 || (x && w && rstd && gy && gx)), "rq_rmsnorm_bwd: null pointer");
  hipStream_t s = (hipStream_t)stream;
  if (B == 0) {
    if (!accumulate_gw) RQ_HIP(zero_async(gw, (size_t)D * sizeof(float), s));
    return 0;
  }
  RQ_CHECK_ARG(workspace && ws_bytes >= rq_rmsnorm_bwd_workspace(B, D), "rq_rmsnorm_bwd: workspace too small");
  uint32_t thr;
  float dscale;
  dropout_params(p, &thr, &dscale);
  float* part = static_cast<float*>(workspace);
  const int rows = rms_rows_per_blk(B);
  const int nblk = (int)((B + rows - 1) / rows);
#define RMS_B(V) hipLaunchKernelGGL((rmsnorm_bwd_kernel<V>), dim3((unsigned)nblk), dim3(256), 0, s, x, w, rstd, gy, B, (int)D, thr, dscale, seed, gres, gx, part, rows);
  RMS_SWITCH((int)((D + 255) / 256), RMS_B)
#undef RMS_B
  RQ_LAUNCH_CHECK("rq_rmsnorm_bwd");
  if (defer && parts) {   // gw partials [nblk][D] left in the workspace: rq_reduce_partials (layout 1) sums them
    *parts = nblk;
    return 0;
  }
  hipLaunchKernelGGL(rms_reduce_kernel, dim3((unsigned)((D / 4 + kRedCols - 1) / kRedCols)), dim3(256), 0, s, part, nblk, D, gw,
                     accumulate_gw);
  RQ_LAUNCH_CHECK("rq_rmsnorm_bwd(reduce)");
  return 0;
}

int rq_rmsnorm2_dropout_fwd(const float* x, const float* w1, const float* w2, int64_t B, int64_t D, float eps, float p1,
                            uint64_t seed1, float p2, uint64_t seed2, float* y1, float* y2, float* rstd, void* stream) {
  RQ_CHECK_ARG(B >= 0 && D > 0 && D % 4 == 0 && D <= 4096, "rq_rmsnorm2_fwd: need D %% 4 == 0, D <= 4096");
  if (B == 0) return 0;
  RQ_CHECK_ARG(x && w1 && w2 && y1 && y2 && rstd, "rq_rmsnorm2_fwd: null pointer");
  uint32_t thr1, thr2;
  float ds1, ds2;
  dropout_params(p1, &thr1, &ds1);
  dropout_params(p2, &thr2, &ds2);
  dim3 g((unsigned)((B + 3) / 4));
  hipStream_t s = (hipStream_t)stream;
#define RMS_F2(V) hipLaunchKernelGGL((rmsnorm2_fwd_kernel<V>), g, dim3(256), 0, s, x, w1, w2, B, (int)D, eps, thr1, ds1, seed1, thr2, ds2, seed2, y1, y2, rstd);
  RMS_SWITCH((int)((D + 255) / 256), RMS_F2)
#undef RMS_F2
  RQ_LAUNCH_CHECK("rq_rmsnorm2_fwd");
  return 0;
}

int rq_rmsnorm2_dropout_bwd(const float* x, const float* w1, const float* w2, const float* rstd, const float* gy1,
                            const float* gy2, const float* gres, int64_t B, int64_t D, float p1, uint64_t seed1, float p2,
                            uint64_t seed2, float* gx, float* gw1, float* gw2, int accumulate_gw, int defer, int* parts,
                            void* workspace, size_t ws_bytes, void* stream) {
  if (parts) *parts = 0;
  RQ_CHECK_ARG(B >= 0 && D > 0 && D % 4 == 0 && D <= 4096, "rq_rmsnorm2_bwd: need D %% 4 == 0, D <= 4096");
  RQ_CHECK_ARG(gw1 && gw2 && (B == 0 || (x && w1 && w2 && rstd && gy1 && gy2 && gx)), "rq_rmsnorm2_bwd: null pointer");
  hipStream_t s = (hipStream_t)stream;
  if (B == 0) {
    if (!accumulate_gw) {
      RQ_HIP(zero_async(gw1, (size_t)D * sizeof(float), s));
      RQ_HIP(zero_async(gw2, (size_t)D * sizeof(float), s));
    }
    return 0;
  }
  const size_t half = rq_rmsnorm_bwd_workspace(B, D);
  RQ_CHECK_ARG(workspace && ws_bytes >= 2 * half, "rq_rmsnorm2_bwd: workspace too small (2 x rq_rmsnorm_bwd_workspace)");
  uint32_t thr1, thr2;
  float ds1, ds2;
  dropout_params(p1, &thr1, &ds1);
  dropout_params(p2, &thr2, &ds2);
  float* part1 = static_cast<float*>(workspace);
  float* part2 = part1 + half / sizeof(float);
  const int rows = rms_rows_per_blk(B);
  const int nblk = (int)((B + rows - 1) / rows);
#define RMS_B2(V) hipLaunchKernelGGL((rmsnorm2_bwd_kernel<V>), dim3((unsigned)nblk), dim3(256), 0, s, x, w1, w2, rstd, gy1, gy2, B, (int)D, thr1, ds1, seed1, thr2, ds2, seed2, gres, gx, part1, part2, rows);
  RMS_SWITCH((int)((D + 255) / 256), RMS_B2)
#undef RMS_B2
  RQ_LAUNCH_CHECK("rq_rmsnorm2_bwd");
  if (defer && parts) {   // both weights' partials [nblk][D] at workspace and workspace + half: rq_reduce_partials
    *parts = nblk;
    return 0;
  }
  const dim3 rg((unsigned)((D / 4 + kRedCols - 1) / kRedCols));
  hipLaunchKernelGGL(rms_reduce_kernel, rg, dim3(256), 0, s, part1, nblk, D, gw1, accumulate_gw);
  hipLaunchKernelGGL(rms_reduce_kernel, rg, dim3(256), 0, s, part2, nblk, D, gw2, accumulate_gw);
  RQ_LAUNCH_CHECK("rq_rmsnorm2_bwd(reduce)");
  return 0;
}

int rq_rmsnorm_bwd(const float* x, const float* w, const float* rstd, const float* gy, int64_t B, int64_t D,
                   float* gx, float* gw, void* workspace, size_t ws_bytes, void* stream) {
  return rq_rmsnorm_dropout_bwd(x, w, rstd, gy, nullptr, B, D, 0.f, 0, gx, gw, 0, 0, nullptr, workspace, ws_bytes,
                                stream);
}



int rq_gumbel_softmax_fwd(const float* x, int64_t B, int64_t D, const float* codebook, int64_t K, const float* noise,
                          float temperature, float* weights, float* emb, int64_t* ids, void* stream) {
  RQ_CHECK_ARG(B >= 0 && D > 0 && D <= rqhip::kGsMaxD && K > 0 && K <= rqhip::kGsMaxK && temperature > 0.f,
               "rq_gumbel_softmax_fwd: need 0 < D <= %d, 0 < K <= %d, temperature > 0", rqhip::kGsMaxD,
               rqhip::kGsMaxK);
  if (B == 0) return 0;
  RQ_CHECK_ARG(x && codebook && noise && weights && emb && ids, "rq_gumbel_softmax_fwd: null pointer");
  const dim3 g((unsigned)((B + rqhip::kGsWaves - 1) / rqhip::kGsWaves));
  hipLaunchKernelGGL(rqhip::gumbel_softmax_fwd_kernel, g, dim3(64 * rqhip::kGsWaves), 0, (hipStream_t)stream, x, B,
                     (int)D, codebook, (int)K, noise, 1.f / temperature, weights, emb, ids);
  RQ_LAUNCH_CHECK("rq_gumbel_softmax_fwd");
  return 0;
}

int rq_gumbel_softmax_bwd(const float* x, const float* codebook, const float* weights, const float* g_emb, int64_t B,
                          int64_t D, int64_t K, float temperature, float* dx, float* ddist, void* stream) {
  RQ_CHECK_ARG(B >= 0 && D > 0 && D <= rqhip::kGsMaxD && K > 0 && K <= rqhip::kGsMaxK && temperature > 0.f,
               "rq_gumbel_softmax_bwd: need 0 < D <= %d, 0 < K <= %d, temperature > 0", rqhip::kGsMaxD,
               rqhip::kGsMaxK);
  if (B == 0) return 0;
  RQ_CHECK_ARG(x && codebook && weights && g_emb && dx && ddist, "rq_gumbel_softmax_bwd: null pointer");
  const dim3 g((unsigned)((B + rqhip::kGsWaves - 1) / rqhip::kGsWaves));
  hipLaunchKernelGGL(rqhip::gumbel_softmax_bwd_kernel, g, dim3(64 * rqhip::kGsWaves), 0, (hipStream_t)stream, x,
                     codebook, weights, g_emb, B, (int)D, (int)K, 1.f / temperature, dx, ddist);
  RQ_LAUNCH_CHECK("rq_gumbel_softmax_bwd");
  return 0;
}

}  // extern "C"

int rqhip::seed_epoch_addr_rowwise(void** out) { return (int)hipGetSymbolAddress(out, HIP_SYMBOL(rqhip::rq_seed_epoch)); }
