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
#include "common.h"

namespace rqhip {

template <int VPL>   // float4 vectors per lane (C = 256 * VPL)
__global__ void __launch_bounds__(256) l2norm_recon_fwd_kernel(const float* __restrict__ pre, const float* __restrict__ x,
                                                                int64_t B, int C, float* __restrict__ recon,
                                                                float* __restrict__ nrm) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= B) return;
  const float* p = pre + r * C;
  const float* q = x + r * C;
  float4 pv[VPL], xv[VPL];
  float s = 0.f;
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    const int c = (v * 64 + lane) * 4;
    const bool ok = c < C;
    pv[v] = ok ? *reinterpret_cast<const float4*>(p + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    xv[v] = ok ? *reinterpret_cast<const float4*>(q + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    s += pv[v].x * pv[v].x + pv[v].y * pv[v].y + pv[v].z * pv[v].z + pv[v].w * pv[v].w;
  }
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
}

template <int VPL>
__global__ void __launch_bounds__(256) l2norm_recon_bwd_kernel(const float* __restrict__ pre, const float* __restrict__ x,
                                                                const float* __restrict__ nrm,
                                                                const float* __restrict__ g_recon, int64_t B, int C,
                                                                float* __restrict__ g_pre) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= B) return;
  const float* p = pre + r * C;
  const float* q = x + r * C;
  const float raw = nrm[r];
  const float n = fmaxf(raw, 1e-12f);
  const float g2 = 2.f * g_recon[r];
  float4 yv[VPL], gy[VPL];
  float dot = 0.f;
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    const int c = (v * 64 + lane) * 4;
    const bool ok = c < C;
    const float4 a = ok ? *reinterpret_cast<const float4*>(p + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 b = ok ? *reinterpret_cast<const float4*>(q + c) : make_float4(0.f, 0.f, 0.f, 0.f);
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
    *reinterpret_cast<float4*>(g_pre + r * C + c) = o;
  }
}

}  // namespace rqhip

using namespace rqhip;

extern "C" {

int rq_l2norm_recon_fwd(const float* pre, const float* x, int64_t B, int64_t C, float* recon, float* norms,
                        void* stream) {
  RQ_CHECK_ARG(pre && x && recon && norms, "rq_l2norm_recon_fwd: null pointer");
  RQ_CHECK_ARG(B >= 0 && C > 0 && C % 4 == 0 && C <= 4096, "rq_l2norm_recon_fwd: need C %% 4 == 0, C <= 4096");
  if (B == 0) return 0;
  dim3 g((unsigned)((B + 3) / 4));
  hipStream_t s = (hipStream_t)stream;
  const int vpl = (int)((C + 255) / 256);
  switch (vpl) {
#define L2R_CASE(V) case V: hipLaunchKernelGGL((l2norm_recon_fwd_kernel<V>), g, dim3(256), 0, s, pre, x, B, (int)C, recon, norms); break;
    L2R_CASE(1) L2R_CASE(2) L2R_CASE(3) L2R_CASE(4) L2R_CASE(5) L2R_CASE(6) L2R_CASE(7) L2R_CASE(8)
    L2R_CASE(9) L2R_CASE(10) L2R_CASE(11) L2R_CASE(12) L2R_CASE(13) L2R_CASE(14) L2R_CASE(15) L2R_CASE(16)
#undef L2R_CASE
  }
  RQ_LAUNCH_CHECK("rq_l2norm_recon_fwd");
  return 0;
}

int rq_l2norm_recon_bwd(const float* pre, const float* x, const float* norms, const float* g_recon, int64_t B,
                        int64_t C, float* g_pre, void* stream) {
  RQ_CHECK_ARG(pre && x && norms && g_recon && g_pre, "rq_l2norm_recon_bwd: null pointer");
  RQ_CHECK_ARG(B >= 0 && C > 0 && C % 4 == 0 && C <= 4096, "rq_l2norm_recon_bwd: need C %% 4 == 0, C <= 4096");
  if (B == 0) return 0;
  dim3 g((unsigned)((B + 3) / 4));
  hipStream_t s = (hipStream_t)stream;
  const int vpl = (int)((C + 255) / 256);
  switch (vpl) {
#define L2R_CASE(V) case V: hipLaunchKernelGGL((l2norm_recon_bwd_kernel<V>), g, dim3(256), 0, s, pre, x, norms, g_recon, B, (int)C, g_pre); break;
    L2R_CASE(1) L2R_CASE(2) L2R_CASE(3) L2R_CASE(4) L2R_CASE(5) L2R_CASE(6) L2R_CASE(7) L2R_CASE(8)
    L2R_CASE(9) L2R_CASE(10) L2R_CASE(11) L2R_CASE(12) L2R_CASE(13) L2R_CASE(14) L2R_CASE(15) L2R_CASE(16)
#undef L2R_CASE
  }
  RQ_LAUNCH_CHECK("rq_l2norm_recon_bwd");
  return 0;
}

}  // extern "C"
