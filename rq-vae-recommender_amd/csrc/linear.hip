// Weight gradient of a Linear layer over a large batch: dW = g^T x, db = sum_b g  (fp32 MFMA).
//
// Reference: every nn.Linear in modules/encoder.py:7-36 (the RQ-VAE encoder / decoder MLPs) and
// modules/transformer/* — torch autograd computes grad_weight = grad_out^T @ input. At the RQ-VAE
// batch (B = 65,536 rows) that product has a tiny output (O x I <= 768 x 512) and a huge
// reduction axis, which the library GEMM tiles poorly (5-29 TFLOP/s measured on gfx950, where
// forward / data-grad GEMMs of the same layers reach 100-128). Here the reduction axis is split
// across workgroups (split-K) so a launch covers every CU:
//
//   pass 1  wgrad_partial_kernel: workgroup (s, tile) computes the 128 x 128 output tile over
//           rows [s*chunk, (s+1)*chunk) on v_mfma_f32_32x32x2_f32, operands staged through a
//           double-buffered LDS ring (rows stay in their HBM layout: b-major, coalesced float4
//           loads; one conflict-free ds_read_b64 per operand feeds two MFMA tiles).
//           Tile-column-0 workgroups also sum g over their rows for db. Partials go to a
//           workspace [S][O][I] (+ [S][O]).
//   pass 2  wgrad_reduce_kernel: fixed-order sum over s — deterministic, no atomics.
//
// Workgroups that share a row chunk are placed on the same XCD (blockIdx % 8 selects the XCD)
// so the tiles re-reading the same g / x rows hit one L2.
#include "common.h"

namespace rqhip {

constexpr int kWT = 128;    // output tile (o and i)
constexpr int kWBK = 32;    // rows per LDS stage
constexpr int kWLD = 128;   // LDS row stride in floats (float2 operand reads: 32 lanes x 8 B = all 64 banks)

// Operand mapping: a wave owns a 64 (o) x 64 (i) block as 2 x 2 MFMA tiles, interleaved so that
// one ds_read_b64 feeds both tiles of a pair: tile p's MFMA row m is o = 2m + p (and tile q's
// column n is i = 2n + q). The MFMA k index is the lane half (rows b = 2kp, 2kp+1 of the stage).
__global__ void __launch_bounds__(256, 2)
wgrad_partial_kernel(const float* __restrict__ g, int64_t ldg, const float* __restrict__ x, int64_t ldx, int64_t Bn,
                     int O, int I, int tiles_i, int tiles, int S, int64_t chunk, int per, float* __restrict__ P,
                     float* __restrict__ Pb) {
  __shared__ __attribute__((aligned(16))) float As[2][kWBK][kWLD];
  __shared__ __attribute__((aligned(16))) float Bs[2][kWBK][kWLD];
  const int bid = blockIdx.x;
  const int lw = (bid & 7) * per + (bid >> 3);   // XCD-major order: consecutive lw share an XCD
  if (lw >= tiles * S) return;
  const int s = lw / tiles, t = lw % tiles;
  const int o0 = (t / tiles_i) * kWT, i0 = (t % tiles_i) * kWT;
  const int64_t b_lo = (int64_t)s * chunk;
  const int64_t b_hi = b_lo + chunk < Bn ? b_lo + chunk : Bn;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, h = lane >> 5, c32 = lane & 31;
  const int wo = wave >> 1, wi = wave & 1;
  const bool do_bias = Pb != nullptr && (t % tiles_i) == 0 && wi == 0;

  constexpr int kF = kWBK * kWT / 4 / 256;   // float4 per thread per operand per stage
  float4 ra[kF], rb[kF];
  auto load = [&](int64_t b0) {
#pragma unroll
    for (int j = 0; j < kF; ++j) {
      const int f = tid + 256 * j, r = f >> 5, c = (f & 31) * 4;
      const int64_t b = b0 + r;
      const bool okb = b < b_hi;
      ra[j] = (okb && o0 + c < O) ? *reinterpret_cast<const float4*>(g + b * ldg + o0 + c) : make_float4(0.f, 0.f, 0.f, 0.f);
      rb[j] = (okb && i0 + c < I) ? *reinterpret_cast<const float4*>(x + b * ldx + i0 + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto stash = [&](int buf) {
#pragma unroll
    for (int j = 0; j < kF; ++j) {
      const int f = tid + 256 * j, r = f >> 5, c = (f & 31) * 4;
      *reinterpret_cast<float4*>(&As[buf][r][c]) = ra[j];
      *reinterpret_cast<float4*>(&Bs[buf][r][c]) = rb[j];
    }
  };

  floatx16 acc[2][2];
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[p][q][r] = 0.f;
  float bsum = 0.f;

  const int nst = (int)((b_hi - b_lo + kWBK - 1) / kWBK);
  load(b_lo);
  stash(0);
  __syncthreads();
  for (int st = 0; st < nst; ++st) {
    const int buf = st & 1;
    if (st + 1 < nst) load(b_lo + (int64_t)(st + 1) * kWBK);   // in flight during the MFMAs
#pragma unroll
    for (int kp = 0; kp < kWBK / 2; ++kp) {
      const int k = 2 * kp + h;   // A[o][k] = g[b][o], B[k][i] = x[b][i]
      const float2 a = *reinterpret_cast<const float2*>(&As[buf][k][wo * 64 + 2 * c32]);
      const float2 v = *reinterpret_cast<const float2*>(&Bs[buf][k][wi * 64 + 2 * c32]);
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, v.x, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, v.y, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, v.x, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, v.y, acc[1][1], 0, 0, 0);
    }
    if (do_bias) {
#pragma unroll
      for (int k = 0; k < kWBK; ++k) bsum += As[buf][k][wo * 64 + lane];
    }
    if (st + 1 < nst) stash(buf ^ 1);
    __syncthreads();
  }

  // C/D map: MFMA row m = (r&3) + 8(r>>2) + 4h, column n = lane&31; o = 2m + p, i = 2n + q.
  float* Ps = P + (int64_t)s * O * I;
  const int i = i0 + wi * 64 + 2 * c32;
  if (i < I) {
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int o = o0 + wo * 64 + 2 * ((r & 3) + 8 * (r >> 2) + 4 * h) + p;
        if (o < O) *reinterpret_cast<float2*>(Ps + (int64_t)o * I + i) = make_float2(acc[p][0][r], acc[p][1][r]);
      }
  }
  if (do_bias) {
    const int o = o0 + wo * 64 + lane;
    if (o < O) Pb[(int64_t)s * O + o] = bsum;
  }
}

// out[j] = sum_{s=0}^{S-1} P[s*n + j] in a fixed order (n % 4 == 0): workgroup = 64 float4
// columns x 4 waves; wave w sums s = w, w+4, ... (4 independent loads in flight per step), then
// the four wave partials are added in wave order through LDS. Deterministic, no atomics.
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* __restrict__ P, int S, int64_t n,
                                                           float* __restrict__ out) {
  __shared__ float4 part[4][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t j = ((int64_t)blockIdx.x * 64 + lane) * 4;
  const bool ok = j < n;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (ok) {
    int s = wave;
    for (; s + 12 < S; s += 16) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const float4*>(P + (int64_t)(s + 4 * u) * n + j);
#pragma unroll
      for (int u = 0; u < 4; ++u) { a.x += v[u].x; a.y += v[u].y; a.z += v[u].z; a.w += v[u].w; }
    }
    for (; s < S; s += 4) {
      const float4 v = *reinterpret_cast<const float4*>(P + (int64_t)s * n + j);
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
  }
  part[wave][lane] = a;
  __syncthreads();
  if (wave == 0 && ok) {
    float4 r = part[0][lane];
#pragma unroll
    for (int w = 1; w < 4; ++w) {
      const float4 v = part[w][lane];
      r.x += v.x; r.y += v.y; r.z += v.z; r.w += v.w;
    }
    *reinterpret_cast<float4*>(out + j) = r;
  }
}

struct WgradPlan {
  int tiles_i, tiles, S, per;
  int64_t chunk;
};

static int resident_slots() {   // 2 workgroups per CU (launch bounds), queried once
  static int slots = 0;
  if (slots == 0) {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || cus <= 0)
      cus = 256;
    slots = 2 * cus;
  }
  return slots;
}

static WgradPlan wgrad_plan(int64_t Bn, int64_t O, int64_t I) {
  WgradPlan p;
  p.tiles_i = (int)((I + kWT - 1) / kWT);
  p.tiles = (int)((O + kWT - 1) / kWT) * p.tiles_i;
  // one full round of resident workgroups: a partial second round would double the time
  int64_t S = resident_slots() / p.tiles;
  const int64_t max_s = (Bn + 4 * kWBK - 1) / (4 * kWBK);   // at least 4 stages per workgroup
  if (S > max_s) S = max_s;
  if (S < 1) S = 1;
  int64_t chunk = (Bn + S - 1) / S;
  chunk = (chunk + kWBK - 1) / kWBK * kWBK;
  if (chunk < kWBK) chunk = kWBK;
  p.chunk = chunk;
  p.S = (int)((Bn + chunk - 1) / chunk);
  if (p.S < 1) p.S = 1;
  p.per = (p.tiles * p.S + 7) / 8;
  return p;
}

}  // namespace rqhip

using namespace rqhip;

extern "C" {

size_t rq_linear_wgrad_workspace(int64_t Bn, int64_t O, int64_t I) {
  if (Bn <= 0 || O <= 0 || I <= 0) return 0;
  const WgradPlan p = wgrad_plan(Bn, O, I);
  return (size_t)p.S * (size_t)(O * I + O) * sizeof(float);
}

int rq_linear_wgrad(const float* g, int64_t ldg, const float* x, int64_t ldx, int64_t Bn, int64_t O, int64_t I,
                    float* dW, float* db, void* workspace, size_t ws_bytes, void* stream) {
  RQ_CHECK_ARG(((g && x) || Bn == 0) && dW && Bn >= 0 && O > 0 && I > 0 && O < (1 << 30) && I < (1 << 30),
               "rq_linear_wgrad: bad arguments");
  RQ_CHECK_ARG(O % 4 == 0 && I % 4 == 0 && ldg % 4 == 0 && ldx % 4 == 0 && ldg >= O && ldx >= I,
               "rq_linear_wgrad: O, I and leading dims must be multiples of 4 (float4 rows)");
  RQ_CHECK_ARG(((uintptr_t)g | (uintptr_t)x | (uintptr_t)dW | (uintptr_t)db) % 16 == 0,
               "rq_linear_wgrad: pointers must be 16-byte aligned");
  hipStream_t s = (hipStream_t)stream;
  if (Bn == 0) {
    RQ_HIP(hipMemsetAsync(dW, 0, (size_t)(O * I) * sizeof(float), s));
    if (db) RQ_HIP(hipMemsetAsync(db, 0, (size_t)O * sizeof(float), s));
    return 0;
  }
  const WgradPlan p = wgrad_plan(Bn, O, I);
  const size_t need = (size_t)p.S * (size_t)(O * I + O) * sizeof(float);
  RQ_CHECK_ARG(workspace != nullptr && ws_bytes >= need, "rq_linear_wgrad: workspace %zu < %zu bytes", ws_bytes, need);
  float* P = static_cast<float*>(workspace);
  float* Pb = db ? P + (int64_t)p.S * O * I : nullptr;
  hipLaunchKernelGGL(wgrad_partial_kernel, dim3((unsigned)(p.per * 8)), dim3(256), 0, s, g, ldg, x, ldx, Bn, (int)O,
                     (int)I, p.tiles_i, p.tiles, p.S, p.chunk, p.per, P, Pb);
  RQ_LAUNCH_CHECK("wgrad_partial_kernel");
  const int64_t n = O * I;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((n / 4 + 63) / 64)), dim3(256), 0, s, P, p.S, n, dW);
  RQ_LAUNCH_CHECK("wgrad_reduce_kernel");
  if (db) {
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((O / 4 + 63) / 64)), dim3(256), 0, s, Pb, p.S, O, db);
    RQ_LAUNCH_CHECK("wgrad_reduce_kernel(bias)");
  }
  return 0;
}

}  // extern "C"
