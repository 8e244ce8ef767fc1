// Residual quantization for the RQ-VAE hot path — fused L-level forward, its VJP, and the
// deterministic codebook-gradient reduction. gfx950 / wave64 / fp32 MFMA.
//
// Reference semantics (AdamLTy/RQ-VAE-Recommender):
//   modules/quantize.py:99-156  Quantize.forward (L2 dist :108-112, argmin :121,
//                               STE :130-132, rotation trick :133-142 with :34-45, eval :148-150)
//   modules/loss.py:34-42       QuantizeLoss (per-row, beta = commitment_weight)
//   modules/rqvae.py:114-138    get_semantic_ids: res_{l+1} = res_l - emb_out_l over L levels
//
// Layout in HBM (row-major, fp32):
//   x          (B, D)      encoder output = level-0 residual
//   codebooks  (L, K, D)   one nn.Embedding weight per level (out_proj = Identity)
//   cb_sqnorm  (L, K)      |c|^2 per codeword (rq_codebook_sqnorm)
//   ids        (B, L)      int64 semantic ids
//   emb_out    (L, B, D)   per-level quantized output (returned to Python as a (B,D,L) view)
//   residuals  (L, B, D)   res_l fed to level l (residuals[0] = x)
//   qloss      (B,)        sum over levels of the per-row VQ loss
//   emb_sum    (B, D)      sum_l emb_out_l (decoder input), optional
//
// Forward kernel: one workgroup = 4 waves = TB=128 items. Per level: the distance GEMM
// C_l (K x D) . X^T (D x 128) runs on v_mfma_f32_32x32x2_f32 (exact fp32 fma chain, no xf32
// on gfx950) with codewords on the MFMA row axis and items on the lane axis, so each lane
// owns one item's distances and the argmin is a register scan (+1 lane swap) — no cross-lane
// reduction per codeword. Codebook chunks (NB=128 codewords x BK) and item chunks are staged
// through LDS with conflict-free padded rows read by ds_read_b128. The row epilogue
// (gather, rotation trick, VQ loss, residual update) runs LPI lanes per item, all levels
// chained inside the launch so the residual never round-trips through a separate kernel.
#include "common.h"

#include <algorithm>
#include <math.h>

namespace rqhip {

constexpr int kTB = 128;   // items per workgroup (4 waves x 32)
constexpr int kNB = 128;   // codewords per LDS chunk (4 MFMA row tiles)

enum Mode { kEval = 0, kGumbel = 1, kSte = 2, kRotation = 3 };

// ---------------------------------------------------------------------------------------
// |c|^2 per codeword: one wave per row.
__global__ void __launch_bounds__(256) rq_sqnorm_kernel(const float* __restrict__ rows, int64_t n, int D,
                                                        float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= n) return;
  const float* p = rows + r * D;
  float s = 0.f;
  for (int d = lane; d < D; d += 64) s += p[d] * p[d];
  s = group_sum<64>(s);
  if (lane == 0) out[r] = s;
}

// Rotation-trick constants for one item held by an aligned group of LPI lanes (EPL elems each).
template <int LPI, int EPL>
struct RowRot {
  float u[EPL], q[EPL], w[EPL];
  float lam;
  __device__ __forceinline__ void build(const float (&x)[EPL], const float (&e)[EPL], float xn, float en) {
    // u = x/(|x|+1e-8), q = e/(|e|+1e-8), w = normalize(u+q, eps 1e-6)   (quantize.py:34-39,135-138)
    const float xd = xn + 1e-8f, ed = en + 1e-8f;
    const float rx = 1.0f / xd, re = 1.0f / ed;
    float mnx = INFINITY, mxx = 0.f, mne = INFINITY, mxe = 0.f;
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
      mnx = fminf(mnx, fabsf(x[k])); mxx = fmaxf(mxx, fabsf(x[k]));
      mne = fminf(mne, fabsf(e[k])); mxe = fmaxf(mxe, fabsf(e[k]));
    }
    const bool fast = div_rn_ok(mnx, mxx, xd) && div_rn_ok(mne, mxe, ed);
    float s2 = 0.f, mns = INFINITY, mxs = 0.f;
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
      u[k] = fast ? div_rn(x[k], xd, rx) : x[k] / xd;
      q[k] = fast ? div_rn(e[k], ed, re) : e[k] / ed;
      const float s = u[k] + q[k];
      w[k] = s;
      s2 += s * s;
      mns = fminf(mns, fabsf(s)); mxs = fmaxf(mxs, fabsf(s));
    }
    s2 = group_sum<LPI>(s2);
    const float sn = fmaxf(sqrtf(s2), 1e-6f), rs = 1.0f / sn;
    const bool fast_w = div_rn_ok(mns, mxs, sn);
#pragma unroll
    for (int k = 0; k < EPL; ++k) w[k] = fast_w ? div_rn(w[k], sn, rs) : w[k] / sn;
    lam = en / (xn + 1e-6f);   // (|emb| / (|x| + 1e-6)).detach()   (quantize.py:140-142)
  }
};

// ---------------------------------------------------------------------------------------
// Fused L-level forward.
template <int BK, int LPI, int EPL>
__global__ void __launch_bounds__(256, 2)
rq_fwd_kernel(const float* __restrict__ x, int B, int D, const float* __restrict__ cbs,
              const float* __restrict__ csq, int K, int L, int mode, float beta,
              int64_t* __restrict__ ids, float* __restrict__ emb_out, float* __restrict__ res,
              float* __restrict__ qloss, float* __restrict__ emb_sum) {
  constexpr int LDA = BK + 4;             // padded LDS row (16-B aligned, ds_read_b128 conflict-free)
  constexpr int G = 64 / LPI;             // items processed concurrently per wave in the epilogue
  __shared__ __attribute__((aligned(16))) float smem[(kNB + kTB) * LDA + kNB + 3 * kTB];
  float* A_s = smem;                       // codeword chunk  [kNB][LDA]
  float* X_s = A_s + kNB * LDA;            // item chunk      [kTB][LDA]
  float* cs_s = X_s + kTB * LDA;           // |c|^2 chunk     [kNB]
  float* xsq_s = cs_s + kNB;               // |res_l|^2       [kTB]
  float* ql_s = xsq_s + kTB;               // running qloss   [kTB]
  int* id_s = reinterpret_cast<int*>(ql_s + kTB);  //        [kTB]

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, h = lane >> 5;
  const int row0 = blockIdx.x * kTB;
  const int64_t BD = (int64_t)B * D;
  const int sub = lane % LPI, grp = lane / LPI;

  // Prologue: residuals[0] = x, |x|^2, qloss accumulator.
  for (int it = 0; it < 32 / G; ++it) {
    const int jl = wave * 32 + it * G + grp;
    const int b = row0 + jl;
    const bool valid = b < B;
    const int64_t o = (int64_t)(valid ? b : B - 1) * D + sub * EPL;
    float xv[EPL];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < EPL; k += 4) {
      const float4 v = *reinterpret_cast<const float4*>(x + o + k);
      xv[k] = v.x; xv[k + 1] = v.y; xv[k + 2] = v.z; xv[k + 3] = v.w;
    }
#pragma unroll
    for (int k = 0; k < EPL; ++k) s += xv[k] * xv[k];
    s = group_sum<LPI>(s);
    if (valid) {
#pragma unroll
      for (int k = 0; k < EPL; k += 4)
        *reinterpret_cast<float4*>(res + o + k) = make_float4(xv[k], xv[k + 1], xv[k + 2], xv[k + 3]);
    }
    if (sub == 0) { xsq_s[jl] = s; ql_s[jl] = 0.f; }
  }

  for (int l = 0; l < L; ++l) {
    const float* src = res + (int64_t)l * BD;
    const float* cb = cbs + (int64_t)l * K * D;
    const float* cq = csq + (int64_t)l * K;
    float best_d = INFINITY;
    int best_i = 0;
    __syncthreads();   // residual rows of level l written by every wave of the block
    const float xs = xsq_s[wave * 32 + (lane & 31)];

    for (int n0 = 0; n0 < K; n0 += kNB) {
      floatx16 acc[4];
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

      for (int k0 = 0; k0 < D; k0 += BK) {
        __syncthreads();   // previous chunk fully consumed
        constexpr int F4 = BK / 4;   // float4 per staged row
        for (int f = tid; f < kNB * F4; f += 256) {
          const int r = f / F4, c = (f % F4) * 4;
          float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
          if (n0 + r < K) v = *reinterpret_cast<const float4*>(cb + (int64_t)(n0 + r) * D + k0 + c);
          *reinterpret_cast<float4*>(A_s + r * LDA + c) = v;
        }
        for (int f = tid; f < kTB * F4; f += 256) {
          const int r = f / F4, c = (f % F4) * 4;
          float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
          if (row0 + r < B) v = *reinterpret_cast<const float4*>(src + (int64_t)(row0 + r) * D + k0 + c);
          *reinterpret_cast<float4*>(X_s + r * LDA + c) = v;
        }
        if (k0 == 0 && tid < kNB) cs_s[tid] = (n0 + tid < K) ? cq[n0 + tid] : 0.f;
        __syncthreads();

        // Lane half h supplies logical k=h of every MFMA; physical k = h*BK/2 + step, the
        // same permutation for both operands, so sum_k A[i][k] B[k][j] is unchanged.
        const float* bp = X_s + (wave * 32 + (lane & 31)) * LDA + h * (BK / 2);
        const float* ap = A_s + (lane & 31) * LDA + h * (BK / 2);
#pragma unroll
        for (int s4 = 0; s4 < BK / 2; s4 += 4) {
          const float4 bv = *reinterpret_cast<const float4*>(bp + s4);
          float4 av[4];
#pragma unroll
          for (int t = 0; t < 4; ++t) av[t] = *reinterpret_cast<const float4*>(ap + t * 32 * LDA + s4);
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[t].x, bv.x, acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[t].y, bv.y, acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[t].z, bv.z, acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[t].w, bv.w, acc[t], 0, 0, 0);
          }
        }
      }
      // dist = (|x|^2 + |c|^2) - 2 x.c  (quantize.py:108-112); C/D map: row i = codeword,
      // col = lane&31 = item. Lowest index wins ties (torch min, quantize.py:121).
#pragma unroll
      for (int t = 0; t < 4; ++t) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          // indices visited in increasing order per lane: strict '<' keeps the lowest one
          const int il = t * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          const int i = n0 + il;
          float d = (xs + cs_s[il]) - 2.f * acc[t][r];
          d = i < K ? d : INFINITY;
          const bool lt = d < best_d;
          best_d = lt ? d : best_d;
          best_i = lt ? i : best_i;
        }
      }
    }
    {
      const float od = __shfl_xor(best_d, 32, 64);
      const int oi = __shfl_xor(best_i, 32, 64);
      if (od < best_d || (od == best_d && oi < best_i)) { best_d = od; best_i = oi; }
      if (h == 0) id_s[wave * 32 + lane] = best_i;
    }
    __syncthreads();

    // Row epilogue: gather codeword, emb_out per mode, VQ loss, next residual.
    float* eo = emb_out + (int64_t)l * BD;
    float* rn = res + (int64_t)(l + 1) * BD;
    for (int it = 0; it < 32 / G; ++it) {
      const int jl = wave * 32 + it * G + grp;
      const int b = row0 + jl;
      const bool valid = b < B;
      const int64_t o = (int64_t)(valid ? b : B - 1) * D + sub * EPL;
      const int id = id_s[jl];
      const float* cr = cb + (int64_t)id * D + sub * EPL;
      float xv[EPL], ev[EPL], out[EPL];
#pragma unroll
      for (int k = 0; k < EPL; k += 4) {
        const float4 a = *reinterpret_cast<const float4*>(src + o + k);
        const float4 c = *reinterpret_cast<const float4*>(cr + k);
        xv[k] = a.x; xv[k + 1] = a.y; xv[k + 2] = a.z; xv[k + 3] = a.w;
        ev[k] = c.x; ev[k + 1] = c.y; ev[k + 2] = c.z; ev[k + 3] = c.w;
      }
      float dl = 0.f;
#pragma unroll
      for (int k = 0; k < EPL; ++k) { const float t = xv[k] - ev[k]; dl += t * t; }
      dl = group_sum<LPI>(dl);
      if (mode == kRotation) {
        float x2 = 0.f, e2 = 0.f;
#pragma unroll
        for (int k = 0; k < EPL; ++k) { x2 += xv[k] * xv[k]; e2 += ev[k] * ev[k]; }
        x2 = group_sum<LPI>(x2);
        e2 = group_sum<LPI>(e2);
        RowRot<LPI, EPL> rr;
        rr.build(xv, ev, sqrtf(x2), sqrtf(e2));
        float ew = 0.f, eu = 0.f;
#pragma unroll
        for (int k = 0; k < EPL; ++k) { ew += xv[k] * rr.w[k]; eu += xv[k] * rr.u[k]; }
        ew = group_sum<LPI>(ew);
        eu = group_sum<LPI>(eu);
        // out = e - 2 (e.w) w + 2 (e.u) q, then * lam   (quantize.py:41-45, :140-142)
#pragma unroll
        for (int k = 0; k < EPL; ++k) out[k] = ((xv[k] - 2.f * (ew * rr.w[k])) + 2.f * (eu * rr.q[k])) * rr.lam;
      } else if (mode == kSte) {
#pragma unroll
        for (int k = 0; k < EPL; ++k) out[k] = xv[k] + (ev[k] - xv[k]);   // x + (emb - x).detach()
      } else {
#pragma unroll
        for (int k = 0; k < EPL; ++k) out[k] = ev[k];
      }
      float r2 = 0.f;
      float nr[EPL];
#pragma unroll
      for (int k = 0; k < EPL; ++k) { nr[k] = xv[k] - out[k]; r2 += nr[k] * nr[k]; }
      r2 = group_sum<LPI>(r2);
      if (valid) {
#pragma unroll
        for (int k = 0; k < EPL; k += 4) {
          *reinterpret_cast<float4*>(eo + o + k) = make_float4(out[k], out[k + 1], out[k + 2], out[k + 3]);
          if (l + 1 < L)
            *reinterpret_cast<float4*>(rn + o + k) = make_float4(nr[k], nr[k + 1], nr[k + 2], nr[k + 3]);
        }
        if (emb_sum != nullptr && l == L - 1) {
          // sum over the level axis in level order: ((e0 + e1) + e2) ...
#pragma unroll
          for (int k = 0; k < EPL; k += 4) {
            float4 s = *reinterpret_cast<const float4*>(emb_out + o + k);
            for (int m = 1; m < L; ++m) {
              const float4 v = (m == l) ? make_float4(out[k], out[k + 1], out[k + 2], out[k + 3])
                                        : *reinterpret_cast<const float4*>(emb_out + (int64_t)m * BD + o + k);
              s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
            }
            if (L == 1) s = make_float4(out[k], out[k + 1], out[k + 2], out[k + 3]);
            *reinterpret_cast<float4*>(emb_sum + o + k) = s;
          }
        }
        if (sub == 0) {
          ids[(int64_t)b * L + l] = id;
          const float lq = dl + beta * dl;   // emb_loss + beta * query_loss (equal values fwd)
          const float acc_l = ql_s[jl] + lq;
          ql_s[jl] = acc_l;
          xsq_s[jl] = r2;
          if (l == L - 1) qloss[b] = acc_l;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// Backward, per item: walk the levels last -> first.
//   g_out_l = g_emb_l + g_emb_sum - g_{res_{l+1}}
//   rotation: g_x = lam*g - 2 ((lam*g).w) w + 2 ((lam*g).q) u   (autograd order of :41-45,140)
//   ste:      g_x = g_out_l ;  eval: g_x = 0, codeword row gets g_out_l
//   VQ loss:  g_x += 2 beta gl (x - e) ; codeword += 2 gl (e - x)
//   g_{res_l} = g_{res_{l+1}} + g_x (+ g_res_l)
// Codeword contributions go to `contrib` (L,B,D); rq_cb_segsum reduces them per codeword.
template <int LPI, int EPL>
__global__ void __launch_bounds__(256)
rq_bwd_rows_kernel(const float* __restrict__ res, const int64_t* __restrict__ ids, const float* __restrict__ cbs,
                   int B, int D, int K, int L, int mode, float beta, const float* __restrict__ g_emb,
                   const float* __restrict__ g_emb_sum, const float* __restrict__ g_res,
                   const float* __restrict__ g_qloss, float* __restrict__ grad_x, float* __restrict__ contrib) {
  constexpr int G = 64 / LPI;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = lane % LPI, grp = lane / LPI;
  const int b = (blockIdx.x * 4 + wave) * G + grp;
  const bool valid = b < B;
  const int bb = valid ? b : B - 1;
  const int64_t BD = (int64_t)B * D;
  const int64_t o = (int64_t)bb * D + sub * EPL;
  const float gl = g_qloss ? g_qloss[bb] : 0.f;
  float gn[EPL];
#pragma unroll
  for (int k = 0; k < EPL; ++k) gn[k] = 0.f;
  for (int l = L - 1; l >= 0; --l) {
    int id = (int)ids[(int64_t)bb * L + l];
    const float* cr = cbs + ((int64_t)l * K + id) * D + sub * EPL;
    float xv[EPL], ev[EPL], go[EPL], gx[EPL];
#pragma unroll
    for (int k = 0; k < EPL; k += 4) {
      const float4 a = *reinterpret_cast<const float4*>(res + (int64_t)l * BD + o + k);
      const float4 c = *reinterpret_cast<const float4*>(cr + k);
      xv[k] = a.x; xv[k + 1] = a.y; xv[k + 2] = a.z; xv[k + 3] = a.w;
      ev[k] = c.x; ev[k + 1] = c.y; ev[k + 2] = c.z; ev[k + 3] = c.w;
    }
#pragma unroll
    for (int k = 0; k < EPL; ++k) go[k] = 0.f;
    if (g_emb_sum) {
#pragma unroll
      for (int k = 0; k < EPL; ++k) go[k] += g_emb_sum[o + k];
    }
    if (g_emb) {
#pragma unroll
      for (int k = 0; k < EPL; ++k) go[k] += g_emb[(int64_t)l * BD + o + k];
    }
#pragma unroll
    for (int k = 0; k < EPL; ++k) go[k] -= gn[k];

    if (mode == kRotation) {
      float x2 = 0.f, e2 = 0.f;
#pragma unroll
      for (int k = 0; k < EPL; ++k) { x2 += xv[k] * xv[k]; e2 += ev[k] * ev[k]; }
      x2 = group_sum<LPI>(x2);
      e2 = group_sum<LPI>(e2);
      RowRot<LPI, EPL> rr;
      rr.build(xv, ev, sqrtf(x2), sqrtf(e2));
      float gw = 0.f, gq = 0.f, gs[EPL];
#pragma unroll
      for (int k = 0; k < EPL; ++k) { gs[k] = go[k] * rr.lam; gw += gs[k] * rr.w[k]; gq += gs[k] * rr.q[k]; }
      gw = group_sum<LPI>(gw);
      gq = group_sum<LPI>(gq);
#pragma unroll
      for (int k = 0; k < EPL; ++k) gx[k] = (gs[k] - 2.f * (gw * rr.w[k])) + 2.f * (gq * rr.u[k]);
    } else if (mode == kSte) {
#pragma unroll
      for (int k = 0; k < EPL; ++k) gx[k] = go[k];
    } else {
#pragma unroll
      for (int k = 0; k < EPL; ++k) gx[k] = 0.f;
    }
    float cc[EPL];
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
      gx[k] += (2.f * beta * gl) * (xv[k] - ev[k]);
      cc[k] = (2.f * gl) * (ev[k] - xv[k]);
      if (mode == kEval) cc[k] += go[k];
      gn[k] = gn[k] + gx[k];
      if (g_res) gn[k] += g_res[(int64_t)l * BD + o + k];
    }
    if (valid && contrib != nullptr) {   // eval mode only: the codeword also gets the emb_out grad
#pragma unroll
      for (int k = 0; k < EPL; k += 4)
        *reinterpret_cast<float4*>(contrib + (int64_t)l * BD + o + k) = make_float4(cc[k], cc[k + 1], cc[k + 2], cc[k + 3]);
    }
  }
  if (valid) {
#pragma unroll
    for (int k = 0; k < EPL; k += 4)
      *reinterpret_cast<float4*>(grad_x + o + k) = make_float4(gn[k], gn[k + 1], gn[k + 2], gn[k + 3]);
  }
}

// ---------------------------------------------------------------------------------------
// Stable counting sort of ids per level (keys < K <= 4096) -> perm (rows grouped by codeword,
// ascending row index inside a codeword): per-block histograms hist[l][blk][k] (key fastest,
// coalesced), a per-key scan over blocks, an exclusive scan over keys, then an in-order scatter
// (per-block LDS bitonic sort of (key, row) pairs). Deterministic by construction (no atomics decide any order).
constexpr int kSortRows = 256;   // rows per sort block

__global__ void __launch_bounds__(256) sort_hist_kernel(const int64_t* __restrict__ ids, int B, int L, int K,
                                                         int nblk, int* __restrict__ hist) {
  extern __shared__ int cnt[];
  const int l = blockIdx.y, blk = blockIdx.x;
  for (int k = threadIdx.x; k < K; k += 256) cnt[k] = 0;
  __syncthreads();
  const int r = blk * kSortRows + threadIdx.x;
  if (r < B) {
    const int64_t key = ids[(int64_t)r * L + l];
    if (key >= 0 && key < K) atomicAdd(&cnt[(int)key], 1);   // counts only: order-free; bad keys dropped
  }
  __syncthreads();
  int* h = hist + ((int64_t)l * nblk + blk) * K;
  for (int k = threadIdx.x; k < K; k += 256) h[k] = cnt[k];
}

// Per key: exclusive scan over blocks (in place) and the key's total -> key_off[l][k].
// Per (level, key): exclusive scan over the histogram blocks in place (hist[l][blk][k] becomes the
// key's first slot within the key for block blk) and the key's total into key_off[l][k]. 16 keys per
// workgroup x 16 block segments (one thread each: a sum pass, then the write pass), segment sums
// combined in LDS: the one-thread-per-key serial walk over 256 blocks was latency-bound (~13 us at
// B = 65,536).
constexpr int kScanSeg = 16;
__global__ void __launch_bounds__(256) sort_keyscan_kernel(int* __restrict__ hist, int K, int nblk,
                                                            int* __restrict__ key_off) {
  __shared__ int part[kScanSeg][16];
  const int l = blockIdx.y, seg = threadIdx.x / 16, kk = threadIdx.x % 16, k = blockIdx.x * 16 + kk;
  const int per = (nblk + kScanSeg - 1) / kScanSeg, b0 = seg * per, b1 = min(nblk, b0 + per);
  int* h = hist + (int64_t)l * nblk * K + k;
  int sum = 0;
  if (k < K)
    for (int u = b0; u < b1; ++u) sum += h[(int64_t)u * K];
  part[seg][kk] = sum;
  __syncthreads();
  if (k >= K) return;
  int run = 0;
  for (int j = 0; j < seg; ++j) run += part[j][kk];
  for (int u = b0; u < b1; ++u) {
    const int x = h[(int64_t)u * K];
    h[(int64_t)u * K] = run;
    run += x;
  }
  if (seg == kScanSeg - 1) key_off[(int64_t)l * (K + 1) + k] = run;
}

// Exclusive scan of the per-key totals in place: key_off[l][k] = first slot of key k; [K] = B.
__global__ void __launch_bounds__(1024) sort_offsets_kernel(int* __restrict__ key_off, int K, int B) {
  __shared__ int part[1024];
  const int l = blockIdx.x, t = threadIdx.x;
  int* ko = key_off + (int64_t)l * (K + 1);
  const int per = (K + 1023) / 1024;
  const int a = t * per, e = min(a + per, K);
  int s = 0;
  for (int i = a; i < e; ++i) s += ko[i];
  part[t] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const int v = t >= o ? part[t - o] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int run = part[t] - s;
  for (int i = a; i < e; ++i) { const int c = ko[i]; ko[i] = run; run += c; }
  if (t == 1023) ko[K] = part[1023];   // rows placed (B unless out-of-range keys were dropped)
}

// Stable placement of one block's 256 rows: a bitonic sort of (key << 8 | row-in-block) in LDS
// orders the rows by key then row index; a row's rank inside its key run is its sorted position
// minus the run's first position. 36 compare-exchange stages, no per-key serial loop.
__global__ void __launch_bounds__(256) sort_scatter_kernel(const int64_t* __restrict__ ids, int B, int L, int K,
                                                           int nblk, const int* __restrict__ hist,
                                                           const int* __restrict__ key_off, int* __restrict__ perm) {
  extern __shared__ int sm[];
  int* base = sm;                                          // [K] first output slot of key k for this block
  int* first = sm + K;                                     // [K] sorted position where key k's run starts
  unsigned* sk = reinterpret_cast<unsigned*>(sm + 2 * K);  // [256]
  const int l = blockIdx.y, blk = blockIdx.x, t = threadIdx.x;
  const int* h = hist + ((int64_t)l * nblk + blk) * K;
  const int* ko = key_off + (int64_t)l * (K + 1);
  for (int k = t; k < K; k += 256) base[k] = ko[k] + h[k];
  const int r = blk * kSortRows + t;
  const int64_t k64 = r < B ? ids[(int64_t)r * L + l] : -1;
  const bool valid = k64 >= 0 && k64 < K;   // rows with out-of-range keys are not placed
  sk[t] = valid ? ((unsigned)k64 << 8) | (unsigned)t : 0xFFFFFFFFu;
  __syncthreads();
  for (int size = 2; size <= kSortRows; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const int j = t ^ stride;
      if (j > t) {
        const unsigned a = sk[t], b = sk[j];
        if ((a > b) == ((t & size) == 0)) { sk[t] = b; sk[j] = a; }
      }
      __syncthreads();
    }
  }
  const unsigned v = sk[t];
  const bool placed = v != 0xFFFFFFFFu;
  const int key = (int)(v >> 8);
  if (placed && (t == 0 || (sk[t - 1] >> 8) != (unsigned)key)) first[key] = t;
  __syncthreads();
  if (placed) perm[(int64_t)l * B + base[key] + (t - first[key])] = blk * kSortRows + (int)(v & 255u);
}

// grad_cb[l][k] = sum over the rows b of codeword k of c_b, with
//   c_b = (2 gl_b) (e_k - x_b)            (rotation / STE: recomputed from residuals, no buffer)
//   c_b = contrib[l][b]                   (eval mode / generic segment sum: the given rows)
// Workgroup (k, g, l), 4 waves: a segment of at most kSegDirect rows is reduced entirely by g = 0
// and written to grad_cb; a longer one (e.g. the dedup-column token every item shares) is cut into
// kSegSplit contiguous parts whose partial sums go to scratch[g][l][k] and rq_segsum_finalize adds
// them in g order. Inside a workgroup wave w reduces the w-th contiguous quarter of its rows, lanes
// hold float4 columns (RPW rows per wave-step when D < 256), partials combine in a fixed order:
// bitwise deterministic for any placement.
constexpr int kSegSplit = 8;
constexpr int kSegDirect = 256;

__global__ void __launch_bounds__(256) rq_cb_segsum_kernel(const float* __restrict__ res, const float* __restrict__ cbs,
                                                           const float* __restrict__ g_qloss,
                                                           const float* __restrict__ contrib, const int* __restrict__ perm,
                                                           const int* __restrict__ key_off, int B, int D, int K,
                                                           float* __restrict__ grad_cb, float* __restrict__ scratch) {
  __shared__ float4 part[4 * 64];
  const int k = blockIdx.x, g = blockIdx.y, l = blockIdx.z, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int L = gridDim.z;
  const int a0 = key_off[(int64_t)l * (K + 1) + k], e0 = key_off[(int64_t)l * (K + 1) + k + 1];
  const int n0 = e0 - a0;
  const bool direct = n0 <= kSegDirect;
  if (direct && g > 0) return;
  const int a = direct ? a0 : a0 + (int)((int64_t)n0 * g / kSegSplit);
  const int e = direct ? e0 : a0 + (int)((int64_t)n0 * (g + 1) / kSegSplit);
  const int n = e - a, q = (n + 3) / 4;
  const int wa = a + min(n, wave * q), we = a + min(n, (wave + 1) * q);
  const int* p = perm + (int64_t)l * B;
  const int64_t BD = (int64_t)B * D;
  const float* xb = contrib ? contrib + (int64_t)l * BD : res + (int64_t)l * BD;
  const float* ek = cbs ? cbs + ((int64_t)l * K + k) * D : nullptr;
  float* dst = direct ? grad_cb + ((int64_t)l * K + k) * D : scratch + (((int64_t)g * L + l) * K + k) * D;
  const int D4 = D / 4;
  const int cpw = D4 < 64 ? D4 : 64, rpw = 64 / cpw;
  const int rs = lane / cpw, c4 = lane % cpw;
  for (int d0 = 0; d0 < D4; d0 += 64) {
    const int d = d0 + c4;
    const bool dok = d < D4;
    const float4 e_d = (contrib || !dok) ? make_float4(0.f, 0.f, 0.f, 0.f) : reinterpret_cast<const float4*>(ek)[d];
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    int i = wa + rs;
    for (; i + 7 * rpw < we; i += 8 * rpw) {
      int rr[8];
      float4 v[8];
      float gg[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) rr[u] = p[i + u * rpw];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        v[u] = dok ? reinterpret_cast<const float4*>(xb + (int64_t)rr[u] * D)[d] : make_float4(0.f, 0.f, 0.f, 0.f);
        gg[u] = contrib ? 1.f : 2.f * (g_qloss ? g_qloss[rr[u]] : 0.f);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (contrib) {
          acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w;
        } else {
          acc.x += gg[u] * (e_d.x - v[u].x); acc.y += gg[u] * (e_d.y - v[u].y);
          acc.z += gg[u] * (e_d.z - v[u].z); acc.w += gg[u] * (e_d.w - v[u].w);
        }
      }
    }
    for (; i < we; i += rpw) {
      const int r = p[i];
      const float4 v = dok ? reinterpret_cast<const float4*>(xb + (int64_t)r * D)[d] : make_float4(0.f, 0.f, 0.f, 0.f);
      if (contrib) {
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      } else {
        const float gr = 2.f * (g_qloss ? g_qloss[r] : 0.f);
        acc.x += gr * (e_d.x - v.x); acc.y += gr * (e_d.y - v.y); acc.z += gr * (e_d.z - v.z); acc.w += gr * (e_d.w - v.w);
      }
    }
    part[(wave * rpw + rs) * cpw + c4] = acc;
    __syncthreads();
    if (tid < cpw && d0 + tid < D4) {
      float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int j = 0; j < 4 * rpw; ++j) {
        const float4 v = part[j * cpw + tid];
        t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
      }
      reinterpret_cast<float4*>(dst)[d0 + tid] = t;
    }
    __syncthreads();
  }
}

// Heavy segments: grad_cb[l][k] = sum_g scratch[g][l][k] in g order.
__global__ void __launch_bounds__(256) rq_segsum_finalize_kernel(const int* __restrict__ key_off, int D, int K,
                                                                 const float* __restrict__ scratch,
                                                                 float* __restrict__ grad_cb) {
  const int k = blockIdx.x, l = blockIdx.y, L = gridDim.y;
  const int n = key_off[(int64_t)l * (K + 1) + k + 1] - key_off[(int64_t)l * (K + 1) + k];
  if (n <= kSegDirect) return;
  for (int d = threadIdx.x; d < D; d += 256) {
    float s = 0.f;
#pragma unroll
    for (int g = 0; g < kSegSplit; ++g) s += scratch[(((int64_t)g * L + l) * K + k) * D + d];
    grad_cb[((int64_t)l * K + k) * D + d] = s;
  }
}

// ---------------------------------------------------------------------------------------
// Codebook gradient without the sort (rotation / STE at K D <= 16,384: the RQ-VAE's 256 x 64 levels), two
// launches instead of six. Workgroup (c, l) owns rows [c R, (c + 1) R) of level l and sums their codeword
// contributions 2 gl_b (e_k - x_b) into an LDS image acc[K][D]: wave w of 16 owns the codewords k with
// 16 k / K == w and walks the chunk's rows in order (a ballot per 64 rows, matches taken lowest row first,
// their residual and codeword rows loaded sixteen at a time), so every acc[k] is a row-ordered sum —
// deterministic with no atomics. The
// image goes to partial[l][c] (zeros where the chunk has no row of k); rq_cb_chunk_reduce sums the chunks in
// c order (four interleaved partial sums, slab_sum_w4). Lane = VPL consecutive dims (D = 64 VPL).
#ifndef RQ_CB_CHUNK
#define RQ_CB_CHUNK 1   // 0: the sort + segmented-sum codebook gradient for every mode (A/B)
#endif
constexpr int kCbRows = 1024;   // rows per workgroup
constexpr int kCbWaves = 16, kCbBatch = 16;
constexpr int kCbList = 256;   // match-list entries per wave (a skewed chunk drains it more often)
template <int VPL>
__global__ void __launch_bounds__(64 * kCbWaves) rq_cb_chunk_kernel(const float* __restrict__ res, const float* __restrict__ cbs,
                                                          const float* __restrict__ g_qloss,
                                                          const int64_t* __restrict__ ids, int B, int K, int L,
                                                          float* __restrict__ partial) {
  constexpr int D = 64 * VPL, NB = kCbBatch / VPL;   // matches per batch (VGPRs: 16 waves per workgroup)
  extern __shared__ __attribute__((aligned(16))) float acc[];   // [K][D], the chunk's ids, the waves' match lists
  int* ids_s = reinterpret_cast<int*>(acc + (int64_t)K * D);
  const int c = blockIdx.x, l = blockIdx.y, nchunk = gridDim.x, tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  unsigned short* list = reinterpret_cast<unsigned short*>(ids_s + kCbRows) + wave * kCbList;
  const int r0 = c * kCbRows;
  for (int i = tid; i < K * D / 4; i += 64 * kCbWaves) reinterpret_cast<float4*>(acc)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int i = tid; i < kCbRows; i += 64 * kCbWaves) {
    const int r = r0 + i;
    const int64_t k = r < B ? ids[(int64_t)r * L + l] : -1;
    ids_s[i] = (k >= 0 && k < K) ? (int)k : -1;
  }
  __syncthreads();
  const int64_t BD = (int64_t)B * D;
  const float* xl = res + (int64_t)l * BD;
  const float* el = cbs + (int64_t)l * K * D;
  // this wave's rows (ascending) in batches of NB: loads first, then the row-ordered accumulation
  auto drain = [&](int n_list) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the list entries other lanes wrote
    for (int i0 = 0; i0 < n_list; i0 += NB) {
      int rr[NB], kc[NB];
      float xv[NB][VPL], ev[NB][VPL], gg[NB];
      // every load unconditional (entries past the list repeat its last one, not accumulated): a branch
      // around a load makes the compiler wait for it at the merge, one round trip per match
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        const int row = list[min(i0 + u, n_list - 1)];
        rr[u] = r0 + row;
        kc[u] = ids_s[row];
        gg[u] = 2.f * g_qloss[rr[u]];
#pragma unroll
        for (int j = 0; j < VPL; ++j) {
          xv[u][j] = xl[(int64_t)rr[u] * D + lane * VPL + j];
          ev[u][j] = el[(int64_t)kc[u] * D + lane * VPL + j];
        }
      }
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        if (i0 + u < n_list) {
          float* a = acc + (int64_t)kc[u] * D + lane * VPL;
#pragma unroll
          for (int j = 0; j < VPL; ++j) a[j] += gg[u] * (ev[u][j] - xv[u][j]);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the list is rewritten after this
  };
  int n_list = 0;
  for (int g0 = 0; g0 < kCbRows; g0 += 64) {
    const int kk = ids_s[g0 + lane];
    const bool mine = kk >= 0 && (kCbWaves * kk) / K == wave;
    const unsigned long long m = __ballot(mine);
    const int cnt = __popcll(m);
    if (n_list + cnt > kCbList) {
      drain(n_list);
      n_list = 0;
    }
    const int before = __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
    if (mine) list[n_list + before] = (unsigned short)(g0 + lane);
    n_list += cnt;
  }
  drain(n_list);
  __syncthreads();
  float4* dst = reinterpret_cast<float4*>(partial + ((int64_t)l * nchunk + c) * K * D);
  for (int i = tid; i < K * D / 4; i += 64 * kCbWaves) dst[i] = reinterpret_cast<const float4*>(acc)[i];
}

// grad_cb[l][j] = sum over chunks c (in order) of partial[l][c][j], one float4 column per thread.
__global__ void __launch_bounds__(256) rq_cb_chunk_reduce_kernel(const float* __restrict__ partial, int nchunk,
                                                                 int64_t KD, float* __restrict__ grad_cb) {
  const int l = blockIdx.y;
  const int64_t j = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (j >= KD) return;
  const float4 r = slab_sum_w4(partial + (int64_t)l * nchunk * KD, nchunk, KD, j);
  *reinterpret_cast<float4*>(grad_cb + (int64_t)l * KD + j) = r;
}

static bool cb_chunk_path(int64_t B, int64_t D, int64_t K, int mode, const float* g_qloss) {
  return mode != kEval && g_qloss && (D == 64 || D == 128 || D == 256) && K * D <= 16384 && B >= 4 * kCbRows;
}
static int64_t cb_chunks(int64_t B) { return (B + kCbRows - 1) / kCbRows; }

// ---------------------------------------------------------------------------------------
// Register-resident forward for small D (D <= 64): items stay on the MFMA lane axis for the
// whole L-level chain. Lane (j, h) holds item j's half-row x[j][h*D/2 .. +D/2) — exactly its
// B-operand fragment — so the distance GEMM reads only codewords from LDS, the argmin is a
// register scan, and the epilogue (rotation trick / STE / eval, VQ loss, next residual) runs on
// the same registers with one xor-32 lane swap per row reduction. The next level's residual never
// leaves the VGPRs; the codeword row for the epilogue comes from the LDS copy of the level.
// RESIDENT: the whole level codebook fits one LDS image (K rows); otherwise it is streamed in
// chunks of NB rows and the epilogue reads the chosen codeword from global memory (L2).
template <int D, bool RESIDENT, int WPI>
__global__ void __launch_bounds__(256, 2)
rq_fwd_reg_kernel(const float* __restrict__ x, int B, const float* __restrict__ cbs, const float* __restrict__ csq,
                  int K, int L, int mode, float beta, int NB, int64_t* __restrict__ ids, float* __restrict__ emb_out,
                  float* __restrict__ res, float* __restrict__ qloss, float* __restrict__ emb_sum) {
  // WPI waves share one 32-item tile and split its codeword tiles (small-B latency mode);
  // items per workgroup = 128 / WPI. All WPI waves run the (cheap) epilogue redundantly so each
  // keeps the next residual in its own registers; only sub-wave 0 stores.
  // SWZ: the resident D=64 image is filled by LDS-DMA (global_load_lds_dwordx4, no VGPR staging)
  // into unpadded 256-B rows whose 16-B chunks are XOR-swizzled by (row & 15): chunk c of row r
  // sits at c ^ (r & 15), so the 16 rows a ds_read_b128 lane group touches hit 16 distinct
  // 4-bank groups. Otherwise rows are padded to D + 4 floats and filled through registers.
  constexpr bool SWZ = RESIDENT && D == 64;
  constexpr int H2 = D / 2, LD = SWZ ? D : D + 4;
  extern __shared__ __attribute__((aligned(16))) float dsm[];
  const int NBp = (NB + 31) & ~31;
  float* A_s = dsm;                                  // [NBp][LD] codewords of the current level / chunk
  float* cs_s = dsm + NBp * LD;                      // [NBp]     |c|^2
  float* rd_s = cs_s + NBp;                          // [4][32]  per-wave best distance (WPI > 1)
  int* ri_s = reinterpret_cast<int*>(rd_s + 128);    // [4][32]  per-wave best index
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, h = lane >> 5;
  const int tile = wave / WPI, wsub = wave % WPI;
  const int b = blockIdx.x * (128 / WPI) + tile * 32 + (lane & 31);
  const bool valid = b < B;
  const bool writer = valid && wsub == 0;
  const int64_t BD = (int64_t)B * D;
  const int64_t o = (int64_t)(valid ? b : 0) * D + h * H2;
  float xv[H2], es[H2];
#pragma unroll
  for (int k = 0; k < H2; k += 4) {
    const float4 v = valid ? *reinterpret_cast<const float4*>(x + o + k) : make_float4(0.f, 0.f, 0.f, 0.f);
    xv[k] = v.x; xv[k + 1] = v.y; xv[k + 2] = v.z; xv[k + 3] = v.w;
  }
#pragma unroll
  for (int k = 0; k < H2; ++k) es[k] = 0.f;
  float ql = 0.f;

  // Stores are deferred until the NEXT level's codebook staging has landed in LDS: gfx950 has one
  // in-order vmcnt for loads and stores, so a store issued before the staging loads would make
  // their wait drain it (HBM write latency on the critical path). Issued after, the stores drain
  // under the level's MFMA phase. pend_e = emb_out[l-1] still to store.
  float pend_e[H2];
  auto flush = [&](int l) {   // residuals[l] (= current xv) and emb_out[l-1]
    if (!writer) return;
#pragma unroll
    for (int k = 0; k < H2; k += 4)
      *reinterpret_cast<float4*>(res + (int64_t)l * BD + o + k) = make_float4(xv[k], xv[k + 1], xv[k + 2], xv[k + 3]);
    if (l > 0) {
#pragma unroll
      for (int k = 0; k < H2; k += 4)
        *reinterpret_cast<float4*>(emb_out + (int64_t)(l - 1) * BD + o + k) =
            make_float4(pend_e[k], pend_e[k + 1], pend_e[k + 2], pend_e[k + 3]);
    }
  };

  for (int l = 0; l < L; ++l) {
    const float* cb = cbs + (int64_t)l * K * D;
    float xs = 0.f;
#pragma unroll
    for (int k = 0; k < H2; ++k) xs = __builtin_fmaf(xv[k], xv[k], xs);
    xs += __shfl_xor(xs, 32, 64);
    float best_d = INFINITY;
    int best_i = 0;
    for (int n0 = 0; n0 < K; n0 += NB) {
      const int nrows = min(NB, K - n0);
      __syncthreads();   // previous level / chunk fully consumed (incl. epilogue codeword reads)
      if constexpr (SWZ) {
        // wave-instruction q moves rows 4q..4q+3 (1 KiB): lane i lands at LDS chunk i%16 of row
        // 4q + i/16 and therefore loads logical chunk (i%16) ^ (row & 15) of that row
        const int nq = (nrows + 3) / 4;
        for (int q = wave; q < nq; q += 4) {
          const int row = min(4 * q + (lane >> 4), nrows - 1);
          const int c = (lane & 15) ^ (row & 15);
          __builtin_amdgcn_global_load_lds(cb + (int64_t)(n0 + row) * D + 4 * c, A_s + q * 256, 16, 0, 0);
        }
      } else {
        // 8 float4 loads in flight per thread before their LDS writes (a plain strided loop
        // compiles to load -> vmcnt(0) -> ds_write per element); indices past the chunk are
        // clamped, so neither the loads nor the writes sit behind a branch
        const int total = nrows * (D / 4);
        const float* cbn = cb + (int64_t)n0 * D;
        for (int f0 = 0; f0 < total; f0 += 256 * 8) {
          float4 v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int f = min(f0 + u * 256 + tid, total - 1);
            v[u] = *reinterpret_cast<const float4*>(cbn + (int64_t)(f / (D / 4)) * D + (f % (D / 4)) * 4);
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) {   // clamped lanes rewrite the last element with its own value
            const int f = min(f0 + u * 256 + tid, total - 1);
            *reinterpret_cast<float4*>(A_s + (f / (D / 4)) * LD + (f % (D / 4)) * 4) = v[u];
          }
        }
      }
      for (int r = tid; r < NBp; r += 256) cs_s[r] = r < nrows ? csq[(int64_t)l * K + n0 + r] : INFINITY;
      __syncthreads();
      if (n0 == 0) flush(l);   // after the barrier: the stores drain under this level's MFMAs
      // One-tile software pipeline: the argmin scan of tile t (VALU) is independent of tile
      // t+1's MFMA chain, so it fills the 64-cycle dependent-MFMA gaps instead of draining them.
      // Rows past nrows (last partial tile) read stale LDS; their distances are forced to +inf.
      // Each lane visits its codeword indices in increasing order, so a strict '<' keeps the
      // lowest index among equal distances (torch.argmin); the lane-pair merge below breaks ties.
      // d = (|x|^2 + |c|^2) - 2 x.c as fma(-2, x.c, |x|^2 + |c|^2): 2 x.c is exact, so this is the
      // reference expression's rounding. The tile's best (d, register) is found first, then merged
      // into the running best once per tile (strict '<' keeps the earlier tile on ties).
      auto scan = [&](const floatx16& a, const float4 (&c)[4], int t0) {
        float td = INFINITY;
        int tr = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float cr = (r & 3) == 0 ? c[r >> 2].x : (r & 3) == 1 ? c[r >> 2].y : (r & 3) == 2 ? c[r >> 2].z
                                                                                                  : c[r >> 2].w;
          const float d = __builtin_fmaf(-2.f, a[r], xs + cr);
          const bool lt = d < td;
          td = lt ? d : td;
          tr = lt ? r : tr;
        }
        const bool lt = td < best_d;
        best_d = lt ? td : best_d;
        best_i = lt ? n0 + t0 + (tr & 3) + 8 * (tr >> 2) + 4 * h : best_i;
      };
      auto chain = [&](int t0, floatx16& acc, float4 (&c)[4]) {
#pragma unroll
        for (int j = 0; j < 4; ++j) c[j] = *reinterpret_cast<const float4*>(cs_s + t0 + 8 * j + 4 * h);
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.f;
        const int arow = t0 + (lane & 31);
        const float* ap = A_s + arow * LD + h * H2;
#pragma unroll
        for (int s4 = 0; s4 < H2; s4 += 4) {
          const float4 a = SWZ ? *reinterpret_cast<const float4*>(A_s + arow * LD + 4 * (((h * H2 + s4) >> 2) ^ (arow & 15)))
                               : *reinterpret_cast<const float4*>(ap + s4);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, xv[s4], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, xv[s4 + 1], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, xv[s4 + 2], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, xv[s4 + 3], acc, 0, 0, 0);
        }
      };
      int t0 = wsub * 32;
      if (t0 < nrows) {
        floatx16 acc_p;
        float4 cp[4];
        chain(t0, acc_p, cp);
        int tp = t0;
        for (t0 += 32 * WPI; t0 < nrows; t0 += 32 * WPI) {
          floatx16 acc;
          float4 cn[4];
          chain(t0, acc, cn);
          scan(acc_p, cp, tp);
          // interleave: 2 MFMAs (128 cycles of matrix work) then a slice of the previous
          // tile's scan, with the codeword ds_reads spread ahead of the MFMAs that use them
          __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);
#pragma unroll
          for (int i = 0; i < H2 / 2; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);
            if (i < H2 / 4 - 2) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          }
          acc_p = acc;
#pragma unroll
          for (int j = 0; j < 4; ++j) cp[j] = cn[j];
          tp = t0;
        }
        scan(acc_p, cp, tp);
      }
    }
    {
      const float od = __shfl_xor(best_d, 32, 64);
      const int oi = __shfl_xor(best_i, 32, 64);
      if (od < best_d || (od == best_d && oi < best_i)) { best_d = od; best_i = oi; }
    }
    if constexpr (WPI > 1) {   // combine the sub-waves' candidates in a fixed order
      if (h == 0) { rd_s[wave * 32 + lane] = best_d; ri_s[wave * 32 + lane] = best_i; }
      __syncthreads();
      best_d = INFINITY;
      best_i = 0;
#pragma unroll
      for (int w = 0; w < WPI; ++w) {
        const float od = rd_s[(tile * WPI + w) * 32 + (lane & 31)];
        const int oi = ri_s[(tile * WPI + w) * 32 + (lane & 31)];
        if (od < best_d || (od == best_d && oi < best_i)) { best_d = od; best_i = oi; }
      }
    }
    const int id = best_i;
    // ---- epilogue on the item's two lanes
    float ev[H2];
    const float* er = RESIDENT ? (A_s + id * LD + h * H2) : (cb + (int64_t)id * D + h * H2);
#pragma unroll
    for (int k = 0; k < H2; k += 4) {
      const float4 c = SWZ ? *reinterpret_cast<const float4*>(A_s + id * LD + 4 * (((h * H2 + k) >> 2) ^ (id & 15)))
                           : *reinterpret_cast<const float4*>(er + k);
      ev[k] = c.x; ev[k + 1] = c.y; ev[k + 2] = c.z; ev[k + 3] = c.w;
    }
    // Row sums use fma (one rounding per term); |x|^2 is the level's xs. The reference's torch
    // reductions round in their own order, so parity here is tolerance-level for the embeddings
    // (ids: exact up to reference top-2 ties within that tolerance), as for every reduction.
    float e2 = 0.f, dl = 0.f;
#pragma unroll
    for (int k = 0; k < H2; ++k) {
      e2 = __builtin_fmaf(ev[k], ev[k], e2);
      const float t = xv[k] - ev[k];
      dl = __builtin_fmaf(t, t, dl);
    }
    e2 += __shfl_xor(e2, 32, 64);
    dl += __shfl_xor(dl, 32, 64);
    float out[H2];
    if (mode == kRotation) {
      const float xn = sqrtf(xs), en = sqrtf(e2);
      const float xd = xn + 1e-8f, ed = en + 1e-8f;
      const float rx = 1.0f / xd, re = 1.0f / ed;
      float mnx = INFINITY, mxx = 0.f, mne = INFINITY, mxe = 0.f;
#pragma unroll
      for (int k = 0; k < H2; ++k) {
        mnx = fminf(mnx, fabsf(xv[k])); mxx = fmaxf(mxx, fabsf(xv[k]));
        mne = fminf(mne, fabsf(ev[k])); mxe = fmaxf(mxe, fabsf(ev[k]));
      }
      const bool fast = div_rn_ok(mnx, mxx, xd) && div_rn_ok(mne, mxe, ed);
      float u[H2], q[H2];
      float s2 = 0.f, eu = 0.f, mns = INFINITY, mxs = 0.f;
#pragma unroll
      for (int k = 0; k < H2; ++k) {
        u[k] = fast ? div_rn(xv[k], xd, rx) : xv[k] / xd;
        q[k] = fast ? div_rn(ev[k], ed, re) : ev[k] / ed;
        const float sk = u[k] + q[k];
        out[k] = sk;   // holds u+q until normalised
        s2 = __builtin_fmaf(sk, sk, s2);
        eu = __builtin_fmaf(xv[k], u[k], eu);
        mns = fminf(mns, fabsf(sk)); mxs = fmaxf(mxs, fabsf(sk));
      }
      s2 += __shfl_xor(s2, 32, 64);
      eu += __shfl_xor(eu, 32, 64);
      const float sn = fmaxf(sqrtf(s2), 1e-6f), rs = 1.0f / sn;
      const bool fast_w = div_rn_ok(mns, mxs, sn);
      float ew = 0.f;
#pragma unroll
      for (int k = 0; k < H2; ++k) {
        out[k] = fast_w ? div_rn(out[k], sn, rs) : out[k] / sn;   // w
        ew = __builtin_fmaf(xv[k], out[k], ew);
      }
      ew += __shfl_xor(ew, 32, 64);
      const float lam = en / (xn + 1e-6f);
      const float m2ew = -2.f * ew, p2eu = 2.f * eu;
      // (x - 2 (x.w) w + 2 (x.u) q) * lam   (quantize.py:41-45,140-142)
#pragma unroll
      for (int k = 0; k < H2; ++k) out[k] = __builtin_fmaf(p2eu, q[k], __builtin_fmaf(m2ew, out[k], xv[k])) * lam;
    } else if (mode == kSte) {
#pragma unroll
      for (int k = 0; k < H2; ++k) out[k] = xv[k] + (ev[k] - xv[k]);
    } else {
#pragma unroll
      for (int k = 0; k < H2; ++k) out[k] = ev[k];
    }
    ql = ql + (dl + beta * dl);
    if (writer && h == 0) ids[(int64_t)b * L + l] = id;
#pragma unroll
    for (int k = 0; k < H2; ++k) {
      pend_e[k] = out[k];
      es[k] = es[k] + out[k];
      xv[k] = xv[k] - out[k];   // next level's residual stays in registers
    }
  }
  if (writer) {
#pragma unroll
    for (int k = 0; k < H2; k += 4)
      *reinterpret_cast<float4*>(emb_out + (int64_t)(L - 1) * BD + o + k) =
          make_float4(pend_e[k], pend_e[k + 1], pend_e[k + 2], pend_e[k + 3]);
    if (h == 0) qloss[b] = ql;
    if (emb_sum != nullptr) {
#pragma unroll
      for (int k = 0; k < H2; k += 4)
        *reinterpret_cast<float4*>(emb_sum + o + k) = make_float4(es[k], es[k + 1], es[k + 2], es[k + 3]);
    }
  }
}

// ---------------------------------------------------------------------------------------
// D = 64, whole level codebook resident in LDS, large B: the register kernel rebuilt on
// v_mfma_f32_16x16x4_f32 with 16 items per wave. Lane (j = lane & 15, g = lane >> 4) holds item
// j's 16 columns {16q + 4g + i : q, i < 4}, which is its B-operand fragment for k-step (q, i)
// (lane group g supplies k = g; the same k permutation on both operands). Each 16-row tile's
// distances land 4 per lane (codewords t0 + 4g + r of item j); the four lane groups merge with
// two xor shuffles at the end of the level. Compared with the 32x32x2 kernel this halves the
// per-lane row state (16 floats), so the kernel fits 4 waves per SIMD (8-wave workgroups sharing
// one 64 KiB LDS-DMA-filled codebook image, two per CU) and two independent accumulator chains
// per wave cover the 16x16x4 dependent-issue latency. The codebook image is XOR-swizzled by
// (row & 15): with the (q, g) column order the 16 rows of a ds_read_b128 lane group hit 16
// distinct 4-bank groups.
constexpr int kR16Items = 128;   // items per 8-wave workgroup

__global__ void __launch_bounds__(512, 2)
rq_fwd_r16_kernel(const float* __restrict__ x, int B, const float* __restrict__ cbs, const float* __restrict__ csq,
                  int K, int L, int mode, float beta, int64_t* __restrict__ ids, float* __restrict__ emb_out,
                  float* __restrict__ res, float* __restrict__ qloss, float* __restrict__ emb_sum,
                  float* __restrict__ enorm) {
  constexpr int D = 64, QD = 16;
  extern __shared__ __attribute__((aligned(16))) float dsm[];
  const int KP = (K + 31) & ~31;                     // rows padded to whole tile pairs
  float* A_s = dsm;                                  // [KP][64] swizzled codeword image
  float* cs_s = dsm + KP * D;                        // [KP] |c|^2 (+inf past K)
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int j = lane & 15, g = lane >> 4;
  const int b = blockIdx.x * kR16Items + wave * 16 + j;
  const bool valid = b < B;
  const int64_t BD = (int64_t)B * D;
  const int64_t ob = (int64_t)(valid ? b : 0) * D + 4 * g;   // + 16 q for column block q
  float xv[QD], es[QD], pend[QD];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 v = valid ? *reinterpret_cast<const float4*>(x + ob + 16 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
    xv[4 * q] = v.x; xv[4 * q + 1] = v.y; xv[4 * q + 2] = v.z; xv[4 * q + 3] = v.w;
  }
#pragma unroll
  for (int k = 0; k < QD; ++k) es[k] = 0.f;
  float ql = 0.f;
  auto store_row = [&](float* dst, const float (&v)[QD]) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      *reinterpret_cast<float4*>(dst + ob + 16 * q) = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
  };
  auto rsum = [](float v) {   // sum over the item's four lane groups
    v += __shfl_xor(v, 16, 64);
    return v + __shfl_xor(v, 32, 64);
  };

  for (int l = 0; l < L; ++l) {
    const float* cb = cbs + (int64_t)l * K * D;
    float xs = 0.f;
#pragma unroll
    for (int k = 0; k < QD; ++k) xs = __builtin_fmaf(xv[k], xv[k], xs);
    xs = rsum(xs);
    __syncthreads();   // previous level's image fully consumed (incl. epilogue codeword reads)
    // LDS-DMA: wave-instruction q moves rows 4q..4q+3 (1 KiB); lane i lands at chunk i%16 of row
    // 4q + i/16, i.e. loads logical chunk (i%16) ^ (row & 15) of that row (rows past K clamp)
    for (int q = wave; q < KP / 4; q += 8) {
      const int row = 4 * q + (lane >> 4);
      const int c = (lane & 15) ^ (row & 15);
      __builtin_amdgcn_global_load_lds(cb + (int64_t)min(row, K - 1) * D + 4 * c, A_s + q * 256, 16, 0, 0);
    }
    for (int r = tid; r < KP; r += 512) cs_s[r] = r < K ? csq[(int64_t)l * K + r] : INFINITY;
    __syncthreads();
    if (valid && g < 4 && l > 0) {   // deferred stores of the previous level (drain under the MFMAs)
      store_row(res + (int64_t)l * BD, xv);
      store_row(emb_out + (int64_t)(l - 1) * BD, pend);
    } else if (valid && l == 0) {
      store_row(res, xv);
    }
    float best_d = INFINITY;
    int best_i = 0;
    // dist = fma(-2, x.c, |x|^2 + |c|^2): 2 x.c is exact, so this is the reference expression's
    // rounding; the tile's best (d, r) is merged once per tile, tiles in increasing order
    auto scan = [&](const floatx4v& a, const float4& c, int t0) {
      const float cr[4] = {c.x, c.y, c.z, c.w};
      float td = INFINITY;
      int tr = 0;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float d = __builtin_fmaf(-2.f, a[r], xs + cr[r]);
        const bool lt = d < td;
        td = lt ? d : td;
        tr = lt ? r : tr;
      }
      const bool lt = td < best_d;
      best_d = lt ? td : best_d;
      best_i = lt ? t0 + 4 * g + tr : best_i;
    };
    for (int t0 = 0; t0 < KP; t0 += 32) {
      floatx4v acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      const int r0 = t0 + j, r1 = t0 + 16 + j;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = 4 * q + g;
        const float4 a0 = *reinterpret_cast<const float4*>(A_s + r0 * D + 4 * (c ^ (r0 & 15)));
        const float4 a1 = *reinterpret_cast<const float4*>(A_s + r1 * D + 4 * (c ^ (r1 & 15)));
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, xv[4 * q], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.x, xv[4 * q], acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, xv[4 * q + 1], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.y, xv[4 * q + 1], acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.z, xv[4 * q + 2], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.z, xv[4 * q + 2], acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.w, xv[4 * q + 3], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.w, xv[4 * q + 3], acc1, 0, 0, 0);
      }
      const float4 c0 = *reinterpret_cast<const float4*>(cs_s + t0 + 4 * g);
      const float4 c1 = *reinterpret_cast<const float4*>(cs_s + t0 + 16 + 4 * g);
      scan(acc0, c0, t0);
      scan(acc1, c1, t0 + 16);
    }
#pragma unroll
    for (int s = 16; s <= 32; s <<= 1) {   // merge the four lane groups (lowest index on ties)
      const float od = __shfl_xor(best_d, s, 64);
      const int oi = __shfl_xor(best_i, s, 64);
      if (od < best_d || (od == best_d && oi < best_i)) { best_d = od; best_i = oi; }
    }
    const int id = best_i;
    float ev[QD];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 c = *reinterpret_cast<const float4*>(A_s + id * D + 4 * ((4 * q + g) ^ (id & 15)));
      ev[4 * q] = c.x; ev[4 * q + 1] = c.y; ev[4 * q + 2] = c.z; ev[4 * q + 3] = c.w;
    }
    float e2 = 0.f, dl = 0.f;
#pragma unroll
    for (int k = 0; k < QD; ++k) {
      e2 = __builtin_fmaf(ev[k], ev[k], e2);
      const float t = xv[k] - ev[k];
      dl = __builtin_fmaf(t, t, dl);
    }
    e2 = rsum(e2);
    dl = rsum(dl);
    float out[QD];
    if (mode == kRotation) {
      const float xn = sqrtf(xs), en = sqrtf(e2);
      const float xd = xn + 1e-8f, ed = en + 1e-8f;
      const float rx = 1.0f / xd, re = 1.0f / ed;
      float mnx = INFINITY, mxx = 0.f, mne = INFINITY, mxe = 0.f;
#pragma unroll
      for (int k = 0; k < QD; ++k) {
        mnx = fminf(mnx, fabsf(xv[k])); mxx = fmaxf(mxx, fabsf(xv[k]));
        mne = fminf(mne, fabsf(ev[k])); mxe = fmaxf(mxe, fabsf(ev[k]));
      }
      // per-lane choice: either branch yields the correctly rounded quotient
      const bool fast = div_rn_ok(mnx, mxx, xd) && div_rn_ok(mne, mxe, ed);
      float u[QD], qv[QD];
      float s2 = 0.f, eu = 0.f, mns = INFINITY, mxs = 0.f;
#pragma unroll
      for (int k = 0; k < QD; ++k) {
        u[k] = fast ? div_rn(xv[k], xd, rx) : xv[k] / xd;
        qv[k] = fast ? div_rn(ev[k], ed, re) : ev[k] / ed;
        const float sk = u[k] + qv[k];
        out[k] = sk;
        s2 = __builtin_fmaf(sk, sk, s2);
        eu = __builtin_fmaf(xv[k], u[k], eu);
        mns = fminf(mns, fabsf(sk)); mxs = fmaxf(mxs, fabsf(sk));
      }
      s2 = rsum(s2);
      eu = rsum(eu);
      const float sn = fmaxf(sqrtf(s2), 1e-6f), rs = 1.0f / sn;
      const bool fast_w = div_rn_ok(mns, mxs, sn);
      float ew = 0.f;
#pragma unroll
      for (int k = 0; k < QD; ++k) {
        out[k] = fast_w ? div_rn(out[k], sn, rs) : out[k] / sn;   // w
        ew = __builtin_fmaf(xv[k], out[k], ew);
      }
      ew = rsum(ew);
      const float lam = en / (xn + 1e-6f);
      const float m2ew = -2.f * ew, p2eu = 2.f * eu;
      // (x - 2 (x.w) w + 2 (x.u) q) * lam   (quantize.py:41-45,140-142)
#pragma unroll
      for (int k = 0; k < QD; ++k) out[k] = __builtin_fmaf(p2eu, qv[k], __builtin_fmaf(m2ew, out[k], xv[k])) * lam;
    } else if (mode == kSte) {
#pragma unroll
      for (int k = 0; k < QD; ++k) out[k] = xv[k] + (ev[k] - xv[k]);
    } else {
#pragma unroll
      for (int k = 0; k < QD; ++k) out[k] = ev[k];
    }
    ql = ql + (dl + beta * dl);
    if (valid && g == 0) ids[(int64_t)b * L + l] = id;
    if (enorm != nullptr) {   // |emb_out[l][b]| (RqVae.forward's embs_norm, modules/rqvae.py:151)
      float n2 = 0.f;
#pragma unroll
      for (int k = 0; k < QD; ++k) n2 = __builtin_fmaf(out[k], out[k], n2);
      n2 = rsum(n2);
      if (valid && g == 0) enorm[(int64_t)l * B + b] = sqrtf(n2);
    }
#pragma unroll
    for (int k = 0; k < QD; ++k) {
      pend[k] = out[k];
      es[k] = es[k] + out[k];
      xv[k] = xv[k] - out[k];   // next level's residual stays in registers
    }
  }
  if (valid) {
    store_row(emb_out + (int64_t)(L - 1) * BD, pend);
    if (g == 0) qloss[b] = ql;
    if (emb_sum != nullptr) store_row(emb_sum, es);
  }
}

static int launch_fwd_r16(int B, hipStream_t s, const float* x, const float* cbs, const float* csq, int K, int L,
                          int mode, float beta, int64_t* ids, float* eo, float* res, float* ql, float* es,
                          float* enorm) {
  const int KP = (K + 31) & ~31;
  const size_t lds = (size_t)KP * (64 + 1) * sizeof(float);
  hipLaunchKernelGGL(rq_fwd_r16_kernel, dim3((B + kR16Items - 1) / kR16Items), dim3(512), lds, s, x, B, cbs, csq, K, L,
                     mode, beta, ids, eo, res, ql, es, enorm);
  return 0;
}

template <int D, int WPI>
static void launch_fwd_reg_w(int B, hipStream_t s, const float* x, const float* cbs, const float* csq, int K, int L,
                             int mode, float beta, int64_t* ids, float* eo, float* res, float* ql, float* es) {
  constexpr int LD = D + 4;
  constexpr int kMaxLds = 75 * 1024;              // two workgroups per CU
  const int fit = (kMaxLds - 1024) / ((LD + 1) * 4);
  const bool resident = (K + 31) / 32 * 32 <= fit;
  const int NB = resident ? K : (fit / 32) * 32;
  const int LDk = (resident && D == 64) ? D : LD;   // swizzled unpadded image (kernel's SWZ)
  // rows / |c|^2 entries up to the next multiple of 32 are read (|c|^2 = +inf) by the last tile
  const size_t lds = (size_t)((NB + 31) / 32 * 32) * (LDk + 1) * sizeof(float) + 1024;
  dim3 g((B + 128 / WPI - 1) / (128 / WPI));
  if (resident)
    hipLaunchKernelGGL((rq_fwd_reg_kernel<D, true, WPI>), g, dim3(256), lds, s, x, B, cbs, csq, K, L, mode, beta, NB,
                       ids, eo, res, ql, es);
  else
    hipLaunchKernelGGL((rq_fwd_reg_kernel<D, false, WPI>), g, dim3(256), lds, s, x, B, cbs, csq, K, L, mode, beta, NB,
                       ids, eo, res, ql, es);
}

template <int D>
static void launch_fwd_reg(int B, hipStream_t s, const float* x, const float* cbs, const float* csq, int K, int L,
                           int mode, float beta, int64_t* ids, float* eo, float* res, float* ql, float* es) {
  // fewer 128-item workgroups than CUs: let 2 or 4 waves split each 32-item tile's codewords
  if (B <= 256 * 32)
    launch_fwd_reg_w<D, 4>(B, s, x, cbs, csq, K, L, mode, beta, ids, eo, res, ql, es);
  else if (B <= 256 * 128)
    launch_fwd_reg_w<D, 2>(B, s, x, cbs, csq, K, L, mode, beta, ids, eo, res, ql, es);
  else
    launch_fwd_reg_w<D, 1>(B, s, x, cbs, csq, K, L, mode, beta, ids, eo, res, ql, es);
}

// ---------------------------------------------------------------------------------------
// Split path for large D / K (D >= 128, e.g. the synthetic roofline shape D=1024, K=2048, L=4).
// The fused kernel above gives one workgroup per 128 items, so B=16,384 leaves half the CUs
// idle and every workgroup walks all K codewords alone. Here each level runs as
//   rq_dist_argmin_kernel  one workgroup per (128-item tile, 128-codeword block): the distance
//                          GEMM on v_mfma_f32_32x32x2_f32 (register-prefetched LDS stages of
//                          32 D-columns, conflict-free ds_read_b128) with the argmin over its
//                          block fused into the epilogue -> one (dist, index) partial per item
//   rq_level_epi_kernel    LPI lanes per item: merge the partials (lowest index among equal
//                          minima, as torch.min), then the same row epilogue as the fused kernel
//                          (rotation trick / STE / eval, VQ loss, next residual and its |r|^2)
// Workgroup order is XCD-major (T1) so the 16 codeword blocks of one item tile share an L2.
// Scratch: level l's (dist, index) partials and its |res_l|^2 live in item b's own emb_out[l]
// row (columns [0, 2*nblk] — needs 2*nblk + 1 <= D) until the epilogue overwrites that row.
constexpr int kSB = 128;           // items per tile
constexpr int kSN = 128;           // codewords per block
constexpr int kSK = 32;            // D columns per LDS stage
constexpr int kSLD = kSK + 4;      // padded LDS row: ds_read_b128 over 32 rows hits 16 distinct 4-bank groups

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3)))
rq_dist_argmin_kernel(const float* __restrict__ res, const float* __restrict__ cb, const float* __restrict__ csq, int B,
                      int D, int K, int nblk, int tilesB, float* __restrict__ scratch) {
  __shared__ __attribute__((aligned(16))) float A_s[kSN * kSLD];   // codeword stage [128][36]
  __shared__ __attribute__((aligned(16))) float X_s[kSB * kSLD];   // residual stage [128][36]
  __shared__ float cs_s[kSN];
  __shared__ float xs_s[kSB];
  __shared__ float md_s[kSB];
  __shared__ int mi_s[kSB];
  const int n = tilesB * nblk, o = blockIdx.x, xcd = o & 7, q = n >> 3, rr = n & 7;
  const int w = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (o >> 3);
  const int tb = w / nblk, cbk = w % nblk;
  const int b0 = tb * kSB, n0 = cbk * kSN;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, h = lane >> 5, c32 = lane & 31;
  const int wr = wave >> 1, wc = wave & 1;   // wave block: codewords wr*64.., items wc*64..

  // stage loads: thread t moves rows t/8 + 32j (j < 4), 16 B at column (t%8)*4 of each operand;
  // rows past K / B are clamped (their results are masked later), so no load sits behind a
  // runtime branch. Plain unrolled code (no captured arrays) keeps the staging in VGPRs.
  const int srow = tid >> 3, scol = (tid & 7) * 4;
  const float* ag = cb + (int64_t)min(n0 + srow, K - 1) * D + scol;
  const float* xg = res + (int64_t)min(b0 + srow, B - 1) * D + scol;
  int64_t aoff[4], xoff[4];
#pragma unroll
  for (int j = 1; j < 4; ++j) {
    aoff[j] = (int64_t)(min(n0 + srow + 32 * j, K - 1) - min(n0 + srow, K - 1)) * D;
    xoff[j] = (int64_t)(min(b0 + srow + 32 * j, B - 1) - min(b0 + srow, B - 1)) * D;
  }
  aoff[0] = xoff[0] = 0;
  float* as_w = A_s + srow * kSLD + scol;
  float* xs_w = X_s + srow * kSLD + scol;
  float4 ra0, ra1, ra2, ra3, rx0, rx1, rx2, rx3;
#define RQ_SPLIT_LOAD(k0)                                                        \
  ra0 = *reinterpret_cast<const float4*>(ag + aoff[0] + (k0));                   \
  ra1 = *reinterpret_cast<const float4*>(ag + aoff[1] + (k0));                   \
  ra2 = *reinterpret_cast<const float4*>(ag + aoff[2] + (k0));                   \
  ra3 = *reinterpret_cast<const float4*>(ag + aoff[3] + (k0));                   \
  rx0 = *reinterpret_cast<const float4*>(xg + xoff[0] + (k0));                   \
  rx1 = *reinterpret_cast<const float4*>(xg + xoff[1] + (k0));                   \
  rx2 = *reinterpret_cast<const float4*>(xg + xoff[2] + (k0));                   \
  rx3 = *reinterpret_cast<const float4*>(xg + xoff[3] + (k0));
#define RQ_SPLIT_STASH()                                                         \
  *reinterpret_cast<float4*>(as_w) = ra0;                                        \
  *reinterpret_cast<float4*>(as_w + 32 * kSLD) = ra1;                            \
  *reinterpret_cast<float4*>(as_w + 64 * kSLD) = ra2;                            \
  *reinterpret_cast<float4*>(as_w + 96 * kSLD) = ra3;                            \
  *reinterpret_cast<float4*>(xs_w) = rx0;                                        \
  *reinterpret_cast<float4*>(xs_w + 32 * kSLD) = rx1;                            \
  *reinterpret_cast<float4*>(xs_w + 64 * kSLD) = rx2;                            \
  *reinterpret_cast<float4*>(xs_w + 96 * kSLD) = rx3;

  RQ_SPLIT_LOAD(0)
  if (tid < kSN) cs_s[tid] = csq[min(n0 + tid, K - 1)];
  else xs_s[tid - kSN] = scratch[(int64_t)min(b0 + tid - kSN, B - 1) * D + 2 * nblk];
  RQ_SPLIT_STASH()
  __syncthreads();

  floatx16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][c][r] = 0.f;

  // lane half h supplies physical columns h*16 + s of each stage for logical k = h (same
  // permutation for both operands: the dot products are unchanged)
  const float* ap = A_s + (wr * 64 + c32) * kSLD + h * (kSK / 2);
  const float* bp = X_s + (wc * 64 + c32) * kSLD + h * (kSK / 2);
  for (int k0 = 0; k0 < D; k0 += kSK) {
    {
      const int kn = k0 + kSK < D ? k0 + kSK : k0;   // last stage: a harmless reload, no branch
      RQ_SPLIT_LOAD(kn)                       // in flight under this stage's MFMAs
    }
    __builtin_amdgcn_sched_barrier(0);        // keep the loads ahead of the MFMAs (no sinking)
#pragma unroll
    for (int s4 = 0; s4 < kSK / 2; s4 += 4) {
      const float4 a0 = *reinterpret_cast<const float4*>(ap + s4);
      const float4 a1 = *reinterpret_cast<const float4*>(ap + 32 * kSLD + s4);
      const float4 x0 = *reinterpret_cast<const float4*>(bp + s4);
      const float4 x1 = *reinterpret_cast<const float4*>(bp + 32 * kSLD + s4);
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.x, x0.x, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.x, x1.x, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.x, x0.x, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.x, x1.x, acc[1][1], 0, 0, 0);
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.y, x0.y, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.y, x1.y, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.y, x0.y, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.y, x1.y, acc[1][1], 0, 0, 0);
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.z, x0.z, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.z, x1.z, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.z, x0.z, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.z, x1.z, acc[1][1], 0, 0, 0);
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.w, x0.w, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.w, x1.w, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.w, x0.w, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.w, x1.w, acc[1][1], 0, 0, 0);
    }
    __syncthreads();   // stage consumed
    RQ_SPLIT_STASH()   // unconditional (last stage: a harmless rewrite) so the loads stay above the MFMAs
    __syncthreads();
  }
#undef RQ_SPLIT_LOAD
#undef RQ_SPLIT_STASH

  // dist = (|x|^2 + |c|^2) - 2 x.c (quantize.py:108-112); C/D map: row = codeword, column = item.
  // Each lane scans its codewords in increasing index order (strict '<' keeps the lowest).
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int jl = wc * 64 + c * 32 + c32;
    const float xs = xs_s[jl];
    float bd = INFINITY;
    int bi = 0;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int il = wr * 64 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        float d = (xs + cs_s[il]) - 2.f * acc[a][c][r];
        d = n0 + il < K ? d : INFINITY;
        const bool lt = d < bd;
        bd = lt ? d : bd;
        bi = lt ? n0 + il : bi;
      }
    const float od = __shfl_xor(bd, 32, 64);
    const int oi = __shfl_xor(bi, 32, 64);
    if (od < bd || (od == bd && oi < bi)) { bd = od; bi = oi; }
    if (wr == 1 && h == 0) { md_s[jl] = bd; mi_s[jl] = bi; }
    __syncthreads();
    if (wr == 0 && h == 0) {
      const float od2 = md_s[jl];
      const int oi2 = mi_s[jl];
      if (od2 < bd || (od2 == bd && oi2 < bi)) { bd = od2; bi = oi2; }
      const int b = b0 + jl;
      if (b < B) *reinterpret_cast<float2*>(scratch + (int64_t)b * D + 2 * cbk) = make_float2(bd, __int_as_float(bi));
    }
  }
}

// Level-0 prologue of the split path: residuals[0] = x and |x|^2 into the level-0 scratch slot.
template <int LPI, int EPL>
__global__ void __launch_bounds__(256) rq_split_prep_kernel(const float* __restrict__ x, int B, int D, int nblk,
                                                            float* __restrict__ res0, float* __restrict__ scratch0) {
  constexpr int G = 64 / LPI;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = lane % LPI, grp = lane / LPI;
  const int b = (blockIdx.x * 4 + wave) * G + grp;
  const bool valid = b < B;
  const int64_t o = (int64_t)(valid ? b : B - 1) * D + sub * EPL;
  float xv[EPL];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < EPL; k += 4) {
    const float4 v = *reinterpret_cast<const float4*>(x + o + k);
    xv[k] = v.x; xv[k + 1] = v.y; xv[k + 2] = v.z; xv[k + 3] = v.w;
  }
#pragma unroll
  for (int k = 0; k < EPL; ++k) s += xv[k] * xv[k];
  s = group_sum<LPI>(s);
  if (valid) {
#pragma unroll
    for (int k = 0; k < EPL; k += 4)
      *reinterpret_cast<float4*>(res0 + o + k) = make_float4(xv[k], xv[k + 1], xv[k + 2], xv[k + 3]);
    if (sub == 0) scratch0[(int64_t)b * D + 2 * nblk] = s;
  }
}

// Level-l epilogue of the split path (same row math as rq_fwd_kernel's epilogue).
template <int LPI, int EPL>
__global__ void __launch_bounds__(256) rq_level_epi_kernel(const float* __restrict__ res_l, const float* __restrict__ cb,
                                                           int B, int D, int L, int l, int nblk, int mode, float beta,
                                                           int64_t* __restrict__ ids, float* __restrict__ emb_out,
                                                           float* __restrict__ res_next, float* __restrict__ qloss,
                                                           float* __restrict__ emb_sum) {
  constexpr int G = 64 / LPI;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = lane % LPI, grp = lane / LPI;
  const int b = (blockIdx.x * 4 + wave) * G + grp;
  const bool valid = b < B;
  const int64_t BD = (int64_t)B * D;
  const int64_t o = (int64_t)(valid ? b : B - 1) * D + sub * EPL;
  float* eo = emb_out + (int64_t)l * BD;
  // merge the per-block partials of this item (read before the row is overwritten below)
  float bd = INFINITY;
  int bi = 0;
  for (int p = sub; p < nblk; p += LPI) {
    const float2 v = *reinterpret_cast<const float2*>(eo + (o - sub * EPL) + 2 * p);
    const int vi = __float_as_int(v.y);
    if (v.x < bd || (v.x == bd && vi < bi)) { bd = v.x; bi = vi; }
  }
#pragma unroll
  for (int s = LPI / 2; s >= 1; s >>= 1) {
    const float od = __shfl_xor(bd, s, 64);
    const int oi = __shfl_xor(bi, s, 64);
    if (od < bd || (od == bd && oi < bi)) { bd = od; bi = oi; }
  }
  const int id = bi;
  const float* cr = cb + (int64_t)id * D + sub * EPL;
  float xv[EPL], ev[EPL], out[EPL];
#pragma unroll
  for (int k = 0; k < EPL; k += 4) {
    const float4 a = *reinterpret_cast<const float4*>(res_l + o + k);
    const float4 c = *reinterpret_cast<const float4*>(cr + k);
    xv[k] = a.x; xv[k + 1] = a.y; xv[k + 2] = a.z; xv[k + 3] = a.w;
    ev[k] = c.x; ev[k + 1] = c.y; ev[k + 2] = c.z; ev[k + 3] = c.w;
  }
  float dl = 0.f;
#pragma unroll
  for (int k = 0; k < EPL; ++k) { const float t = xv[k] - ev[k]; dl += t * t; }
  dl = group_sum<LPI>(dl);
  if (mode == kRotation) {
    float x2 = 0.f, e2 = 0.f;
#pragma unroll
    for (int k = 0; k < EPL; ++k) { x2 += xv[k] * xv[k]; e2 += ev[k] * ev[k]; }
    x2 = group_sum<LPI>(x2);
    e2 = group_sum<LPI>(e2);
    RowRot<LPI, EPL> rot;
    rot.build(xv, ev, sqrtf(x2), sqrtf(e2));
    float ew = 0.f, eu = 0.f;
#pragma unroll
    for (int k = 0; k < EPL; ++k) { ew += xv[k] * rot.w[k]; eu += xv[k] * rot.u[k]; }
    ew = group_sum<LPI>(ew);
    eu = group_sum<LPI>(eu);
#pragma unroll
    for (int k = 0; k < EPL; ++k) out[k] = ((xv[k] - 2.f * (ew * rot.w[k])) + 2.f * (eu * rot.q[k])) * rot.lam;
  } else if (mode == kSte) {
#pragma unroll
    for (int k = 0; k < EPL; ++k) out[k] = xv[k] + (ev[k] - xv[k]);
  } else {
#pragma unroll
    for (int k = 0; k < EPL; ++k) out[k] = ev[k];
  }
  float r2 = 0.f;
  float nr[EPL];
#pragma unroll
  for (int k = 0; k < EPL; ++k) { nr[k] = xv[k] - out[k]; r2 += nr[k] * nr[k]; }
  r2 = group_sum<LPI>(r2);
  if (!valid) return;
#pragma unroll
  for (int k = 0; k < EPL; k += 4) {
    *reinterpret_cast<float4*>(eo + o + k) = make_float4(out[k], out[k + 1], out[k + 2], out[k + 3]);
    if (res_next != nullptr)
      *reinterpret_cast<float4*>(res_next + o + k) = make_float4(nr[k], nr[k + 1], nr[k + 2], nr[k + 3]);
  }
  if (emb_sum != nullptr && l == L - 1) {
#pragma unroll
    for (int k = 0; k < EPL; k += 4) {
      float4 s = *reinterpret_cast<const float4*>(emb_out + o + k);
      for (int m = 1; m < L; ++m) {
        const float4 v = (m == l) ? make_float4(out[k], out[k + 1], out[k + 2], out[k + 3])
                                  : *reinterpret_cast<const float4*>(emb_out + (int64_t)m * BD + o + k);
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
      }
      if (L == 1) s = make_float4(out[k], out[k + 1], out[k + 2], out[k + 3]);
      *reinterpret_cast<float4*>(emb_sum + o + k) = s;
    }
  }
  if (sub == 0) {
    ids[(int64_t)b * L + l] = id;
    const float lq = dl + beta * dl;
    qloss[b] = l == 0 ? 0.f + lq : qloss[b] + lq;
    if (l + 1 < L) emb_out[(int64_t)(l + 1) * BD + (int64_t)b * D + 2 * nblk] = r2;   // next level's |res|^2
  }
}

template <int LPI, int EPL>
static void launch_split(int B, hipStream_t s, const float* x, int D, const float* cbs, const float* csq, int K, int L,
                         int mode, float beta, int64_t* ids, float* eo, float* res, float* ql, float* es) {
  constexpr int G = 64 / LPI;
  const int nblk = (K + kSN - 1) / kSN, tilesB = (B + kSB - 1) / kSB;
  const int64_t BD = (int64_t)B * D;
  const dim3 gr((B + 4 * G - 1) / (4 * G));
  hipLaunchKernelGGL((rq_split_prep_kernel<LPI, EPL>), gr, dim3(256), 0, s, x, B, D, nblk, res, eo);
  for (int l = 0; l < L; ++l) {
    hipLaunchKernelGGL(rq_dist_argmin_kernel, dim3(tilesB * nblk), dim3(256), 0, s, res + l * BD, cbs + (int64_t)l * K * D,
                       csq + (int64_t)l * K, B, D, K, nblk, tilesB, eo + l * BD);
    hipLaunchKernelGGL((rq_level_epi_kernel<LPI, EPL>), gr, dim3(256), 0, s, res + l * BD, cbs + (int64_t)l * K * D, B,
                       D, L, l, nblk, mode, beta, ids, eo, l + 1 < L ? res + (l + 1) * BD : nullptr, ql, es);
  }
}

__global__ void __launch_bounds__(256) segment_counts_kernel(const int* __restrict__ key_off, int K,
                                                             int64_t* __restrict__ counts) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k < K) counts[k] = key_off[k + 1] - key_off[k];
}

// ---------------------------------------------------------------------------------------
static bool row_split(int D, int& lpi, int& epl) {
  if (D < 8 || D > 1024 || (D & (D - 1)) != 0) return false;
  lpi = D / 4 < 64 ? D / 4 : 64;
  epl = D / lpi;
  return true;
}

template <int BK, int LPI, int EPL>
static void launch_fwd(dim3 g, hipStream_t s, const float* x, int B, int D, const float* cbs, const float* csq, int K,
                       int L, int mode, float beta, int64_t* ids, float* eo, float* res, float* ql, float* es) {
  hipLaunchKernelGGL((rq_fwd_kernel<BK, LPI, EPL>), g, dim3(256), 0, s, x, B, D, cbs, csq, K, L, mode, beta, ids, eo,
                     res, ql, es);
}

template <int LPI, int EPL>
static void launch_bwd(int B, hipStream_t s, const float* res, const int64_t* ids, const float* cbs, int D, int K,
                       int L, int mode, float beta, const float* ge, const float* ges, const float* gr, const float* gq,
                       float* gx, float* contrib) {
  constexpr int G = 64 / LPI;
  dim3 g((B + 4 * G - 1) / (4 * G));
  hipLaunchKernelGGL((rq_bwd_rows_kernel<LPI, EPL>), g, dim3(256), 0, s, res, ids, cbs, B, D, K, L, mode, beta, ge, ges,
                     gr, gq, gx, contrib);
}

}  // namespace rqhip

using namespace rqhip;

extern "C" {

int rq_codebook_sqnorm(const float* rows, int64_t n, int64_t D, float* out, void* stream) {
  RQ_CHECK_ARG(rows && out && n >= 0 && D > 0, "rq_codebook_sqnorm: bad arguments");
  if (n == 0) return 0;
  hipLaunchKernelGGL(rq_sqnorm_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, (hipStream_t)stream, rows, n,
                     (int)D, out);
  RQ_LAUNCH_CHECK("rq_codebook_sqnorm");
  return 0;
}

static int quantize_fwd(const float* x, int64_t B, int64_t D, const float* codebooks, const float* cb_sqnorm,
                        int64_t K, int64_t L, int mode, float beta, int64_t* ids, float* emb_out, float* residuals,
                        float* qloss, float* emb_sum, int impl, float* emb_norms, void* stream);

int rq_quantize_fwd(const float* x, int64_t B, int64_t D, const float* codebooks, const float* cb_sqnorm, int64_t K,
                    int64_t L, int mode, float beta, int64_t* ids, float* emb_out, float* residuals, float* qloss,
                    float* emb_sum, float* emb_norms, int impl, void* stream) {
  return quantize_fwd(x, B, D, codebooks, cb_sqnorm, K, L, mode, beta, ids, emb_out, residuals, qloss, emb_sum, impl,
                      emb_norms, stream);
}

static int quantize_fwd(const float* x, int64_t B, int64_t D, const float* codebooks, const float* cb_sqnorm,
                        int64_t K, int64_t L, int mode, float beta, int64_t* ids, float* emb_out, float* residuals,
                        float* qloss, float* emb_sum, int impl, float* emb_norms, void* stream) {
  int lpi, epl;
  RQ_CHECK_ARG(codebooks && cb_sqnorm && (B == 0 || (x && ids && emb_out && residuals && qloss)),
               "rq_quantize_fwd: null pointer");   // an empty batch may come as NULL buffers
  RQ_CHECK_ARG(row_split((int)D, lpi, epl), "rq_quantize_fwd: D=%lld must be a power of two in [8, 1024]", (long long)D);
  RQ_CHECK_ARG(K >= 1 && K <= (1 << 20) && L >= 1 && L <= 64, "rq_quantize_fwd: bad K=%lld / L=%lld", (long long)K,
               (long long)L);
  RQ_CHECK_ARG(B >= 0 && B < (1ll << 31) && B * D < (1ll << 40), "rq_quantize_fwd: bad B=%lld", (long long)B);
  RQ_CHECK_ARG(mode == kEval || mode == kSte || mode == kRotation, "rq_quantize_fwd: mode %d has no fused kernel", mode);
  if (B == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  dim3 g((unsigned)((B + kTB - 1) / kTB));
  const int b = (int)B, d = (int)D, k = (int)K, l = (int)L;
  RQ_CHECK_ARG(impl >= 0 && impl <= 4,
               "rq_quantize_fwd: impl must be 0 (auto), 1 (tiled), 2 (register), 3 (split) or 4 (register 16x16)");
  const bool split_ok = D >= 128 && 2 * ((K + kSN - 1) / kSN) + 1 <= D;
  const bool r16_ok = D == 64 && K <= 288;   // two 65 * K * 4-byte images per CU
  if (impl == 0) impl = (r16_ok && B >= 32768) ? 4 : D <= 64 ? 2 : (split_ok ? 3 : 1);
  RQ_CHECK_ARG(impl != 4 || r16_ok, "rq_quantize_fwd: 16x16 register kernel needs D == 64 and K <= 288");
  if (emb_norms != nullptr && impl != 4) {   // only the 16x16 kernel fuses the norms: one extra row pass otherwise
    const int rc = quantize_fwd(x, B, D, codebooks, cb_sqnorm, K, L, mode, beta, ids, emb_out, residuals, qloss,
                                emb_sum, impl, nullptr, stream);
    return rc != 0 ? rc : rq_row_norms(emb_out, L * B, D, emb_norms, stream);
  }
  if (impl == 4) {
    launch_fwd_r16(b, s, x, codebooks, cb_sqnorm, k, l, mode, beta, ids, emb_out, residuals, qloss, emb_sum, emb_norms);
    RQ_LAUNCH_CHECK("rq_quantize_fwd(register 16x16)");
    return 0;
  }
  RQ_CHECK_ARG(impl != 2 || D <= 64, "rq_quantize_fwd_impl: register kernel needs D <= 64");
  RQ_CHECK_ARG(impl != 3 || split_ok, "rq_quantize_fwd_impl: split path needs D >= 128 and 2*ceil(K/128)+1 <= D");
  if (impl == 3) {
    switch (D) {
#define RQ_SPLIT_CASE(DD, LPI, EPL) \
  case DD: launch_split<LPI, EPL>(b, s, x, d, codebooks, cb_sqnorm, k, l, mode, beta, ids, emb_out, residuals, qloss, emb_sum); break;
      RQ_SPLIT_CASE(128, 32, 4)
      RQ_SPLIT_CASE(256, 64, 4)
      RQ_SPLIT_CASE(512, 64, 8)
      RQ_SPLIT_CASE(1024, 64, 16)
#undef RQ_SPLIT_CASE
    }
    RQ_LAUNCH_CHECK("rq_quantize_fwd(split)");
    return 0;
  }
  if (impl == 2) {
    switch (D) {
      case 8: launch_fwd_reg<8>(b, s, x, codebooks, cb_sqnorm, k, l, mode, beta, ids, emb_out, residuals, qloss, emb_sum); break;
      case 16: launch_fwd_reg<16>(b, s, x, codebooks, cb_sqnorm, k, l, mode, beta, ids, emb_out, residuals, qloss, emb_sum); break;
      case 32: launch_fwd_reg<32>(b, s, x, codebooks, cb_sqnorm, k, l, mode, beta, ids, emb_out, residuals, qloss, emb_sum); break;
      case 64: launch_fwd_reg<64>(b, s, x, codebooks, cb_sqnorm, k, l, mode, beta, ids, emb_out, residuals, qloss, emb_sum); break;
    }
    RQ_LAUNCH_CHECK("rq_quantize_fwd(register)");
    return 0;
  }
  switch (D) {
#define RQ_FWD_CASE(DD, BK, LPI, EPL) \
  case DD: launch_fwd<BK, LPI, EPL>(g, s, x, b, d, codebooks, cb_sqnorm, k, l, mode, beta, ids, emb_out, residuals, qloss, emb_sum); break;
    RQ_FWD_CASE(8, 8, 2, 4)
    RQ_FWD_CASE(16, 16, 4, 4)
    RQ_FWD_CASE(32, 32, 8, 4)
    RQ_FWD_CASE(64, 64, 16, 4)
    RQ_FWD_CASE(128, 64, 32, 4)
    RQ_FWD_CASE(256, 64, 64, 4)
    RQ_FWD_CASE(512, 64, 64, 8)
    RQ_FWD_CASE(1024, 64, 64, 16)
#undef RQ_FWD_CASE
    default: RQ_CHECK_ARG(false, "rq_quantize_fwd: unsupported D");
  }
  RQ_LAUNCH_CHECK("rq_quantize_fwd");
  return 0;
}

size_t rq_quantize_bwd_workspace(int64_t B, int64_t D, int64_t K, int64_t L) {
  const int64_t nblk = (B + kSortRows - 1) / kSortRows;
  size_t bytes = 0;
  // the chunk path's partial images (every mode but eval; the sort path's buffers below cover the rest)
  const size_t chunk_bytes = (size_t)(L * cb_chunks(B) * K * D) * sizeof(float) + 256;
  bytes += (size_t)(L * B * D) * sizeof(float);          // contrib
  bytes += (size_t)(L * K * nblk) * sizeof(int);         // hist / scanned positions
  bytes += (size_t)(L * (K + 1)) * sizeof(int);          // key offsets
  bytes += (size_t)(L * B) * sizeof(int);                // perm
  bytes += (size_t)(kSegSplit * L * K * D) * sizeof(float);   // heavy-segment partials
  return std::max(bytes + 256, chunk_bytes);
}

int rq_quantize_bwd(const float* residuals, const int64_t* ids, const float* codebooks, int64_t B, int64_t D, int64_t K,
                    int64_t L, int mode, float beta, const float* g_emb, const float* g_emb_sum, const float* g_res,
                    const float* g_qloss, float* grad_x, float* grad_codebooks, void* workspace, size_t ws_bytes,
                    void* stream) {
  int lpi, epl;
  RQ_CHECK_ARG(residuals && ids && codebooks && grad_x && grad_codebooks, "rq_quantize_bwd: null pointer");
  RQ_CHECK_ARG(row_split((int)D, lpi, epl), "rq_quantize_bwd: D=%lld must be a power of two in [8, 1024]", (long long)D);
  RQ_CHECK_ARG(K >= 1 && K <= 4096 && L >= 1 && L <= 64, "rq_quantize_bwd: bad K/L");
  RQ_CHECK_ARG(mode == kEval || mode == kSte || mode == kRotation, "rq_quantize_bwd: bad mode %d", mode);
  RQ_CHECK_ARG(B >= 0 && B < (1ll << 31), "rq_quantize_bwd: bad B");
  RQ_CHECK_ARG(workspace && ws_bytes >= rq_quantize_bwd_workspace(B, D, K, L), "rq_quantize_bwd: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int b = (int)B, d = (int)D, k = (int)K, l = (int)L;
  const int nblk = (b + kSortRows - 1) / kSortRows;
  char* w = (char*)workspace;
  float* contrib = (float*)w; w += (size_t)(L * B * D) * sizeof(float);
  int* hist = (int*)w;        w += (size_t)(L * K * nblk) * sizeof(int);
  int* key_off = (int*)w;     w += (size_t)(L * (K + 1)) * sizeof(int);
  int* perm = (int*)w;        w += (size_t)(L * B) * sizeof(int);
  float* segs = (float*)(((uintptr_t)w + 15) & ~(uintptr_t)15);
  if (B == 0) {
    RQ_HIP(zero_async(grad_codebooks, (size_t)(L * K * D) * sizeof(float), s));
    return 0;
  }
  switch (D) {
#define RQ_BWD_CASE(DD, LPI, EPL) \
  case DD: launch_bwd<LPI, EPL>(b, s, residuals, ids, codebooks, d, k, l, mode, beta, g_emb, g_emb_sum, g_res, g_qloss, grad_x, mode == kEval ? contrib : nullptr); break;
    RQ_BWD_CASE(8, 2, 4)
    RQ_BWD_CASE(16, 4, 4)
    RQ_BWD_CASE(32, 8, 4)
    RQ_BWD_CASE(64, 16, 4)
    RQ_BWD_CASE(128, 32, 4)
    RQ_BWD_CASE(256, 64, 4)
    RQ_BWD_CASE(512, 64, 8)
    RQ_BWD_CASE(1024, 64, 16)
#undef RQ_BWD_CASE
    default: RQ_CHECK_ARG(false, "rq_quantize_bwd: unsupported D");
  }
  RQ_LAUNCH_CHECK("rq_bwd_rows");
  if (RQ_CB_CHUNK && cb_chunk_path(B, D, K, mode, g_qloss)) {
    float* partial = (float*)(((uintptr_t)workspace + 15) & ~(uintptr_t)15);
    const int nchunk = (int)cb_chunks(B);
    const size_t lds = (size_t)K * D * sizeof(float) + kCbRows * sizeof(int) + kCbWaves * kCbList * sizeof(unsigned short);
    switch (D) {
      case 64: hipLaunchKernelGGL(rq_cb_chunk_kernel<1>, dim3(nchunk, l), dim3(64 * kCbWaves), lds, s, residuals, codebooks, g_qloss, ids, b, k, l, partial); break;
      case 128: hipLaunchKernelGGL(rq_cb_chunk_kernel<2>, dim3(nchunk, l), dim3(64 * kCbWaves), lds, s, residuals, codebooks, g_qloss, ids, b, k, l, partial); break;
      default: hipLaunchKernelGGL(rq_cb_chunk_kernel<4>, dim3(nchunk, l), dim3(64 * kCbWaves), lds, s, residuals, codebooks, g_qloss, ids, b, k, l, partial); break;
    }
    const int64_t KD = K * D;
    hipLaunchKernelGGL(rq_cb_chunk_reduce_kernel, dim3((unsigned)((KD / 4 + 255) / 256), l), dim3(256), 0, s, partial,
                       nchunk, KD, grad_codebooks);
    RQ_LAUNCH_CHECK("rq_codebook_grad");
    return 0;
  }
  hipLaunchKernelGGL(sort_hist_kernel, dim3(nblk, l), dim3(256), k * sizeof(int), s, ids, b, l, k, nblk, hist);
  hipLaunchKernelGGL(sort_keyscan_kernel, dim3((k + 15) / 16, l), dim3(256), 0, s, hist, k, nblk, key_off);
  hipLaunchKernelGGL(sort_offsets_kernel, dim3(l), dim3(1024), 0, s, key_off, k, b);
  hipLaunchKernelGGL(sort_scatter_kernel, dim3(nblk, l), dim3(256), (2 * k + kSortRows) * sizeof(int), s, ids, b, l, k,
                     nblk, hist, key_off, perm);
  hipLaunchKernelGGL(rq_cb_segsum_kernel, dim3(k, kSegSplit, l), dim3(256), 0, s, residuals, codebooks, g_qloss,
                     mode == kEval ? contrib : nullptr, perm, key_off, b, d, k, grad_codebooks, segs);
  hipLaunchKernelGGL(rq_segsum_finalize_kernel, dim3(k, l), dim3(256), 0, s, key_off, d, k, segs, grad_codebooks);
  RQ_LAUNCH_CHECK("rq_codebook_grad");
  return 0;
}


// Deterministic segmented sum by key (k-means centroid update, generic scatter-add):
// out[k] = sum of rows[b] over b with keys[b] == k (fixed reduction order), counts[k] = #rows.
size_t rq_segment_sum_workspace(int64_t B, int64_t K) {
  const int64_t nblk = (B + kSortRows - 1) / kSortRows;
  return (size_t)(K * nblk + (K + 1) + B) * sizeof(int) + 256 + (size_t)(kSegSplit * K) * 1024 * sizeof(float);
}

}  // extern "C"

namespace rqhip {
// Pack of several (rows, keys) sources into one: global row i of source t = i - rowbase[t] (t by a scan over
// <= kSegMultiMax bases), key -> -1 (skipped) when outside [0, K_t) or the source's padding index, else
// keybase[t] + key. One thread per float4 of a row; the row's first lane writes the key.
constexpr int kSegMultiMax = 16;
struct SegMultiTable {
  const float* rows[kSegMultiMax];
  const int64_t* keys[kSegMultiMax];
  int64_t rowbase[kSegMultiMax + 1];
  int64_t keybase[kSegMultiMax];
  int64_t K[kSegMultiMax];
  int64_t pad[kSegMultiMax];
  int count;
};
__global__ void __launch_bounds__(256) seg_multi_pack_kernel(SegMultiTable t, int D, float* __restrict__ rows_out,
                                                             int64_t* __restrict__ keys_out) {
  const int F4 = D / 4;
  const int64_t total = t.rowbase[t.count];
  for (int64_t f = (int64_t)blockIdx.x * 256 + threadIdx.x; f < total * F4; f += (int64_t)gridDim.x * 256) {
    const int64_t i = f / F4;
    const int c = (int)(f - i * F4);
    int s = 0;
    while (s + 1 < t.count && i >= t.rowbase[s + 1]) ++s;
    const int64_t r = i - t.rowbase[s];
    reinterpret_cast<float4*>(rows_out + i * D)[c] = reinterpret_cast<const float4*>(t.rows[s] + r * D)[c];
    if (c == 0) {
      const int64_t k = t.keys[s][r];
      keys_out[i] = (k < 0 || k >= t.K[s] || k == t.pad[s]) ? -1 : t.keybase[s] + k;
    }
  }
}
}  // namespace rqhip

extern "C" {

int rq_segment_sum(const float* rows, const int64_t* keys, int64_t B, int64_t D, int64_t K, float* out, int64_t* counts,
                   void* workspace, size_t ws_bytes, void* stream);

size_t rq_segment_sum_multi_workspace(int count, const int64_t* n, const int64_t* K, int64_t D) {
  if (count <= 0 || !n || !K) return 0;
  int64_t rows = 0, keys = 0;
  for (int i = 0; i < count; ++i) {
    rows += n[i];
    keys += K[i];
  }
  return (size_t)rows * (size_t)D * sizeof(float) + (size_t)rows * sizeof(int64_t) + 256 +
         rq_segment_sum_workspace(rows, keys);
}

int rq_segment_sum_multi(int count, const float* const* rows, const int64_t* const* keys, const int64_t* n,
                         const int64_t* K, const int64_t* pad, int64_t D, float* out, void* workspace, size_t ws_bytes,
                         void* stream) {
  RQ_CHECK_ARG(count >= 1 && count <= kSegMultiMax && rows && keys && n && K && pad && out && workspace,
               "rq_segment_sum_multi: 1 <= count <= %d sources, non-null arrays", kSegMultiMax);
  SegMultiTable t;
  t.count = count;
  t.rowbase[0] = 0;
  int64_t kb = 0;
  for (int i = 0; i < count; ++i) {
    RQ_CHECK_ARG(n[i] >= 0 && K[i] >= 1 && (n[i] == 0 || (rows[i] && keys[i])) && (uintptr_t)rows[i] % 16 == 0,
                 "rq_segment_sum_multi: source %d: bad rows / keys / K", i);
    t.rows[i] = rows[i];
    t.keys[i] = keys[i];
    t.rowbase[i + 1] = t.rowbase[i] + n[i];
    t.keybase[i] = kb;
    t.K[i] = K[i];
    t.pad[i] = pad[i];
    kb += K[i];
  }
  const int64_t total = t.rowbase[count];
  RQ_CHECK_ARG(ws_bytes >= rq_segment_sum_multi_workspace(count, n, K, D), "rq_segment_sum_multi: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  float* prow = static_cast<float*>(workspace);
  int64_t* pkey = reinterpret_cast<int64_t*>(prow + total * D);
  char* rest = reinterpret_cast<char*>((((uintptr_t)(pkey + total)) + 255) & ~(uintptr_t)255);
  const size_t used = (size_t)(rest - static_cast<char*>(workspace));
  if (total > 0) {
    const int64_t f4 = total * (D / 4);
    const unsigned grid = (unsigned)std::min<int64_t>((f4 + 255) / 256, 4096);
    hipLaunchKernelGGL(seg_multi_pack_kernel, dim3(grid), dim3(256), 0, s, t, (int)D, prow, pkey);
    RQ_LAUNCH_CHECK("seg_multi_pack_kernel");
  }
  return rq_segment_sum(prow, pkey, total, D, kb, out, nullptr, rest, ws_bytes - used, stream);
}

int rq_segment_sum(const float* rows, const int64_t* keys, int64_t B, int64_t D, int64_t K, float* out, int64_t* counts,
                   void* workspace, size_t ws_bytes, void* stream) {
  RQ_CHECK_ARG(rows && keys && out && workspace, "rq_segment_sum: null pointer");
  RQ_CHECK_ARG(B >= 0 && B < (1ll << 31) && D >= 4 && D <= 1024 && D % 4 == 0 && K >= 1 && K <= 4096,
               "rq_segment_sum: bad shape (need D %% 4 == 0, 4 <= D <= 1024, K <= 4096)");
  RQ_CHECK_ARG(((uintptr_t)rows | (uintptr_t)out) % 16 == 0, "rq_segment_sum: rows / out must be 16-byte aligned");
  RQ_CHECK_ARG(ws_bytes >= rq_segment_sum_workspace(B, K), "rq_segment_sum: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  if (B == 0) {
    RQ_HIP(zero_async(out, (size_t)(K * D) * sizeof(float), s));
    if (counts) RQ_HIP(zero_async(counts, (size_t)K * sizeof(int64_t), s));
    return 0;
  }
  const int b = (int)B, d = (int)D, k = (int)K;
  const int nblk = (b + kSortRows - 1) / kSortRows;
  int* hist = (int*)workspace;
  int* key_off = hist + (size_t)K * nblk;
  int* perm = key_off + (K + 1);
  float* segs = (float*)(((uintptr_t)(perm + B) + 15) & ~(uintptr_t)15);
  hipLaunchKernelGGL(sort_hist_kernel, dim3(nblk, 1), dim3(256), k * sizeof(int), s, keys, b, 1, k, nblk, hist);
  hipLaunchKernelGGL(sort_keyscan_kernel, dim3((k + 15) / 16, 1), dim3(256), 0, s, hist, k, nblk, key_off);
  hipLaunchKernelGGL(sort_offsets_kernel, dim3(1), dim3(1024), 0, s, key_off, k, b);
  hipLaunchKernelGGL(sort_scatter_kernel, dim3(nblk, 1), dim3(256), (2 * k + kSortRows) * sizeof(int), s, keys, b, 1, k,
                     nblk, hist, key_off, perm);
  hipLaunchKernelGGL(rq_cb_segsum_kernel, dim3(k, kSegSplit, 1), dim3(256), 0, s, (const float*)nullptr,
                     (const float*)nullptr, (const float*)nullptr, rows, perm, key_off, b, d, k, out, segs);
  hipLaunchKernelGGL(rq_segsum_finalize_kernel, dim3(k, 1), dim3(256), 0, s, key_off, d, k, segs, out);
  if (counts) hipLaunchKernelGGL(segment_counts_kernel, dim3((k + 255) / 256), dim3(256), 0, s, key_off, k, counts);
  RQ_LAUNCH_CHECK("rq_segment_sum");
  return 0;
}

}  // extern "C"
