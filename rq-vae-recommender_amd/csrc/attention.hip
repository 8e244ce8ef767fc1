// Varlen (jagged) multi-head attention, forward + backward, exact fp32 on v_mfma_f32_16x16x4_f32.
//
// Reference: modules/transformer/attention.py:113-124 (Attend.jagged_forward) —
// F.scaled_dot_product_attention on NJT q/k/v (B, H, j, hd), dropout 0 (:177), scale
// 1/sqrt(hd), is_causal = top-left aligned tril mask. Three call shapes in the model:
// encoder self-attention (non-causal), decoder self-attention (causal) and cross-attention
// (decoder queries x encoder keys, non-causal) — all served by this one kernel family.
//
// Layout: packed token-major rows. q[t][h][d] at q + t*sq + h*HD + d (sq = row stride, so the
// (T, 3A) qkv projection is consumed in place); cu_q / cu_k int64 (B+1) NJT offsets;
// out (Tq, H*HD) rows with stride so; lse (H, Tq) = m + log(l) per query (natural log, saved
// for the backward). Tq / Tk are the ALLOCATED row counts of the q-side / kv-side buffers: rows
// past cu_q[B] / cu_k[B] (a row-bucketed tail) get zero outputs and zero gradients, written by an
// extra grid slice, so no host-side valid row count is needed (graph-capturable).
//
// Tiling (CDNA4, wave64). The unit is a 16 x 16 tile of the 16x16x4 fp32 MFMA, so a ragged
// sequence pads to a multiple of 16 rows (not 32): at the decoder's Amazon contexts
// (4*U{2..20}+1 <= 81 tokens, mean ~45) 73 % of the MFMA work is useful instead of 56 %.
// Each wave owns 16 query rows (forward / dQ) or 16 key rows (dK/dV) for one (sequence, head);
// a workgroup of NW waves shares 32- or 64-row K/V (or Q/dO) chunks staged through LDS (row stride
// HD+4 floats: conflict-free 16-B row reads and 4-B column reads). The wave's own 16 rows stay
// in registers as the MFMA B operand for the whole key (query) loop.
//
// Orientation: score tiles are computed TRANSPOSED in the forward and dQ passes (S^T = K Q^T:
// keys on the accumulator rows, queries on the lanes), so each lane's 4 accumulator registers
// are 4 keys of ONE query and P^T / dS^T feed the next MFMA (O^T += V^T P^T, dQ^T += K^T dS^T)
// straight from the accumulators (key order 4*(lane>>4)+i matches the B operand k index). The
// dK/dV pass computes S = Q K^T (queries on rows, keys on lanes) for the same reason. A query's
// running max needs a 4-lane reduction per staged key chunk (not per tile); its running sum stays
// per lane until the end. exp via v_exp_f32 on log2e-prescaled scores.
// Backward = two launches (dQ per query block, which also stores delta = rowsum(dO*O); then
// dK, dV per key block) with recomputed P: no atomics, bitwise deterministic.
#include "common.h"

#include <math.h>
#include <stdlib.h>

#include <algorithm>

// Build switches (A/B-measured on MI355X, profiles/r02/attn_ab.txt; register prefetch of the next
// staged chunk was measured slower everywhere — +33-64 VGPRs cost more occupancy than the overlap gains —
// and is not built): the number of 16-row tiles whose S / dP chains the backward passes interleave (2: 4 would
// drop the dK/dV pass to one wave per SIMD). The Makefile builds this file with
// -mllvm -amdgpu-mfma-vgpr-form (accumulators in VGPRs: no accvgpr moves around the softmax).
// The few-query / short kernels' per-wave partial tiles (part / part_o [NW][16][HD]) are written by lane
// (row c = lane % 16, columns 16 (lane / 16) + 4 i): with 256-byte rows all 16 rows hit the same banks
// (16-way conflicts on every ds_write_b128: 8-17 conflict cycles per LDS instruction in the Amazon SQ
// pass). 4 floats of row padding put the 16 rows on disjoint 4-bank groups; same values, same order.
#ifndef RQ_ATTN_PART_PAD
#define RQ_ATTN_PART_PAD 1
#endif
constexpr int kPartPad = RQ_ATTN_PART_PAD ? 4 : 0;
#ifndef RQ_ATTN_BWD_GROUP
#define RQ_ATTN_BWD_GROUP 2
#endif

namespace rqhip {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;
// rows of K/V (or Q/dO) staged per LDS round: 64 for 4-wave workgroups, 32 for narrower ones (LDS per
// workgroup 2 x CH x (HD+4) x 4 B: 34.8 KB / 17.4 KB at HD = 64, i.e. 4 / 9 workgroups per CU)
template <int NW>
struct Chunk {
  static constexpr int CH = NW >= 4 ? 64 : 32;
  static constexpr int T = CH / 16;   // 16-row tiles per chunk
};

__device__ __forceinline__ float exp2_fast(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Register-staged chunk copy: CH rows x HD floats of a strided row source, global -> registers
// (load) and registers -> LDS [CH][HD+4] (store), so the NEXT chunk's global loads are in flight
// while the current chunk is multiplied. Rows >= n are zero.
template <int HD, int NT, int CH>
struct RowStage {
  static constexpr int F4 = HD / 4, PER = (CH * F4 + NT - 1) / NT;
  float4 r[PER];
  __device__ __forceinline__ void load(const float* __restrict__ src, int64_t stride, int row0, int n, int tid) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int f = tid + i * NT;
      const int row = f / F4, c = (f % F4) * 4;
      r[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (f < CH * F4 && row0 + row < n) r[i] = *reinterpret_cast<const float4*>(src + (int64_t)(row0 + row) * stride + c);
    }
  }
  __device__ __forceinline__ void store(float* dst, int tid) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int f = tid + i * NT;
      if (f < CH * F4) *reinterpret_cast<float4*>(dst + (f / F4) * (HD + 4) + (f % F4) * 4) = r[i];
    }
  }
};

// This lane's HD/4 consecutive elements of a row (lane group g = lane >> 4 holds d in [g*HD/4, (g+1)*HD/4)).
template <int HD>
__device__ __forceinline__ void load_frag(const float* p, bool valid, float (&f)[HD / 4]) {
#pragma unroll
  for (int s = 0; s < HD / 4; s += 4) {
    const float4 v = valid ? *reinterpret_cast<const float4*>(p + s) : make_float4(0.f, 0.f, 0.f, 0.f);
    f[s] = v.x; f[s + 1] = v.y; f[s + 2] = v.z; f[s + 3] = v.w;
  }
}

// acc[t][row = tile row (lane&15)][col = lane&15] += LDS rows (A operand: NTT consecutive 16-row tiles of a
// row-major [.][HD+4] image) x frag (B operand: this lane's HD/4 elements of the shared dimension).
// The NTT tile products are independent MFMA chains, interleaved so the 16x16x4's 40-cycle
// dependent latency hides behind the other chains' 32-cycle issues.
template <int HD, int NTT>
__device__ __forceinline__ void tiles_x_frag(const float* rows, const float (&frag)[HD / 4], int lane, f32x4 (&acc)[NTT]) {
  constexpr int LD = HD + 4;
  const float* ap = rows + (lane & 15) * LD + (lane >> 4) * (HD / 4);
#pragma unroll
  for (int s = 0; s < HD / 4; s += 4) {
    float4 a[NTT];
#pragma unroll
    for (int t = 0; t < NTT; ++t) a[t] = *reinterpret_cast<const float4*>(ap + t * 16 * LD + s);
#pragma unroll
    for (int t = 0; t < NTT; ++t) acc[t] = mfma4(a[t].x, frag[s], acc[t]);
#pragma unroll
    for (int t = 0; t < NTT; ++t) acc[t] = mfma4(a[t].y, frag[s + 1], acc[t]);
#pragma unroll
    for (int t = 0; t < NTT; ++t) acc[t] = mfma4(a[t].z, frag[s + 2], acc[t]);
#pragma unroll
    for (int t = 0; t < NTT; ++t) acc[t] = mfma4(a[t].w, frag[s + 3], acc[t]);
  }
}

// Two such products over the same tiles (S and dP in the backward passes): 2 x NTT chains.
template <int HD, int NTT>
__device__ __forceinline__ void tiles_x_frag2(const float* rows_a, const float (&fa)[HD / 4], const float* rows_b,
                                              const float (&fb)[HD / 4], int lane, f32x4 (&acc_a)[NTT],
                                              f32x4 (&acc_b)[NTT]) {
  constexpr int LD = HD + 4;
  const int off = (lane & 15) * LD + (lane >> 4) * (HD / 4);
#pragma unroll
  for (int s = 0; s < HD / 4; s += 4) {
    float4 a[NTT], b[NTT];
#pragma unroll
    for (int t = 0; t < NTT; ++t) {
      a[t] = *reinterpret_cast<const float4*>(rows_a + off + t * 16 * LD + s);
      b[t] = *reinterpret_cast<const float4*>(rows_b + off + t * 16 * LD + s);
    }
#pragma unroll
    for (int t = 0; t < NTT; ++t) { acc_a[t] = mfma4(a[t].x, fa[s], acc_a[t]); acc_b[t] = mfma4(b[t].x, fb[s], acc_b[t]); }
#pragma unroll
    for (int t = 0; t < NTT; ++t) { acc_a[t] = mfma4(a[t].y, fa[s + 1], acc_a[t]); acc_b[t] = mfma4(b[t].y, fb[s + 1], acc_b[t]); }
#pragma unroll
    for (int t = 0; t < NTT; ++t) { acc_a[t] = mfma4(a[t].z, fa[s + 2], acc_a[t]); acc_b[t] = mfma4(b[t].z, fb[s + 2], acc_b[t]); }
#pragma unroll
    for (int t = 0; t < NTT; ++t) { acc_a[t] = mfma4(a[t].w, fa[s + 3], acc_a[t]); acc_b[t] = mfma4(b[t].w, fb[s + 3], acc_b[t]); }
  }
}

// acc[dt] (rows d = 16 dt + (lane&15) of the transposed product, cols = lane&15 of w) +=
// M^T[d][t] * w[t] over the 16 rows t of the LDS tile M (row-major [.][HD+4]) whose order
// 4*(lane>>4)+i matches the accumulator layout of w (register i).
template <int HD>
__device__ __forceinline__ void colsT_x_acc(const float* tile, const f32x4& w, int lane, f32x4 (&acc)[HD / 16]) {
  const float* base = tile + 4 * (lane >> 4) * (HD + 4) + (lane & 15);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) acc[dt] = mfma4(base[i * (HD + 4) + dt * 16], w[i], acc[dt]);
  }
}

// Store the transposed accumulators of one row (this lane's column): d = 16 dt + 4 (lane>>4) + 0..3.
template <int HD>
__device__ __forceinline__ void store_rowT(float* rowp, const f32x4 (&acc)[HD / 16], float mul, int lane) {
#pragma unroll
  for (int dt = 0; dt < HD / 16; ++dt)
    *reinterpret_cast<float4*>(rowp + dt * 16 + 4 * (lane >> 4)) =
        make_float4(acc[dt][0] * mul, acc[dt][1] * mul, acc[dt][2] * mul, acc[dt][3] * mul);
}

// Zero rows [r0, r1) of one head's HD columns of a row-major buffer (grid-stride over the x extent):
// the extra grid slice z == nseq clears a row-bucketed buffer's tail past the last sequence, so a
// caller never needs the valid row count on the host (graph-capturable).
template <int HD, int NT>
__device__ __forceinline__ void zero_rows(float* base, int64_t stride, int64_t r0, int64_t r1, int hh, int tid) {
  constexpr int F4 = HD / 4;
  const int64_t n = (r1 - r0) * F4;
  for (int64_t f = (int64_t)blockIdx.x * NT + tid; f < n; f += (int64_t)gridDim.x * NT)
    *reinterpret_cast<float4*>(base + (r0 + f / F4) * stride + hh * HD + (f % F4) * 4) = make_float4(0.f, 0.f, 0.f, 0.f);
}

// Calls f.template run<NTT, MASK>() for a chunk of `nt` 16-row tiles: every tile unmasked when the
// chunk is interior (all NTL tiles present, every row valid, no causal diagonal), else masked.
template <int NTL, typename F>
__device__ __forceinline__ void dispatch_tiles(int nt, bool interior, F& f) {
  if (nt <= 0) return;
  if (interior && nt == NTL) { f.template run<NTL, false>(); return; }
  if (nt == 1) { f.template run<1, true>(); return; }
  if constexpr (NTL >= 3) {
    if (nt == 2) { f.template run<2, true>(); return; }
    if (nt == 3) { f.template run<3, true>(); return; }
  }
  f.template run<NTL, true>();
}

// ------------------------------------------------------------------------- sequence order
// Longest-first dispatch order of the sequences (LPT): order[r] = the sequence of rank r by segment
// length (descending, ties by index). The chunked forward and the fused backward map grid z through it,
// so the longest sequences' workgroups (whose run time grows with the length) start first and the
// launch does not end on one long straggler. One workgroup, lengths staged in LDS, B <= kOrderMax.
constexpr int kOrderMax = 4096;
__global__ void __launch_bounds__(1024) attn_order_kernel(const int64_t* __restrict__ cu, int B, int* __restrict__ order) {
  __shared__ int len[kOrderMax];
  for (int b = threadIdx.x; b < B; b += 1024) len[b] = (int)(cu[b + 1] - cu[b]);
  __syncthreads();
  for (int b = threadIdx.x; b < B; b += 1024) {
    const int lb = len[b];
    int rank = 0;
    for (int j = 0; j < B; ++j) rank += (len[j] > lb) || (len[j] == lb && j < b);
    order[rank] = b;
  }
}

// sequence of grid slice z (z < B): through the LPT order when one is given
__device__ __forceinline__ int seq_of(const int* __restrict__ order, int z) { return order ? order[z] : z; }

// ---------------------------------------------------------------------------------------- fwd
template <int HD>
struct FwdChunk {
  const float* K_s;
  const float* V_s;
  const float* qf;
  int lane, kc, lk, qi, causal;
  float sl2;
  float* m;
  float* l;
  f32x4* o;
  template <int NTT, bool MASK>
  __device__ __forceinline__ void run() {
    constexpr int LD = HD + 4;
    const int g = lane >> 4;
    f32x4 s[NTT];
#pragma unroll
    for (int t = 0; t < NTT; ++t) s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    tiles_x_frag<HD, NTT>(K_s, *reinterpret_cast<const float(*)[HD / 4]>(qf), lane, s);   // S^T: rows = keys
    float mt = -INFINITY;
#pragma unroll
    for (int t = 0; t < NTT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr (MASK) {
          const int key = kc + t * 16 + 4 * g + i;
          if (!(key < lk && (!causal || key <= qi))) s[t][i] = -INFINITY;
        }
        mt = fmaxf(mt, s[t][i]);
      }
    mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    const float mn = fmaxf(*m, mt * sl2);         // running max in log2 units (sl2 > 0 keeps the order)
    const bool none = MASK && mn == -INFINITY;    // every key so far masked (causal padding lanes)
    const float alpha = none ? 1.f : exp2_fast(*m - mn);
    float ls = 0.f;
#pragma unroll
    for (int t = 0; t < NTT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        s[t][i] = none ? 0.f : exp2_fast(__builtin_fmaf(s[t][i], sl2, -mn));
        ls += s[t][i];
      }
    *l = *l * alpha + ls;                         // per-lane partial sum (alpha is uniform per query)
    *m = mn;
    f32x4(&oa)[HD / 16] = *reinterpret_cast<f32x4(*)[HD / 16]>(o);
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) oa[dt] *= alpha;
#pragma unroll
    for (int t = 0; t < NTT; ++t) colsT_x_acc<HD>(V_s + t * 16 * LD, s[t], lane, oa);   // O^T += V^T P^T
  }
};

// ------------------------------------------------------------- split-bf16 forward (matmul 'high')
// At the reference's matmul precision 'high' (modules/model.py:27, the same setting that puts every Linear
// on the split-bf16 GEMM) the long-range forwards (HD = 64, 4-wave workgroups, 64-key chunks) multiply
// S = Q K^T and O = P V as a = hi + lo bf16 pairs: hi*lo + lo*hi + hi*hi on v_mfma_f32_16x16x32_bf16
// (fp32 accumulate; per-product relative error <= ~2^-16), 5.3x less MFMA time than the 16x16x4 fp32
// chain. The softmax (max, exp, running sums, lse) stays fp32. K and V are staged as row-major hi / lo
// planes: K fragments are one 16-B row read per plane, V^T fragments two ds_read_b64_tr_b16 transposed
// reads (x3_tr_frag) whose 8 keys per lane follow the order the S^T accumulator hands P^T to the PV
// product (lane group g holds keys 4g..4g+3 of the block's two 16-key tiles: position 8g + j <- key
// 4g + j (j < 4) / 16 + 4g + j - 4). (A transposed V image written by 16-bit scattered stores measured
// 2-way+ bank conflicts on 72% of the LDS cycles: profiles/r04/attn_tr/.)
typedef __bf16 abf16x8 __attribute__((ext_vector_type(8)));
constexpr int kX3Ld = 80;   // bf16 per plane row (160 B): the 16-row fragment reads (ds_read_b128) and the transposed
                            // reads of 4-row blocks 4 rows apart (ds_read_b64_tr_b16) are both bank-conflict-free

__device__ __forceinline__ void split8(const float (&v)[8], abf16x8& h, abf16x8& l) {
  uint4 hh, ll;
  split_bf16x2(v[0], v[1], hh.x, ll.x);
  split_bf16x2(v[2], v[3], hh.y, ll.y);
  split_bf16x2(v[4], v[5], hh.z, ll.z);
  split_bf16x2(v[6], v[7], hh.w, ll.w);
  h = __builtin_bit_cast(abf16x8, hh);
  l = __builtin_bit_cast(abf16x8, ll);
}

__device__ __forceinline__ f32x4 mfma_x3(const abf16x8& ah, const abf16x8& al, const abf16x8& bh,
                                         const abf16x8& bl, f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, c, 0, 0, 0);
}

// A RowStage's registers (CH rows x 64 fp32) written as row-major split planes [row][ld]
template <int NT, int CH>
__device__ __forceinline__ void x3_store_rows(const RowStage<64, NT, CH>& st, uint16_t* Xh, uint16_t* Xl, int ld,
                                              int tid) {
  constexpr int F4 = 16;
#pragma unroll
  for (int i = 0; i < RowStage<64, NT, CH>::PER; ++i) {
    const int f = tid + i * NT;
    if (f < CH * F4) {
      const int row = f / F4, c = (f % F4) * 4;
      uint2 h, l;
      split_bf16x2(st.r[i].x, st.r[i].y, h.x, l.x);
      split_bf16x2(st.r[i].z, st.r[i].w, h.y, l.y);
      *reinterpret_cast<uint2*>(Xh + row * ld + c) = h;
      *reinterpret_cast<uint2*>(Xl + row * ld + c) = l;
    }
  }
}
typedef short x3s4 __attribute__((ext_vector_type(4)));
// Fragment (8 bf16, k = 8 g + e) of a product contracting over the ROWS of a row-major bf16 plane [.][ld]:
// element e of lane (g, c) = plane[row0 + x3 order(8 g + e)][col0 + c] with x3 order 4 g + e (e < 4) /
// 16 + 4 g + e - 4 — the S accumulator's query order (two ds_read_b64_tr_b16 of 4-row blocks). EXEC must be
// all ones (wave-uniform control flow only).
__device__ __forceinline__ abf16x8 x3_tr_frag(const uint16_t* plane, int ld, int row0, int col0, int lane) {
  const uint16_t* a = plane + (row0 + 4 * (lane >> 4) + ((lane >> 2) & 3)) * ld + col0 + 4 * (lane & 3);
  const x3s4 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) x3s4*)a);
  const x3s4 y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) x3s4*)(a + 16 * ld));
  typedef short x3s8 __attribute__((ext_vector_type(8)));
  const x3s8 v = {x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
  return __builtin_bit_cast(abf16x8, v);
}
// this lane's query fragments (d = 32 b + 8 (lane >> 4) + 0..7, b = 0, 1) as split planes
__device__ __forceinline__ void x3_load_q(const float* p, bool valid, int lane, abf16x8 (&qh)[2], abf16x8 (&ql)[2]) {
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    float v[8];
    const float* src = p + 32 * b + 8 * (lane >> 4);
    const float4 x = valid ? *reinterpret_cast<const float4*>(src) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 y = valid ? *reinterpret_cast<const float4*>(src + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w; v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
    split8(v, qh[b], ql[b]);
  }
}

// FwdChunk's online-softmax step on the split planes (HD = 64, 64-key chunk of NTT <= 4 tiles)
struct FwdChunkX3 {
  const uint16_t* Kh;
  const uint16_t* Kl;
  const uint16_t* Vh;
  const uint16_t* Vl;
  const abf16x8* qh;
  const abf16x8* ql;
  int lane, kc, lk, qi, causal;
  float sl2;
  float* m;
  float* l;
  f32x4* o;
  template <int NTT, bool MASK>
  __device__ __forceinline__ void run() {
    const int g = lane >> 4, r = lane & 15;
    f32x4 s[NTT];
#pragma unroll
    for (int t = 0; t < NTT; ++t) s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int b = 0; b < 2; ++b) {   // S^T = K Q^T: rows = keys, columns = queries
#pragma unroll
      for (int t = 0; t < NTT; ++t) {
        const int off = (16 * t + r) * kX3Ld + 32 * b + 8 * g;
        const abf16x8 kh = *reinterpret_cast<const abf16x8*>(Kh + off);
        const abf16x8 kl = *reinterpret_cast<const abf16x8*>(Kl + off);
        s[t] = mfma_x3(kh, kl, qh[b], ql[b], s[t]);
      }
    }
    float mt = -INFINITY;
#pragma unroll
    for (int t = 0; t < NTT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr (MASK) {
          const int key = kc + t * 16 + 4 * g + i;
          if (!(key < lk && (!causal || key <= qi))) s[t][i] = -INFINITY;
        }
        mt = fmaxf(mt, s[t][i]);
      }
    mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    const float mn = fmaxf(*m, mt * sl2);
    const bool none = MASK && mn == -INFINITY;
    const float alpha = none ? 1.f : exp2_fast(*m - mn);
    float ls = 0.f;
#pragma unroll
    for (int t = 0; t < NTT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        s[t][i] = none ? 0.f : exp2_fast(__builtin_fmaf(s[t][i], sl2, -mn));
        ls += s[t][i];
      }
    *l = *l * alpha + ls;
    *m = mn;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;
    constexpr int NKB = (NTT + 1) / 2;
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) {   // O^T += V^T P^T over the block's 32 keys (permuted order)
      float p8[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        p8[i] = s[2 * kb][i];
        p8[4 + i] = 2 * kb + 1 < NTT ? s[2 * kb + 1 < NTT ? 2 * kb + 1 : 0][i] : 0.f;
      }
      abf16x8 ph, pl;
      split8(p8, ph, pl);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const abf16x8 vh = x3_tr_frag(Vh, kX3Ld, 32 * kb, 16 * dt, lane);
        const abf16x8 vl = x3_tr_frag(Vl, kX3Ld, 32 * kb, 16 * dt, lane);
        o[dt] = mfma_x3(vh, vl, ph, pl, o[dt]);
      }
    }
  }
};

// X3: the split-bf16 products (matmul 'high'; HD = 64, NW = 4 only)
template <int HD, int NW, bool X3 = false>
__global__ void __launch_bounds__(64 * NW) attn_fwd_kernel(const float* __restrict__ q, int64_t sq, const float* __restrict__ k,
                                                        int64_t sk, const float* __restrict__ v, int64_t sv,
                                                        const int64_t* __restrict__ cu_q, const int64_t* __restrict__ cu_k,
                                                        int causal, float scale, float* __restrict__ out, int64_t so,
                                                        float* __restrict__ lse, int64_t Tq, const int* __restrict__ order) {
  constexpr int LD = HD + 4, DT = HD / 16, CH = Chunk<NW>::CH, NTL = Chunk<NW>::T;
  static_assert(!X3 || (HD == 64 && CH == 64), "split-bf16 form: HD 64, 64-key chunks");
  constexpr int kSmemF = X3 ? (4 * 64 * kX3Ld) / 2 : 2 * CH * LD;   // floats
  __shared__ __attribute__((aligned(16))) float smem[kSmemF];
  float* K_s = smem;
  float* V_s = smem + CH * LD;
  uint16_t* const Kh = reinterpret_cast<uint16_t*>(smem);
  uint16_t* const Kl = Kh + 64 * kX3Ld;
  uint16_t* const Vh = Kl + 64 * kX3Ld;
  uint16_t* const Vl = Vh + 64 * kX3Ld;
  const int z = blockIdx.z, hh = blockIdx.y, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int g = lane >> 4;
  if (z == (int)gridDim.z - 1) {              // tail slice: output rows past the last sequence
    zero_rows<HD, 64 * NW>(out, so, cu_q[z], Tq, hh, tid);
    return;
  }
  const int b = seq_of(order, z);
  const int64_t q0 = cu_q[b], k0 = cu_k[b];
  const int lq = (int)(cu_q[b + 1] - q0), lk = (int)(cu_k[b + 1] - k0);
  const int qwg = blockIdx.x * 16 * NW;
  if (qwg >= lq) return;                      // uniform over the workgroup
  const int qb = qwg + wave * 16, qi = qb + (lane & 15);
  const bool wave_on = qb < lq, qv = qi < lq;
  float qf[HD / 4];
  abf16x8 qh[2], ql[2];
  const float* qrow = q + (q0 + (qv ? qi : 0)) * sq + hh * HD;
  if constexpr (X3)
    x3_load_q(qrow, qv, lane, qh, ql);
  else
    load_frag<HD>(qrow + g * (HD / 4), qv, qf);
  f32x4 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;
  const int kend = causal ? min(lk, qwg + 16 * NW) : lk;   // workgroup's last key (staging loop)
  const int kend_w = causal ? min(lk, qb + 16) : lk;        // this wave's last key
  const float* kb_ = k + k0 * sk + hh * HD;
  const float* vb_ = v + k0 * sv + hh * HD;
  RowStage<HD, 64 * NW, CH> stk, stv;
  FwdChunk<HD> fc{K_s, V_s, qf, lane, 0, lk, qi, causal, scale * kLog2e, &m, &l, o};
  FwdChunkX3 fx{Kh, Kl, Vh, Vl, qh, ql, lane, 0, lk, qi, causal, scale * kLog2e, &m, &l, o};
  for (int kc = 0; kc < kend; kc += CH) {
    stk.load(kb_, sk, kc, lk, tid);
    stv.load(vb_, sv, kc, lk, tid);
    __syncthreads();                          // the previous chunk's LDS reads are done
    if constexpr (X3) {
      x3_store_rows<64 * NW, 64>(stk, Kh, Kl, kX3Ld, tid);
      x3_store_rows<64 * NW, 64>(stv, Vh, Vl, kX3Ld, tid);
    } else {
      stk.store(K_s, tid);
      stv.store(V_s, tid);
    }
    __syncthreads();
    const int nt = __builtin_amdgcn_readfirstlane(wave_on ? min(NTL, (kend_w - kc + 15) >> 4) : 0);
    if constexpr (X3) {
      fx.kc = kc;
      dispatch_tiles<NTL>(nt, !causal && kc + CH <= lk, fx);
    } else {
      fc.kc = kc;
      dispatch_tiles<NTL>(nt, !causal && kc + CH <= lk, fc);
    }
  }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  if (!qv) return;
  const float inv = l > 0.f ? 1.f / l : 0.f;
  store_rowT<HD>(out + (q0 + qi) * so + hh * HD, o, inv, lane);
  if (g == 0) lse[(int64_t)hh * Tq + q0 + qi] = l > 0.f ? (m + log2f(l)) * kLn2 : 0.f;
}

// ------------------------------------------------------------------------------------ bwd: dQ
template <int HD>
struct DqChunk {
  const float* K_s;
  const float* V_s;
  const float* qf;
  const float* dof;
  int lane, kc, lk, qi, causal;
  float sl2, lse2, delta;
  f32x4* acc;
  template <int NTT, bool MASK>
  __device__ __forceinline__ void run() { groups<NTT, MASK>(0); }
  template <int N, bool MASK>   // tiles [tb, tb + N) in groups of RQ_ATTN_BWD_GROUP
  __device__ __forceinline__ void groups(int tb) {
    constexpr int NG = N < RQ_ATTN_BWD_GROUP ? N : RQ_ATTN_BWD_GROUP;
    group<NG, MASK>(tb);
    if constexpr (N > NG) groups<N - NG, MASK>(tb + NG);
  }
  template <int NG, bool MASK>
  __device__ __forceinline__ void group(int tb) {
    constexpr int LD = HD + 4;
    const int g = lane >> 4;
    f32x4 s[NG], dp[NG];
#pragma unroll
    for (int t = 0; t < NG; ++t) { s[t] = f32x4{0.f, 0.f, 0.f, 0.f}; dp[t] = f32x4{0.f, 0.f, 0.f, 0.f}; }
    tiles_x_frag2<HD, NG>(K_s + tb * 16 * LD, *reinterpret_cast<const float(*)[HD / 4]>(qf), V_s + tb * 16 * LD,
                          *reinterpret_cast<const float(*)[HD / 4]>(dof), lane, s, dp);   // S^T, dP^T = V dO^T
#pragma unroll
    for (int t = 0; t < NG; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float p = exp2_fast(__builtin_fmaf(s[t][i], sl2, -lse2));
        if constexpr (MASK) {
          const int key = kc + (tb + t) * 16 + 4 * g + i;
          if (!(key < lk && (!causal || key <= qi))) p = 0.f;
        }
        s[t][i] = p * (dp[t][i] - delta);       // dS^T
      }
    f32x4(&aa)[HD / 16] = *reinterpret_cast<f32x4(*)[HD / 16]>(acc);
#pragma unroll
    for (int t = 0; t < NG; ++t) colsT_x_acc<HD>(K_s + (tb + t) * 16 * LD, s[t], lane, aa);   // dQ^T += K^T dS^T
  }
};

template <int HD, int NW>
__global__ void __launch_bounds__(64 * NW) attn_bwd_dq_kernel(
    const float* __restrict__ q, int64_t sq, const float* __restrict__ k, int64_t sk, const float* __restrict__ v,
    int64_t sv, const float* __restrict__ out, int64_t so, const float* __restrict__ dout, int64_t sdo,
    const float* __restrict__ lse, int64_t Tq, const int64_t* __restrict__ cu_q, const int64_t* __restrict__ cu_k,
    int causal, float scale, float* __restrict__ dq, int64_t sdq, float* __restrict__ delta_out) {
  constexpr int LD = HD + 4, DT = HD / 16, CH = Chunk<NW>::CH, NTL = Chunk<NW>::T;
  __shared__ __attribute__((aligned(16))) float smem[2 * CH * LD];
  float* K_s = smem;
  float* V_s = smem + CH * LD;
  const int b = blockIdx.z, hh = blockIdx.y, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int g = lane >> 4;
  if (b == (int)gridDim.z - 1) {              // tail slice: dQ rows past the last sequence
    zero_rows<HD, 64 * NW>(dq, sdq, cu_q[b], Tq, hh, tid);
    return;
  }
  const int64_t q0 = cu_q[b], k0 = cu_k[b];
  const int lq = (int)(cu_q[b + 1] - q0), lk = (int)(cu_k[b + 1] - k0);
  const int qwg = blockIdx.x * 16 * NW;
  if (qwg >= lq) return;
  const int qb = qwg + wave * 16, qi = qb + (lane & 15);
  const bool wave_on = qb < lq, qv = qi < lq;
  const int64_t qrow = q0 + (qv ? qi : 0);
  float qf[HD / 4], dof[HD / 4];
  load_frag<HD>(q + qrow * sq + hh * HD + g * (HD / 4), qv, qf);
  load_frag<HD>(dout + qrow * sdo + hh * HD + g * (HD / 4), qv, dof);
  float delta = 0.f;
  {
    float of[HD / 4];
    load_frag<HD>(out + qrow * so + hh * HD + g * (HD / 4), qv, of);
#pragma unroll
    for (int d = 0; d < HD / 4; ++d) delta += dof[d] * of[d];
    delta += __shfl_xor(delta, 16, 64);
    delta += __shfl_xor(delta, 32, 64);
    if (qv && g == 0) delta_out[(int64_t)hh * Tq + qrow] = delta;   // reused by the dK/dV pass
  }
  f32x4 acc[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) acc[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int kend = causal ? min(lk, qwg + 16 * NW) : lk;
  const int kend_w = causal ? min(lk, qb + 16) : lk;
  const float* kb_ = k + k0 * sk + hh * HD;
  const float* vb_ = v + k0 * sv + hh * HD;
  RowStage<HD, 64 * NW, CH> stk, stv;
  DqChunk<HD> fc{K_s, V_s, qf, dof, lane, 0, lk, qi, causal, scale * kLog2e,
                 qv ? lse[(int64_t)hh * Tq + qrow] * kLog2e : 0.f, delta, acc};
  for (int kc = 0; kc < kend; kc += CH) {
    stk.load(kb_, sk, kc, lk, tid);
    stv.load(vb_, sv, kc, lk, tid);
    __syncthreads();
    stk.store(K_s, tid);
    stv.store(V_s, tid);
    __syncthreads();
    const int nt = __builtin_amdgcn_readfirstlane(wave_on ? min(NTL, (kend_w - kc + 15) >> 4) : 0);
    fc.kc = kc;
    dispatch_tiles<NTL>(nt, !causal && kc + CH <= lk, fc);
  }
  if (!qv) return;
  store_rowT<HD>(dq + (q0 + qi) * sdq + hh * HD, acc, scale, lane);
}

// ------------------------------------------------------------------------------- bwd: dK, dV
template <int HD>
struct DkdvChunk {
  const float* Q_s;
  const float* O_s;
  const float* lse_s;
  const float* dl_s;
  const float* kf;
  const float* vf;
  int lane, qc, t0, lq, kj, causal;
  float sl2;
  f32x4* dka;
  f32x4* dva;
  template <int NTT, bool MASK>
  __device__ __forceinline__ void run() { groups<NTT, MASK>(t0); }
  template <int N, bool MASK>   // tiles [tb, tb + N) in groups of RQ_ATTN_BWD_GROUP
  __device__ __forceinline__ void groups(int tb) {
    constexpr int NG = N < RQ_ATTN_BWD_GROUP ? N : RQ_ATTN_BWD_GROUP;
    group<NG, MASK>(tb);
    if constexpr (N > NG) groups<N - NG, MASK>(tb + NG);
  }
  template <int NG, bool MASK>
  __device__ __forceinline__ void group(int tb) {
    constexpr int LD = HD + 4;
    const int g = lane >> 4;
    const float* Qt = Q_s + tb * 16 * LD;
    const float* Ot = O_s + tb * 16 * LD;
    f32x4 s[NG], dp[NG];
#pragma unroll
    for (int t = 0; t < NG; ++t) { s[t] = f32x4{0.f, 0.f, 0.f, 0.f}; dp[t] = f32x4{0.f, 0.f, 0.f, 0.f}; }
    tiles_x_frag2<HD, NG>(Qt, *reinterpret_cast<const float(*)[HD / 4]>(kf), Ot,
                          *reinterpret_cast<const float(*)[HD / 4]>(vf), lane, s, dp);   // S, dP = dO V^T
#pragma unroll
    for (int t = 0; t < NG; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int qr = (tb + t) * 16 + 4 * g + i;
        float p = exp2_fast(__builtin_fmaf(s[t][i], sl2, -lse_s[qr]));
        if constexpr (MASK) {
          const int qq = qc + qr;
          if (!(qq < lq && (!causal || kj <= qq))) p = 0.f;
        }
        s[t][i] = p;
        dp[t][i] = p * (dp[t][i] - dl_s[qr]);   // dS
      }
    f32x4(&dk_)[HD / 16] = *reinterpret_cast<f32x4(*)[HD / 16]>(dka);
    f32x4(&dv_)[HD / 16] = *reinterpret_cast<f32x4(*)[HD / 16]>(dva);
#pragma unroll
    for (int t = 0; t < NG; ++t) {
      colsT_x_acc<HD>(Ot + t * 16 * LD, s[t], lane, dv_);    // dV^T += dO^T P
      colsT_x_acc<HD>(Qt + t * 16 * LD, dp[t], lane, dk_);   // dK^T += Q^T dS
    }
  }
};

template <int HD, int NW>
__global__ void __launch_bounds__(64 * NW) attn_bwd_dkdv_kernel(
    const float* __restrict__ q, int64_t sq, const float* __restrict__ k, int64_t sk, const float* __restrict__ v,
    int64_t sv, const float* __restrict__ dout, int64_t sdo, const float* __restrict__ lse,
    const float* __restrict__ delta, int64_t Tq, const int64_t* __restrict__ cu_q, const int64_t* __restrict__ cu_k,
    int causal, float scale, float* __restrict__ dk, int64_t sdk, float* __restrict__ dv, int64_t sdv, int64_t Tk) {
  constexpr int LD = HD + 4, DT = HD / 16, CH = Chunk<NW>::CH, NTL = Chunk<NW>::T;
  __shared__ __attribute__((aligned(16))) float smem[2 * CH * LD + 2 * CH];
  float* Q_s = smem;
  float* O_s = smem + CH * LD;   // dO tile
  float* lse_s = O_s + CH * LD;
  float* dl_s = lse_s + CH;
  const int b = blockIdx.z, hh = blockIdx.y, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int g = lane >> 4;
  if (b == (int)gridDim.z - 1) {              // tail slice: dK / dV rows past the last sequence
    zero_rows<HD, 64 * NW>(dk, sdk, cu_k[b], Tk, hh, tid);
    zero_rows<HD, 64 * NW>(dv, sdv, cu_k[b], Tk, hh, tid);
    return;
  }
  const int64_t q0 = cu_q[b], k0 = cu_k[b];
  const int lq = (int)(cu_q[b + 1] - q0), lk = (int)(cu_k[b + 1] - k0);
  const int kwg = blockIdx.x * 16 * NW;
  if (kwg >= lk) return;
  const int kb = kwg + wave * 16, kj = kb + (lane & 15);
  const bool wave_on = kb < lk, kv = kj < lk;
  const int64_t krow = k0 + (kv ? kj : 0);
  float kf[HD / 4], vf[HD / 4];
  load_frag<HD>(k + krow * sk + hh * HD + g * (HD / 4), kv, kf);
  load_frag<HD>(v + krow * sv + hh * HD + g * (HD / 4), kv, vf);
  f32x4 dka[DT], dva[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) { dka[dt] = f32x4{0.f, 0.f, 0.f, 0.f}; dva[dt] = f32x4{0.f, 0.f, 0.f, 0.f}; }
  // causal (key <= query): query chunks that end before this workgroup's first key contribute nothing
  const int qstart = causal ? (kwg / CH) * CH : 0;
  const float* qb_ = q + q0 * sq + hh * HD;
  const float* ob_ = dout + q0 * sdo + hh * HD;
  const float* lse_h = lse + (int64_t)hh * Tq + q0;
  const float* dl_h = delta + (int64_t)hh * Tq + q0;
  RowStage<HD, 64 * NW, CH> stq, sto;
  float lse_r = 0.f, dl_r = 0.f;              // thread tid < CH stages the chunk's row tid
  auto load_chunk = [&](int qc) {
    stq.load(qb_, sq, qc, lq, tid);
    sto.load(ob_, sdo, qc, lq, tid);
    const bool ok = tid < CH && qc + tid < lq;
    lse_r = ok ? lse_h[qc + tid] * kLog2e : 0.f;
    dl_r = ok ? dl_h[qc + tid] : 0.f;
  };
  DkdvChunk<HD> fc{Q_s, O_s, lse_s, dl_s, kf, vf, lane, 0, 0, lq, kj, causal, scale * kLog2e, dka, dva};
  for (int qc = qstart; qc < lq; qc += CH) {
    load_chunk(qc);
    __syncthreads();
    stq.store(Q_s, tid);
    sto.store(O_s, tid);
    if (tid < CH) {
      lse_s[tid] = lse_r;
      dl_s[tid] = dl_r;
    }
    __syncthreads();
    const int t0 = __builtin_amdgcn_readfirstlane(causal ? max(0, (kb - qc) >> 4) : 0);   // tiles wholly before the keys
    const int nt = __builtin_amdgcn_readfirstlane(wave_on ? min(NTL, (lq - qc + 15) >> 4) - t0 : 0);
    fc.qc = qc;
    fc.t0 = t0;
    dispatch_tiles<NTL>(nt, !causal && qc + CH <= lq, fc);
  }
  if (!kv) return;
  store_rowT<HD>(dk + (k0 + kj) * sdk + hh * HD, dka, scale, lane);
  store_rowT<HD>(dv + (k0 + kj) * sdv + hh * HD, dva, 1.f, lane);
}

template <int HD>
__global__ void __launch_bounds__(256) attn_kv_reduce_kernel(const float* __restrict__ kvpart, int qsplit, int64_t Tk,
                                                             int64_t H, const int64_t* __restrict__ cu_k, int B,
                                                             float scale, float* __restrict__ dk, int64_t sdk,
                                                             float* __restrict__ dv, int64_t sdv) {
  constexpr int F4 = HD / 4;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t HH = H * HD;
  const int64_t row = i / (H * F4), c = (i % (H * F4)) * 4;
  if (row >= cu_k[B]) return;
  const int64_t slab = Tk * HH;
  const float* p = kvpart + row * HH + c;
  float4 a = *reinterpret_cast<const float4*>(p), e = *reinterpret_cast<const float4*>(p + qsplit * slab);
  for (int s = 1; s < qsplit; ++s) {
    const float4 x = *reinterpret_cast<const float4*>(p + s * slab);
    const float4 y = *reinterpret_cast<const float4*>(p + (qsplit + s) * slab);
    a.x += x.x; a.y += x.y; a.z += x.z; a.w += x.w;
    e.x += y.x; e.y += y.y; e.z += y.z; e.w += y.w;
  }
  *reinterpret_cast<float4*>(dk + row * sdk + c) = make_float4(a.x * scale, a.y * scale, a.z * scale, a.w * scale);
  *reinterpret_cast<float4*>(dv + row * sdv + c) = e;
}

// ------------------------------------------------------------- fwd: split keys (few queries)
// Few queries over a long key range (the decoder's cross-attention: 5-6 future tokens x a context of
// up to 81 / 801 / 1281 rows): the chunked forward gives each (sequence, head) ONE wave that walks every
// 32-key chunk serially. Here key block j of kSplitKB (32 for ranges <= 128, else 128) keys is its own
// one-wave workgroup (FwdChunk over the block, the same online softmax), which writes its unnormalised
// partial (o, m, l) to `part`; attn_fwd_combine_kernel merges a query's blocks in block order (deterministic):
// M = max m_j, L = sum l_j 2^(m_j - M), o = sum o_j 2^(m_j - M) / L, lse = (M + log2 L) ln 2.
// part layout: o (nsplit, Tq, H, HD) then m, l (nsplit, H, Tq) each.
template <int HD, int kSplitKB>
__global__ void __launch_bounds__(64) attn_fwd_split_kernel(const float* __restrict__ q, int64_t sq,
                                                            const float* __restrict__ k, int64_t sk,
                                                            const float* __restrict__ v, int64_t sv,
                                                            const int64_t* __restrict__ cu_q,
                                                            const int64_t* __restrict__ cu_k, float scale, int64_t Tq,
                                                            float* __restrict__ part, int nsplit) {
  constexpr int CH = 32, LD = HD + 4, DT = HD / 16;
  __shared__ __attribute__((aligned(16))) float smem[2 * CH * LD];
  float* K_s = smem;
  float* V_s = smem + CH * LD;
  const int b = blockIdx.z, hh = blockIdx.y, j = blockIdx.x, lane = threadIdx.x, g = lane >> 4;
  const int64_t q0 = cu_q[b], k0 = cu_k[b];
  const int lq = (int)(cu_q[b + 1] - q0), lk = (int)(cu_k[b + 1] - k0);
  const int kbeg = j * kSplitKB;
  if (lq <= 0 || kbeg >= lk) return;         // no partial for this block (the combine skips it)
  const int kend = min(lk, kbeg + kSplitKB);
  const int qi = lane & 15;
  const bool qv = qi < lq;
  float qf[HD / 4];
  load_frag<HD>(q + (q0 + (qv ? qi : 0)) * sq + hh * HD + g * (HD / 4), qv, qf);
  f32x4 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;
  const float* kb_ = k + k0 * sk + hh * HD;
  const float* vb_ = v + k0 * sv + hh * HD;
  RowStage<HD, 64, CH> stk, stv;
  FwdChunk<HD> fc{K_s, V_s, qf, lane, 0, kend, qi, 0, scale * kLog2e, &m, &l, o};
  for (int kc = kbeg; kc < kend; kc += CH) {
    stk.load(kb_, sk, kc, kend, lane);
    stv.load(vb_, sv, kc, kend, lane);
    __syncthreads();
    stk.store(K_s, lane);
    stv.store(V_s, lane);
    __syncthreads();
    const int nt = __builtin_amdgcn_readfirstlane(min(CH / 16, (kend - kc + 15) >> 4));
    fc.kc = kc;
    dispatch_tiles<CH / 16>(nt, kc + CH <= kend, fc);
  }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  if (!qv) return;
  const int64_t H = gridDim.y, row = q0 + qi;
  store_rowT<HD>(part + (((int64_t)j * Tq + row) * H + hh) * HD, o, 1.f, lane);
  if (g == 0) {
    float* ml = part + (int64_t)nsplit * Tq * H * HD;
    ml[((int64_t)j * H + hh) * Tq + row] = m;
    ml[((int64_t)(nsplit + j) * H + hh) * Tq + row] = l;
  }
}

// Key-split form of attn_fwd_kernel for long, few sequences (the C4 per-rank config: 8 sequences of up to
// 801 keys, 6 heads): with one workgroup per 64-query block walking every key, the launch lasts as long
// as the longest sequence's chain (51 key tiles). Here grid x = query block x key block (kSplitKB keys,
// non-causal), each workgroup runs the same staged online softmax over its key block and writes the
// unnormalised (o, m, l) partial in attn_fwd_split_kernel's layout; attn_fwd_combine_kernel merges them
// in key-block order (deterministic).
template <int HD, int NW, int kSplitKB, bool X3 = false>
__global__ void __launch_bounds__(64 * NW) attn_fwd_kvsplit_kernel(
    const float* __restrict__ q, int64_t sq, const float* __restrict__ k, int64_t sk, const float* __restrict__ v,
    int64_t sv, const int64_t* __restrict__ cu_q, const int64_t* __restrict__ cu_k, float scale, int64_t Tq,
    float* __restrict__ part, int nsplit) {
  constexpr int LD = HD + 4, DT = HD / 16, CH = Chunk<NW>::CH, NTL = Chunk<NW>::T;
  static_assert(kSplitKB % CH == 0, "key block of whole chunks");
  static_assert(!X3 || (HD == 64 && CH == 64), "split-bf16 form: HD 64, 64-key chunks");
  constexpr int kSmemF = X3 ? (4 * 64 * kX3Ld) / 2 : 2 * CH * LD;   // floats
  __shared__ __attribute__((aligned(16))) float smem[kSmemF];
  float* K_s = smem;
  float* V_s = smem + CH * LD;
  uint16_t* const Kh = reinterpret_cast<uint16_t*>(smem);
  uint16_t* const Kl = Kh + 64 * kX3Ld;
  uint16_t* const Vh = Kl + 64 * kX3Ld;
  uint16_t* const Vl = Vh + 64 * kX3Ld;
  const int b = blockIdx.z, hh = blockIdx.y, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int g = lane >> 4;
  const int j = blockIdx.x % nsplit, qblk = blockIdx.x / nsplit;
  const int64_t q0 = cu_q[b], k0 = cu_k[b];
  const int lq = (int)(cu_q[b + 1] - q0), lk = (int)(cu_k[b + 1] - k0);
  const int qwg = qblk * 16 * NW, kbeg = j * kSplitKB;
  if (qwg >= lq || kbeg >= lk) return;        // uniform: no partial for this block (the combine skips it)
  const int kend = min(lk, kbeg + kSplitKB);
  const int qb = qwg + wave * 16, qi = qb + (lane & 15);
  const bool wave_on = qb < lq, qv = qi < lq;
  float qf[HD / 4];
  abf16x8 qh[2], ql[2];
  const float* qrow = q + (q0 + (qv ? qi : 0)) * sq + hh * HD;
  if constexpr (X3)
    x3_load_q(qrow, qv, lane, qh, ql);
  else
    load_frag<HD>(qrow + g * (HD / 4), qv, qf);
  f32x4 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;
  const float* kb_ = k + k0 * sk + hh * HD;
  const float* vb_ = v + k0 * sv + hh * HD;
  RowStage<HD, 64 * NW, CH> stk, stv;
  FwdChunk<HD> fc{K_s, V_s, qf, lane, 0, kend, qi, 0, scale * kLog2e, &m, &l, o};
  FwdChunkX3 fx{Kh, Kl, Vh, Vl, qh, ql, lane, 0, kend, qi, 0, scale * kLog2e, &m, &l, o};
  for (int kc = kbeg; kc < kend; kc += CH) {
    stk.load(kb_, sk, kc, kend, tid);
    stv.load(vb_, sv, kc, kend, tid);
    __syncthreads();                          // the previous chunk's LDS reads are done
    if constexpr (X3) {
      x3_store_rows<64 * NW, 64>(stk, Kh, Kl, kX3Ld, tid);
      x3_store_rows<64 * NW, 64>(stv, Vh, Vl, kX3Ld, tid);
    } else {
      stk.store(K_s, tid);
      stv.store(V_s, tid);
    }
    __syncthreads();
    const int nt = __builtin_amdgcn_readfirstlane(wave_on ? min(NTL, (kend - kc + 15) >> 4) : 0);
    if constexpr (X3) {
      fx.kc = kc;
      dispatch_tiles<NTL>(nt, kc + CH <= kend, fx);
    } else {
      fc.kc = kc;
      dispatch_tiles<NTL>(nt, kc + CH <= kend, fc);
    }
  }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  if (!qv) return;
  const int64_t H = gridDim.y, row = q0 + qi;
  store_rowT<HD>(part + (((int64_t)j * Tq + row) * H + hh) * HD, o, 1.f, lane);
  if (g == 0) {
    float* ml = part + (int64_t)nsplit * Tq * H * HD;
    ml[((int64_t)j * H + hh) * Tq + row] = m;
    ml[((int64_t)(nsplit + j) * H + hh) * Tq + row] = l;
  }
}

// one 16-lane group per (query row, head): the split partials' merge, out / lse rows; rows past the last
// sequence (grid row z == B) get zeros
template <int HD, int kSplitKB>
__global__ void __launch_bounds__(256) attn_fwd_combine_kernel(const float* __restrict__ part, int nsplit,
                                                               const int64_t* __restrict__ cu_q,
                                                               const int64_t* __restrict__ cu_k, int64_t Tq,
                                                               float* __restrict__ out, int64_t so,
                                                               float* __restrict__ lse) {
  constexpr int F4 = HD / 4, RPB = 256 / F4;
  const int z = blockIdx.z, hh = blockIdx.y, c = (threadIdx.x % F4) * 4;
  const int64_t H = gridDim.y;
  if (z == (int)gridDim.z - 1) {              // tail slice
    zero_rows<HD, 256>(out, so, cu_q[z], Tq, hh, threadIdx.x);
    return;
  }
  const int64_t q0 = cu_q[z];
  const int lq = (int)(cu_q[z + 1] - q0), lk = (int)(cu_k[z + 1] - cu_k[z]);
  const int r = blockIdx.x * RPB + threadIdx.x / F4;
  if (r >= lq) return;
  const int64_t row = q0 + r;
  const int n = (lk + kSplitKB - 1) / kSplitKB;
  const float* ml = part + (int64_t)nsplit * Tq * H * HD;
  float M = -INFINITY;
  for (int j = 0; j < n; ++j) M = fmaxf(M, ml[((int64_t)j * H + hh) * Tq + row]);
  float L = 0.f;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int j = 0; j < n; ++j) {
    const float mj = ml[((int64_t)j * H + hh) * Tq + row];
    const float w = M == -INFINITY ? 0.f : exp2_fast(mj - M);
    L += ml[((int64_t)(nsplit + j) * H + hh) * Tq + row] * w;
    const float4 a = *reinterpret_cast<const float4*>(part + (((int64_t)j * Tq + row) * H + hh) * HD + c);
    acc.x += a.x * w; acc.y += a.y * w; acc.z += a.z * w; acc.w += a.w * w;
  }
  const float inv = L > 0.f ? 1.f / L : 0.f;
  *reinterpret_cast<float4*>(out + row * so + hh * HD + c) = make_float4(acc.x * inv, acc.y * inv, acc.z * inv, acc.w * inv);
  if (c == 0) lse[hh * Tq + row] = L > 0.f ? (M + log2f(L)) * kLn2 : 0.f;
}

// ------------------------------------------------------------------ bwd: fused dQ, dK, dV
// One launch per key block of KB = 16 NW keys computes S and dP ONCE per (query tile, key tile)
// pair — 5 MFMA products per pair (S, dP, dV, dK, dQ) instead of the two-pass form's 7 (the dQ pass
// recomputes S and dP). The block's dS (CH queries x KB keys) goes through LDS so each wave can
// form dQ rows over ALL KB keys against the staged K block: dQ^T(16 q) += K^T dS^T. A sequence with
// one key block (lk <= KB) gets dQ written directly; longer ones write one partial per key block
// into `part` (nkb_max, Tq, H*HD) and attn_dq_reduce_kernel sums them in key-block order — no
// atomics, bitwise deterministic. delta = rowsum(dO * O) comes from attn_delta_kernel beforehand.
template <int HD>
struct FusedChunk {
  const float* Q_s;
  const float* O_s;
  const float* lse_s;
  const float* dl_s;
  const float* kf;
  const float* vf;
  float* dS_s;   // [CH][KB + 4]: this wave writes columns [16 wave, 16 wave + 16)
  int lane, qc, t0, lq, kj, causal, col, ldS;
  bool kv;
  float sl2;
  f32x4* dka;
  f32x4* dva;
  template <int NTT, bool MASK>
  __device__ __forceinline__ void run() { groups<NTT, MASK>(t0); }
  template <int N, bool MASK>
  __device__ __forceinline__ void groups(int tb) {
    constexpr int NG = N < RQ_ATTN_BWD_GROUP ? N : RQ_ATTN_BWD_GROUP;
    group<NG, MASK>(tb);
    if constexpr (N > NG) groups<N - NG, MASK>(tb + NG);
  }
  template <int NG, bool MASK>
  __device__ __forceinline__ void group(int tb) {
    constexpr int LD = HD + 4;
    const int g = lane >> 4;
    const float* Qt = Q_s + tb * 16 * LD;
    const float* Ot = O_s + tb * 16 * LD;
    f32x4 s[NG], dp[NG];
#pragma unroll
    for (int t = 0; t < NG; ++t) { s[t] = f32x4{0.f, 0.f, 0.f, 0.f}; dp[t] = f32x4{0.f, 0.f, 0.f, 0.f}; }
    tiles_x_frag2<HD, NG>(Qt, *reinterpret_cast<const float(*)[HD / 4]>(kf), Ot,
                          *reinterpret_cast<const float(*)[HD / 4]>(vf), lane, s, dp);   // S, dP = dO V^T
#pragma unroll
    for (int t = 0; t < NG; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int qr = (tb + t) * 16 + 4 * g + i;
        float p = exp2_fast(__builtin_fmaf(s[t][i], sl2, -lse_s[qr]));
        if constexpr (MASK) {
          const int qq = qc + qr;
          if (!(qq < lq && (!causal || kj <= qq))) p = 0.f;
        }
        s[t][i] = p;
        dp[t][i] = p * (dp[t][i] - dl_s[qr]);   // dS
        dS_s[qr * ldS + col] = kv ? dp[t][i] : 0.f;
      }
    f32x4(&dk_)[HD / 16] = *reinterpret_cast<f32x4(*)[HD / 16]>(dka);
    f32x4(&dv_)[HD / 16] = *reinterpret_cast<f32x4(*)[HD / 16]>(dva);
#pragma unroll
    for (int t = 0; t < NG; ++t) {
      colsT_x_acc<HD>(Ot + t * 16 * LD, s[t], lane, dv_);    // dV^T += dO^T P
      colsT_x_acc<HD>(Qt + t * 16 * LD, dp[t], lane, dk_);   // dK^T += Q^T dS
    }
  }
};

// delta[h][t] = sum_d dO[t][h HD + d] * O[t][h HD + d] over every allocated row (16 lanes per (row, head))
template <int HD>
__global__ void __launch_bounds__(256) attn_delta_kernel(const float* __restrict__ out, int64_t so,
                                                         const float* __restrict__ dout, int64_t sdo, int64_t Tq,
                                                         int64_t H, float* __restrict__ delta) {
  constexpr int LPR = HD / 4 < 16 ? HD / 4 : 16;   // lanes per (row, head)
  constexpr int PER = HD / (4 * LPR);              // float4 per lane
  const int64_t item = ((int64_t)blockIdx.x * 256 + threadIdx.x) / LPR;
  const int sub = threadIdx.x % LPR;
  float acc = 0.f;
  const bool ok = item < Tq * H;
  const int64_t t = ok ? item / H : 0, hh = ok ? item % H : 0;
  if (ok) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int c = (j * LPR + sub) * 4;
      const float4 a = *reinterpret_cast<const float4*>(out + t * so + hh * HD + c);
      const float4 b = *reinterpret_cast<const float4*>(dout + t * sdo + hh * HD + c);
      acc += a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w;
    }
  }
#pragma unroll
  for (int o = LPR / 2; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (ok && sub == 0) delta[hh * Tq + t] = acc;
}

template <int HD, int NW, int CH>
__global__ void __launch_bounds__(64 * NW) attn_bwd_fused_kernel(
    const float* __restrict__ q, int64_t sq, const float* __restrict__ k, int64_t sk, const float* __restrict__ v,
    int64_t sv, const float* __restrict__ dout, int64_t sdo, const float* __restrict__ lse,
    const float* __restrict__ delta, int64_t Tq, const int64_t* __restrict__ cu_q, const int64_t* __restrict__ cu_k,
    int causal, float scale, float* __restrict__ dq, int64_t sdq, float* __restrict__ part, float* __restrict__ dk,
    int64_t sdk, float* __restrict__ dv, int64_t sdv, int64_t Tk, const int* __restrict__ order, int qsplit,
    float* __restrict__ kvpart) {
  constexpr int LD = HD + 4, DT = HD / 16, KB = 16 * NW, NTL = CH / 16, LDS_ = KB + 4;
  constexpr int DSPLIT = NW >= NTL ? NW / NTL : 1, DTW = DT / DSPLIT;
  static_assert(DT % DSPLIT == 0, "dQ split");
  __shared__ __attribute__((aligned(16))) float smem[2 * CH * LD + 2 * CH + KB * LD + CH * LDS_];
  float* Q_s = smem;
  float* O_s = Q_s + CH * LD;   // dO
  float* lse_s = O_s + CH * LD;
  float* dl_s = lse_s + CH;
  float* K_s = dl_s + CH;       // the block's KB key rows (A operand of dQ^T = K^T dS^T)
  float* dS_s = K_s + KB * LD;
  const int z = blockIdx.z, hh = blockIdx.y, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int g = lane >> 4;
  if (z == (int)gridDim.z - 1) {              // tail slice: gradient rows past the last sequence
    zero_rows<HD, 64 * NW>(dk, sdk, cu_k[z], Tk, hh, tid);
    zero_rows<HD, 64 * NW>(dv, sdv, cu_k[z], Tk, hh, tid);
    zero_rows<HD, 64 * NW>(dq, sdq, cu_q[z], Tq, hh, tid);
    return;
  }
  const int b = seq_of(order, z);
  const int64_t q0 = cu_q[b], k0 = cu_k[b];
  const int lq = (int)(cu_q[b + 1] - q0), lk = (int)(cu_k[b + 1] - k0);
  const int kbi = (int)blockIdx.x / qsplit, qs = (int)blockIdx.x - kbi * qsplit;   // key block, query split
  const int kwg = kbi * KB;
  if (kwg >= lk) {
    if (lk == 0) zero_rows<HD, 64 * NW>(dq, sdq, q0, q0 + lq, hh, tid);   // no keys: dQ = 0 (grid-stride over x)
    return;
  }
  const int nkb = (lk + KB - 1) / KB;
  const int kb = kwg + wave * 16, kj = kb + (lane & 15);
  const bool wave_on = kb < lk, kv = kj < lk;
  const int64_t krow = k0 + (kv ? kj : 0);
  float kf[HD / 4], vf[HD / 4];
  load_frag<HD>(k + krow * sk + hh * HD + g * (HD / 4), kv, kf);
  load_frag<HD>(v + krow * sv + hh * HD + g * (HD / 4), kv, vf);
  {
    RowStage<HD, 64 * NW, KB> stk;
    stk.load(k + k0 * sk + hh * HD, sk, kwg, lk, tid);
    stk.store(K_s, tid);                      // published by the first chunk's barrier
  }
  f32x4 dka[DT], dva[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) { dka[dt] = f32x4{0.f, 0.f, 0.f, 0.f}; dva[dt] = f32x4{0.f, 0.f, 0.f, 0.f}; }
  const int qstart = causal ? (kwg / CH) * CH : 0;
  const float* qb_ = q + q0 * sq + hh * HD;
  const float* ob_ = dout + q0 * sdo + hh * HD;
  const float* lse_h = lse + (int64_t)hh * Tq + q0;
  const float* dl_h = delta + (int64_t)hh * Tq + q0;
  const int64_t HH = (int64_t)gridDim.y * HD;
  float* dst;
  int64_t dstride;
  float mul;
  if (nkb == 1) { dst = dq + q0 * sdq + hh * HD; dstride = sdq; mul = scale; }
  else { dst = part + ((int64_t)kbi * Tq + q0) * HH + hh * HD; dstride = HH; mul = 1.f; }
  // query split qs of qsplit: whole CH chunks [c_lo, c_hi) of the block's range (disjoint dQ rows;
  // dK / dV partials per split, summed in split order by attn_kv_reduce_kernel)
  const int nch = lq > qstart ? (lq - qstart + CH - 1) / CH : 0;
  const int c_lo = qstart + (qs * nch / qsplit) * CH;
  const int c_hi = min(lq, qstart + ((qs + 1) * nch / qsplit) * CH);
  RowStage<HD, 64 * NW, CH> stq, sto;
  FusedChunk<HD> fc{Q_s, O_s, lse_s, dl_s, kf, vf, dS_s, lane, 0, 0, lq, kj, causal, wave * 16 + (lane & 15), LDS_, kv,
                    scale * kLog2e, dka, dva};
  // Q / dO / lse / delta of a chunk: global -> registers, then LDS (prefetching the next chunk into
  // registers measured slower: 158 -> 177 VGPRs, 3 -> 2 waves per SIMD, profiles/r03/attn_bwd_prefetch_ab.txt)
  float lse_r = 0.f, dl_r = 0.f;
  auto load_chunk = [&](int qc) {
    stq.load(qb_, sq, qc, lq, tid);
    sto.load(ob_, sdo, qc, lq, tid);
    const bool ok = tid < CH && qc + tid < lq;
    lse_r = ok ? lse_h[qc + tid] * kLog2e : 0.f;
    dl_r = ok ? dl_h[qc + tid] : 0.f;
  };
  for (int qc = c_lo; qc < c_hi; qc += CH) {
    load_chunk(qc);
    __syncthreads();                          // previous chunk's Q/dO/dS reads are done
    stq.store(Q_s, tid);
    sto.store(O_s, tid);
    if (tid < CH) {
      lse_s[tid] = lse_r;
      dl_s[tid] = dl_r;
    }
    __syncthreads();
    const int t0 = __builtin_amdgcn_readfirstlane(causal ? max(0, (kb - qc) >> 4) : 0);
    const int nt = __builtin_amdgcn_readfirstlane(wave_on ? max(0, min(NTL, (lq - qc + 15) >> 4) - t0) : 0);
    // dS columns of tiles this wave does not compute are zero (K_s rows past lk are zero too, but
    // stale LDS could hold NaN bit patterns)
    for (int t = 0; t < NTL; ++t)
      if (t < t0 || t >= t0 + nt)
#pragma unroll
        for (int i = 0; i < 4; ++i) dS_s[(t * 16 + 4 * g + i) * LDS_ + fc.col] = 0.f;
    fc.qc = qc;
    fc.t0 = t0;
    dispatch_tiles<NTL>(nt, !causal && qc + CH <= lq, fc);
    __syncthreads();                          // dS of every wave in LDS
    // dQ^T (16 queries x DTW*16 dims) += K^T dS^T over the block's keys (key tiles past lk are zero)
    const int nkt = __builtin_amdgcn_readfirstlane(min(NW, (lk - kwg + 15) >> 4));
    for (int u = wave; u < NTL * DSPLIT; u += NW) {
      const int qt = u % NTL, d0 = (u / NTL) * DTW;
      if (qc + qt * 16 >= lq) continue;
      f32x4 acc[DTW];
#pragma unroll
      for (int j = 0; j < DTW; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      const float* dsrow = dS_s + (qt * 16 + (lane & 15)) * LDS_ + 4 * g;
      for (int kt = 0; kt < nkt; ++kt) {
        const float4 w4 = *reinterpret_cast<const float4*>(dsrow + kt * 16);
        const float w[4] = {w4.x, w4.y, w4.z, w4.w};
        const float* base = K_s + (kt * 16 + 4 * g) * LD + d0 * 16 + (lane & 15);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < DTW; ++j) acc[j] = mfma4(base[i * LD + j * 16], w[i], acc[j]);
      }
      const int qi = qc + qt * 16 + (lane & 15);
      if (qi < lq) {
        float* rowp = dst + (int64_t)qi * dstride + d0 * 16 + 4 * g;
#pragma unroll
        for (int j = 0; j < DTW; ++j)
          *reinterpret_cast<float4*>(rowp + j * 16) =
              make_float4(acc[j][0] * mul, acc[j][1] * mul, acc[j][2] * mul, acc[j][3] * mul);
      }
    }
  }
  if (!kv) return;
  if (qsplit == 1) {
    store_rowT<HD>(dk + (k0 + kj) * sdk + hh * HD, dka, scale, lane);
    store_rowT<HD>(dv + (k0 + kj) * sdv + hh * HD, dva, 1.f, lane);
  } else {   // partials [2][qsplit][Tk][H HD], unscaled
    store_rowT<HD>(kvpart + (((int64_t)qs * Tk + k0 + kj) * HH + hh * HD), dka, 1.f, lane);
    store_rowT<HD>(kvpart + (((int64_t)(qsplit + qs) * Tk + k0 + kj) * HH + hh * HD), dva, 1.f, lane);
  }
}

// ------------------------------------------------- split-bf16 fused backward (matmul 'high')
// attn_bwd_fused_kernel's schedule (64-key block per workgroup, 32-query chunks, 4 waves of 16 keys, dQ
// from the chunk's dS in LDS) with every product on v_mfma_f32_16x16x32_bf16 over hi / lo pairs: S = Q K^T
// and dP = dO V^T (Q, dO row-major planes x this wave's K / V fragments), dV^T += dO^T P and dK^T += Q^T dS
// (the same Q / dO planes read transposed by ds_read_b64_tr_b16, the chunk's 32 queries in the S
// accumulator's order, x the P / dS values split in registers), dQ^T += K^T dS^T (the block's row-major K
// planes read transposed, keys in that order, x the fp32 dS rows split at the read). One row-major image
// per operand: no transposed copies, no 16-bit scattered stores. P, dS, the softmax statistics and all
// accumulation stay fp32.
template <int NW, int CH>
__global__ void __launch_bounds__(64 * NW) attn_bwd_fused_x3_kernel(
    const float* __restrict__ q, int64_t sq, const float* __restrict__ k, int64_t sk, const float* __restrict__ v,
    int64_t sv, const float* __restrict__ dout, int64_t sdo, const float* __restrict__ lse,
    const float* __restrict__ delta, int64_t Tq, const int64_t* __restrict__ cu_q, const int64_t* __restrict__ cu_k,
    int causal, float scale, float* __restrict__ dq, int64_t sdq, float* __restrict__ part, float* __restrict__ dk,
    int64_t sdk, float* __restrict__ dv, int64_t sdv, int64_t Tk, const int* __restrict__ order, int qsplit,
    float* __restrict__ kvpart) {
  constexpr int HD = 64, DT = 4, KB = 16 * NW, NTL = CH / 16, LDS_ = KB + 4;
  constexpr int DSPLIT = NW >= NTL ? NW / NTL : 1, DTW = DT / DSPLIT;
  static_assert(CH == 32 && NW == 4 && DT % DSPLIT == 0, "split-bf16 fused backward: 32-query chunks, 4 waves");
  constexpr int kRow = CH * kX3Ld, kKr = KB * kX3Ld;   // bf16 per plane
  __shared__ __attribute__((aligned(16))) uint16_t planes[2 * (2 * kRow + kKr)];
  __shared__ __attribute__((aligned(16))) float fsm[CH * LDS_ + 2 * CH];
  uint16_t* const Qh = planes;
  uint16_t* const Ql = Qh + kRow;
  uint16_t* const Oh = Ql + kRow;   // dO
  uint16_t* const Ol = Oh + kRow;
  uint16_t* const Kh = Ol + kRow;
  uint16_t* const Kl = Kh + kKr;
  float* const dS_s = fsm;
  float* const lse_s = dS_s + CH * LDS_;
  float* const dl_s = lse_s + CH;
  const int z = blockIdx.z, hh = blockIdx.y, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int g = lane >> 4, r = lane & 15;
  if (z == (int)gridDim.z - 1) {              // tail slice: gradient rows past the last sequence
    zero_rows<HD, 64 * NW>(dk, sdk, cu_k[z], Tk, hh, tid);
    zero_rows<HD, 64 * NW>(dv, sdv, cu_k[z], Tk, hh, tid);
    zero_rows<HD, 64 * NW>(dq, sdq, cu_q[z], Tq, hh, tid);
    return;
  }
  const int b = seq_of(order, z);
  const int64_t q0 = cu_q[b], k0 = cu_k[b];
  const int lq = (int)(cu_q[b + 1] - q0), lk = (int)(cu_k[b + 1] - k0);
  const int kbi = (int)blockIdx.x / qsplit, qs = (int)blockIdx.x - kbi * qsplit;
  const int kwg = kbi * KB;
  if (kwg >= lk) {
    if (lk == 0) zero_rows<HD, 64 * NW>(dq, sdq, q0, q0 + lq, hh, tid);
    return;
  }
  const int nkb = (lk + KB - 1) / KB;
  const int kb = kwg + wave * 16, kj = kb + r;
  const bool wave_on = kb < lk, kv = kj < lk;
  const int64_t krow = k0 + (kv ? kj : 0);
  abf16x8 kh[2], kl[2], vh[2], vl[2];   // this lane's key row (d = 32 b + 8 g + 0..7)
  x3_load_q(k + krow * sk + hh * HD, kv, lane, kh, kl);
  x3_load_q(v + krow * sv + hh * HD, kv, lane, vh, vl);
  {
    RowStage<HD, 64 * NW, KB> stk;
    stk.load(k + k0 * sk + hh * HD, sk, kwg, lk, tid);
    x3_store_rows<64 * NW, KB>(stk, Kh, Kl, kX3Ld, tid);   // published by the first chunk's barrier
  }
  f32x4 dka[DT], dva[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) { dka[dt] = f32x4{0.f, 0.f, 0.f, 0.f}; dva[dt] = f32x4{0.f, 0.f, 0.f, 0.f}; }
  const int qstart = causal ? (kwg / CH) * CH : 0;
  const float* qb_ = q + q0 * sq + hh * HD;
  const float* ob_ = dout + q0 * sdo + hh * HD;
  const float* lse_h = lse + (int64_t)hh * Tq + q0;
  const float* dl_h = delta + (int64_t)hh * Tq + q0;
  const int64_t HH = (int64_t)gridDim.y * HD;
  float* dst;
  int64_t dstride;
  float mul;
  if (nkb == 1) { dst = dq + q0 * sdq + hh * HD; dstride = sdq; mul = scale; }
  else { dst = part + ((int64_t)kbi * Tq + q0) * HH + hh * HD; dstride = HH; mul = 1.f; }
  const int nch = lq > qstart ? (lq - qstart + CH - 1) / CH : 0;
  const int c_lo = qstart + (qs * nch / qsplit) * CH;
  const int c_hi = min(lq, qstart + ((qs + 1) * nch / qsplit) * CH);
  RowStage<HD, 64 * NW, CH> stq, sto;
  const float sl2 = scale * kLog2e;
  const int col = wave * 16 + r;
  // Q / dO / lse / delta of a chunk: global -> registers, then LDS; the next chunk's loads are issued
  // once the current one is in LDS, so they fly while it is multiplied (no occupancy cost here: the
  // kernel holds 2 waves per SIMD either way)
  float lse_r = 0.f, dl_r = 0.f;
  auto load_chunk = [&](int qc) {
    stq.load(qb_, sq, qc, lq, tid);
    sto.load(ob_, sdo, qc, lq, tid);
    const bool ok = tid < CH && qc + tid < lq;
    lse_r = ok ? lse_h[qc + tid] * kLog2e : 0.f;
    dl_r = ok ? dl_h[qc + tid] : 0.f;
  };
  if (c_lo < c_hi) load_chunk(c_lo);
  for (int qc = c_lo; qc < c_hi; qc += CH) {
    __syncthreads();                          // previous chunk's plane / dS reads are done
    x3_store_rows<64 * NW, CH>(stq, Qh, Ql, kX3Ld, tid);
    x3_store_rows<64 * NW, CH>(sto, Oh, Ol, kX3Ld, tid);
    if (tid < CH) {
      lse_s[tid] = lse_r;
      dl_s[tid] = dl_r;
    }
    __syncthreads();
    if (qc + CH < c_hi) load_chunk(qc + CH);
    const int t0 = __builtin_amdgcn_readfirstlane(causal ? max(0, (kb - qc) >> 4) : 0);
    const int nt = __builtin_amdgcn_readfirstlane(wave_on ? max(0, min(NTL, (lq - qc + 15) >> 4) - t0) : 0);
    f32x4 s[NTL], dp[NTL];
#pragma unroll
    for (int t = 0; t < NTL; ++t) {
      s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      dp[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      const bool on = t >= t0 && t < t0 + nt;
      if (on) {
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {   // S = Q K^T, dP = dO V^T: rows = queries, columns = keys
          const int off = (16 * t + r) * kX3Ld + 32 * bb + 8 * g;
          const abf16x8 ah = *reinterpret_cast<const abf16x8*>(Qh + off), al = *reinterpret_cast<const abf16x8*>(Ql + off);
          const abf16x8 oh = *reinterpret_cast<const abf16x8*>(Oh + off), ol = *reinterpret_cast<const abf16x8*>(Ol + off);
          s[t] = mfma_x3(ah, al, kh[bb], kl[bb], s[t]);
          dp[t] = mfma_x3(oh, ol, vh[bb], vl[bb], dp[t]);
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int qr = t * 16 + 4 * g + i;
        const int qq = qc + qr;
        float p = exp2_fast(__builtin_fmaf(s[t][i], sl2, -lse_s[qr]));
        if (!(on && qq < lq && (!causal || kj <= qq))) p = 0.f;
        s[t][i] = p;
        dp[t][i] = p * (dp[t][i] - dl_s[qr]);   // dS
        dS_s[qr * LDS_ + col] = kv ? dp[t][i] : 0.f;
      }
    }
    {   // dV^T += dO^T P, dK^T += Q^T dS over the chunk's 32 queries (the accumulator's order)
      float p8[8], d8[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        p8[i] = s[0][i];
        p8[4 + i] = s[1][i];
        d8[i] = dp[0][i];
        d8[4 + i] = dp[1][i];
      }
      abf16x8 ph, pl, dh, dl;
      split8(p8, ph, pl);
      split8(d8, dh, dl);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const abf16x8 oth = x3_tr_frag(Oh, kX3Ld, 0, 16 * dt, lane), otl = x3_tr_frag(Ol, kX3Ld, 0, 16 * dt, lane);
        const abf16x8 qth = x3_tr_frag(Qh, kX3Ld, 0, 16 * dt, lane), qtl = x3_tr_frag(Ql, kX3Ld, 0, 16 * dt, lane);
        dva[dt] = mfma_x3(oth, otl, ph, pl, dva[dt]);
        dka[dt] = mfma_x3(qth, qtl, dh, dl, dka[dt]);
      }
    }
    __syncthreads();                          // dS of every wave in LDS
    // dQ^T (16 queries x DTW*16 dims) += K^T dS^T over the block's keys in the x3 order of each 32-key block
    // (keys past lk: zero K rows, zero dS)
    const int nkk = __builtin_amdgcn_readfirstlane((min(NW, (lk - kwg + 15) >> 4) + 1) >> 1);   // 32-key blocks
    for (int u = wave; u < NTL * DSPLIT; u += NW) {
      const int qt = u % NTL, d0 = (u / NTL) * DTW;
      if (qc + qt * 16 >= lq) continue;
      f32x4 acc[DTW];
#pragma unroll
      for (int j = 0; j < DTW; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int kk = 0; kk < nkk; ++kk) {
        const float* dsrow = dS_s + (qt * 16 + r) * LDS_ + 32 * kk + 4 * g;
        const float4 x = *reinterpret_cast<const float4*>(dsrow), y = *reinterpret_cast<const float4*>(dsrow + 16);
        const float w8[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
        abf16x8 wh, wl;
        split8(w8, wh, wl);
#pragma unroll
        for (int j = 0; j < DTW; ++j) {
          const abf16x8 th = x3_tr_frag(Kh, kX3Ld, 32 * kk, 16 * (d0 + j), lane);
          const abf16x8 tl = x3_tr_frag(Kl, kX3Ld, 32 * kk, 16 * (d0 + j), lane);
          acc[j] = mfma_x3(th, tl, wh, wl, acc[j]);
        }
      }
      const int qi = qc + qt * 16 + r;
      if (qi < lq) {
        float* rowp = dst + (int64_t)qi * dstride + d0 * 16 + 4 * g;
#pragma unroll
        for (int j = 0; j < DTW; ++j)
          *reinterpret_cast<float4*>(rowp + j * 16) =
              make_float4(acc[j][0] * mul, acc[j][1] * mul, acc[j][2] * mul, acc[j][3] * mul);
      }
    }
  }
  if (!kv) return;
  if (qsplit == 1) {
    store_rowT<HD>(dk + (k0 + kj) * sdk + hh * HD, dka, scale, lane);
    store_rowT<HD>(dv + (k0 + kj) * sdv + hh * HD, dva, 1.f, lane);
  } else {   // partials [2][qsplit][Tk][H HD], unscaled
    store_rowT<HD>(kvpart + (((int64_t)qs * Tk + k0 + kj) * HH + hh * HD), dka, 1.f, lane);
    store_rowT<HD>(kvpart + (((int64_t)(qsplit + qs) * Tk + k0 + kj) * HH + hh * HD), dva, 1.f, lane);
  }
}

// dK = scale * sum_s dK_s, dV = sum_s dV_s over the fused backward's query splits, in split order
// (deterministic), rows < cu_k[B] (the bucket tail was zeroed by the fused kernel's tail slice).


// dQ rows of sequences with more than one key block: scale * sum over key blocks (in block order) of
// the fused kernel's partials. Causal: query r sees key blocks kb <= r / KB only (the others never
// wrote row r). One thread per float4 of a (row, head) slice; grid (row blocks of 16, H, B).
template <int HD, int KB>
__global__ void __launch_bounds__(256) attn_dq_reduce_kernel(const float* __restrict__ part, int64_t Tq,
                                                             const int64_t* __restrict__ cu_q,
                                                             const int64_t* __restrict__ cu_k, int causal, float scale,
                                                             float* __restrict__ dq, int64_t sdq) {
  constexpr int F4 = HD / 4, RPB = 256 / F4;   // rows per block
  const int b = blockIdx.z, hh = blockIdx.y;
  const int64_t q0 = cu_q[b];
  const int lq = (int)(cu_q[b + 1] - q0), lk = (int)(cu_k[b + 1] - cu_k[b]);
  const int nkb = (lk + KB - 1) / KB;
  if (nkb <= 1) return;                        // written directly by the fused kernel
  const int r = blockIdx.x * RPB + threadIdx.x / F4, c = (threadIdx.x % F4) * 4;
  if (r >= lq) return;
  const int n = causal ? min(nkb, r / KB + 1) : nkb;
  const int64_t HH = (int64_t)gridDim.y * HD;
  const float* p = part + (q0 + r) * HH + hh * HD + c;
  const int64_t slab = Tq * HH;
  float4 s = *reinterpret_cast<const float4*>(p);
  for (int j = 1; j < n; ++j) {
    const float4 a = *reinterpret_cast<const float4*>(p + j * slab);
    s.x += a.x; s.y += a.y; s.z += a.z; s.w += a.w;
  }
  *reinterpret_cast<float4*>(dq + (q0 + r) * sdq + hh * HD + c) =
      make_float4(s.x * scale, s.y * scale, s.z * scale, s.w * scale);
}

// ------------------------------------------------------------------------ short sequences
// Short-sequence forms (the decoder's Amazon contexts, <= 81 tokens, and its 5 future tokens): one
// workgroup per (sequence, head) stages the head's WHOLE key range (forward, dQ) or query range (dK/dV)
// through LDS in a single round trip — every load of the stage in flight at once, one barrier — and
// its NW waves then run their 16-row tiles (wave w: tiles w, w + NW, ...) against every staged tile.
// The chunked kernels above stage 32 rows per round trip and re-stage K/V once per 32-query
// workgroup; at n ~ 45 that is 2-3 serial round trips per workgroup and 2-3 workgroups per head.
// CH = staged rows (>= the longest range, multiple of 16, <= 128).
// Stage rows [0, CH) of a strided source (rows >= n zero) into LDS [CH][HD+4] with NT threads, in
// pieces of at most 8 float4 per thread per source (a one-wave workgroup staging 96 rows at once would
// hold 24 float4 per source in VGPRs and drop to one wave per SIMD).
template <int HD, int NT, int CH>
__device__ __forceinline__ void stage2(const float* __restrict__ a, int64_t sa, const float* __restrict__ b, int64_t sb,
                                       int n, float* da, float* db, int tid) {
  constexpr int PIECE = CH * (HD / 4) <= 8 * NT ? CH : (8 * NT) / (HD / 4);
  static_assert(CH % PIECE == 0, "piece");
#pragma unroll
  for (int r0 = 0; r0 < CH; r0 += PIECE) {
    RowStage<HD, NT, PIECE> sta, stb;
    sta.load(a, sa, r0, n, tid);
    stb.load(b, sb, r0, n, tid);
    sta.store(da + r0 * (HD + 4), tid);
    stb.store(db + r0 * (HD + 4), tid);
  }
}

template <int NTL, typename F>
__device__ __forceinline__ void dispatch_short(int nt, F& f) {
  switch (nt) {
    case 1: f.template run<1, true>(); break;
    case 2: if constexpr (NTL >= 2) f.template run<2, true>(); break;
    case 3: if constexpr (NTL >= 3) f.template run<3, true>(); break;
    case 4: if constexpr (NTL >= 4) f.template run<4, true>(); break;
    case 5: if constexpr (NTL >= 5) f.template run<5, true>(); break;
    case 6: if constexpr (NTL >= 6) f.template run<6, true>(); break;
    case 7: if constexpr (NTL >= 7) f.template run<7, true>(); break;
    case 8: if constexpr (NTL >= 8) f.template run<8, true>(); break;
    default: break;
  }
}

template <int HD, int NW, int CH>
__global__ void __launch_bounds__(64 * NW) attn_fwd_short_kernel(
    const float* __restrict__ q, int64_t sq, const float* __restrict__ k, int64_t sk, const float* __restrict__ v,
    int64_t sv, const int64_t* __restrict__ cu_q, const int64_t* __restrict__ cu_k, int causal, float scale,
    float* __restrict__ out, int64_t so, float* __restrict__ lse, int64_t Tq) {
  constexpr int LD = HD + 4, DT = HD / 16, NTL = CH / 16;
  __shared__ __attribute__((aligned(16))) float smem[2 * CH * LD];
  float* K_s = smem;
  float* V_s = smem + CH * LD;
  const int b = blockIdx.z, hh = blockIdx.y, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int g = lane >> 4;
  if (b == (int)gridDim.z - 1) {
    zero_rows<HD, 64 * NW>(out, so, cu_q[b], Tq, hh, tid);
    return;
  }
  const int64_t q0 = cu_q[b], k0 = cu_k[b];
  const int lq = (int)(cu_q[b + 1] - q0), lk = (int)(cu_k[b + 1] - k0);
  if (lq <= 0) return;
  stage2<HD, 64 * NW, CH>(k + k0 * sk + hh * HD, sk, v + k0 * sv + hh * HD, sv, lk, K_s, V_s, tid);
  __syncthreads();
  const float sl2 = scale * kLog2e;
  for (int qt = wave; qt * 16 < lq; qt += NW) {
    const int qb = qt * 16, qi = qb + (lane & 15);
    const bool qv = qi < lq;
    float qf[HD / 4];
    load_frag<HD>(q + (q0 + (qv ? qi : 0)) * sq + hh * HD + g * (HD / 4), qv, qf);
    f32x4 o[DT];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m = -INFINITY, l = 0.f;
    const int kend = causal ? min(lk, qb + 16) : lk;
    const int nt = __builtin_amdgcn_readfirstlane((kend + 15) >> 4);
    FwdChunk<HD> fc{K_s, V_s, qf, lane, 0, lk, qi, causal, sl2, &m, &l, o};
    dispatch_short<NTL>(nt, fc);
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    if (qv) {
      store_rowT<HD>(out + (q0 + qi) * so + hh * HD, o, l > 0.f ? 1.f / l : 0.f, lane);
      if (g == 0) lse[(int64_t)hh * Tq + q0 + qi] = l > 0.f ? (m + log2f(l)) * kLn2 : 0.f;
    }
  }
}

template <int HD, int NW, int CH>
__global__ void __launch_bounds__(64 * NW) attn_bwd_dq_short_kernel(
    const float* __restrict__ q, int64_t sq, const float* __restrict__ k, int64_t sk, const float* __restrict__ v,
    int64_t sv, const float* __restrict__ out, int64_t so, const float* __restrict__ dout, int64_t sdo,
    const float* __restrict__ lse, int64_t Tq, const int64_t* __restrict__ cu_q, const int64_t* __restrict__ cu_k,
    int causal, float scale, float* __restrict__ dq, int64_t sdq, float* __restrict__ delta_out) {
  constexpr int LD = HD + 4, DT = HD / 16, NTL = CH / 16;
  __shared__ __attribute__((aligned(16))) float smem[2 * CH * LD];
  float* K_s = smem;
  float* V_s = smem + CH * LD;
  const int b = blockIdx.z, hh = blockIdx.y, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int g = lane >> 4;
  if (b == (int)gridDim.z - 1) {
    zero_rows<HD, 64 * NW>(dq, sdq, cu_q[b], Tq, hh, tid);
    return;
  }
  const int64_t q0 = cu_q[b], k0 = cu_k[b];
  const int lq = (int)(cu_q[b + 1] - q0), lk = (int)(cu_k[b + 1] - k0);
  if (lq <= 0) return;
  stage2<HD, 64 * NW, CH>(k + k0 * sk + hh * HD, sk, v + k0 * sv + hh * HD, sv, lk, K_s, V_s, tid);
  __syncthreads();
  const float sl2 = scale * kLog2e;
  for (int qt = wave; qt * 16 < lq; qt += NW) {
    const int qb = qt * 16, qi = qb + (lane & 15);
    const bool qv = qi < lq;
    const int64_t qrow = q0 + (qv ? qi : 0);
    float qf[HD / 4], dof[HD / 4];
    load_frag<HD>(q + qrow * sq + hh * HD + g * (HD / 4), qv, qf);
    load_frag<HD>(dout + qrow * sdo + hh * HD + g * (HD / 4), qv, dof);
    float delta = 0.f;
    {
      float of[HD / 4];
      load_frag<HD>(out + qrow * so + hh * HD + g * (HD / 4), qv, of);
#pragma unroll
      for (int d = 0; d < HD / 4; ++d) delta += dof[d] * of[d];
      delta += __shfl_xor(delta, 16, 64);
      delta += __shfl_xor(delta, 32, 64);
      if (qv && g == 0) delta_out[(int64_t)hh * Tq + qrow] = delta;
    }
    f32x4 acc[DT];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) acc[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int kend = causal ? min(lk, qb + 16) : lk;
    const int nt = __builtin_amdgcn_readfirstlane((kend + 15) >> 4);
    DqChunk<HD> fc{K_s, V_s, qf, dof, lane, 0, lk, qi, causal, sl2,
                   qv ? lse[(int64_t)hh * Tq + qrow] * kLog2e : 0.f, delta, acc};
    dispatch_short<NTL>(nt, fc);
    if (qv) store_rowT<HD>(dq + (q0 + qi) * sdq + hh * HD, acc, scale, lane);
  }
}

template <int HD, int NW, int CH>
__global__ void __launch_bounds__(64 * NW) attn_bwd_dkdv_short_kernel(
    const float* __restrict__ q, int64_t sq, const float* __restrict__ k, int64_t sk, const float* __restrict__ v,
    int64_t sv, const float* __restrict__ dout, int64_t sdo, const float* __restrict__ lse,
    const float* __restrict__ delta, int64_t Tq, const int64_t* __restrict__ cu_q, const int64_t* __restrict__ cu_k,
    int causal, float scale, float* __restrict__ dk, int64_t sdk, float* __restrict__ dv, int64_t sdv, int64_t Tk) {
  constexpr int LD = HD + 4, DT = HD / 16, NTL = CH / 16;
  __shared__ __attribute__((aligned(16))) float smem[2 * CH * LD + 2 * CH];
  float* Q_s = smem;
  float* O_s = smem + CH * LD;   // dO
  float* lse_s = O_s + CH * LD;
  float* dl_s = lse_s + CH;
  const int b = blockIdx.z, hh = blockIdx.y, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int g = lane >> 4;
  if (b == (int)gridDim.z - 1) {
    zero_rows<HD, 64 * NW>(dk, sdk, cu_k[b], Tk, hh, tid);
    zero_rows<HD, 64 * NW>(dv, sdv, cu_k[b], Tk, hh, tid);
    return;
  }
  const int64_t q0 = cu_q[b], k0 = cu_k[b];
  const int lq = (int)(cu_q[b + 1] - q0), lk = (int)(cu_k[b + 1] - k0);
  if (lk <= 0) return;
  for (int r = tid; r < CH; r += 64 * NW) {
    const bool ok = r < lq;
    lse_s[r] = ok ? lse[(int64_t)hh * Tq + q0 + r] * kLog2e : 0.f;
    dl_s[r] = ok ? delta[(int64_t)hh * Tq + q0 + r] : 0.f;
  }
  stage2<HD, 64 * NW, CH>(q + q0 * sq + hh * HD, sq, dout + q0 * sdo + hh * HD, sdo, lq, Q_s, O_s, tid);
  __syncthreads();
  const float sl2 = scale * kLog2e;
  const int nqt = (lq + 15) >> 4;
  for (int kt = wave; kt * 16 < lk; kt += NW) {
    const int kb = kt * 16, kj = kb + (lane & 15);
    const bool kv = kj < lk;
    const int64_t krow = k0 + (kv ? kj : 0);
    float kf[HD / 4], vf[HD / 4];
    load_frag<HD>(k + krow * sk + hh * HD + g * (HD / 4), kv, kf);
    load_frag<HD>(v + krow * sv + hh * HD + g * (HD / 4), kv, vf);
    f32x4 dka[DT], dva[DT];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) { dka[dt] = f32x4{0.f, 0.f, 0.f, 0.f}; dva[dt] = f32x4{0.f, 0.f, 0.f, 0.f}; }
    const int t0 = __builtin_amdgcn_readfirstlane(causal ? (kb >> 4) : 0);   // query tiles wholly before the keys
    const int nt = __builtin_amdgcn_readfirstlane(nqt - t0);
    DkdvChunk<HD> fc{Q_s, O_s, lse_s, dl_s, kf, vf, lane, 0, t0, lq, kj, causal, sl2, dka, dva};
    dispatch_short<NTL>(nt, fc);
    if (kv) {
      store_rowT<HD>(dk + (k0 + kj) * sdk + hh * HD, dka, scale, lane);
      store_rowT<HD>(dv + (k0 + kj) * sdv + hh * HD, dva, 1.f, lane);
    }
  }
}

// ----------------------------------------------------------- LDS-DMA staged short forms (HD = 64)
// One workgroup of NW waves per (sequence, head) whose key range (forward) fits R <= 128 rows: the
// head's K and V rows go global -> LDS by LDS-DMA (global_load_lds_dwordx4: no VGPR round trip, no
// staging VALU, every row of the head in flight at once), one wait + barrier, then each wave runs its
// 16-query tiles (w, w + NW, ...) against ALL key tiles in one pass: the whole S^T row block of a query
// tile stays in registers, so its max and sum are exact (no running rescale of O).
// LDS image: a row of 64 fp32 (256 B = 16 chunks of 16 B) per key, no padding; chunk c of row r sits at
// position c ^ swz(r) (the XOR goes on each DMA lane's SOURCE address, the LDS side of a DMA is
// lane-linear: lane L of an instruction writes position L & 15 of row 4j + (L >> 4)). swz keeps both
// fragment reads conflict-free (checked per ds_read_b128 lane group):
//   K pattern  S^T = K Q^T:  lane (row = lane & 15, chunk = 4 (lane >> 4) + s), s = 0..3
//   V pattern  O^T += V^T P^T: lane (row = 4 (lane >> 4) + i, chunk = lane & 15),  i = 0..3
// The V product runs over a PERMUTED d: accumulator tile dt, row m holds d = 4 m + dt, so one
// ds_read_b128 of V[key][4m .. 4m+3] feeds the 4 output tiles; each lane then owns the 16 contiguous
// d = 16 (lane >> 4) + 4 i + dt of its query — whole float4 stores.
// Rows past the sequence read its last row (finite data: masked keys get P = 0; never read past it).
__device__ __forceinline__ int swz16(int r) {
  r &= 15;
  return r ^ ((((r >> 2) ^ (r >> 3)) & 1) << 2);
}

__device__ __forceinline__ void glds16f(const float* src, char* lds_dst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_dst, 16, 0, 0);
}

// DMA rows [0, 16 nt) of two strided row sources (rows >= n read row n - 1) into two swizzled LDS images,
// instruction j (4 rows) by wave j % NW.
template <int NW>
__device__ __forceinline__ void dma_rows2(const float* __restrict__ a, int64_t sa, const float* __restrict__ b,
                                          int64_t sb, int n, int nt, char* da, char* db, int wave, int lane) {
  const int ninstr = 4 * nt;
  for (int j = wave; j < ninstr; j += NW) {
    const int r = 4 * j + (lane >> 4);
    const int64_t rr = min(r, n - 1);
    const int c = (lane & 15) ^ swz16(r);
    glds16f(a + rr * sa + 4 * c, da + j * 1024);
    glds16f(b + rr * sb + 4 * c, db + j * 1024);
  }
}

// float4 at chunk c of image row r
__device__ __forceinline__ float4 lds_chunk(const char* img, int r, int c) {
  return *reinterpret_cast<const float4*>(img + r * 256 + ((c ^ swz16(r)) << 4));
}

// One query tile of the DMA forward against its N key tiles (compile-time N: every array in registers).
template <int N>
__device__ __forceinline__ void fwd_dma_tile(const char* K_s, const char* V_s, const float (&qf)[16], int lane, int lk,
                                             int qi, int causal, float sl2, f32x4 (&o)[4], float& mn_out, float& l_out) {
  const int g = lane >> 4;
  f32x4 st[N];
#pragma unroll
  for (int t = 0; t < N; ++t) st[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  // S^T (keys on rows): N independent MFMA chains
#pragma unroll
  for (int s4 = 0; s4 < 4; ++s4) {
    float4 a[N];
#pragma unroll
    for (int t = 0; t < N; ++t) a[t] = lds_chunk(K_s, t * 16 + (lane & 15), 4 * g + s4);
#pragma unroll
    for (int t = 0; t < N; ++t) {
      st[t] = mfma4(a[t].x, qf[4 * s4], st[t]);
      st[t] = mfma4(a[t].y, qf[4 * s4 + 1], st[t]);
      st[t] = mfma4(a[t].z, qf[4 * s4 + 2], st[t]);
      st[t] = mfma4(a[t].w, qf[4 * s4 + 3], st[t]);
    }
  }
  // exact row max / sum over every key of the query (keys >= lk, causal keys > query: masked)
  float mt = -INFINITY;
#pragma unroll
  for (int t = 0; t < N; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int key = t * 16 + 4 * g + i;
      if (!(key < lk && (!causal || key <= qi))) st[t][i] = -INFINITY;
      mt = fmaxf(mt, st[t][i]);
    }
  mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
  mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
  const float mn = mt * sl2;
  const bool none = mn == -INFINITY;          // no key (padding query rows, empty key range)
  float l = 0.f;
#pragma unroll
  for (int t = 0; t < N; ++t) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      st[t][i] = none ? 0.f : exp2_fast(__builtin_fmaf(st[t][i], sl2, -mn));
      l += st[t][i];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {             // O^T += V^T P^T, d permuted
      const float4 vv = lds_chunk(V_s, t * 16 + 4 * g + i, lane & 15);
      o[0] = mfma4(vv.x, st[t][i], o[0]);
      o[1] = mfma4(vv.y, st[t][i], o[1]);
      o[2] = mfma4(vv.z, st[t][i], o[2]);
      o[3] = mfma4(vv.w, st[t][i], o[3]);
    }
  }
  mn_out = mn;
  l_out = l;
}

template <int NW, int R>
__global__ void __launch_bounds__(64 * NW, R <= 64 ? 4 : 3) attn_fwd_dma_kernel(
    const float* __restrict__ q, int64_t sq, const float* __restrict__ k, int64_t sk, const float* __restrict__ v,
    int64_t sv, const int64_t* __restrict__ cu_q, const int64_t* __restrict__ cu_k, int causal, float scale,
    float* __restrict__ out, int64_t so, float* __restrict__ lse, int64_t Tq) {
  constexpr int HD = 64, NKT = R / 16;
  static_assert(R % 16 == 0 && R <= 128, "staged rows");
  __shared__ __attribute__((aligned(16))) char lds[2 * R * 256];
  char* K_s = lds;
  char* V_s = lds + R * 256;
  const int b = blockIdx.z, hh = blockIdx.y, tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;
  if (b == (int)gridDim.z - 1) {              // tail slice: output rows past the last sequence
    zero_rows<HD, 64 * NW>(out, so, cu_q[b], Tq, hh, tid);
    return;
  }
  const int64_t q0 = cu_q[b], k0 = cu_k[b];
  const int lq = (int)(cu_q[b + 1] - q0), lk = (int)(cu_k[b + 1] - k0);
  if (lq <= 0) return;
  const int nkt_all = min((lk + 15) >> 4, NKT);   // lk <= max_k <= R by the plan; never stage past the image
  if (lk > 0) dma_rows2<NW>(k + k0 * sk + hh * HD, sk, v + k0 * sv + hh * HD, sv, lk, nkt_all, K_s, V_s, wave, lane);
  const float sl2 = scale * kLog2e;
  const int nqt = (lq + 15) >> 4;
  float qf[HD / 4];
  if (wave < nqt) {   // the first tile's Q rows fly with the DMAs
    const int qi = wave * 16 + (lane & 15);
    load_frag<HD>(q + (q0 + (qi < lq ? qi : 0)) * sq + hh * HD + g * (HD / 4), qi < lq, qf);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMAs (and Q) landed
  __syncthreads();                                     // ... and every other wave's
  for (int qt = wave; qt < nqt; qt += NW) {
    const int qb = qt * 16, qi = qb + (lane & 15);
    const bool qv = qi < lq;
    if (qt != wave) load_frag<HD>(q + (q0 + (qv ? qi : 0)) * sq + hh * HD + g * (HD / 4), qv, qf);
    const int kend = causal ? min(lk, qb + 16) : lk;
    const int nkt = __builtin_amdgcn_readfirstlane(min((kend + 15) >> 4, NKT));
    f32x4 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    float mn = -INFINITY, l = 0.f;
    switch (nkt) {
      case 1: fwd_dma_tile<1>(K_s, V_s, qf, lane, lk, qi, causal, sl2, o, mn, l); break;
      case 2: if constexpr (NKT >= 2) fwd_dma_tile<2>(K_s, V_s, qf, lane, lk, qi, causal, sl2, o, mn, l); break;
      case 3: if constexpr (NKT >= 3) fwd_dma_tile<3>(K_s, V_s, qf, lane, lk, qi, causal, sl2, o, mn, l); break;
      case 4: if constexpr (NKT >= 4) fwd_dma_tile<4>(K_s, V_s, qf, lane, lk, qi, causal, sl2, o, mn, l); break;
      case 5: if constexpr (NKT >= 5) fwd_dma_tile<5>(K_s, V_s, qf, lane, lk, qi, causal, sl2, o, mn, l); break;
      case 6: if constexpr (NKT >= 6) fwd_dma_tile<6>(K_s, V_s, qf, lane, lk, qi, causal, sl2, o, mn, l); break;
      case 7: if constexpr (NKT >= 7) fwd_dma_tile<7>(K_s, V_s, qf, lane, lk, qi, causal, sl2, o, mn, l); break;
      case 8: if constexpr (NKT >= 8) fwd_dma_tile<8>(K_s, V_s, qf, lane, lk, qi, causal, sl2, o, mn, l); break;
      default: break;                         // no key: zero output, lse 0
    }
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    if (qv) {
      const float inv = l > 0.f ? 1.f / l : 0.f;
      float* orow = out + (q0 + qi) * so + hh * HD + 16 * g;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        *reinterpret_cast<float4*>(orow + 4 * i) = make_float4(o[0][i] * inv, o[1][i] * inv, o[2][i] * inv, o[3][i] * inv);
      if (g == 0) lse[(int64_t)hh * Tq + q0 + qi] = l > 0.f ? (mn + log2f(l)) * kLn2 : 0.f;
    }
  }
}

// Split-bf16 form of the short forward (matmul 'high'): the head's K and V rows (<= R) staged once as
// row-major hi / lo planes, each wave's 16-query tiles (w, w + 4, ...) run FwdChunkX3 over ALL key tiles in
// one pass (a single chunk from m = -inf: the max and sum are exact, as in attn_fwd_dma_kernel).
template <int R>
__global__ void __launch_bounds__(256) attn_fwd_short_x3_kernel(
    const float* __restrict__ q, int64_t sq, const float* __restrict__ k, int64_t sk, const float* __restrict__ v,
    int64_t sv, const int64_t* __restrict__ cu_q, const int64_t* __restrict__ cu_k, int causal, float scale,
    float* __restrict__ out, int64_t so, float* __restrict__ lse, int64_t Tq, const int* __restrict__ order) {
  constexpr int HD = 64, NW = 4, NKT = R / 16;
  static_assert(R % 32 == 0 && R <= 128, "staged rows");
  __shared__ __attribute__((aligned(16))) uint16_t planes[4 * R * kX3Ld];
  uint16_t* const Kh = planes;
  uint16_t* const Kl = Kh + R * kX3Ld;
  uint16_t* const Vh = Kl + R * kX3Ld;
  uint16_t* const Vl = Vh + R * kX3Ld;
  const int z = blockIdx.z, hh = blockIdx.y, tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;
  if (z == (int)gridDim.z - 1) {              // tail slice: output rows past the last sequence
    zero_rows<HD, 256>(out, so, cu_q[z], Tq, hh, tid);
    return;
  }
  const int b = seq_of(order, z);   // longest-first when an LPT order is given
  const int64_t q0 = cu_q[b], k0 = cu_k[b];
  const int lq = (int)(cu_q[b + 1] - q0), lk = (int)(cu_k[b + 1] - k0);
  if (lq <= 0) return;
  {
    RowStage<HD, 256, R> stk, stv;   // rows past lk are zero
    stk.load(k + k0 * sk + hh * HD, sk, 0, lk, tid);
    stv.load(v + k0 * sv + hh * HD, sv, 0, lk, tid);
    x3_store_rows<256, R>(stk, Kh, Kl, kX3Ld, tid);
    x3_store_rows<256, R>(stv, Vh, Vl, kX3Ld, tid);
  }
  __syncthreads();
  const float sl2 = scale * kLog2e;
  const int nqt = (lq + 15) >> 4;
  for (int qt = wave; qt < nqt; qt += NW) {
    const int qi = qt * 16 + (lane & 15);
    const bool qv = qi < lq;
    abf16x8 qh[2], ql[2];
    x3_load_q(q + (q0 + (qv ? qi : 0)) * sq + hh * HD, qv, lane, qh, ql);
    const int kend = causal ? min(lk, qt * 16 + 16) : lk;
    const int nkt = __builtin_amdgcn_readfirstlane(min((kend + 15) >> 4, NKT));
    f32x4 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m = -INFINITY, l = 0.f;
    FwdChunkX3 fx{Kh, Kl, Vh, Vl, qh, ql, lane, 0, lk, qi, causal, sl2, &m, &l, o};
    switch (nkt) {
      case 1: fx.run<1, true>(); break;
      case 2: fx.run<2, true>(); break;
      case 3: if constexpr (NKT >= 3) fx.run<3, true>(); break;
      case 4: if constexpr (NKT >= 4) fx.run<4, true>(); break;
      case 5: if constexpr (NKT >= 5) fx.run<5, true>(); break;
      case 6: if constexpr (NKT >= 6) fx.run<6, true>(); break;
      case 7: if constexpr (NKT >= 7) fx.run<7, true>(); break;
      case 8: if constexpr (NKT >= 8) fx.run<8, true>(); break;
      default: break;                         // no key: zero output, lse 0
    }
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    if (qv) {
      const float inv = l > 0.f ? 1.f / l : 0.f;
      store_rowT<HD>(out + (q0 + qi) * so + hh * HD, o, inv, lane);
      if (g == 0) lse[(int64_t)hh * Tq + q0 + qi] = l > 0.f ? (m + log2f(l)) * kLn2 : 0.f;
    }
  }
}

// dQ of one query tile against its N key tiles (DMA images of K and V): S^T and dP^T = V dO^T per key
// tile (K pattern), P from the saved lse, dS^T = P (dP^T - delta), dQ^T += K^T dS^T (V pattern, d permuted).
template <int N>
__device__ __forceinline__ void dq_dma_tile(const char* K_s, const char* V_s, const float (&qf)[16],
                                            const float (&dof)[16], int lane, int lk, int qi, int causal, float sl2,
                                            float lse2, float delta, f32x4 (&acc)[4]) {
  const int g = lane >> 4;
  f32x4 st[N], dp[N];
#pragma unroll
  for (int t = 0; t < N; ++t) { st[t] = f32x4{0.f, 0.f, 0.f, 0.f}; dp[t] = f32x4{0.f, 0.f, 0.f, 0.f}; }
#pragma unroll
  for (int s4 = 0; s4 < 4; ++s4) {
    float4 a[N], c[N];
#pragma unroll
    for (int t = 0; t < N; ++t) {
      a[t] = lds_chunk(K_s, t * 16 + (lane & 15), 4 * g + s4);
      c[t] = lds_chunk(V_s, t * 16 + (lane & 15), 4 * g + s4);
    }
#pragma unroll
    for (int t = 0; t < N; ++t) {
      st[t] = mfma4(a[t].x, qf[4 * s4], st[t]);
      dp[t] = mfma4(c[t].x, dof[4 * s4], dp[t]);
      st[t] = mfma4(a[t].y, qf[4 * s4 + 1], st[t]);
      dp[t] = mfma4(c[t].y, dof[4 * s4 + 1], dp[t]);
      st[t] = mfma4(a[t].z, qf[4 * s4 + 2], st[t]);
      dp[t] = mfma4(c[t].z, dof[4 * s4 + 2], dp[t]);
      st[t] = mfma4(a[t].w, qf[4 * s4 + 3], st[t]);
      dp[t] = mfma4(c[t].w, dof[4 * s4 + 3], dp[t]);
    }
  }
#pragma unroll
  for (int t = 0; t < N; ++t) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int key = t * 16 + 4 * g + i;
      float p = exp2_fast(__builtin_fmaf(st[t][i], sl2, -lse2));
      if (!(key < lk && (!causal || key <= qi))) p = 0.f;
      st[t][i] = p * (dp[t][i] - delta);      // dS^T
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {             // dQ^T += K^T dS^T
      const float4 kk = lds_chunk(K_s, t * 16 + 4 * g + i, lane & 15);
      acc[0] = mfma4(kk.x, st[t][i], acc[0]);
      acc[1] = mfma4(kk.y, st[t][i], acc[1]);
      acc[2] = mfma4(kk.z, st[t][i], acc[2]);
      acc[3] = mfma4(kk.w, st[t][i], acc[3]);
    }
  }
}

// dQ (+ delta = rowsum(dO * O), saved for the dK/dV pass): one workgroup per (sequence, head), K / V by
// LDS-DMA, waves over 16-query tiles against every key tile.
template <int NW, int R>
__global__ void __launch_bounds__(64 * NW, R <= 64 ? 4 : 3) attn_bwd_dq_dma_kernel(
    const float* __restrict__ q, int64_t sq, const float* __restrict__ k, int64_t sk, const float* __restrict__ v,
    int64_t sv, const float* __restrict__ out, int64_t so, const float* __restrict__ dout, int64_t sdo,
    const float* __restrict__ lse, int64_t Tq, const int64_t* __restrict__ cu_q, const int64_t* __restrict__ cu_k,
    int causal, float scale, float* __restrict__ dq, int64_t sdq, float* __restrict__ delta_out) {
  constexpr int HD = 64, NKT = R / 16;
  __shared__ __attribute__((aligned(16))) char lds[2 * R * 256];
  char* K_s = lds;
  char* V_s = lds + R * 256;
  const int b = blockIdx.z, hh = blockIdx.y, tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;
  if (b == (int)gridDim.z - 1) {
    zero_rows<HD, 64 * NW>(dq, sdq, cu_q[b], Tq, hh, tid);
    return;
  }
  const int64_t q0 = cu_q[b], k0 = cu_k[b];
  const int lq = (int)(cu_q[b + 1] - q0), lk = (int)(cu_k[b + 1] - k0);
  if (lq <= 0) return;
  const int nkt_all = min((lk + 15) >> 4, NKT);
  if (lk > 0) dma_rows2<NW>(k + k0 * sk + hh * HD, sk, v + k0 * sv + hh * HD, sv, lk, nkt_all, K_s, V_s, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const float sl2 = scale * kLog2e;
  const int nqt = (lq + 15) >> 4;
  for (int qt = wave; qt < nqt; qt += NW) {
    const int qb = qt * 16, qi = qb + (lane & 15);
    const bool qv = qi < lq;
    const int64_t qrow = q0 + (qv ? qi : 0);
    float qf[HD / 4], dof[HD / 4];
    load_frag<HD>(q + qrow * sq + hh * HD + g * (HD / 4), qv, qf);
    load_frag<HD>(dout + qrow * sdo + hh * HD + g * (HD / 4), qv, dof);
    float delta = 0.f;
    {
      float of[HD / 4];
      load_frag<HD>(out + qrow * so + hh * HD + g * (HD / 4), qv, of);
#pragma unroll
      for (int d = 0; d < HD / 4; ++d) delta += dof[d] * of[d];
      delta += __shfl_xor(delta, 16, 64);
      delta += __shfl_xor(delta, 32, 64);
      if (qv && g == 0) delta_out[(int64_t)hh * Tq + qrow] = delta;
    }
    const float lse2 = qv ? lse[(int64_t)hh * Tq + qrow] * kLog2e : 0.f;
    const int kend = causal ? min(lk, qb + 16) : lk;
    const int nkt = __builtin_amdgcn_readfirstlane(min((kend + 15) >> 4, NKT));
    f32x4 acc[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) acc[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    switch (nkt) {
      case 1: dq_dma_tile<1>(K_s, V_s, qf, dof, lane, lk, qi, causal, sl2, lse2, delta, acc); break;
      case 2: if constexpr (NKT >= 2) dq_dma_tile<2>(K_s, V_s, qf, dof, lane, lk, qi, causal, sl2, lse2, delta, acc); break;
      case 3: if constexpr (NKT >= 3) dq_dma_tile<3>(K_s, V_s, qf, dof, lane, lk, qi, causal, sl2, lse2, delta, acc); break;
      case 4: if constexpr (NKT >= 4) dq_dma_tile<4>(K_s, V_s, qf, dof, lane, lk, qi, causal, sl2, lse2, delta, acc); break;
      case 5: if constexpr (NKT >= 5) dq_dma_tile<5>(K_s, V_s, qf, dof, lane, lk, qi, causal, sl2, lse2, delta, acc); break;
      case 6: if constexpr (NKT >= 6) dq_dma_tile<6>(K_s, V_s, qf, dof, lane, lk, qi, causal, sl2, lse2, delta, acc); break;
      case 7: if constexpr (NKT >= 7) dq_dma_tile<7>(K_s, V_s, qf, dof, lane, lk, qi, causal, sl2, lse2, delta, acc); break;
      case 8: if constexpr (NKT >= 8) dq_dma_tile<8>(K_s, V_s, qf, dof, lane, lk, qi, causal, sl2, lse2, delta, acc); break;
      default: break;
    }
    if (qv) {
      float* row = dq + (q0 + qi) * sdq + hh * HD + 16 * g;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        *reinterpret_cast<float4*>(row + 4 * i) =
            make_float4(acc[0][i] * scale, acc[1][i] * scale, acc[2][i] * scale, acc[3][i] * scale);
    }
  }
}

// dK, dV of one key tile against its N query tiles (DMA images of Q and dO; lse / delta per query in LDS):
// S = Q K^T, dP = dO V^T (queries on rows, K pattern), P, dS = P (dP - delta), dV^T += dO^T P and
// dK^T += Q^T dS (V pattern, d permuted). Query tiles [t0, t0 + N).
template <int N>
__device__ __forceinline__ void dkdv_dma_tile(const char* Q_s, const char* O_s, const float* lse_s, const float* dl_s,
                                              const float (&kf)[16], const float (&vf)[16], int lane, int t0, int lq,
                                              int kj, int causal, float sl2, f32x4 (&dka)[4], f32x4 (&dva)[4]) {
  const int g = lane >> 4;
  f32x4 st[N], dp[N];
#pragma unroll
  for (int t = 0; t < N; ++t) { st[t] = f32x4{0.f, 0.f, 0.f, 0.f}; dp[t] = f32x4{0.f, 0.f, 0.f, 0.f}; }
#pragma unroll
  for (int s4 = 0; s4 < 4; ++s4) {
    float4 a[N], c[N];
#pragma unroll
    for (int t = 0; t < N; ++t) {
      a[t] = lds_chunk(Q_s, (t0 + t) * 16 + (lane & 15), 4 * g + s4);
      c[t] = lds_chunk(O_s, (t0 + t) * 16 + (lane & 15), 4 * g + s4);
    }
#pragma unroll
    for (int t = 0; t < N; ++t) {
      st[t] = mfma4(a[t].x, kf[4 * s4], st[t]);
      dp[t] = mfma4(c[t].x, vf[4 * s4], dp[t]);
      st[t] = mfma4(a[t].y, kf[4 * s4 + 1], st[t]);
      dp[t] = mfma4(c[t].y, vf[4 * s4 + 1], dp[t]);
      st[t] = mfma4(a[t].z, kf[4 * s4 + 2], st[t]);
      dp[t] = mfma4(c[t].z, vf[4 * s4 + 2], dp[t]);
      st[t] = mfma4(a[t].w, kf[4 * s4 + 3], st[t]);
      dp[t] = mfma4(c[t].w, vf[4 * s4 + 3], dp[t]);
    }
  }
#pragma unroll
  for (int t = 0; t < N; ++t) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int qr = (t0 + t) * 16 + 4 * g + i;
      float p = exp2_fast(__builtin_fmaf(st[t][i], sl2, -lse_s[qr]));
      if (!(qr < lq && (!causal || kj <= qr))) p = 0.f;
      st[t][i] = p;
      dp[t][i] = p * (dp[t][i] - dl_s[qr]);   // dS
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = (t0 + t) * 16 + 4 * g + i;
      const float4 oo = lds_chunk(O_s, r, lane & 15);   // dV^T += dO^T P
      dva[0] = mfma4(oo.x, st[t][i], dva[0]);
      dva[1] = mfma4(oo.y, st[t][i], dva[1]);
      dva[2] = mfma4(oo.z, st[t][i], dva[2]);
      dva[3] = mfma4(oo.w, st[t][i], dva[3]);
      const float4 qq = lds_chunk(Q_s, r, lane & 15);   // dK^T += Q^T dS
      dka[0] = mfma4(qq.x, dp[t][i], dka[0]);
      dka[1] = mfma4(qq.y, dp[t][i], dka[1]);
      dka[2] = mfma4(qq.z, dp[t][i], dka[2]);
      dka[3] = mfma4(qq.w, dp[t][i], dka[3]);
    }
  }
}

template <int NW, int R>
__global__ void __launch_bounds__(64 * NW, R <= 64 ? 4 : 3) attn_bwd_dkdv_dma_kernel(
    const float* __restrict__ q, int64_t sq, const float* __restrict__ k, int64_t sk, const float* __restrict__ v,
    int64_t sv, const float* __restrict__ dout, int64_t sdo, const float* __restrict__ lse,
    const float* __restrict__ delta, int64_t Tq, const int64_t* __restrict__ cu_q, const int64_t* __restrict__ cu_k,
    int causal, float scale, float* __restrict__ dk, int64_t sdk, float* __restrict__ dv, int64_t sdv, int64_t Tk) {
  constexpr int HD = 64, NQT = R / 16;
  __shared__ __attribute__((aligned(16))) char lds[2 * R * 256];
  __shared__ float lse_s[R], dl_s[R];
  char* Q_s = lds;
  char* O_s = lds + R * 256;
  const int b = blockIdx.z, hh = blockIdx.y, tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;
  if (b == (int)gridDim.z - 1) {
    zero_rows<HD, 64 * NW>(dk, sdk, cu_k[b], Tk, hh, tid);
    zero_rows<HD, 64 * NW>(dv, sdv, cu_k[b], Tk, hh, tid);
    return;
  }
  const int64_t q0 = cu_q[b], k0 = cu_k[b];
  const int lq = (int)(cu_q[b + 1] - q0), lk = (int)(cu_k[b + 1] - k0);
  if (lk <= 0) return;
  const int nqt_all = min((lq + 15) >> 4, NQT);
  if (lq > 0) dma_rows2<NW>(q + q0 * sq + hh * HD, sq, dout + q0 * sdo + hh * HD, sdo, lq, nqt_all, Q_s, O_s, wave, lane);
  for (int r = tid; r < R; r += 64 * NW) {
    const bool ok = r < lq;
    lse_s[r] = ok ? lse[(int64_t)hh * Tq + q0 + r] * kLog2e : 0.f;
    dl_s[r] = ok ? delta[(int64_t)hh * Tq + q0 + r] : 0.f;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const float sl2 = scale * kLog2e;
  for (int kt = wave; kt * 16 < lk; kt += NW) {
    const int kb = kt * 16, kj = kb + (lane & 15);
    const bool kvv = kj < lk;
    const int64_t krow = k0 + (kvv ? kj : 0);
    float kf[HD / 4], vf[HD / 4];
    load_frag<HD>(k + krow * sk + hh * HD + g * (HD / 4), kvv, kf);
    load_frag<HD>(v + krow * sv + hh * HD + g * (HD / 4), kvv, vf);
    f32x4 dka[4], dva[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) { dka[dt] = f32x4{0.f, 0.f, 0.f, 0.f}; dva[dt] = f32x4{0.f, 0.f, 0.f, 0.f}; }
    const int t0 = __builtin_amdgcn_readfirstlane(causal ? min(kb >> 4, nqt_all) : 0);   // query tiles wholly before the keys
    const int nt = __builtin_amdgcn_readfirstlane(nqt_all - t0);
    switch (nt) {
      case 1: dkdv_dma_tile<1>(Q_s, O_s, lse_s, dl_s, kf, vf, lane, t0, lq, kj, causal, sl2, dka, dva); break;
      case 2: if constexpr (NQT >= 2) dkdv_dma_tile<2>(Q_s, O_s, lse_s, dl_s, kf, vf, lane, t0, lq, kj, causal, sl2, dka, dva); break;
      case 3: if constexpr (NQT >= 3) dkdv_dma_tile<3>(Q_s, O_s, lse_s, dl_s, kf, vf, lane, t0, lq, kj, causal, sl2, dka, dva); break;
      case 4: if constexpr (NQT >= 4) dkdv_dma_tile<4>(Q_s, O_s, lse_s, dl_s, kf, vf, lane, t0, lq, kj, causal, sl2, dka, dva); break;
      case 5: if constexpr (NQT >= 5) dkdv_dma_tile<5>(Q_s, O_s, lse_s, dl_s, kf, vf, lane, t0, lq, kj, causal, sl2, dka, dva); break;
      case 6: if constexpr (NQT >= 6) dkdv_dma_tile<6>(Q_s, O_s, lse_s, dl_s, kf, vf, lane, t0, lq, kj, causal, sl2, dka, dva); break;
      case 7: if constexpr (NQT >= 7) dkdv_dma_tile<7>(Q_s, O_s, lse_s, dl_s, kf, vf, lane, t0, lq, kj, causal, sl2, dka, dva); break;
      case 8: if constexpr (NQT >= 8) dkdv_dma_tile<8>(Q_s, O_s, lse_s, dl_s, kf, vf, lane, t0, lq, kj, causal, sl2, dka, dva); break;
      default: break;
    }
    if (kvv) {
      float* rk = dk + (k0 + kj) * sdk + hh * HD + 16 * g;
      float* rv = dv + (k0 + kj) * sdv + hh * HD + 16 * g;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        *reinterpret_cast<float4*>(rk + 4 * i) =
            make_float4(dka[0][i] * scale, dka[1][i] * scale, dka[2][i] * scale, dka[3][i] * scale);
        *reinterpret_cast<float4*>(rv + 4 * i) = make_float4(dva[0][i], dva[1][i], dva[2][i], dva[3][i]);
      }
    }
  }
}

// ---------------------------------------------------- few queries over a short key range (HD = 64)
// One query tile per (sequence, head) (the decoder's cross-attention: 5-6 future tokens over <= 128
// context keys; its causal self-attention over 5-6 tokens): the key tiles are split over the NW waves of
// the workgroup (wave w: tiles w, w + NW, ...) so each wave issues all the loads of its one or two tiles
// at once, straight into registers in the two fragment layouts (K pattern for S^T, permuted-d V pattern
// for the O^T product: no LDS staging, no reuse to stage for), and the waves' partial (m, l, O) — or dQ —
// merge through LDS in wave order (deterministic).
// Register fragments of key tile t of a strided row source (rows >= lk read row lk - 1):
//   K pattern: row t*16 + (lane & 15), d = 16 (lane >> 4) + 0..15
//   V pattern: rows t*16 + 4 (lane >> 4) + i, d = 4 (lane & 15) + 0..3   (permuted-d products)
__device__ __forceinline__ void frag_kpat(const float* __restrict__ base, int64_t stride, int t, int lk, int lane,
                                          float4 (&f)[4]) {
  const int rk = min(t * 16 + (lane & 15), lk - 1);
  const float* p = base + (int64_t)rk * stride + 16 * (lane >> 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) f[j] = *reinterpret_cast<const float4*>(p + 4 * j);
}
__device__ __forceinline__ void frag_vpat(const float* __restrict__ base, int64_t stride, int t, int lk, int lane,
                                          float4 (&f)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rv = min(t * 16 + 4 * (lane >> 4) + i, lk - 1);
    f[i] = *reinterpret_cast<const float4*>(base + (int64_t)rv * stride + 4 * (lane & 15));
  }
}

template <int NW>
__global__ void __launch_bounds__(64 * NW) attn_fwd_fewq_kernel(
    const float* __restrict__ q, int64_t sq, const float* __restrict__ k, int64_t sk, const float* __restrict__ v,
    int64_t sv, const int64_t* __restrict__ cu_q, const int64_t* __restrict__ cu_k, int causal, float scale,
    float* __restrict__ out, int64_t so, float* __restrict__ lse, int64_t Tq, const int* __restrict__ order) {
  constexpr int HD = 64, TPW = 2;   // key tiles per wave (<= 128 keys over 4 waves)
  __shared__ __attribute__((aligned(16))) float part_o[NW][16][HD + kPartPad];
  __shared__ float part_m[NW][16], part_l[NW][16];
  const int z = blockIdx.z, hh = blockIdx.y, tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;
  if (z == (int)gridDim.z - 1) {
    zero_rows<HD, 64 * NW>(out, so, cu_q[z], Tq, hh, tid);
    return;
  }
  const int b = seq_of(order, z);   // longest-first when an LPT order is given
  const int64_t q0 = cu_q[b], k0 = cu_k[b];
  const int lq = (int)(cu_q[b + 1] - q0), lk = (int)(cu_k[b + 1] - k0);
  if (lq <= 0) return;
  const int qi = lane & 15;
  const bool qv = qi < lq;
  const int kend = causal ? min(lk, 16) : lk;
  const int nkt = (kend + 15) >> 4;
  float qf[HD / 4];
  load_frag<HD>(q + (q0 + (qv ? qi : 0)) * sq + hh * HD + g * (HD / 4), qv, qf);
  const float* kb_ = k + k0 * sk + hh * HD;
  const float* vb_ = v + k0 * sv + hh * HD;
  float4 kp[TPW][4], vp[TPW][4];
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int t = wave + j * NW;
    if (t < nkt) {
      frag_kpat(kb_, sk, t, lk, lane, kp[j]);
      frag_vpat(vb_, sv, t, lk, lane, vp[j]);
    }
  }
  const float sl2 = scale * kLog2e;
  f32x4 st[TPW];
  float mt = -INFINITY;
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int t = wave + j * NW;
    st[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (t < nkt) {
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        st[j] = mfma4(kp[j][s4].x, qf[4 * s4], st[j]);
        st[j] = mfma4(kp[j][s4].y, qf[4 * s4 + 1], st[j]);
        st[j] = mfma4(kp[j][s4].z, qf[4 * s4 + 2], st[j]);
        st[j] = mfma4(kp[j][s4].w, qf[4 * s4 + 3], st[j]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = t * 16 + 4 * g + i;
        if (!(key < lk && (!causal || key <= qi))) st[j][i] = -INFINITY;
        mt = fmaxf(mt, st[j][i]);
      }
    }
  }
  mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
  mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
  const float mn = mt * sl2;
  const bool none = mn == -INFINITY;
  float l = 0.f;
  f32x4 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int t = wave + j * NW;
    if (t < nkt) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        st[j][i] = none ? 0.f : exp2_fast(__builtin_fmaf(st[j][i], sl2, -mn));
        l += st[j][i];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        o[0] = mfma4(vp[j][i].x, st[j][i], o[0]);
        o[1] = mfma4(vp[j][i].y, st[j][i], o[1]);
        o[2] = mfma4(vp[j][i].z, st[j][i], o[2]);
        o[3] = mfma4(vp[j][i].w, st[j][i], o[3]);
      }
    }
  }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
#pragma unroll
  for (int i = 0; i < 4; ++i)
    *reinterpret_cast<float4*>(&part_o[wave][qi][16 * g + 4 * i]) = make_float4(o[0][i], o[1][i], o[2][i], o[3][i]);
  if (g == 0) {
    part_m[wave][qi] = mn;
    part_l[wave][qi] = l;
  }
  __syncthreads();
  // merge: thread -> (query r, 4 d); waves in order
  constexpr int TPR = HD / 4;   // threads per query row
  for (int e = tid; e < 16 * TPR; e += 64 * NW) {
    const int r = e / TPR, c = (e % TPR) * 4;
    if (r >= lq) continue;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < NW; ++w) M = fmaxf(M, part_m[w][r]);
    float L = 0.f;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (M != -INFINITY) {
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        const float a = part_m[w][r] == -INFINITY ? 0.f : exp2_fast(part_m[w][r] - M);
        L += part_l[w][r] * a;
        const float4 pv = *reinterpret_cast<const float4*>(&part_o[w][r][c]);
        acc.x += pv.x * a; acc.y += pv.y * a; acc.z += pv.z * a; acc.w += pv.w * a;
      }
    }
    const float inv = L > 0.f ? 1.f / L : 0.f;
    *reinterpret_cast<float4*>(out + (q0 + r) * so + hh * HD + c) = make_float4(acc.x * inv, acc.y * inv, acc.z * inv, acc.w * inv);
    if (c == 0) lse[(int64_t)hh * Tq + q0 + r] = L > 0.f ? (M + log2f(L)) * kLn2 : 0.f;
  }
}

// dQ (+ delta) of the one query tile: key tiles split over the waves as in the forward, partial dQ^T
// summed through LDS in wave order.
template <int NW>
__global__ void __launch_bounds__(64 * NW) attn_bwd_dq_fewq_kernel(
    const float* __restrict__ q, int64_t sq, const float* __restrict__ k, int64_t sk, const float* __restrict__ v,
    int64_t sv, const float* __restrict__ out, int64_t so, const float* __restrict__ dout, int64_t sdo,
    const float* __restrict__ lse, int64_t Tq, const int64_t* __restrict__ cu_q, const int64_t* __restrict__ cu_k,
    int causal, float scale, float* __restrict__ dq, int64_t sdq, float* __restrict__ delta_out) {
  constexpr int HD = 64, TPW = 2;
  __shared__ __attribute__((aligned(16))) float part[NW][16][HD + kPartPad];
  const int b = blockIdx.z, hh = blockIdx.y, tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;
  if (b == (int)gridDim.z - 1) {
    zero_rows<HD, 64 * NW>(dq, sdq, cu_q[b], Tq, hh, tid);
    return;
  }
  const int64_t q0 = cu_q[b], k0 = cu_k[b];
  const int lq = (int)(cu_q[b + 1] - q0), lk = (int)(cu_k[b + 1] - k0);
  if (lq <= 0) return;
  const int qi = lane & 15;
  const bool qv = qi < lq;
  const int64_t qrow = q0 + (qv ? qi : 0);
  const int kend = causal ? min(lk, 16) : lk;
  const int nkt = (kend + 15) >> 4;
  float qf[HD / 4], dof[HD / 4];
  load_frag<HD>(q + qrow * sq + hh * HD + g * (HD / 4), qv, qf);
  load_frag<HD>(dout + qrow * sdo + hh * HD + g * (HD / 4), qv, dof);
  const float* kb_ = k + k0 * sk + hh * HD;
  const float* vb_ = v + k0 * sv + hh * HD;
  float4 kp[TPW][4], kv[TPW][4], vk[TPW][4];   // K (K pattern), K (V pattern), V (K pattern)
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int t = wave + j * NW;
    if (t < nkt) {
      frag_kpat(kb_, sk, t, lk, lane, kp[j]);
      frag_vpat(kb_, sk, t, lk, lane, kv[j]);
      frag_kpat(vb_, sv, t, lk, lane, vk[j]);
    }
  }
  float delta = 0.f;
  {
    float of[HD / 4];
    load_frag<HD>(out + qrow * so + hh * HD + g * (HD / 4), qv, of);
#pragma unroll
    for (int d = 0; d < HD / 4; ++d) delta += dof[d] * of[d];
    delta += __shfl_xor(delta, 16, 64);
    delta += __shfl_xor(delta, 32, 64);
    if (wave == 0 && qv && g == 0) delta_out[(int64_t)hh * Tq + qrow] = delta;
  }
  const float sl2 = scale * kLog2e;
  const float lse2 = qv ? lse[(int64_t)hh * Tq + qrow] * kLog2e : 0.f;
  f32x4 acc[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) acc[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int t = wave + j * NW;
    if (t < nkt) {
      f32x4 st = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        st = mfma4(kp[j][s4].x, qf[4 * s4], st);
        dp = mfma4(vk[j][s4].x, dof[4 * s4], dp);
        st = mfma4(kp[j][s4].y, qf[4 * s4 + 1], st);
        dp = mfma4(vk[j][s4].y, dof[4 * s4 + 1], dp);
        st = mfma4(kp[j][s4].z, qf[4 * s4 + 2], st);
        dp = mfma4(vk[j][s4].z, dof[4 * s4 + 2], dp);
        st = mfma4(kp[j][s4].w, qf[4 * s4 + 3], st);
        dp = mfma4(vk[j][s4].w, dof[4 * s4 + 3], dp);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = t * 16 + 4 * g + i;
        float p = exp2_fast(__builtin_fmaf(st[i], sl2, -lse2));
        if (!(key < lk && (!causal || key <= qi))) p = 0.f;
        st[i] = p * (dp[i] - delta);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        acc[0] = mfma4(kv[j][i].x, st[i], acc[0]);
        acc[1] = mfma4(kv[j][i].y, st[i], acc[1]);
        acc[2] = mfma4(kv[j][i].z, st[i], acc[2]);
        acc[3] = mfma4(kv[j][i].w, st[i], acc[3]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
    *reinterpret_cast<float4*>(&part[wave][qi][16 * g + 4 * i]) = make_float4(acc[0][i], acc[1][i], acc[2][i], acc[3][i]);
  __syncthreads();
  constexpr int TPR = HD / 4;
  for (int e = tid; e < 16 * TPR; e += 64 * NW) {
    const int r = e / TPR, c = (e % TPR) * 4;
    if (r >= lq) continue;
    float4 s4 = *reinterpret_cast<const float4*>(&part[0][r][c]);
#pragma unroll
    for (int w = 1; w < NW; ++w) {
      const float4 a = *reinterpret_cast<const float4*>(&part[w][r][c]);
      s4.x += a.x; s4.y += a.y; s4.z += a.z; s4.w += a.w;
    }
    *reinterpret_cast<float4*>(dq + (q0 + r) * sdq + hh * HD + c) = make_float4(s4.x * scale, s4.y * scale, s4.z * scale, s4.w * scale);
  }
}

// ------------------------------------------ fused backward of one query tile over a short key range
// dQ, dK and dV in ONE pass (the decoder's cross-attention: <= 16 future queries per sequence over <= 128
// context keys; its causal self-attention over <= 16 tokens). The two-pass form reads every key twice and
// forms S and dP twice (7 products per tile pair); here each wave owns key tiles (t = wave, wave + NW),
// forms S and dP once in the dK/dV orientation (queries on the accumulator rows 4 (lane >> 4) + i, keys on
// the lanes), and from them P, dS -> dV^T += dO^T P, dK^T += Q^T dS (permuted-d products); dS is turned into
// dS^T by four exact MFMAs against a 0/1 permutation operand (each output is one x * 1 plus zeros), which
// feeds dQ^T += K^T dS^T. The waves' partial dQ^T sum through LDS in wave order (deterministic). 5 products
// + the transpose per tile pair; keys are read once. delta = rowsum(dO * O) per query comes in by lane
// shuffles from the lanes that computed it (lane & 15 = query).
template <int NW>
#ifndef RQ_FEWQ_BWD_MINWG
#define RQ_FEWQ_BWD_MINWG 1   // workgroups per CU the 4-wave few-query backward is compiled for (register budget)
#endif
__global__ void __launch_bounds__(64 * NW, NW == 4 ? RQ_FEWQ_BWD_MINWG : 1) attn_bwd_fewq_fused_kernel(
    const float* __restrict__ q, int64_t sq, const float* __restrict__ k, int64_t sk, const float* __restrict__ v,
    int64_t sv, const float* __restrict__ out, int64_t so, const float* __restrict__ dout, int64_t sdo,
    const float* __restrict__ lse, int64_t Tq, const int64_t* __restrict__ cu_q, const int64_t* __restrict__ cu_k,
    int causal, float scale, float* __restrict__ dq, int64_t sdq, float* __restrict__ dk, int64_t sdk,
    float* __restrict__ dv, int64_t sdv, int64_t Tk, float* __restrict__ delta_out,
    const int* __restrict__ order) {
  constexpr int HD = 64, TPW = 2;   // key tiles per wave (<= 128 keys over 4 waves)
  __shared__ __attribute__((aligned(16))) float part[NW][16][HD + kPartPad];
  const int z = blockIdx.z, hh = blockIdx.y, tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, c = lane & 15;
  if (z == (int)gridDim.z - 1) {   // tail slice: rows past the last sequence
    zero_rows<HD, 64 * NW>(dq, sdq, cu_q[z], Tq, hh, tid);
    zero_rows<HD, 64 * NW>(dk, sdk, cu_k[z], Tk, hh, tid);
    zero_rows<HD, 64 * NW>(dv, sdv, cu_k[z], Tk, hh, tid);
    return;
  }
  const int b = seq_of(order, z);   // longest-first when an LPT order is given
  const int64_t q0 = cu_q[b], k0 = cu_k[b];
  const int lq = (int)(cu_q[b + 1] - q0), lk = (int)(cu_k[b + 1] - k0);
  const int nkt = (lk + 15) >> 4;   // every key tile gets its dK / dV rows written (zeros past the queries)
  const float* kb_ = k + k0 * sk + hh * HD;
  const float* vb_ = v + k0 * sv + hh * HD;
  // this wave's key tiles: K and V in the K pattern (S, dP), K in the V pattern (dQ^T)
  float4 kp[TPW][4], vk[TPW][4], kv[TPW][4];
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int t = wave + j * NW;
    if (t < nkt) {
      frag_kpat(kb_, sk, t, lk, lane, kp[j]);
      frag_kpat(vb_, sv, t, lk, lane, vk[j]);
      frag_vpat(kb_, sk, t, lk, lane, kv[j]);
    }
  }
  // the query tile: Q, dO in the A pattern (row c, d = 16 g + 0..15) and the V pattern (rows 4 g + i,
  // d = 4 c + 0..3); O (A pattern) only for delta
  const bool qv = c < lq;
  const int64_t qrow = q0 + (qv ? c : 0);
  float qf[HD / 4], dof[HD / 4];
  load_frag<HD>(q + qrow * sq + hh * HD + g * (HD / 4), qv && lq > 0, qf);
  load_frag<HD>(dout + qrow * sdo + hh * HD + g * (HD / 4), qv && lq > 0, dof);
  float4 qvp[4], dvp[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) qvp[i] = dvp[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (lq > 0) {
    frag_vpat(q + q0 * sq + hh * HD, sq, 0, lq, lane, qvp);
    frag_vpat(dout + q0 * sdo + hh * HD, sdo, 0, lq, lane, dvp);
  }
  float delta = 0.f, lse2 = 0.f;
  if (lq > 0) {
    float of[HD / 4];
    load_frag<HD>(out + qrow * so + hh * HD + g * (HD / 4), qv, of);
#pragma unroll
    for (int d = 0; d < HD / 4; ++d) delta += dof[d] * of[d];
    delta += __shfl_xor(delta, 16, 64);
    delta += __shfl_xor(delta, 32, 64);
    if (wave == 0 && qv && g == 0) delta_out[(int64_t)hh * Tq + qrow] = delta;
    lse2 = qv ? lse[(int64_t)hh * Tq + qrow] * kLog2e : 0.f;
  }
  // per-lane values of the queries 4 g + i (held by lane 4 g + i)
  float dl[4], ls[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    dl[i] = __shfl(delta, 4 * g + i, 64);
    ls[i] = __shfl(lse2, 4 * g + i, 64);
  }
  // 0/1 permutation operand of the transpose: step s, lane (g, c) = [c == 4 g + s]
  float pe[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) pe[s] = c == 4 * g + s ? 1.f : 0.f;
  const float sl2 = scale * kLog2e;
  f32x4 acc[4];   // partial dQ^T (d permuted) over this wave's key tiles
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) acc[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int t = wave + j * NW;
    if (t < nkt) {
      // S = Q K^T, dP = dO V^T: rows = queries 4 g + i, columns = keys t * 16 + c
      f32x4 st = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        st = mfma4(qf[4 * s4], kp[j][s4].x, st);
        dp = mfma4(dof[4 * s4], vk[j][s4].x, dp);
        st = mfma4(qf[4 * s4 + 1], kp[j][s4].y, st);
        dp = mfma4(dof[4 * s4 + 1], vk[j][s4].y, dp);
        st = mfma4(qf[4 * s4 + 2], kp[j][s4].z, st);
        dp = mfma4(dof[4 * s4 + 2], vk[j][s4].z, dp);
        st = mfma4(qf[4 * s4 + 3], kp[j][s4].w, st);
        dp = mfma4(dof[4 * s4 + 3], vk[j][s4].w, dp);
      }
      const int key = t * 16 + c;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int qr = 4 * g + i;
        float p = exp2_fast(__builtin_fmaf(st[i], sl2, -ls[i]));
        if (!(qr < lq && key < lk && (!causal || key <= qr))) p = 0.f;
        st[i] = p;
        dp[i] = p * (dp[i] - dl[i]);   // dS
      }
      f32x4 dka[4], dva[4], dst = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) { dka[dt] = f32x4{0.f, 0.f, 0.f, 0.f}; dva[dt] = f32x4{0.f, 0.f, 0.f, 0.f}; }
#pragma unroll
      for (int i = 0; i < 4; ++i) {   // dV^T += dO^T P, dK^T += Q^T dS (k = the query index 4 g + i)
        dva[0] = mfma4(dvp[i].x, st[i], dva[0]);
        dva[1] = mfma4(dvp[i].y, st[i], dva[1]);
        dva[2] = mfma4(dvp[i].z, st[i], dva[2]);
        dva[3] = mfma4(dvp[i].w, st[i], dva[3]);
        dka[0] = mfma4(qvp[i].x, dp[i], dka[0]);
        dka[1] = mfma4(qvp[i].y, dp[i], dka[1]);
        dka[2] = mfma4(qvp[i].z, dp[i], dka[2]);
        dka[3] = mfma4(qvp[i].w, dp[i], dka[3]);
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) dst = mfma4(dp[s], pe[s], dst);   // dS^T: rows = keys 4 g + i, lanes = queries
#pragma unroll
      for (int i = 0; i < 4; ++i) {   // dQ^T += K^T dS^T (k = the key index 4 g + i of the tile)
        acc[0] = mfma4(kv[j][i].x, dst[i], acc[0]);
        acc[1] = mfma4(kv[j][i].y, dst[i], acc[1]);
        acc[2] = mfma4(kv[j][i].z, dst[i], acc[2]);
        acc[3] = mfma4(kv[j][i].w, dst[i], acc[3]);
      }
      if (key < lk) {
        float* rk = dk + (k0 + key) * sdk + hh * HD + 16 * g;
        float* rv = dv + (k0 + key) * sdv + hh * HD + 16 * g;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          *reinterpret_cast<float4*>(rk + 4 * i) =
              make_float4(dka[0][i] * scale, dka[1][i] * scale, dka[2][i] * scale, dka[3][i] * scale);
          *reinterpret_cast<float4*>(rv + 4 * i) = make_float4(dva[0][i], dva[1][i], dva[2][i], dva[3][i]);
        }
      }
    }
  }
  if (lq <= 0) return;   // uniform per workgroup: no dQ rows
#pragma unroll
  for (int i = 0; i < 4; ++i)
    *reinterpret_cast<float4*>(&part[wave][c][16 * g + 4 * i]) = make_float4(acc[0][i], acc[1][i], acc[2][i], acc[3][i]);
  __syncthreads();
  constexpr int TPR = HD / 4;
  for (int e = tid; e < 16 * TPR; e += 64 * NW) {
    const int r = e / TPR, cc = (e % TPR) * 4;
    if (r >= lq) continue;
    float4 s4 = *reinterpret_cast<const float4*>(&part[0][r][cc]);
#pragma unroll
    for (int w = 1; w < NW; ++w) {
      const float4 a = *reinterpret_cast<const float4*>(&part[w][r][cc]);
      s4.x += a.x; s4.y += a.y; s4.z += a.z; s4.w += a.w;
    }
    *reinterpret_cast<float4*>(dq + (q0 + r) * sdq + hh * HD + cc) =
        make_float4(s4.x * scale, s4.y * scale, s4.z * scale, s4.w * scale);
  }
}

// -------------------------------- few-query fused backward, persistent, next unit staged by LDS-DMA
// attn_bwd_fewq_fused_kernel with the unit loop inside: a workgroup walks units u = blockIdx.x + i gridDim.x
// (unit = LPT rank u / H, head u % H) and, while it multiplies unit u, its K / V rows (R staged rows), its
// Q / dO / O rows (16) and lse are already on their way into LDS for unit u + gridDim.x by LDS-DMA. The
// workgroup form paid one load round trip per unit with nothing to overlap it (2,048 workgroups in ~4
// dependent rounds: 44 us for the Amazon cross-attention, 0.034 of fp32 peak). Per unit the fragments are
// read from the images into the registers the workgroup form loads from global memory (K / V in the K
// pattern, K in the V pattern, Q / dO in the A and V patterns, rows past a segment = its last row), so the
// products, the wave-order dQ sum and every stored value are the workgroup form's bit for bit.
// The images are refilled in two phases so that a wave holds one key tile's fragments at a time: phase A
// (key rows < 64 = every wave's first tile, Q / dO / O, lse) right after the first tiles were read, phase B
// (key rows >= 64, the second tiles) after the second tiles were read, at the dQ-reduction barrier.
// vmcnt discipline (it retires in issue order): per unit every wave issues the same counts — 12 phase-A DMA
// instructions, 8 dK / dV stores per tile slot (buffer stores whose descriptor range drops rows past the
// segment, so no branch changes a count), 2 (R - 64) / 16 phase-B instructions, the dQ and delta stores — and
// the next unit starts with s_waitcnt vmcnt(2) (R = 64: vmcnt(18)): its DMA landed, the stores issued after it
// may still be in flight. Barriers are bare s_barrier (__syncthreads would wait vmcnt(0)).
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wave_rsrc(const float* base, int64_t bytes) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const int n = __builtin_amdgcn_readfirstlane((int)(bytes < 0x7fffffff ? (bytes > 0 ? bytes : 0) : 0x7fffffff));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<float*>((uintptr_t)(((uint64_t)hi << 32) | lo)), (short)0, n,
                                           0x00020000);
}
__device__ __forceinline__ void rsrc_st4(__amdgpu_buffer_rsrc_t r, int64_t off_floats, float4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), r, (int)(off_floats * 4), 0, 0);
}
__device__ __forceinline__ void rsrc_st1(__amdgpu_buffer_rsrc_t r, int64_t off_floats, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, (int)(off_floats * 4), 0, 0);
}
// rows [rlo, rhi) of a strided head slice into a swizzled image (rows >= n read row n - 1, clamped to the
// buffer's last row T - 1); instruction j (4 rows) by wave j % NW: (rhi - rlo) / (4 NW) instructions per wave
template <int NW>
__device__ __forceinline__ void dma_img(const float* __restrict__ head0, int64_t stride, int64_t row0, int n, int64_t T,
                                        int rlo, int rhi, char* img, int wave, int lane) {
  for (int j = rlo / 4 + wave; j < rhi / 4; j += NW) {
    const int r = 4 * j + (lane >> 4);
    const int64_t rr = min(row0 + min(r, max(n, 1) - 1), T - 1);
    const int c = (lane & 15) ^ swz16(r);
    glds16f(head0 + rr * stride + 4 * c, img + j * 1024);
  }
}

template <int R>
__global__ void __launch_bounds__(256, R <= 96 ? 2 : 1) attn_bwd_fewq_stream_kernel(
    const float* __restrict__ q, int64_t sq, const float* __restrict__ k, int64_t sk, const float* __restrict__ v,
    int64_t sv, const float* __restrict__ out, int64_t so, const float* __restrict__ dout, int64_t sdo,
    const float* __restrict__ lse, int64_t Tq, const int64_t* __restrict__ cu_q, const int64_t* __restrict__ cu_k,
    int causal, float scale, float* __restrict__ dq, int64_t sdq, float* __restrict__ dk, int64_t sdk,
    float* __restrict__ dv, int64_t sdv, int64_t Tk, float* __restrict__ delta_out, const int* __restrict__ order,
    int B, int H) {
  constexpr int HD = 64, NW = 4, TPW = 2, NKT = R / 16;
  static_assert(R % 64 == 0 || R == 96, "staged key rows: whole 4-row DMA instructions on every wave");
  __shared__ __attribute__((aligned(16))) char K_s[R * 256];
  __shared__ __attribute__((aligned(16))) char V_s[R * 256];
  __shared__ __attribute__((aligned(16))) char Q_s[16 * 256];
  __shared__ __attribute__((aligned(16))) char D_s[16 * 256];
  __shared__ __attribute__((aligned(16))) char O_s[16 * 256];
  __shared__ __attribute__((aligned(16))) float L_s[64];
  __shared__ __attribute__((aligned(16))) float part[NW][16][HD + kPartPad];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, c = lane & 15;
  {   // rows past the last sequence: zero dq / dk / dv over every head (before the first unit's wait)
    const int64_t f4 = (int64_t)H * (HD / 4), nth = (int64_t)gridDim.x * 256, me = (int64_t)blockIdx.x * 256 + tid;
    const int64_t rq = cu_q[B], rk = cu_k[B];
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t f = me; f < (Tq - rq) * f4; f += nth)
      *reinterpret_cast<float4*>(dq + (rq + f / f4) * sdq + (f % f4) * 4) = z4;
    for (int64_t f = me; f < (Tk - rk) * f4; f += nth) {
      *reinterpret_cast<float4*>(dk + (rk + f / f4) * sdk + (f % f4) * 4) = z4;
      *reinterpret_cast<float4*>(dv + (rk + f / f4) * sdv + (f % f4) * 4) = z4;
    }
  }
  const int nunits = B * H;
  // DMA of unit uu's rows into the images in two phases: A = key rows [0, 64) (the first tile of every
  // wave), Q / dO / O, lse (12 instructions per wave); B = key rows [64, R) (the second tiles: 2 (R - 64) / 16
  // per wave). The same counts for every unit.
  auto stage_a = [&](int uu) {
    const int bb = seq_of(order, uu / H), h2 = uu % H;
    const int64_t qa = cu_q[bb], ka = cu_k[bb];
    const int nq = (int)(cu_q[bb + 1] - qa), nk = (int)(cu_k[bb + 1] - ka);
    dma_img<NW>(k + h2 * HD, sk, ka, nk, Tk, 0, 64, K_s, wave, lane);
    dma_img<NW>(v + h2 * HD, sv, ka, nk, Tk, 0, 64, V_s, wave, lane);
    dma_img<NW>(q + h2 * HD, sq, qa, nq, Tq, 0, 16, Q_s, wave, lane);
    dma_img<NW>(dout + h2 * HD, sdo, qa, nq, Tq, 0, 16, D_s, wave, lane);
    dma_img<NW>(out + h2 * HD, so, qa, nq, Tq, 0, 16, O_s, wave, lane);
    const int64_t lr = min(qa + min(lane, max(nq, 1) - 1), Tq - 1);   // lse (H, Tq): 4 B per lane, lanes 16.. repeat
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(lse + (int64_t)h2 * Tq + lr),
                                     (__attribute__((address_space(3))) void*)L_s, 4, 0, 0);
  };
  auto stage_b = [&](int uu) {
    if constexpr (R > 64) {
      const int bb = seq_of(order, uu / H), h2 = uu % H;
      const int64_t ka = cu_k[bb];
      const int nk = (int)(cu_k[bb + 1] - ka);
      dma_img<NW>(k + h2 * HD, sk, ka, nk, Tk, 64, R, K_s, wave, lane);
      dma_img<NW>(v + h2 * HD, sv, ka, nk, Tk, 64, R, V_s, wave, lane);
    }
  };
  int u = blockIdx.x;
  if (u < nunits) { stage_a(u); stage_b(u); }
  const float sl2 = scale * kLog2e;
  bool first = true;
  for (; u < nunits; u += gridDim.x) {
    // this unit's DMA landed; what may still fly: the last unit's stores issued after its phase-B DMA
    // (R > 64: dQ, delta) or after its phase-A DMA (R = 64: 16 dK / dV pieces, dQ, delta)
    if (first) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if constexpr (R > 64) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
    first = false;
    __builtin_amdgcn_s_barrier();   // every wave's DMA landed: the images are complete
    const int b = seq_of(order, u / H), hh = u % H;
    const int64_t q0 = cu_q[b], k0 = cu_k[b];
    const int lq = (int)(cu_q[b + 1] - q0), lk = (int)(cu_k[b + 1] - k0);
    const int nkt = min((lk + 15) >> 4, NKT);
    // fragments from the images (the workgroup form's global-load layouts): the first tile's now (rows < 64,
    // phase A), the second tile's after the first tile is done (rows >= 64, phase B)
    float4 kp[4], vk[4], kv[4];
    auto read_tile = [&](int t) {
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        kp[s4] = lds_chunk(K_s, t * 16 + c, 4 * g + s4);
        vk[s4] = lds_chunk(V_s, t * 16 + c, 4 * g + s4);
        kv[s4] = lds_chunk(K_s, t * 16 + 4 * g + s4, c);
      }
    };
    read_tile(min(wave, NKT - 1));
    const bool qv = c < lq;
    float qf[HD / 4], dof[HD / 4], of[HD / 4];
    float4 qvp[4], dvp[4];
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      const float4 a = lds_chunk(Q_s, c, 4 * g + s4), d = lds_chunk(D_s, c, 4 * g + s4), o = lds_chunk(O_s, c, 4 * g + s4);
      qf[4 * s4] = a.x; qf[4 * s4 + 1] = a.y; qf[4 * s4 + 2] = a.z; qf[4 * s4 + 3] = a.w;
      dof[4 * s4] = d.x; dof[4 * s4 + 1] = d.y; dof[4 * s4 + 2] = d.z; dof[4 * s4 + 3] = d.w;
      of[4 * s4] = o.x; of[4 * s4 + 1] = o.y; of[4 * s4 + 2] = o.z; of[4 * s4 + 3] = o.w;
      qvp[s4] = lds_chunk(Q_s, 4 * g + s4, c);
      dvp[s4] = lds_chunk(D_s, 4 * g + s4, c);
    }
    const float lraw = L_s[c];
#pragma unroll
    for (int d = 0; d < HD / 4; ++d) {   // queries past lq: zero (the workgroup form's masked loads)
      qf[d] = qv ? qf[d] : 0.f;
      dof[d] = qv ? dof[d] : 0.f;
      of[d] = qv ? of[d] : 0.f;
    }
    float delta = 0.f;   // before the barrier: O's fragment is dead after it
#pragma unroll
    for (int d = 0; d < HD / 4; ++d) delta += dof[d] * of[d];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();   // every wave has its fragments: the images are free
    asm volatile("" ::: "memory");
    const int un = u + (int)gridDim.x < nunits ? u + (int)gridDim.x : u;   // the next unit (past the end: this one)
    stage_a(un);   // rows < 64 and Q / dO / O / lse are free: every wave holds its first tile and query fragments
    asm volatile("" ::: "memory");
    delta += __shfl_xor(delta, 16, 64);
    delta += __shfl_xor(delta, 32, 64);
    const float lse2 = qv ? lraw * kLog2e : 0.f;
    float dl[4], ls[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      dl[i] = __shfl(delta, 4 * g + i, 64);
      ls[i] = __shfl(lse2, 4 * g + i, 64);
    }
    f32x4 acc[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) acc[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    // dK / dV of each tile stored right after it is formed (one accumulator set live; 8 stores per tile
    // always — a tile past nkt stores its zero rows past lk, dropped by the descriptor range)
    const __amdgpu_buffer_rsrc_t rk_ = wave_rsrc(dk + k0 * sdk + hh * HD, (int64_t)lk * sdk * 4);
    const __amdgpu_buffer_rsrc_t rv_ = wave_rsrc(dv + k0 * sdv + hh * HD, (int64_t)lk * sdv * 4);
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const int t = wave + j * NW;
      if (j > 0) read_tile(min(t, NKT - 1));
      f32x4 dka[1][4], dva[1][4];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) { dka[0][dt] = f32x4{0.f, 0.f, 0.f, 0.f}; dva[0][dt] = f32x4{0.f, 0.f, 0.f, 0.f}; }
      if (t < nkt) {
        f32x4 st = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          st = mfma4(qf[4 * s4], kp[s4].x, st);
          dp = mfma4(dof[4 * s4], vk[s4].x, dp);
          st = mfma4(qf[4 * s4 + 1], kp[s4].y, st);
          dp = mfma4(dof[4 * s4 + 1], vk[s4].y, dp);
          st = mfma4(qf[4 * s4 + 2], kp[s4].z, st);
          dp = mfma4(dof[4 * s4 + 2], vk[s4].z, dp);
          st = mfma4(qf[4 * s4 + 3], kp[s4].w, st);
          dp = mfma4(dof[4 * s4 + 3], vk[s4].w, dp);
        }
        const int key = t * 16 + c;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int qr = 4 * g + i;
          float p = exp2_fast(__builtin_fmaf(st[i], sl2, -ls[i]));
          if (!(qr < lq && key < lk && (!causal || key <= qr))) p = 0.f;
          st[i] = p;
          dp[i] = p * (dp[i] - dl[i]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          dva[0][0] = mfma4(dvp[i].x, st[i], dva[0][0]);
          dva[0][1] = mfma4(dvp[i].y, st[i], dva[0][1]);
          dva[0][2] = mfma4(dvp[i].z, st[i], dva[0][2]);
          dva[0][3] = mfma4(dvp[i].w, st[i], dva[0][3]);
          dka[0][0] = mfma4(qvp[i].x, dp[i], dka[0][0]);
          dka[0][1] = mfma4(qvp[i].y, dp[i], dka[0][1]);
          dka[0][2] = mfma4(qvp[i].z, dp[i], dka[0][2]);
          dka[0][3] = mfma4(qvp[i].w, dp[i], dka[0][3]);
        }
        f32x4 dst = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) dst = mfma4(dp[s2], c == 4 * g + s2 ? 1.f : 0.f, dst);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          acc[0] = mfma4(kv[i].x, dst[i], acc[0]);
          acc[1] = mfma4(kv[i].y, dst[i], acc[1]);
          acc[2] = mfma4(kv[i].z, dst[i], acc[2]);
          acc[3] = mfma4(kv[i].w, dst[i], acc[3]);
        }
      }
      const int key = t * 16 + c;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        rsrc_st4(rk_, (int64_t)key * sdk + 16 * g + 4 * i,
                 make_float4(dka[0][0][i] * scale, dka[0][1][i] * scale, dka[0][2][i] * scale, dka[0][3][i] * scale));
        rsrc_st4(rv_, (int64_t)key * sdv + 16 * g + 4 * i, make_float4(dva[0][0][i], dva[0][1][i], dva[0][2][i], dva[0][3][i]));
      }
    }
    // dQ: partials through LDS in wave order (the workgroup form's sum), one float4 per thread
#pragma unroll
    for (int i = 0; i < 4; ++i)
      *reinterpret_cast<float4*>(&part[wave][c][16 * g + 4 * i]) = make_float4(acc[0][i], acc[1][i], acc[2][i], acc[3][i]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();   // every wave read its second tile: rows >= 64 are free
    asm volatile("" ::: "memory");
    stage_b(un);
    asm volatile("" ::: "memory");
    {
      const int r = tid >> 4, cc = (tid & 15) * 4;
      float4 s4 = *reinterpret_cast<const float4*>(&part[0][r][cc]);
#pragma unroll
      for (int w = 1; w < NW; ++w) {
        const float4 a = *reinterpret_cast<const float4*>(&part[w][r][cc]);
        s4.x += a.x; s4.y += a.y; s4.z += a.z; s4.w += a.w;
      }
      // stores (18 per wave): dQ row r (dropped past lq), dK / dV rows of both tiles (dropped past lk), delta
      const __amdgpu_buffer_rsrc_t rq_ = wave_rsrc(dq + q0 * sdq + hh * HD, (int64_t)lq * sdq * 4);
      rsrc_st4(rq_, (int64_t)r * sdq + cc, make_float4(s4.x * scale, s4.y * scale, s4.z * scale, s4.w * scale));
    }
    {
      const __amdgpu_buffer_rsrc_t rd_ = wave_rsrc(delta_out + (int64_t)hh * Tq + q0, (int64_t)lq * 4);
      rsrc_st1(rd_, c, delta);   // (every wave and lane group: the same value to the same row)
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the extra DMA of the last unit lands before the exit
}

// ----------------------------------------------- fused backward over short query and key ranges
// The one-pass form of the few-query kernel above for self-attention over <= R rows (the Amazon encoder's
// contexts, n <= 81: R = 96): one workgroup per (sequence, head), Q and dO staged by LDS-DMA (swizzled
// images, as the dK/dV pass), each wave owning key tiles t = wave, wave + NW with K / V fragments and its
// dK / dV accumulators in registers for the whole launch. Query tiles run in lock-step over the waves: per
// tile each wave forms S and dP against its keys (once), P and dS -> dV^T, dK^T, then dS^T (exact
// permutation MFMAs) -> its partial dQ^T of the tile; the partials meet in an LDS slot per wave and are
// summed in wave order (deterministic) by the whole workgroup. delta = rowsum(dO * O) and lse per query are
// staged in LDS first. 5 products + the transpose per tile pair (the two-pass form: 7), Q / dO / K / V read
// once.
#ifndef RQ_ATTN_SHORT_PAIR
#define RQ_ATTN_SHORT_PAIR 1   // 0: a wave's two key tiles one after the other (A/B: same bits)
#endif
template <int NW, int R>
__global__ void __launch_bounds__(64 * NW, 2) attn_bwd_short_fused_kernel(
    const float* __restrict__ q, int64_t sq, const float* __restrict__ k, int64_t sk, const float* __restrict__ v,
    int64_t sv, const float* __restrict__ out, int64_t so, const float* __restrict__ dout, int64_t sdo,
    const float* __restrict__ lse, int64_t Tq, const int64_t* __restrict__ cu_q, const int64_t* __restrict__ cu_k,
    int causal, float scale, float* __restrict__ dq, int64_t sdq, float* __restrict__ dk, int64_t sdk,
    float* __restrict__ dv, int64_t sdv, int64_t Tk, float* __restrict__ delta_out,
    const int* __restrict__ order) {
  constexpr int HD = 64, NT = R / 16, TPW = (NT + NW - 1) / NW;
  static_assert(R % 16 == 0 && R <= 128 && TPW <= 2, "staged rows");
  __shared__ __attribute__((aligned(16))) char lds[2 * R * 256];
  __shared__ __attribute__((aligned(16))) float part[NW][16][HD + kPartPad];
  __shared__ float lse_s[R], dl_s[R];
  char* Q_s = lds;
  char* O_s = lds + R * 256;
  const int z = blockIdx.z, hh = blockIdx.y, tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, c = lane & 15;
  if (z == (int)gridDim.z - 1) {   // tail slice: rows past the last sequence
    zero_rows<HD, 64 * NW>(dq, sdq, cu_q[z], Tq, hh, tid);
    zero_rows<HD, 64 * NW>(dk, sdk, cu_k[z], Tk, hh, tid);
    zero_rows<HD, 64 * NW>(dv, sdv, cu_k[z], Tk, hh, tid);
    return;
  }
  const int b = seq_of(order, z);   // longest-first when an LPT order is given
  const int64_t q0 = cu_q[b], k0 = cu_k[b];
  const int lq = (int)(cu_q[b + 1] - q0), lk = (int)(cu_k[b + 1] - k0);
  const int nqt = min((lq + 15) >> 4, NT), nkt = min((lk + 15) >> 4, NT);
  if (lq > 0) dma_rows2<NW>(q + q0 * sq + hh * HD, sq, dout + q0 * sdo + hh * HD, sdo, lq, nqt, Q_s, O_s, wave, lane);
  // this wave's key tiles (registers for the whole launch): K, V in the K pattern, K in the V pattern
  const float* kb_ = k + k0 * sk + hh * HD;
  const float* vb_ = v + k0 * sv + hh * HD;
  float4 kp[TPW][4], vk[TPW][4], kv[TPW][4];
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int t = wave + j * NW;
    if (t < nkt) {
      frag_kpat(kb_, sk, t, lk, lane, kp[j]);
      frag_kpat(vb_, sv, t, lk, lane, vk[j]);
      frag_vpat(kb_, sk, t, lk, lane, kv[j]);
    }
  }
  // lse (log2 units) and delta = rowsum(dO * O) per query: 4 lanes per row, 16 d each
  for (int r0 = 0; r0 < 16 * nqt; r0 += 16 * NW) {
    const int r = r0 + (tid >> 2);
    const bool ok = r < lq;
    const int64_t row = q0 + (ok ? r : 0);
    float d = 0.f;
    if (ok) {
      const float* po = out + row * so + hh * HD + 16 * (tid & 3);
      const float* pd = dout + row * sdo + hh * HD + 16 * (tid & 3);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float4 a = *reinterpret_cast<const float4*>(po + 4 * u);
        const float4 e = *reinterpret_cast<const float4*>(pd + 4 * u);
        d += a.x * e.x + a.y * e.y + a.z * e.z + a.w * e.w;
      }
    }
    d += __shfl_xor(d, 1, 64);
    d += __shfl_xor(d, 2, 64);
    if ((tid & 3) == 0 && r < R) {
      dl_s[r] = ok ? d : 0.f;
      lse_s[r] = ok ? lse[(int64_t)hh * Tq + row] * kLog2e : 0.f;
      if (ok) delta_out[(int64_t)hh * Tq + row] = d;
    }
  }
  float pe[4];   // 0/1 permutation operand of the dS transpose (attn_bwd_fewq_fused_kernel)
#pragma unroll
  for (int s = 0; s < 4; ++s) pe[s] = c == 4 * g + s ? 1.f : 0.f;
  f32x4 dka[TPW][4], dva[TPW][4];
#pragma unroll
  for (int j = 0; j < TPW; ++j)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) { dka[j][dt] = f32x4{0.f, 0.f, 0.f, 0.f}; dva[j][dt] = f32x4{0.f, 0.f, 0.f, 0.f}; }
  const float sl2 = scale * kLog2e;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMAs (and fragments) landed
  __syncthreads();                                     // ... and every other wave's; lse / delta staged
  for (int qt = 0; qt < nqt; ++qt) {
    f32x4 acc[4];   // this wave's partial dQ^T of query tile qt
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) acc[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    float dl[4], ls[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      dl[i] = dl_s[qt * 16 + 4 * g + i];
      ls[i] = lse_s[qt * 16 + 4 * g + i];
    }
    // both key tiles of this wave live for this query tile (wave-uniform): their S / dP, dV / dK and dS^T chains
    // interleaved, each Q / dO chunk read from LDS once for both — the same products in the same per-
    // accumulator order as the tile-by-tile loop below (dQ^T: tile 0's terms, then tile 1's), so the same bits
    const bool two = RQ_ATTN_SHORT_PAIR && TPW == 2 && wave + NW < nkt && (!causal || wave + NW <= qt);
    if constexpr (TPW == 2) {
      if (two) {
        f32x4 st0 = f32x4{0.f, 0.f, 0.f, 0.f}, st1 = st0, dp0 = st0, dp1 = st0;
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          const float4 a = lds_chunk(Q_s, qt * 16 + c, 4 * g + s4);
          const float4 e = lds_chunk(O_s, qt * 16 + c, 4 * g + s4);
          st0 = mfma4(a.x, kp[0][s4].x, st0);
          st1 = mfma4(a.x, kp[1][s4].x, st1);
          dp0 = mfma4(e.x, vk[0][s4].x, dp0);
          dp1 = mfma4(e.x, vk[1][s4].x, dp1);
          st0 = mfma4(a.y, kp[0][s4].y, st0);
          st1 = mfma4(a.y, kp[1][s4].y, st1);
          dp0 = mfma4(e.y, vk[0][s4].y, dp0);
          dp1 = mfma4(e.y, vk[1][s4].y, dp1);
          st0 = mfma4(a.z, kp[0][s4].z, st0);
          st1 = mfma4(a.z, kp[1][s4].z, st1);
          dp0 = mfma4(e.z, vk[0][s4].z, dp0);
          dp1 = mfma4(e.z, vk[1][s4].z, dp1);
          st0 = mfma4(a.w, kp[0][s4].w, st0);
          st1 = mfma4(a.w, kp[1][s4].w, st1);
          dp0 = mfma4(e.w, vk[0][s4].w, dp0);
          dp1 = mfma4(e.w, vk[1][s4].w, dp1);
        }
        const int key0 = wave * 16 + c, key1 = (wave + NW) * 16 + c;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int qr = qt * 16 + 4 * g + i;
          float p0 = exp2_fast(__builtin_fmaf(st0[i], sl2, -ls[i]));
          float p1 = exp2_fast(__builtin_fmaf(st1[i], sl2, -ls[i]));
          if (!(qr < lq && key0 < lk && (!causal || key0 <= qr))) p0 = 0.f;
          if (!(qr < lq && key1 < lk && (!causal || key1 <= qr))) p1 = 0.f;
          st0[i] = p0;
          st1[i] = p1;
          dp0[i] = p0 * (dp0[i] - dl[i]);
          dp1[i] = p1 * (dp1[i] - dl[i]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float4 oo = lds_chunk(O_s, qt * 16 + 4 * g + i, c);
          const float4 qq = lds_chunk(Q_s, qt * 16 + 4 * g + i, c);
          dva[0][0] = mfma4(oo.x, st0[i], dva[0][0]);
          dva[1][0] = mfma4(oo.x, st1[i], dva[1][0]);
          dva[0][1] = mfma4(oo.y, st0[i], dva[0][1]);
          dva[1][1] = mfma4(oo.y, st1[i], dva[1][1]);
          dva[0][2] = mfma4(oo.z, st0[i], dva[0][2]);
          dva[1][2] = mfma4(oo.z, st1[i], dva[1][2]);
          dva[0][3] = mfma4(oo.w, st0[i], dva[0][3]);
          dva[1][3] = mfma4(oo.w, st1[i], dva[1][3]);
          dka[0][0] = mfma4(qq.x, dp0[i], dka[0][0]);
          dka[1][0] = mfma4(qq.x, dp1[i], dka[1][0]);
          dka[0][1] = mfma4(qq.y, dp0[i], dka[0][1]);
          dka[1][1] = mfma4(qq.y, dp1[i], dka[1][1]);
          dka[0][2] = mfma4(qq.z, dp0[i], dka[0][2]);
          dka[1][2] = mfma4(qq.z, dp1[i], dka[1][2]);
          dka[0][3] = mfma4(qq.w, dp0[i], dka[0][3]);
          dka[1][3] = mfma4(qq.w, dp1[i], dka[1][3]);
        }
        f32x4 dst0 = f32x4{0.f, 0.f, 0.f, 0.f}, dst1 = dst0;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          dst0 = mfma4(dp0[s], pe[s], dst0);
          dst1 = mfma4(dp1[s], pe[s], dst1);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {   // tile 0's dQ^T terms first (the loop's order)
          acc[0] = mfma4(kv[0][i].x, dst0[i], acc[0]);
          acc[1] = mfma4(kv[0][i].y, dst0[i], acc[1]);
          acc[2] = mfma4(kv[0][i].z, dst0[i], acc[2]);
          acc[3] = mfma4(kv[0][i].w, dst0[i], acc[3]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          acc[0] = mfma4(kv[1][i].x, dst1[i], acc[0]);
          acc[1] = mfma4(kv[1][i].y, dst1[i], acc[1]);
          acc[2] = mfma4(kv[1][i].z, dst1[i], acc[2]);
          acc[3] = mfma4(kv[1][i].w, dst1[i], acc[3]);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const int t = wave + j * NW;
      if (!two && t < nkt && (!causal || t <= qt)) {
        f32x4 st = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {   // S = Q K^T, dP = dO V^T (queries on rows, keys on lanes)
          const float4 a = lds_chunk(Q_s, qt * 16 + c, 4 * g + s4);
          const float4 e = lds_chunk(O_s, qt * 16 + c, 4 * g + s4);
          st = mfma4(a.x, kp[j][s4].x, st);
          dp = mfma4(e.x, vk[j][s4].x, dp);
          st = mfma4(a.y, kp[j][s4].y, st);
          dp = mfma4(e.y, vk[j][s4].y, dp);
          st = mfma4(a.z, kp[j][s4].z, st);
          dp = mfma4(e.z, vk[j][s4].z, dp);
          st = mfma4(a.w, kp[j][s4].w, st);
          dp = mfma4(e.w, vk[j][s4].w, dp);
        }
        const int key = t * 16 + c;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int qr = qt * 16 + 4 * g + i;
          float p = exp2_fast(__builtin_fmaf(st[i], sl2, -ls[i]));
          if (!(qr < lq && key < lk && (!causal || key <= qr))) p = 0.f;
          st[i] = p;
          dp[i] = p * (dp[i] - dl[i]);   // dS
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {   // dV^T += dO^T P, dK^T += Q^T dS (k = query 4 g + i of the tile)
          const float4 oo = lds_chunk(O_s, qt * 16 + 4 * g + i, c);
          const float4 qq = lds_chunk(Q_s, qt * 16 + 4 * g + i, c);
          dva[j][0] = mfma4(oo.x, st[i], dva[j][0]);
          dva[j][1] = mfma4(oo.y, st[i], dva[j][1]);
          dva[j][2] = mfma4(oo.z, st[i], dva[j][2]);
          dva[j][3] = mfma4(oo.w, st[i], dva[j][3]);
          dka[j][0] = mfma4(qq.x, dp[i], dka[j][0]);
          dka[j][1] = mfma4(qq.y, dp[i], dka[j][1]);
          dka[j][2] = mfma4(qq.z, dp[i], dka[j][2]);
          dka[j][3] = mfma4(qq.w, dp[i], dka[j][3]);
        }
        f32x4 dst = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 4; ++s) dst = mfma4(dp[s], pe[s], dst);   // dS^T
#pragma unroll
        for (int i = 0; i < 4; ++i) {   // dQ^T += K^T dS^T
          acc[0] = mfma4(kv[j][i].x, dst[i], acc[0]);
          acc[1] = mfma4(kv[j][i].y, dst[i], acc[1]);
          acc[2] = mfma4(kv[j][i].z, dst[i], acc[2]);
          acc[3] = mfma4(kv[j][i].w, dst[i], acc[3]);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
      *reinterpret_cast<float4*>(&part[wave][c][16 * g + 4 * i]) = make_float4(acc[0][i], acc[1][i], acc[2][i], acc[3][i]);
    __syncthreads();
    constexpr int TPR = HD / 4;
    for (int e = tid; e < 16 * TPR; e += 64 * NW) {
      const int r = e / TPR, cc = (e % TPR) * 4;
      if (qt * 16 + r >= lq) continue;
      float4 s4 = *reinterpret_cast<const float4*>(&part[0][r][cc]);
#pragma unroll
      for (int w = 1; w < NW; ++w) {
        const float4 a = *reinterpret_cast<const float4*>(&part[w][r][cc]);
        s4.x += a.x; s4.y += a.y; s4.z += a.z; s4.w += a.w;
      }
      *reinterpret_cast<float4*>(dq + (q0 + qt * 16 + r) * sdq + hh * HD + cc) =
          make_float4(s4.x * scale, s4.y * scale, s4.z * scale, s4.w * scale);
    }
    __syncthreads();   // the slots are rewritten by the next query tile
  }
#pragma unroll
  for (int j = 0; j < TPW; ++j) {   // dK / dV of this wave's key tiles (zeros when no query sees them)
    const int t = wave + j * NW;
    const int key = t * 16 + c;
    if (t < nkt && key < lk) {
      float* rk = dk + (k0 + key) * sdk + hh * HD + 16 * g;
      float* rv = dv + (k0 + key) * sdv + hh * HD + 16 * g;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        *reinterpret_cast<float4*>(rk + 4 * i) =
            make_float4(dka[j][0][i] * scale, dka[j][1][i] * scale, dka[j][2][i] * scale, dka[j][3][i] * scale);
        *reinterpret_cast<float4*>(rv + 4 * i) = make_float4(dva[j][0][i], dva[j][1][i], dva[j][2][i], dva[j][3][i]);
      }
    }
  }
}

#ifndef RQ_ATTN_SHORT
#define RQ_ATTN_SHORT 1   // 0: the chunked kernels for every length (A/B switch)
#endif
#ifndef RQ_ATTN_SHORT_MAX_STAGED
#define RQ_ATTN_SHORT_MAX_STAGED 32   // longest staged range served by the short forms (A/B: 32 / 128)
#endif
constexpr int kShortMax = 128;   // longest staged range of the short forms

// (waves, staged rows) of a short-form launch whose tiles run over `rows` (queries for fwd / dQ, keys
// for dK/dV) against a staged range of `staged` rows; false when the chunked kernels serve it
static bool short_plan(int64_t rows, int64_t staged, int* nw, int* ch) {
  if (!RQ_ATTN_SHORT || rows > kShortMax || staged > kShortMax) return false;
  // Measured on MI355X (decoder Amazon step, rocprofv3): the short forms win where the staged range
  // is one 32-row chunk (decoder self-attention 5 x 5: fwd 11.6 -> 6.4 us, dQ 15.6 -> 8.9 us; the
  // cross-attention dK/dV over 5 staged queries 41 -> 24 us) and lose at 96 staged rows (encoder
  // self-attention, n <= 81: fwd 35 -> 39 us, dQ 54 -> 59 us, dK/dV 41 -> 64 us: 52 KB of LDS per
  // workgroup leaves 3 workgroups per CU, and a one-wave workgroup would hold it alone), so longer
  // staged ranges keep the chunked kernels.
  if (staged > RQ_ATTN_SHORT_MAX_STAGED) return false;
  *nw = rows <= 16 ? 1 : 4;
  *ch = staged <= 32 ? 32 : (staged <= 64 ? 64 : (staged <= 96 ? 96 : 128));
  return true;
}

#define RQ_SHORT_SWITCH(NW_, CH_, LAUNCH)                          \
  do {                                                           \
    if ((NW_) == 1) {                                            \
      LAUNCH(1, 32);                                             \
    } else {                                                     \
      switch (CH_) {                                             \
        case 32: LAUNCH(4, 32); break;                           \
        case 64: LAUNCH(4, 64); break;                           \
        case 96: LAUNCH(4, 96); break;                           \
        default: LAUNCH(4, 128); break;                          \
      }                                                          \
    }                                                            \
  } while (0)

// Waves per workgroup by the longest row count: 16 rows per wave; short sequences (the Amazon
// decoder's contexts <= 81 tokens, its 5-6 future tokens) use narrow workgroups so few waves idle
// on padding, long ones (ML-32M <= 801, C5 <= 1281) share each staged 64-row chunk between 4 waves.
static int waves_for(int64_t rows) { return rows <= 16 ? 1 : (rows <= 96 ? 2 : 4); }

#ifndef RQ_ATTN_LPT
#define RQ_ATTN_LPT 1   // longest-first sequence order for long ranges (A/B switch)
#endif
// LPT order where a workgroup's run time varies enough with the sequence to leave a straggler tail
static bool lpt_plan(int64_t B, int64_t max_len) { return RQ_ATTN_LPT && B >= 2 && B <= kOrderMax && max_len > 128; }

#ifndef RQ_ATTN_SPLIT
#define RQ_ATTN_SPLIT 1   // split-key forward for <= 16 queries over > 128 keys (A/B switch)
#endif
// split-key forward: one query tile per sequence, non-causal, long key ranges (cross-attention)
#ifndef RQ_ATTN_SPLIT_MIN_K
#define RQ_ATTN_SPLIT_MIN_K 129   // key ranges from here use the split-key forward (A/B: at the Amazon
#endif                            // contexts, <= 81 keys in 32-key blocks, it ties the chunked form)
// The kernel policy of one call, from its `flags` argument (RQ_ATTN_* in include/rqvae_hip.h; 0 = the
// measured-best forms): LDS-DMA short forms, one-pass backwards, split-key / key-split forwards, and the
// fused backward's query splits (0 = automatic).
struct AttnPolicy {
  bool dma, fused, split;
  int qsplit;
  bool x3;   // RQ_ATTN_SPLIT_BF16: the long-range forwards multiply in split-bf16 (matmul precision 'high')
  bool lpt_short;   // RQ_ATTN_LPT_SHORT: longest-first sequence order for the short / few-query forms too
  bool order_given;   // RQ_ATTN_ORDER_GIVEN: ws[0, B) already holds the LPT order of cu_k (no order launch)
  bool fewq_stream;   // !RQ_ATTN_FEWQ_WG: the 4-wave few-query backward as the persistent LDS-DMA-staged walk
};
static AttnPolicy attn_policy(int flags) {
  return AttnPolicy{!(flags & RQ_ATTN_NO_DMA), !(flags & RQ_ATTN_TWO_PASS), !(flags & RQ_ATTN_NO_SPLIT),
                    (flags >> RQ_ATTN_QSPLIT_SHIFT) & 15, (flags & RQ_ATTN_SPLIT_BF16) != 0,
                    (flags & RQ_ATTN_LPT_SHORT) != 0, (flags & RQ_ATTN_ORDER_GIVEN) != 0,
                    !(flags & RQ_ATTN_FEWQ_WG)};
}
// LPT order of the short / few-query forms (by key length: their work per workgroup grows with it)
static bool short_lpt_plan(int64_t B, const AttnPolicy& pol) { return RQ_ATTN_LPT && pol.lpt_short && B >= 2 && B <= kOrderMax; }

static bool split_plan(int64_t hd, int64_t max_q, int64_t max_k, int causal, const AttnPolicy& pol) {
  return RQ_ATTN_SPLIT && pol.split && hd == 64 && !causal && max_q <= 16 && max_k >= RQ_ATTN_SPLIT_MIN_K;
}
static int split_kb(int64_t max_k) { return max_k <= 128 ? 32 : 128; }   // 32: RQ_ATTN_SPLIT_MIN_K <= 128 builds
// key-split forward for many queries over long keys at low occupancy (attn_fwd_kvsplit_kernel): the C4
// per-rank config (8 sequences x 6 heads x <= 13 query blocks); RQ_ATTN_NO_SPLIT disables it (A/B)
#ifndef RQ_ATTN_KVSPLIT_MAX_WG
#define RQ_ATTN_KVSPLIT_MAX_WG 1024   // unsplit workgroups (B x H x 64-query blocks) up to which it applies
#endif
constexpr int kKvSplitKB = 128;
static bool kvsplit_plan(int64_t B, int64_t H, int64_t hd, int64_t max_q, int64_t max_k, int causal,
                         const AttnPolicy& pol) {
  return pol.split && RQ_ATTN_SPLIT && hd == 64 && !causal && max_q > 16 && max_k > 2 * kKvSplitKB &&
         B * H * ((max_q + 63) / 64) <= RQ_ATTN_KVSPLIT_MAX_WG;
}
static int64_t split_ws_elems(int64_t B, int64_t H, int64_t hd, int64_t max_q, int64_t max_k, int64_t Tq, int causal,
                              const AttnPolicy& pol) {
  if (kvsplit_plan(B, H, hd, max_q, max_k, causal, pol)) return (max_k + kKvSplitKB - 1) / kKvSplitKB * Tq * H * (hd + 2);
  if (!split_plan(hd, max_q, max_k, causal, pol)) return 0;
  const int kb = split_kb(max_k);
  return (max_k + kb - 1) / kb * Tq * H * (hd + 2);
}

// LDS-DMA short forms (attn_fwd_dma_kernel): self-attention style launches (more than one query tile)
// whose key range fits 128 staged rows; RQ_ATTN_NO_DMA keeps the register-staged kernels (A/B).
static int dma_rows_for(int64_t max_k) { return max_k <= 32 ? 32 : (max_k <= 64 ? 64 : (max_k <= 96 ? 96 : 128)); }
static bool dma_fwd_plan(int64_t hd, int64_t max_q, int64_t max_k, const AttnPolicy& pol) {   // also the dQ pass
  return pol.dma && hd == 64 && max_q > 16 && max_k <= 128;
}
static bool dma_kv_plan(int64_t hd, int64_t max_q, int64_t max_k, const AttnPolicy& pol) {    // dK / dV: queries staged
  return pol.dma && hd == 64 && max_k > 16 && max_q <= 128;
}
// one query tile over <= 128 keys (cross-attention, the decoder's short causal self-attention): forward and
// dQ with the key tiles split over the waves (attn_fwd_fewq_kernel / attn_bwd_dq_fewq_kernel)
static bool fewq_plan(int64_t hd, int64_t max_q, int64_t max_k, const AttnPolicy& pol) {
  return pol.dma && hd == 64 && max_q <= 16 && max_k <= 128;
}
static int fewq_waves(int64_t max_k) { return max_k <= 16 ? 1 : (max_k <= 32 ? 2 : 4); }
#ifndef RQ_ATTN_FEWQ_STREAM
#define RQ_ATTN_FEWQ_STREAM 1   // 0: the workgroup-per-unit few-query backward for 4-wave launches too (A/B)
#endif
static int attn_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                hipSuccess || cus <= 0)
      cus = 256;
  }
  return cus;
}
// one-pass backward of the self-attention style short launches (attn_bwd_short_fused_kernel) and of the
// few-query launches (attn_bwd_fewq_fused_kernel); RQ_ATTN_TWO_PASS keeps the two-pass dQ + dK/dV kernels
static bool short_fused_plan(int64_t hd, int64_t max_q, int64_t max_k, const AttnPolicy& pol) {
  return pol.dma && pol.fused && hd == 64 && max_q > 16 && max_q <= 128 && max_k <= 128;
}

template <int HD, int NW>
static void fwd_nw(int64_t B, int64_t H, int64_t max_q, hipStream_t st, const float* q, int64_t sq, const float* k,
                   int64_t sk, const float* v, int64_t sv, const int64_t* cq, const int64_t* ck, int causal, float scale,
                   float* out, int64_t so, float* lse, int64_t Tq, const int* order, bool x3) {
  dim3 g((unsigned)std::max<int64_t>(1, (max_q + 16 * NW - 1) / (16 * NW)), (unsigned)H, (unsigned)B + 1);   // + tail slice
  if constexpr (HD == 64 && NW == 4) {
    if (x3) {
      hipLaunchKernelGGL((attn_fwd_kernel<HD, NW, true>), g, dim3(64 * NW), 0, st, q, sq, k, sk, v, sv, cq, ck, causal,
                         scale, out, so, lse, Tq, order);
      return;
    }
  }
  hipLaunchKernelGGL((attn_fwd_kernel<HD, NW>), g, dim3(64 * NW), 0, st, q, sq, k, sk, v, sv, cq, ck, causal, scale, out,
                     so, lse, Tq, order);
}

template <int HD>
static void launch_fwd(int64_t B, int64_t H, int64_t max_q, int64_t max_k, hipStream_t st, const float* q, int64_t sq,
                       const float* k,
                       int64_t sk, const float* v, int64_t sv, const int64_t* cq, const int64_t* ck, int causal,
                       float scale, float* out, int64_t so, float* lse, int64_t Tq, int* order, float* split_ws,
                       const AttnPolicy& pol) {
  if constexpr (HD == 64) {
    if (split_ws && kvsplit_plan(B, H, HD, max_q, max_k, causal, pol)) {
      const int nsplit = (int)((max_k + kKvSplitKB - 1) / kKvSplitKB);
      constexpr int RPB = 256 / (HD / 4);
      const dim3 gs((unsigned)(((max_q + 63) / 64) * nsplit), (unsigned)H, (unsigned)B);
      const dim3 gc((unsigned)std::max<int64_t>(1, (max_q + RPB - 1) / RPB), (unsigned)H, (unsigned)B + 1);
      if (pol.x3)
        hipLaunchKernelGGL((attn_fwd_kvsplit_kernel<HD, 4, kKvSplitKB, true>), gs, dim3(256), 0, st, q, sq, k, sk, v, sv,
                           cq, ck, scale, Tq, split_ws, nsplit);
      else
        hipLaunchKernelGGL((attn_fwd_kvsplit_kernel<HD, 4, kKvSplitKB>), gs, dim3(256), 0, st, q, sq, k, sk, v, sv, cq,
                           ck, scale, Tq, split_ws, nsplit);
      hipLaunchKernelGGL((attn_fwd_combine_kernel<HD, kKvSplitKB>), gc, dim3(256), 0, st, split_ws, nsplit, cq, ck, Tq, out,
                         so, lse);
      return;
    }
    if (split_ws && split_plan(HD, max_q, max_k, causal, pol)) {
      const int kb = split_kb(max_k);
      const int nsplit = (int)((max_k + kb - 1) / kb);
      constexpr int RPB = 256 / (HD / 4);
      const dim3 gs((unsigned)nsplit, (unsigned)H, (unsigned)B);
      const dim3 gc((unsigned)std::max<int64_t>(1, (max_q + RPB - 1) / RPB), (unsigned)H, (unsigned)B + 1);
      if (pol.x3 && kb == kKvSplitKB) {   // split-bf16: the key-split form (4 waves stage each 128-key block)
        hipLaunchKernelGGL((attn_fwd_kvsplit_kernel<HD, 4, kKvSplitKB, true>), gs, dim3(256), 0, st, q, sq, k, sk, v,
                           sv, cq, ck, scale, Tq, split_ws, nsplit);
        hipLaunchKernelGGL((attn_fwd_combine_kernel<HD, kKvSplitKB>), gc, dim3(256), 0, st, split_ws, nsplit, cq, ck, Tq,
                           out, so, lse);
        return;
      }
#define RQ_SPL(KB_)                                                                                                \
  hipLaunchKernelGGL((attn_fwd_split_kernel<HD, KB_>), gs, dim3(64), 0, st, q, sq, k, sk, v, sv, cq, ck, scale, Tq, \
                     split_ws, nsplit);                                                                            \
  hipLaunchKernelGGL((attn_fwd_combine_kernel<HD, KB_>), gc, dim3(256), 0, st, split_ws, nsplit, cq, ck, Tq, out, so, lse)
      if (kb == 32) { RQ_SPL(32); } else { RQ_SPL(128); }
#undef RQ_SPL
      return;
    }
    const int* sord = nullptr;   // LPT order of the short / few-query forms
    if (order && short_lpt_plan(B, pol) && (fewq_plan(HD, max_q, max_k, pol) || dma_fwd_plan(HD, max_q, max_k, pol))) {
      if (!pol.order_given) hipLaunchKernelGGL(attn_order_kernel, dim3(1), dim3(1024), 0, st, ck, (int)B, order);
      sord = order;
    }
    if (fewq_plan(HD, max_q, max_k, pol)) {
      const dim3 g(1, (unsigned)H, (unsigned)B + 1);   // + tail slice
      switch (fewq_waves(max_k)) {
        case 1: hipLaunchKernelGGL((attn_fwd_fewq_kernel<1>), g, dim3(64), 0, st, q, sq, k, sk, v, sv, cq, ck, causal, scale, out, so, lse, Tq, sord); break;
        case 2: hipLaunchKernelGGL((attn_fwd_fewq_kernel<2>), g, dim3(128), 0, st, q, sq, k, sk, v, sv, cq, ck, causal, scale, out, so, lse, Tq, sord); break;
        default: hipLaunchKernelGGL((attn_fwd_fewq_kernel<4>), g, dim3(256), 0, st, q, sq, k, sk, v, sv, cq, ck, causal, scale, out, so, lse, Tq, sord); break;
      }
      return;
    }
    if (dma_fwd_plan(HD, max_q, max_k, pol)) {
      const dim3 g(1, (unsigned)H, (unsigned)B + 1);   // + tail slice
      if (pol.x3 && max_k > 32) {   // split-bf16 form at matmul 'high'
#define RQ_FX(R_)                                                                                                \
  hipLaunchKernelGGL((attn_fwd_short_x3_kernel<R_>), g, dim3(256), 0, st, q, sq, k, sk, v, sv, cq, ck, causal, scale, \
                     out, so, lse, Tq, sord)
        switch (dma_rows_for(max_k)) {
          case 64: RQ_FX(64); break;
          case 96: RQ_FX(96); break;
          default: RQ_FX(128); break;
        }
#undef RQ_FX
        return;
      }
#define RQ_FD(R_)                                                                                              \
  hipLaunchKernelGGL((attn_fwd_dma_kernel<4, R_>), g, dim3(256), 0, st, q, sq, k, sk, v, sv, cq, ck, causal, scale, \
                     out, so, lse, Tq)
      switch (dma_rows_for(max_k)) {
        case 32: RQ_FD(32); break;
        case 64: RQ_FD(64); break;
        case 96: RQ_FD(96); break;
        default: RQ_FD(128); break;
      }
#undef RQ_FD
      return;
    }
    int nw = 0, ch = 0;
    if (short_plan(max_q, max_k, &nw, &ch)) {
      const dim3 g(1, (unsigned)H, (unsigned)B + 1);   // + tail slice
#define RQ_FS(NW_, CH_)                                                                                            \
  hipLaunchKernelGGL((attn_fwd_short_kernel<HD, NW_, CH_>), g, dim3(64 * NW_), 0, st, q, sq, k, sk, v, sv, cq, ck, \
                     causal, scale, out, so, lse, Tq)
      RQ_SHORT_SWITCH(nw, ch, RQ_FS);
#undef RQ_FS
      return;
    }
  }
  const int* ord = nullptr;
  if (order && lpt_plan(B, max_k)) {
    if (!pol.order_given) hipLaunchKernelGGL(attn_order_kernel, dim3(1), dim3(1024), 0, st, ck, (int)B, order);
    ord = order;
  }
  switch (waves_for(max_q)) {
    case 1: fwd_nw<HD, 1>(B, H, max_q, st, q, sq, k, sk, v, sv, cq, ck, causal, scale, out, so, lse, Tq, ord, false); break;
    case 2: fwd_nw<HD, 2>(B, H, max_q, st, q, sq, k, sk, v, sv, cq, ck, causal, scale, out, so, lse, Tq, ord, false); break;
    default: fwd_nw<HD, 4>(B, H, max_q, st, q, sq, k, sk, v, sv, cq, ck, causal, scale, out, so, lse, Tq, ord, pol.x3); break;
  }
}

template <int HD, int NW>
static void dq_nw(int64_t B, int64_t H, int64_t max_q, hipStream_t st, const float* q, int64_t sq, const float* k,
                  int64_t sk, const float* v, int64_t sv, const float* out, int64_t so, const float* dout, int64_t sdo,
                  const float* lse, int64_t Tq, const int64_t* cq, const int64_t* ck, int causal, float scale, float* dq,
                  int64_t sdq, float* delta) {
  dim3 g((unsigned)std::max<int64_t>(1, (max_q + 16 * NW - 1) / (16 * NW)), (unsigned)H, (unsigned)B + 1);   // + tail slice
  hipLaunchKernelGGL((attn_bwd_dq_kernel<HD, NW>), g, dim3(64 * NW), 0, st, q, sq, k, sk, v, sv, out, so, dout, sdo, lse,
                     Tq, cq, ck, causal, scale, dq, sdq, delta);
}

template <int HD, int NW>
static void dkdv_nw(int64_t B, int64_t H, int64_t max_k, hipStream_t st, const float* q, int64_t sq, const float* k,
                    int64_t sk, const float* v, int64_t sv, const float* dout, int64_t sdo, const float* lse,
                    const float* delta, int64_t Tq, const int64_t* cq, const int64_t* ck, int causal, float scale,
                    float* dk, int64_t sdk, float* dv, int64_t sdv, int64_t Tk) {
  dim3 g((unsigned)std::max<int64_t>(1, (max_k + 16 * NW - 1) / (16 * NW)), (unsigned)H, (unsigned)B + 1);   // + tail slice
  hipLaunchKernelGGL((attn_bwd_dkdv_kernel<HD, NW>), g, dim3(64 * NW), 0, st, q, sq, k, sk, v, sv, dout, sdo, lse, delta,
                     Tq, cq, ck, causal, scale, dk, sdk, dv, sdv, Tk);
}

template <int HD>
static void launch_dq_chunked(int64_t B, int64_t H, int64_t max_q, hipStream_t st, const float* q, int64_t sq,
                              const float* k, int64_t sk, const float* v, int64_t sv, const float* out, int64_t so,
                              const float* dout, int64_t sdo, const float* lse, int64_t Tq, const int64_t* cq,
                              const int64_t* ck, int causal, float scale, float* dq, int64_t sdq, float* delta) {
  switch (waves_for(max_q)) {
    case 1: dq_nw<HD, 1>(B, H, max_q, st, q, sq, k, sk, v, sv, out, so, dout, sdo, lse, Tq, cq, ck, causal, scale, dq, sdq, delta); break;
    case 2: dq_nw<HD, 2>(B, H, max_q, st, q, sq, k, sk, v, sv, out, so, dout, sdo, lse, Tq, cq, ck, causal, scale, dq, sdq, delta); break;
    default: dq_nw<HD, 4>(B, H, max_q, st, q, sq, k, sk, v, sv, out, so, dout, sdo, lse, Tq, cq, ck, causal, scale, dq, sdq, delta); break;
  }
}

template <int HD>
static void launch_bwd(int64_t B, int64_t H, int64_t max_q, int64_t max_k, hipStream_t st, const float* q, int64_t sq,
                       const float* k, int64_t sk, const float* v, int64_t sv, const float* out, int64_t so,
                       const float* dout, int64_t sdo, const float* lse, int64_t Tq, const int64_t* cq, const int64_t* ck,
                       int causal, float scale, float* dq, int64_t sdq, float* dk, int64_t sdk, float* dv, int64_t sdv,
                       int64_t Tk, float* delta, const AttnPolicy& pol, const int* order = nullptr) {
  // dQ pass first: it also writes delta_q = dO.O, which the dK/dV pass reads per query chunk
  bool dq_done = false, kv_done = false;
  if constexpr (HD == 64) {
    int nw = 0, ch = 0;
    const dim3 g(1, (unsigned)H, (unsigned)B + 1);   // + tail slice
    if (short_fused_plan(HD, max_q, max_k, pol)) {
#define RQ_SHF(NW_, R_)                                                                                              \
  hipLaunchKernelGGL((attn_bwd_short_fused_kernel<NW_, R_>), g, dim3(64 * NW_), 0, st, q, sq, k, sk, v, sv, out, so, \
                     dout, sdo, lse, Tq, cq, ck, causal, scale, dq, sdq, dk, sdk, dv, sdv, Tk, delta, order)
      // 4 waves with up to two key tiles each (one key tile per wave, R / 16 waves, measured slower on the
      // Amazon step: 6.20-6.22 vs 6.10-6.15 ms, profiles/r03/short_tpw_ab.txt — more waves idle on short
      // sequences)
      switch (dma_rows_for(std::max(max_q, max_k))) {
        case 32: RQ_SHF(2, 32); break;
        case 64: RQ_SHF(4, 64); break;
        case 96: RQ_SHF(4, 96); break;
        default: RQ_SHF(4, 128); break;
      }
#undef RQ_SHF
      return;
    }
    if (fewq_plan(HD, max_q, max_k, pol) && pol.fused && fewq_waves(max_k) == 4 && RQ_ATTN_FEWQ_STREAM && pol.fewq_stream && Tq > 0 &&
        Tk > 0) {   // persistent workgroups, the next unit staged by LDS-DMA
      const int64_t slots = (int64_t)attn_cus() * (max_k <= 96 ? 2 : 1);
      const dim3 gs((unsigned)std::max<int64_t>(1, std::min<int64_t>(B * H, slots)));
#define RQ_FQS(R_)                                                                                                 \
  hipLaunchKernelGGL((attn_bwd_fewq_stream_kernel<R_>), gs, dim3(256), 0, st, q, sq, k, sk, v, sv, out, so, dout, sdo, \
                     lse, Tq, cq, ck, causal, scale, dq, sdq, dk, sdk, dv, sdv, Tk, delta, order, (int)B, (int)H)
      if (max_k <= 64) { RQ_FQS(64); } else if (max_k <= 96) { RQ_FQS(96); } else { RQ_FQS(128); }
#undef RQ_FQS
      return;
    }
    if (fewq_plan(HD, max_q, max_k, pol) && pol.fused) {
#define RQ_FQF(NW_)                                                                                                   \
  hipLaunchKernelGGL((attn_bwd_fewq_fused_kernel<NW_>), g, dim3(64 * NW_), 0, st, q, sq, k, sk, v, sv, out, so, dout, \
                     sdo, lse, Tq, cq, ck, causal, scale, dq, sdq, dk, sdk, dv, sdv, Tk, delta, order)
      switch (fewq_waves(max_k)) {
        case 1: RQ_FQF(1); break;
        case 2: RQ_FQF(2); break;
        default: RQ_FQF(4); break;
      }
#undef RQ_FQF
      return;
    }
    if (fewq_plan(HD, max_q, max_k, pol)) {
#define RQ_DQF(NW_)                                                                                                   \
  hipLaunchKernelGGL((attn_bwd_dq_fewq_kernel<NW_>), g, dim3(64 * NW_), 0, st, q, sq, k, sk, v, sv, out, so, dout, sdo, \
                     lse, Tq, cq, ck, causal, scale, dq, sdq, delta)
      switch (fewq_waves(max_k)) {
        case 1: RQ_DQF(1); break;
        case 2: RQ_DQF(2); break;
        default: RQ_DQF(4); break;
      }
#undef RQ_DQF
      dq_done = true;
    } else if (dma_fwd_plan(HD, max_q, max_k, pol)) {
#define RQ_DQD(R_)                                                                                                  \
  hipLaunchKernelGGL((attn_bwd_dq_dma_kernel<4, R_>), g, dim3(256), 0, st, q, sq, k, sk, v, sv, out, so, dout, sdo, lse, \
                     Tq, cq, ck, causal, scale, dq, sdq, delta)
      switch (dma_rows_for(max_k)) {
        case 32: RQ_DQD(32); break;
        case 64: RQ_DQD(64); break;
        case 96: RQ_DQD(96); break;
        default: RQ_DQD(128); break;
      }
#undef RQ_DQD
      dq_done = true;
    } else if (short_plan(max_q, max_k, &nw, &ch)) {
#define RQ_DQS(NW_, CH_)                                                                                              \
  hipLaunchKernelGGL((attn_bwd_dq_short_kernel<HD, NW_, CH_>), g, dim3(64 * NW_), 0, st, q, sq, k, sk, v, sv, out, so, \
                     dout, sdo, lse, Tq, cq, ck, causal, scale, dq, sdq, delta)
      RQ_SHORT_SWITCH(nw, ch, RQ_DQS);
#undef RQ_DQS
      dq_done = true;
    }
    if (dma_kv_plan(HD, max_q, max_k, pol)) {
      if (!dq_done) {   // the dK/dV pass reads delta: chunked dQ first
        launch_dq_chunked<HD>(B, H, max_q, st, q, sq, k, sk, v, sv, out, so, dout, sdo, lse, Tq, cq, ck, causal, scale, dq,
                              sdq, delta);
        dq_done = true;
      }
#define RQ_KVD(R_)                                                                                                     \
  hipLaunchKernelGGL((attn_bwd_dkdv_dma_kernel<4, R_>), g, dim3(256), 0, st, q, sq, k, sk, v, sv, dout, sdo, lse, delta, \
                     Tq, cq, ck, causal, scale, dk, sdk, dv, sdv, Tk)
      switch (dma_rows_for(max_q)) {
        case 32: RQ_KVD(32); break;
        case 64: RQ_KVD(64); break;
        case 96: RQ_KVD(96); break;
        default: RQ_KVD(128); break;
      }
#undef RQ_KVD
      kv_done = true;
    } else if (short_plan(max_k, max_q, &nw, &ch)) {
      if (!dq_done) {   // the dK/dV pass reads delta: chunked dQ first
        launch_dq_chunked<HD>(B, H, max_q, st, q, sq, k, sk, v, sv, out, so, dout, sdo, lse, Tq, cq, ck, causal, scale, dq,
                              sdq, delta);
        dq_done = true;
      }
#define RQ_KVS(NW_, CH_)                                                                                                \
  hipLaunchKernelGGL((attn_bwd_dkdv_short_kernel<HD, NW_, CH_>), g, dim3(64 * NW_), 0, st, q, sq, k, sk, v, sv, dout, \
                     sdo, lse, delta, Tq, cq, ck, causal, scale, dk, sdk, dv, sdv, Tk)
      RQ_SHORT_SWITCH(nw, ch, RQ_KVS);
#undef RQ_KVS
      kv_done = true;
    }
  }
  if (!dq_done)
    launch_dq_chunked<HD>(B, H, max_q, st, q, sq, k, sk, v, sv, out, so, dout, sdo, lse, Tq, cq, ck, causal, scale, dq, sdq,
                          delta);
  if (kv_done) return;
  switch (waves_for(max_k)) {
    case 1: dkdv_nw<HD, 1>(B, H, max_k, st, q, sq, k, sk, v, sv, dout, sdo, lse, delta, Tq, cq, ck, causal, scale, dk, sdk, dv, sdv, Tk); break;
    case 2: dkdv_nw<HD, 2>(B, H, max_k, st, q, sq, k, sk, v, sv, dout, sdo, lse, delta, Tq, cq, ck, causal, scale, dk, sdk, dv, sdv, Tk); break;
    default: dkdv_nw<HD, 4>(B, H, max_k, st, q, sq, k, sk, v, sv, dout, sdo, lse, delta, Tq, cq, ck, causal, scale, dk, sdk, dv, sdv, Tk); break;
  }
}

// Fused backward (one launch for dQ, dK, dV: attn_bwd_fused_kernel) where the two-pass form would use the
// chunked dK/dV kernel; the short forms keep the decoder's 5-token self- and cross-attention.
#ifndef RQ_ATTN_FUSED
#define RQ_ATTN_FUSED 1
#endif
#ifndef RQ_ATTN_FUSED_NW
#define RQ_ATTN_FUSED_NW 4   // waves per workgroup = key block / 16
#endif
#ifndef RQ_ATTN_FUSED_CH
#define RQ_ATTN_FUSED_CH 32  // staged query rows per LDS round trip (A/B on MI355X: 32 beats 64 by 4-5 %)
#endif
#ifndef RQ_ATTN_FUSED_MIN_K
#define RQ_ATTN_FUSED_MIN_K 129   // shorter key ranges keep the two-pass form (Amazon n <= 81: 0.25 vs 0.30 ms)
#endif
#ifndef RQ_ATTN_FUSED_MIN_K_FEWQ
#define RQ_ATTN_FUSED_MIN_K_FEWQ 129   // the same threshold for <= 16 queries per sequence (cross-attention;
#endif                                 // A/B from 33 keys: Amazon decoder step 6.53 -> 6.60 ms, fewq_ab.txt)
constexpr int kFusedKB = 16 * RQ_ATTN_FUSED_NW;

static bool fused_plan(int64_t hd, int64_t max_q, int64_t max_k, const AttnPolicy& pol) {
  if (!RQ_ATTN_FUSED || !pol.fused || hd != 64) return false;
  if (max_q <= 16) return max_k >= RQ_ATTN_FUSED_MIN_K_FEWQ;   // few queries (cross-attention): own threshold
  if (max_k < RQ_ATTN_FUSED_MIN_K) return false;
  int nw = 0, ch = 0;
  return !short_plan(max_k, max_q, &nw, &ch);
}

// Query splits of the fused backward: when (sequences x heads x key blocks) workgroups cannot fill the
// chip twice over (ML-32M at 8 sequences per GPU: ~300 workgroups, each walking up to 801 queries), each
// key block's query range is split over up to 4 workgroups (whole 32-query chunks, >= 2 per split);
// their dK / dV partials are summed by attn_kv_reduce_kernel. A call's RQ_ATTN_QSPLIT(n) forces n (1 = off).
static int fused_qsplit(int64_t B, int64_t H, int64_t max_q, int64_t max_k, const AttnPolicy& pol) {
  const int forced = pol.qsplit;
  if (max_q <= 16) return 1;
  const int64_t max_by_len = std::max<int64_t>(1, max_q / (2 * RQ_ATTN_FUSED_CH));
  if (forced > 0) return (int)std::min<int64_t>(std::min(forced, 8), max_by_len);
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                hipSuccess || cus <= 0)
      cus = 256;
  }
  const int64_t wgs = B * H * ((max_k + kFusedKB - 1) / kFusedKB);
  const int64_t want = (6 * (int64_t)cus + wgs - 1) / std::max<int64_t>(1, wgs);   // ~2 rounds of 3 per CU
  return (int)std::max<int64_t>(1, std::min<int64_t>(std::min<int64_t>(want, 4), max_by_len));
}

// floats of dQ partials the fused backward needs: one (Tq, H*hd) slab per key block when a sequence may
// span more than one block
static int64_t fused_part_elems(int64_t H, int64_t hd, int64_t max_q, int64_t max_k, int64_t Tq, const AttnPolicy& pol) {
  if (!fused_plan(hd, max_q, max_k, pol)) return 0;
  const int64_t nkb = (max_k + kFusedKB - 1) / kFusedKB;
  return nkb > 1 ? nkb * Tq * H * hd : 0;
}
// + B ints of LPT order (float slots, padded to 16 B) [+ the query splits' dK / dV partials, Tk >= 0]
static int64_t fused_ws_elems(int64_t B, int64_t H, int64_t hd, int64_t max_q, int64_t max_k, int64_t Tq,
                              const AttnPolicy& pol, int64_t Tk = -1) {
  if (!fused_plan(hd, max_q, max_k, pol)) return 0;
  const int64_t base =
      fused_part_elems(H, hd, max_q, max_k, Tq, pol) + (lpt_plan(B, max_q) ? ((B + 3) & ~(int64_t)3) : 0);
  const int qs = Tk >= 0 ? fused_qsplit(B, H, max_q, max_k, pol) : 1;
  return base + (qs > 1 ? 2 * qs * Tk * H * hd : 0);
}

// the one-pass short / few-query backwards in LPT order (scratch: B ints)
static bool short_lpt_bwd(int64_t B, int64_t hd, int64_t max_q, int64_t max_k, const AttnPolicy& pol) {
  return short_lpt_plan(B, pol) && !fused_plan(hd, max_q, max_k, pol) &&
         (short_fused_plan(hd, max_q, max_k, pol) || (fewq_plan(hd, max_q, max_k, pol) && pol.fused));
}

template <int HD>
static void launch_bwd_fused(int64_t B, int64_t H, int64_t max_q, int64_t max_k, hipStream_t st, const float* q,
                             int64_t sq, const float* k, int64_t sk, const float* v, int64_t sv, const float* out,
                             int64_t so, const float* dout, int64_t sdo, const float* lse, int64_t Tq, const int64_t* cq,
                             const int64_t* ck, int causal, float scale, float* dq, int64_t sdq, float* dk, int64_t sdk,
                             float* dv, int64_t sdv, int64_t Tk, float* delta, float* ws, int64_t ws_elems,
                             const AttnPolicy& pol) {
  if constexpr (HD == 64) {
    constexpr int NW = RQ_ATTN_FUSED_NW, CH = RQ_ATTN_FUSED_CH, KB = 16 * NW;
    const int* ord = nullptr;
    if (lpt_plan(B, max_q)) {   // the order lives after the dQ partials in ws
      int* o = reinterpret_cast<int*>(ws + fused_part_elems(H, HD, max_q, max_k, Tq, pol));
      hipLaunchKernelGGL(attn_order_kernel, dim3(1), dim3(1024), 0, st, cq, (int)B, o);
      ord = o;
    }
    constexpr int LPR = HD / 4 < 16 ? HD / 4 : 16;
    const int64_t threads = Tq * H * LPR;
    if (threads > 0)
      hipLaunchKernelGGL((attn_delta_kernel<HD>), dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, out, so, dout,
                         sdo, Tq, H, delta);
    // query splits only when the caller sized the workspace for them (varlen_attn_bwd_ws_elems with Tk)
    int qs = fused_qsplit(B, H, max_q, max_k, pol);
    if (qs > 1 && ws_elems < fused_ws_elems(B, H, HD, max_q, max_k, Tq, pol, Tk)) qs = 1;
    float* kvpart = qs > 1 ? ws + fused_ws_elems(B, H, HD, max_q, max_k, Tq, pol) : nullptr;
    const dim3 g((unsigned)(std::max<int64_t>(1, (max_k + KB - 1) / KB) * qs), (unsigned)H, (unsigned)B + 1);   // + tail
    if (pol.x3 && NW == 4 && CH == 32)
      hipLaunchKernelGGL((attn_bwd_fused_x3_kernel<NW, CH>), g, dim3(64 * NW), 0, st, q, sq, k, sk, v, sv, dout, sdo, lse,
                         delta, Tq, cq, ck, causal, scale, dq, sdq, ws, dk, sdk, dv, sdv, Tk, ord, qs, kvpart);
    else
      hipLaunchKernelGGL((attn_bwd_fused_kernel<HD, NW, CH>), g, dim3(64 * NW), 0, st, q, sq, k, sk, v, sv, dout, sdo,
                         lse, delta, Tq, cq, ck, causal, scale, dq, sdq, ws, dk, sdk, dv, sdv, Tk, ord, qs, kvpart);
    if (qs > 1 && Tk > 0) {
      const int64_t n = Tk * H * (HD / 4);
      hipLaunchKernelGGL((attn_kv_reduce_kernel<HD>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, kvpart, qs, Tk,
                         H, ck, (int)B, scale, dk, sdk, dv, sdv);
    }
    if ((max_k + KB - 1) / KB > 1 && max_q > 0) {
      constexpr int RPB = 256 / (HD / 4);
      const dim3 gr((unsigned)((max_q + RPB - 1) / RPB), (unsigned)H, (unsigned)B);
      hipLaunchKernelGGL((attn_dq_reduce_kernel<HD, KB>), gr, dim3(256), 0, st, ws, Tq, cq, ck, causal, scale, dq, sdq);
    }
  }
}

static bool attn_args_ok(int64_t B, int64_t H, int64_t hd, int64_t max_q, int64_t max_k) {
  // max_q / max_k bound the grid's x extent and every in-kernel int index (row * stride fits int64)
  return B >= 0 && B < 65535 && H >= 1 && H <= 65535 && (hd == 16 || hd == 32 || hd == 64 || hd == 128) && max_q >= 0 &&
         max_k >= 0 && max_q <= (1 << 24) && max_k <= (1 << 24);
}

}  // namespace rqhip

using namespace rqhip;

extern "C" {

int varlen_attn_fwd_ws_elems(int64_t B, int64_t H, int64_t hd, int64_t max_q, int64_t max_k, int64_t Tq, int causal,
                             int flags, int64_t* elems) {
  RQ_CHECK_ARG(elems, "varlen_attn_fwd_ws_elems: null pointer");
  RQ_CHECK_ARG(attn_args_ok(B, H, hd, max_q, max_k) && Tq >= 0, "varlen_attn_fwd_ws_elems: bad shape");
  // order (B ints, 16-B padded) + split-key partials
  *elems = ((B + 3) & ~(int64_t)3) + split_ws_elems(B, H, hd, max_q, max_k, Tq, causal, attn_policy(flags));
  return 0;
}

int varlen_attn_fwd(const float* q, int64_t sq, const float* k, int64_t sk, const float* v, int64_t sv,
                    const int64_t* cu_q, const int64_t* cu_k, int64_t B, int64_t H, int64_t hd, int64_t max_q,
                    int64_t max_k, int causal, float scale, float* out, int64_t so, float* lse, int64_t Tq, float* ws,
                    int64_t ws_elems, int flags, void* stream) {
  RQ_CHECK_ARG(q && k && v && cu_q && cu_k && out && lse, "varlen_attn_fwd: null pointer");
  RQ_CHECK_ARG(attn_args_ok(B, H, hd, max_q, max_k), "varlen_attn_fwd: bad shape (hd must be 16/32/64/128, B<65535)");
  RQ_CHECK_ARG(sq % 4 == 0 && sk % 4 == 0 && sv % 4 == 0 && so % 4 == 0, "varlen_attn_fwd: row strides must be x4");
  const AttnPolicy pol = attn_policy(flags);
  int* order = nullptr;
  float* split_ws = nullptr;
  if (ws != nullptr) {   // no scratch (ws NULL): natural sequence order, no split-key / key-split forms
    const int64_t ob = (B + 3) & ~(int64_t)3, sp = split_ws_elems(B, H, hd, max_q, max_k, Tq, causal, pol);
    RQ_CHECK_ARG(ws_elems >= ob + sp, "varlen_attn_fwd: workspace %lld < varlen_attn_fwd_ws_elems %lld floats",
                 (long long)ws_elems, (long long)(ob + sp));
    order = reinterpret_cast<int*>(ws);
    split_ws = sp ? ws + ob : nullptr;
  }
  if (B == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  switch (hd) {
    case 16: launch_fwd<16>(B, H, max_q, max_k, st, q, sq, k, sk, v, sv, cu_q, cu_k, causal, scale, out, so, lse, Tq, order, split_ws, pol); break;
    case 32: launch_fwd<32>(B, H, max_q, max_k, st, q, sq, k, sk, v, sv, cu_q, cu_k, causal, scale, out, so, lse, Tq, order, split_ws, pol); break;
    case 64: launch_fwd<64>(B, H, max_q, max_k, st, q, sq, k, sk, v, sv, cu_q, cu_k, causal, scale, out, so, lse, Tq, order, split_ws, pol); break;
    case 128: launch_fwd<128>(B, H, max_q, max_k, st, q, sq, k, sk, v, sv, cu_q, cu_k, causal, scale, out, so, lse, Tq, order, split_ws, pol); break;
  }
  RQ_LAUNCH_CHECK("varlen_attn_fwd");
  return 0;
}

int varlen_attn_bwd_ws_elems(int64_t B, int64_t H, int64_t hd, int64_t max_q, int64_t max_k, int64_t Tq, int64_t Tk,
                             int flags, int64_t* elems) {
  RQ_CHECK_ARG(elems, "varlen_attn_bwd_ws_elems: null pointer");
  RQ_CHECK_ARG(attn_args_ok(B, H, hd, max_q, max_k) && Tq >= 0, "varlen_attn_bwd_ws_elems: bad shape");
  const AttnPolicy pol = attn_policy(flags);
  *elems = fused_ws_elems(B, H, hd, max_q, max_k, Tq, pol, Tk);
  if (*elems == 0 && short_lpt_bwd(B, hd, max_q, max_k, pol)) *elems = (B + 3) & ~(int64_t)3;   // the LPT order
  return 0;
}

int varlen_attn_bwd(const float* q, int64_t sq, const float* k, int64_t sk, const float* v, int64_t sv, const float* out,
                    int64_t so, const float* dout, int64_t sdo, const float* lse, int64_t Tq, const int64_t* cu_q,
                    const int64_t* cu_k, int64_t B, int64_t H, int64_t hd, int64_t max_q, int64_t max_k, int causal,
                    float scale, float* dq, int64_t sdq, float* dk, int64_t sdk, float* dv, int64_t sdv, int64_t Tk,
                    float* delta, float* ws, int64_t ws_elems, int flags, void* stream) {
  RQ_CHECK_ARG(q && k && v && out && dout && lse && cu_q && cu_k && dq && dk && dv && delta,
               "varlen_attn_bwd: null pointer");
  RQ_CHECK_ARG(attn_args_ok(B, H, hd, max_q, max_k), "varlen_attn_bwd: bad shape (hd must be 16/32/64/128, B<65535)");
  RQ_CHECK_ARG(sq % 4 == 0 && sk % 4 == 0 && sv % 4 == 0 && so % 4 == 0 && sdo % 4 == 0 && sdq % 4 == 0 &&
                   sdk % 4 == 0 && sdv % 4 == 0,
               "varlen_attn_bwd: row strides must be x4");
  const AttnPolicy pol = attn_policy(flags);
  // the fused long-range form needs its scratch; a call without one (ws NULL) runs the two-pass form there
  const bool fused = fused_plan(hd, max_q, max_k, pol) && ws != nullptr;
  if (fused) {
    const int64_t need = fused_ws_elems(B, H, hd, max_q, max_k, Tq, pol);
    RQ_CHECK_ARG(ws_elems >= need, "varlen_attn_bwd: workspace %lld < varlen_attn_bwd_ws_elems %lld floats",
                 (long long)ws_elems, (long long)need);
  }
  if (B == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  int* sord = nullptr;
  if (!fused && ws != nullptr && ws_elems >= B && short_lpt_bwd(B, hd, max_q, max_k, pol)) {
    sord = reinterpret_cast<int*>(ws);
    if (!pol.order_given) hipLaunchKernelGGL(attn_order_kernel, dim3(1), dim3(1024), 0, st, cu_k, (int)B, sord);
  }
  if (fused) {
    launch_bwd_fused<64>(B, H, max_q, max_k, st, q, sq, k, sk, v, sv, out, so, dout, sdo, lse, Tq, cu_q, cu_k, causal,
                         scale, dq, sdq, dk, sdk, dv, sdv, Tk, delta, ws, ws_elems, pol);
    RQ_LAUNCH_CHECK("varlen_attn_bwd");
    return 0;
  }
  switch (hd) {
    case 16: launch_bwd<16>(B, H, max_q, max_k, st, q, sq, k, sk, v, sv, out, so, dout, sdo, lse, Tq, cu_q, cu_k, causal, scale, dq, sdq, dk, sdk, dv, sdv, Tk, delta, pol); break;
    case 32: launch_bwd<32>(B, H, max_q, max_k, st, q, sq, k, sk, v, sv, out, so, dout, sdo, lse, Tq, cu_q, cu_k, causal, scale, dq, sdq, dk, sdk, dv, sdv, Tk, delta, pol); break;
    case 64: launch_bwd<64>(B, H, max_q, max_k, st, q, sq, k, sk, v, sv, out, so, dout, sdo, lse, Tq, cu_q, cu_k, causal, scale, dq, sdq, dk, sdk, dv, sdv, Tk, delta, pol, sord); break;
    case 128: launch_bwd<128>(B, H, max_q, max_k, st, q, sq, k, sk, v, sv, out, so, dout, sdo, lse, Tq, cu_q, cu_k, causal, scale, dq, sdq, dk, sdk, dv, sdv, Tk, delta, pol); break;
  }
  RQ_LAUNCH_CHECK("varlen_attn_bwd");
  return 0;
}

}  // extern "C"
