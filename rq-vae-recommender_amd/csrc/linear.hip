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
  bool okm[kF];
  // Branch-free staging: every load is issued (a guarded load compiles to a branch around it and
  // a vmcnt(0) per element). Rows past the chunk read row b_lo and are zeroed by a select (they
  // would add into valid outputs); columns past O / I are clamped in range and left as they are —
  // they only feed output rows / columns >= O / I, which are never written.
  const int scol = (tid & 31) * 4;
  const int64_t gcol = min(o0 + scol, O - 4), xcol = min(i0 + scol, I - 4);
  auto load = [&](int64_t b0) {
#pragma unroll
    for (int j = 0; j < kF; ++j) {
      const int r = (tid >> 5) + 8 * j;
      const int64_t b = b0 + r;
      const bool okb = b < b_hi;
      const int64_t bb = okb ? b : b_lo;
      ra[j] = *reinterpret_cast<const float4*>(g + bb * ldg + gcol);
      rb[j] = *reinterpret_cast<const float4*>(x + bb * ldx + xcol);
      okm[j] = okb;
    }
  };
  // The zero-select happens here, after the loads have landed (a select right after the load
  // would wait for it); per component, since a whole-float4 select lowers through scratch.
  auto stash = [&](int buf) {
#pragma unroll
    for (int j = 0; j < kF; ++j) {
      const int f = tid + 256 * j, r = f >> 5, c = (f & 31) * 4;
      const bool k = okm[j];
      const float4 a = make_float4(k ? ra[j].x : 0.f, k ? ra[j].y : 0.f, k ? ra[j].z : 0.f, k ? ra[j].w : 0.f);
      const float4 v = make_float4(k ? rb[j].x : 0.f, k ? rb[j].y : 0.f, k ? rb[j].z : 0.f, k ? rb[j].w : 0.f);
      *reinterpret_cast<float4*>(&As[buf][r][c]) = a;
      *reinterpret_cast<float4*>(&Bs[buf][r][c]) = v;
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
    // LDS operand pipeline: the two reads for k-pair kp+1 are issued ahead of k-pair kp's four
    // MFMAs (sched_group_barrier pins that order), so no MFMA group waits on its own ds_read.
    // A[o][k] = g[b][o], B[k][i] = x[b][i].
    float2 a = *reinterpret_cast<const float2*>(&As[buf][h][wo * 64 + 2 * c32]);
    float2 v = *reinterpret_cast<const float2*>(&Bs[buf][h][wi * 64 + 2 * c32]);
#pragma unroll
    for (int kp = 0; kp < kWBK / 2; ++kp) {
      float2 an = a, vn = v;
      if (kp + 1 < kWBK / 2) {
        const int k = 2 * (kp + 1) + h;
        an = *reinterpret_cast<const float2*>(&As[buf][k][wo * 64 + 2 * c32]);
        vn = *reinterpret_cast<const float2*>(&Bs[buf][k][wi * 64 + 2 * c32]);
      }
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, v.x, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, v.y, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, v.x, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, v.y, acc[1][1], 0, 0, 0);
      a = an;
      v = vn;
    }
#pragma unroll
    for (int kp = 0; kp < kWBK / 2; ++kp) {
      if (kp + 1 < kWBK / 2) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);   // next k-pair's reads
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);                          // this k-pair's MFMAs
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
// columns x 4 waves; wave w sums s = w, w+4, ... (strided_slab_sum), then
// the four wave partials are added in wave order through LDS. Deterministic, no atomics.
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* __restrict__ P, int S, int64_t n,
                                                           float* __restrict__ out) {
  __shared__ float4 part[4][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t j = ((int64_t)blockIdx.x * 64 + lane) * 4;
  const bool ok = j < n;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (ok) a = strided_slab_sum(P, S, n, j, wave, 4);
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


// ---------------------------------------------------------------------------------------------
// Split-bf16 ("bf16x3") GEMM: the fp32 matmul at torch.set_float32_matmul_precision('high'),
// which the reference selects at import (modules/rqvae.py:19, modules/model.py:27). PyTorch
// defines 'high' as TF32 or "each float32 as the sum of two bfloat16 numbers"; gfx950 has no
// xf32 MFMA, so this is the second form on v_mfma_f32_32x32x16_bf16: a = a_hi + a_lo with
// a_hi = RN_bf16(a), a_lo = RN_bf16(a - a_hi) (the subtraction is exact), and
//   a.b ~ a_hi.b_hi + a_hi.b_lo + a_lo.b_hi        (fp32 accumulation; a_lo.b_lo dropped)
// — per-product relative error <= ~2^-17 (TF32: 2^-11), at 3 bf16 MFMAs per product = 5.3x the
// f32-MFMA rate. 'highest' keeps the exact-f32 path (library GEMM + wgrad_partial_kernel).
//
//   C[m][n] = sum_k A(m, k) B(n, k)
//   A(m, k) = A[m*lda + k] (a_kc: k-contiguous) or A[k*lda + m] (m-contiguous); B likewise.
//   forward  y = x W^T : A = x (k-contig),  B = W (k-contig)
//   dgrad   dx = g W   : A = g (k-contig),  B(n=i, k=o) = W[o][i] (n-contig)
//   wgrad   dW = g^T x : A(m=o, k=b) = g[b][o], B(n=i, k=b) = x[b][i] (both m/n-contig), split-K
//
// Tile 128 x 128 x 32 per workgroup (4 waves, 64 x 64 each = 2 x 2 MFMA tiles). Operands are
// converted to (hi, lo) bf16 planes while staged into LDS (register staging, double-buffered):
//   k-contig operand -> "row image" [128 rows][32 k] (64-B rows, 16-B chunk c stored at
//                       c ^ ((row >> 2) & 3)): fragments by conflict-free ds_read_b128;
//   m/n-contig       -> "column image" [32 k][128 rows] (256-B rows, chunk XOR
//                       ((k & 3) << 2 | (k >> 2) & 3)): fragments by ds_read_b64_tr_b16 (the
//                       hardware transpose read), conflict-free per 32-lane half.
// Both images come from coalesced float4 loads in the operand's HBM layout.
// ---------------------------------------------------------------------------------------------

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));

#ifndef RQ_X3_BK16
#define RQ_X3_BK16 0   // 1: 16-deep k stages (32 KiB LDS, 3 workgroups/CU, 32x32x16 MFMA)
#endif
constexpr int kXT = 128;                       // output tile (m and n)
constexpr int kXK = RQ_X3_BK16 ? 16 : 32;      // k per LDS stage
constexpr int kXCPR = kXK / 8;                 // 16-byte bf16 chunks per row of the row image
constexpr int kXWG = RQ_X3_BK16 ? 3 : 2;       // resident workgroups per CU
constexpr int kXPlane = kXT * kXK * 2;         // bytes of one bf16 plane (8 KiB)
constexpr int kXOp = 2 * kXPlane;              // hi + lo planes of one operand
constexpr int kXBuf = 2 * kXOp;                // A + B
constexpr int kXLds = 2 * kXBuf;               // double buffer: 64 KiB (the 64-tile form: half)
static_assert(kXLds == 65536, "LDS of the 128-tile form");

__device__ __forceinline__ int col_swz(int k) { return ((k & 3) << 2) | ((k >> 2) & 3); }
#ifndef RQ_X3S_COMPACT
#define RQ_X3S_COMPACT 1   // 64-tile form: 128-B column-image rows and 32 KiB of LDS (4 workgroups / CU)
#endif
constexpr int kXWG64 = RQ_X3S_COMPACT ? 4 : kXWG;   // resident workgroups per CU of the 64-tile form
// Byte offset of 16-B chunk `c` of k-row kr in a column image of TR columns: 256-B rows with col_swz
// for TR = 128 (and the wide kernel); for TR = 64 (compact) 128-B rows with a swizzle over the 8 chunks,
// s = 2 ((kr >> 1) & 1) + 4 ((kr >> 3) & 1): a ds_read_b64_tr_b16 half-wave touches k-rows {4u..4u+3,
// 4u+8..4u+11} (+16), chunk pairs (c0, c0 + 1) with c0 even — the even rows land on banks 0-31 and the
// odd rows on 32-63, each row's pair at a distinct s: conflict-free; the staging stores write whole
// 128-B rows per 8- / 16-lane group.
template <int TR>
__device__ __forceinline__ int col_off(int kr, int c) {
  if constexpr (TR == 64 && RQ_X3S_COMPACT) return 128 * kr + ((c ^ ((((kr >> 1) & 1) << 1) | (((kr >> 3) & 1) << 2))) << 4);
  else return 256 * kr + ((c ^ col_swz(kr)) << 4);
}
// Row image: row rr of 2 kXK bytes, 16-B chunk c stored at c ^ row_swz(rr). With the 16x16x32 MFMA
// (default) a fragment read (xfrag16) is a ds_read_b128 whose lane groups {0-3,12-15,20-27},
// {4-11,16-19,28-31} (+32) touch rows {0-3, 12-15} at chunk c and rows 4-11 at chunk c ^ 1: the
// swizzle (rr >> 2) & 2 puts the four rows of equal rr % 4 on four distinct 16-B bank slots (the
// wide kernel's image; (rr >> 2) & 3, designed for the 32x32x16 reads, was 2-way conflicted here:
// SQ_LDS_BANK_CONFLICT 2.6 cycles per LDS instruction). Staging writes (ds_write_b128, 8-lane
// groups over 2 rows) stay conflict-free.
#if RQ_X3_BK16 || (defined(RQ_X3_MFMA16) && !RQ_X3_MFMA16)
__device__ __forceinline__ int row_swz(int rr) { return kXCPR == 4 ? ((rr >> 2) & 3) : ((rr >> 3) & 1); }
#else
__device__ __forceinline__ int row_swz(int rr) { return (rr >> 2) & 2; }
#endif
__device__ __forceinline__ int row_off(int rr, int c) { return rr * (2 * kXK) + ((c ^ row_swz(rr)) << 4); }

// One operand's staging registers (a TR x 32 tile per stage, 256 threads; TR = 128 or 64 rows of m / n).
// Operand formats:
//   fp32  (SP = false): TR / 32 float4 per thread, split into (hi, lo) bf16 while written to LDS;
//   split (SP = true):  two bf16 planes (hi, lo) of the operand's shape, produced once upstream
//                       (rq_split_bf16x3, or a GEMM epilogue): TR / 64 + TR / 64 16-byte chunks per
//                       thread, copied to LDS as they are.
// The LDS images do not depend on TR (a 64-row tile uses the first 64 rows of a row image and the
// first 64 columns of a column image's 256-B rows, with the same swizzles).
// KF ("k full"): every stage of the launch lies inside [k_lo, k_hi) (K and the split-K chunk multiples of
// the stage depth), so no k mask, masked address or zeroing select is emitted.
template <bool KC, bool SP, int TR = 128, bool KF = false>
struct XStage {
  static_assert(TR == 128 || (TR == 64 && kXK == 32), "tile rows (64-row tiles need 32-deep k stages)");
  // fp32, k-contig: float4 per thread (two per 16-B bf16 chunk of the row image)
  static constexpr int NJ_FK = 2 * TR * kXCPR / 256;
  // fp32, m/n-contig: CT threads across the TR columns (4 each), KR k-rows per pass
  static constexpr int CT_F = TR / 4, KR_F = 256 / CT_F, NJ_FM = kXK / KR_F;
  // split, k-contig: hi + lo 16-B chunks per thread
  static constexpr int NJ_SK = TR * kXCPR / 256;
  // split, m/n-contig: CT threads across the TR columns (8 each), KR k-rows per pass
  static constexpr int CT_S = TR / 8, KR_S = 256 / CT_S, NJ_SM = kXK / KR_S;
  uint4 v[4];
  bool ok[4];   // k of the loaded vector < k_hi (else it read k_lo and is zeroed at store time)

  // rows [r0, r0 + TR) of the operand (clamped to R - 1: they feed only outputs >= R, never
  // written); k in [kb, kb + 32), positions >= k_hi read k_lo and are zeroed at store time. Every
  // load is unconditional and its address branch-free (a select), so the compiler can count the
  // loads in flight statically: with separate full-stage / masked-stage load paths it merged the
  // paths' counts and waited vmcnt(0) at the top of every k iteration, draining the prefetch.
  __device__ __forceinline__ void load(const void* __restrict__ Xv, const void* __restrict__ Xlv, int64_t ld, int r0,
                                       int R, int64_t kb, int64_t k_lo, int64_t k_hi, int tid) {
    if constexpr (!SP) {
      const float* __restrict__ X = static_cast<const float*>(Xv);
      if constexpr (KC) {   // thread: chunk tid % CPR of rows tid / CPR (+ 256 / CPR), 2 float4 per chunk
#pragma unroll
        for (int j = 0; j < NJ_FK; ++j) {
          const int64_t row = min(r0 + (tid / kXCPR) + (256 / kXCPR) * (j >> 1), R - 1);
          const int64_t k = kb + (tid % kXCPR) * 8 + 4 * (j & 1);
          ok[j] = KF || k < k_hi;
          v[j] = *reinterpret_cast<const uint4*>(X + row * ld + (ok[j] ? k : k_lo));
        }
      } else {              // thread: 4 consecutive rows 4 (tid % CT), k rows tid / CT + KR j
        const int64_t col = min(r0 + 4 * (tid % CT_F), R - 4);
#pragma unroll
        for (int j = 0; j < NJ_FM; ++j) {
          const int64_t k = kb + (tid / CT_F) + KR_F * j;
          ok[j] = KF || k < k_hi;
          v[j] = *reinterpret_cast<const uint4*>(X + (ok[j] ? k : k_lo) * ld + col);
        }
      }
    } else {
      const uint16_t* __restrict__ Xh = static_cast<const uint16_t*>(Xv);
      const uint16_t* __restrict__ Xl = static_cast<const uint16_t*>(Xlv);
      if constexpr (KC) {   // thread: chunk tid % CPR of rows tid / CPR (+ 256 / CPR)
#pragma unroll
        for (int j = 0; j < NJ_SK; ++j) {
          const int64_t row = min(r0 + (tid / kXCPR) + (256 / kXCPR) * j, R - 1);
          const int64_t k = kb + (tid % kXCPR) * 8;
          ok[j] = KF || k < k_hi;
          const int64_t o = row * ld + (ok[j] ? k : k_lo);
          v[j] = *reinterpret_cast<const uint4*>(Xh + o);
          v[2 + j] = *reinterpret_cast<const uint4*>(Xl + o);
        }
      } else {              // thread: 8 consecutive rows 8 (tid % CT), k rows tid / CT + KR j
        const int64_t col = min(r0 + 8 * (tid % CT_S), R - 8);
#pragma unroll
        for (int j = 0; j < NJ_SM; ++j) {
          const int64_t k = kb + (tid / CT_S) + KR_S * j;
          ok[j] = KF || k < k_hi;
          const int64_t o = (ok[j] ? k : k_lo) * ld + col;
          v[j] = *reinterpret_cast<const uint4*>(Xh + o);
          v[2 + j] = *reinterpret_cast<const uint4*>(Xl + o);
        }
      }
    }
  }

  __device__ __forceinline__ void store(char* hi_plane, char* lo_plane, int tid) const {
    if constexpr (!SP) {
      constexpr int NJ = KC ? NJ_FK : NJ_FM;
      float4 w[4];
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const float4 f = __builtin_bit_cast(float4, v[j]);
        const bool k = ok[j];
        w[j] = make_float4(k ? f.x : 0.f, k ? f.y : 0.f, k ? f.z : 0.f, k ? f.w : 0.f);
      }
      if constexpr (KC) {
#pragma unroll
        for (int c2 = 0; c2 < NJ_FK / 2; ++c2) {
          const int rr = (tid / kXCPR) + (256 / kXCPR) * c2, c = tid % kXCPR;
          const int off = row_off(rr, c);
          uint4 h, l;
          split_bf16x2(w[2 * c2].x, w[2 * c2].y, h.x, l.x);
          split_bf16x2(w[2 * c2].z, w[2 * c2].w, h.y, l.y);
          split_bf16x2(w[2 * c2 + 1].x, w[2 * c2 + 1].y, h.z, l.z);
          split_bf16x2(w[2 * c2 + 1].z, w[2 * c2 + 1].w, h.w, l.w);
          *reinterpret_cast<uint4*>(hi_plane + off) = h;
          *reinterpret_cast<uint4*>(lo_plane + off) = l;
        }
      } else {
        const int m = 4 * (tid % CT_F);
#pragma unroll
        for (int j = 0; j < NJ_FM; ++j) {
          const int kr = (tid / CT_F) + KR_F * j;
          const int off = col_off<TR>(kr, m >> 3) + (((m >> 2) & 1) << 3);
          uint2 h, l;
          split_bf16x2(w[j].x, w[j].y, h.x, l.x);
          split_bf16x2(w[j].z, w[j].w, h.y, l.y);
          *reinterpret_cast<uint2*>(hi_plane + off) = h;
          *reinterpret_cast<uint2*>(lo_plane + off) = l;
        }
      }
    } else {
      constexpr int NJ = KC ? NJ_SK : NJ_SM;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const bool k = ok[j];
        const uint4 h0 = v[j], l0 = v[2 + j];
        const uint4 h = make_uint4(k ? h0.x : 0u, k ? h0.y : 0u, k ? h0.z : 0u, k ? h0.w : 0u);
        const uint4 l = make_uint4(k ? l0.x : 0u, k ? l0.y : 0u, k ? l0.z : 0u, k ? l0.w : 0u);
        int off;
        if constexpr (KC) {
          const int rr = (tid / kXCPR) + (256 / kXCPR) * j, c = tid % kXCPR;
          off = row_off(rr, c);
        } else {
          const int kr = (tid / CT_S) + KR_S * j;
          off = col_off<TR>(kr, tid % CT_S);
        }
        *reinterpret_cast<uint4*>(hi_plane + off) = h;
        *reinterpret_cast<uint4*>(lo_plane + off) = l;
      }
    }
  }
};

// MFMA operand fragment (8 bf16: row rb + lane % 32, k = 16 s + 8 (lane / 32) + 0..7) of a plane.
template <bool KC>
__device__ __forceinline__ bf16x8_t xfrag(const char* plane, int rb, int s, int lane) {
  if constexpr (KC) {
    const int rr = rb + (lane & 31), c = 2 * s + (lane >> 5);
    return *reinterpret_cast<const bf16x8_t*>(plane + row_off(rr, c));
  } else {
    // ds_read_b64_tr_b16: 16-lane group G reads a 4 (k) x 16 (row) block; lane 4q + p supplies
    // the address of k-row q, rows 4p..4p+3, and receives row (lane % 16) of all 4 k-rows.
    const int G = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int m = rb + 16 * (G & 1) + 4 * p;
    s16x4_t t[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int kr = 16 * s + 8 * (G >> 1) + 4 * u + q;
      const int off = 256 * kr + (((m >> 3) ^ col_swz(kr)) << 4) + (((m >> 2) & 1) << 3);
      t[u] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s16x4_t*)(plane + off));
    }
    typedef short s16x8_t __attribute__((ext_vector_type(8)));
    const s16x8_t r = {t[0].x, t[0].y, t[0].z, t[0].w, t[1].x, t[1].y, t[1].z, t[1].w};
    return __builtin_bit_cast(bf16x8_t, r);
  }
}

// 16x16x32 operand fragment (8 bf16: row rb + lane % 16, k = 8 (lane / 16) + 0..7 of the stage).
template <bool KC, int TR = 128>
__device__ __forceinline__ bf16x8_t xfrag16(const char* plane, int rb, int lane) {
  if constexpr (KC) {
    const int rr = rb + (lane & 15), c = lane >> 4;
    return *reinterpret_cast<const bf16x8_t*>(plane + row_off(rr, c));
  } else {
    // ds_read_b64_tr_b16 per 16-lane group G (k-rows 8G .. 8G + 7 in two 4-row blocks): lane
    // 4q + p supplies the address of k-row q, rows 4p..4p+3, and receives row (lane % 16).
    const int G = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int m = rb + 4 * p;
    s16x4_t t[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int kr = 8 * G + 4 * u + q;
      const int off = col_off<TR>(kr, m >> 3) + (((m >> 2) & 1) << 3);
      t[u] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s16x4_t*)(plane + off));
    }
    typedef short s16x8_t __attribute__((ext_vector_type(8)));
    const s16x8_t r = {t[0].x, t[0].y, t[0].z, t[0].w, t[1].x, t[1].y, t[1].z, t[1].w};
    return __builtin_bit_cast(bf16x8_t, r);
  }
}

#ifndef RQ_X3_DEPTH
#define RQ_X3_DEPTH 2    // register stage sets in flight (2 or 3; 3 spills on the transposed-B variants)
#endif

#ifndef RQ_X3S_DEPTH
#define RQ_X3S_DEPTH 2   // stage sets in flight of the 64-tile form (A/B on MI355X: 2, 3, 4 within 3 %)
#endif

#ifndef RQ_X3_SETPRIO
#define RQ_X3_SETPRIO 0   // 1: s_setprio(1) around each stage's MFMA cluster (guide T5; measured -1 %)
#endif
#if RQ_X3_SETPRIO
#define RQ_X3_PRIO(P) __builtin_amdgcn_s_setprio(P);
#else
#define RQ_X3_PRIO(P)
#endif

#ifndef RQ_X3_MAX_SPLIT
#define RQ_X3_MAX_SPLIT 64   // split-K: at most this many k chunks
#endif

#ifndef RQ_X3_MIN_STAGES
#define RQ_X3_MIN_STAGES 2   // split-K: k-stages per workgroup at least (fewer slabs to reduce)
#endif

#ifndef RQ_X3_INTERLEAVE
#define RQ_X3_INTERLEAVE 0   // 1: next-stage LDS writes between the MFMAs (measured 20 % slower); 2: the
                             // 128-tile stage as 8 groups of (6 MFMA, 1 LDS write, 7 VALU) after its reads
#endif

#ifndef RQ_X3_PEEL
#define RQ_X3_PEEL 1   // 0: the second stage slot of each loop iteration multiplies under a runtime test (the
                       // round-4 loop; the MFMAs then sit in their own basic block, apart from the staging)
#endif

#ifndef RQ_X3_MFMA16
#define RQ_X3_MFMA16 (RQ_X3_BK16 ? 0 : 1)   // 16x16x32 bf16 MFMA (4 x 4 tiles per wave); 0: 32x32x16 (2 x 2)
#endif
static_assert(!(RQ_X3_MFMA16 && RQ_X3_BK16), "16x16x32 MFMA needs 32-deep k stages");

// Epilogues: what the accumulator tile becomes (all fp32 math; dropout mask = keep1(seed, m N + n),
// the convention of the standalone dropout kernels, dropout.hip).
enum X3Epi : int {
  kEpiStore = 0,     // C = A B^T (fp32; split-K slabs when S > 1)
  kEpiSiluFwd = 1,   // C = z = A B^T (fp32, kept for the backward); H = split(Dropout(SiLU(z)))
  kEpiSiluBwd = 2,   // H = split(SiLU'(Z) * Dropout(A B^T)): the pre-activation grad of a hidden layer
  kEpiAdd = 3,       // C = A B^T + Z (fp32; the residual add after an attention projection); with dropout
                     // C = Z + Dropout(A B^T) (the block output h + Dropout(MLP(.)))
};

struct X3Epilogue {
  const float* Z;    // kEpiSiluBwd: pre-activations (ld = ldc)
  uint16_t* Hh;      // split output planes (ld = ldh)
  uint16_t* Hl;
  int64_t ldh;
  uint32_t thr;      // dropout threshold (0 = none) and scale
  float scale;
  uint64_t seed;
  int acc;           // kEpiStore, unsplit: C += A B^T (an accumulating call without the slab reduction)
};

// Epilogue SiLU on the hardware exp / reciprocal (v_exp_f32, v_rcp_f32: ~1 ulp each) instead of
// the IEEE expf + division of the standalone kernels (dropout.hip): the result is split to bf16
// planes at ~2^-17 right after, so the last bits do not survive anyway, and the epilogue VALU drops
// ~3x. s = sigmoid(z) = 1 / (1 + 2^(-z log2 e)).
__device__ __forceinline__ float sigmoid_fast(float z) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * z));
}

// Epilogue stores; NT: non-temporal (the wide kernel's all-CU write bursts, A/B RQ_X3W_NT)
typedef unsigned ux4_t __attribute__((ext_vector_type(4)));
typedef unsigned ux2_t __attribute__((ext_vector_type(2)));
template <bool NT>
__device__ __forceinline__ void epi_st16(void* p, float4 v) {
  if constexpr (NT) __builtin_nontemporal_store(__builtin_bit_cast(ux4_t, v), reinterpret_cast<ux4_t*>(p));
  else *reinterpret_cast<float4*>(p) = v;
}
template <bool NT>
__device__ __forceinline__ void epi_st8(void* p, uint2 v) {
  if constexpr (NT) __builtin_nontemporal_store(__builtin_bit_cast(ux2_t, v), reinterpret_cast<ux2_t*>(p));
  else *reinterpret_cast<uint2*>(p) = v;
}

// What the epilogue of lane quad (m, n .. n + 3) reads besides the accumulators: Z (SiLU', residual add) or,
// for an accumulating plain store, the current C quad; zeros otherwise. Loaded for a whole group of quads
// before any of their stores (x3_epi4z): the output pointers may alias Z for the compiler, so a load written
// after a store waits for that store and its own round trip, one quad at a time.
template <int EPI>
__device__ __forceinline__ float4 x3_epi_in(int m, int n, float* __restrict__ Cs, int64_t ldc, const X3Epilogue& ep) {
  if constexpr (EPI == kEpiSiluBwd || EPI == kEpiAdd) {
    return *reinterpret_cast<const float4*>(ep.Z + (int64_t)m * ldc + n);
  } else if constexpr (EPI == kEpiStore) {
    if (ep.acc) return *reinterpret_cast<const float4*>(Cs + (int64_t)m * ldc + n);
  }
  return make_float4(0.f, 0.f, 0.f, 0.f);
}

// Epilogue of one lane quad C[m][n .. n + 3] = v (fp32 accumulator values) with its input quad z
// (x3_epi_in); Cs = the split-K slab (kEpiStore) or C itself.
template <int EPI, bool DROP, bool NT = false>
__device__ __forceinline__ void x3_epi4z(const float4 v, const float4 z, int m, int n, int N, float* __restrict__ C,
                                         float* __restrict__ Cs, int64_t ldc, const X3Epilogue& ep) {
  if constexpr (EPI == kEpiStore) {
    float4* c = reinterpret_cast<float4*>(Cs + (int64_t)m * ldc + n);
    if (ep.acc) {   // fixed order c + v: bitwise the slab reduction's C[j] + P[0][j]
      const float4 o = z;
      epi_st16<NT>(c, make_float4(o.x + v.x, o.y + v.y, o.z + v.z, o.w + v.w));
    } else {
      epi_st16<NT>(c, v);
    }
  } else if constexpr (EPI == kEpiAdd) {
    const float4 r = z;
    if constexpr (DROP) {   // C = Z + Dropout(A B^T): dropout_add_fwd's mask (element m N + n) and arithmetic
      const uint64_t e = (uint64_t)m * N + n;
      float d[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) d[j] = keep1(ep.seed, e + j, ep.thr) ? ep.scale : 0.f;
      epi_st16<NT>(C + (int64_t)m * ldc + n, make_float4(r.x + v.x * d[0], r.y + v.y * d[1], r.z + v.z * d[2], r.w + v.w * d[3]));
    } else {
      epi_st16<NT>(C + (int64_t)m * ldc + n, make_float4(v.x + r.x, v.y + r.y, v.z + r.z, v.w + r.w));
    }
  } else {
    const uint64_t e = (uint64_t)m * N + n;
    float d[4] = {1.f, 1.f, 1.f, 1.f};   // dropout multipliers (0 or 1 / (1 - p))
    if constexpr (DROP) {
#pragma unroll
      for (int j = 0; j < 4; ++j) d[j] = keep1(ep.seed, e + j, ep.thr) ? ep.scale : 0.f;
    }
    float4 o;
    if constexpr (EPI == kEpiSiluFwd) {
      epi_st16<NT>(C + (int64_t)m * ldc + n, v);
      o = make_float4(v.x * sigmoid_fast(v.x) * d[0], v.y * sigmoid_fast(v.y) * d[1], v.z * sigmoid_fast(v.z) * d[2],
                      v.w * sigmoid_fast(v.w) * d[3]);
    } else {   // silu'(z) g = g s (1 + z (1 - s)), g = Dropout(A B^T)
      const float sx = sigmoid_fast(z.x), sy = sigmoid_fast(z.y), sz = sigmoid_fast(z.z), sw = sigmoid_fast(z.w);
      o = make_float4(v.x * d[0] * sx * (1.f + z.x * (1.f - sx)), v.y * d[1] * sy * (1.f + z.y * (1.f - sy)),
                      v.z * d[2] * sz * (1.f + z.z * (1.f - sz)), v.w * d[3] * sw * (1.f + z.w * (1.f - sw)));
    }
    uint2 hi, lo;
    split_bf16x2(o.x, o.y, hi.x, lo.x);
    split_bf16x2(o.z, o.w, hi.y, lo.y);
    epi_st8<NT>(ep.Hh + (int64_t)m * ep.ldh + n, hi);
    epi_st8<NT>(ep.Hl + (int64_t)m * ep.ldh + n, lo);
  }
}

template <int EPI, bool DROP, bool NT = false>
__device__ __forceinline__ void x3_epi4(const float4 v, int m, int n, int N, float* __restrict__ C,
                                        float* __restrict__ Cs, int64_t ldc, const X3Epilogue& ep) {
  x3_epi4z<EPI, DROP, NT>(v, x3_epi_in<EPI>(m, n, Cs, ldc, ep), m, n, N, C, Cs, ldc, ep);
}

__device__ __forceinline__ void split_store1(float v, uint16_t* hi, uint16_t* lo) {
  const __bf16 h = (__bf16)v;
  *hi = __builtin_bit_cast(uint16_t, h);
  *lo = __builtin_bit_cast(uint16_t, (__bf16)(v - (float)h));
}

// One LDS stage of MFMA work per wave. Transposed product D = B A^T (tile rows = n, columns = m):
// each lane then holds consecutive n of one row m, so the epilogue stores vectors.
#if RQ_X3_MFMA16
#define RQ_X3_MMA                                                                                             \
  {                                                                                                           \
    bf16x8_t fa_h[kP], fa_l[kP], fb_h[kP], fb_l[kP];                                                          \
    _Pragma("unroll") for (int p = 0; p < kP; ++p) {                                                          \
      fa_h[p] = xfrag16<AKC, TS>(ah, wm * kWTile + 16 * p, lane);                                             \
      fa_l[p] = xfrag16<AKC, TS>(al, wm * kWTile + 16 * p, lane);                                             \
      fb_h[p] = xfrag16<BKC, TS>(bh, wn * kWTile + 16 * p, lane);                                             \
      fb_l[p] = xfrag16<BKC, TS>(bl, wn * kWTile + 16 * p, lane);                                             \
    }                                                                                                         \
    _Pragma("unroll") for (int p = 0; p < kP; ++p) _Pragma("unroll") for (int q = 0; q < kP; ++q) {          \
      acc[p][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb_h[q], fa_l[p], acc[p][q], 0, 0, 0);              \
      acc[p][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb_l[q], fa_h[p], acc[p][q], 0, 0, 0);              \
      acc[p][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb_h[q], fa_h[p], acc[p][q], 0, 0, 0);              \
    }                                                                                                         \
  }
// The same products in two halves (A fragment rows [0, kP/2) then [kP/2, kP)) with MID between them.
#define RQ_X3_MMA2(MID)                                                                                       \
  {                                                                                                           \
    bf16x8_t fa_h[kP], fa_l[kP], fb_h[kP], fb_l[kP];                                                          \
    _Pragma("unroll") for (int p = 0; p < kP; ++p) {                                                          \
      fb_h[p] = xfrag16<BKC, TS>(bh, wn * kWTile + 16 * p, lane);                                             \
      fb_l[p] = xfrag16<BKC, TS>(bl, wn * kWTile + 16 * p, lane);                                             \
    }                                                                                                         \
    _Pragma("unroll") for (int h_ = 0; h_ < 2; ++h_) {                                                        \
      _Pragma("unroll") for (int p = h_ * kP / 2; p < (h_ + 1) * kP / 2; ++p) {                               \
        fa_h[p] = xfrag16<AKC, TS>(ah, wm * kWTile + 16 * p, lane);                                           \
        fa_l[p] = xfrag16<AKC, TS>(al, wm * kWTile + 16 * p, lane);                                           \
      }                                                                                                       \
      _Pragma("unroll") for (int p = h_ * kP / 2; p < (h_ + 1) * kP / 2; ++p)                                 \
      _Pragma("unroll") for (int q = 0; q < kP; ++q) {                                                        \
        acc[p][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb_h[q], fa_l[p], acc[p][q], 0, 0, 0);            \
        acc[p][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb_l[q], fa_h[p], acc[p][q], 0, 0, 0);            \
        acc[p][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb_h[q], fa_h[p], acc[p][q], 0, 0, 0);            \
      }                                                                                                       \
      if (h_ == 0) { MID }                                                                                    \
    }                                                                                                         \
  }
#else
#define RQ_X3_MMA                                                                                             \
  _Pragma("unroll") for (int ks = 0; ks < kXK / 16; ++ks) {                                                   \
    bf16x8_t fa_h[2], fa_l[2], fb_h[2], fb_l[2];                                                              \
    _Pragma("unroll") for (int p = 0; p < 2; ++p) {                                                           \
      fa_h[p] = xfrag<AKC>(ah, wm * 64 + 32 * p, ks, lane);                                                   \
      fa_l[p] = xfrag<AKC>(al, wm * 64 + 32 * p, ks, lane);                                                   \
      fb_h[p] = xfrag<BKC>(bh, wn * 64 + 32 * p, ks, lane);                                                   \
      fb_l[p] = xfrag<BKC>(bl, wn * 64 + 32 * p, ks, lane);                                                   \
    }                                                                                                         \
    _Pragma("unroll") for (int p = 0; p < 2; ++p) _Pragma("unroll") for (int q = 0; q < 2; ++q) {            \
      acc[p][q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb_h[q], fa_l[p], acc[p][q], 0, 0, 0);              \
      acc[p][q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb_l[q], fa_h[p], acc[p][q], 0, 0, 0);              \
      acc[p][q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb_h[q], fa_h[p], acc[p][q], 0, 0, 0);              \
    }                                                                                                         \
  }
#endif

// One launch's problem (operands, shape, plan, output, epilogue): the kernel argument of the 128-/64-tile
// kernel and of the paired launch (gemm_x3_pair_kernel) that runs two problems' workgroups in one grid.
struct X3Args {
  const void* A;
  const void* Al;
  int64_t lda;
  const void* B;
  const void* Bl;
  int64_t ldb;
  int M, N;
  int64_t K;
  int tiles_n, tiles, S;
  int64_t chunk;
  int per;
  float* C;
  int64_t ldc;
  X3Epilogue ep;
  int kf;   // 1: K and chunk are multiples of kXK (the unmasked staging path)
};

// LDS bytes of one plane of the TS-tile form (the 64-tile form's compact images: half of every plane)
template <int TS>
constexpr int x3_plane_bytes() { return (TS == 64 && RQ_X3S_COMPACT) ? kXPlane / 2 : kXPlane; }

// TS = output tile (128, or 64 for launches whose 128-tiles cannot fill the chip: the decoder's 1,280
// future-token rows): 4 waves of (TS / 2)^2 outputs, the same k order (so the same result) either way.
// The body of one workgroup `bid` of problem `a` over the LDS block `lds` (8 planes).
template <bool AKC, bool ASP, bool BKC, bool BSP, int EPI, bool DROP, int TS, bool KF>
__device__ __forceinline__ void x3_body_k(const X3Args& a, int bid, char* __restrict__ lds) {
  const void* __restrict__ A = a.A;
  const void* __restrict__ Al = a.Al;
  const void* __restrict__ B = a.B;
  const void* __restrict__ Bl = a.Bl;
  const int64_t lda = a.lda, ldb = a.ldb, K = a.K, chunk = a.chunk, ldc = a.ldc;
  const int M = a.M, N = a.N, tiles_n = a.tiles_n, tiles = a.tiles, S = a.S, per = a.per;
  float* __restrict__ C = a.C;
  X3Epilogue ep = a.ep;
  ep.seed = epoch_seed(ep.seed);
  constexpr int kPl = x3_plane_bytes<TS>();
  const int lw = (bid & 7) * per + (bid >> 3);   // XCD-major: neighbours (same A rows / same k chunk) share an L2
  if (lw >= tiles * S) return;
  const int s = lw / tiles, t = lw % tiles;
  const int m0 = (t / tiles_n) * TS, n0 = (t % tiles_n) * TS;
  static_assert(TS == 128 || (TS == 64 && RQ_X3_MFMA16), "64-row tiles run on the 16x16x32 MFMA");
  constexpr int kWTile = TS / 2, kP = TS / 32;   // per-wave tile, 16-row MFMA tiles per wave side
  const int64_t k_lo = (int64_t)s * chunk;
  const int64_t k_hi = k_lo + chunk < K ? k_lo + chunk : K;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;

#if RQ_X3_MFMA16
  floatx4v acc[kP][kP];
#pragma unroll
  for (int p = 0; p < kP; ++p)
#pragma unroll
    for (int q = 0; q < kP; ++q) acc[p][q] = floatx4v{0.f, 0.f, 0.f, 0.f};
#else
  floatx16 acc[2][2];
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[p][q][r] = 0.f;
#endif

  auto plane = [&](int buf, int op, int hl) { return lds + buf * 4 * kPl + op * 2 * kPl + hl * kPl; };
  const int nst = (int)((k_hi - k_lo + kXK - 1) / kXK);
  // kDepth register stage sets: stage st + kDepth is loaded while stage st is multiplied and
  // stage st + 1 (loaded earlier) is written to the other LDS buffer, so each load has kDepth stages
  // of MFMA work to land in (HBM latency under load is ~2-4k cycles, one 128-tile stage ~1.5k; a
  // 64-tile stage is 4x less MFMA work, so that form keeps 4 stages in flight).
  constexpr int kDepth = TS == 64 ? RQ_X3S_DEPTH : RQ_X3_DEPTH;
  static_assert(kDepth >= 2 && kDepth <= 4, "stage sets");
  XStage<AKC, ASP, TS, KF> sa0, sa1, sa2, sa3;
  XStage<BKC, BSP, TS, KF> sb0, sb1, sb2, sb3;
  sa0.load(A, Al, lda, m0, M, k_lo, k_lo, k_hi, tid);
  sb0.load(B, Bl, ldb, n0, N, k_lo, k_lo, k_hi, tid);
  sa1.load(A, Al, lda, m0, M, k_lo + (int64_t)min(1, nst - 1) * kXK, k_lo, k_hi, tid);
  sb1.load(B, Bl, ldb, n0, N, k_lo + (int64_t)min(1, nst - 1) * kXK, k_lo, k_hi, tid);
  if constexpr (kDepth >= 3) {
    sa2.load(A, Al, lda, m0, M, k_lo + (int64_t)min(2, nst - 1) * kXK, k_lo, k_hi, tid);
    sb2.load(B, Bl, ldb, n0, N, k_lo + (int64_t)min(2, nst - 1) * kXK, k_lo, k_hi, tid);
  }
  if constexpr (kDepth >= 4) {
    sa3.load(A, Al, lda, m0, M, k_lo + (int64_t)min(3, nst - 1) * kXK, k_lo, k_hi, tid);
    sb3.load(B, Bl, ldb, n0, N, k_lo + (int64_t)min(3, nst - 1) * kXK, k_lo, k_hi, tid);
  }
  sa0.store(plane(0, 0, 0), plane(0, 0, 1), tid);
  sb0.store(plane(0, 1, 0), plane(0, 1, 1), tid);
  __syncthreads();

#define RQ_X3_STAGE(ST, LA, LB, SA, SB, ON)                                                                   \
  {                                                                                                           \
    const int st_ = (ST), buf = st_ & 1;                                                                      \
    const bool on_ = (ON);                                                                                    \
    {  /* unconditional (past the end: the last stage again, an L2 hit) so vmcnt counts stay static */       \
      const int64_t kb = k_lo + (int64_t)min(st_ + kDepth, nst - 1) * kXK;                                    \
      LA.load(A, Al, lda, m0, M, kb, k_lo, k_hi, tid);                                                        \
      LB.load(B, Bl, ldb, n0, N, kb, k_lo, k_hi, tid);                                                        \
    }                                                                                                         \
    const char* ah = plane(buf, 0, 0);                                                                        \
    const char* al = plane(buf, 0, 1);                                                                        \
    const char* bh = plane(buf, 1, 0);                                                                        \
    const char* bl = plane(buf, 1, 1);                                                                        \
    RQ_X3_BODY(SA, SB)                                                                                        \
    __syncthreads();                                                                                          \
  }
  // Stage body: the MFMAs on buffer buf and the write of the next stage's registers into buf ^ 1
  // (free since the previous barrier; unconditional: past the last stage it writes a buffer nobody
  // reads, and a conditional store would leave the set's loads possibly pending, so the compiler
  // would wait vmcnt(0) before reloading it). RQ_X3_INTERLEAVE issues the write (its VALU and
  // ds_writes) between the MFMAs instead of after them.
#if RQ_X3_INTERLEAVE == 1
#define RQ_X3_BODY(SA, SB)                                                                                    \
  SA.store(plane(buf ^ 1, 0, 0), plane(buf ^ 1, 0, 1), tid);                                                  \
  SB.store(plane(buf ^ 1, 1, 0), plane(buf ^ 1, 1, 1), tid);                                                  \
  if (on_) RQ_X3_MMA                                                                                          \
  _Pragma("unroll") for (int i_ = 0; i_ < 8; ++i_) {                                                          \
    __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);                                                        \
    __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);                                                        \
    __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);                                                        \
  }
#elif RQ_X3_INTERLEAVE == 2
#define RQ_X3_BODY(SA, SB)                                                                                    \
  if constexpr (TS == 128) {                                                                                  \
    SA.store(plane(buf ^ 1, 0, 0), plane(buf ^ 1, 0, 1), tid);                                                \
    SB.store(plane(buf ^ 1, 1, 0), plane(buf ^ 1, 1, 1), tid);                                                \
    if (on_) RQ_X3_MMA                                                                                        \
    __builtin_amdgcn_sched_group_barrier(0x020, 8, 0);                                                        \
    __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);                                                       \
    _Pragma("unroll") for (int i_ = 0; i_ < 8; ++i_) {                                                        \
      __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);                                                      \
      __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);                                                      \
      __builtin_amdgcn_sched_group_barrier(0x002, 7, 0);                                                      \
    }                                                                                                         \
  } else {                                                                                                    \
    if (on_) RQ_X3_MMA                                                                                        \
    SA.store(plane(buf ^ 1, 0, 0), plane(buf ^ 1, 0, 1), tid);                                                \
    SB.store(plane(buf ^ 1, 1, 0), plane(buf ^ 1, 1, 1), tid);                                                \
  }
#elif RQ_X3_INTERLEAVE == 3   // A's staging store before the MFMAs, B's after
#define RQ_X3_BODY(SA, SB)                                                                                    \
  SA.store(plane(buf ^ 1, 0, 0), plane(buf ^ 1, 0, 1), tid);                                                  \
  if (on_) RQ_X3_MMA                                                                                          \
  SB.store(plane(buf ^ 1, 1, 0), plane(buf ^ 1, 1, 1), tid);
#elif RQ_X3_INTERLEAVE == 4   // the MFMAs in two halves, A's staging store between them, B's after
#define RQ_X3_BODY(SA, SB)                                                                                    \
  static_assert(RQ_X3_PEEL, "every slot multiplies");                                                         \
  RQ_X3_MMA2(SA.store(plane(buf ^ 1, 0, 0), plane(buf ^ 1, 0, 1), tid);)                                      \
  SB.store(plane(buf ^ 1, 1, 0), plane(buf ^ 1, 1, 1), tid);
#else
#define RQ_X3_BODY(SA, SB)                                                                                    \
  if (on_) {                                                                                                  \
    RQ_X3_PRIO(1)                                                                                             \
    RQ_X3_MMA                                                                                                 \
    RQ_X3_PRIO(0)                                                                                             \
  }                                                                                                           \
  SA.store(plane(buf ^ 1, 0, 0), plane(buf ^ 1, 0, 1), tid);                                                  \
  SB.store(plane(buf ^ 1, 1, 0), plane(buf ^ 1, 1, 1), tid);
#endif
  // set j % kDepth holds stage j: after multiplying stage st its set is reloaded with st + kDepth.
  // Every stage slot of an iteration issues its loads, stores and barrier; only the MFMAs of slots
  // past the last stage are skipped (a skipped slot's loads would leave the counts path-dependent).
  if constexpr (kDepth == 4) {
    for (int st = 0; st < nst; st += 4) {
      RQ_X3_STAGE(st, sa0, sb0, sa1, sb1, true)
      RQ_X3_STAGE(st + 1, sa1, sb1, sa2, sb2, st + 1 < nst)
      RQ_X3_STAGE(st + 2, sa2, sb2, sa3, sb3, st + 2 < nst)
      RQ_X3_STAGE(st + 3, sa3, sb3, sa0, sb0, st + 3 < nst)
    }
  } else if constexpr (kDepth == 3) {
#if RQ_X3_PEEL
    int st = 0;
    for (; st + 2 < nst; st += 3) {
      RQ_X3_STAGE(st, sa0, sb0, sa1, sb1, true)
      RQ_X3_STAGE(st + 1, sa1, sb1, sa2, sb2, true)
      RQ_X3_STAGE(st + 2, sa2, sb2, sa0, sb0, true)
    }
    if (st < nst) RQ_X3_STAGE(st, sa0, sb0, sa1, sb1, true)
    if (st + 1 < nst) RQ_X3_STAGE(st + 1, sa1, sb1, sa2, sb2, true)
#else
    for (int st = 0; st < nst; st += 3) {
      RQ_X3_STAGE(st, sa0, sb0, sa1, sb1, true)
      RQ_X3_STAGE(st + 1, sa1, sb1, sa2, sb2, st + 1 < nst)
      RQ_X3_STAGE(st + 2, sa2, sb2, sa0, sb0, st + 2 < nst)
    }
#endif
  } else {
#if RQ_X3_PEEL
    int st = 0;
    for (; st + 1 < nst; st += 2) {
      RQ_X3_STAGE(st, sa0, sb0, sa1, sb1, true)
      RQ_X3_STAGE(st + 1, sa1, sb1, sa0, sb0, true)
    }
    if (st < nst) RQ_X3_STAGE(st, sa0, sb0, sa1, sb1, true)
#else
    for (int st = 0; st < nst; st += 2) {
      RQ_X3_STAGE(st, sa0, sb0, sa1, sb1, true)
      RQ_X3_STAGE(st + 1, sa1, sb1, sa0, sb0, st + 1 < nst)
    }
#endif
  }
#undef RQ_X3_STAGE
#undef RQ_X3_BODY
#undef RQ_X3_MMA
#undef RQ_X3_MMA2

  // Each lane stores C[m][n .. n + 3] quads: 16-B fp32 / 8-B bf16 stores (N % 4 == 0).
  float* Cs = C + (int64_t)s * M * N;   // split-K partial slab (S > 1: ldc == N)
#if RQ_X3_MFMA16
  // 16x16 C/D map of D = B A^T: column (lane & 15) = m, row 4 (lane >> 4) + j = n (j = register).
  constexpr int kPM = kP, kPN = kP, kG = 1;
#else
  // 32x32 C/D map: column (lane & 31) = m, row (r & 3) + 8 (r >> 2) + 4 (lane >> 5) = n: register
  // quad g holds n = 8 g + 4 (lane >> 5) + 0..3.
  constexpr int kPM = 2, kPN = 2, kG = 4;
#endif
  auto quad_m = [&](int p) {
#if RQ_X3_MFMA16
    return m0 + wm * kWTile + 16 * p + (lane & 15);
#else
    return m0 + wm * 64 + 32 * p + (lane & 31);
#endif
  };
  auto quad_n = [&](int q, int g) {
#if RQ_X3_MFMA16
    return n0 + wn * kWTile + 16 * q + 4 * (lane >> 4);
#else
    return n0 + wn * 64 + 32 * q + 8 * g + 4 * (lane >> 5);
#endif
  };
  // the SiLU' epilogue's Z quads for every quad first: one round trip, not one per quad (the residual add
  // keeps its per-quad reads: preloaded it measured 2 us slower per decoder launch, profiles/r06/epi_z)
  constexpr bool kZ = EPI == kEpiSiluBwd;
  float4 zin[kPM][kPN][kG];
#pragma unroll
  for (int p = 0; p < kPM; ++p)
#pragma unroll
    for (int q = 0; q < kPN; ++q)
#pragma unroll
      for (int g = 0; g < kG; ++g) {
        const int m = quad_m(p), n = quad_n(q, g);
        zin[p][q][g] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (kZ && m < M && n < N) zin[p][q][g] = x3_epi_in<EPI>(m, n, Cs, ldc, ep);
      }
#pragma unroll
  for (int p = 0; p < kPM; ++p) {
    const int m = quad_m(p);
    if (m < M) {
#pragma unroll
      for (int q = 0; q < kPN; ++q)
#pragma unroll
        for (int g = 0; g < kG; ++g) {
          const int n = quad_n(q, g);
#if RQ_X3_MFMA16
          const float4 v = make_float4(acc[p][q][0], acc[p][q][1], acc[p][q][2], acc[p][q][3]);
#else
          const float4 v = make_float4(acc[p][q][4 * g], acc[p][q][4 * g + 1], acc[p][q][4 * g + 2], acc[p][q][4 * g + 3]);
#endif
          if (n >= N) continue;
          if constexpr (kZ) x3_epi4z<EPI, DROP>(v, zin[p][q][g], m, n, N, C, Cs, ldc, ep);
          else x3_epi4<EPI, DROP>(v, m, n, N, C, Cs, ldc, ep);
        }
    }
  }
}

// The body with the staging path picked once per workgroup (uniform): unmasked when every stage is full.
template <bool AKC, bool ASP, bool BKC, bool BSP, int EPI, bool DROP, int TS>
__device__ __forceinline__ void x3_body(const X3Args& a, int bid, char* __restrict__ lds) {
  if (a.kf)
    x3_body_k<AKC, ASP, BKC, BSP, EPI, DROP, TS, true>(a, bid, lds);
  else
    x3_body_k<AKC, ASP, BKC, BSP, EPI, DROP, TS, false>(a, bid, lds);
}

template <bool AKC, bool ASP, bool BKC, bool BSP, int EPI, bool DROP = false, int TS = 128>
__global__ void __launch_bounds__(256, TS == 64 ? kXWG64 : kXWG) gemm_bf16x3_kernel(X3Args a) {
  __shared__ __attribute__((aligned(16))) char lds[8 * x3_plane_bytes<TS>()];
  x3_body<AKC, ASP, BKC, BSP, EPI, DROP, TS>(a, blockIdx.x, lds);
}

// Two problems in ONE launch: workgroups [0, n1) run problem 1, the rest problem 2 (each with its own
// XCD-major tile order and plan). The backward's data-gradient and weight-gradient GEMMs of a Linear are
// independent; one launch instead of two saves a launch and lets the pair fill the chip together (the
// decoder's 1,280-row launches fill 160..480 of 1,024 slots each; the 11,332-row data gradients 356 of 512).
// P1 / P2: x3_body instantiations (X3Body<form..., TS>); both the same tile size.
template <bool AKC, bool ASP, bool BKC, bool BSP, int EPI, bool DROP, int TS>
struct X3Body {
  static constexpr int kTS = TS;
  __device__ __forceinline__ static void run(const X3Args& a, int bid, char* lds) {
    x3_body<AKC, ASP, BKC, BSP, EPI, DROP, TS>(a, bid, lds);
  }
};

template <class P1, class P2>
__global__ void __launch_bounds__(256, P1::kTS == 64 ? kXWG64 : kXWG) gemm_x3_pair_kernel(X3Args a1, X3Args a2, int n1) {
  static_assert(P1::kTS == P2::kTS, "paired problems share the tile size");
  __shared__ __attribute__((aligned(16))) char lds[8 * x3_plane_bytes<P1::kTS>()];
  const int bid = blockIdx.x;
  if (bid < n1)
    P1::run(a1, bid, lds);
  else
    P2::run(a2, bid - n1, lds);
}

// ---------------------------------------------------------------------------------------------
// Wide split-bf16 GEMM ("x3w"): 256 x 256 output tile per workgroup, 8 waves (2 along m x 4
// along n, 128 x 64 outputs each), both operands already split into bf16 planes. The operand tile
// of one 32-deep k step is four "halves" (A rows 0-127 / 128-255, B rows 0-127 / 128-255), each a
// hi and a lo plane of 8 KiB: a row image for a k-contiguous operand (64-B rows, 16-B chunk c of
// row r at c ^ ((r >> 2) & 2): conflict-free for the 16x16x32 fragment's ds_read_b128 lane
// groups), else the column image of gemm_bf16x3_kernel read by ds_read_b64_tr_b16. A (the
// streamed activation: HBM / Infinity-Cache misses) has THREE k-step slots, B (the weights, L2
// hits) two: 3 x 32 + 2 x 32 KiB = 160 KiB, the whole LDS, one workgroup per CU.
//
// Staging is LDS-DMA (global_load_lds_dwordx4: no VGPR round trip; the images' XOR swizzles go on
// the per-lane SOURCE address, the LDS side stays lane-linear: wave w fills bytes [1 KiB w,
// 1 KiB (w + 1)) of every half-plane). A k step is four phases, one per C quadrant of the wave
// (A half h x B half g), in the order (0,0) (0,1) (1,1) (1,0); reads: A0 + B0 (phase 0), B1 (1),
// A1 (2), none (3: B0 kept in registers). Phase p of step t issues, 2 DMA instructions per wave
// each, B0 (t + 1), B1 (t + 1), A0 (t + 2), A1 (t + 2): A lands 5-7 phases after issue, B in 4,
// and since vmcnt retires in issue order, B issued after A never waits on A's misses early. The
// only waits are a counted vmcnt(6) (three halves left in flight) at the end of phases 3 and 0;
// phase 2's A1 was retired by phase 0's. Never vmcnt(0) inside the loop. The two wave groups
// (waves 0-3 / 4-7: one of each per SIMD) run staggered by one barrier with two barriers per
// phase, so on every SIMD one wave issues its LDS reads and DMAs while the other runs its 24
// MFMAs. Ordering rules:
//  * RAW: data read in phase f is retired (each wave's own vmcnt) before the barrier that ends
//    the interval BEFORE either group's read interval of phase f: group 0 waits at the end of its
//    MFMA interval of phase f - 1, group 1 (one interval behind) at the end of its read interval;
//  * WAR: a DMA overwrites a slot last read >= 3 phases earlier (A: step t - 1's copy; B: step
//    t - 1's), those reads retired by lgkmcnt(0) before their phase's MFMAs.
// Per k step and wave: 24 ds_read_b128 / tr reads, 8 DMA instructions, 96 MFMAs (16x16x32 bf16).
// The accumulation order over k equals gemm_bf16x3_kernel's (same 32-deep steps, same product
// order), so for the same split the two kernels agree bitwise.
// ---------------------------------------------------------------------------------------------
#ifndef RQ_X3W_STAGGER
#define RQ_X3W_STAGGER 1   // 0: both wave groups in lock-step (A/B switch)
#endif
#ifndef RQ_X3W_EPI_LDS
#define RQ_X3W_EPI_LDS 1   // epilogue through LDS in whole rows (0: straight from the accumulators)
#endif
#ifndef RQ_X3W_DIAG
#define RQ_X3W_DIAG 0      // diagnostic builds only: 1 = no operand loads, 2 = no MFMAs, 3 = no epilogue, 4 = B re-read
                           // from its first k step (cache-resident), 5 = A likewise, 6 = k-contiguous operands DMA whole
                           // 128-B lines (8 rows per KiB, each line once per k-step pair), 7 = phases 1 / 2 skip
                           // their fragment reads after the first k step (half the LDS reads) (wrong results)
#endif
#ifndef RQ_X3W_BUFLDS
#define RQ_X3W_BUFLDS 1    // operand DMA as buffer_load ... lds (SGPR descriptor rebased at the workgroup's first
                           // row / k chunk + 32-bit byte offset): 1-2.5 % faster than global_load_lds with 64-bit
                           // per-lane addresses (profiles/r06/gemm_diag); 0 = global_load_lds (A/B switch)
#endif
#ifndef RQ_X3W_NT
#define RQ_X3W_NT 1        // the wide kernel's epilogue stores non-temporal (0: default policy; A/B)
#endif
#ifndef RQ_X3W_PRIO
#define RQ_X3W_PRIO 1      // s_setprio(1) around each MFMA cluster (keeps hipcc from moving it)
#endif

constexpr int kWT2 = 256;          // output tile (m and n)
constexpr int kWH = 8192;          // one half-plane: 128 rows x 32 k bf16
constexpr int kWStep = 4 * kWH;    // one operand's k step: 2 halves x 2 planes
constexpr int kWB0 = 3 * kWStep;   // B's slots follow A's three
constexpr int kWLds = 5 * kWStep;  // 160 KiB

__device__ __forceinline__ void glds16(const uint16_t* src, char* lds_dst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_dst, 16, 0, 0);
}

__device__ __forceinline__ int wrow_swz(int r) { return (r >> 2) & 2; }

// Element offset (from the k step's base) of the 16 bytes lane `lane` of wave `wave` DMAs into its
// slot of a half-plane image whose first row (m or n) is r0.
template <bool KC>
__device__ __forceinline__ int64_t x3w_src(int64_t ld, int r0, int R, int wave, int lane) {
  if constexpr (KC) {   // row image: 16 rows x 4 chunks per 1 KiB; position c holds k-chunk c ^ swz
    if (RQ_X3W_DIAG == 6) {   // diagnostic: 8 rows x one whole 128-B line per 1 KiB (wrong results)
      const int row = 8 * wave + (lane >> 3);
      return (int64_t)min(r0 + row, R - 1) * ld + 8 * (lane & 7);
    }
    const int row = 16 * wave + (lane >> 2);
    const int kc = (lane & 3) ^ wrow_swz(row);
    return (int64_t)min(r0 + row, R - 1) * ld + 8 * kc;
  } else {              // column image: 4 k-rows x 16 chunks per 1 KiB; position c holds m-chunk c ^ col_swz
    const int kr = 4 * wave + (lane >> 4);
    const int mc = (lane & 15) ^ col_swz(kr);
    return (int64_t)kr * ld + min(r0 + 8 * mc, R - 8);
  }
}

// 16x16x32 operand fragment of a wide-kernel half-plane (row rb + lane % 16, k = 8 (lane / 16) + 0..7).
template <bool KC>
__device__ __forceinline__ bf16x8_t wfrag16(const char* plane, int rb, int lane) {
  if constexpr (KC) {
    const int rr = rb + (lane & 15), c = lane >> 4;
    return *reinterpret_cast<const bf16x8_t*>(plane + rr * 64 + ((c ^ wrow_swz(rr)) << 4));
  } else {
    return xfrag16<false>(plane, rb, lane);
  }
}

#define RQ_W_BAR() __builtin_amdgcn_s_barrier()
#define RQ_W_VM6() asm volatile("s_waitcnt vmcnt(6)" ::: "memory")

#define RQ_W_LGKM0() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")

template <bool AKC, bool BKC, int EPI, bool DROP>
__global__ void __launch_bounds__(512, 1)
gemm_x3w_kernel(const uint16_t* __restrict__ Ah, const uint16_t* __restrict__ Al, int64_t lda,
                const uint16_t* __restrict__ Bh, const uint16_t* __restrict__ Bl, int64_t ldb, int M, int N, int64_t K,
                int tiles_n, int tiles, int64_t chunk, float* __restrict__ C, int64_t ldc, X3Epilogue ep) {
  ep.seed = epoch_seed(ep.seed);
  __shared__ __attribute__((aligned(16))) char lds[kWLds];   // the kernel's only LDS object (DMA waits)
  // bijective XCD-major remap: consecutive work items (same A rows, same k chunk) share an L2
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xq = nwg >> 3, xr = nwg & 7, xcd = bid & 7;
  const int lw = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + (bid >> 3);
  const int s = lw / tiles, t = lw - s * tiles;
  const int m0 = (t / tiles_n) * kWT2, n0 = (t % tiles_n) * kWT2;
  const int64_t k_lo = (int64_t)s * chunk;
  const int64_t k_hi = k_lo + chunk < K ? k_lo + chunk : K;
  const int nk = (int)((k_hi - k_lo) >> 5);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const bool g1 = RQ_X3W_STAGGER && wr != 0;

  const int64_t da = AKC ? 32 : 32 * lda, db = BKC ? 32 : 32 * ldb;
  const int64_t ka = AKC ? k_lo : k_lo * lda, kb = BKC ? k_lo : k_lo * ldb;
  const int64_t oa0 = ka + x3w_src<AKC>(lda, m0, M, wave, lane), oa1 = ka + x3w_src<AKC>(lda, m0 + 128, M, wave, lane);
  const int64_t ob0 = kb + x3w_src<BKC>(ldb, n0, N, wave, lane), ob1 = kb + x3w_src<BKC>(ldb, n0 + 128, N, wave, lane);
  char* const wl = lds + 1024 * wave;
  // A half h of k step `step` into A slot `slot`; B half g of step `step` into B parity step & 1.
  // Steps past the end are clamped (the last step again, into a slot nobody reads), so every wave
  // issues the same DMA count in every phase and the vmcnt counts stay static.
#if RQ_X3W_BUFLDS
  // descriptors based at the workgroup's first A / B row (k-contiguous) or first k row (m/n-contiguous): every
  // offset below is then < x3w_span() elements, which x3w_choose keeps under 2^30 (32-bit byte offsets)
  const int64_t abase = AKC ? (int64_t)m0 * lda : k_lo * lda, bbase = BKC ? (int64_t)n0 * ldb : k_lo * ldb;
  const __amdgpu_buffer_rsrc_t rah = __builtin_amdgcn_make_buffer_rsrc((void*)(Ah + abase), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t ral = __builtin_amdgcn_make_buffer_rsrc((void*)(Al + abase), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rbh = __builtin_amdgcn_make_buffer_rsrc((void*)(Bh + bbase), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rbl = __builtin_amdgcn_make_buffer_rsrc((void*)(Bl + bbase), (short)0, 0x7fffffff, 0x00020000);
  auto bdma = [](__amdgpu_buffer_rsrc_t r, int64_t rel, char* dst) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)dst, 16, (int)(rel * 2), 0, 0, 0);
  };
#endif
  auto issue_a = [&](int h, int step, int slot) {
    if (RQ_X3W_DIAG == 1) return;   // diagnostic build: no operand loads (wrong results)
    const int sa = step < nk ? step : nk - 1;
    const int64_t o = (h == 0 ? oa0 : oa1) + (RQ_X3W_DIAG == 5 ? 0 : (RQ_X3W_DIAG == 6 && AKC ? (int64_t)(sa & ~1) * da + (int64_t)(sa & 1) * 64 * lda : (int64_t)sa * da));
    char* dst = wl + slot * kWStep + h * 2 * kWH;
#if RQ_X3W_BUFLDS
    bdma(rah, o - abase, dst);
    bdma(ral, o - abase, dst + kWH);
#else
    glds16(Ah + o, dst);
    glds16(Al + o, dst + kWH);
#endif
  };
  auto issue_b = [&](int g, int step) {
    if (RQ_X3W_DIAG == 1) return;
    const int sb = step < nk ? step : nk - 1;
    const int64_t o = (g == 0 ? ob0 : ob1) + (RQ_X3W_DIAG == 4 ? 0 : (RQ_X3W_DIAG == 6 && BKC ? (int64_t)(sb & ~1) * db + (int64_t)(sb & 1) * 64 * ldb : (int64_t)sb * db));
    char* dst = wl + kWB0 + (step & 1) * kWStep + g * 2 * kWH;
#if RQ_X3W_BUFLDS
    bdma(rbh, o - bbase, dst);
    bdma(rbl, o - bbase, dst + kWH);
#else
    glds16(Bh + o, dst);
    glds16(Bl + o, dst + kWH);
#endif
  };
  auto aplane = [&](int slot, int h, int pl) -> const char* { return lds + slot * kWStep + (h * 2 + pl) * kWH; };
  auto bplane = [&](int par, int g, int pl) -> const char* {
    return lds + kWB0 + par * kWStep + (g * 2 + pl) * kWH;
  };

  floatx4v acc[2][2][4][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[h][g][i][j] = floatx4v{0.f, 0.f, 0.f, 0.f};
  bf16x8_t fah[4], fal[4], fb0h[2], fb0l[2], fb1h[2], fb1l[2];

#define RQ_W_READ_A(SLOT, H)                                                                   \
  _Pragma("unroll") for (int i = 0; i < 4; ++i) {                                              \
    fah[i] = wfrag16<AKC>(aplane(SLOT, H, 0), wr * 64 + 16 * i, lane);                         \
    fal[i] = wfrag16<AKC>(aplane(SLOT, H, 1), wr * 64 + 16 * i, lane);                         \
  }
#define RQ_W_READ_B(PAR, G, BH, BL)                                                            \
  _Pragma("unroll") for (int j = 0; j < 2; ++j) {                                              \
    BH[j] = wfrag16<BKC>(bplane(PAR, G, 0), wc * 32 + 16 * j, lane);                           \
    BL[j] = wfrag16<BKC>(bplane(PAR, G, 1), wc * 32 + 16 * j, lane);                           \
  }
#define RQ_W_MMA(H, G, BH, BL)                                                                 \
  if (RQ_X3W_DIAG != 2) {                                                                      \
  if (RQ_X3W_PRIO) __builtin_amdgcn_s_setprio(1);                                              \
  _Pragma("unroll") for (int i = 0; i < 4; ++i) _Pragma("unroll") for (int j = 0; j < 2; ++j) { \
    floatx4v& c_ = acc[H][G][i][j];                                                            \
    c_ = __builtin_amdgcn_mfma_f32_16x16x32_bf16(BH[j], fal[i], c_, 0, 0, 0);                  \
    c_ = __builtin_amdgcn_mfma_f32_16x16x32_bf16(BL[j], fah[i], c_, 0, 0, 0);                  \
    c_ = __builtin_amdgcn_mfma_f32_16x16x32_bf16(BH[j], fah[i], c_, 0, 0, 0);                  \
  }                                                                                            \
  if (RQ_X3W_PRIO) __builtin_amdgcn_s_setprio(0);                                              \
  }

  // prologue, in the steady state's issue order (A of steps 0 and 1, B of step 0); phase 0 of
  // step 0 needs A0 (0) and B0 (0): B1 (0), A0 (1), A1 (1) may stay in flight
  issue_a(0, 0, 0);
  issue_a(1, 0, 0);
  issue_b(0, 0);
  issue_b(1, 0);
  issue_a(0, 1, 1);
  issue_a(1, 1, 1);
  RQ_W_VM6();
  RQ_W_BAR();
  if (g1) RQ_W_BAR();   // group 1 runs one barrier behind
  int slot = 0;         // A slot of step st (st % 3); step st + 2 goes to (st + 2) % 3
  for (int st = 0; st < nk; ++st) {
    const int par = st & 1, slot2 = slot == 0 ? 2 : slot - 1;
    // phase 0: quadrant (A0, B0)
    RQ_W_READ_A(slot, 0)
    RQ_W_READ_B(par, 0, fb0h, fb0l)
    issue_b(0, st + 1);
    if (g1) RQ_W_VM6();   // B1 (and A1) of this step, for phases 1 and 2
    RQ_W_BAR();
    RQ_W_LGKM0();
    RQ_W_MMA(0, 0, fb0h, fb0l)
    if (!g1) RQ_W_VM6();
    RQ_W_BAR();
    // phase 1: (A0, B1)
    if (RQ_X3W_DIAG != 7 || st == 0) RQ_W_READ_B(par, 1, fb1h, fb1l)
    issue_b(1, st + 1);
    RQ_W_BAR();
    RQ_W_LGKM0();
    RQ_W_MMA(0, 1, fb1h, fb1l)
    RQ_W_BAR();
    // phase 2: (A1, B1)
    if (RQ_X3W_DIAG != 7 || st == 0) RQ_W_READ_A(slot, 1)
    issue_a(0, st + 2, slot2);
    RQ_W_BAR();
    RQ_W_LGKM0();
    RQ_W_MMA(1, 1, fb1h, fb1l)
    RQ_W_BAR();
    // phase 3: (A1, B0) from registers
    issue_a(1, st + 2, slot2);
    if (g1) RQ_W_VM6();   // A0 and B0 of the next step, for its phase 0
    RQ_W_BAR();
    RQ_W_MMA(1, 0, fb0h, fb0l)
    if (!g1) RQ_W_VM6();
    RQ_W_BAR();
    slot = slot == 2 ? 0 : slot + 1;
  }
#undef RQ_W_READ_A
#undef RQ_W_READ_B
#undef RQ_W_MMA
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (!g1) RQ_W_BAR();   // balance group 1's extra barrier

  float* Cs = C + (int64_t)s * M * N;   // split-K partial slab (S > 1: ldc == N)
  if (RQ_X3W_DIAG == 3) {   // diagnostic build: no epilogue (the accumulators must look used)
    float keep = 0.f;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) keep += acc[h][g][i][j][0] + acc[h][g][i][j][3];
    if (keep == 12345.678f && tid == 0) C[0] = keep;
    return;
  }
#if RQ_X3W_EPI_LDS
  // Epilogue through LDS, one 128-row half of the tile at a time (128 KiB): the waves scatter their
  // accumulator quads into a [128][256] fp32 image (16-B chunk c of row r at c ^ (r & 15): the
  // 16 rows of a quad store and the 16 chunks of a row read hit distinct bank groups), then each
  // wave runs the epilogue on 16 whole rows, one 1 KiB row segment per instruction (coalesced
  // stores / Z reads instead of 64-B pieces of 16 rows).
  __syncthreads();   // every wave's DMAs retired (vmcnt(0) above) and its reads done: LDS is free
  float* const img = reinterpret_cast<float*>(lds);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int r = wr * 64 + 16 * i + (lane & 15);
          const int c = 32 * g + 8 * wc + 4 * j + (lane >> 4);
          *reinterpret_cast<floatx4v*>(img + r * 256 + 4 * (c ^ (r & 15))) = acc[h][g][i][j];
        }
    const int n = n0 + 4 * lane;
    if constexpr (EPI == kEpiSiluBwd) {
      // the 16 rows' Z quads in flight together, in the registers this half's accumulators just left
      // (x3_epi_in: one round trip instead of one per row)
      float4 zin[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int m = m0 + 128 * h + wave * 16 + q;
        zin[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (m < M && n < N) zin[q] = x3_epi_in<EPI>(m, n, Cs, ldc, ep);
      }
      __syncthreads();
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int r = wave * 16 + q, m = m0 + 128 * h + r;
        const floatx4v a = *reinterpret_cast<const floatx4v*>(img + r * 256 + 4 * (lane ^ (r & 15)));
        if (m < M && n < N)
          x3_epi4z<EPI, DROP, RQ_X3W_NT>(make_float4(a[0], a[1], a[2], a[3]), zin[q], m, n, N, C, Cs, ldc, ep);
      }
    } else {   // store-only epilogues (the accumulating store's C read stays per row: unsplit wide calls only)
      __syncthreads();
#pragma unroll 4
      for (int q = 0; q < 16; ++q) {
        const int r = wave * 16 + q, m = m0 + 128 * h + r;
        const floatx4v a = *reinterpret_cast<const floatx4v*>(img + r * 256 + 4 * (lane ^ (r & 15)));
        if (m < M && n < N) x3_epi4<EPI, DROP, RQ_X3W_NT>(make_float4(a[0], a[1], a[2], a[3]), m, n, N, C, Cs, ldc, ep);
      }
    }
    __syncthreads();
  }
#else
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + 128 * h + wr * 64 + 16 * i + (lane & 15);
      if (m >= M) continue;
#pragma unroll
      for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int n = n0 + 128 * g + wc * 32 + 16 * j + 4 * (lane >> 4);
          if (n >= N) continue;
          const floatx4v a = acc[h][g][i][j];
          x3_epi4<EPI, DROP>(make_float4(a[0], a[1], a[2], a[3]), m, n, N, C, Cs, ldc, ep);
        }
    }
#endif
}
#undef RQ_W_BAR
#undef RQ_W_VM6
#undef RQ_W_LGKM0

// Split-K slab reduction with the GEMM's epilogue: element j of the (M, N) output (ldc == N) is the
// fixed-order sum over s of P[s][j] (wave w sums s = w, w + 4, ...; the four wave partials are added
// in wave order: deterministic, no atomics), then (ACC) plus the current C[j], then the epilogue of
// x3_epi4 at (m, n) = (j / N, j % N). Lets every epilogue — SiLU fwd / bwd with dropout, residual
// add, accumulation into an existing gradient — use split-K when the output tiles cannot fill the
// chip (the decoder's 1,280 future-token rows: 40 tiles of 128 x 128).
#ifndef RQ_SLAB_THREAD
#define RQ_SLAB_THREAD 1   // 0: four waves over s per float4 column combined through LDS (the round-4 form)
#endif
constexpr int kRedColsPerWg = RQ_SLAB_THREAD ? 256 : 64;   // float4 columns per workgroup (layout 0)

template <int EPI, bool DROP, bool ACC>
__global__ void __launch_bounds__(256) x3_reduce_kernel(const float* __restrict__ P, int S, int64_t n, int N,
                                                        float* __restrict__ C, X3Epilogue ep) {
  ep.seed = epoch_seed(ep.seed);
#if RQ_SLAB_THREAD   // one thread per float4 column, the same order (slab_sum_w4)
  {
    const int64_t j = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (j >= n) return;
    float4 r = slab_sum_w4(P, S, n, j);
    if constexpr (ACC) {
      const float4 c = *reinterpret_cast<const float4*>(C + j);
      r = make_float4(c.x + r.x, c.y + r.y, c.z + r.z, c.w + r.w);
    }
    x3_epi4<EPI, DROP>(r, (int)(j / N), (int)(j % N), N, C, C, N, ep);
    return;
  }
#endif
  __shared__ float4 part[4][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t j = ((int64_t)blockIdx.x * 64 + lane) * 4;
  const bool ok = j < n;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (ok) a = strided_slab_sum(P, S, n, j, wave, 4);
  part[wave][lane] = a;
  __syncthreads();
  if (wave == 0 && ok) {
    float4 r = part[0][lane];
#pragma unroll
    for (int w = 1; w < 4; ++w) {
      const float4 v = part[w][lane];
      r.x += v.x; r.y += v.y; r.z += v.z; r.w += v.w;
    }
    if constexpr (ACC) {
      const float4 c = *reinterpret_cast<const float4*>(C + j);
      r = make_float4(c.x + r.x, c.y + r.y, c.z + r.z, c.w + r.w);
    }
    x3_epi4<EPI, DROP>(r, (int)(j / N), (int)(j % N), N, C, C, N, ep);
  }
}

// Elementwise split (weights once per step, a large chain input once per step). HBM-bound: 4 B
// read + 2 x 2 B written per element. VEC: float4 loads and 8-B plane stores, 2 float4 in flight
// per thread per iteration (n % 4 == 0, 16-B aligned x, 8-B aligned planes); else scalar.
template <bool VEC>
__global__ void __launch_bounds__(256) split_bf16x3_kernel(const float* __restrict__ x, int64_t n,
                                                           uint16_t* __restrict__ hi, uint16_t* __restrict__ lo) {
  if constexpr (VEC) {
    const int64_t n4 = n >> 2, stride = (int64_t)gridDim.x * 256;
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + stride < n4; i += 2 * stride) {
      const float4 a = reinterpret_cast<const float4*>(x)[i];
      const float4 b = reinterpret_cast<const float4*>(x)[i + stride];
      split_store4(a, hi + 4 * i, lo + 4 * i);
      split_store4(b, hi + 4 * (i + stride), lo + 4 * (i + stride));
    }
    if (i < n4) split_store4(reinterpret_cast<const float4*>(x)[i], hi + 4 * i, lo + 4 * i);
  } else {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
      split_store1(x[i], hi + i, lo + i);
  }
}

// Several tensors at once (all weights of an MLP chain: one launch instead of one per weight).
constexpr int kSplitMax = 48;   // a decoder's every GEMM weight in one launch (kernel arguments ~1.6 KB)
constexpr int kSplitPer = 4;    // units (float4 / scalars) per thread: one workgroup = 1,024 units of ONE tensor
struct SplitMulti {
  const float* x[kSplitMax];
  uint16_t* hi[kSplitMax];
  uint16_t* lo[kSplitMax];
  int64_t n[kSplitMax];           // units per tensor
  int blk0[kSplitMax + 1];        // prefix sums of the workgroups per tensor
  int count;
};

// VEC: every tensor's element count % 4 == 0 and its pointers aligned (16 B x, 8 B planes): float4 units
// with two 8-B plane stores each; else scalar units. Each workgroup owns 1,024 consecutive units of one
// tensor, found by a uniform scan of blk0 (scalar kernel-argument loads: the per-thread binary search it
// replaces indexed the argument block per lane, one dependent search per float4 — 2.6 TB/s on the
// decoder's weights), and keeps its thread's 4 loads in flight.
template <bool VEC>
__global__ void __launch_bounds__(256) split_bf16x3_multi_kernel(SplitMulti sm) {
  const int b = blockIdx.x;
  int t = 0;
  while (t + 1 < sm.count && b >= sm.blk0[t + 1]) ++t;
  const int64_t n = sm.n[t];
  const int64_t j0 = (int64_t)(b - sm.blk0[t]) * (256 * kSplitPer) + threadIdx.x;
  const float* __restrict__ x = sm.x[t];
  uint16_t* __restrict__ hi = sm.hi[t];
  uint16_t* __restrict__ lo = sm.lo[t];
  if constexpr (VEC) {
    float4 v[kSplitPer];
#pragma unroll
    for (int u = 0; u < kSplitPer; ++u) {
      const int64_t j = j0 + 256 * u;
      if (j < n) v[u] = reinterpret_cast<const float4*>(x)[j];
    }
#pragma unroll
    for (int u = 0; u < kSplitPer; ++u) {
      const int64_t j = j0 + 256 * u;
      if (j < n) split_store4(v[u], hi + 4 * j, lo + 4 * j);
    }
  } else {
#pragma unroll
    for (int u = 0; u < kSplitPer; ++u) {
      const int64_t j = j0 + 256 * u;
      if (j < n) split_store1(x[j], hi + j, lo + j);
    }
  }
}

struct X3Plan {
  int tiles_n, tiles, S, per;
  int64_t chunk;
  int ts;   // output tile of the 128-tile kernel family: 128 or 64 (the wide kernel: 256)
};

static int x3_slots() { return resident_slots() / 2 * kXWG; }

#ifndef RQ_X3_SLAB_MB
#define RQ_X3_SLAB_MB 64   // split-K: slab bytes (S x M x N fp32) allowed beyond RQ_X3_MAX_SPLIT slabs
#endif
// Split-K count cap: RQ_X3_MAX_SPLIT slabs, or more while the slabs stay within RQ_X3_SLAB_MB — the
// small weight grads (e.g. 128 x 64 over 65,536 rows: one output tile) need hundreds of k chunks to
// cover the chip, and their slabs are tiny.
static int64_t x3_split_cap(int64_t M, int64_t N) {
  const int64_t by_bytes = ((int64_t)RQ_X3_SLAB_MB << 20) / (4 * M * N);
  return by_bytes > RQ_X3_MAX_SPLIT ? by_bytes : RQ_X3_MAX_SPLIT;
}

// The 64-tile form's compact LDS (32 KiB) lets 4 workgroups share a CU. A launch that fits in 2 per CU
// gets 32 KiB of padding LDS instead (dynamic, unused), so the dispatcher spreads it over every CU rather
// than packing them 4 per CU onto fewer CUs (measured: 1280 x 1536 x 512, 480 workgroups: 14.5 us spread,
// 24.8 us packed; 26,880 x 384 x 1152, 2,520 workgroups: 122.6 -> 109.1 us at 4 per CU).
static int x3s_resident(int64_t wgs) {
  return RQ_X3S_COMPACT && wgs > (int64_t)resident_slots() ? kXWG64 : kXWG;
}
template <typename P>
static unsigned x3s_pad_lds(const P& pl) {
  return RQ_X3S_COMPACT && x3s_resident((int64_t)pl.tiles * pl.S) == kXWG ? 32768u : 0u;
}

// Modelled time (us) of a plan, to choose the split-K factor and between the two kernels:
//  * MMA: rounds of resident workgroups (fractional: a partly filled last round costs its share — fitted
//    on measured plan sweeps, tools/plan_model_fit.py over profiles/r05/plan_sweep/; the whole-round count
//    it replaced mispriced the 64-tile form at 4 per CU, e.g. C4's 4,608 x 1,024 x 384 SiLU launches) x the
//    MACs a CU does per round, at the measured per-CU rates (128-tile kernel ~0.53 M fp32-MAC/us per
//    CU with its two workgroups, ~0.4 for a lone workgroup; wide kernel 1.3x) — the wide kernel's
//    256 x 256 tiles quantise into 4x coarser rounds (decoder context rows: a 1,536-wide projection is
//    270 wide tiles, two rounds, the second nearly empty);
//  * split-K: the slabs written by the GEMM and read back by the reduction, 2 S M N fp32 at ~3 TB/s (the
//    rate the batched deferred reductions reach), plus a ~4 us reduce launch. Round 4 priced (S + 1) M N at
//    5 TB/s, which chose 256 x 256-tile plans with S = 21..30 for the decoder's 11k-row weight gradients:
//    ~64 MB of slabs per weight, 444 MB (C4) / 800 MB (Amazon) a step. Same-process A/B on MI355X: C4
//    2.766 -> 2.678 ms, Amazon 5.415 -> 5.355, RQ-VAE 1.957 -> 1.924 (half the rate, 1.5 TB/s, loses).
// Checked against tools/gemm_ab.py on MI355X (RQ-VAE and decoder shapes, both kernels forced).
#ifndef RQ_X3W_SPEED
#define RQ_X3W_SPEED 1.3
#endif
#ifndef RQ_X3S_RATE1
#define RQ_X3S_RATE1 0.3    // 64-tile kernel, one workgroup per CU: M fp32-MAC / us
#endif
#ifndef RQ_X3S_RATE2
#define RQ_X3S_RATE2 0.35   // 64-tile kernel, kXWG64 workgroups per CU
#endif
// Modelled cost (us) of the separate slab-reduction launch of a split-K call: the reduction kernel plus the
// gap it adds between launches in a replayed step (4 us measured best of 4 / 8 / 16 at both decoder
// configs in round 3, profiles/r03/reduce_us_ab.txt; 3 with the fractional rounds, fitted on the round-5
// plan sweeps: a back-to-back tiny launch costs ~2.7 us in a replayed graph).
#ifndef RQ_X3_FRAC_ROUNDS
#define RQ_X3_FRAC_ROUNDS 1   // 0: whole rounds and a 4 us reduction (the model before the round-5 sweeps; A/B)
#endif
constexpr double kX3ReduceUs = RQ_X3_FRAC_ROUNDS ? 3.0 : 4.0;
#ifndef RQ_X3_SLAB_BPUS
#define RQ_X3_SLAB_BPUS 3.0e6   // slab bytes per us (written + read back)
#endif
static double x3_plan_time(const X3Plan& p, int64_t M, int64_t N, bool wide) {
  const int64_t cus = resident_slots() / 2;
  const int64_t wgs = (int64_t)p.tiles * p.S;
  const bool small = p.ts == 64;
  const double tile = wide ? (double)kWT2 * kWT2 : (double)p.ts * p.ts;
  const double rate = small ? RQ_X3S_RATE2 : 0.53 * (wide ? RQ_X3W_SPEED : 1.0);   // M MAC / us per CU
  double t;
  if (wgs <= cus) {   // at most one workgroup per CU
    t = tile * (double)p.chunk / ((wide ? rate : (small ? RQ_X3S_RATE1 : 0.4)) * 1e6);
  } else {
    const int per_cu = wide ? 1 : (small ? x3s_resident(wgs) : kXWG);
    const int64_t slots = cus * per_cu;
    // a partly filled last round costs its share; one round at least
    const double rounds = !RQ_X3_FRAC_ROUNDS ? (double)((wgs + slots - 1) / slots)
                                             : (wgs > slots ? (double)wgs / (double)slots : 1.0);
    t = rounds * per_cu * tile * (double)p.chunk / (rate * 1e6);
  }
  if (p.S > 1) t += (double)(2 * p.S) * (double)(M * N) * 4.0 / RQ_X3_SLAB_BPUS + kX3ReduceUs;
  return t;
}

static X3Plan x3_plan_s(int64_t M, int64_t N, int64_t K, int64_t S, bool wide, int ts = kXT) {
  X3Plan p;
  const int T = wide ? kWT2 : ts, KS = wide ? 32 : kXK;
  p.ts = T;
  p.tiles_n = (int)((N + T - 1) / T);
  p.tiles = (int)((M + T - 1) / T) * p.tiles_n;
  int64_t chunk = (K + S - 1) / S;
  chunk = (chunk + KS - 1) / KS * KS;
  p.chunk = chunk;
  p.S = (int)((K + chunk - 1) / chunk);
  if (p.S < 1) p.S = 1;
  p.per = wide ? 0 : (p.tiles * p.S + 7) / 8;
  return p;
}

// Best split-K plan of one tile size: split K when the output tiles cannot fill the chip (weight
// gradients, the decoder's future rows) and the model says the slabs pay for themselves.
static X3Plan x3_plan_t(int64_t M, int64_t N, int64_t K, bool allow_split, int ts) {
  X3Plan p = x3_plan_s(M, N, K, 1, false, ts);
  const int64_t slots_t = (int64_t)(resident_slots() / 2) * kXWG;   // split-K fills the 2-per-CU slots
  if (allow_split && p.tiles < slots_t / 2 && (M * N) % 4 == 0) {   // slab reduction reads float4
    int64_t S = slots_t / p.tiles;
    const int64_t max_s = (K + RQ_X3_MIN_STAGES * kXK - 1) / (RQ_X3_MIN_STAGES * kXK);   // min stages per workgroup
    if (S > max_s) S = max_s;
    if (S > x3_split_cap(M, N)) S = x3_split_cap(M, N);   // slab traffic of the reduction grows with S
    if (ts == 64) {   // small tiles: the best of S = 2, 4, ... up to the one-round heuristic
      for (int64_t s2 = 2; s2 < S; s2 *= 2) {
        const X3Plan q = x3_plan_s(M, N, K, s2, false, ts);
        if (x3_plan_time(q, M, N, false) < x3_plan_time(p, M, N, false)) p = q;
      }
    }
    if (S > 1) {
      const X3Plan q = x3_plan_s(M, N, K, S, false, ts);
      if (x3_plan_time(q, M, N, false) < x3_plan_time(p, M, N, false)) p = q;
    }
  }
  return p;
}

// 128-tile kernel, or its 64-tile form where the time model prefers it (the 128-tiles of a
// 1,280-row operand are 40 workgroups: split-K slabs and their reduction cost more than the GEMM).
// flags (the call's rq_gemm_desc.flags): RQ_GEMM_ONLY_128 / RQ_GEMM_ONLY_64 pin one tile size.
#ifndef RQ_X3_SHORTK_64
#define RQ_X3_SHORTK_64 1   // 0: the time model picks the tile size for K <= 128 too
#endif
#ifndef RQ_X3_SKINNY_UNSPLIT
#define RQ_X3_SKINNY_UNSPLIT 1   // 0: the time model decides split-K for one-row-of-tiles, short-K calls too
#endif

static X3Plan x3_plan(int64_t M, int64_t N, int64_t K, int flags, bool allow_split = true, int epilogue = 0) {
  // One row of 64-tiles (the C4 decoder's 40 future-token rows) over K <= 384 with a plain or residual
  // epilogue: unsplit. Measured per call (profiles/r05/plan_sweep2/sweep_c4.jsonl, hipGraph of 10 calls with
  // their reductions): 6.7-7.2 us unsplit vs 7.1-7.3 at the model's S = 6 plus a reduction launch per call
  // — the model underprices the short-K workgroups' fixed latency; the SiLU epilogues keep the model's split.
  if (RQ_X3_SKINNY_UNSPLIT && !(flags & (RQ_GEMM_ONLY_128 | RQ_GEMM_ONLY_64)) && M <= 64 && K <= 384 &&
      (epilogue == kEpiStore || epilogue == kEpiAdd))
    allow_split = false;
  const X3Plan p = x3_plan_t(M, N, K, allow_split, kXT);
  if (flags & RQ_GEMM_ONLY_128) return p;
  const X3Plan q = x3_plan_t(M, N, K, allow_split, 64);
  if (flags & RQ_GEMM_ONLY_64) return q;
  // K <= 128 (at most four 32-deep stages): the 64-tile form, whose 4 resident workgroups per CU hide the
  // per-workgroup prologue / epilogue latency that such short k loops cannot — measured faster than the
  // 128-tile kernel for every short-K call of the three bench steps (plan_sweep2: RQ-VAE 65,536 x 128 x 64
  // SiLU' epilogue 27.6 -> 20.6 us, SiLU 23.4 -> 22.0; Amazon 11,520 x 512 x 128 14.6 -> 13.8)
  if (RQ_X3_SHORTK_64 && K <= 128) return q;
  return x3_plan_time(q, M, N, false) < x3_plan_time(p, M, N, false) ? q : p;
}

#ifndef RQ_X3W_MIN_STEPS
#define RQ_X3W_MIN_STEPS 8   // split-K of the wide kernel: k steps per workgroup at least
#endif

// Plan of the wide kernel, or false when the 128-tile kernel serves the shape better: k steps
// must be whole (K % 32), padding of a partial 256-row tile must stay small (R % 256 == 0 or
// R >= 2048), and the launch must cover at least a quarter of the CUs (split-K when allowed).
static bool x3w_plan(int64_t M, int64_t N, int64_t K, bool allow_split, X3Plan* p) {
  if (K % 32 != 0 || K <= 0) return false;
  auto fits = [](int64_t R) { return R % kWT2 == 0 || R >= 2048; };
  if (!fits(M) || !fits(N)) return false;
  const int cus = resident_slots() / 2;
  *p = x3_plan_s(M, N, K, 1, true);
  if (allow_split && p->tiles < cus / 2 && (M * N) % 4 == 0) {
    int64_t S = cus / p->tiles;
    const int64_t max_s = K / (32 * RQ_X3W_MIN_STEPS);
    if (S > max_s) S = max_s;
    if (S > x3_split_cap(M, N)) S = x3_split_cap(M, N);
    if (S > 1) {
      const X3Plan q = x3_plan_s(M, N, K, S, true);
      if (x3_plan_time(q, M, N, true) < x3_plan_time(*p, M, N, true)) *p = q;
    }
  }
  return (int64_t)p->tiles * p->S >= cus / 4;
}

// Elements one wide workgroup's operand DMA spans from its descriptor base (RQ_X3W_BUFLDS: 32-bit byte offsets):
// 256 rows of a k-contiguous operand (+ K), or one k chunk of rows of an m/n-contiguous one (+ its rows).
static int64_t x3w_span(int64_t R, int64_t K, int64_t ld, bool kc, int64_t chunk) {
  return kc ? (int64_t)kWT2 * ld + K : (chunk + 32) * ld + R;
}

// The wide kernel runs when both operands are split planes, the (layout, epilogue) pair is
// instantiated (every layout for the plain store; the fused MLP chain's layouts otherwise), the shape
// plans (x3w_plan) and the time model prefers it — or wherever it can run under RQ_GEMM_FORCE_WIDE;
// never under RQ_GEMM_NO_WIDE / RQ_GEMM_ONLY_128 / RQ_GEMM_ONLY_64.
static bool x3w_choose(int64_t M, int64_t N, int64_t K, bool asp, bool bsp, bool a_kc, bool b_kc, int epilogue,
                       int flags, X3Plan* p) {
  if (flags & (RQ_GEMM_NO_WIDE | RQ_GEMM_ONLY_128 | RQ_GEMM_ONLY_64)) return false;
  const bool combo = epilogue == kEpiStore || (epilogue == kEpiSiluFwd && a_kc && b_kc) ||
                     (epilogue == kEpiSiluBwd && a_kc && !b_kc) || (epilogue == kEpiAdd && a_kc && b_kc);
  if (!(asp && bsp && combo && x3w_plan(M, N, K, true, p))) return false;
  // priced against the 128-/64-tile plan this call would really get (same epilogue: the skinny-unsplit rule
  // applies to the store / add epilogues only)
  return (flags & RQ_GEMM_FORCE_WIDE) ||
         x3_plan_time(*p, M, N, true) < x3_plan_time(x3_plan(M, N, K, flags, true, epilogue), M, N, false);
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
    RQ_HIP(zero_async(dW, (size_t)(O * I) * sizeof(float), s));
    if (db) RQ_HIP(zero_async(db, (size_t)O * sizeof(float), s));
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


// Slab bytes of a call: split-K slabs (S > 1) of whichever kernel may run for the shape (the largest of
// the 128-tile, 64-tile and wide plans, so one workspace serves every rq_gemm_desc.flags policy). An
// unsplit accumulating call adds in the GEMM's own epilogue: no slab.
static size_t x3_workspace_bytes(int64_t M, int64_t N, int64_t K) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  const X3Plan p = x3_plan_t(M, N, K, true, kXT), q = x3_plan_t(M, N, K, true, 64);
  X3Plan pw;
  int S = p.S > q.S ? p.S : q.S;
  if (x3w_plan(M, N, K, true, &pw) && pw.S > S) S = pw.S;
  return S > 1 ? (size_t)S * (size_t)(M * N) * sizeof(float) : 0;
}

size_t rq_gemm_bf16x3_workspace(int64_t M, int64_t N, int64_t K) { return x3_workspace_bytes(M, N, K); }

}  // extern "C"

namespace rqhip {

// One validated and planned rq_gemm_bf16x3 call (x3_prepare), its kernel launch (x3_launch) and its slab
// reduction or deferral (x3_post): rq_gemm_bf16x3_run runs the three in a row, rq_gemm_bf16x3_pair prepares
// two calls and, where an instantiation exists, launches both problems in one gemm_x3_pair_kernel.
struct X3Call {
  X3Plan pl;
  bool wide, slab, asp, bsp, trivial;
  int a_kc, b_kc, epilogue, epi_k, code, accumulate, defer, flags;
  int64_t M, N, K;
  float* C;
  float* out;
  X3Args xa;
};

// Validate and plan one call. dry = planning only (rq_gemm_bf16x3_plan): no stream work, no workspace check.
static int x3_prepare(const rq_gemm_desc& d, hipStream_t s, X3Call* c, bool dry = false) {
  const void *A = d.A, *A_lo = d.A_lo, *B = d.B, *B_lo = d.B_lo;
  const int64_t lda = d.lda, ldb = d.ldb, M = d.M, N = d.N, K = d.K, ldc = d.ldc, ldh = d.ldh;
  const int a_kcontig = d.a_kcontig, b_kcontig = d.b_kcontig, epilogue = d.epilogue, accumulate = d.accumulate;
  float* C = d.C;
  const bool asp = A_lo != nullptr, bsp = B_lo != nullptr;
  RQ_CHECK_ARG(dry || (((A && B) || K == 0) && M > 0 && N > 0), "rq_gemm_bf16x3: bad arguments");
  RQ_CHECK_ARG(K >= 0 && M > 0 && N > 0 && M < (1 << 30) && N < (1 << 30) && epilogue >= 0 && epilogue <= 3,
               "rq_gemm_bf16x3: bad arguments");
  const bool needs_h = epilogue == kEpiSiluFwd || epilogue == kEpiSiluBwd;
  RQ_CHECK_ARG(dry || ((epilogue == kEpiSiluBwd || C) && (!needs_h || (d.H_hi && d.H_lo && ldh >= N)) &&
                       ((epilogue != kEpiSiluBwd && epilogue != kEpiAdd) || d.Z)),
               "rq_gemm_bf16x3: epilogue %d needs %s", epilogue,
               epilogue == kEpiSiluBwd ? "Z and H planes"
                                       : (epilogue == kEpiSiluFwd ? "C and H planes" : (epilogue ? "C and Z" : "C")));
  // float4 (fp32) / 8 x bf16 (split) vectors along each operand's contiguous axis
  const int64_t va = asp ? 8 : 4, vb = bsp ? 8 : 4;
  RQ_CHECK_ARG((a_kcontig ? K % va == 0 : M % va == 0) && (b_kcontig ? K % vb == 0 : N % vb == 0) && lda % va == 0 &&
                   ldb % vb == 0,
               "rq_gemm_bf16x3: the contiguous axis of each operand and its leading dim must be multiples of %d "
               "(fp32) / 8 (split)", 4);
  RQ_CHECK_ARG(lda >= (a_kcontig ? K : M) && ldb >= (b_kcontig ? K : N) && (epilogue == kEpiSiluBwd || ldc >= N),
               "rq_gemm_bf16x3: leading dimension too small");
  RQ_CHECK_ARG(N % 4 == 0 && ldc % 4 == 0 && ldh % 4 == 0 && ((uintptr_t)C | (uintptr_t)d.Z) % 16 == 0 &&
                   ((uintptr_t)d.H_hi | (uintptr_t)d.H_lo) % 8 == 0,
               "rq_gemm_bf16x3: N and the output leading dims must be multiples of 4 (vector stores), outputs aligned");
  RQ_CHECK_ARG(((uintptr_t)A | (uintptr_t)A_lo | (uintptr_t)B | (uintptr_t)B_lo) % 16 == 0,
               "rq_gemm_bf16x3: operand pointers must be 16-byte aligned");
  X3Epilogue ep{d.Z, d.H_hi, d.H_lo, ldh, 0u, 1.f, d.seed, 0};
  dropout_params(d.p, &ep.thr, &ep.scale);
  RQ_CHECK_ARG(!accumulate || epilogue == kEpiStore, "rq_gemm_bf16x3: accumulate needs the plain epilogue");
  c->trivial = K == 0;
  if (K == 0) {
    RQ_CHECK_ARG(epilogue == kEpiStore, "rq_gemm_bf16x3: K == 0 needs the plain epilogue");
    if (!accumulate && !dry)
      RQ_HIP(hipMemset2DAsync(C, (size_t)ldc * sizeof(float), 0, (size_t)N * sizeof(float), (size_t)M, s));
    return 0;
  }
  const int flags = d.flags;
  X3Plan pl = x3_plan(M, N, K, flags, true, epilogue);
  X3Plan pw;
  // (the span at the largest chunk, K: a forced split count below only shortens it)
  const bool wide = x3w_choose(M, N, K, asp, bsp, a_kcontig, b_kcontig, epilogue, flags, &pw) &&
                    x3w_span(M, K, lda, a_kcontig, K) < (1ll << 30) && x3w_span(N, K, ldb, b_kcontig, K) < (1ll << 30);
  if (wide) pl = pw;
  // a tuned plan: RQ_GEMM_SPLIT(S) forces the split-K count on the kernel the policy picked
  const int forced_s = (flags >> RQ_GEMM_SPLIT_SHIFT) & RQ_GEMM_SPLIT_MASK;
  if (forced_s > 0) pl = x3_plan_s(M, N, K, forced_s, wide, wide ? kWT2 : pl.ts);
  // slab path: split-K partials go to the workspace with the plain store, and x3_reduce_kernel applies
  // the real epilogue (and the accumulation); an unsplit accumulating call adds in the GEMM's epilogue
  const bool slab = pl.S > 1;
  ep.acc = accumulate && !slab;
  float* out = C;
  if (slab && !dry) {
    const size_t need = (size_t)pl.S * (size_t)(M * N) * sizeof(float);
    RQ_CHECK_ARG(d.workspace != nullptr && d.ws_bytes >= need && ldc == N,
                 "rq_gemm_bf16x3: split-K / accumulate needs ldc == N and workspace %zu >= %zu bytes", d.ws_bytes, need);
    out = static_cast<float*>(d.workspace);
  }
  c->pl = pl;
  c->wide = wide;
  c->slab = slab;
  c->asp = asp;
  c->bsp = bsp;
  c->a_kc = a_kcontig;
  c->b_kc = b_kcontig;
  c->epilogue = epilogue;
  c->epi_k = slab ? (int)kEpiStore : epilogue;   // the epilogue the GEMM kernel itself runs
  c->code = (a_kcontig ? 16 : 0) | (asp ? 8 : 0) | (b_kcontig ? 4 : 0) | (bsp ? 2 : 0);
  c->accumulate = accumulate;
  c->defer = d.defer;
  c->flags = flags;
  c->M = M;
  c->N = N;
  c->K = K;
  c->C = C;
  c->out = out;
  const int64_t ldo = pl.S > 1 ? N : ldc;
  // whole 32-deep stages: unmasked staging (bitwise the masked path; RQ_GEMM_MASKED keeps the masked one)
  const int kfull = !(flags & RQ_GEMM_MASKED) && K % kXK == 0 && pl.chunk % kXK == 0;
  c->xa = X3Args{A, A_lo, lda, B, B_lo, ldb, (int)M, (int)N, K, pl.tiles_n, pl.tiles, pl.S, pl.chunk, pl.per, out, ldo, ep,
                 kfull};
  return 0;
}

static int x3_launch(const X3Call& c, hipStream_t s) {
  const X3Plan& pl = c.pl;
  const X3Args& xa = c.xa;
  const X3Epilogue& ep = xa.ep;
  const int64_t M = c.M, N = c.N, K = c.K, lda = xa.lda, ldb = xa.ldb, ldo = xa.ldc;
  const int epi_k = c.epi_k, code = c.code, a_kcontig = c.a_kc, b_kcontig = c.b_kc;
  const void *A = xa.A, *A_lo = xa.Al, *B = xa.B, *B_lo = xa.Bl;
  float* out = c.out;
  const dim3 grid((unsigned)(pl.per * 8)), block(256);
#define RQ_X3D(AK, AS, BK, BS, EP, DR)                                                                               \
  do {                                                                                                               \
    if (pl.ts == 64)                                                                                                 \
      hipLaunchKernelGGL((gemm_bf16x3_kernel<AK, AS, BK, BS, EP, DR, 64>), grid, block, x3s_pad_lds(pl), s, xa);     \
    else                                                                                                             \
      hipLaunchKernelGGL((gemm_bf16x3_kernel<AK, AS, BK, BS, EP, DR>), grid, block, 0, s, xa);                       \
  } while (0)
#define RQ_X3(AK, AS, BK, BS, EP)                                                                                    \
  do {                                                                                                               \
    if (ep.thr != 0)                                                                                                 \
      RQ_X3D(AK, AS, BK, BS, EP, (EP != kEpiStore));                                                                 \
    else                                                                                                             \
      RQ_X3D(AK, AS, BK, BS, EP, false);                                                                             \
  } while (0)
  bool launched = true;
  if (c.wide) {
    const uint16_t *ah = static_cast<const uint16_t*>(A), *al = static_cast<const uint16_t*>(A_lo);
    const uint16_t *bh = static_cast<const uint16_t*>(B), *bl = static_cast<const uint16_t*>(B_lo);
    const dim3 wgrid((unsigned)(pl.tiles * pl.S)), wblock(512);
#define RQ_X3W(AK, BK, EP, DR)                                                                                        \
  hipLaunchKernelGGL((gemm_x3w_kernel<AK, BK, EP, DR>), wgrid, wblock, 0, s, ah, al, lda, bh, bl, ldb, (int)M, (int)N, \
                     K, pl.tiles_n, pl.tiles, pl.chunk, out, ldo, ep)
    const bool drop = ep.thr != 0;
    const int kc = (a_kcontig ? 2 : 0) | (b_kcontig ? 1 : 0);
    if (epi_k == kEpiStore) {
      switch (kc) {
        case 3: RQ_X3W(true, true, kEpiStore, false); break;
        case 2: RQ_X3W(true, false, kEpiStore, false); break;
        case 1: RQ_X3W(false, true, kEpiStore, false); break;
        default: RQ_X3W(false, false, kEpiStore, false); break;
      }
    } else if (epi_k == kEpiSiluFwd && kc == 3) {
      if (drop) RQ_X3W(true, true, kEpiSiluFwd, true); else RQ_X3W(true, true, kEpiSiluFwd, false);
    } else if (epi_k == kEpiSiluBwd && kc == 2) {
      if (drop) RQ_X3W(true, false, kEpiSiluBwd, true); else RQ_X3W(true, false, kEpiSiluBwd, false);
    } else if (epi_k == kEpiAdd && kc == 3) {
      if (drop) RQ_X3W(true, true, kEpiAdd, true); else RQ_X3W(true, true, kEpiAdd, false);
    } else {
      launched = false;
    }
#undef RQ_X3W
  } else if (epi_k == kEpiStore) {
    switch (code) {
      // every layout with fp32 operands (the generic entry point)
      case 16 | 4: RQ_X3(true, false, true, false, kEpiStore); break;
      case 16: RQ_X3(true, false, false, false, kEpiStore); break;
      case 4: RQ_X3(false, false, true, false, kEpiStore); break;
      case 0: RQ_X3(false, false, false, false, kEpiStore); break;
      // fused MLP chain: forward of the last layer, data grads with split weights, weight grads
      case 16 | 8 | 4 | 2: RQ_X3(true, true, true, true, kEpiStore); break;
      case 16 | 4 | 2: RQ_X3(true, false, true, true, kEpiStore); break;
      case 16 | 8 | 2: RQ_X3(true, true, false, true, kEpiStore); break;
      case 16 | 2: RQ_X3(true, false, false, true, kEpiStore); break;
      case 8 | 2: RQ_X3(false, true, false, true, kEpiStore); break;
      case 8: RQ_X3(false, true, false, false, kEpiStore); break;
      case 2: RQ_X3(false, false, false, true, kEpiStore); break;
      default: launched = false;
    }
  } else if (epi_k == kEpiSiluFwd) {
    switch (code) {
      case 16 | 4 | 2: RQ_X3(true, false, true, true, kEpiSiluFwd); break;
      case 16 | 8 | 4 | 2: RQ_X3(true, true, true, true, kEpiSiluFwd); break;
      default: launched = false;
    }
  } else if (epi_k == kEpiSiluBwd) {
    switch (code) {
      case 16 | 2: RQ_X3(true, false, false, true, kEpiSiluBwd); break;
      case 16 | 8 | 2: RQ_X3(true, true, false, true, kEpiSiluBwd); break;
      default: launched = false;
    }
  } else {
    switch (code) {
      case 16 | 4 | 2: RQ_X3(true, false, true, true, kEpiAdd); break;   // Linear (split weight) + residual
      case 16 | 8 | 4 | 2: RQ_X3(true, true, true, true, kEpiAdd); break;  // MLP chain's last layer + residual
      default: launched = false;
    }
  }
#undef RQ_X3
#undef RQ_X3D
  RQ_CHECK_ARG(launched, "rq_gemm_bf16x3: operand combination (a_kcontig %d, a_split %d, b_kcontig %d, b_split %d) "
                         "not built for epilogue %d", a_kcontig, (int)c.asp, b_kcontig, (int)c.bsp, c.epilogue);
  RQ_LAUNCH_CHECK("gemm_bf16x3_kernel");
  return 0;
}

static int x3_post(const X3Call& c, int* splits, hipStream_t s) {
  if (!c.slab) return 0;
  if (c.defer && c.accumulate && c.epilogue == kEpiStore && splits) {   // the caller reduces later
    *splits = c.pl.S;                                                  // (rq_reduce_partials, layout 0)
    return 0;
  }
  const int64_t n = c.M * c.N;
  const int N = (int)c.N;
  const dim3 rg((unsigned)((n / 4 + kRedColsPerWg - 1) / kRedColsPerWg)), rb(256);
  const X3Epilogue& ep = c.xa.ep;
  const bool drop = ep.thr != 0 && c.epilogue != kEpiStore;
  float* out = c.out;
  float* C = c.C;
  const int S = c.pl.S;
#define RQ_X3R(EP, DR, AC) hipLaunchKernelGGL((x3_reduce_kernel<EP, DR, AC>), rg, rb, 0, s, out, S, n, N, C, ep)
  switch (c.epilogue) {
    case kEpiStore: if (c.accumulate) RQ_X3R(kEpiStore, false, true); else RQ_X3R(kEpiStore, false, false); break;
    case kEpiSiluFwd: if (drop) RQ_X3R(kEpiSiluFwd, true, false); else RQ_X3R(kEpiSiluFwd, false, false); break;
    case kEpiSiluBwd: if (drop) RQ_X3R(kEpiSiluBwd, true, false); else RQ_X3R(kEpiSiluBwd, false, false); break;
    default: if (drop) RQ_X3R(kEpiAdd, true, false); else RQ_X3R(kEpiAdd, false, false); break;
  }
#undef RQ_X3R
  RQ_LAUNCH_CHECK("x3_reduce_kernel");
  return 0;
}

template <class P1, class P2>
static void x3_pair_go(const X3Call& c1, const X3Call& c2, dim3 grid, unsigned pad, hipStream_t s, int n1) {
  hipLaunchKernelGGL((gemm_x3_pair_kernel<P1, P2>), grid, dim3(256), pad, s, c1.xa, c2.xa, n1);
}
template <class P1, int TS>
static void x3_pair_p2(const X3Call& c1, const X3Call& c2, dim3 grid, unsigned pad, hipStream_t s, int n1) {
  switch (c2.code) {   // c2: m-contiguous A (fp32 / split) x n-contiguous B (fp32 / split), plain store
    case 0: x3_pair_go<P1, X3Body<false, false, false, false, kEpiStore, false, TS>>(c1, c2, grid, pad, s, n1); break;
    case 2: x3_pair_go<P1, X3Body<false, false, false, true, kEpiStore, false, TS>>(c1, c2, grid, pad, s, n1); break;
    case 8: x3_pair_go<P1, X3Body<false, true, false, false, kEpiStore, false, TS>>(c1, c2, grid, pad, s, n1); break;
    default: x3_pair_go<P1, X3Body<false, true, false, true, kEpiStore, false, TS>>(c1, c2, grid, pad, s, n1); break;
  }
}
template <int TS>
static bool x3_pair_ts(int k1, const X3Call& c1, const X3Call& c2, dim3 grid, unsigned pad, hipStream_t s, int n1) {
  switch (k1) {   // c1: k-contiguous A (fp32 / split) x n-contiguous split B; plain or SiLU' (+ dropout)
    case 16 | 2: x3_pair_p2<X3Body<true, false, false, true, kEpiStore, false, TS>, TS>(c1, c2, grid, pad, s, n1); return true;
    case 16 | 8 | 2: x3_pair_p2<X3Body<true, true, false, true, kEpiStore, false, TS>, TS>(c1, c2, grid, pad, s, n1); return true;
    case 16 | 2 | 32: x3_pair_p2<X3Body<true, false, false, true, kEpiSiluBwd, false, TS>, TS>(c1, c2, grid, pad, s, n1); return true;
    case 16 | 2 | 64: x3_pair_p2<X3Body<true, false, false, true, kEpiSiluBwd, true, TS>, TS>(c1, c2, grid, pad, s, n1); return true;
    default: return false;
  }
}

template <int TS>
static bool x3_pair_fwd_ts(const X3Call& c1, const X3Call& c2, dim3 grid, unsigned pad, hipStream_t s, int n1) {
  using F32 = X3Body<true, false, true, true, kEpiStore, false, TS>;   // fp32 A
  using SPL = X3Body<true, true, true, true, kEpiStore, false, TS>;    // split A
  const bool a1 = c1.asp, a2 = c2.asp;
  if (!a1 && !a2) x3_pair_go<F32, F32>(c1, c2, grid, pad, s, n1);
  else if (!a1) x3_pair_go<F32, SPL>(c1, c2, grid, pad, s, n1);
  else if (!a2) x3_pair_go<SPL, F32>(c1, c2, grid, pad, s, n1);
  else x3_pair_go<SPL, SPL>(c1, c2, grid, pad, s, n1);
  return true;
}

// The paired launch of a data-gradient problem c1 and a weight-gradient problem c2 (both on the 128- or
// 64-tile kernel with the same tile size), for the operand forms of the decoder's backward: c1 = g W
// (A fp32 or split k-contiguous, B split n-contiguous; plain or SiLU'-with-dropout epilogue), c2 = g^T x
// (A fp32 or split m-contiguous, B fp32 or split n-contiguous, plain). false: no instantiation.
static int x3_pair_k1(const X3Call& c1) {
  const bool drop1 = c1.xa.ep.thr != 0 && c1.epi_k != kEpiStore;
  return c1.code | (c1.epi_k == kEpiSiluBwd ? (drop1 ? 64 : 32) : (c1.epi_k == kEpiStore ? 0 : 128));
}

// The two problems can share a launch: both on the 128- / 64-tile kernel with one tile size, an instantiated
// form pair, and at least one of them leaving resident slots idle alone (the decoder's 40..11,332-row
// launches; two launches that each fill the chip already — the RQ-VAE's 65,536-row 64-tile layers — gain
// nothing and measured 4 us slower paired).
// Two forward projections of different inputs (the decoder block's self-attention qkv of attn_norm(x) and
// cross-attention q of cross_attn_norm(x)): k-contiguous A (fp32 / split) x k-contiguous split B, plain store.
static bool x3_fwd_form(const X3Call& c) {
  return c.epi_k == kEpiStore && (c.code == (16 | 4 | 2) || c.code == (16 | 8 | 4 | 2));
}

static bool x3_pairable(const X3Call& c1, const X3Call& c2) {
  if (c1.wide || c2.wide || c1.pl.ts != c2.pl.ts) return false;
  const bool fwd = x3_fwd_form(c1) && x3_fwd_form(c2);
  if (!fwd) {
    if (c2.epi_k != kEpiStore || c2.code != (c2.code & (8 | 2))) return false;   // c2: m-contig A, n-contig B
    const int k1 = x3_pair_k1(c1);
    if (k1 != (16 | 2) && k1 != (16 | 8 | 2) && k1 != (16 | 2 | 32) && k1 != (16 | 2 | 64)) return false;
  }
  const int64_t w1 = (int64_t)c1.pl.tiles * c1.pl.S, w2 = (int64_t)c2.pl.tiles * c2.pl.S;
  const int64_t slots = c1.pl.ts == 64 ? (int64_t)x3s_resident(w1 + w2) * (resident_slots() / 2) : x3_slots();
  return !(w1 >= slots && w2 >= slots);
}

static bool x3_pair_launch(const X3Call& c1, const X3Call& c2, hipStream_t s) {
  if (!x3_pairable(c1, c2)) return false;
  const int64_t w1 = (int64_t)c1.pl.tiles * c1.pl.S, w2 = (int64_t)c2.pl.tiles * c2.pl.S;
  const int n1 = c1.pl.per * 8, n2 = c2.pl.per * 8;
  const dim3 grid((unsigned)(n1 + n2));
  const bool t64 = c1.pl.ts == 64;
  unsigned pad = 0;
  if (t64 && RQ_X3S_COMPACT && x3s_resident(w1 + w2) == kXWG) pad = 32768u;   // few workgroups: 2 per CU (x3s_pad_lds)
  if (x3_fwd_form(c1) && x3_fwd_form(c2))
    return t64 ? x3_pair_fwd_ts<64>(c1, c2, grid, pad, s, n1) : x3_pair_fwd_ts<128>(c1, c2, grid, 0u, s, n1);
  const int k1 = x3_pair_k1(c1);
  return t64 ? x3_pair_ts<64>(k1, c1, c2, grid, pad, s, n1) : x3_pair_ts<128>(k1, c1, c2, grid, 0u, s, n1);
}

}  // namespace rqhip

extern "C" {

static_assert(sizeof(rq_gemm_desc) == 192, "rq_gemm_desc layout (the ctypes mirror in rqvae_hip/ops.py)");

int rq_gemm_bf16x3_run(const rq_gemm_desc* d, int* splits, void* stream) {
  RQ_CHECK_ARG(d != nullptr, "rq_gemm_bf16x3_run: null descriptor");
  if (splits) *splits = 0;
  hipStream_t s = (hipStream_t)stream;
  X3Call c;
  const int rc = x3_prepare(*d, s, &c);
  if (rc || c.trivial) return rc;
  const int rl = x3_launch(c, s);
  if (rl) return rl;
  return x3_post(c, splits, s);
}

int rq_gemm_bf16x3_pair(const rq_gemm_desc* d, int* splits, void* stream) {
  RQ_CHECK_ARG(d != nullptr, "rq_gemm_bf16x3_pair: null descriptors");
  if (splits) splits[0] = splits[1] = 0;
  hipStream_t s = (hipStream_t)stream;
  X3Call c[2];
  for (int i = 0; i < 2; ++i) {
    const int rc = x3_prepare(d[i], s, &c[i]);
    if (rc) return rc;
  }
  const bool no_pair = ((d[0].flags | d[1].flags) & RQ_GEMM_NO_PAIR) != 0;
  if (c[0].trivial || c[1].trivial || no_pair || !x3_pair_launch(c[0], c[1], s)) {
    for (int i = 0; i < 2; ++i) {
      if (c[i].trivial) continue;
      const int rl = x3_launch(c[i], s);
      if (rl) return rl;
    }
  } else {
    RQ_LAUNCH_CHECK("gemm_x3_pair_kernel");
  }
  // two plain-store slab outputs: one batched reduction (rq_reduce_partials layout 0 = x3_reduce_kernel's
  // order, bitwise) instead of two launches
  auto plain_slab = [](const X3Call& x) { return !x.trivial && x.slab && x.epilogue == kEpiStore && !x.accumulate; };
  if (plain_slab(c[0]) && plain_slab(c[1])) {
    const float* P[2] = {c[0].out, c[1].out};
    float* out[2] = {c[0].C, c[1].C};
    const int64_t n[2] = {c[0].M * c[0].N, c[1].M * c[1].N};
    const int S[2] = {c[0].pl.S, c[1].pl.S}, layout[2] = {0, 0}, acc[2] = {0, 0};
    return rq_reduce_partials(2, P, out, n, S, layout, acc, stream);
  }
  for (int i = 0; i < 2; ++i) {
    if (c[i].trivial) continue;
    const int rp = x3_post(c[i], splits ? splits + i : nullptr, s);
    if (rp) return rp;
  }
  return 0;
}

int rq_gemm_bf16x3_plan(const rq_gemm_desc* d, int* splits) {
  if (splits) *splits = 0;
  if (!d || d->M <= 0 || d->N <= 0 || d->K <= 0) return -1;
  X3Call c;
  if (x3_prepare(*d, nullptr, &c, true) != 0) return -1;
  if (splits) *splits = c.pl.S;
  return c.wide ? 1 : (c.pl.ts == 64 ? 2 : 0);
}

int rq_gemm_bf16x3_pair_plan(const rq_gemm_desc* d) {
  if (!d || ((d[0].flags | d[1].flags) & RQ_GEMM_NO_PAIR)) return 0;
  X3Call c[2];
  for (int i = 0; i < 2; ++i) {
    if (d[i].M <= 0 || d[i].N <= 0 || d[i].K <= 0) return 0;
    if (x3_prepare(d[i], nullptr, &c[i], true) != 0) return 0;
  }
  return x3_pairable(c[0], c[1]) ? 1 : 0;
}

// Deferred partial reductions, many in one launch: out_i[j] (+)= sum_s P_i[s n_i + j] for every entry i,
// each in the SAME order as the reduction it replaces — layout 0 = x3_reduce_kernel's (4 wave lanes over
// s, combined in wave order; a workgroup owns 64 float4 columns), layout 1 = rms_reduce_kernel's (64 lanes
// over s, fixed LDS tree; 4 float4 columns) — so a deferred result is bitwise the immediate one.
constexpr int kRedSegMax = 48;
struct RedSegTable {
  const float* P[kRedSegMax];
  float* out[kRedSegMax];
  int64_t n[kRedSegMax];
  int S[kRedSegMax];
  int layout[kRedSegMax];
  int acc[kRedSegMax];
  int blk0[kRedSegMax + 1];
  int count;
};

__global__ void __launch_bounds__(256) reduce_partials_kernel(RedSegTable t) {
  __shared__ float4 red[256];
  const int b = blockIdx.x;
  int e = 0;
  while (e + 1 < t.count && b >= t.blk0[e + 1]) ++e;
  const int lb = b - t.blk0[e];
  const float* __restrict__ P = t.P[e];
  float* __restrict__ out = t.out[e];
  const int64_t n = t.n[e];
  const int S = t.S[e];
  const int tid = threadIdx.x;
  if (t.layout[e] == 0 && RQ_SLAB_THREAD) {   // one thread per float4 column (slab_sum_w4: the same order)
    const int64_t j = ((int64_t)lb * 256 + tid) * 4;
    if (j >= n) return;
    float4 r = slab_sum_w4(P, S, n, j);
    if (t.acc[e]) {
      const float4 c = *reinterpret_cast<const float4*>(out + j);
      r = make_float4(c.x + r.x, c.y + r.y, c.z + r.z, c.w + r.w);
    }
    *reinterpret_cast<float4*>(out + j) = r;
  } else if (t.layout[e] == 0) {
    const int wave = tid >> 6, lane = tid & 63;
    const int64_t j = ((int64_t)lb * 64 + lane) * 4;
    const bool ok = j < n;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    if (ok) a = strided_slab_sum(P, S, n, j, wave, 4);
    red[wave * 64 + lane] = a;
    __syncthreads();
    if (wave == 0 && ok) {
      float4 r = red[lane];
#pragma unroll
      for (int w = 1; w < 4; ++w) {
        const float4 v = red[w * 64 + lane];
        r.x += v.x; r.y += v.y; r.z += v.z; r.w += v.w;
      }
      if (t.acc[e]) {
        const float4 c = *reinterpret_cast<const float4*>(out + j);
        r = make_float4(c.x + r.x, c.y + r.y, c.z + r.z, c.w + r.w);
      }
      *reinterpret_cast<float4*>(out + j) = r;
    }
  } else {
    constexpr int kC = 4, kQ = 256 / kC;
    const int c = tid % kC, q = tid / kC;
    const int64_t j = ((int64_t)lb * kC + c) * 4;
    const bool ok = j < n;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    if (ok) a = strided_slab_sum(P, S, n, j, q, kQ);
    red[q * kC + c] = a;
    __syncthreads();
#pragma unroll
    for (int h = kQ / 2; h >= 1; h >>= 1) {
      if (q < h) {
        const float4 u = red[q * kC + c], v = red[(q + h) * kC + c];
        red[q * kC + c] = make_float4(u.x + v.x, u.y + v.y, u.z + v.z, u.w + v.w);
      }
      __syncthreads();
    }
    if (q == 0 && ok) {
      float4 r = red[c];
      if (t.acc[e]) {
        const float4 o = *reinterpret_cast<const float4*>(out + j);
        r = make_float4(o.x + r.x, o.y + r.y, o.z + r.z, o.w + r.w);
      }
      *reinterpret_cast<float4*>(out + j) = r;
    }
  }
}

int rq_reduce_partials(int count, const float* const* P, float* const* out, const int64_t* n, const int* S,
                       const int* layout, const int* accumulate, void* stream) {
  RQ_CHECK_ARG(count >= 0 && (count == 0 || (P && out && n && S && layout && accumulate)),
               "rq_reduce_partials: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  for (int base = 0; base < count; base += kRedSegMax) {
    RedSegTable t;
    t.count = std::min(kRedSegMax, count - base);
    int blk = 0;
    for (int i = 0; i < t.count; ++i) {
      const int k = base + i;
      RQ_CHECK_ARG(P[k] && out[k] && n[k] > 0 && n[k] % 4 == 0 && S[k] >= 1 && (layout[k] == 0 || layout[k] == 1) &&
                       ((uintptr_t)P[k] | (uintptr_t)out[k]) % 16 == 0,
                   "rq_reduce_partials: entry %d: need n %% 4 == 0, S >= 1, layout 0/1, 16-B aligned pointers", k);
      t.P[i] = P[k];
      t.out[i] = out[k];
      t.n[i] = n[k];
      t.S[i] = S[k];
      t.layout[i] = layout[k];
      t.acc[i] = accumulate[k] != 0;
      t.blk0[i] = blk;
      blk += (int)((n[k] / 4 + (layout[k] == 0 ? kRedColsPerWg - 1 : 3)) / (layout[k] == 0 ? kRedColsPerWg : 4));
    }
    t.blk0[t.count] = blk;
    if (blk == 0) continue;
    hipLaunchKernelGGL(reduce_partials_kernel, dim3((unsigned)blk), dim3(256), 0, st, t);
    RQ_LAUNCH_CHECK("reduce_partials_kernel");
  }
  return 0;
}

int rq_gemm_bf16x3(const float* A, int64_t lda, int a_kcontig, const float* B, int64_t ldb, int b_kcontig, int64_t M,
                   int64_t N, int64_t K, float* C, int64_t ldc, void* workspace, size_t ws_bytes, void* stream) {
  rq_gemm_desc d{};
  d.A = A;
  d.lda = lda;
  d.a_kcontig = a_kcontig;
  d.B = B;
  d.ldb = ldb;
  d.b_kcontig = b_kcontig;
  d.M = M;
  d.N = N;
  d.K = K;
  d.C = C;
  d.ldc = ldc;
  d.epilogue = kEpiStore;
  d.workspace = workspace;
  d.ws_bytes = ws_bytes;
  return rq_gemm_bf16x3_run(&d, nullptr, stream);
}

int rq_split_bf16x3_multi(int count, const float* const* x, const int64_t* n, uint16_t* const* hi,
                          uint16_t* const* lo, void* stream) {
  RQ_CHECK_ARG(count >= 0 && count <= kSplitMax && (count == 0 || (x && n && hi && lo)),
               "rq_split_bf16x3_multi: 0 <= count <= %d tensors", kSplitMax);
  SplitMulti sm;
  sm.count = count;
  sm.blk0[0] = 0;
  bool vec = true;
  for (int t = 0; t < count; ++t) {
    RQ_CHECK_ARG(n[t] >= 0 && (n[t] == 0 || (x[t] && hi[t] && lo[t])), "rq_split_bf16x3_multi: bad tensor %d", t);
    vec = vec && n[t] % 4 == 0 && (uintptr_t)x[t] % 16 == 0 && ((uintptr_t)hi[t] | (uintptr_t)lo[t]) % 8 == 0;
  }
  int64_t blocks = 0;
  for (int t = 0; t < count; ++t) {
    sm.x[t] = x[t];
    sm.hi[t] = hi[t];
    sm.lo[t] = lo[t];
    sm.n[t] = vec ? n[t] / 4 : n[t];
    blocks += (sm.n[t] + 256 * kSplitPer - 1) / (256 * kSplitPer);
    RQ_CHECK_ARG(blocks < (1ll << 31), "rq_split_bf16x3_multi: too many elements");
    sm.blk0[t + 1] = (int)blocks;
  }
  if (count == 0 || blocks == 0) return 0;
  const dim3 grid((unsigned)blocks);
  if (vec)
    hipLaunchKernelGGL((split_bf16x3_multi_kernel<true>), grid, dim3(256), 0, (hipStream_t)stream, sm);
  else
    hipLaunchKernelGGL((split_bf16x3_multi_kernel<false>), grid, dim3(256), 0, (hipStream_t)stream, sm);
  RQ_LAUNCH_CHECK("split_bf16x3_multi_kernel");
  return 0;
}

// x (n fp32) -> hi = RN_bf16(x), lo = RN_bf16(x - hi): the split form the GEMM consumes.
int rq_split_bf16x3(const float* x, int64_t n, uint16_t* hi, uint16_t* lo, void* stream) {
  RQ_CHECK_ARG(n >= 0 && (n == 0 || (x && hi && lo)), "rq_split_bf16x3: bad arguments");
  if (n == 0) return 0;
  const bool vec = n % 4 == 0 && (uintptr_t)x % 16 == 0 && ((uintptr_t)hi | (uintptr_t)lo) % 8 == 0;
  // vector path: 8 elements per thread per iteration; a grid of 8 x 256 workgroups keeps every CU busy
  const int64_t blocks = vec ? (n / 4 + 511) / 512 : (n + 255) / 256;
  const dim3 grid((unsigned)(blocks < 2048 ? blocks : 2048));
  if (vec)
    hipLaunchKernelGGL((split_bf16x3_kernel<true>), grid, dim3(256), 0, (hipStream_t)stream, x, n, hi, lo);
  else
    hipLaunchKernelGGL((split_bf16x3_kernel<false>), grid, dim3(256), 0, (hipStream_t)stream, x, n, hi, lo);
  RQ_LAUNCH_CHECK("split_bf16x3_kernel");
  return 0;
}


}  // extern "C"

int rqhip::seed_epoch_addr_linear(void** out) { return (int)hipGetSymbolAddress(out, HIP_SYMBOL(rqhip::rq_seed_epoch)); }
