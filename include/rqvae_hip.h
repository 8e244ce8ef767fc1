/* rqvae_hip.h — C ABI of the MI355X (gfx950) RQ-VAE training hot path.
 *
 * Library: rq-vae-recommender_amd/rqvae_hip/librqvae_hip.so (built by `make -C
 * rq-vae-recommender_amd/csrc`). Plain pointers and sizes only; no framework types.
 *
 * Conventions (every entry point):
 *   - All data pointers are DEVICE pointers owned by the caller; kernels never allocate/free.
 *   - `stream` is a hipStream_t (NULL = legacy default stream). Calls are asynchronous,
 *     stream-ordered, never synchronise the host, and are safe to capture in a hipGraph.
 *   - Return 0 on success, a hipError_t (> 0) on a launch/runtime failure, or a negative
 *     argument-check code (-22); rq_last_error() returns the message (thread-local).
 *   - Stateless and re-entrant (autograd may call backward from another host thread).
 *
 * The reference (AdamLTy/RQ-VAE-Recommender) has no FFI of its own: its hot path is Python
 * over ATen + one Triton kernel. Each entry point below names the reference function whose
 * semantics it implements; INTEGRATION.md shows the ctypes binding used by the drop-in
 * nn.Module / autograd.Function surface.
 */
#ifndef RQVAE_HIP_H_
#define RQVAE_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Library identification / errors. */
int rq_abi_version(void);
const char* rq_last_error(void);

/* Quantize modes (modules/quantize.py:16-20 QuantizeForwardMode; 0 = eval path :148-150). */
#define RQ_MODE_EVAL 0
#define RQ_MODE_STE 2
#define RQ_MODE_ROTATION 3

/* out[r] = sum_d rows[r][d]^2 for r < n — the (codebook.T**2).sum(0) term of the L2 distance
 * (modules/quantize.py:110). rows: (n, D) fp32. */
int rq_codebook_sqnorm(const float* rows, int64_t n, int64_t D, float* out, void* stream);

/* Fused L-level residual quantization forward = RqVae.get_semantic_ids' level loop
 * (modules/rqvae.py:114-138) over Quantize.forward (modules/quantize.py:99-156, L2 distance,
 * out_proj = Identity) with QuantizeLoss (modules/loss.py:34-42).
 *   x (B,D) fp32 encoder output; codebooks (L,K,D); cb_sqnorm (L,K) from rq_codebook_sqnorm.
 *   mode RQ_MODE_ROTATION / RQ_MODE_STE (training) or RQ_MODE_EVAL; beta = commitment weight.
 * Outputs: ids (B,L) int64; emb_out (L,B,D); residuals (L,B,D) with residuals[0] = x;
 *   qloss (B,) = sum_l loss_l; emb_sum (B,D) = sum_l emb_out_l, or NULL; emb_norms (L,B) =
 *   |emb_out[l][b]|_2, the embs_norm diagnostic of RqVae.forward (modules/rqvae.py:151), or NULL (the
 *   16x16 kernel writes them from its level epilogue; every other kernel adds one row-norm pass).
 * Requires D a power of two in [8, 1024], 1 <= K <= 2^20, 1 <= L <= 64. Ids are the lowest
 * index among equal minimum distances (torch.min semantics, quantize.py:121).
 * impl: the kernel (0 = auto: 4 for D == 64, K <= 288, B >= 32768; else 2 for D <= 64; else 3 when
 * allowed; else 1), 1 = fused LDS-tiled kernel (any D), 2 = register-resident 32x32x2 kernel (D <= 64),
 * 3 = split path for D >= 128 with 2*ceil(K/128)+1 <= D (per level: distance GEMM + partial argmin over
 * 128x128 tiles, then a row epilogue; emb_out doubles as the level's scratch before it is written),
 * 4 = register-resident 16x16x4 kernel (D == 64, K <= 288; 4 waves per SIMD). Every kernel gives the
 * same ids and the same outputs within fp32 summation order (kernel-vs-kernel tests). */
int rq_quantize_fwd(const float* x, int64_t B, int64_t D, const float* codebooks, const float* cb_sqnorm, int64_t K,
                    int64_t L, int mode, float beta, int64_t* ids, float* emb_out, float* residuals, float* qloss,
                    float* emb_sum, float* emb_norms, int impl, void* stream);

/* Backward of rq_quantize_fwd (the autograd graph of modules/quantize.py:99-156 chained by
 * modules/rqvae.py:129): grads of emb_out (g_emb, (L,B,D) or NULL), of sum_l emb_out
 * (g_emb_sum, (B,D) or NULL), of residuals (g_res, (L,B,D) or NULL) and of qloss (g_qloss,
 * (B,) or NULL). Writes grad_x (B,D) and grad_codebooks (L,K,D) (every element written).
 * The codebook gradient is reduced in ascending row order per codeword (stable counting
 * sort + segmented sum): bitwise deterministic. K <= 4096.
 * workspace: device scratch of at least rq_quantize_bwd_workspace(B,D,K,L) bytes. */
size_t rq_quantize_bwd_workspace(int64_t B, int64_t D, int64_t K, int64_t L);
int rq_quantize_bwd(const float* residuals, const int64_t* ids, const float* codebooks, int64_t B, int64_t D, int64_t K,
                    int64_t L, int mode, float beta, const float* g_emb, const float* g_emb_sum, const float* g_res,
                    const float* g_qloss, float* grad_x, float* grad_codebooks, void* workspace, size_t ws_bytes,
                    void* stream);

/* Deterministic segmented sum: out[k] = sum of rows[b] (B, D) over b with keys[b] == k (int64, in
 * [0, K)), reduced in a fixed order; counts[k] = #rows (or NULL). Used by the k-means codebook
 * init (init/kmeans.py:40-58 centroid means). D <= 1024, K <= 4096. */
size_t rq_segment_sum_workspace(int64_t B, int64_t K);
int rq_segment_sum(const float* rows, const int64_t* keys, int64_t B, int64_t D, int64_t K, float* out, int64_t* counts,
                   void* workspace, size_t ws_bytes, void* stream);

/* RMSNorm (modules/normalize.py:22-32): y = (x * rstd) * w, rstd = rsqrt(mean_j x^2 + eps) per row.
 * x, y: (B, D) fp32 rows, D % 4 == 0, D <= 4096; rstd (B,) saved for the backward. bwd: gx (B, D)
 * and gw (D,) = sum_b gy_b x_b rstd_b (fixed-order reduction; workspace >=
 * rq_rmsnorm_bwd_workspace(B, D) bytes). Replaces torch's pow/mean/rsqrt/mul chain (6 kernels fwd,
 * ~10 bwd) in the decoder (modules/model.py:54-55, modules/transformer/model.py:47-57). */
int rq_rmsnorm_fwd(const float* x, const float* w, int64_t B, int64_t D, float eps, float* y, float* rstd,
                   void* stream);
size_t rq_rmsnorm_bwd_workspace(int64_t B, int64_t D);
int rq_rmsnorm_bwd(const float* x, const float* w, const float* rstd, const float* gy, int64_t B, int64_t D,
                   float* gx, float* gw, void* workspace, size_t ws_bytes, void* stream);

/* RMSNorm followed by nn.Dropout(p) (modules/transformer/model.py:71,74 `self.do(self.attn_norm(x))`,
 * modules/model.py:128-129 `self.do(self.norm(...))`): y = keep * scale * rmsnorm(x), keep drawn from
 * a counter-based generator keyed by `seed` (element e of y keeps iff word e of SplitMix64(seed) >=
 * round(p 2^32); kept values scaled by 1/(1-p)), so the backward regenerates the mask from
 * (seed, e) instead of storing it. p = 0 is plain RMSNorm. */
int rq_rmsnorm_dropout_fwd(const float* x, const float* w, int64_t B, int64_t D, float eps, float p, uint64_t seed,
                           float* y, float* rstd, void* stream);
/* Its backward, with two fusions and a deferral: gres (NULL or B x D) is added to gx — the gradient that
 * reaches x along the residual stream (modules/transformer/model.py:75-82: x feeds both the norm and the
 * residual add; autograd would sum the two in a separate pass) — and accumulate_gw = 1 adds the weight
 * gradient into gw instead of overwriting it (a flat data-parallel gradient bucket). defer = 1 leaves gw's
 * per-workgroup partials (*parts rows of D floats) at the start of the workspace and skips their reduction
 * (*parts = 0 when nothing was deferred); rq_reduce_partials (layout 1) later adds them into gw, batched
 * with other deferred reductions into one launch. workspace >= rq_rmsnorm_bwd_workspace(B, D) bytes. */
int rq_rmsnorm_dropout_bwd(const float* x, const float* w, const float* rstd, const float* gy, const float* gres,
                           int64_t B, int64_t D, float p, uint64_t seed, float* gx, float* gw, int accumulate_gw,
                           int defer, int* parts, void* workspace, size_t ws_bytes, void* stream);
/* Two RMSNorms of the same rows (the decoder block's attn_norm and cross_attn_norm of x,
 * modules/transformer/model.py:75-82), each with its own weight, dropout p and seed: one rstd, y1 and y2 —
 * bitwise two rq_rmsnorm_dropout_fwd calls, in one launch. The backward returns gx = norm2'(gy2) +
 * (norm1'(gy1) + gres) (the chained single-norm calls' roundings) and both weight gradients (accumulate /
 * defer as rq_rmsnorm_dropout_bwd; deferred: w1's partials at workspace, w2's at workspace +
 * rq_rmsnorm_bwd_workspace(B, D), *parts rows each). workspace >= 2 rq_rmsnorm_bwd_workspace(B, D) bytes. */
int rq_rmsnorm2_dropout_fwd(const float* x, const float* w1, const float* w2, int64_t B, int64_t D, float eps, float p1,
                            uint64_t seed1, float p2, uint64_t seed2, float* y1, float* y2, float* rstd, void* stream);
int rq_rmsnorm2_dropout_bwd(const float* x, const float* w1, const float* w2, const float* rstd, const float* gy1,
                            const float* gy2, const float* gres, int64_t B, int64_t D, float p1, uint64_t seed1, float p2,
                            uint64_t seed2, float* gx, float* gw1, float* gw2, int accumulate_gw, int defer, int* parts,
                            void* workspace, size_t ws_bytes, void* stream);
/* Elementwise dropout fusions over n fp32 elements (n % 4 == 0, 16-byte aligned), same mask
 * generator as above (element index = position in the buffer):
 *   rq_silu_dropout_fwd  h = Dropout(SiLU(z))         the MLP hidden layer (modules/encoder.py:20-28)
 *   rq_silu_dropout_bwd  gz = SiLU'(z) * keep * scale * g
 *   rq_dropout_add_fwd   out = h + Dropout(y)          the block output (modules/transformer/model.py:82)
 *   rq_dropout_bwd       gy = keep * scale * g         (grad of y; h's grad is g itself)
 * rq_dropout_params returns the (threshold, scale) pair the kernels use for p. */
int rq_dropout_params(float p, uint32_t* thr, float* scale);
int rq_silu_dropout_fwd(const float* z, int64_t n, float p, uint64_t seed, float* h, void* stream);
int rq_silu_dropout_bwd(const float* g, const float* z, int64_t n, float p, uint64_t seed, float* gz, void* stream);
int rq_dropout_add_fwd(const float* h, const float* y, int64_t n, float p, uint64_t seed, float* out, void* stream);
int rq_dropout_bwd(const float* g, int64_t n, float p, uint64_t seed, float* gy, void* stream);

/* Dropout epoch: a device-side word mixed into every mask key of the functions above and of
 * rq_gemm_bf16x3_run (key = seed + epoch * C). 0 by default (keys = the host seeds). A train step
 * captured into a hipGraph ends with rq_seed_epoch_advance, so every replay draws fresh masks while
 * the forward and backward of one step share the epoch (replaces the per-step host RNG state that
 * torch.compile's cudagraphs trees manage for the reference's nn.Dropout, modules/model.py:247).
 * Both are stream-ordered kernel launches (capturable). */
int rq_seed_epoch_advance(void* stream);
int rq_seed_epoch_set(uint64_t value, void* stream);

/* Weight / bias gradient of a Linear layer over a large batch: dW (O,I) = g^T x, db (O,) = sum_b g
 * (or NULL). g: (Bn, O) rows of stride ldg, x: (Bn, I) rows of stride ldx, fp32, O, I, ld % 4 == 0,
 * 16-byte aligned. Replaces torch autograd's grad_weight = grad_out^T @ input for the nn.Linear
 * layers of modules/encoder.py:7-36 (RQ-VAE encoder/decoder MLPs): split-K over the batch with a
 * fixed-order reduction (deterministic). workspace >= rq_linear_wgrad_workspace(Bn, O, I) bytes. */
size_t rq_linear_wgrad_workspace(int64_t Bn, int64_t O, int64_t I);
int rq_linear_wgrad(const float* g, int64_t ldg, const float* x, int64_t ldx, int64_t Bn, int64_t O, int64_t I,
                    float* dW, float* db, void* workspace, size_t ws_bytes, void* stream);

/* fp32 GEMM at PyTorch's 'high' matmul precision, which the reference selects at import
 * (modules/rqvae.py:19, modules/model.py:27): each operand split as a = hi + lo in bf16, products
 * hi.hi + hi.lo + lo.hi accumulated in fp32 on bf16 MFMA (per-product relative error <= ~2^-17;
 * TF32's is 2^-11). Replaces the nn.Linear matmuls of modules/encoder.py:7-36 and
 * modules/transformer (forward x W^T, data grad g W, weight grad g^T x).
 *   C[m*ldc + n] = sum_k A(m,k) B(n,k),  A(m,k) = a_kcontig ? A[m*lda + k] : A[k*lda + m],
 *                                         B(n,k) = b_kcontig ? B[n*ldb + k] : B[k*ldb + n].
 * The contiguous axis of each operand (K for a k-contiguous one, else M or N) and lda, ldb % 4 == 0,
 * 16-byte aligned pointers. When the output tiles cannot fill the GPU, K is split across workgroups
 * with a fixed-order reduction (deterministic); that case needs ldc == N and workspace >=
 * rq_gemm_bf16x3_workspace(M, N, K) bytes (0 = the shape never splits). */
size_t rq_gemm_bf16x3_workspace(int64_t M, int64_t N, int64_t K);
int rq_gemm_bf16x3(const float* A, int64_t lda, int a_kcontig, const float* B, int64_t ldb, int b_kcontig, int64_t M,
                   int64_t N, int64_t K, float* C, int64_t ldc, void* workspace, size_t ws_bytes, void* stream);

/* Kernel policy of one call (rq_gemm_desc.flags; 0 = the time model picks per shape). For kernel-vs-kernel
 * tests and A/B measurements; every policy gives the same bits for the same split operands. */
#define RQ_GEMM_ONLY_128 1    /* the 128 x 128-tile kernel only (no wide kernel, no 64-tile form) */
#define RQ_GEMM_ONLY_64 2     /* the 64 x 64-tile form wherever the 128-tile kernel would run */
#define RQ_GEMM_FORCE_WIDE 4  /* the wide 256 x 256-tile kernel wherever it can run */
#define RQ_GEMM_NO_WIDE 8     /* never the wide kernel (128- / 64-tile chosen by the model) */
#define RQ_GEMM_MASKED 16     /* masked k staging even for whole 32-deep stages (bitwise the unmasked path) */
#define RQ_GEMM_NO_PAIR 32    /* rq_gemm_bf16x3_pair: two launches */
/* flags | RQ_GEMM_SPLIT(S): split K into S chunks (1..4095; 0 = the planner's count) on the kernel the other
 * flags / the planner pick — a tuned plan for a known shape. S > 1 needs S x M x N fp32 of workspace (which
 * rq_gemm_bf16x3_workspace does not size for a forced S). Bits of a result depend on the chunking. */
#define RQ_GEMM_SPLIT_SHIFT 16
#define RQ_GEMM_SPLIT_MASK 0xFFF
#define RQ_GEMM_SPLIT(S) ((int)(S) << RQ_GEMM_SPLIT_SHIFT)

/* One general split-bf16 GEMM call (the fused MLP chain, modules/encoder.py:7-36 — Linear, SiLU,
 * [Dropout], ..., Linear — and every decoder Linear). An operand is fp32 (X_lo == NULL) or pre-split:
 * two bf16 planes (X = hi, X_lo = lo) of the operand's shape; split operands need their contiguous axis
 * and ld % 8 == 0. The epilogue turns the tile into:
 *   0  C = A B^T                                                  (accumulate = 1: C += A B^T)
 *   3  C = A B^T + Z                                              (a residual add after a projection);
 *      with p > 0: C = Z + Dropout_p(A B^T), the mask of rq_dropout_add_fwd (element m N + n), so
 *      rq_dropout_bwd regenerates it — the transformer block's h + Dropout(MLP(..)) in the MLP's last GEMM
 *   1  C = z = A B^T, and H = split(Dropout_p(SiLU(z)))          (a hidden layer's forward)
 *   2  H = split(SiLU'(Z) * Dropout_p(A B^T)), C unused          (its pre-activation grad)
 * H_hi / H_lo: bf16 planes (M, N) of row stride ldh; Z: (M, N) of stride ldc. The dropout mask is element
 * e = m N + n of the same counter-based mask as rq_silu_dropout_fwd (seed). Split-K applies to every
 * epilogue (partials in the workspace, a fixed-order reduction applies the epilogue). accumulate = 1
 * (plain epilogue only): C += A B^T — a weight gradient added straight into a flat data-parallel
 * gradient bucket (replaces autograd's AccumulateGrad add). defer = 1 (with accumulate): a split call
 * leaves its *splits partial slabs (M x N fp32 each) at the start of the workspace and does not reduce
 * them (*splits = 0: the call completed C itself); the caller adds them into C later with
 * rq_reduce_partials (layout 0), batched with other deferred reductions. */
typedef struct rq_gemm_desc {
  const void* A;
  const void* A_lo;
  int64_t lda;
  int a_kcontig;
  const void* B;
  const void* B_lo;
  int64_t ldb;
  int b_kcontig;
  int64_t M, N, K;
  float* C;
  int64_t ldc;
  int epilogue;
  const float* Z;
  uint16_t* H_hi;
  uint16_t* H_lo;
  int64_t ldh;
  float p;
  uint64_t seed;
  int accumulate;
  int defer;
  void* workspace;
  size_t ws_bytes;
  int flags;     /* RQ_GEMM_* kernel policy, 0 = automatic */
  int reserved;  /* 0 */
} rq_gemm_desc;
int rq_gemm_bf16x3_run(const rq_gemm_desc* d, int* splits, void* stream);
/* Two independent calls d[0], d[1] (splits[i] as rq_gemm_bf16x3_run's `splits`), results identical to the
 * two calls in a row; where both run on the 128- or 64-tile kernel with the same tile size and a paired
 * instantiation exists — a Linear's backward: d[0] the data gradient g W (SiLU'-with-dropout epilogue
 * allowed), d[1] the weight gradient g^T x (modules/encoder.py:7-36, modules/transformer: autograd's
 * grad_input / grad_weight of nn.Linear) — both problems' workgroups run in ONE launch (one launch instead
 * of two; together they fill the chip where each alone cannot). Also two forward projections of different
 * inputs (k-contiguous A, k-contiguous split B, plain store: the decoder block's self-attention qkv and
 * cross-attention q, modules/transformer/model.py:75-80); when both then use split-K, their slabs are
 * reduced in one launch (rq_reduce_partials' layout 0, bitwise the two reductions). RQ_GEMM_NO_PAIR in
 * either: two launches. */
int rq_gemm_bf16x3_pair(const rq_gemm_desc* d, int* splits, void* stream);
/* Host-only planning of a descriptor (pointers may be NULL): the kernel rq_gemm_bf16x3_run would launch —
 * 1 = the wide 256 x 256-tile kernel (both operands split, LDS-DMA staged, 8 waves), 0 = the 128 x 128-tile
 * kernel, 2 = its 64 x 64-tile form, -1 = empty shape / invalid — and *splits its split-K factor. */
int rq_gemm_bf16x3_plan(const rq_gemm_desc* d, int* splits);
/* 1 when rq_gemm_bf16x3_pair would run d[0], d[1] in one launch (host-only planning), else 0. */
int rq_gemm_bf16x3_pair_plan(const rq_gemm_desc* d);
/* Deferred partial reductions, up to 48 per launch: for each entry i, out_i[j] = (accumulate_i ? out_i[j] :
 * 0) + sum_{s < S_i} P_i[s n_i + j], j < n_i (n_i % 4 == 0, 16-B aligned pointers), in the order of the
 * reduction it replaces (layout 0: rq_gemm_bf16x3_run's slab reduction; layout 1: rq_rmsnorm_dropout_bwd's
 * weight-gradient partials) — bitwise the immediate result. Entries must not share an output. Host arrays. */
int rq_reduce_partials(int count, const float* const* P, float* const* out, const int64_t* n, const int* S,
                       const int* layout, const int* accumulate, void* stream);

/* rq_segment_sum over up to 16 sources at once (every embedding table of a decoder step: modules/model.py:59-63,
 * modules/embedding/id_embedder.py): source t's rows (n[t], D) with keys in [0, K[t]) (others and pad[t]
 * skipped) sum into rows [sum_{u<t} K[u], + K[t]) of out (sum K, D). One pack launch + one segmented-sum
 * chain instead of one chain per table; sum K <= 4096. */
size_t rq_segment_sum_multi_workspace(int count, const int64_t* n, const int64_t* K, int64_t D);
int rq_segment_sum_multi(int count, const float* const* rows, const int64_t* const* keys, const int64_t* n,
                         const int64_t* K, const int64_t* pad, int64_t D, float* out, void* workspace, size_t ws_bytes,
                         void* stream);
/* Decoder loss head (modules/model.py:137-143): X = out_proj output rows (B * npos_x, K), row stride ldx;
 * logits row r = b * npos + j is X row b * npos_x + j (the reference drops the last position);
 * u[r] = cross_entropy(logits[r], tgt[r], ignore_index=-1) (NaN for a target >= K), lse[r] saved for the
 * backward, logits = the contiguous (B * npos, K) copy, loss = sum(u) / B, loss_d[j] = sum_b u[b][j] / B
 * (fixed-order sums). K <= 1024. */
int rq_ce_loss_fwd(const float* X, int64_t ldx, int64_t K, const int64_t* tgt, int64_t B, int64_t npos, int64_t npos_x,
                   float* u, float* lse, float* logits, float* loss, float* loss_d, void* stream);
/* Its backward: dX (B * npos_x, K, contiguous) from g_loss (scalar), g_loss_d (npos) and g_logits
 * (B * npos, K), each optional (NULL = zero); rows of the dropped position and ignored targets get only
 * the g_logits part (or zeros). */
int rq_ce_loss_bwd(const float* X, int64_t ldx, int64_t K, const int64_t* tgt, const float* lse, int64_t B, int64_t npos,
                   int64_t npos_x, const float* g_loss, const float* g_loss_d, const float* g_logits, float* dX,
                   void* stream);
/* x (n fp32) -> hi = RN_bf16(x), lo = RN_bf16(x - hi) (bf16 bit patterns). */
int rq_split_bf16x3(const float* x, int64_t n, uint16_t* hi, uint16_t* lo, void* stream);
/* The same for count <= 48 tensors in one launch (x[t], n[t], hi[t], lo[t]: host arrays of device
 * pointers / element counts). */
int rq_split_bf16x3_multi(int count, const float* const* x, const int64_t* n, uint16_t* const* hi,
                          uint16_t* const* lo, void* stream);

/* Number of distinct L-tuples among the B rows of ids (B,L) -> *out_count (device int64).
 * p_unique_ids = count / B (modules/rqvae.py:152-157, which computes it in O(B^2 L)).
 * Requires K^L < 2^63. workspace >= rq_unique_workspace(B, L, K) bytes: where K^L <= 2^24 a byte map
 * of K^L bytes (counted in one pass, no scattered atomics), else a hash table of ~2B slots. */
size_t rq_unique_workspace(int64_t B, int64_t L, int64_t K);
int rq_unique_count(const int64_t* ids, int64_t B, int64_t L, int64_t K, int64_t* out_count, void* workspace,
                    size_t ws_bytes, void* stream);

/* p_unique_ids itself (modules/rqvae.py:152-157: the count / B the train step logs, as torch's true_divide by
 * the scalar B computes it, count * (1 / B) in fp32) -> *out_frac (device float), and the count -> *out_count
 * (either may be NULL, not both); B >= 1. Two launches where K^L <= 2^24 at large B: a bit map of the keys
 * (atomicOr) and one counting pass that also clears it — the workspace (>= rq_unique_fraction_workspace bytes)
 * must then be ALL ZERO on entry and is left all zero (keep one per stream; zero it once). Else the hash table
 * of rq_unique_count (self-initialising) and a division launch. */
size_t rq_unique_fraction_workspace(int64_t B, int64_t L, int64_t K);
int rq_unique_fraction(const int64_t* ids, int64_t B, int64_t L, int64_t K, int64_t* out_count, float* out_frac,
                       void* workspace, size_t ws_bytes, void* stream);

/* out[j] (+)= sum_{s < S} P[s * n + j] for j < n, in a fixed order (deterministic, no atomics):
 * the batch-sum gradient of a parameter broadcast over the batch — `pos + seq_emb` and
 * `bos_emb.repeat(B, 1, 1)` of EncoderDecoderRetrievalModel._predict (modules/model.py:91-95).
 * n % 4 == 0; P and out 16-byte aligned. accumulate != 0: out += sum. */
int rq_col_sum(const float* P, int64_t S, int64_t n, float* out, int accumulate, void* stream);

/* Fused decoder head of RqVae.forward (modules/rqvae.py:145-150): x_hat = l2norm(pre) (decoder MLP's
 * final L2NormalizationLayer, F.normalize eps 1e-12) and recon[b] = sum_c (x_hat - x)^2
 * (modules/loss.py:5-10). pre, x: (B, C) fp32, C % 4 == 0, C <= 4096. fwd writes recon (B,) and
 * norms (B,) = |pre_b| (saved for bwd); bwd writes g_pre (B, C) from g_recon (B,). */
int rq_l2norm_recon_fwd(const float* pre, const float* x, int64_t B, int64_t C, float* recon, float* norms,
                        void* stream);
int rq_l2norm_recon_bwd(const float* pre, const float* x, const float* norms, const float* g_recon, int64_t B,
                        int64_t C, float* g_pre, void* stream);
/* The same gradient emitted as split-bf16 planes (g = hi + lo, rq_split_bf16x3's form): the input of the
 * decoder MLP's last data-grad / weight-grad GEMMs at matmul precision 'high'. */
int rq_l2norm_recon_bwd_split(const float* pre, const float* x, const float* norms, const float* g_recon, int64_t B,
                              int64_t C, uint16_t* g_hi, uint16_t* g_lo, void* stream);
/* rq_l2norm_recon_fwd plus, in the same pass over pre and x, the split gradient rq_l2norm_recon_bwd_split
 * would write if g_recon[b] = gs for every row (the batch-mean loss, loss_means: gs = 1 / B) — speculative:
 * the backward then only checks g_recon (rq_l2norm_recon_bwd_fix) instead of reading pre and x again. */
int rq_l2norm_recon_fwd_grad(const float* pre, const float* x, int64_t B, int64_t C, float* recon, float* norms,
                             float gs, uint16_t* g_hi, uint16_t* g_lo, void* stream);
/* The backward after rq_l2norm_recon_fwd_grad: rows whose g_recon[b * g_stride] (g_stride 0: one value for
 * every row, 1: one per row) is bitwise gs keep the planes the forward wrote; every other row is recomputed
 * with rq_l2norm_recon_bwd_split's arithmetic (same bits as that call). */
int rq_l2norm_recon_bwd_fix(const float* pre, const float* x, const float* norms, const float* g_recon,
                            int64_t g_stride, int64_t B, int64_t C, float gs, uint16_t* g_hi, uint16_t* g_lo,
                            void* stream);

/* RqVae.forward statistics (modules/rqvae.py:151-162):
 *   rq_row_norms   out[r] = |x_r|_2 for rows (rows, D), D % 4 == 0 — embs_norm = emb.norm(dim=-1)
 *   rq_loss_means  out[3] = {mean(recon + qloss), mean(recon), mean(qloss)} over B rows, one
 *                  deterministic pass (the loss and the two logged components). */
int rq_row_norms(const float* x, int64_t rows, int64_t D, float* out, void* stream);
int rq_loss_means(const float* recon, const float* qloss, int64_t B, float* out, void* stream);
/* Its backward when only the total loss out[0] has a gradient g (device scalar): *out_scalar = g * (1 / B)
 * (torch: g / B), and out_vec[0..B) = the same value (the per-row qloss gradient) — one launch. */
int rq_loss_means_bwd(const float* g, int64_t B, float* out_scalar, float* out_vec, void* stream);

/* Gumbel-softmax quantize, training (replaces modules/quantize.py:107-112,121,124-129 with
 * distributions/gumbel.py:14-18 for GUMBEL_SOFTMAX + L2): per row b, dist_k = |x|^2 + |c_k|^2 - 2 x.c_k,
 * ids[b] = argmin_k dist (lowest index on ties), weights = softmax((noise - dist) / temperature) over the K
 * codes (noise: (B, K) Gumbel samples drawn by the caller, as the reference's sample_gumbel), emb = weights @
 * codebook. x (B, D), codebook (K, D), weights (B, K), emb (B, D), all contiguous fp32; D <= 256, K <= 4096.
 * rq_gumbel_softmax_bwd: g_emb (B, D) -> dx (B, D) and ddist (B, K) = d loss / d dist; the codebook gradient
 * weights^T g_emb + 2 colsum(ddist) (.) codebook - 2 ddist^T x is the caller's GEMMs. */
int rq_gumbel_softmax_fwd(const float* x, int64_t B, int64_t D, const float* codebook, int64_t K, const float* noise,
                          float temperature, float* weights, float* emb, int64_t* ids, void* stream);
int rq_gumbel_softmax_bwd(const float* x, const float* codebook, const float* weights, const float* g_emb, int64_t B,
                          int64_t D, int64_t K, float temperature, float* dx, float* ddist, void* stream);

/* Jagged (NJT) conversion — ops/triton/jagged.py. dtype: 0 fp32, 1 bf16, 2 fp16.
 * jagged_offsets: offsets (B+1) int64 = [0, cumsum(clamp(lengths, 0, N))]   (jagged.py:30-33)
 * jagged_from_padded: values[offsets[b]+t] = x[b,t] (+1-1 rounding when add_one_sub_one, as
 *   `target + 1 - 1` at jagged.py:65), x (B,N,D) contiguous            (jagged.py:11-66,92-125)
 * jagged_from_padded_rows: the same into a values buffer of alloc_rows (>= offsets[B]) rows whose tail
 *   rows [offsets[B], alloc_rows) are zero-filled on the device (a row-bucketed allocation: the
 *   caller never needs the valid total on the host, so the call is graph-capturable per bucket)
 * jagged_to_padded: x = zeros(B,N,D); x[b,t] = values[offsets[b]+t] for t < len_b (jagged.py:69-77)
 * B < 65535 per call. */
int jagged_offsets(const int64_t* lengths, int64_t B, int64_t N, int64_t* offsets, void* stream);
int jagged_from_padded(const void* x, int64_t B, int64_t N, int64_t D, const int64_t* offsets, void* values, int dtype,
                       int add_one_sub_one, void* stream);
int jagged_from_padded_rows(const void* x, int64_t B, int64_t N, int64_t D, const int64_t* offsets, void* values,
                            int64_t alloc_rows, int dtype, int add_one_sub_one, void* stream);
int jagged_to_padded(const void* values, const int64_t* offsets, int64_t B, int64_t N, int64_t D, void* x, int dtype,
                     void* stream);

/* Decoder input embeddings straight into the two jagged batches (reference modules/model.py:101-129
 * `_predict` up to padded_to_jagged_tensor, with modules/embedding/id_embedder.py:28-53 SemIdEmbedder /
 * UserIdEmbedder): context row 0 = user_w[user_ids[b] mod n_buckets]; context row 1 + j = wpe_w[j] +
 * sem_w[seq_mask ? type_ids * K + sem_ids : pad] for j < sum(seq_mask[b]); future row 0 = bos, future row
 * 1 + t = sem_w[type_ids_fut * K + sem_ids_fut] + tte_w[type_ids_fut]; every value through the jagged
 * gather's (v + 1) - 1 (ops/triton/jagged.py:65): bitwise the reference composition.
 *   ids (B, N) / (B, L) int64, seq_mask (B, N) bool, tables fp32 row-major with E columns (E % 4 == 0);
 *   ctx_values (ctx_alloc_rows, E): rows past ctx_offsets[B] zero; ctx_offsets (B+1) = [0, cumsum(sum(mask)+1)];
 *   fut_values (B * (L+1), E), fut_offsets (B+1) = b (L+1); keys (B, N+L) int64 = the context's sem-table rows
 *   then the future's (the backward's segmented-sum keys), uid_mod (B) int64; lpt_order (NULL or B int32, B <= 4096):
 *   the contexts longest-first (the ranking of the attention LPT order, for RQ_ATTN_ORDER_GIVEN). Two launches;
 *   graph-capturable. */
int rq_dec_prologue_fwd(const int64_t* user_ids, const int64_t* sem_ids, const int64_t* type_ids, const bool* seq_mask,
                        const int64_t* sem_ids_fut, const int64_t* type_ids_fut, int64_t B, int64_t N, int64_t L,
                        int64_t E, const float* user_w, int64_t n_buckets, const float* sem_w, int64_t n_sem_rows,
                        int64_t K, int64_t pad, const float* wpe_w, int64_t n_wpe_rows, const float* tte_w,
                        int64_t n_tte_rows, const float* bos, float* ctx_values, int64_t ctx_alloc_rows,
                        int64_t* ctx_offsets, float* fut_values, int64_t* fut_offsets, int64_t* keys, int64_t* uid_mod,
                        int* lpt_order, void* stream);

/* Varlen multi-head attention on packed rows = F.scaled_dot_product_attention on NJT q/k/v
 * (modules/transformer/attention.py:113-124), dropout 0, is_causal top-left.
 *   q[t][h][d] at q + t*sq + h*hd + d (likewise k, v, out, dout, dq, dk, dv with their strides);
 *   cu_q, cu_k (B+1) int64 offsets; max_q / max_k >= the longest segment (grid bound);
 *   lse (H, Tq) fp32 log-sum-exp per query (written by fwd, read by bwd). hd in {16, 32, 64, 128}.
 *   Tq / Tk: ALLOCATED rows of the q-side / kv-side buffers (>= cu_q[B] / cu_k[B]); rows past the
 *   last sequence get zero out / dq / dk / dv (written by the kernels: graph-capturable per bucket).
 *   ws / ws_elems: caller-provided fp32 scratch of at least varlen_attn_{fwd,bwd}_ws_elems(...) floats, or
 *   NULL / 0 (the forms that need none).
 *   flags: RQ_ATTN_* kernel policy, 0 = the measured-best forms (kernel-vs-kernel tests / A/B runs; every
 *   policy computes the same function within fp32 summation order).
 * Forward: with scratch, long ranges (max_k > 128, 2 <= B <= 4096) rank the sequences longest-first and
 * dispatch their workgroups in that order (no straggler tail); <= 16 queries per sequence over > 128 keys
 * (non-causal: the decoder's cross-attention) run split-key partials (one one-wave workgroup per 128-key
 * block) merged per query in block order (deterministic); many queries over long keys at low occupancy run
 * the key-split form. Backward is deterministic (no atomics): short ranges run one-pass forms (dQ, dK, dV
 * from S and dP formed once per tile pair); with scratch, longer ranges (hd == 64) run ONE fused launch
 * per key block (after a delta = rowsum(dO*O) pre-pass) whose dQ partials are summed in block order by a
 * reduction launch, and — when varlen_attn_bwd_ws_elems was given Tk >= 0 — may split each key block's
 * query range over up to 4 workgroups when the grid cannot fill the GPU (few long sequences per GPU),
 * their dK / dV partials summed in split order. Without scratch those ranges run the two-pass form (dQ per
 * query block, writing delta (H, Tq) to the caller's `delta`, then dK / dV per key block). */
#define RQ_ATTN_NO_DMA 1          /* register-staged short forms instead of the LDS-DMA ones */
#define RQ_ATTN_TWO_PASS 2        /* two-pass backward everywhere (no one-pass / fused forms) */
#define RQ_ATTN_NO_SPLIT 4        /* no split-key / key-split forward */
#define RQ_ATTN_SPLIT_BF16 8      /* matmul precision 'high': the hd-64 forwards over more than 32 keys with more
                                     than 16 queries per sequence (chunked, key-split and short forms) or with
                                     few queries over long key ranges (cross-attention, key-split form) multiply
                                     Q K^T and P V in split-bf16 (3 bf16 MFMA products, fp32 accumulate and
                                     softmax) instead of exact fp32; so does the fused long-range backward (S, dP,
                                     dV, dK and dQ products; P, dS fp32) */
#define RQ_ATTN_FEWQ_WG 16        /* few-query backward over 49..128 keys: one workgroup per (sequence, head) instead of
                                     the persistent walk with the next unit staged by LDS-DMA (same bits) */
#define RQ_ATTN_LPT_SHORT 32      /* the short / few-query forms (<= 128 keys) also dispatch their sequences longest-first
                                     (an order launch; the backward's scratch then holds B ints) */
#define RQ_ATTN_ORDER_GIVEN 64    /* ws[0, B) (as int32) already holds the longest-first order of cu_k's segments (e.g. from
                                     rq_dec_prologue_fwd): the forwards and the short backwards use it without an order
                                     launch (the fused long-range backward keeps its own) */
#define RQ_ATTN_QSPLIT_SHIFT 8
#define RQ_ATTN_QSPLIT(n) ((n) << RQ_ATTN_QSPLIT_SHIFT)   /* fused backward query splits forced to n (1..8; 1 = off) */
int varlen_attn_fwd_ws_elems(int64_t B, int64_t H, int64_t hd, int64_t max_q, int64_t max_k, int64_t Tq, int causal,
                             int flags, int64_t* elems);
int varlen_attn_fwd(const float* q, int64_t sq, const float* k, int64_t sk, const float* v, int64_t sv,
                    const int64_t* cu_q, const int64_t* cu_k, int64_t B, int64_t H, int64_t hd, int64_t max_q,
                    int64_t max_k, int causal, float scale, float* out, int64_t so, float* lse, int64_t Tq, float* ws,
                    int64_t ws_elems, int flags, void* stream);
/* Tk < 0: scratch without the query splits' dK / dV partials. */
int varlen_attn_bwd_ws_elems(int64_t B, int64_t H, int64_t hd, int64_t max_q, int64_t max_k, int64_t Tq, int64_t Tk,
                             int flags, int64_t* elems);
int varlen_attn_bwd(const float* q, int64_t sq, const float* k, int64_t sk, const float* v, int64_t sv, const float* out,
                    int64_t so, const float* dout, int64_t sdo, const float* lse, int64_t Tq, const int64_t* cu_q,
                    const int64_t* cu_k, int64_t B, int64_t H, int64_t hd, int64_t max_q, int64_t max_k, int causal,
                    float scale, float* dq, int64_t sdq, float* dk, int64_t sdk, float* dv, int64_t sdv, int64_t Tk,
                    float* delta, float* ws, int64_t ws_elems, int flags, void* stream);

/* AdamW step (torch.optim.AdamW as stepped by train_rqvae.py:168-172 / train_decoder.py:203) over
 * every fp32 parameter of a group, one launch per 64 tensors. segs: HOST array of nseg records of 5
 * int64 {p, g, exp_avg, exp_avg_sq (device pointers), n}; it is copied into the kernel arguments, so
 * the call needs no device-side table and is graph-capturable. Per element (rq_adamw_chunk_elems()
 * elements per workgroup):
 *   p -= lr*wd*p; m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2; p -= (lr/bc1) m / (sqrt(v)/bc2_sqrt + eps).
 * bias_correction1 = 1 - b1^step, bias_correction2_sqrt = sqrt(1 - b2^step) (caller-computed). */
int rq_adamw_step(const int64_t* segs, int64_t nseg, float lr, float beta1, float beta2, float eps,
                  float weight_decay, float bias_correction1, float bias_correction2_sqrt, void* stream);
size_t rq_adamw_chunk_elems(void);

#ifdef __cplusplus
}
#endif

#endif /* RQVAE_HIP_H_ */
