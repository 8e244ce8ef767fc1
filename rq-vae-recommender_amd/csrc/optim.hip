// Multi-tensor AdamW step over every fp32 parameter of a group in ONE launch.
//
// Reference: the training loops step torch.optim.AdamW (train_rqvae.py:96-100,168-172,
// train_decoder.py:151-160,203). torch's fused AdamW chunks each tensor into 64 Ki-element
// blocks: the RQ-VAE's 1.18 M parameters become ~18 workgroups on a 256-CU part (~46 us for
// ~33 MB of traffic). Here a workgroup owns kAdamChunk = 4096 elements of one tensor (289
// workgroups for the RQ-VAE, 5.3 k for the decoder), found from a per-group segment table
// (binary search on the first chunk index). Per element, the torch AdamW update (decoupled decay):
//   p -= lr*wd*p;  m = b1*m + (1-b1)*g;  v = b2*v + (1-b2)*g*g;
//   p -= (lr/bc1) * m / (sqrt(v)/bc2_sqrt + eps)
// with bc1 = 1 - b1^step and bc2_sqrt = sqrt(1 - b2^step) computed by the caller.
// HBM-bound: 4 reads + 3 writes of 4 B per element.
#include "common.h"

namespace rqhip {

struct AdamSeg {        // one parameter tensor
  float* p;
  const float* g;
  float* m;
  float* v;
  int64_t n;            // elements
  int64_t first_chunk;  // prefix sum of ceil(n / kAdamChunk) over the preceding segments of the launch
};

// The segment table travels BY VALUE in the kernel arguments (48 B x 64 < the 4 KiB kernarg limit): no
// device-side table, so nothing to upload when grads are re-allocated between steps, and the launch
// stays graph-capturable. Larger groups are split into several launches on the host.
constexpr int kAdamMaxSegs = 64;
struct AdamSegTable {
  AdamSeg s[kAdamMaxSegs];
};

constexpr int kAdamChunk = 4096;   // elements per 256-thread workgroup (16 per thread)

__global__ void __launch_bounds__(256) adamw_kernel(const AdamSegTable segs, int nseg, float lr, float b1,
                                                     float b2, float eps, float wd, float step_size, float bc2s) {
  __shared__ int s_idx;
  if (threadIdx.x == 0) {   // last segment whose first chunk <= this workgroup's chunk
    int lo = 0, hi = nseg - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (segs.s[mid].first_chunk <= (int64_t)blockIdx.x) lo = mid; else hi = mid - 1;
    }
    s_idx = lo;
  }
  __syncthreads();
  const AdamSeg s = segs.s[s_idx];
  const int64_t base = ((int64_t)blockIdx.x - s.first_chunk) * kAdamChunk;
  const int64_t end = min(base + (int64_t)kAdamChunk, s.n);
  const float one_m_b1 = 1.f - b1, one_m_b2 = 1.f - b2, decay = lr * wd;
  constexpr int U = kAdamChunk / 256;
  float p[U], g[U], m[U], v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {   // all loads first: 4 x 16 independent loads in flight per lane
    const int64_t i = base + u * 256 + threadIdx.x;
    const bool ok = i < end;
    p[u] = ok ? s.p[i] : 0.f;
    g[u] = ok ? s.g[i] : 0.f;
    m[u] = ok ? s.m[i] : 0.f;
    v[u] = ok ? s.v[i] : 0.f;
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * 256 + threadIdx.x;
    if (i >= end) continue;
    float pu = p[u] - decay * p[u];
    const float mu = b1 * m[u] + one_m_b1 * g[u];
    const float vu = b2 * v[u] + one_m_b2 * g[u] * g[u];
    const float denom = sqrtf(vu) / bc2s + eps;
    pu = pu - step_size * mu / denom;
    s.p[i] = pu;
    s.m[i] = mu;
    s.v[i] = vu;
  }
}

}  // namespace rqhip

using namespace rqhip;

extern "C" {

int rq_adamw_step(const int64_t* segs, int64_t nseg, float lr, float beta1, float beta2, float eps,
                  float weight_decay, float bias_correction1, float bias_correction2_sqrt, void* stream) {
  RQ_CHECK_ARG(nseg >= 0, "rq_adamw_step: nseg < 0");
  if (nseg == 0) return 0;
  RQ_CHECK_ARG(segs != nullptr, "rq_adamw_step: null segment table");
  RQ_CHECK_ARG(bias_correction1 > 0.f && bias_correction2_sqrt > 0.f, "rq_adamw_step: bias corrections must be > 0");
  const float step_size = lr / bias_correction1;
  int64_t i = 0;
  while (i < nseg) {   // up to kAdamMaxSegs non-empty tensors per launch
    AdamSegTable tab;
    int cnt = 0;
    int64_t chunks = 0;
    for (; i < nseg && cnt < kAdamMaxSegs; ++i) {
      const int64_t* r = segs + 5 * i;
      RQ_CHECK_ARG(r[4] >= 0, "rq_adamw_step: negative element count");
      if (r[4] == 0) continue;
      RQ_CHECK_ARG(r[0] && r[1] && r[2] && r[3], "rq_adamw_step: null tensor pointer");
      tab.s[cnt] = AdamSeg{(float*)r[0], (const float*)r[1], (float*)r[2], (float*)r[3], r[4], chunks};
      chunks += (r[4] + kAdamChunk - 1) / kAdamChunk;
      ++cnt;
    }
    if (cnt == 0) continue;
    RQ_CHECK_ARG(chunks < (1ll << 31), "rq_adamw_step: too many chunks");
    hipLaunchKernelGGL(adamw_kernel, dim3((unsigned)chunks), dim3(256), 0, (hipStream_t)stream, tab, cnt, lr, beta1,
                       beta2, eps, weight_decay, step_size, bias_correction2_sqrt);
    RQ_LAUNCH_CHECK("rq_adamw_step");
  }
  return 0;
}

size_t rq_adamw_chunk_elems(void) { return (size_t)kAdamChunk; }

}  // extern "C"
