// Distinct semantic-ID tuples in a batch (RqVae debug metric p_unique_ids).
//
// Reference: modules/rqvae.py:152-157 computes (~triu(eq_all(B x B x L), 1)).all(1).sum() / B,
// an O(B^2 L) comparison. The count of rows with no identical earlier row equals the number
// of distinct tuples, so this path inserts each packed tuple key into an open-addressing
// table (linear probing, 64-bit CAS) and counts successful inserts: O(B L) and exact.
// Keys pack the L ids in base K (requires K^L < 2^63); the table holds >= 2B slots so the
// probe sequence always terminates.
#include "common.h"

namespace rqhip {

constexpr unsigned long long kEmpty = ~0ull;

__device__ __forceinline__ unsigned long long mix64(unsigned long long k) {
  k ^= k >> 33; k *= 0xff51afd7ed558ccdull; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ull; k ^= k >> 33;
  return k;
}

__global__ void __launch_bounds__(256) unique_insert_kernel(const int64_t* __restrict__ ids, int64_t B, int L, int64_t K,
                                                             unsigned long long* __restrict__ table, int64_t mask,
                                                             unsigned long long* __restrict__ count) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= B) return;
  unsigned long long key = 0;
  for (int l = L - 1; l >= 0; --l) key = key * (unsigned long long)K + (unsigned long long)ids[r * L + l];
  int64_t slot = (int64_t)(mix64(key) & (unsigned long long)mask);
  for (int64_t probe = 0; probe <= mask; ++probe) {
    const unsigned long long prev = atomicCAS(table + slot, kEmpty, key);
    if (prev == kEmpty) { atomicAdd(count, 1ull); return; }
    if (prev == key) return;
    slot = (slot + 1) & mask;
  }
}

}  // namespace rqhip

using namespace rqhip;

extern "C" {

static int64_t table_slots(int64_t B) {
  int64_t t = 1;
  while (t < 2 * B) t <<= 1;
  return t < 64 ? 64 : t;
}

size_t rq_unique_workspace(int64_t B) { return (size_t)table_slots(B) * sizeof(unsigned long long); }

int rq_unique_count(const int64_t* ids, int64_t B, int64_t L, int64_t K, int64_t* out_count, void* workspace,
                    size_t ws_bytes, void* stream) {
  RQ_CHECK_ARG(ids && out_count && workspace, "rq_unique_count: null pointer");
  RQ_CHECK_ARG(B >= 0 && L >= 1 && K >= 1, "rq_unique_count: bad shape");
  double bits = 0;
  for (int64_t k = K - 1; k > 0; k >>= 1) bits += 1;
  RQ_CHECK_ARG(bits * L <= 63, "rq_unique_count: K^L must fit 63 bits (K=%lld, L=%lld)", (long long)K, (long long)L);
  RQ_CHECK_ARG(ws_bytes >= rq_unique_workspace(B), "rq_unique_count: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int64_t slots = table_slots(B);
  RQ_HIP(hipMemsetAsync(workspace, 0xFF, (size_t)slots * sizeof(unsigned long long), s));
  RQ_HIP(hipMemsetAsync(out_count, 0, sizeof(int64_t), s));
  if (B > 0)
    hipLaunchKernelGGL(unique_insert_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, s, ids, B, (int)L, K,
                       (unsigned long long*)workspace, slots - 1, (unsigned long long*)out_count);
  RQ_LAUNCH_CHECK("rq_unique_count");
  return 0;
}

}  // extern "C"
