// Distinct semantic-ID tuples in a batch (RqVae debug metric p_unique_ids).
//
// Reference: modules/rqvae.py:152-157 computes (~triu(eq_all(B x B x L), 1)).all(1).sum() / B,
// an O(B^2 L) comparison. The count of rows with no identical earlier row equals the number
// of distinct tuples, so this path inserts each packed tuple key into an open-addressing
// table (linear probing, 64-bit CAS) and counts successful inserts: O(B L) and exact.
// Keys pack the L ids in base K (requires K^L < 2^63); the table holds >= 2B slots so the
// probe sequence always terminates.
#include "common.h"

#include <algorithm>

namespace rqhip {

constexpr unsigned long long kEmpty = ~0ull;

__device__ __forceinline__ unsigned long long mix64(unsigned long long k) {
  k ^= k >> 33; k *= 0xff51afd7ed558ccdull; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ull; k ^= k >> 33;
  return k;
}

// Hash path set-up in one launch (no memset nodes): every slot empty, the count zero.
__global__ void __launch_bounds__(256) unique_table_init_kernel(unsigned long long* __restrict__ table, int64_t slots,
                                                                 unsigned long long* __restrict__ count) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < slots) table[i] = kEmpty;
  if (i == 0) *count = 0ull;
}

__global__ void __launch_bounds__(256) unique_insert_kernel(const int64_t* __restrict__ ids, int64_t B, int L, int64_t K,
                                                             unsigned long long* __restrict__ table, int64_t mask,
                                                             unsigned long long* __restrict__ count) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  bool inserted = false;
  if (r < B) {
    unsigned long long key = 0;
    for (int l = L - 1; l >= 0; --l) key = key * (unsigned long long)K + (unsigned long long)ids[r * L + l];
    int64_t slot = (int64_t)(mix64(key) & (unsigned long long)mask);
    for (int64_t probe = 0; probe <= mask; ++probe) {
      const unsigned long long prev = atomicCAS(table + slot, kEmpty, key);
      if (prev == kEmpty) { inserted = true; break; }
      if (prev == key) break;
      slot = (slot + 1) & mask;
    }
  }
  // one counter update per wave (a single hot address took one atomic per distinct row: ~23 us at B = 65,536)
  const unsigned long long n = __popcll(__ballot(inserted));
  if ((threadIdx.x & 63) == 0 && n) atomicAdd(count, n);
}

// Small key spaces (K^L <= 2^24, e.g. ML-32M: 256^3) at large batches: a byte map instead of the hash
// table — each row stores 1 at its key (plain byte stores: racing writers all store 1), then one pass
// counts the set bytes. No atomics on the scattered side (the table's device-scope CAS traffic took
// ~22 us at B = 65,536; the map is ~3x cheaper including its 16 MiB memset). The map's memset and
// counting pass cost O(K^L) whatever B is, so small batches (eval, B = 64..4,096) keep the hash table:
// the map is used only when B >= K^L / kMapRowsDiv.
constexpr int64_t kMapKeys = 1 << 24;
constexpr int64_t kMapRowsDiv = 512;

static bool use_byte_map(int64_t B, double keys) { return keys <= (double)kMapKeys && (double)B * kMapRowsDiv >= keys; }

// A row with an id outside [0, K) has no slot in the map: it is not marked and counts as one distinct
// tuple of its own (the quantizer never produces such ids; rq_unique_count is a public entry point, so
// a bad row must not turn into an out-of-bounds store).
__global__ void __launch_bounds__(256) unique_mark_kernel(const int64_t* __restrict__ ids, int64_t B, int L, int64_t K,
                                                           unsigned char* __restrict__ map,
                                                           unsigned long long* __restrict__ bad,
                                                           unsigned long long* __restrict__ count) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r == 0) *count = 0ull;   // the count kernel runs after this launch
  bool out_of_range = false;
  if (r < B) {
    int64_t key = 0;
    for (int l = L - 1; l >= 0; --l) {
      const int64_t v = ids[r * L + l];
      out_of_range |= v < 0 || v >= K;
      key = key * K + v;
    }
    if (!out_of_range) map[key] = 1;
  }
  const unsigned long long n = __popcll(__ballot(out_of_range));
  if ((threadIdx.x & 63) == 0 && n) atomicAdd(bad, n);
}

// 16 bytes per thread per step; one atomic per workgroup (workgroup 0 adds the out-of-range rows)
__global__ void __launch_bounds__(256) unique_map_count_kernel(const uint4* __restrict__ map, int64_t n16,
                                                                const unsigned long long* __restrict__ bad,
                                                                unsigned long long* __restrict__ count) {
  __shared__ unsigned int part[4];
  unsigned int c = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256) {
    const uint4 v = map[i];
    // bytes are 0 or 1: the sum of a word's bytes is its popcount
    c += __popc(v.x) + __popc(v.y) + __popc(v.z) + __popc(v.w);
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0)
    atomicAdd(count, (unsigned long long)(part[0] + part[1] + part[2] + part[3]) + (blockIdx.x == 0 ? *bad : 0ull));
}

// p_unique_ids in two launches with a workspace that stays zero between calls: a bit map of the K^L keys
// (<= 2^24: 2 MiB) marked with atomicOr, then one pass that counts the set bits, clears the words it found set
// and adds (1 << 40 | its count) to a packed counter with ONE atomic per workgroup — the workgroup that sees
// every other one's increment in the returned value writes the count and count * inv_b (torch's true_divide by
// a scalar multiplies by the host reciprocal), and clears the out-of-range counter. The map's memset, the
// byte-map count and the division kernel of the rq_unique_count route are gone.
__global__ void __launch_bounds__(256) unique_mark_bits_kernel(const int64_t* __restrict__ ids, int64_t B, int L, int64_t K,
                                                                unsigned* __restrict__ bits,
                                                                unsigned long long* __restrict__ bad,
                                                                unsigned long long* __restrict__ packed) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r == 0) *packed = 0ull;   // the count kernel runs after this launch
  bool out_of_range = false;
  if (r < B) {
    int64_t key = 0;
    for (int l = L - 1; l >= 0; --l) {
      const int64_t v = ids[r * L + l];
      out_of_range |= v < 0 || v >= K;
      key = key * K + v;
    }
    if (!out_of_range) atomicOr(bits + (key >> 5), 1u << (key & 31));
  }
  const unsigned long long n = __popcll(__ballot(out_of_range));
  if ((threadIdx.x & 63) == 0 && n) atomicAdd(bad, n);
}

__global__ void __launch_bounds__(256) unique_count_clear_kernel(uint4* __restrict__ bits, int64_t n16,
                                                                  unsigned long long* __restrict__ bad,
                                                                  unsigned long long* __restrict__ packed,
                                                                  int64_t* __restrict__ out_count,
                                                                  float* __restrict__ out_frac, float inv_b) {
  __shared__ unsigned int part[4];
  unsigned int c = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256) {
    const uint4 v = bits[i];
    if (v.x | v.y | v.z | v.w) {
      c += __popc(v.x) + __popc(v.y) + __popc(v.z) + __popc(v.w);
      bits[i] = make_uint4(0u, 0u, 0u, 0u);
    }
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long t = (unsigned long long)(part[0] + part[1] + part[2] + part[3]);
    const unsigned long long old = atomicAdd(packed, (1ull << 40) | t);
    if ((old >> 40) == (unsigned long long)(gridDim.x - 1)) {   // the last workgroup
      const unsigned long long total = (old & ((1ull << 40) - 1)) + t + *bad;
      if (out_count) *out_count = (int64_t)total;
      if (out_frac) *out_frac = (float)total * inv_b;
      *bad = 0ull;
      *packed = 0ull;   // every workgroup's increment is in: the workspace is all zero again
    }
  }
}

// The hash-table route's count -> count and count * inv_b.
__global__ void unique_fraction_kernel(const unsigned long long* __restrict__ count, int64_t* __restrict__ out_count,
                                       float* __restrict__ out_frac, float inv_b) {
  const unsigned long long c = *count;
  if (out_count) *out_count = (int64_t)c;
  if (out_frac) *out_frac = (float)c * inv_b;
}

}  // namespace rqhip

using namespace rqhip;

extern "C" {

static int64_t table_slots(int64_t B) {
  int64_t t = 1;
  while (t < 2 * B) t <<= 1;
  return t < 64 ? 64 : t;
}

static size_t table_bytes(int64_t B) { return (size_t)table_slots(B) * sizeof(unsigned long long); }

// workspace of rq_unique_count for these K, L: the byte map where K^L <= 2^24, else the hash table
size_t rq_unique_workspace(int64_t B, int64_t L, int64_t K) {
  double keys = 1;
  for (int64_t l = 0; l < L; ++l) keys *= (double)K;
  // the map (rounded to 16 B) + the out-of-range row counter
  return use_byte_map(B, keys) ? (size_t)(((int64_t)keys + 15) / 16 * 16 + 16) : table_bytes(B);
}

int rq_unique_count(const int64_t* ids, int64_t B, int64_t L, int64_t K, int64_t* out_count, void* workspace,
                    size_t ws_bytes, void* stream) {
  RQ_CHECK_ARG(ids && out_count && workspace, "rq_unique_count: null pointer");
  RQ_CHECK_ARG(B >= 0 && L >= 1 && K >= 1, "rq_unique_count: bad shape");
  double bits = 0;
  for (int64_t k = K - 1; k > 0; k >>= 1) bits += 1;
  RQ_CHECK_ARG(bits * L <= 63, "rq_unique_count: K^L must fit 63 bits (K=%lld, L=%lld)", (long long)K, (long long)L);
  hipStream_t s = (hipStream_t)stream;
  double keys = 1;
  for (int64_t l = 0; l < L; ++l) keys *= (double)K;
  if (use_byte_map(B, keys) && ws_bytes >= rq_unique_workspace(B, L, K)) {
    const int64_t nb = ((int64_t)keys + 15) / 16 * 16;
    unsigned long long* bad = reinterpret_cast<unsigned long long*>(static_cast<char*>(workspace) + nb);
    RQ_HIP(zero_async(workspace, (size_t)nb + 16, s));
    hipLaunchKernelGGL(unique_mark_kernel, dim3((unsigned)std::max<int64_t>(1, (B + 255) / 256)), dim3(256), 0, s, ids, B,
                       (int)L, K, (unsigned char*)workspace, bad, (unsigned long long*)out_count);
    const int64_t n16 = nb / 16;
    // few workgroups: their one device-scope atomic each on a single address serialises (~10 ns apiece)
    hipLaunchKernelGGL(unique_map_count_kernel, dim3((unsigned)std::min<int64_t>(128, (n16 + 255) / 256)), dim3(256), 0, s,
                       (const uint4*)workspace, n16, bad, (unsigned long long*)out_count);
    RQ_LAUNCH_CHECK("rq_unique_count");
    return 0;
  }
  RQ_CHECK_ARG(ws_bytes >= table_bytes(B), "rq_unique_count: workspace too small");
  const int64_t slots = table_slots(B);
  hipLaunchKernelGGL(unique_table_init_kernel, dim3((unsigned)((slots + 255) / 256)), dim3(256), 0, s,
                     (unsigned long long*)workspace, slots, (unsigned long long*)out_count);
  if (B > 0)
    hipLaunchKernelGGL(unique_insert_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, s, ids, B, (int)L, K,
                       (unsigned long long*)workspace, slots - 1, (unsigned long long*)out_count);
  RQ_LAUNCH_CHECK("rq_unique_count");
  return 0;
}

// rq_unique_fraction: the bit-map route where K^L <= 2^24 and B * kMapRowsDiv >= K^L (the map + two 8-B
// counters, ZERO on entry and left zero), else the hash table (+ its count word)
static bool use_bit_map(int64_t B, double keys) { return use_byte_map(B, keys); }

size_t rq_unique_fraction_workspace(int64_t B, int64_t L, int64_t K) {
  double keys = 1;
  for (int64_t l = 0; l < L; ++l) keys *= (double)K;
  return use_bit_map(B, keys) ? (size_t)(((int64_t)keys + 127) / 128 * 16 + 16) : table_bytes(B) + 16;
}

int rq_unique_fraction(const int64_t* ids, int64_t B, int64_t L, int64_t K, int64_t* out_count, float* out_frac,
                       void* workspace, size_t ws_bytes, void* stream) {
  RQ_CHECK_ARG(ids && (out_count || out_frac) && workspace, "rq_unique_fraction: null pointer");
  RQ_CHECK_ARG(B >= 1 && L >= 1 && K >= 1, "rq_unique_fraction: bad shape");
  double bits = 0;
  for (int64_t k = K - 1; k > 0; k >>= 1) bits += 1;
  RQ_CHECK_ARG(bits * L <= 63, "rq_unique_fraction: K^L must fit 63 bits (K=%lld, L=%lld)", (long long)K, (long long)L);
  RQ_CHECK_ARG(ws_bytes >= rq_unique_fraction_workspace(B, L, K), "rq_unique_fraction: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const float inv_b = 1.0f / (float)B;   // torch: true_divide(count, B) = count * (1 / B) in fp32
  double keys = 1;
  for (int64_t l = 0; l < L; ++l) keys *= (double)K;
  if (use_bit_map(B, keys)) {
    const int64_t nb = ((int64_t)keys + 127) / 128 * 16;   // bytes of the bit map (whole uint4 words)
    unsigned long long* bad = reinterpret_cast<unsigned long long*>(static_cast<char*>(workspace) + nb);
    hipLaunchKernelGGL(unique_mark_bits_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, s, ids, B, (int)L, K,
                       (unsigned*)workspace, bad, bad + 1);
    const int64_t n16 = nb / 16;
    hipLaunchKernelGGL(unique_count_clear_kernel, dim3((unsigned)std::min<int64_t>(128, (n16 + 255) / 256)), dim3(256),
                       0, s, (uint4*)workspace, n16, bad, bad + 1, out_count, out_frac, inv_b);
    RQ_LAUNCH_CHECK("rq_unique_fraction");
    return 0;
  }
  const int64_t slots = table_slots(B);
  unsigned long long* cnt = reinterpret_cast<unsigned long long*>(static_cast<char*>(workspace) + table_bytes(B));
  hipLaunchKernelGGL(unique_table_init_kernel, dim3((unsigned)((slots + 255) / 256)), dim3(256), 0, s,
                     (unsigned long long*)workspace, slots, cnt);
  hipLaunchKernelGGL(unique_insert_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, s, ids, B, (int)L, K,
                     (unsigned long long*)workspace, slots - 1, cnt);
  hipLaunchKernelGGL(unique_fraction_kernel, dim3(1), dim3(1), 0, s, cnt, out_count, out_frac, inv_b);
  RQ_LAUNCH_CHECK("rq_unique_fraction");
  return 0;
}

}  // extern "C"
