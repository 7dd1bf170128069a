// topk_wave.h — the best k of one query's short candidate list (<= 512) by ONE wave: lane-local
// sorted lists of K 64-bit words (key order bits, row id) over a strided slice, then k rounds of
// a wave minimum over the heads (shuffles, no block barrier).  The body of select.hip's
// merge_wave_kernel, shared with scan.hip's gated exact fallback, whose last block per query tile
// merges that tile's flagged queries itself (no separate merge launch).
#pragma once

#include "kernels.h"

namespace mpr {
namespace tkw {

__device__ __forceinline__ uint32_t order_bits(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
// ids < 0 never rank; -0.0 keys count as +0.0 (as key_less's float compare)
__device__ __forceinline__ uint64_t head_word(float key, int64_t id) {
  return id < 0 ? ~0ull : ((uint64_t)order_bits(key + 0.0f) << 32) | (uint32_t)id;
}
__device__ __forceinline__ float word_key(uint64_t w) {
  const uint32_t o = (uint32_t)(w >> 32);
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o);
}

// Query q's best k of n_cand candidates, load(c) -> (key, id) giving candidate c (keys already
// signed so that smaller ranks first; NaN keys never rank).  Outputs value (metric 1: -key),
// id, and the float64 pair when pack_out; ranks past the valid candidates get (NaN, -1).  Every
// lane of the calling wave takes part; k <= 64.
template <int K, class Load>
__device__ __forceinline__ void merge_query(Load load, int64_t n_cand, int k, int metric, int q,
                                            float* out_val, int64_t* out_id, double2* pack_out) {
  const int lane = threadIdx.x & 63;
  uint64_t w[K];
#pragma unroll
  for (int t = 0; t < K; ++t) w[t] = ~0ull;
  for (int64_t c = lane; c < n_cand; c += 64) {
    float kk;
    int64_t id;
    load(c, kk, id);
    uint64_t v = head_word(kk, kk == kk ? id : -1);
#pragma unroll
    for (int t = 0; t < K; ++t) {  // sorted insert (words are unique per valid candidate)
      const uint64_t lo = v < w[t] ? v : w[t], hi = v < w[t] ? w[t] : v;
      w[t] = lo;
      v = hi;
    }
  }
  for (int r = 0; r < k; ++r) {
    uint64_t m = w[0];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const uint64_t o = __shfl_xor(m, off, 64);
      m = o < m ? o : m;
    }
    if (m != ~0ull && w[0] == m) {
#pragma unroll
      for (int t = 0; t < K - 1; ++t) w[t] = w[t + 1];
      w[K - 1] = ~0ull;
    }
    if (lane == 0) {
      const bool none = m == ~0ull;
      const float kk = word_key(m);
      const float v = none ? NAN : (metric == 1 ? -kk : kk);
      const int64_t id = none ? -1 : (int64_t)(uint32_t)m;
      out_val[(int64_t)q * k + r] = v;
      out_id[(int64_t)q * k + r] = id;
      if (pack_out) pack_out[(int64_t)q * k + r] = make_double2((double)v, (double)id);
    }
  }
}

}  // namespace tkw
}  // namespace mpr
