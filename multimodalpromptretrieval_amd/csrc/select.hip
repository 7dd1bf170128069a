// select.hip — the final top-k of a scan: per query, the best k of n_cand (key, id) candidate
// lists (scan_kernel / scan_small_kernel / scan_mm_kernel block lists, the coarse scan's lane
// lists, a sharded search's per-shard lists).  Its own translation unit: inside scan.hip the
// k-round kernel below did not finish compiling under hipcc 7.2; alone it compiles in seconds for
// every list length but 16, which takes the 32 kernel).
#include <climits>
#include <cmath>
#include <cstdlib>

#include "kernels.h"
#include "topk_wave.h"

namespace mpr {
namespace {

__device__ __forceinline__ bool key_less(float ka, int64_t ia, float kb, int64_t ib) {
  return ka < kb || (ka == kb && ia < ib);
}
__device__ __forceinline__ uint32_t order_bits(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// Final selection: per query, best k of n_cand (key, id) candidates.  Thread-local sorted lists
// over a strided slice, then k rounds of a block-wide minimum over the lists' heads, each head one
// 64-bit word (key order bits, row id): the winner's list shifts.  (Replaces a pairwise tree
// merge through LDS: log2(NT) levels of K dependent steps.)  Row ids are < 2^31 (every scan
// keeps them in 32 bits); -0.0 keys count as +0.0, as the float compare of key_less does.
__device__ __forceinline__ uint64_t head_word(float key, int64_t id) {
  return id < 0 ? ~0ull : ((uint64_t)order_bits(key + 0.0f) << 32) | (uint32_t)id;
}
__device__ __forceinline__ float word_key(uint64_t w) {
  const uint32_t o = (uint32_t)(w >> 32);
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o);
}

template <int K, int NT>
__global__ __launch_bounds__(NT) void merge_kernel(const float* cand_key, const int64_t* cand_id,
                                                   int64_t n_cand, int k, int keys_are_values,
                                                   int metric, float* out_val, int64_t* out_id,
                                                   const int* gate) {
  if (gate && gate[blockIdx.x] == 0) return;  // coarse path fallback: flagged queries only
  constexpr int NW = NT / 64;
  __shared__ uint64_t wmin[2][NW];
  const int q = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* ck = cand_key + (int64_t)q * n_cand;
  const int64_t* ci = cand_id + (int64_t)q * n_cand;
  // keys_are_values && cosine: candidate values are similarities (descending) -> negate.
  const float sign = (keys_are_values && metric == 1) ? -1.f : 1.f;
  float bk[K];
  int64_t bi[K];
#pragma unroll
  for (int t = 0; t < K; ++t) {
    bk[t] = INFINITY;
    bi[t] = INT64_MAX;
  }
  for (int64_t c = tid; c < n_cand; c += NT) {
    const int64_t id = ci[c];
    if (id < 0) continue;
    float kk = sign * ck[c];
    int64_t ii = id;
    if (!key_less(kk, ii, bk[K - 1], bi[K - 1])) continue;
#pragma unroll
    for (int t = 0; t < K; ++t) {
      const bool sw = key_less(kk, ii, bk[t], bi[t]);
      const float tk = sw ? bk[t] : kk;
      const int64_t ti = sw ? bi[t] : ii;
      bk[t] = sw ? kk : bk[t];
      bi[t] = sw ? ii : bi[t];
      kk = tk;
      ii = ti;
    }
  }
  uint64_t w[K];
#pragma unroll
  for (int t = 0; t < K; ++t) w[t] = head_word(bk[t], bi[t] == INT64_MAX ? -1 : bi[t]);
  for (int r = 0; r < k; ++r) {
    uint64_t m = w[0];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const uint64_t o = __shfl_xor(m, off, 64);
      m = o < m ? o : m;
    }
    if (lane == 0) wmin[r & 1][wave] = m;
    __syncthreads();
    uint64_t g = wmin[r & 1][0];
#pragma unroll
    for (int v = 1; v < NW; ++v) g = wmin[r & 1][v] < g ? wmin[r & 1][v] : g;
    if (g != ~0ull && w[0] == g) {  // (key, id) words are unique: one winner
#pragma unroll
      for (int t = 0; t < K - 1; ++t) w[t] = w[t + 1];
      w[K - 1] = ~0ull;
    }
    if (tid == 0) {
      const bool none = g == ~0ull;
      const float kk = word_key(g);
      out_val[(int64_t)q * k + r] = none ? NAN : (metric == 1 ? -kk : kk);
      out_id[(int64_t)q * k + r] = none ? -1 : (int64_t)(uint32_t)g;
    }
  }
}


// Short candidate lists (a sharded search's W x k per query, <= MW_MAX): one WAVE per query, four
// queries per block, so the k rounds are wave shuffles with no block barrier (the block kernel
// above spends a barrier per round).  Same (key, id) order, same outputs.
constexpr int MW_MAX = 512;
// PK: the candidates are a sharded search's all_gathered per-shard top-k as they arrive, packed
// (dist, id) float64 pairs [W shards][Bp query slots][kc][2] (distributed.py); query q's list is
// shard-major, candidate c = (shard c / kc, rank c % kc) — the order of the unpacked [b, W kc]
// lists, so the outputs are the unpacked merge's.
// pack_out (gated merges only): the merged queries' final (dist, id) also as float64 pairs
// [b][k][2]; the coarse re-rank wrote every query's, so the sharded search's exchange needs no
// separate pack launch (mpr_sharded_search_all).
template <int K, bool PK = false>
__global__ __launch_bounds__(256) void merge_wave_kernel(const float* cand_key,
                                                         const int64_t* cand_id, int64_t n_cand,
                                                         int b, int k, int keys_are_values,
                                                         int metric, float* out_val,
                                                         int64_t* out_id, const int* gate,
                                                         const double* packed = nullptr,
                                                         int Bp = 0, int kc = 1,
                                                         double2* pack_out = nullptr) {
  const int q = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= b) return;  // wave-uniform
  if (gate && gate[q] == 0) return;  // the re-rank's result stands (its packed pair too)
  const float sign = (keys_are_values && metric == 1) ? -1.f : 1.f;
  if constexpr (PK) {
    tkw::merge_query<K>(
        [&](int64_t c, float& key, int64_t& id) {
          const double* e = packed + (((c / kc) * (int64_t)Bp + q) * kc + c % kc) * 2;
          key = sign * (float)e[0];
          id = (int64_t)e[1];
        },
        n_cand, k, metric, q, out_val, out_id, pack_out);
  } else {
    const float* ck = cand_key + (int64_t)q * n_cand;
    const int64_t* ci = cand_id + (int64_t)q * n_cand;
    tkw::merge_query<K>(
        [&](int64_t c, float& key, int64_t& id) {
          key = sign * ck[c];
          id = ci[c];
        },
        n_cand, k, metric, q, out_val, out_id, pack_out);
  }
}


// Large k (> 64; the reference slices any retrieval_k out of a full argsort,
// dataset/VQAFeatureDataset.py:194-197): per query one block finds the k smallest 64-bit words
// (key order bits, id) — unique, so the set is exact with ties going to the lowest id — by a
// radix select over 8 passes of 8-bit digits (MSB first, LDS histograms), gathers them into LDS
// and sorts them there (bitonic, padded to a power of two).  ids == null: candidate c of the row
// has id c (a full score row), output ids + id_offset.  Ids are < 2^32 (n < 2^31 everywhere).
constexpr int SL_NT = 1024;

__device__ __forceinline__ uint64_t sl_word(float key, uint32_t id) {
  return ((uint64_t)order_bits(key + 0.0f) << 32) | id;
}

__global__ __launch_bounds__(SL_NT) void select_large_kernel(const float* keys,
                                                             const int64_t* ids, int64_t n,
                                                             int k, int P, float sign,
                                                             int64_t id_offset, float* out_val,
                                                             int64_t* out_id) {
  extern __shared__ __attribute__((aligned(16))) uint64_t sl_lds[];
  uint64_t* items = sl_lds;                                 // [P]
  uint32_t* hist = reinterpret_cast<uint32_t*>(sl_lds + P);  // [256]
  __shared__ uint64_t s_prefix;
  __shared__ uint32_t s_rem, s_count, s_all;
  const int q = blockIdx.x, tid = threadIdx.x;
  const float* kr = keys + (int64_t)q * n;
  const int64_t* ir = ids ? ids + (int64_t)q * n : nullptr;
  auto word_at = [&](int64_t c, bool& ok) -> uint64_t {
    if (ir) {
      const int64_t id = ir[c];
      ok = id >= 0;
      return sl_word(sign * kr[c], (uint32_t)id);
    }
    ok = true;
    return sl_word(sign * kr[c], (uint32_t)c);
  };
  if (tid == 0) {
    s_prefix = 0;
    s_rem = (uint32_t)k;
    s_all = 0;
  }
  uint64_t mask = 0;
  for (int pass = 7; pass >= 0; --pass) {
    __syncthreads();
    if (s_all) break;  // fewer than k valid candidates (ids < 0 dropped): every one is kept
    for (int i = tid; i < 256; i += SL_NT) hist[i] = 0;
    __syncthreads();
    const uint64_t prefix = s_prefix;
    const int sh = pass * 8;
    for (int64_t c = tid; c < n; c += SL_NT) {
      bool ok;
      const uint64_t w = word_at(c, ok);
      if (ok && (w & mask) == prefix) atomicAdd(&hist[(w >> sh) & 255], 1u);
    }
    __syncthreads();
    if (tid == 0) {  // the digit whose cumulative count reaches the rank still to place
      uint32_t rem = s_rem, cum = 0;
      int dgt = 0;
      for (; dgt < 256; ++dgt) {
        if (cum + hist[dgt] >= rem) break;
        cum += hist[dgt];
      }
      if (dgt == 256) {  // only reachable in the first pass: fewer than k valid words in all
        s_all = 1;
        s_prefix = ~0ull;
      } else {
        s_rem = rem - cum;
        s_prefix = prefix | ((uint64_t)dgt << sh);
      }
    }
    mask |= (uint64_t)255 << sh;
    __syncthreads();
  }
  const uint64_t thr = s_prefix;  // the k-th smallest word
  if (tid == 0) s_count = 0;
  for (int i = tid; i < P; i += SL_NT) items[i] = ~0ull;
  __syncthreads();
  for (int64_t c = tid; c < n; c += SL_NT) {
    bool ok;
    const uint64_t w = word_at(c, ok);
    if (ok && w <= thr) items[atomicAdd(&s_count, 1u)] = w;
  }
  __syncthreads();
  // bitonic sort of the P words (ascending)
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < P / 2; i += SL_NT) {
        const int lo = 2 * i - (i & (stride - 1));
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const uint64_t a = items[lo], b = items[hi];
        if ((a > b) == up) {
          items[lo] = b;
          items[hi] = a;
        }
      }
      __syncthreads();
    }
  }
  for (int t = tid; t < k; t += SL_NT) {  // ranks past the valid candidates: NaN / -1 (as merge)
    const uint64_t w = items[t];
    const bool none = w == ~0ull;
    out_val[(int64_t)q * k + t] = none ? NAN : sign * word_key(w);
    out_id[(int64_t)q * k + t] = none ? -1 : (int64_t)(uint32_t)w + (ir ? 0 : id_offset);
  }
}

template <int K>
int launch_merge(const float* ck, const int64_t* ci, int b, int64_t n_cand, int k,
                 int keys_are_values, int metric, float* od, int64_t* oi, hipStream_t s,
                 const int* gate, double* pack_out) {
  if constexpr (K <= 8) {
    if (n_cand <= MW_MAX && !getenv("MPR_MERGE_BLOCK")) {
      hipLaunchKernelGGL((merge_wave_kernel<K>), dim3((unsigned)((b + 3) / 4)), dim3(256), 0, s,
                         ck, ci, n_cand, b, k, keys_are_values, metric, od, oi, gate, nullptr, 0,
                         1, reinterpret_cast<double2*>(pack_out));
      MPR_LAUNCHED();
      return MPR_OK;
    }
  }
  MPR_REQUIRE(!pack_out, "merge: packed output on the wave merge only (k <= 8, <= %d lists)",
              MW_MAX);
  constexpr int NT = K >= 32 ? 128 : 256;
  hipLaunchKernelGGL((merge_kernel<K, NT>), dim3(b), dim3(NT), 0, s, ck, ci, n_cand, k,
                     keys_are_values, metric, od, oi, gate);
  MPR_LAUNCHED();
  return MPR_OK;
}

// rows of kk (dist, id) -> rows of k >= kk float64 pairs, ranks past kk empty (NaN, -1): a
// shard holding fewer than k rows
__global__ __launch_bounds__(256) void topk_pack_kernel(const float* __restrict__ d,
                                                        const int64_t* __restrict__ ids, int64_t n,
                                                        int kk, int k, double2* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int64_t r = i / k;
  const int j = (int)(i - r * k);
  out[i] = j < kk ? make_double2((double)d[r * kk + j], (double)ids[r * kk + j])
                  : make_double2((double)NAN, -1.0);
}

template <int K>
int launch_merge_packed(const double* packed, int W, int Bp, int b, int kc, int k, int metric,
                        float* od, int64_t* oi, hipStream_t s) {
  hipLaunchKernelGGL((merge_wave_kernel<K, true>), dim3((unsigned)((b + 3) / 4)), dim3(256), 0, s,
                     nullptr, nullptr, (int64_t)W * kc, b, k, /*keys_are_values=*/1, metric, od,
                     oi, nullptr, packed, Bp, kc);
  MPR_LAUNCHED();
  return MPR_OK;
}

}  // namespace

// (dist fp32, id int64) [n] -> float64 pairs [n][2] (ids < 2^53 and fp32 values are exact)
int topk_pack(const float* d, const int64_t* ids, int64_t n, double* out, hipStream_t s, int kk,
              int k) {
  if (n == 0) return MPR_OK;
  MPR_REQUIRE(kk >= 1 && k >= kk && n % k == 0, "topk_pack: kk=%d k=%d n=%lld", kk, k,
              (long long)n);
  hipLaunchKernelGGL(topk_pack_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, s, d, ids, n,
                     kk, k, reinterpret_cast<double2*>(out));
  MPR_LAUNCHED();
  return MPR_OK;
}

int merge_packed(const double* packed, int W, int Bp, int b, int kc, int k, int metric,
                 float* od, int64_t* oi, hipStream_t s) {
  MPR_REQUIRE(W >= 1 && Bp >= b && b >= 0 && kc >= 1 && k >= 1 && k <= 64 && k <= W * kc &&
                  (int64_t)W * kc <= MW_MAX,
              "merge_packed: W=%d Bp=%d b=%d kc=%d k=%d (k <= 64, W kc <= %d)", W, Bp, b, kc, k,
              MW_MAX);
  if (b == 0) return MPR_OK;
  // a lane's sorted list never needs more than the candidates it sees: W kc <= 512 over 64 lanes
  // is <= 8 each, so lists of min(next_pow2(k), 8) give the same result at any k
  int c = 1;
  while (c < k && c < 8) c <<= 1;
  switch (c) {
    case 1: return launch_merge_packed<1>(packed, W, Bp, b, kc, k, metric, od, oi, s);
    case 2: return launch_merge_packed<2>(packed, W, Bp, b, kc, k, metric, od, oi, s);
    case 4: return launch_merge_packed<4>(packed, W, Bp, b, kc, k, metric, od, oi, s);
    default: return launch_merge_packed<8>(packed, W, Bp, b, kc, k, metric, od, oi, s);
  }
}

int merge_lists(const float* ck, const int64_t* ci, int b, int64_t n_cand, int k,
                int keys_are_values, int metric, float* od, int64_t* oi, hipStream_t s,
                const int* gate, double* pack_out) {
  MPR_REQUIRE(!pack_out || gate, "merge: packed output only on a gated merge");
  int c = 1;
  while (c < k) c <<= 1;
  if (c == 16) c = 32;  // merge_kernel<16, *> hangs hipcc 7.2's backend (every other K compiles)
#define MPR_MG(K) \
  case K: return launch_merge<K>(ck, ci, b, n_cand, k, keys_are_values, metric, od, oi, s, gate, \
                                 pack_out);
  switch (c) {
    MPR_MG(1) MPR_MG(2) MPR_MG(4) MPR_MG(8) MPR_MG(32) MPR_MG(64)
  }
#undef MPR_MG
  MPR_REQUIRE(!gate, "top-k: gated merge of k=%d > 64", k);
  const float sign = (keys_are_values && metric == 1) ? -1.f : 1.f;
  return select_large(ck, ci, b, n_cand, k, sign, 0, od, oi, s);
}

int select_large(const float* keys, const int64_t* ids, int b, int64_t n, int k, float sign,
                 int64_t id_offset, float* od, int64_t* oi, hipStream_t s) {
  MPR_REQUIRE(k >= 1 && k <= SELECT_MAX_K && k <= n, "top-k: k=%d (1..%d, <= %lld candidates)",
              k, SELECT_MAX_K, (long long)n);
  MPR_REQUIRE(n < ((int64_t)1 << 31), "top-k: %lld candidates per row", (long long)n);
  if (b == 0) return MPR_OK;
  int P = 1;
  while (P < k) P <<= 1;
  const size_t lds = (size_t)P * 8 + 256 * 4;
  if (lds > 64 * 1024)
    MPR_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(select_large_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(select_large_kernel, dim3((unsigned)b), dim3(SL_NT), lds, s, keys, ids, n, k,
                     P, sign, id_offset, od, oi);
  MPR_LAUNCHED();
  return MPR_OK;
}

}  // namespace mpr
