// scan.hip — exhaustive nearest-neighbour scan with fused top-k over the retrieval index.
//
// Replaces dataset/VQAFeatureDataset.py:192-197:
//     dist_matrix = torch.cdist(combined, retrieval_embeddings)          # mm path, rows > 25
//     top = torch.argsort(dist_matrix, axis=1)[:, s:s+k]
// and utils.py:57-62 cosine_similarity for the cosine metric.
//
// Layout: index rows X [n, d] fp32 row-major (4 KiB per row at d = 1024), squared row norms
// precomputed once at index creation.  A block = 4 waves; each wave streams 16-row tiles of X
// straight from HBM into registers (each lane one float4 of its row per 16 columns: every row is
// read as 64-byte contiguous segments, 16 rows per wave-instruction) and multiplies them against
// a group of 16 queries held in LDS with v_mfma_f32_16x16x4_f32: one MFMA consumes 256 B of index
// per 2048 FLOP, so at batch 16 the tile math runs ~3x faster than HBM delivers and the scan is
// HBM-bound.  The 16x16 distance tile lands as 4 rows x 1 query per lane; each lane keeps a
// sorted register list of its best K (key, row) and the block merges its 16 lists per query in
// LDS, so only K candidates per (query, block) leave the kernel; topk_merge_kernel finishes.
//
// Ordering contract (ids parity with the reference): keys are the reported values — L2 distance
// sqrt(max(|q|^2 + |x|^2 - 2 q.x, 0)) (the cdist mm-path formula) or minus the cosine similarity —
// sorted ascending, exact ties broken by the lowest row id (argsort(stable=True) semantics).
#include <algorithm>
#include <cfloat>
#include <climits>
#include <cstdlib>
#include <vector>

#include "kernels.h"
#include "topk_wave.h"

namespace mpr {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int QG = 16;  // queries per group (MFMA N)
constexpr float COS_EPS = 1e-8f;

__device__ __forceinline__ bool key_less(float ka, int64_t ia, float kb, int64_t ib) {
  return ka < kb || (ka == kb && ia < ib);
}

// Wave minimum by DPP row operations (a few cycles each, where a __shfl_xor butterfly waits on
// six LDS-unit permutes): quad xor 1 and xor 2, half-row and row mirrors leave each row's minimum
// in all its lanes; row_bcast15 / row_bcast31 fold rows 0-2 into row 3, whose lane 63 is read
// out (wave-uniform result).  The whole wave must be active.  Min is order-free, so this equals
// the butterfly's result (for the non-negative or infinite keys it is used on).
#define MPR_DPP_MIN(v, CTRL, ROWS)                                                               \
  v = fminf(v, __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), \
                                                          CTRL, ROWS, 0xF, false)))
__device__ __forceinline__ float wave_min(float v) {
  MPR_DPP_MIN(v, 0xB1, 0xF);   // quad_perm [1, 0, 3, 2]
  MPR_DPP_MIN(v, 0x4E, 0xF);   // quad_perm [2, 3, 0, 1]
  MPR_DPP_MIN(v, 0x141, 0xF);  // row_half_mirror
  MPR_DPP_MIN(v, 0x140, 0xF);  // row_mirror
  MPR_DPP_MIN(v, 0x142, 0xA);  // row_bcast15 -> rows 1, 3
  MPR_DPP_MIN(v, 0x143, 0xC);  // row_bcast31 -> rows 2, 3
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
#undef MPR_DPP_MIN

__device__ __forceinline__ float score_key(int metric, float dot, float qn, float xn) {
  if (metric == 0) return sqrtf(fmaxf(qn + xn - 2.0f * dot, 0.0f));
  return -(dot / fmaxf(sqrtf(qn) * sqrtf(xn), COS_EPS));
}

// Dynamic LDS: Qs [16][d+4] during the scan, reused for the per-block merge afterwards.
template <int K, bool ALL>
__global__ __launch_bounds__(256) void scan_kernel(const float* __restrict__ X,
                                                   const float* __restrict__ xnorm, int64_t n,
                                                   int d, int64_t row_offset, int metric,
                                                   const float* __restrict__ Q, int b,
                                                   float* cand_key, int64_t* cand_id,
                                                   float* scores) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int ldq = d + 4;
  float* Qs = lds;
  __shared__ float qn_s[QG];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR)
  const int g = blockIdx.y, qbase = g * QG;
  // Stage the query group (zero rows past b).
  for (int idx = tid; idx < QG * (d / 4); idx += 256) {
    const int r = idx / (d / 4), c4 = (idx % (d / 4)) * 4, q = qbase + r;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (q < b) v = *reinterpret_cast<const f32x4*>(Q + (int64_t)q * d + c4);
    *reinterpret_cast<f32x4*>(Qs + r * ldq + c4) = v;
  }
  __syncthreads();
  // Query squared norms: 16 threads per query.
  {
    const int r = tid >> 4, sub = tid & 15;
    float ss = 0.f;
    for (int c = sub; c < d; c += 16) {
      const float v = Qs[r * ldq + c];
      ss += v * v;
    }
#pragma unroll
    for (int off = 8; off >= 1; off >>= 1) ss += __shfl_xor(ss, off, 64);
    if (sub == 0) qn_s[r] = ss;
  }
  __syncthreads();

  const int i = lane & 15, h = lane >> 4;
  const int j = lane & 15;  // this lane's query in the output tile
  const bool qok = qbase + j < b;
  const float qn = qn_s[j];
  float bk[K];
  int bi[K];
#pragma unroll
  for (int t = 0; t < K; ++t) {
    bk[t] = INFINITY;
    bi[t] = INT_MAX;
  }

  const int64_t ntiles = (n + 15) / 16;
  const float* qrow = Qs + i * ldq + h * 4;
  for (int64_t tile = (int64_t)blockIdx.x * 4 + wave; tile < ntiles;
       tile += (int64_t)gridDim.x * 4) {
    const int64_t row = tile * 16 + i;
    const bool rok = row < n;
    const float* xp = X + (rok ? row : 0) * (int64_t)d + h * 4;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    constexpr int U = 8;
    int c = 0;
    const int nc = d / 16;
    for (; c + U <= nc; c += U) {
      f32x4 xv[U];
#pragma unroll
      for (int u = 0; u < U; ++u)
        xv[u] = rok ? *reinterpret_cast<const f32x4*>(xp + (c + u) * 16)
                    : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const f32x4 qv = *reinterpret_cast<const f32x4*>(qrow + (c + u) * 16);
#pragma unroll
        for (int e = 0; e < 4; ++e)
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[u][e], qv[e], acc, 0, 0, 0);
      }
    }
    for (; c < nc; ++c) {
      const f32x4 xv = rok ? *reinterpret_cast<const f32x4*>(xp + c * 16)
                           : f32x4{0.f, 0.f, 0.f, 0.f};
      const f32x4 qv = *reinterpret_cast<const f32x4*>(qrow + c * 16);
#pragma unroll
      for (int e = 0; e < 4; ++e)
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[e], qv[e], acc, 0, 0, 0);
    }
    // acc[r] = dot(X[tile*16 + h*4 + r], Q[qbase + j])
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t row2 = tile * 16 + h * 4 + r;
      if (row2 >= n || !qok) continue;
      const float key = score_key(metric, acc[r], qn, xnorm[row2]);
      if (ALL) {
        scores[(int64_t)(qbase + j) * n + row2] = metric == 0 ? key : -key;
      } else if (key < bk[K - 1]) {
        float ck = key;
        int ci = (int)row2;
#pragma unroll
        for (int t = 0; t < K; ++t) {
          const bool sw = ck < bk[t];
          const float tk = sw ? bk[t] : ck;
          const int ti = sw ? bi[t] : ci;
          bk[t] = sw ? ck : bk[t];
          bi[t] = sw ? ci : bi[t];
          ck = tk;
          ci = ti;
        }
      }
    }
  }
  if (ALL) return;

  // Block merge: 16 sorted lists (4 waves x 4 lane-quarters) per query -> best K.
  __syncthreads();  // Qs no longer needed
  float* Lk = lds;                                            // [QG][16][K]
  int* Li = reinterpret_cast<int*>(lds + QG * 16 * K);        // [QG][16][K]
  {
    const int list = wave * 4 + h;
#pragma unroll
    for (int t = 0; t < K; ++t) {
      Lk[(j * 16 + list) * K + t] = bk[t];
      Li[(j * 16 + list) * K + t] = bi[t];
    }
  }
  __syncthreads();
  if (tid < QG && qbase + tid < b) {
    const int q = tid;
    int head[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) head[s] = 0;
    float* ok = cand_key + ((int64_t)(qbase + q) * gridDim.x + blockIdx.x) * K;
    int64_t* oi = cand_id + ((int64_t)(qbase + q) * gridDim.x + blockIdx.x) * K;
    for (int t = 0; t < K; ++t) {
      float best = INFINITY;
      int bidx = INT_MAX, bs = 0;
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        if (head[s] < K) {
          const float kk = Lk[(q * 16 + s) * K + head[s]];
          const int ii = Li[(q * 16 + s) * K + head[s]];
          if (kk < best || (kk == best && ii < bidx)) {
            best = kk;
            bidx = ii;
            bs = s;
          }
        }
      }
#pragma unroll
      for (int s = 0; s < 16; ++s) head[s] += (s == bs) ? 1 : 0;
      ok[t] = best;
      oi[t] = bidx == INT_MAX ? -1 : (int64_t)bidx + row_offset;
    }
  }
}

__device__ __forceinline__ uint32_t order_bits(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

constexpr int SS_TT = 1;  // 16-row tiles per small-scan block (2 and 4 measured slower at C2)
// ---- small-index scan (the C2 regime: n of a few thousand rows, <= 16 queries per group) -------
// scan_kernel gives each wave whole 16-row tiles, so at n = 6,500 it launches ~100 blocks and each
// wave walks its 4 KiB rows in d/128 dependent load rounds.  Here a block is ONE 16-row tile x 16
// queries and its 4 waves split d: every load of the block (rows and query fragments, both read
// straight from global memory, the queries L2-resident) is in flight at once, the 4 partial dot
// tiles and query norms are summed through LDS, and the block emits its best min(K, 16) rows per
// query (K-list padded with empty slots).
template <int K, int CH, int TT>  // CH = d / 64 chunks of 16 columns per wave; TT tiles a block
__global__ __launch_bounds__(256) void scan_small_kernel(const float* __restrict__ X,
                                                         const float* __restrict__ xnorm,
                                                         int64_t n, int64_t row_offset,
                                                         int metric, const float* __restrict__ Q,
                                                         int b, float* cand_key,
                                                         int64_t* cand_id) {
  constexpr int d = 64 * CH, R = 16 * TT;  // R = rows per block
  __shared__ f32x4 red[TT][4][64];
  __shared__ float qss[4][QG];
  __shared__ float lk[QG][R];
  __shared__ int li[QG][R];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i = lane & 15, h = lane >> 4;
  const int64_t row0 = (int64_t)blockIdx.x * R;
  const int qbase = blockIdx.y * QG;
  const int c0 = wave * CH;
  const bool qok_i = qbase + i < b;
  const float* qp = Q + (int64_t)(qok_i ? qbase + i : 0) * d + c0 * 16 + h * 4;
  f32x4 xv[TT][CH], qv[CH];
#pragma unroll
  for (int u = 0; u < CH; ++u) qv[u] = *reinterpret_cast<const f32x4*>(qp + u * 16);
#pragma unroll
  for (int t = 0; t < TT; ++t) {
    const int64_t row = row0 + t * 16 + i;
    const float* xp = X + (row < n ? row : n - 1) * (int64_t)d + c0 * 16 + h * 4;
#pragma unroll
    for (int u = 0; u < CH; ++u) xv[t][u] = *reinterpret_cast<const f32x4*>(xp + u * 16);
  }
  // the epilogue's row norms (wave 0: rows t*16 + h*4 .. +3), fetched with the rest
  float xnr[TT][4];
#pragma unroll
  for (int t = 0; t < TT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t row2 = row0 + t * 16 + h * 4 + r;
      xnr[t][r] = xnorm[row2 < n ? row2 : n - 1];
    }
  __builtin_amdgcn_sched_barrier(0);  // every load in flight before the first wait
  float ss = 0.f;
  const float qscale = qok_i ? 1.f : 0.f;  // rows past b: zero query (no select on the loads)
#pragma unroll
  for (int u = 0; u < CH; ++u)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      qv[u][e] *= qscale;
      ss += qv[u][e] * qv[u][e];
    }
#pragma unroll
  for (int t = 0; t < TT; ++t) {
    // four independent accumulation chains (one per k of the 4-deep MFMA step)
    f32x4 acc4[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) acc4[e] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < CH; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        acc4[e] = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[t][u][e], qv[u][e], acc4[e], 0, 0, 0);
    red[t][wave][lane] = (acc4[0] + acc4[1]) + (acc4[2] + acc4[3]);
  }
  ss += __shfl_xor(ss, 16, 64);
  ss += __shfl_xor(ss, 32, 64);
  if (h == 0) qss[wave][i] = ss;
  __syncthreads();
  if (wave == 0) {
    const int j = lane & 15;  // this lane's query (D column); rows h*4 .. h*4+3 of each tile
    const float qn = ((qss[0][j] + qss[1][j]) + qss[2][j]) + qss[3][j];
#pragma unroll
    for (int t = 0; t < TT; ++t) {
      const f32x4 a = ((red[t][0][lane] + red[t][1][lane]) + red[t][2][lane]) + red[t][3][lane];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row2 = row0 + t * 16 + h * 4 + r;
        const bool ok = row2 < n && qbase + j < b;
        lk[j][t * 16 + h * 4 + r] = ok ? score_key(metric, a[r], qn, xnr[t][r]) : INFINITY;
        li[j][t * 16 + h * 4 + r] = ok ? (int)row2 : INT_MAX;
      }
    }
  }
  __syncthreads();
  // thread (query q, slots t): rank of row t among the block's R by (key, row, slot); best
  // min(K, R)
  const int q = tid >> 4;
  if (qbase + q < b) {
    float* ok = cand_key + ((int64_t)(qbase + q) * gridDim.x + blockIdx.x) * K;
    int64_t* oi = cand_id + ((int64_t)(qbase + q) * gridDim.x + blockIdx.x) * K;
    for (int t = tid & 15; t < R; t += 16) {
      const float kk = lk[q][t];
      const int ii = li[q][t];
      // (key, row, slot) order as one 64-bit word per slot (empty slots rank by slot, so every
      // rank is written); branch-free count
      const uint64_t ct = ((uint64_t)order_bits(kk) << 32) | (uint32_t)ii;
      int rank = 0;
#pragma unroll
      for (int u = 0; u < R; ++u) {
        const uint64_t cu = ((uint64_t)order_bits(lk[q][u]) << 32) | (uint32_t)li[q][u];
        rank += (int)((cu < ct) | ((cu == ct) & (u < t)));
      }
      if (rank < K) {
        ok[rank] = kk;
        oi[rank] = ii == INT_MAX ? -1 : (int64_t)ii + row_offset;
      }
    }
    for (int e = R + (tid & 15); e < K; e += 16) {  // K > R: the list's empty tail
      ok[e] = INFINITY;
      oi[e] = -1;
    }
  }
}

// ---- large-batch scan (b >= 64): the similarity GEMM with a top-k epilogue ------------------
// At b = 256 the scan is MFMA-bound in fp32 (2 FLOP per index byte per query),
// and the 16-query kernel above would stream the index once per query group.  Here a block owns
// a 64-query tile (Q rows, L2-resident) and a strided set of 64-row index tiles; each k-step stages
// a 64 x 32 slice of X and of Q through LDS (register prefetch SM_D tiles ahead, two LDS stages:
// the tiled-GEMM pipeline of gemm.hip) into v_mfma_f32_32x32x2_f32 (4 waves, 2 x 2 of 32x32).
// At the end of each row tile the accumulators become keys in registers (row norms are summed
// from the same staged fragments) and enter per-lane sorted top-K lists; scores never reach HBM.
// Blocks of one row-tile set are adjacent after an XCD-aware remap, so they share an XCD's L2
// and the index is fetched from HBM about once.  Keys, order and ties as scan_kernel.
constexpr int SM_B = 64, SM_BK = 32, SM_D = 2, SM_LDK = SM_BK + 4;
constexpr int SM_STAGE = 2 * SM_B * SM_LDK;  // floats: X rows then Q rows

template <int K>
__global__ __launch_bounds__(256) void scan_mm_kernel(const float* __restrict__ X, int64_t n,
                                                      int d, int64_t row_offset, int metric,
                                                      const float* __restrict__ Q,
                                                      const float* __restrict__ qnorm, int b,
                                                      int nqt, int RB, float* cand_key,
                                                      int64_t* cand_id, const int* gate,
                                                      int* tile_cnt = nullptr, int k = 0,
                                                      float* out_dist = nullptr,
                                                      int64_t* out_id = nullptr,
                                                      double2* pack_out = nullptr) {
  __shared__ __attribute__((aligned(16))) float smem[2 * SM_STAGE];
  constexpr int KQ = SM_BK / 4, LA = SM_B * KQ / 256;  // float4 per thread and operand: 2
  int qt, rb;
  {
    const int total = gridDim.x, hw = blockIdx.x;
    const int xcd = hw & 7, slot = hw >> 3, q8 = total >> 3, r8 = total & 7;
    const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
    qt = t % nqt;
    rb = t / nqt;
  }
  if (gate) {  // the coarse path's exact fallback: only query tiles holding a flagged query run
    // (one vector load of the tile's 64 flags per wave and a ballot: a scalar loop over them
    // waited on 64 dependent loads, ~5 us for a grid that does nothing)
    const int qf = qt * SM_B + (int)(threadIdx.x & 63);
    if (__ballot(qf < b && gate[qf] != 0) == 0) return;
  }
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int li = lane & 31, lh = lane >> 5;
  const int64_t ntile = (n + SM_B - 1) / SM_B;
  const int ntb = (int)((ntile - rb + RB - 1) / RB);  // row tiles of this block
  const int KS = (d + SM_BK - 1) / SM_BK;
  const int S = ntb * KS, Sr = (S + SM_D - 1) / SM_D * SM_D;
  const int q0 = qt * SM_B;

  f32x4 ra[SM_D][LA], rq[SM_D][LA];
  bool oka[SM_D][LA], okq[SM_D][LA];
  auto gload = [&](int j, int step) {
    const int tt = step / KS, ks = step - tt * KS;
    const int64_t row0 = (int64_t)(rb + (int64_t)tt * RB) * SM_B;
    const int k0 = ks * SM_BK;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int idx = tid + i * 256, r = idx / KQ, c = k0 + (idx % KQ) * 4;
      const int64_t row = row0 + r;
      oka[j][i] = row < n && c < d && tt < ntb;
      ra[j][i] = *reinterpret_cast<const f32x4*>(X + (row < n ? row : n - 1) * (int64_t)d +
                                                 min(c, d - 4));
      const int q = q0 + r;
      okq[j][i] = q < b && c < d;
      rq[j][i] = *reinterpret_cast<const f32x4*>(Q + (int64_t)min(q, b - 1) * d + min(c, d - 4));
    }
  };
  auto swrite = [&](int st, int j) {
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
    float* base = smem + st * SM_STAGE;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int idx = tid + i * 256, r = idx / KQ, c4 = (idx % KQ) * 4;
      *reinterpret_cast<f32x4*>(base + r * SM_LDK + c4) = oka[j][i] ? ra[j][i] : z;
      *reinterpret_cast<f32x4*>(base + (SM_B + r) * SM_LDK + c4) = okq[j][i] ? rq[j][i] : z;
    }
  };
  // fragments: lane (li, lh) holds row li's k = 16 lh .. 16 lh + 15 of the tile (as gemm.hip)
  f32x4 fa[4], fb[4], na[4], nb[4];
  auto sread = [&](int st, f32x4(&xa)[4], f32x4(&xb)[4]) {
    const float* base = smem + st * SM_STAGE;
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      xa[s4] = *reinterpret_cast<const f32x4*>(base + (wm * 32 + li) * SM_LDK + lh * 16 + s4 * 4);
      xb[s4] = *reinterpret_cast<const f32x4*>(base + (SM_B + wn * 32 + li) * SM_LDK + lh * 16 +
                                               s4 * 4);
    }
  };

  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  float ssq = 0.f;  // this lane's half of row (wm*32 + li)'s squared norm, current tile
  const int jq = q0 + wn * 32 + li;  // this lane's query in the accumulator
  const float qn = qnorm[min(jq, b - 1)];
  float bk[K];
  int bi[K];
#pragma unroll
  for (int t = 0; t < K; ++t) {
    bk[t] = INFINITY;
    bi[t] = INT_MAX;
  }

  gload(0, 0);
  swrite(0, 0);
  gload(0, 1);
  swrite(1, 0);
#pragma unroll
  for (int j = 0; j < SM_D; ++j) gload(j, 2 + j);
  __syncthreads();
  sread(0, fa, fb);
  // Iteration 0 overwrites stage 0 (tile 2) while a slower wave may still be reading tile 0's
  // fragments from it here: every wave's reads must land first (this race made ~3% of grouped
  // launches nondeterministic before the barrier was added).
  __syncthreads();
  for (int s0 = 0; s0 < Sr; s0 += SM_D) {
#pragma unroll
    for (int j = 0; j < SM_D; ++j) {
      const int step = s0 + j, st = step & 1;
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[s4][c], fb[s4][c], acc, 0, 0, 0);
          ssq += fa[s4][c] * fa[s4][c];
        }
      sread(st ^ 1, na, nb);
      swrite(st, j);
      gload(j, step + 2 + SM_D);
      const int tt = step / KS;
      if (step - tt * KS == KS - 1 && tt < ntb) {  // last k-step of a row tile: keys -> top-K
        const float full = ssq + __shfl_xor(ssq, 32, 64);  // norm of row wm*32 + li
        const int64_t row0 = (int64_t)(rb + (int64_t)tt * RB) * SM_B + wm * 32;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rr = (r & 3) + 8 * (r >> 2) + 4 * lh;
          const float xn = __shfl(full, rr, 64);
          const int64_t row = row0 + rr;
          const float key = score_key(metric, acc[r], qn, xn);
          if (row < n && key < bk[K - 1]) {
            float ck = key;
            int ci = (int)row;
#pragma unroll
            for (int t = 0; t < K; ++t) {
              const bool sw = ck < bk[t];
              const float tk = sw ? bk[t] : ck;
              const int ti = sw ? bi[t] : ci;
              bk[t] = sw ? ck : bk[t];
              bi[t] = sw ? ci : bi[t];
              ck = tk;
              ci = ti;
            }
          }
          acc[r] = 0.f;
        }
        ssq = 0.f;
      }
      __syncthreads();
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        fa[s4] = na[s4];
        fb[s4] = nb[s4];
      }
    }
  }

  // Block merge: per query 4 sorted lists (lh x wm) -> best K, written as this block's
  // candidates (the stages are free: the loop ended on a barrier).
  float* Lk = smem;                                         // [64 q][4][K]
  int* Li = reinterpret_cast<int*>(smem + SM_B * 4 * K);    // [64 q][4][K]
  {
    const int ql = wn * 32 + li, list = wm * 2 + lh;
#pragma unroll
    for (int t = 0; t < K; ++t) {
      Lk[(ql * 4 + list) * K + t] = bk[t];
      Li[(ql * 4 + list) * K + t] = bi[t];
    }
  }
  __syncthreads();
  if (tid < SM_B && q0 + tid < b) {
    const int ql = tid;
    int head[4] = {0, 0, 0, 0};
    float* ok = cand_key + ((int64_t)(q0 + ql) * RB + rb) * K;
    int64_t* oi = cand_id + ((int64_t)(q0 + ql) * RB + rb) * K;
    for (int t = 0; t < K; ++t) {
      float best = INFINITY;
      int bidx = INT_MAX, bs = 0;
#pragma unroll
      for (int l = 0; l < 4; ++l) {
        if (head[l] < K) {
          const float kk = Lk[(ql * 4 + l) * K + head[l]];
          const int ii = Li[(ql * 4 + l) * K + head[l]];
          if (kk < best || (kk == best && ii < bidx)) {
            best = kk;
            bidx = ii;
            bs = l;
          }
        }
      }
#pragma unroll
      for (int l = 0; l < 4; ++l) head[l] += (l == bs) ? 1 : 0;
      ok[t] = best;
      oi[t] = bidx == INT_MAX ? -1 : (int64_t)bidx + row_offset;
    }
  }
  if (!tile_cnt) return;
  // The gated fallback's merge, folded in: the tile's last block to finish (agent-scope release
  // of every block's lists, counter, acquire) merges its flagged queries' RB x K candidates, one
  // wave per query (select.hip's wave merge).  Only flagged tiles get here, so the fences cost
  // nothing on the common path, which makes no merge launch at all.
  __shared__ int s_last;
  __threadfence();
  __syncthreads();
  if (tid == 0) s_last = atomicAdd(tile_cnt + qt, 1) == RB - 1;
  __syncthreads();
  if (!s_last) return;
  __threadfence();
  const int64_t nc = (int64_t)RB * K;
  for (int ql = wave; ql < SM_B; ql += 4) {
    const int q = q0 + ql;
    if (q >= b || gate[q] == 0) continue;  // wave-uniform
    const float* ck = cand_key + (int64_t)q * nc;
    const int64_t* ci = cand_id + (int64_t)q * nc;
    tkw::merge_query<K>(
        [&](int64_t c, float& key, int64_t& id) {
          key = ck[c];
          id = ci[c];
        },
        nc, k, metric, q, out_dist, out_id, pack_out);
  }
}

__global__ void qnorm_kernel(const float* Q, int b, int d, float* out) {
  const int q = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (q >= b) return;
  float s = 0.f;
  for (int c = lane; c < d; c += 64) s += Q[(int64_t)q * d + c] * Q[(int64_t)q * d + c];
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
  if (lane == 0) out[q] = s;
}

// ---- coarse bf16 scan + exact fp32 re-rank (b >= 64 queries, L2, d in {256, 512}) -------------
// At C5 (256 queries x 1,048,576 x 512) the exact scan is fp32-MFMA-bound (275 GFLOP, ~3.2 ms).
// Here the index is also kept as bf16 (rows rounded to nearest, 1 GiB) and scanned with
// v_mfma_f32_32x32x16_bf16 (16x the f32 MFMA rate, half the bytes: the HBM regime), keeping per
// query the best coarse keys s~ = |x|^2 - 2 q~.x~ (|x|^2 exact; |q|^2 is constant per query): a
// sorted list of CB_L per lane (its share of the rows), then the best CB_C over all lists; every
// one of those is re-scored exactly in fp32 and the best k returned.  The coarse error is
// bounded: with r = x~ - x and e = q~ - q the rounding residuals, |q~.x~ - q.x| <= |e| |x| +
// |q| |r| + |e| |r| (Cauchy-Schwarz), so with the index's max |x| and max |r| and the query's own
// |e|, |s~ - s| <= E = 2 (|e| X + |q| R + |e| R + 2 d 2^-24 (|q| + |e|)(X + R)) (the fp32
// accumulations of the coarse and the exact dot included; rounding residuals are <= 2^-9 of each
// component, so E ~ 2^-8 |q| X at worst, ~2^-9 for random data).  Every row of the exact top k
// (ties included) has s~ <= T = s~(k) + 2E, s~(k) the coarse k-th best.  The re-rank is exact
// when no such row can be missing: the CB_C-th selected key and every lane's bound (no row the
// lane left out has a smaller key) lie beyond T.  Otherwise the
// query's device flag is set and
// the exact scan recomputes the flagged queries (its blocks exit at once for query tiles without
// a flag) — never a silently approximate id.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
constexpr int CB_L = 8;                // coarse candidates kept per lane list
constexpr int CB_C = 64;               // coarse candidates re-ranked per query

__global__ void to_bf16_kernel(const float* __restrict__ x, int64_t n4, bf16x4* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256)
    out[i] = __builtin_convertvector(reinterpret_cast<const f32x4*>(x)[i], bf16x4);
}

// The coarse path's query prep in one launch: Q rounded to bf16 (as to_bf16_kernel) and |q|^2
// (qnorm_kernel's summation order, so the gated exact fallback reuses it bit for bit).
__global__ void qprep_kernel(const float* __restrict__ Q, int b, int d, __bf16* __restrict__ qb,
                             float* __restrict__ out) {
  const int q = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (q >= b) return;
  float s = 0.f;
#pragma unroll 8  // d <= 512 in one batch of loads (the sum keeps qnorm_kernel's order)
  for (int c = lane; c < d; c += 64) {
    const float v = Q[(int64_t)q * d + c];
    qb[(int64_t)q * d + c] = (__bf16)v;
    s += v * v;
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
  if (lane == 0) out[q] = s;
}

// |bf16(x) - x|^2 per row (wave per row; runs once per index)
__global__ void bf16_residual_kernel(const float* __restrict__ X, int64_t n, int d, float* out) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  float s = 0.f;
  for (int c = lane; c < d; c += 64) {
    const float v = X[row * d + c];
    const float r = (float)(__bf16)v - v;
    s += r * r;
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
  if (lane == 0) out[row] = s;
}

// max of n floats by one block (runs once per index)
__global__ __launch_bounds__(1024) void max_kernel(const float* __restrict__ x, int64_t n,
                                                   float* out) {
  __shared__ float red[16];
  float m = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += 1024) m = fmaxf(m, x[i]);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float r = 0.f;
    for (int i = 0; i < 16; ++i) r = fmaxf(r, red[i]);
    out[0] = r;
  }
}

// The coarse scan with the queries in REGISTERS, so one block covers up to 256 queries and the
// bf16 index is streamed from HBM once per search (round 2's kernel held 128 queries in LDS and
// read the index once per 128-query tile: twice at C5).  Block = NW waves x 32 queries; wave w's
// lane keeps its query's bf16 row as the MFMA B operand for every 16-deep k-step (KS x 16 B:
// 128 VGPRs at d = 512), so only the index tile passes through LDS: 64-row x 64-deep stages
// (register prefetch CB2_D stages ahead, two LDS buffers, one barrier per stage), every wave reading
// the A fragments of all 64 rows (1 KiB of LDS per 32x32x16 MFMA: 128 B/clk/CU at the MFMA rate,
// half the array's 256).  Two waves per SIMD at NW = 8, so one wave's key epilogue runs beside the
// other's MFMAs.  Keys: the coarse value quantised with the row tag in its low 6 bits (so
// the quantisation is < 2^-17 relative, inside the re-rank's 2^-16 margin); one sorted list of
// CB_L per (query, block) ([q][RB][CB_L]: the two lane halves merged in-kernel) and its lane bound.
constexpr int CB2_RT = 64;             // index rows per tile (2 x 32-row MFMA tiles)
constexpr int CB2_BK = 64;             // k per LDS stage (4 x 16-deep MFMA steps)

__device__ __forceinline__ void bf2_insert(float (&bk)[CB_L], int (&bi)[CB_L], float ck, int ci) {
#pragma unroll
  for (int t = 0; t < CB_L; ++t) {
    const bool sw = ck < bk[t];
    const float tk = sw ? bk[t] : ck;
    const int ti = sw ? bi[t] : ci;
    bk[t] = sw ? ck : bk[t];
    bi[t] = sw ? ci : bi[t];
    ck = tk;
    ci = ti;
  }
}

// The keys of one 64-row tile (the two 32x32 accumulators, zeroed here) into the lane's sorted
// list: each key quantised with its row in the low 6 bits, the best three of the tile by integer
// min / max, the best two inserted, the third bounding what was dropped (`drop`).
__device__ __forceinline__ void bf2_tile_keys(f32x16 (&acc)[2], const float* xn, float qn_l, int lh,
                                              int row0, float (&bk)[CB_L], int (&bi)[CB_L],
                                              float& drop) {
  uint32_t v1 = 0xFFFFFFFFu, v2 = 0xFFFFFFFFu, v3 = 0xFFFFFFFFu;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rr = mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      const float key = fmaxf(fmaf(-2.0f, acc[mi][r], xn[rr]) + qn_l, 0.0f);
      acc[mi][r] = 0.f;
      const uint32_t v = (__float_as_uint(key) & ~63u) | (uint32_t)rr;
      v3 = min(v3, max(v2, v));
      v2 = min(v2, max(v1, v));
      v1 = min(v1, v);
    }
  drop = fminf(drop, __uint_as_float(v3 & ~63u));
  const float k1 = __uint_as_float(v1 & ~63u), k2 = __uint_as_float(v2 & ~63u);
  if (k1 < bk[CB_L - 1]) bf2_insert(bk, bi, k1, row0 + (int)(v1 & 63u));
  if (k2 < bk[CB_L - 1]) bf2_insert(bk, bi, k2, row0 + (int)(v2 & 63u));
}

// One list per (query, block): lane li takes lane li + 32's list (the same query's other rows)
// and keeps the best CB_L of the 16.  Every row the merged list lacks has a key >= the new bound
// min(both lanes' bounds, the smallest key pushed out here), so the re-rank's test is unchanged
// and the select reads half the candidates.
__device__ __forceinline__ void bf2_finish(float (&bk)[CB_L], int (&bi)[CB_L], float drop, int q,
                                           bool qok, int lh, int rb, int RB, int64_t row_offset,
                                           float* cand_key, int64_t* cand_id, float* lane_bound) {
  float bound = fminf(bk[CB_L - 1], drop);
  {
    float ok[CB_L];
    int oi[CB_L];
#pragma unroll
    for (int t = 0; t < CB_L; ++t) {
      ok[t] = __shfl_xor(bk[t], 32, 64);
      oi[t] = __shfl_xor(bi[t], 32, 64);
    }
    bound = fminf(bound, __shfl_xor(bound, 32, 64));
    float pushed = INFINITY;
#pragma unroll
    for (int s = 0; s < CB_L; ++s) {
      float ck = ok[s];
      int ci = oi[s];
#pragma unroll
      for (int t = 0; t < CB_L; ++t) {
        const bool sw = ck < bk[t];
        const float tk = sw ? bk[t] : ck;
        const int ti = sw ? bi[t] : ci;
        bk[t] = sw ? ck : bk[t];
        bi[t] = sw ? ci : bi[t];
        ck = tk;
        ci = ti;
      }
      pushed = fminf(pushed, ck);
    }
    bound = fminf(bound, pushed);
  }
  if (!qok || lh) return;
  float* okp = cand_key + ((int64_t)q * RB + rb) * CB_L;
  int64_t* oip = cand_id + ((int64_t)q * RB + rb) * CB_L;
#pragma unroll
  for (int t = 0; t < CB_L; ++t) {
    okp[t] = bk[t];
    oip[t] = bi[t] == INT_MAX ? -1 : (int64_t)bi[t] + row_offset;
  }
  lane_bound[(int64_t)q * RB + rb] = bound;
}

template <int KS, int NW, int D, int BK = CB2_BK>
__global__ __launch_bounds__(NW * 64, 8 / NW) void scan_bf2_kernel(const __bf16* __restrict__ Xb,
                                                              const float* __restrict__ xnorm,
                                                              int64_t n, int64_t row_offset,
                                                              const __bf16* __restrict__ Qb, int b,
                                                              const float* __restrict__ qnorm,
                                                              int nqt, int RB, float* cand_key,
                                                              int64_t* cand_id, float* lane_bound) {
  constexpr int d = KS * 16, NT = NW * 64;
  constexpr int SPT = d / BK;                       // stages per row tile
  constexpr int LPS = CB2_RT * BK / 8 / NT;         // 16-byte loads per thread per stage
  constexpr int CPR = BK / 8;                       // 16-byte chunks per staged row
  constexpr int LDK = BK + 8;                       // LDS row stride (bf16): conflict-free
  constexpr int STAGE = CB2_RT * LDK;
  static_assert(LPS >= 1 && SPT % D == 0, "stage slots repeat per row tile");
  static_assert(SPT % 2 == 0, "a tile's first stage lands in LDS buffer 0");
  __shared__ __attribute__((aligned(16))) __bf16 xs[2][STAGE];
  __shared__ float xn_s[2][CB2_RT];
  int qt, rb;
  {
    const int total = gridDim.x, hw = blockIdx.x;
    const int xcd = hw & 7, slot = hw >> 3, q8 = total >> 3, r8 = total & 7;
    const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
    qt = t % nqt;
    rb = t / nqt;
  }
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 31, lh = lane >> 5;
  const int64_t ntile = (n + CB2_RT - 1) / CB2_RT;
  const int ntb = (int)((ntile - rb + RB - 1) / RB);

  const int q = qt * NW * 32 + wave * 32 + li;
  const bool qok = q < b;
  const float qn_l = qok ? qnorm[q] : 0.f;
  // B[k = 16 j + 8 lh + e][col li] = Q~[q][16 j + 8 lh + e]; queries past b read row b-1 (their
  // lists are never written)
  bf16x8 qf[KS];
  {
    const __bf16* qp = Qb + (int64_t)(qok ? q : b - 1) * d + 8 * lh;
#pragma unroll
    for (int j = 0; j < KS; ++j) qf[j] = *reinterpret_cast<const bf16x8*>(qp + 16 * j);
  }

  bf16x8 rx[D][LPS];
  float rn[D];
  // stage ks of the block's row tile tt: rows past n load row n-1 (masked by an infinite norm)
  auto gload = [&](int j, int tt, int ks) {
    const int64_t row0 = (int64_t)(rb + (int64_t)tt * RB) * CB2_RT;
#pragma unroll
    for (int i = 0; i < LPS; ++i) {
      const int idx = tid + i * NT, r = idx / CPR, c = ks * BK + (idx % CPR) * 8;
      const int64_t row = row0 + r;
      rx[j][i] = *reinterpret_cast<const bf16x8*>(Xb + (row < n ? row : n - 1) * (int64_t)d + c);
    }
    if (ks == 0) {  // unconditional load (a select on loaded data makes hipcc wait early)
      const int64_t nrow = row0 + (tid & (CB2_RT - 1));
      rn[j] = xnorm[nrow < n ? nrow : n - 1];
    }
  };
  auto swrite = [&](int st, int j, int tt, int ks) {
#pragma unroll
    for (int i = 0; i < LPS; ++i) {
      const int idx = tid + i * NT, r = idx / CPR, c = (idx % CPR) * 8;
      *reinterpret_cast<bf16x8*>(&xs[st][r * LDK + c]) = rx[j][i];
    }
    if (ks == 0 && tid < CB2_RT) {  // rows past n: infinite keys
      const int64_t nrow = (int64_t)(rb + (int64_t)tt * RB) * CB2_RT + tid;
      xn_s[tt & 1][tid] = nrow < n ? rn[j] : INFINITY;
    }
  };

  f32x16 acc[2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[mi][r] = 0.f;
  float bk[CB_L];
  int bi[CB_L];
#pragma unroll
  for (int t = 0; t < CB_L; ++t) {
    bk[t] = INFINITY;
    bi[t] = INT_MAX;
  }
  float drop = INFINITY;

  // prologue: stage 0 in LDS buffer 0, stages 1..D in flight (stage s >= 1 in slot (s - 1) % D)
  gload(0, 0, 0);
  swrite(0, 0, 0, 0);
#pragma unroll
  for (int j = 0; j < D; ++j) gload(j, (1 + j) / SPT, (1 + j) % SPT);
  __syncthreads();
  for (int tt = 0; tt < ntb; ++tt) {
#pragma clang loop unroll(full)
    for (int ks = 0; ks < SPT; ++ks) {
      const int st = ks & 1;  // SPT is even: a tile's first stage is always in buffer 0
#pragma unroll
      for (int u = 0; u < BK / 16; ++u) {
        bf16x8 fa[2];
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
          fa[mi] = *reinterpret_cast<const bf16x8*>(
              &xs[st][(mi * 32 + li) * LDK + 16 * u + 8 * lh]);
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
          acc[mi] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[mi], qf[ks * (BK / 16) + u],
                                                            acc[mi], 0, 0, 0);
      }
      // stage g+1 (held in slot g % D = ks % D) into the other buffer, then re-arm that slot with
      // stage g+1+D
      const int j1 = ks % D;
      swrite(st ^ 1, j1, tt + (ks + 1) / SPT, (ks + 1) % SPT);
      gload(j1, tt + (ks + 1 + D) / SPT, (ks + 1 + D) % SPT);
      __syncthreads();
    }
    // keys of this row tile (n < 2^31: checked by the launcher)
    bf2_tile_keys(acc, xn_s[tt & 1], qn_l, lh, (rb + tt * RB) * CB2_RT, bk, bi, drop);
  }
  bf2_finish(bk, bi, drop, q, qok, lh, rb, RB, row_offset, cand_key, cand_id, lane_bound);
}

// Select + re-rank without a full selection (block per query, the one-list-per-block layout of
// scan_bf2: n_lists sorted lists of CB_L, n_lists <= 512).  The re-rank only ever needs the
// candidates whose coarse key is within T = s~(k) + 2E (rerank_block's bound), so:
//  1. s~(k), the k-th smallest coarse key: each wave walks its lists' sorted heads for k rounds
//     (wave-shuffle minima, no block barrier), then one wave takes the k-th of the 4 x k winners;
//  2. |q|, the query's bf16 residual and E as rerank_block; T, Tcut;
//  3. every entry <= Tcut is gathered (each list's qualifying entries are a prefix; a block scan
//     places them) — at most CB_C, else the query is flagged for the exact scan;
//  4. exact fp32 keys of the gathered rows, the best k by (key, id).
// Sufficient when nothing was cut off: every list's bound > T and the gather did not overflow
// (a row missing from every list has a key >= its lane's bound).  Same outputs as the select +
// rerank_block pair whenever both are exact.
// D = d (256 or 512, scan_coarse_eligible): the exact keys' row loads are straight-line code.
// pack_out: the (dist, id) float64 pairs of every query too (the sharded search's exchange block;
// the gated fallback merge rewrites a flagged query's).
template <int K, int D>
__global__ __launch_bounds__(256) void coarse_rerank2_kernel(
    const float* __restrict__ cand_key, const int64_t* __restrict__ cand_id, int n_lists,
    const float* __restrict__ X, const float* __restrict__ xnorm, int d, int64_t row_offset,
    const float* __restrict__ Q, const float* __restrict__ lane_bound, int k, const float* xmax,
    float* out_dist, int64_t* out_id, int* gate, double2* pack_out, int* tile_cnt) {
  constexpr int LPT = 2;  // lists per thread (n_lists <= 512)
  __shared__ float qs[512];
  __shared__ float wk[4][K];
  __shared__ float red[3][4];
  __shared__ int wcount[4];
  __shared__ float keys[CB_C];
  __shared__ int64_t ids[CB_C];
  __shared__ float s_T;
  const int qi = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* ck = cand_key + (int64_t)qi * n_lists * CB_L;
  const int64_t* ci = cand_id + (int64_t)qi * n_lists * CB_L;
  // Every global operand needed before the exact keys is loaded up front (this thread's lists'
  // keys and ids, their bounds, the query, xmax), so the block waits on memory twice — these,
  // then the gathered rows — instead of once per step.
  static_assert(CB_L == 8, "two float4 per list");
  float lk[LPT][CB_L], lkc[LPT][CB_L];
  int64_t lid[LPT][CB_L];
  float lb = INFINITY;  // the smallest bound of this thread's lists
#pragma unroll
  for (int p = 0; p < LPT; ++p) {
    const int l = tid + p * 256;
    if (l < n_lists) {
      const f32x4* k4 = reinterpret_cast<const f32x4*>(ck + (int64_t)l * CB_L);
      const f32x4 k0 = k4[0], k1 = k4[1];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        lk[p][t] = k0[t];
        lk[p][4 + t] = k1[t];
      }
#pragma unroll
      for (int t = 0; t < CB_L; ++t) lid[p][t] = ci[(int64_t)l * CB_L + t];
      lb = fminf(lb, lane_bound[(int64_t)qi * n_lists + l]);
    } else {
#pragma unroll
      for (int t = 0; t < CB_L; ++t) {
        lk[p][t] = INFINITY;
        lid[p][t] = -1;
      }
    }
#pragma unroll
    for (int t = 0; t < CB_L; ++t) lkc[p][t] = lk[p][t];
  }
  const float* qp = Q + (int64_t)qi * d;
  float qv[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) qv[j] = tid + 256 * j < d ? qp[tid + 256 * j] : 0.f;
  const float xm0 = xmax[0], xm1 = xmax[1];
  // 1. the wave's k smallest keys: k rounds of "minimum head, its owner advances"
  {
    int h0 = 0, h1 = 0;  // heads of the thread's two lists
    for (int r = 0; r < k; ++r) {
      float a = h0 < CB_L ? lk[0][0] : INFINITY, b2 = h1 < CB_L ? lk[1][0] : INFINITY;
      // (static indexing: the head value is rotated to slot 0 as a list advances, below)
      const float mine = fminf(a, b2);
      const float m = wave_min(mine);
      // the lowest lane holding the minimum advances one list
      const uint64_t bal = __ballot(mine == m);
      const int win = __ffsll((unsigned long long)bal) - 1;
      if (lane == win) {
        if (a <= b2) {
#pragma unroll
          for (int t = 0; t < CB_L - 1; ++t) lk[0][t] = lk[0][t + 1];
          lk[0][CB_L - 1] = INFINITY;
          ++h0;
        } else {
#pragma unroll
          for (int t = 0; t < CB_L - 1; ++t) lk[1][t] = lk[1][t + 1];
          lk[1][CB_L - 1] = INFINITY;
          ++h1;
        }
      }
      if (lane == 0) wk[wave][r] = m;
    }
  }
  // 2. the query's norms and E (rerank_block's formulas and summation order)
  float ss = 0.f, ee = 0.f;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int c = tid + 256 * j;
    if (c < d) {
      const float v = qv[j];
      const float r = (float)(__bf16)v - v;
      qs[c] = v;
      ss += v * v;
      ee += r * r;
    }
  }
  float lm = lb;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    ss += __shfl_xor(ss, off, 64);
    ee += __shfl_xor(ee, off, 64);
    lm = fminf(lm, __shfl_xor(lm, off, 64));
  }
  if (lane == 0) {
    red[0][wave] = ss;
    red[1][wave] = ee;
    red[2][wave] = lm;
  }
  __syncthreads();
  const float qn = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
  if (wave == 0) {  // k-th smallest of the 4 waves' k smallest: one per lane, k wave minima
    float v = lane < 4 * k ? wk[lane / k][lane % k] : INFINITY;
    float kth = INFINITY;
    for (int r = 0; r < k; ++r) {
      const float m = wave_min(v);
      kth = m;
      const uint64_t bal = __ballot(v == m);
      if (lane == __ffsll((unsigned long long)bal) - 1) v = INFINITY;
    }
    const float qa = sqrtf(qn), ea = sqrtf((red[1][0] + red[1][1]) + (red[1][2] + red[1][3]));
    const float Xm = sqrtf(xm0), Rm = sqrtf(xm1);
    const float E = 2.0f * (ea * Xm + qa * Rm + ea * Rm + 2.0f * d * 5.9604645e-8f * (qa + ea) *
                                                         (Xm + Rm)) * 1.01f +
                    4.0f * 5.9604645e-8f * (Xm * Xm + 2.0f * qa * Xm + qa * qa);
    if (lane == 0) s_T = kth * (1.0f + 3.0517578e-5f) + 2.0f * E;
  }
  __syncthreads();
  const float T = s_T, Tcut = T * (1.0f + 1.5258789e-5f);
  // 3. gather every entry <= Tcut (from the kept copy of the lists: step 1 consumed lk)
  int cnt[LPT], mycnt = 0;
#pragma unroll
  for (int p = 0; p < LPT; ++p) {
    const int l = tid + p * 256;
    cnt[p] = 0;
    if (l < n_lists)
#pragma unroll
      for (int t = 0; t < CB_L; ++t) cnt[p] += lkc[p][t] <= Tcut ? 1 : 0;
    mycnt += cnt[p];
  }
  int incl = mycnt;  // wave inclusive scan
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int o = __shfl_up(incl, off, 64);
    if (lane >= off) incl += o;
  }
  if (lane == 63) wcount[wave] = incl;
  for (int c = tid; c < CB_C; c += 256) {
    keys[c] = INFINITY;
    ids[c] = INT64_MAX;
  }
  __syncthreads();
  int base = incl - mycnt;
  for (int w = 0; w < wave; ++w) base += wcount[w];
  const int total = (wcount[0] + wcount[1]) + (wcount[2] + wcount[3]);
  // (candidate keys go to LDS as +inf-keyed placeholders first: their exact keys come in step 4;
  // a list's qualifying entries are a prefix, so static register indices suffice)
  int pos = base;
#pragma unroll
  for (int p = 0; p < LPT; ++p) {
#pragma unroll
    for (int t = 0; t < CB_L; ++t)
      if (t < cnt[p] && pos + t < CB_C) ids[pos + t] = lid[p][t];
    pos += cnt[p];
  }
  __syncthreads();
  const int need = min(total, CB_C);
  // 4. exact keys (rerank_block's summation: 64 lanes over the row, lane l summing elements
  // l + 64 j in j order, then the xor butterfly).  Each wave takes CB_C / 4 candidates and loads
  // all their rows and norms before the first product (branch-free: past `need` it re-loads the
  // last candidate and discards it), so the block waits on memory once; the 16 butterflies
  // interleave.
  static_assert(CB_C == 64, "one candidate per lane in the final rank");
  constexpr int J = D / 64, G = CB_C / 4;
  const int c0 = wave * G;
  if (c0 < need) {  // wave-uniform
    float qr[J], xv[G][J], xn[G], dot[G];
#pragma unroll
    for (int j = 0; j < J; ++j) qr[j] = qs[lane + 64 * j];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int64_t id = ids[min(c0 + g, need - 1)];
      const int64_t r = id >= 0 ? id - row_offset : 0;
      const float* xp = X + r * (int64_t)D;
      xn[g] = xnorm[r];
#pragma unroll
      for (int j = 0; j < J; ++j) xv[g][j] = xp[lane + 64 * j];
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      dot[g] = 0.f;
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int e = lane + 64 * j;
        dot[g] += e < d ? qr[j] * xv[g][j] : 0.f;
      }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1)
#pragma unroll
      for (int g = 0; g < G; ++g) dot[g] += __shfl_xor(dot[g], off, 64);
    if (lane == 0) {
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const int c = c0 + g;
        if (c < need) {
          const int64_t id = ids[c];
          keys[c] = id >= 0 ? sqrtf(fmaxf(qn + xn[g] - 2.0f * dot[g], 0.0f)) : INFINITY;
          if (id < 0) ids[c] = INT64_MAX;
        }
      }
    }
  }
  __syncthreads();
  // 5. the best k by (key, id): one wave, lane c holding candidate c, ranks by lane reads (the
  // placeholders past `need`, (+inf, INT64_MAX), never rank below a candidate)
  if (wave != 0) return;
  if (lane == 0 && qi % SM_B == 0) tile_cnt[qi / SM_B] = 0;  // arm the gated fallback's merge
  if (lane == 0) {
    const float lists_bound = fminf(fminf(red[2][0], red[2][1]), fminf(red[2][2], red[2][3]));
    gate[qi] = (total <= CB_C && lists_bound > T) ? 0 : 1;
  }
  const float a = keys[lane];
  const int64_t ia = ids[lane];
  const int alo = (int)(uint32_t)(uint64_t)ia, ahi = (int)(uint32_t)((uint64_t)ia >> 32);
  int rank = 0;
  for (int c = 0; c < need; ++c) {
    const float kc = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(a), c));
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane(alo, c);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane(ahi, c);
    rank += key_less(kc, (int64_t)(((uint64_t)hi << 32) | lo), a, ia) ? 1 : 0;
  }
  if (rank < k) {
    const float v = ia == INT64_MAX ? NAN : a;
    const int64_t id = ia == INT64_MAX ? -1 : ia;
    out_dist[(int64_t)qi * k + rank] = v;
    out_id[(int64_t)qi * k + rank] = id;
    if (pack_out) pack_out[(int64_t)qi * k + rank] = make_double2((double)v, (double)id);
  }
}

__global__ void sqnorm_kernel(const float* X, int64_t n, int d, float* out) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  const float* x = X + row * d;
  float s = 0.f;
  for (int c = lane; c < d; c += 64) s += x[c] * x[c];
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
  if (lane == 0) out[row] = s;
}

__global__ void cosine_rows_kernel(const float* x1, const float* x2, int64_t m, int d, float eps,
                                   float* out) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= m) return;
  const float* a = x1 + row * d;
  const float* b = x2 + row * d;
  float w12 = 0.f, w1 = 0.f, w2 = 0.f;
  for (int c = lane; c < d; c += 64) {
    w12 += a[c] * b[c];
    w1 += a[c] * a[c];
    w2 += b[c] * b[c];
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    w12 += __shfl_xor(w12, off, 64);
    w1 += __shfl_xor(w1, off, 64);
    w2 += __shfl_xor(w2, off, 64);
  }
  if (lane == 0) out[row] = w12 / fmaxf(sqrtf(w1) * sqrtf(w2), eps);
}

int list_cap(int k) {
  int c = 1;
  while (c < k) c <<= 1;
  return c;
}

int64_t scan_blocks(int64_t n) {
  const int64_t ntiles = (n + 15) / 16;
  int64_t nb = (ntiles + 3) / 4;
  return nb < 1 ? 1 : (nb > 2048 ? 2048 : nb);
}

size_t scan_lds_bytes(int d, int K) {
  const size_t q = (size_t)QG * (d + 4) * sizeof(float);
  const size_t m = (size_t)QG * 16 * K * (sizeof(float) + sizeof(int));
  return q > m ? q : m;
}

template <int K>
int launch_scan(const float* X, const float* xnorm, int64_t n, int d, int64_t row_offset,
                int metric, const float* Q, int b, float* ck, int64_t* ci, hipStream_t s) {
  const int64_t nb = scan_blocks(n);
  const size_t lds = scan_lds_bytes(d, K);
  dim3 grid((unsigned)nb, (unsigned)cdiv(b, QG));
  hipLaunchKernelGGL((scan_kernel<K, false>), grid, dim3(256), lds, s, X, xnorm, n, d, row_offset,
                     metric, Q, b, ck, ci, (float*)nullptr);
  MPR_LAUNCHED();
  return MPR_OK;
}


int merge_dispatch(const float* ck, const int64_t* ci, int b, int64_t n_cand, int k,
                   int keys_are_values, int metric, float* od, int64_t* oi, hipStream_t s,
                   const int* gate = nullptr, double* pack_out = nullptr) {
  return merge_lists(ck, ci, b, n_cand, k, keys_are_values, metric, od, oi, s, gate, pack_out);
}

}  // namespace

// The large-batch path: b >= SM_MIN_B queries, k <= 16, d >= 64 (two k-steps per row tile).
constexpr int SM_MIN_B = 64;
bool use_scan_mm(int64_t n, int d, int b, int k) {
  return b >= SM_MIN_B && k <= 16 && d >= 2 * SM_BK && d % 4 == 0 && n >= SM_B;
}
int scan_mm_rowblocks(int64_t n, int b) {
  const int64_t ntile = (n + SM_B - 1) / SM_B;
  const int nqt = (int)cdiv(b, SM_B);
  const int64_t rb = std::max<int64_t>(1, 512 / nqt);  // ~2 blocks per CU
  return (int)std::min(rb, ntile);
}
// As the coarse path's gated fallback the scan runs on few row blocks (8 per query tile): when no
// query is flagged (the common case) its blocks exit at once, and a grid of 32 exits in ~2 us
// where 512 blocks of this LDS-heavy kernel took ~5 us and, beside another stream's coarse scan,
// waited for CUs (profiles/r05_proj_w8_kernel_stats.csv); a flagged query tile scans with 8
// blocks instead of ~128 (rare: rows within the coarse error bound overflowing the candidate
// list).  Any row blocking gives the same keys and the same exact top k.
int scan_mm_rb(int64_t n, int b, bool gated) {
  return gated ? std::min(scan_mm_rowblocks(n, b), 8) : scan_mm_rowblocks(n, b);
}
// whether the coarse path's gated merge is the wave merge writing packed pairs (<= 512
// candidates, k <= 8) — and so the re-rank writes them for every query
bool coarse_packs(int64_t n, int b, int k) {
  return (int64_t)scan_mm_rb(n, b, true) * list_cap(k) <= 512 && k <= 8;
}

template <int K>
int launch_scan_mm(const float* X, int64_t n, int d, int64_t row_offset, int metric,
                   const float* Q, float* qn, int b, float* ck, int64_t* ci, hipStream_t s,
                   const int* gate, const float* qn_pre, int* tile_cnt = nullptr, int k = 0,
                   float* od = nullptr, int64_t* oi = nullptr, double* pack_out = nullptr) {
  const int nqt = (int)cdiv(b, SM_B), RB = scan_mm_rb(n, b, gate != nullptr);
  if (qn_pre)
    qn = const_cast<float*>(qn_pre);
  else
    hipLaunchKernelGGL(qnorm_kernel, dim3((unsigned)cdiv(b, 4)), dim3(256), 0, s, Q, b, d, qn);
  hipLaunchKernelGGL((scan_mm_kernel<K>), dim3((unsigned)(nqt * RB)), dim3(256), 0, s, X, n, d,
                     row_offset, metric, Q, qn, b, nqt, RB, ck, ci, gate, tile_cnt, k, od, oi,
                     reinterpret_cast<double2*>(pack_out));
  MPR_LAUNCHED();
  return MPR_OK;
}

// ---- coarse path launchers --------------------------------------------------------------------
int coarse_waves(int b) { return b <= 128 ? 4 : 8; }
// one 8-wave block (two at 4 waves) per CU, every lane seeing >= 8 row tiles (<= 512: the
// threshold gather of coarse_rerank2_kernel walks at most 512 lists)
int coarse_rowblocks(int64_t n, int b) {
  const int64_t ntile = (n + CB2_RT - 1) / CB2_RT;
  const int NW = coarse_waves(b), nqt = (int)cdiv(b, NW * 32);
  const int64_t per = std::max<int64_t>(1, (NW == 4 ? 512 : 256) / nqt);
  return (int)std::max<int64_t>(1, std::min<int64_t>(per, ntile / 8));
}

bool scan_coarse_eligible(int64_t n, int d, int b, int k, int metric) {
  static const bool off = [] {
    const char* e = getenv("MPR_SCAN_COARSE");
    return e && e[0] == '0';
  }();
  static const bool mm_off = getenv("MPR_SCAN_MM_OFF") != nullptr;
  // the coarse path's gated exact fallback is scan_mm: only where that one runs (k <= 16)
  return !off && !mm_off && metric == 0 && b >= SM_MIN_B && k <= CB_C / 2 &&
         (d == 256 || d == 512) && n >= CB_C && use_scan_mm(n, d, b, k);
}

int bf16_residuals(const float* X, int64_t n, int d, float* out, hipStream_t s) {
  if (n == 0) return MPR_OK;
  hipLaunchKernelGGL(bf16_residual_kernel, dim3((unsigned)cdiv(n, 4)), dim3(256), 0, s, X, n, d,
                     out);
  MPR_LAUNCHED();
  return MPR_OK;
}

int index_to_bf16(const float* X, int64_t count, void* out, hipStream_t s) {
  MPR_REQUIRE(count % 4 == 0, "to_bf16: count %lld", (long long)count);
  if (count == 0) return MPR_OK;
  const int64_t n4 = count / 4;
  hipLaunchKernelGGL(to_bf16_kernel, dim3((unsigned)std::min<int64_t>(cdiv(n4, 256), 8192)),
                     dim3(256), 0, s, X, n4, reinterpret_cast<bf16x4*>(out));
  MPR_LAUNCHED();
  return MPR_OK;
}

int max_of(const float* x, int64_t n, float* out, hipStream_t s) {
  hipLaunchKernelGGL(max_kernel, dim3(1), dim3(1024), 0, s, x, n, out);
  MPR_LAUNCHED();
  return MPR_OK;
}

namespace {
struct CoarseWs {
  float *ck, *sk, *qn, *lb;
  int64_t *ci, *si;
  __bf16* qb;
  int* gate;
  int* cnt;  // per exact-scan query tile: fallback blocks done (zeroed by the re-rank)
  size_t bytes;
};
CoarseWs coarse_ws(void* base, int64_t n, int d, int b) {
  const int RB = coarse_rowblocks(n, b);
  const size_t nc = (size_t)b * RB * 2 * CB_L, ns = (size_t)b * CB_C;
  char* p = reinterpret_cast<char*>(base);
  CoarseWs w;
  w.ci = reinterpret_cast<int64_t*>(p); p += nc * 8;
  w.si = reinterpret_cast<int64_t*>(p); p += ns * 8;
  w.ck = reinterpret_cast<float*>(p); p += nc * 4;
  w.sk = reinterpret_cast<float*>(p); p += ns * 4;
  w.lb = reinterpret_cast<float*>(p); p += ((size_t)b * RB * 2 * 4 + 15) / 16 * 16;
  w.qn = reinterpret_cast<float*>(p); p += ((size_t)b * 4 + 15) / 16 * 16;
  w.qb = reinterpret_cast<__bf16*>(p); p += ((size_t)b * d * 2 + 15) / 16 * 16;
  w.gate = reinterpret_cast<int*>(p); p += ((size_t)b * 4 + 15) / 16 * 16;
  w.cnt = reinterpret_cast<int*>(p); p += ((size_t)cdiv(b, SM_B) * 4 + 15) / 16 * 16;
  w.bytes = (size_t)(p - reinterpret_cast<char*>(base));
  return w;
}
}  // namespace

int coarse_flag_count(const void* ws, int64_t n, int d, int b, int* count) {
  CoarseWs w = coarse_ws(const_cast<void*>(ws), n, d, b);
  std::vector<int> h(b);
  MPR_HIP(hipMemcpy(h.data(), w.gate, (size_t)b * sizeof(int), hipMemcpyDeviceToHost));
  int c = 0;
  for (int v : h) c += v != 0;
  *count = c;
  return MPR_OK;
}

// Slices per query of the two-level merge: enough blocks to spread over the chip (b * P <= 256)
// with >= 512 candidates per slice; 1 = a single merge.
int merge_split(int b, int64_t n_cand) {
  int P = 1;
  while (b * P * 2 <= 256 && n_cand % (P * 2) == 0 && n_cand / (P * 2) >= 512) P *= 2;
  return P;
}

// scan_small_kernel when the tile-per-wave scan would launch fewer than ~2 blocks per CU
bool small_regime(int64_t n, int b) {
  return cdiv(n, 16) <= 16384 && scan_blocks(n) * cdiv(b, QG) < 512;
}
bool use_scan_small(int64_t n, int d, int b) {
  return (d == 256 || d == 512 || d == 1024) && small_regime(n, b) &&
         !getenv("MPR_SCAN_SMALL_OFF");
}

size_t scan_topk_workspace(int64_t n, int b, int k) {
  if (k > 64) return (size_t)b * n * sizeof(float) + 256;  // the full score rows (select_large)
  const int K = list_cap(k);
  const int64_t per_q = std::max<int64_t>(
      std::max<int64_t>(scan_blocks(n), small_regime(n, b) ? cdiv(n, 16) : 0),
      scan_mm_rowblocks(n, b));
  const size_t exact = (size_t)b * per_q * K * (sizeof(float) + sizeof(int64_t)) + (size_t)b * 4 +
                       (size_t)256 * K * (sizeof(float) + sizeof(int64_t)) + 512;
  // the coarse path's buffers (d <= 512) ahead of the exact path's (its gated fallback)
  return exact + coarse_ws(nullptr, n, 512, b).bytes + 256;
}

int scan_topk(const float* X, const float* xnorm, int64_t n, int d, int64_t row_offset,
              int metric, const float* Q, int b, int k, float* ws, size_t ws_bytes,
              float* out_dist, int64_t* out_ids, hipStream_t s, const void* Xb,
              const float* xmax, double* pack_out, bool* packed) {
  if (packed) *packed = false;
  MPR_REQUIRE(k >= 1 && k <= SELECT_MAX_K, "search: k=%d must be in [1, %d]", k, SELECT_MAX_K);
  MPR_REQUIRE(k <= n, "search: k=%d exceeds index rows %lld", k, (long long)n);
  MPR_REQUIRE(d % 16 == 0 && d <= 8192, "search: d=%d must be a multiple of 16", d);
  MPR_REQUIRE(b >= 0, "search: b<0");
  if (b == 0) return MPR_OK;
  MPR_REQUIRE(ws_bytes >= scan_topk_workspace(n, b, k), "search: workspace too small");
  if (k > 64) {
    // a retrieval_k past the fused kernels' register lists: the full score rows (the exact scan
    // kernel's arithmetic, as mpr_index_scores), then a per-query radix select + sort
    MPR_TRY(scan_scores(X, xnorm, n, d, metric, Q, b, ws, s));
    return select_large(ws, nullptr, b, n, k, metric == 1 ? -1.f : 1.f, row_offset, out_dist,
                        out_ids, s);
  }
  const int K = list_cap(k);
  const int* gate = nullptr;
  void* ws_coarse = nullptr;      // the coarse path's buffers (its fallback's tile counters)
  const float* qn_pre = nullptr;  // |q|^2 already computed by the coarse path
  if (Xb && xmax && scan_coarse_eligible(n, d, b, k, metric)) {
    // coarse bf16 scan -> top CB_C per query -> exact re-rank (+ the gated exact fallback below)
    ws_coarse = ws;
    CoarseWs w = coarse_ws(ws, n, d, b);
    ws = reinterpret_cast<float*>(reinterpret_cast<char*>(ws) + (w.bytes + 255) / 256 * 256);
    const int RB = coarse_rowblocks(n, b);
    MPR_REQUIRE(n < (int64_t)1 << 31, "search: coarse scan rows %lld >= 2^31", (long long)n);
    hipLaunchKernelGGL(qprep_kernel, dim3((unsigned)cdiv(b, 4)), dim3(256), 0, s, Q, b, d,
                       reinterpret_cast<__bf16*>(w.qb), w.qn);
    MPR_LAUNCHED();
    qn_pre = w.qn;
    const __bf16* xb = reinterpret_cast<const __bf16*>(Xb);
    const int NW = coarse_waves(b), nqt = (int)cdiv(b, NW * 32);
    const dim3 grid((unsigned)(nqt * RB)), blk((unsigned)(NW * 64));
    // prefetch: 16-byte loads per thread in flight = D x LPS = 4 at 8 waves (d = 512: one
    // 256-deep stage, 4 loads; d = 256: 4 64-deep stages), 4 at 4 waves (2 stages of 2 loads:
    // the 256-VGPR budget of 2 blocks per CU)
#define MPR_BF2(KS_, NW_, D_, BK_)                                                          \
  hipLaunchKernelGGL((scan_bf2_kernel<KS_, NW_, D_, BK_>), grid, blk, 0, s, xb, xnorm, n,     \
                     row_offset, w.qb, b, w.qn, nqt, RB, w.ck, w.ci, w.lb)
    if (d == 512) {
      // 8 waves: 256-deep stages, one in flight (two barriers per 64-row tile instead of 8 at
      // 64-deep x 4 in flight, the same 32 KiB of loads in flight per CU): C5 search 0.389 ->
      // 0.357 ms, 1/8 shard 72 -> 70 us (tools/scan_c5.py)
      // (Measured and dropped: four waves of 64 queries each (two 32-query groups per wave, one
      // wave per SIMD, every A fragment read feeding two MFMAs): 256 VGPRs + 256 AGPRs and still
      // 96-192 B of spills, C5 search 0.49-0.56 vs 0.37 ms, profiles/r05_scan_qg2_ab.txt.
      // The index tile staged by LDS-DMA, global_load_lds_dwordx4 into a
      // 3-buffer ring with 2 stages of 32 KiB in flight, counted vmcnt + raw s_barrier, XOR-
      // swizzled by source address: bit-identical, C5 search 0.382-0.392 vs 0.361-0.374 ms, the
      // 1/8 shard 70 vs 66 us; not bound by HBM bytes in flight, profiles/r05_scan_glds_ab.txt.)
      if (NW == 8) MPR_BF2(32, 8, 1, 256); else MPR_BF2(32, 4, 2, 64);
    } else {
      if (NW == 8) MPR_BF2(16, 8, 4, 64); else MPR_BF2(16, 4, 2, 64);
    }
#undef MPR_BF2
    MPR_LAUNCHED();
    // threshold gather over the sorted per-block lists (no full selection) + exact re-rank
    MPR_REQUIRE(RB <= 512, "search: %d coarse row blocks", RB);
    // the re-rank writes every query's packed pair when the gated merge below would (it rewrites
    // only the flagged queries')
    double2* rr_pack = (pack_out && coarse_packs(n, b, k)) ? reinterpret_cast<double2*>(pack_out)
                                                           : nullptr;
#define MPR_RR(D_)                                                                            \
  hipLaunchKernelGGL((coarse_rerank2_kernel<16, D_>), dim3((unsigned)b), dim3(256), 0, s, w.ck, \
                     w.ci, RB, X, xnorm, d, row_offset, Q, w.lb, k, xmax, out_dist, out_ids, w.gate, \
                     rr_pack, w.cnt)
    if (d == 512) MPR_RR(512); else MPR_RR(256);
#undef MPR_RR
    MPR_LAUNCHED();
    gate = w.gate;
  }
  if (use_scan_mm(n, d, b, k) && !getenv("MPR_SCAN_MM_OFF")) {
    const int RB = scan_mm_rb(n, b, gate != nullptr);
    int64_t* ci = reinterpret_cast<int64_t*>(ws);
    float* ck = reinterpret_cast<float*>(ci + (size_t)b * RB * K);
    float* qn = ck + (size_t)b * RB * K;
    // the coarse path's gated merge also writes the flagged queries' packed pairs when asked (the
    // wave merge: <= 512 candidates, k <= 8; the re-rank wrote every query's); with K <= 8 it is
    // folded into the fallback scan's last block per query tile (coarse_packs: RB * K <= 512)
    // (MPR_MERGE_BLOCK: the block merge, which writes no packed pairs: topk_pack runs instead)
    const bool block_merge = getenv("MPR_MERGE_BLOCK") != nullptr;
    double* po = (gate && pack_out && coarse_packs(n, b, k) && !block_merge) ? pack_out : nullptr;
    if (po && packed) *packed = true;
    const bool fold = gate && K <= 8 && !block_merge;
    int* cnt = fold ? coarse_ws(ws_coarse, n, d, b).cnt : nullptr;
    int rc = MPR_EUNSUP;
    switch (K) {
#define MPR_SM(KK) \
  case KK: rc = launch_scan_mm<KK>(X, n, d, row_offset, metric, Q, qn, b, ck, ci, s, gate, qn_pre, \
                                   cnt, k, out_dist, out_ids, po); \
    break;
      MPR_SM(1) MPR_SM(2) MPR_SM(4) MPR_SM(8) MPR_SM(16)
#undef MPR_SM
    }
    if (rc != MPR_OK || fold) return rc;
    return merge_dispatch(ck, ci, b, (int64_t)RB * K, k, /*keys_are_values=*/0, metric, out_dist,
                          out_ids, s, gate, po);
  }
  MPR_REQUIRE(gate == nullptr, "search: coarse path without its exact fallback");
  const bool small = use_scan_small(n, d, b);
  const int64_t nb = small ? cdiv(n, 16 * SS_TT) : scan_blocks(n);
  int64_t* ci = reinterpret_cast<int64_t*>(ws);
  float* ck = reinterpret_cast<float*>(ci + (size_t)b * nb * K);
  int rc = MPR_EUNSUP;
  if (small) {
    const dim3 grid((unsigned)nb, (unsigned)cdiv(b, QG));
    switch (K) {
#define MPR_SS(KK)                                                                        \
  case KK:                                                                                \
    if (d == 256)                                                                         \
      hipLaunchKernelGGL((scan_small_kernel<KK, 4, SS_TT>), grid, dim3(256), 0, s, X, xnorm, n,  \
                         row_offset, metric, Q, b, ck, ci);                               \
    else if (d == 512)                                                                    \
      hipLaunchKernelGGL((scan_small_kernel<KK, 8, SS_TT>), grid, dim3(256), 0, s, X, xnorm, n,  \
                         row_offset, metric, Q, b, ck, ci);                               \
    else                                                                                  \
      hipLaunchKernelGGL((scan_small_kernel<KK, 16, SS_TT>), grid, dim3(256), 0, s, X, xnorm, n, \
                         row_offset, metric, Q, b, ck, ci);                               \
    rc = MPR_OK;                                                                          \
    break;
      MPR_SS(1) MPR_SS(2) MPR_SS(4) MPR_SS(8) MPR_SS(16) MPR_SS(32) MPR_SS(64)
#undef MPR_SS
    }
    MPR_LAUNCHED();
  } else switch (K) {
    case 1: rc = launch_scan<1>(X, xnorm, n, d, row_offset, metric, Q, b, ck, ci, s); break;
    case 2: rc = launch_scan<2>(X, xnorm, n, d, row_offset, metric, Q, b, ck, ci, s); break;
    case 4: rc = launch_scan<4>(X, xnorm, n, d, row_offset, metric, Q, b, ck, ci, s); break;
    case 8: rc = launch_scan<8>(X, xnorm, n, d, row_offset, metric, Q, b, ck, ci, s); break;
    case 16: rc = launch_scan<16>(X, xnorm, n, d, row_offset, metric, Q, b, ck, ci, s); break;
    case 32: rc = launch_scan<32>(X, xnorm, n, d, row_offset, metric, Q, b, ck, ci, s); break;
    case 64: rc = launch_scan<64>(X, xnorm, n, d, row_offset, metric, Q, b, ck, ci, s); break;
  }
  if (rc != MPR_OK) return rc;
  const int64_t n_cand = nb * K;
  const int P = merge_split(b, n_cand);
  if (P > 1) {
    // few queries, many candidates: P blocks per query each keep the best K of one slice, then one
    // block per query merges the P lists (the (key, id) order makes the result the same list)
    int64_t* ci2 = reinterpret_cast<int64_t*>(ck + (size_t)b * n_cand);
    float* ck2 = reinterpret_cast<float*>(ci2 + (size_t)b * P * K);
    MPR_TRY(merge_dispatch(ck, ci, b * P, n_cand / P, K, /*keys_are_values=*/0, metric, ck2, ci2,
                           s));
    return merge_dispatch(ck2, ci2, b, (int64_t)P * K, k, /*keys_are_values=*/1, metric,
                          out_dist, out_ids, s);
  }
  return merge_dispatch(ck, ci, b, n_cand, k, /*keys_are_values=*/0, metric, out_dist, out_ids, s);
}

int scan_scores(const float* X, const float* xnorm, int64_t n, int d, int metric, const float* Q,
                int b, float* out, hipStream_t s) {
  MPR_REQUIRE(d % 16 == 0, "scores: d=%d must be a multiple of 16", d);
  if (b == 0 || n == 0) return MPR_OK;
  dim3 grid((unsigned)scan_blocks(n), (unsigned)cdiv(b, QG));
  const size_t lds = scan_lds_bytes(d, 1);
  hipLaunchKernelGGL((scan_kernel<1, true>), grid, dim3(256), lds, s, X, xnorm, n, d, (int64_t)0,
                     metric, Q, b, (float*)nullptr, (int64_t*)nullptr, out);
  MPR_LAUNCHED();
  return MPR_OK;
}

int row_sqnorms(const float* X, int64_t n, int d, float* out, hipStream_t s) {
  if (n == 0) return MPR_OK;
  hipLaunchKernelGGL(sqnorm_kernel, dim3((unsigned)cdiv(n, 4)), dim3(256), 0, s, X, n, d, out);
  MPR_LAUNCHED();
  return MPR_OK;
}

int topk_merge(const float* cand_d, const int64_t* cand_i, int b, int64_t n_cand, int k,
               int metric, float* out_d, int64_t* out_i, hipStream_t s) {
  MPR_REQUIRE(k >= 1 && k <= SELECT_MAX_K && k <= n_cand, "merge: k=%d n_cand=%lld", k,
              (long long)n_cand);
  if (b == 0) return MPR_OK;
  return merge_dispatch(cand_d, cand_i, b, n_cand, k, /*keys_are_values=*/1, metric, out_d, out_i,
                        s);
}

int cosine_rows(const float* x1, const float* x2, int64_t m, int d, float eps, float* out,
                hipStream_t s) {
  if (m == 0) return MPR_OK;
  hipLaunchKernelGGL(cosine_rows_kernel, dim3((unsigned)cdiv(m, 4)), dim3(256), 0, s, x1, x2, m,
                     d, eps, out);
  MPR_LAUNCHED();
  return MPR_OK;
}

}  // namespace mpr
