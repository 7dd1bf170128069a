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

#include "kernels.h"

namespace mpr {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int QG = 16;  // queries per group (MFMA N)
constexpr float COS_EPS = 1e-8f;

__device__ __forceinline__ bool key_less(float ka, int64_t ia, float kb, int64_t ib) {
  return ka < kb || (ka == kb && ia < ib);
}

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
                                                      int64_t* cand_id) {
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

// Final selection: per query, best k of n_cand (key, id) candidates.  Thread-local sorted lists
// over a strided slice, then a pairwise tree merge through LDS.
template <int K, int NT>
__global__ __launch_bounds__(NT) void merge_kernel(const float* cand_key, const int64_t* cand_id,
                                                   int64_t n_cand, int k, int keys_are_values,
                                                   int metric, float* out_val, int64_t* out_id) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* Sk = lds;                                            // [NT][K]
  int64_t* Si = reinterpret_cast<int64_t*>(lds + NT * K);     // [NT][K]
  const int q = blockIdx.x, tid = threadIdx.x;
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
#pragma unroll
  for (int t = 0; t < K; ++t) {
    Sk[tid * K + t] = bk[t];
    Si[tid * K + t] = bi[t];
  }
  __syncthreads();
  for (int half = NT / 2; half >= 1; half >>= 1) {
    if (tid < half) {
      const int a = tid, bb = tid + half;
      int pa = 0, pb = 0;
      float mk[K];
      int64_t mi[K];
#pragma unroll
      for (int t = 0; t < K; ++t) {
        const float ka = Sk[a * K + min(pa, K - 1)], kb = Sk[bb * K + min(pb, K - 1)];
        const int64_t ia = pa < K ? Si[a * K + pa] : INT64_MAX;
        const int64_t ib = pb < K ? Si[bb * K + pb] : INT64_MAX;
        const float kav = pa < K ? ka : INFINITY, kbv = pb < K ? kb : INFINITY;
        const bool takea = key_less(kav, ia, kbv, ib);
        mk[t] = takea ? kav : kbv;
        mi[t] = takea ? ia : ib;
        pa += takea ? 1 : 0;
        pb += takea ? 0 : 1;
      }
#pragma unroll
      for (int t = 0; t < K; ++t) {
        Sk[a * K + t] = mk[t];
        Si[a * K + t] = mi[t];
      }
    }
    __syncthreads();
  }
  if (tid < k) {
    const float kk = Sk[tid];
    const int64_t ii = Si[tid];
    const float val = (metric == 1) ? -kk : kk;
    out_val[(int64_t)q * k + tid] = ii == INT64_MAX ? NAN : val;
    out_id[(int64_t)q * k + tid] = ii == INT64_MAX ? -1 : ii;
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

template <int K>
int launch_merge(const float* ck, const int64_t* ci, int b, int64_t n_cand, int k,
                 int keys_are_values, int metric, float* od, int64_t* oi, hipStream_t s) {
  constexpr int NT = K >= 64 ? 128 : 256;
  const size_t lds = (size_t)NT * K * (sizeof(float) + sizeof(int64_t));
  hipLaunchKernelGGL((merge_kernel<K, NT>), dim3(b), dim3(NT), lds, s, ck, ci, n_cand, k,
                     keys_are_values, metric, od, oi);
  MPR_LAUNCHED();
  return MPR_OK;
}

int merge_dispatch(const float* ck, const int64_t* ci, int b, int64_t n_cand, int k,
                   int keys_are_values, int metric, float* od, int64_t* oi, hipStream_t s) {
  switch (list_cap(k)) {
    case 1: return launch_merge<1>(ck, ci, b, n_cand, k, keys_are_values, metric, od, oi, s);
    case 2: return launch_merge<2>(ck, ci, b, n_cand, k, keys_are_values, metric, od, oi, s);
    case 4: return launch_merge<4>(ck, ci, b, n_cand, k, keys_are_values, metric, od, oi, s);
    case 8: return launch_merge<8>(ck, ci, b, n_cand, k, keys_are_values, metric, od, oi, s);
    case 16: return launch_merge<16>(ck, ci, b, n_cand, k, keys_are_values, metric, od, oi, s);
    case 32: return launch_merge<32>(ck, ci, b, n_cand, k, keys_are_values, metric, od, oi, s);
    case 64: return launch_merge<64>(ck, ci, b, n_cand, k, keys_are_values, metric, od, oi, s);
  }
  set_error("top-k: k=%d unsupported (1..64)", k);
  return MPR_EUNSUP;
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

template <int K>
int launch_scan_mm(const float* X, int64_t n, int d, int64_t row_offset, int metric,
                   const float* Q, float* qn, int b, float* ck, int64_t* ci, hipStream_t s) {
  const int nqt = (int)cdiv(b, SM_B), RB = scan_mm_rowblocks(n, b);
  hipLaunchKernelGGL(qnorm_kernel, dim3((unsigned)cdiv(b, 4)), dim3(256), 0, s, Q, b, d, qn);
  hipLaunchKernelGGL((scan_mm_kernel<K>), dim3((unsigned)(nqt * RB)), dim3(256), 0, s, X, n, d,
                     row_offset, metric, Q, qn, b, nqt, RB, ck, ci);
  MPR_LAUNCHED();
  return MPR_OK;
}

size_t scan_topk_workspace(int64_t n, int b, int k) {
  const int K = list_cap(k);
  const int64_t per_q = std::max<int64_t>(scan_blocks(n), scan_mm_rowblocks(n, b));
  return (size_t)b * per_q * K * (sizeof(float) + sizeof(int64_t)) + (size_t)b * 4 + 512;
}

int scan_topk(const float* X, const float* xnorm, int64_t n, int d, int64_t row_offset,
              int metric, const float* Q, int b, int k, float* ws, size_t ws_bytes,
              float* out_dist, int64_t* out_ids, hipStream_t s) {
  MPR_REQUIRE(k >= 1 && k <= 64, "search: k=%d must be in [1, 64]", k);
  MPR_REQUIRE(k <= n, "search: k=%d exceeds index rows %lld", k, (long long)n);
  MPR_REQUIRE(d % 16 == 0 && d <= 8192, "search: d=%d must be a multiple of 16", d);
  MPR_REQUIRE(b >= 0, "search: b<0");
  if (b == 0) return MPR_OK;
  MPR_REQUIRE(ws_bytes >= scan_topk_workspace(n, b, k), "search: workspace too small");
  const int K = list_cap(k);
  if (use_scan_mm(n, d, b, k) && !getenv("MPR_SCAN_MM_OFF")) {
    const int RB = scan_mm_rowblocks(n, b);
    int64_t* ci = reinterpret_cast<int64_t*>(ws);
    float* ck = reinterpret_cast<float*>(ci + (size_t)b * RB * K);
    float* qn = ck + (size_t)b * RB * K;
    int rc = MPR_EUNSUP;
    switch (K) {
      case 1: rc = launch_scan_mm<1>(X, n, d, row_offset, metric, Q, qn, b, ck, ci, s); break;
      case 2: rc = launch_scan_mm<2>(X, n, d, row_offset, metric, Q, qn, b, ck, ci, s); break;
      case 4: rc = launch_scan_mm<4>(X, n, d, row_offset, metric, Q, qn, b, ck, ci, s); break;
      case 8: rc = launch_scan_mm<8>(X, n, d, row_offset, metric, Q, qn, b, ck, ci, s); break;
      case 16: rc = launch_scan_mm<16>(X, n, d, row_offset, metric, Q, qn, b, ck, ci, s); break;
    }
    if (rc != MPR_OK) return rc;
    return merge_dispatch(ck, ci, b, (int64_t)RB * K, k, /*keys_are_values=*/0, metric, out_dist,
                          out_ids, s);
  }
  const int64_t nb = scan_blocks(n);
  int64_t* ci = reinterpret_cast<int64_t*>(ws);
  float* ck = reinterpret_cast<float*>(ci + (size_t)b * nb * K);
  int rc = MPR_EUNSUP;
  switch (K) {
    case 1: rc = launch_scan<1>(X, xnorm, n, d, row_offset, metric, Q, b, ck, ci, s); break;
    case 2: rc = launch_scan<2>(X, xnorm, n, d, row_offset, metric, Q, b, ck, ci, s); break;
    case 4: rc = launch_scan<4>(X, xnorm, n, d, row_offset, metric, Q, b, ck, ci, s); break;
    case 8: rc = launch_scan<8>(X, xnorm, n, d, row_offset, metric, Q, b, ck, ci, s); break;
    case 16: rc = launch_scan<16>(X, xnorm, n, d, row_offset, metric, Q, b, ck, ci, s); break;
    case 32: rc = launch_scan<32>(X, xnorm, n, d, row_offset, metric, Q, b, ck, ci, s); break;
    case 64: rc = launch_scan<64>(X, xnorm, n, d, row_offset, metric, Q, b, ck, ci, s); break;
  }
  if (rc != MPR_OK) return rc;
  return merge_dispatch(ck, ci, b, nb * K, k, /*keys_are_values=*/0, metric, out_dist, out_ids, s);
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
  MPR_REQUIRE(k >= 1 && k <= 64 && k <= n_cand, "merge: k=%d n_cand=%lld", k, (long long)n_cand);
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
