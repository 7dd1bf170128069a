// train.hip — the kernels of the teacher-forced T5 training step (SURVEY.md §8(f) rank 3:
// main.py:177-188 calls loss.backward() on architectures/T5VisionModel.py:219-234, i.e. on
// transformers' T5ForConditionalGeneration(inputs_embeds, attention_mask, labels).loss).
//
// The dense projections and their two backward products run on the tiled fp32-accurate GEMM
// (gemm.hip): Y = X W^T, dX = dY W (W^T staged by transpose_kernel), dW = dY^T X (dY^T, X^T
// staged).  What is T5-specific lives here, each a small latency-bound kernel sized for the
// training shapes (B x L rows of 512-768, L <= 1024 keys, head dim 64):
//   rmsnorm forward (saves 1/rms) and backward (dx per row; dw by a column-block reduction with
//   a fixed summation order — every gradient here is deterministic, no float atomics);
//   attention forward with the probabilities kept ([B, H, Lq, Lk]) and backward in two passes
//   (per query row: dS and dQ; per key row: dK and dV), plus the relative-position-bias
//   gradient by offset (summed over batch and rows) and its scatter onto the bucket table;
//   ReLU backward; cross-entropy forward+backward over the vocabulary; the embedding gather and
//   its backward (rows grouped per token id on the host, summed in order).
#include <cfloat>
#include <climits>
#include <cmath>

#include "kernels.h"

namespace mpr {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// a wave's own LDS writes, seen by all its lanes before they read (wave-private LDS slots)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}

// out[c][r] = in[r][c] (out row stride ld_out >= rows, zeros in r >= rows: a GEMM K padded to
// a multiple of 4); 32 x 32 tiles through LDS (+1 column: conflict-free)
__global__ __launch_bounds__(256) void transpose_kernel(const float* __restrict__ in, int64_t rows,
                                                        int64_t cols, int64_t ld_in,
                                                        float* __restrict__ out, int64_t ld_out) {
  __shared__ float t[32][33];
  const int64_t r0 = (int64_t)blockIdx.y * 32, c0 = (int64_t)blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 8 rows of 32
#pragma unroll
  for (int j = 0; j < 32; j += 8) {
    const int64_t r = r0 + ty + j, c = c0 + tx;
    t[ty + j][tx] = (r < rows && c < cols) ? in[r * ld_in + c] : 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 32; j += 8) {
    const int64_t c = c0 + ty + j, r = r0 + tx;
    if (c < cols && r < ld_out) out[c * ld_out + r] = t[tx][ty + j];
  }
}

// T5LayerNorm: y = (x * rsqrt(mean(x^2) + eps) * w) * scale (scale: the decoder output's
// d_model^-0.5 before the tied lm_head, else 1); wave per row, rstd saved
__global__ __launch_bounds__(256) void rms_fwd_kernel(const float* __restrict__ x, int M, int D,
                                                      const float* __restrict__ w, float eps,
                                                      float scale, float* __restrict__ y,
                                                      float* __restrict__ rstd) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;
  const float* xr = x + (int64_t)row * D;
  float ss = 0.f;
  for (int c = lane; c < D; c += 64) ss += xr[c] * xr[c];
  ss = wave_sum(ss);
  const float r = rsqrtf(ss / (float)D + eps);
  for (int c = lane; c < D; c += 64) y[(int64_t)row * D + c] = xr[c] * r * w[c] * scale;
  if (lane == 0) rstd[row] = r;
}

// dx = r * (w*g - xhat * mean(w*g*xhat)), g = dy*scale, xhat = x*r; dx (+)= (accumulate flag)
__global__ __launch_bounds__(256) void rms_bwd_dx_kernel(const float* __restrict__ x, int M, int D,
                                                         const float* __restrict__ w,
                                                         const float* __restrict__ rstd,
                                                         const float* __restrict__ dy, float scale,
                                                         float* __restrict__ dx, int accumulate) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;
  const float r = rstd[row];
  const float* xr = x + (int64_t)row * D;
  const float* g = dy + (int64_t)row * D;
  float s = 0.f;
  for (int c = lane; c < D; c += 64) s += w[c] * (g[c] * scale) * xr[c] * r;
  s = wave_sum(s) / (float)D;
  float* o = dx + (int64_t)row * D;
  for (int c = lane; c < D; c += 64) {
    const float v = r * (w[c] * (g[c] * scale) - xr[c] * r * s);
    o[c] = accumulate ? o[c] + v : v;
  }
}

// dw[c] = sum_rows dy * scale * x * r: block per 64 columns, 4 row groups, fixed order
__global__ __launch_bounds__(256) void rms_bwd_dw_kernel(const float* __restrict__ x, int M, int D,
                                                         const float* __restrict__ rstd,
                                                         const float* __restrict__ dy, float scale,
                                                         float* __restrict__ dw) {
  __shared__ float part[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), g = threadIdx.x >> 6;
  float s = 0.f;
  if (c < D)
    for (int row = g; row < M; row += 4)
      s += (dy[(int64_t)row * D + c] * scale) * x[(int64_t)row * D + c] * rstd[row];
  part[g][threadIdx.x & 63] = s;
  __syncthreads();
  if (g == 0 && c < D) dw[c] = (part[0][threadIdx.x] + part[1][threadIdx.x]) +
                               (part[2][threadIdx.x] + part[3][threadIdx.x]);
}

// The same sum over 64-row chunks: part[chunk, c] (grid D/64 x chunks: the chip fills at
// training sizes, where one block per 64 columns walked ~2K rows at memory latency, 42 us), then
// dw[c] = sum over chunks in chunk order.  Fixed order: deterministic.
constexpr int RMS_DW_CHUNK = 64;
__global__ __launch_bounds__(256) void rms_dw_part_kernel(const float* __restrict__ x, int M, int D,
                                                          const float* __restrict__ rstd,
                                                          const float* __restrict__ dy,
                                                          float scale, float* __restrict__ part) {
  __shared__ float ps[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), g = threadIdx.x >> 6;
  const int r0 = blockIdx.y * RMS_DW_CHUNK, r1 = min(M, r0 + RMS_DW_CHUNK);
  float s = 0.f;
  if (c < D)
    for (int row = r0 + g; row < r1; row += 4)
      s += (dy[(int64_t)row * D + c] * scale) * x[(int64_t)row * D + c] * rstd[row];
  ps[g][threadIdx.x & 63] = s;
  __syncthreads();
  if (g == 0 && c < D)
    part[(int64_t)blockIdx.y * D + c] = (ps[0][threadIdx.x] + ps[1][threadIdx.x]) +
                                        (ps[2][threadIdx.x] + ps[3][threadIdx.x]);
}

__global__ void sum_rows_kernel(const float* __restrict__ part, int rows, int64_t n,
                                float* __restrict__ out) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= n) return;
  float s = 0.f;
  for (int r = 0; r < rows; ++r) s += part[(int64_t)r * n + c];
  out[c] = s;
}

// Split-K GEMM epilogue: C = act(sum_s part[s]) + R, splits summed in order
__global__ void splitk_reduce_kernel(const float* __restrict__ part, int splits, int M, int N,
                                     int act, const float* R, int64_t ldr, float* C, int64_t ldc) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)M * N) return;
  const int64_t m = e / N, n = e % N;
  float s = 0.f;
  for (int k = 0; k < splits; ++k) s += part[(int64_t)k * M * N + e];
  if (act == ACT_RELU) s = fmaxf(s, 0.f);
  if (R) s += R[m * ldr + n];
  C[m * ldc + n] = s;
}

// Counter-based dropout mask (train mode: T5's nn.Dropout / functional dropout sites): element
// idx of site `site` under a forward's seed is kept iff the top 24 bits of a splitmix64 mix of
// (seed, site, idx) are >= thresh (= p * 2^24), kept elements scaled by 1 / (1 - p).  Nothing is
// stored: the backward regenerates the same mask.  thresh == 0: identity.
struct Drop {
  uint64_t seed;
  uint32_t site, thresh;
  float scale;
};
__device__ __forceinline__ float drop_factor(const Drop& d, uint64_t idx) {
  if (d.thresh == 0) return 1.f;
  uint64_t x = d.seed ^ ((uint64_t)d.site * 0x9E3779B97F4A7C15ull);
  x += idx * 0xD1B54A32D192ED03ull;
  x ^= x >> 30;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27;
  x *= 0x94D049BB133111EBull;
  x ^= x >> 31;
  return (uint32_t)(x >> 40) >= d.thresh ? d.scale : 0.f;
}

// y[e] = (r ? r[e] : 0) + x[e] * mask[e]   (y may alias x or r)
__global__ void dropout_kernel(const float* x, int64_t n, Drop d, const float* r, float* y) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n) return;
  const float v = x[e] * drop_factor(d, (uint64_t)e);
  y[e] = r ? r[e] + v : v;
}

struct TrainAttn {
  const float *q, *k, *v;  // row (b, i) of head h at base + b*bs + i*rs + h*64
  int64_t q_bs, q_rs, k_bs, k_rs, v_bs, v_rs;
  int B, H, Lq, Lk;
  int causal;
  const float* key_mask;  // [B, Lk] 1/0, optional
  const float* rel;       // per offset [(j - i + R) * H + h], optional
  int R;
  Drop drop;              // on the probabilities (index (b, h, i, j) of P), applied in P V only
};

// Wave per (b, h, query row i): lane per key for the scores and the softmax (P row kept in the
// wave's LDS slot and written to P), lane per output column for O = P V.  Masked keys (mask 0,
// or j > i when causal) get probability 0, as the additive finfo.min mask of transformers does
// whenever a row has a visible key.
constexpr int TA_MAXK = 1024;
__global__ __launch_bounds__(256) void attn_fwd_kernel(TrainAttn a, float* __restrict__ o,
                                                       int64_t o_bs, int64_t o_rs,
                                                       float* __restrict__ P) {
  __shared__ float prow[4][TA_MAXK];
  __shared__ float qs[4][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t item = (int64_t)blockIdx.x * 4 + wave;  // (b, h, i)
  if (item >= (int64_t)a.B * a.H * a.Lq) return;
  const int i = (int)(item % a.Lq), h = (int)((item / a.Lq) % a.H), b = (int)(item / ((int64_t)a.Lq * a.H));
  qs[wave][lane] = a.q[b * a.q_bs + i * a.q_rs + h * 64 + lane];
  wave_lds_sync();
  float mx = -INFINITY;
  for (int j = lane; j < a.Lk; j += 64) {
    const bool vis = (!a.causal || j <= i) && (!a.key_mask || a.key_mask[(int64_t)b * a.Lk + j] != 0.f);
    float s = -INFINITY;
    if (vis) {
      const float* kr = a.k + b * a.k_bs + j * a.k_rs + h * 64;
      s = 0.f;
#pragma unroll 16
      for (int c = 0; c < 64; ++c) s += qs[wave][c] * kr[c];
      if (a.rel) s += a.rel[(int64_t)(j - i + a.R) * a.H + h];
    }
    prow[wave][j] = s;
    mx = fmaxf(mx, s);
  }
  mx = wave_max(mx);
  float sum = 0.f;
  for (int j = lane; j < a.Lk; j += 64) {
    const float s = prow[wave][j];
    const float e = s == -INFINITY ? 0.f : expf(s - mx);
    prow[wave][j] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  const float inv = sum > 0.f ? 1.f / sum : 0.f;
  float* Pr = P + item * a.Lk;
  for (int j = lane; j < a.Lk; j += 64) {
    const float p = prow[wave][j] * inv;
    prow[wave][j] = p * drop_factor(a.drop, (uint64_t)item * a.Lk + j);  // dropout(P) V
    Pr[j] = p;
  }
  wave_lds_sync();
  float acc = 0.f;
  for (int j = 0; j < a.Lk; ++j) acc += prow[wave][j] * a.v[b * a.v_bs + j * a.v_rs + h * 64 + lane];
  o[b * o_bs + i * o_rs + h * 64 + lane] = acc;
}

// Pass 1, wave per (b, h, i): dP_ij = (dO_i . V_j) m_ij (lane per key; m the dropout factor of
// P_ij), D_i = sum_j P_ij dP_ij, dS_ij = P_ij (dP_ij - D_i) (kept in dS), dQ_i = sum_j dS_ij K_j
// (lane per column).
__global__ __launch_bounds__(256) void attn_bwd_q_kernel(TrainAttn a, const float* __restrict__ P,
                                                         const float* __restrict__ dO,
                                                         int64_t do_bs, int64_t do_rs,
                                                         float* __restrict__ dS,
                                                         float* __restrict__ dq, int64_t dq_bs,
                                                         int64_t dq_rs) {
  __shared__ float srow[4][TA_MAXK];
  __shared__ float gs[4][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t item = (int64_t)blockIdx.x * 4 + wave;
  if (item >= (int64_t)a.B * a.H * a.Lq) return;
  const int i = (int)(item % a.Lq), h = (int)((item / a.Lq) % a.H), b = (int)(item / ((int64_t)a.Lq * a.H));
  gs[wave][lane] = dO[b * do_bs + i * do_rs + h * 64 + lane];
  wave_lds_sync();
  const float* Pr = P + item * a.Lk;
  float dsum = 0.f;
  for (int j = lane; j < a.Lk; j += 64) {
    const float p = Pr[j];
    float dp = 0.f;
    if (p != 0.f) {
      const float* vr = a.v + b * a.v_bs + j * a.v_rs + h * 64;
#pragma unroll 16
      for (int c = 0; c < 64; ++c) dp += gs[wave][c] * vr[c];
      dp *= drop_factor(a.drop, (uint64_t)item * a.Lk + j);
    }
    srow[wave][j] = dp;
    dsum += p * dp;
  }
  dsum = wave_sum(dsum);
  float* dSr = dS + item * a.Lk;
  for (int j = lane; j < a.Lk; j += 64) {
    const float ds = Pr[j] * (srow[wave][j] - dsum);
    srow[wave][j] = ds;
    dSr[j] = ds;
  }
  wave_lds_sync();
  float acc = 0.f;
  for (int j = 0; j < a.Lk; ++j) acc += srow[wave][j] * a.k[b * a.k_bs + j * a.k_rs + h * 64 + lane];
  dq[b * dq_bs + i * dq_rs + h * 64 + lane] = acc;
}

// Pass 2, wave per (b, h, key row j), lane per column: dV_j = sum_i P_ij m_ij dO_i,
// dK_j = sum_i dS_ij Q_i.
__global__ __launch_bounds__(256) void attn_bwd_kv_kernel(TrainAttn a, const float* __restrict__ P,
                                                          const float* __restrict__ dS,
                                                          const float* __restrict__ dO,
                                                          int64_t do_bs, int64_t do_rs,
                                                          float* __restrict__ dk, int64_t dk_bs,
                                                          int64_t dk_rs, float* __restrict__ dv,
                                                          int64_t dv_bs, int64_t dv_rs) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t item = (int64_t)blockIdx.x * 4 + wave;  // (b, h, j)
  if (item >= (int64_t)a.B * a.H * a.Lk) return;
  const int j = (int)(item % a.Lk), h = (int)((item / a.Lk) % a.H), b = (int)(item / ((int64_t)a.Lk * a.H));
  const int64_t base = ((int64_t)b * a.H + h) * a.Lq;  // (b, h, i = 0) row of P / dS
  float gv = 0.f, gk = 0.f;
  for (int i = 0; i < a.Lq; ++i) {
    const float p = P[(base + i) * a.Lk + j] * drop_factor(a.drop, (uint64_t)(base + i) * a.Lk + j);
    const float ds = dS[(base + i) * a.Lk + j];
    gv += p * dO[b * do_bs + i * do_rs + h * 64 + lane];
    gk += ds * a.q[b * a.q_bs + i * a.q_rs + h * 64 + lane];
  }
  dv[b * dv_bs + j * dv_rs + h * 64 + lane] = gv;
  dk[b * dk_bs + j * dk_rs + h * 64 + lane] = gk;
}

// ---- block per (b, h) forms (Lq, Lk <= 128: the training shapes) ------------------------------
// The wave-per-row kernels above re-read the (b, h) K / V (or dO / Q) rows from L2 once per row:
// at L = 121 that is 121 x 62 KB per (b, h), 24-34 us per launch.  These stage them in LDS once
// per (b, h) block (row stride 65: a lane per key reading its row is conflict-free) and run the
// same per-row arithmetic in the same order — bit-identical results — with 8 waves taking the
// rows in turn.
constexpr int TB_MAXL = 128;
constexpr int TB_LD = 65;
constexpr int TB_WAVES = 8;

__device__ __forceinline__ void tb_stage(const float* __restrict__ src, int64_t rs, int rows,
                                         float* dst) {
  for (int e = threadIdx.x; e < rows * 64; e += 64 * TB_WAVES)
    dst[(e >> 6) * TB_LD + (e & 63)] = src[(int64_t)(e >> 6) * rs + (e & 63)];
}

__global__ __launch_bounds__(64 * TB_WAVES) void attn_fwd_bh_kernel(TrainAttn a,
                                                                    float* __restrict__ o,
                                                                    int64_t o_bs, int64_t o_rs,
                                                                    float* __restrict__ P) {
  __shared__ float Ks[TB_MAXL * TB_LD], Vs[TB_MAXL * TB_LD];
  __shared__ float prow[TB_WAVES][TB_MAXL];
  __shared__ float qs[TB_WAVES][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int h = blockIdx.x % a.H, b = blockIdx.x / a.H;
  tb_stage(a.k + b * a.k_bs + h * 64, a.k_rs, a.Lk, Ks);
  tb_stage(a.v + b * a.v_bs + h * 64, a.v_rs, a.Lk, Vs);
  __syncthreads();
  for (int i = wave; i < a.Lq; i += TB_WAVES) {
    const int64_t item = ((int64_t)b * a.H + h) * a.Lq + i;
    qs[wave][lane] = a.q[b * a.q_bs + i * a.q_rs + h * 64 + lane];
    wave_lds_sync();
    float mx = -INFINITY;
    for (int j = lane; j < a.Lk; j += 64) {
      const bool vis = (!a.causal || j <= i) && (!a.key_mask || a.key_mask[(int64_t)b * a.Lk + j] != 0.f);
      float s = -INFINITY;
      if (vis) {
        const float* kr = Ks + j * TB_LD;
        s = 0.f;
#pragma unroll 16
        for (int c = 0; c < 64; ++c) s += qs[wave][c] * kr[c];
        if (a.rel) s += a.rel[(int64_t)(j - i + a.R) * a.H + h];
      }
      prow[wave][j] = s;
      mx = fmaxf(mx, s);
    }
    mx = wave_max(mx);
    float sum = 0.f;
    for (int j = lane; j < a.Lk; j += 64) {
      const float s = prow[wave][j];
      const float e = s == -INFINITY ? 0.f : expf(s - mx);
      prow[wave][j] = e;
      sum += e;
    }
    sum = wave_sum(sum);
    const float inv = sum > 0.f ? 1.f / sum : 0.f;
    float* Pr = P + item * a.Lk;
    for (int j = lane; j < a.Lk; j += 64) {
      const float p = prow[wave][j] * inv;
      prow[wave][j] = p * drop_factor(a.drop, (uint64_t)item * a.Lk + j);
      Pr[j] = p;
    }
    wave_lds_sync();
    float acc = 0.f;
    for (int j = 0; j < a.Lk; ++j) acc += prow[wave][j] * Vs[j * TB_LD + lane];
    o[b * o_bs + i * o_rs + h * 64 + lane] = acc;
    wave_lds_sync();  // this row's qs / prow reads done before the next row's writes
  }
}

__global__ __launch_bounds__(64 * TB_WAVES) void attn_bwd_q_bh_kernel(
    TrainAttn a, const float* __restrict__ P, const float* __restrict__ dO, int64_t do_bs,
    int64_t do_rs, float* __restrict__ dS, float* __restrict__ dq, int64_t dq_bs, int64_t dq_rs) {
  __shared__ float Ks[TB_MAXL * TB_LD], Vs[TB_MAXL * TB_LD];
  __shared__ float srow[TB_WAVES][TB_MAXL];
  __shared__ float gs[TB_WAVES][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int h = blockIdx.x % a.H, b = blockIdx.x / a.H;
  tb_stage(a.k + b * a.k_bs + h * 64, a.k_rs, a.Lk, Ks);
  tb_stage(a.v + b * a.v_bs + h * 64, a.v_rs, a.Lk, Vs);
  __syncthreads();
  for (int i = wave; i < a.Lq; i += TB_WAVES) {
    const int64_t item = ((int64_t)b * a.H + h) * a.Lq + i;
    gs[wave][lane] = dO[b * do_bs + i * do_rs + h * 64 + lane];
    wave_lds_sync();
    const float* Pr = P + item * a.Lk;
    float dsum = 0.f;
    for (int j = lane; j < a.Lk; j += 64) {
      const float p = Pr[j];
      float dp = 0.f;
      if (p != 0.f) {
        const float* vr = Vs + j * TB_LD;
#pragma unroll 16
        for (int c = 0; c < 64; ++c) dp += gs[wave][c] * vr[c];
        dp *= drop_factor(a.drop, (uint64_t)item * a.Lk + j);
      }
      srow[wave][j] = dp;
      dsum += p * dp;
    }
    dsum = wave_sum(dsum);
    float* dSr = dS + item * a.Lk;
    for (int j = lane; j < a.Lk; j += 64) {
      const float ds = Pr[j] * (srow[wave][j] - dsum);
      srow[wave][j] = ds;
      dSr[j] = ds;
    }
    wave_lds_sync();
    float acc = 0.f;
    for (int j = 0; j < a.Lk; ++j) acc += srow[wave][j] * Ks[j * TB_LD + lane];
    dq[b * dq_bs + i * dq_rs + h * 64 + lane] = acc;
    wave_lds_sync();
  }
}

// per key row j: its column of P (times the dropout factor) and of dS staged per wave, then
// dV_j = sum_i Pm_ij dO_i, dK_j = sum_i dS_ij Q_i in row order
__global__ __launch_bounds__(64 * TB_WAVES) void attn_bwd_kv_bh_kernel(
    TrainAttn a, const float* __restrict__ P, const float* __restrict__ dS,
    const float* __restrict__ dO, int64_t do_bs, int64_t do_rs, float* __restrict__ dk,
    int64_t dk_bs, int64_t dk_rs, float* __restrict__ dv, int64_t dv_bs, int64_t dv_rs) {
  __shared__ float Gs[TB_MAXL * TB_LD], Qs[TB_MAXL * TB_LD];
  __shared__ float pc[TB_WAVES][TB_MAXL], dc[TB_WAVES][TB_MAXL];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int h = blockIdx.x % a.H, b = blockIdx.x / a.H;
  tb_stage(dO + b * do_bs + h * 64, do_rs, a.Lq, Gs);
  tb_stage(a.q + b * a.q_bs + h * 64, a.q_rs, a.Lq, Qs);
  __syncthreads();
  const int64_t base = ((int64_t)b * a.H + h) * a.Lq;  // (b, h, i = 0) row of P / dS
  for (int j = wave; j < a.Lk; j += TB_WAVES) {
    for (int i = lane; i < a.Lq; i += 64) {
      pc[wave][i] = P[(base + i) * a.Lk + j] * drop_factor(a.drop, (uint64_t)(base + i) * a.Lk + j);
      dc[wave][i] = dS[(base + i) * a.Lk + j];
    }
    wave_lds_sync();
    float gv = 0.f, gk = 0.f;
    for (int i = 0; i < a.Lq; ++i) {
      gv += pc[wave][i] * Gs[i * TB_LD + lane];
      gk += dc[wave][i] * Qs[i * TB_LD + lane];
    }
    dv[b * dv_bs + j * dv_rs + h * 64 + lane] = gv;
    dk[b * dk_bs + j * dk_rs + h * 64 + lane] = gk;
    wave_lds_sync();
  }
}

// d(rel)[off][h] += sum_{b, i} dS[b, h, i, i + off - R]: block per (off, h), fixed order
__global__ __launch_bounds__(256) void attn_bwd_rel_kernel(const float* __restrict__ dS, int B,
                                                           int H, int Lq, int Lk, int R,
                                                           float* __restrict__ drel) {
  __shared__ float part[256];
  const int off = blockIdx.x, h = blockIdx.y, t = threadIdx.x;  // off in [0, 2R]
  const int rel = off - R;
  float s = 0.f;
  for (int64_t bi = t; bi < (int64_t)B * Lq; bi += 256) {
    const int b = (int)(bi / Lq), i = (int)(bi % Lq), j = i + rel;
    if (j >= 0 && j < Lk) s += dS[(((int64_t)b * H + h) * Lq + i) * Lk + j];
  }
  part[t] = s;
  __syncthreads();
  for (int w = 128; w >= 1; w >>= 1) {
    if (t < w) part[t] += part[t + w];
    __syncthreads();
  }
  if (t == 0) drel[(int64_t)off * H + h] += part[0];
}

// table gradient: dtab[bucket][h] += sum of drel[off][h] over offsets with lut[off] == bucket
__global__ void rel_scatter_kernel(const float* __restrict__ drel, const int32_t* __restrict__ lut,
                                   int R, int nb, int H, float* __restrict__ dtab) {
  const int bucket = blockIdx.x, h = threadIdx.x;
  if (h >= H) return;
  float s = 0.f;
  for (int off = 0; off <= 2 * R; ++off)
    if (lut[off] == bucket) s += drel[(int64_t)off * H + h];
  dtab[(int64_t)bucket * H + h] += s;
}

// rel[off][h] = table[lut[off]][h]
__global__ void rel_gather_kernel(const float* __restrict__ table, const int32_t* __restrict__ lut,
                                  int R, int H, float* __restrict__ rel) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)(2 * R + 1) * H) return;
  rel[e] = table[(int64_t)lut[e / H] * H + e % H];
}

__global__ void relu_bwd_kernel(const float* __restrict__ y, const float* __restrict__ dy,
                                int64_t n, float* __restrict__ dx) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e < n) dx[e] = y[e] > 0.f ? dy[e] : 0.f;
}

__global__ void add_kernel(const float* __restrict__ a, const float* __restrict__ b, int64_t n,
                           float* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e < n) out[e] = a[e] + b[e];
}

// Cross-entropy over rows of logits (ignore label -100): per row loss = lse - logit[label] into
// row_loss (0 for ignored), dlogits = (softmax - onehot) * grad_scale (0 rows when ignored).
__global__ __launch_bounds__(256) void ce_rows_kernel(const float* __restrict__ logits, int64_t n,
                                                      int V, const int32_t* __restrict__ labels,
                                                      float grad_scale,
                                                      const float* __restrict__ grad_mult,
                                                      float* __restrict__ row_loss,
                                                      float* __restrict__ dlogits, int64_t ldd) {
  __shared__ float red[4];
  const int64_t row = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const float* lr = logits + row * V;
  float* dr = dlogits ? dlogits + row * ldd : nullptr;
  const int lab = labels[row];
  if (lab < 0) {
    if (dr)
      for (int c = t; c < ldd; c += 256) dr[c] = 0.f;
    if (t == 0) row_loss[row] = 0.f;
    return;
  }
  float mx = -INFINITY;
  for (int c = t; c < V; c += 256) mx = fmaxf(mx, lr[c]);
  mx = wave_max(mx);
  if (lane == 0) red[wave] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float s = 0.f;
  for (int c = t; c < V; c += 256) s += expf(lr[c] - mx);
  s = wave_sum(s);
  if (lane == 0) red[wave] = s;
  __syncthreads();
  s = (red[0] + red[1]) + (red[2] + red[3]);
  const float lse = mx + logf(s);
  if (t == 0) row_loss[row] = lse - lr[lab];
  if (dr) {
    const float inv = 1.f / s;
    if (grad_mult) grad_scale *= grad_mult[0];
    for (int c = t; c < ldd; c += 256)  // columns V .. ldd: zero padding (a GEMM K)
      dr[c] = c < V ? (expf(lr[c] - mx) * inv - (c == lab ? 1.f : 0.f)) * grad_scale : 0.f;
  }
}

// loss = sum(row_loss) * scale in row order (one block)
__global__ __launch_bounds__(256) void sum_scale_kernel(const float* __restrict__ x, int64_t n,
                                                        float scale, float* __restrict__ out) {
  __shared__ float part[256];
  float s = 0.f;
  for (int64_t e = threadIdx.x; e < n; e += 256) s += x[e];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w >= 1; w >>= 1) {
    if ((int)threadIdx.x < w) part[threadIdx.x] += part[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = part[0] * scale;
}

__global__ void gather_rows_kernel(const float* __restrict__ table, const int32_t* __restrict__ ids,
                                   int64_t n, int d, float* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n * d) return;
  out[e] = table[(int64_t)ids[e / d] * d + e % d];
}

// dW[uniq[u]] += sum over pos[offs[u] .. offs[u+1]) of dY[pos] (block per unique id, in order)
__global__ __launch_bounds__(256) void embed_bwd_kernel(const float* __restrict__ dY, int d,
                                                        const int32_t* __restrict__ uniq,
                                                        const int32_t* __restrict__ offs,
                                                        const int32_t* __restrict__ pos,
                                                        float* __restrict__ dW) {
  const int u = blockIdx.x;
  const int lo = offs[u], hi = offs[u + 1];
  float* o = dW + (int64_t)uniq[u] * d;
  for (int c = threadIdx.x; c < d; c += 256) {
    float s = 0.f;
    for (int p = lo; p < hi; ++p) s += dY[(int64_t)pos[p] * d + c];
    o[c] += s;
  }
}

template <class F>
int guarded_call(F&& f) {
  try {
    return f();
  } catch (...) {
    set_error("train: exception");
    return MPR_EINVAL;
  }
}
inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

TrainAttn make_attn(const float* q, int64_t q_bs, int64_t q_rs, const float* k, int64_t k_bs,
                    int64_t k_rs, const float* v, int64_t v_bs, int64_t v_rs, int B, int H,
                    int Lq, int Lk, int causal, const float* mask, const float* rel, int R) {
  TrainAttn a;
  a.q = q; a.q_bs = q_bs; a.q_rs = q_rs;
  a.k = k; a.k_bs = k_bs; a.k_rs = k_rs;
  a.v = v; a.v_bs = v_bs; a.v_rs = v_rs;
  a.B = B; a.H = H; a.Lq = Lq; a.Lk = Lk; a.causal = causal;
  a.key_mask = mask; a.rel = rel; a.R = R;
  a.drop = Drop{0, 0, 0, 1.f};
  return a;
}

}  // namespace
}  // namespace mpr

using namespace mpr;

extern "C" {

int mpr_gemm_f32(const float* A, int64_t lda, const float* W, int64_t ldw, float* C, int64_t ldc,
                 int32_t M, int32_t N, int32_t K, const float* R, int64_t ldr, int32_t act,
                 void* stream) {
  return guarded_call([&]() -> int {
    MPR_REQUIRE(act == ACT_NONE || act == ACT_RELU, "gemm: act %d (none or relu)", act);
    GemmArgs g;
    g.A = A; g.lda = lda; g.W = W; g.ldw = ldw; g.C = C; g.ldc = ldc;
    g.M = M; g.N = N; g.K = K; g.R = R; g.ldr = ldr; g.act = act;
    return gemm(g, S(stream));
  });
}

int mpr_pack_x3_bytes(int64_t N, int64_t K, int64_t* bytes) {
  return guarded_call([&]() -> int {
    MPR_REQUIRE(N > 0 && K > 0 && bytes, "pack_x3_bytes: N=%lld K=%lld", (long long)N,
                (long long)K);
    *bytes = packed_x3_bytes(N, K);
    return MPR_OK;
  });
}

int mpr_pack_x3(const float* W, int64_t N, int64_t K, int64_t ldw, void* out, int64_t out_bytes,
                void* stream) {
  return guarded_call([&]() -> int {
    MPR_REQUIRE(W && out && out_bytes >= packed_x3_bytes(N, K),
                "pack_x3: output of %lld bytes, %lld needed", (long long)out_bytes,
                (long long)packed_x3_bytes(N, K));
    return pack_x3(W, N, K, ldw, out, S(stream));
  });
}

int mpr_gemm_f32_packed(const float* A, int64_t lda, const float* W, int64_t ldw, const void* wp,
                        float* C, int64_t ldc, int32_t M, int32_t N, int32_t K, const float* R,
                        int64_t ldr, int32_t act, void* stream) {
  return guarded_call([&]() -> int {
    MPR_REQUIRE(act == ACT_NONE || act == ACT_RELU, "gemm: act %d (none or relu)", act);
    MPR_REQUIRE(wp != nullptr, "gemm_packed: no packed image");
    GemmArgs g;
    g.A = A; g.lda = lda; g.W = W; g.ldw = ldw; g.C = C; g.ldc = ldc; g.wp = wp;
    g.M = M; g.N = N; g.K = K; g.R = R; g.ldr = ldr; g.act = act;
    return gemm(g, S(stream));
  });
}

int mpr_gemm_f32_many(int32_t n, const int64_t* desc, void* stream) {
  return guarded_call([&]() -> int {
    MPR_REQUIRE(n >= 0 && n <= 64 && (n == 0 || desc), "gemm_many: %d problems", n);
    GemmGroup g;
    g.n = 0;
    for (int i = 0; i < n; ++i) {
      const int64_t* d = desc + 12 * i;
      GemmArgs& a = g.g[g.n];
      a = GemmArgs();
      a.A = reinterpret_cast<const float*>(d[0]); a.lda = d[1];
      a.W = reinterpret_cast<const float*>(d[2]); a.ldw = d[3];
      a.C = reinterpret_cast<float*>(d[4]); a.ldc = d[5];
      a.M = (int)d[6]; a.N = (int)d[7]; a.K = (int)d[8];
      a.R = reinterpret_cast<const float*>(d[9]); a.ldr = d[10]; a.act = (int)d[11];
      MPR_REQUIRE(a.act == ACT_NONE || a.act == ACT_RELU, "gemm_many: act %d", a.act);
      MPR_REQUIRE(a.M >= 0 && a.N >= 0 && a.K > 0, "gemm_many: bad shape M=%d N=%d K=%d", a.M,
                  a.N, a.K);
      if (a.M == 0 || a.N == 0) continue;
      if (++g.n == GEMM_GROUP) {
        MPR_TRY(gemm_group(g, S(stream)));
        g.n = 0;
      }
    }
    if (g.n) MPR_TRY(gemm_group(g, S(stream)));
    return MPR_OK;
  });
}

int mpr_gemm_f32_splitk(const float* A, int64_t lda, const float* W, int64_t ldw, float* C,
                        int64_t ldc, int32_t M, int32_t N, int32_t K, const float* R, int64_t ldr,
                        int32_t act, int32_t splits, float* partial, void* stream) {
  return guarded_call([&]() -> int {
    MPR_REQUIRE(act == ACT_NONE || act == ACT_RELU, "gemm: act %d (none or relu)", act);
    MPR_REQUIRE(splits >= 1 && splits <= 64 && partial, "gemm_splitk: splits=%d", splits);
    MPR_REQUIRE(M >= 0 && N >= 0 && K > 0, "gemm_splitk: bad shape M=%d N=%d K=%d", M, N, K);
    if (M == 0 || N == 0) return MPR_OK;
    const int kc = (int)cdiv(cdiv(K, splits), 32) * 32;  // chunk: a multiple of every BK
    const int full = K / kc, rem = K - full * kc, used = full + (rem > 0);
    GemmGroup g;
    g.n = 0;
    auto chunk = [&](int k0, int kk, int nb) {
      GemmArgs& a = g.g[g.n++];
      a = GemmArgs();
      a.A = A + k0; a.lda = lda; a.W = W + k0; a.ldw = ldw;
      a.C = partial + (int64_t)(k0 / kc) * M * N; a.ldc = N;
      a.M = M; a.N = N; a.K = kk;
      a.batch = nb; a.a_bs = kc; a.w_bs = kc; a.cb_bs = (int64_t)M * N;
    };
    if (gemm_uniform_order()) {  // the full chunks as one strided batch, one launch
      if (full) chunk(0, kc, full);
      if (rem) chunk(full * kc, rem, 1);
      MPR_TRY(gemm_group(g, S(stream)));
    } else {
      for (int c = 0; c < used; ++c) {
        chunk(c * kc, std::min(kc, K - c * kc), 1);
        if (g.n == GEMM_GROUP || c == used - 1) {
          MPR_TRY(gemm_group(g, S(stream)));
          g.n = 0;
        }
      }
    }
    const int64_t n = (int64_t)M * N;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, S(stream),
                       partial, used, M, N, act, R, ldr, C, ldc);
    MPR_LAUNCHED();
    return MPR_OK;
  });
}

int mpr_transpose(const float* in, int64_t rows, int64_t cols, int64_t ld_in, float* out,
                  int64_t ld_out, void* stream) {
  MPR_REQUIRE(ld_out >= rows, "transpose: ld_out %lld < rows %lld", (long long)ld_out,
              (long long)rows);
  if (rows == 0 || cols == 0) return MPR_OK;
  hipLaunchKernelGGL(transpose_kernel, dim3((unsigned)cdiv(cols, 32), (unsigned)cdiv(ld_out, 32)),
                     dim3(256), 0, S(stream), in, rows, cols, ld_in, out, ld_out);
  MPR_LAUNCHED();
  return MPR_OK;
}

int mpr_rmsnorm_fwd(const float* x, int32_t M, int32_t D, const float* w, float eps, float scale,
                    float* y, float* rstd, void* stream) {
  if (M == 0) return MPR_OK;
  hipLaunchKernelGGL(rms_fwd_kernel, dim3((unsigned)cdiv(M, 4)), dim3(256), 0, S(stream), x, M,
                     D, w, eps, scale, y, rstd);
  MPR_LAUNCHED();
  return MPR_OK;
}

int mpr_rmsnorm_bwd(const float* x, int32_t M, int32_t D, const float* w, const float* rstd,
                    const float* dy, float scale, float* dx, int32_t accumulate, float* dw,
                    float* dw_partial, void* stream) {
  if (M == 0) return MPR_OK;
  hipLaunchKernelGGL(rms_bwd_dx_kernel, dim3((unsigned)cdiv(M, 4)), dim3(256), 0, S(stream), x, M,
                     D, w, rstd, dy, scale, dx, accumulate);
  MPR_LAUNCHED();
  if (!dw_partial) {
    hipLaunchKernelGGL(rms_bwd_dw_kernel, dim3((unsigned)cdiv(D, 64)), dim3(256), 0, S(stream), x,
                       M, D, rstd, dy, scale, dw);
    MPR_LAUNCHED();
    return MPR_OK;
  }
  const int chunks = (int)cdiv(M, RMS_DW_CHUNK);
  hipLaunchKernelGGL(rms_dw_part_kernel, dim3((unsigned)cdiv(D, 64), (unsigned)chunks), dim3(256),
                     0, S(stream), x, M, D, rstd, dy, scale, dw_partial);
  MPR_LAUNCHED();
  hipLaunchKernelGGL(sum_rows_kernel, dim3((unsigned)cdiv(D, 256)), dim3(256), 0, S(stream),
                     dw_partial, chunks, (int64_t)D, dw);
  MPR_LAUNCHED();
  return MPR_OK;
}

int mpr_attn_train_fwd(const float* q, int64_t q_bs, int64_t q_rs, const float* k, int64_t k_bs,
                       int64_t k_rs, const float* v, int64_t v_bs, int64_t v_rs, int32_t B,
                       int32_t H, int32_t Lq, int32_t Lk, int32_t causal, const float* key_mask,
                       const float* rel, int32_t R, float* o, int64_t o_bs, int64_t o_rs, float* P,
                       uint64_t drop_seed, uint32_t drop_site, uint32_t drop_thresh,
                       float drop_scale, void* stream) {
  MPR_REQUIRE(Lk >= 1 && Lk <= TA_MAXK, "train attention: Lk=%d (1..%d)", Lk, TA_MAXK);
  MPR_REQUIRE(!rel || (Lq - 1 <= R && Lk - 1 <= R), "train attention: L exceeds the bias radius");
  const int64_t items = (int64_t)B * H * Lq;
  if (items == 0) return MPR_OK;
  TrainAttn a = make_attn(q, q_bs, q_rs, k, k_bs, k_rs, v, v_bs, v_rs, B, H, Lq, Lk, causal,
                          key_mask, rel, R);
  a.drop = Drop{drop_seed, drop_site, drop_thresh, drop_scale};
  if (Lq <= TB_MAXL && Lk <= TB_MAXL)
    hipLaunchKernelGGL(attn_fwd_bh_kernel, dim3((unsigned)(B * H)), dim3(64 * TB_WAVES), 0,
                       S(stream), a, o, o_bs, o_rs, P);
  else
    hipLaunchKernelGGL(attn_fwd_kernel, dim3((unsigned)cdiv(items, 4)), dim3(256), 0, S(stream),
                       a, o, o_bs, o_rs, P);
  MPR_LAUNCHED();
  return MPR_OK;
}

int mpr_attn_train_bwd(const float* q, int64_t q_bs, int64_t q_rs, const float* k, int64_t k_bs,
                       int64_t k_rs, const float* v, int64_t v_bs, int64_t v_rs, int32_t B,
                       int32_t H, int32_t Lq, int32_t Lk, const float* P, const float* dO,
                       int64_t do_bs, int64_t do_rs, float* dS, float* dq, int64_t dq_bs,
                       int64_t dq_rs, float* dk, int64_t dk_bs, int64_t dk_rs, float* dv,
                       int64_t dv_bs, int64_t dv_rs, float* drel, int32_t R, uint64_t drop_seed,
                       uint32_t drop_site, uint32_t drop_thresh, float drop_scale, void* stream) {
  MPR_REQUIRE(Lk >= 1 && Lk <= TA_MAXK, "train attention: Lk=%d (1..%d)", Lk, TA_MAXK);
  MPR_REQUIRE(!drel || (Lq - 1 <= R && Lk - 1 <= R), "train attention: L exceeds the bias radius");
  if ((int64_t)B * H * Lq == 0) return MPR_OK;
  TrainAttn a = make_attn(q, q_bs, q_rs, k, k_bs, k_rs, v, v_bs, v_rs, B, H, Lq, Lk, 0, nullptr,
                          nullptr, R);
  a.drop = Drop{drop_seed, drop_site, drop_thresh, drop_scale};
  if (Lq <= TB_MAXL && Lk <= TB_MAXL) {
    hipLaunchKernelGGL(attn_bwd_q_bh_kernel, dim3((unsigned)(B * H)), dim3(64 * TB_WAVES), 0,
                       S(stream), a, P, dO, do_bs, do_rs, dS, dq, dq_bs, dq_rs);
    MPR_LAUNCHED();
    hipLaunchKernelGGL(attn_bwd_kv_bh_kernel, dim3((unsigned)(B * H)), dim3(64 * TB_WAVES), 0,
                       S(stream), a, P, dS, dO, do_bs, do_rs, dk, dk_bs, dk_rs, dv, dv_bs, dv_rs);
    MPR_LAUNCHED();
  } else {
    hipLaunchKernelGGL(attn_bwd_q_kernel, dim3((unsigned)cdiv((int64_t)B * H * Lq, 4)), dim3(256),
                       0, S(stream), a, P, dO, do_bs, do_rs, dS, dq, dq_bs, dq_rs);
    MPR_LAUNCHED();
    hipLaunchKernelGGL(attn_bwd_kv_kernel, dim3((unsigned)cdiv((int64_t)B * H * Lk, 4)),
                       dim3(256), 0, S(stream), a, P, dS, dO, do_bs, do_rs, dk, dk_bs, dk_rs, dv,
                       dv_bs, dv_rs);
    MPR_LAUNCHED();
  }
  if (drel) {
    hipLaunchKernelGGL(attn_bwd_rel_kernel, dim3((unsigned)(2 * R + 1), (unsigned)H), dim3(256), 0,
                       S(stream), dS, B, H, Lq, Lk, R, drel);
    MPR_LAUNCHED();
  }
  return MPR_OK;
}

int mpr_rel_gather(const float* table, const int32_t* lut, int32_t R, int32_t H, float* rel,
                   void* stream) {
  const int64_t n = (int64_t)(2 * R + 1) * H;
  hipLaunchKernelGGL(rel_gather_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, S(stream),
                     table, lut, R, H, rel);
  MPR_LAUNCHED();
  return MPR_OK;
}

int mpr_rel_scatter(const float* drel, const int32_t* lut, int32_t R, int32_t num_buckets,
                    int32_t H, float* dtable, void* stream) {
  MPR_REQUIRE(H <= 1024, "rel scatter: H=%d", H);
  hipLaunchKernelGGL(rel_scatter_kernel, dim3((unsigned)num_buckets), dim3(64 * (int)cdiv(H, 64)),
                     0, S(stream), drel, lut, R, num_buckets, H, dtable);
  MPR_LAUNCHED();
  return MPR_OK;
}

int mpr_dropout(const float* x, int64_t n, uint64_t seed, uint32_t site, uint32_t thresh,
                float scale, const float* residual, float* y, void* stream) {
  if (n == 0) return MPR_OK;
  hipLaunchKernelGGL(dropout_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, S(stream), x, n,
                     Drop{seed, site, thresh, scale}, residual, y);
  MPR_LAUNCHED();
  return MPR_OK;
}

int mpr_relu_bwd(const float* y, const float* dy, int64_t n, float* dx, void* stream) {
  if (n == 0) return MPR_OK;
  hipLaunchKernelGGL(relu_bwd_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, S(stream), y, dy,
                     n, dx);
  MPR_LAUNCHED();
  return MPR_OK;
}

int mpr_add(const float* a, const float* b, int64_t n, float* out, void* stream) {
  if (n == 0) return MPR_OK;
  hipLaunchKernelGGL(add_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, S(stream), a, b, n,
                     out);
  MPR_LAUNCHED();
  return MPR_OK;
}

int mpr_ce_train(const float* logits, int64_t n, int32_t V, const int32_t* labels,
                 float loss_scale, float grad_scale, const float* grad_mult, float* row_loss,
                 float* loss, float* dlogits, int64_t ld_dlogits, void* stream) {
  MPR_REQUIRE(!dlogits || ld_dlogits >= V, "cross-entropy: dlogits row stride < V");
  if (n == 0) return MPR_OK;
  hipLaunchKernelGGL(ce_rows_kernel, dim3((unsigned)n), dim3(256), 0, S(stream), logits, n, V,
                     labels, grad_scale, grad_mult, row_loss, dlogits, ld_dlogits);
  MPR_LAUNCHED();
  hipLaunchKernelGGL(sum_scale_kernel, dim3(1), dim3(256), 0, S(stream), row_loss, n, loss_scale,
                     loss);
  MPR_LAUNCHED();
  return MPR_OK;
}

int mpr_gather_rows(const float* table, const int32_t* ids, int64_t n, int32_t d, float* out,
                    void* stream) {
  if (n == 0) return MPR_OK;
  hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)cdiv(n * d, 256)), dim3(256), 0,
                     S(stream), table, ids, n, d, out);
  MPR_LAUNCHED();
  return MPR_OK;
}

int mpr_embed_bwd(const float* dY, int32_t d, const int32_t* uniq, const int32_t* offs,
                  const int32_t* pos, int32_t n_uniq, float* dW, void* stream) {
  if (n_uniq == 0) return MPR_OK;
  hipLaunchKernelGGL(embed_bwd_kernel, dim3((unsigned)n_uniq), dim3(256), 0, S(stream), dY, d,
                     uniq, offs, pos, dW);
  MPR_LAUNCHED();
  return MPR_OK;
}

}  // extern "C"
