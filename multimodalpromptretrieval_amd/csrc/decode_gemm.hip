// decode_gemm.hip — the decoder projections of grouped greedy decodes (32-256 rows per step).
//
// Reference: the per-token decoder of transformers' T5 as driven by
// architectures/T5VisionModel.py:200-205 (generate, greedy, max_new_tokens=20): every step runs
// q|k|v, o, cross-q, cross-o, wi, wo of every decoder layer over the rows of the batch.  The serving
// loop's grouped decodes put 128 rows (eight 16-row batches) through every projection, config C5's
// 256-question batches 256; a 16-row predict() keeps the skinny GEMV chain (gemm.hip).
//
//   C[m, n] = R[m, n] + act(s_m * sum_k A'[m, k] W[n, k])      (T5's RMSNorm folded: A' = ln_w A,
//                                                              s_m = rsqrt(mean_k A[m,:]^2 + eps))
// on v_mfma_f32_16x16x32_bf16, fp32 accurate: both operands split into three bf16 planes (x3.h),
// six cross products accumulated in fp32.
//
// What bounds a decode projection at these row counts is how many CUs stream distinct weight bytes
// (~25 GB/s per CU from HBM; measured: a 144-block launch over t5-base's q|k|v ran 12 us at
// 0.9 TB/s), so the work is cut along N AND K into >= ~200 blocks, every weight element read by
// exactly one block, and every block covers ALL rows of the launch:
//   * block (column block cb, K slice ks): 16 * DN output columns x every row, K range
//     [ks * Kb, (ks + 1) * Kb).  Its fp32 weight slice is loaded once, split into three bf16 planes
//     in LDS (fragment order: one conflict-free ds_read_b128 per plane and lane);
//   * each wave owns (row tile, column tiles) pairs and sums its outputs sequentially over the K
//     slice, its A fragments loaded straight from L2 into registers and split there;
//   * KS = K / Kb > 1: partial tiles go to a workspace [KS][M][N] and dec_finish_kernel sums them
//     in slice order and applies the epilogue (row scale, ReLU, residual).
// The K partition (Kb) is a function of (K, N) only (dec_plan): a row's result does not depend on
// how many rows share the launch — a batch's rows give the same bits in a 128-row serving-loop
// group and in a 256-row C5 decode.
#include <algorithm>
#include <cstdlib>

#include "kernels.h"
#include "x3.h"

namespace mpr {
namespace {

using x3::bf16x4;
using x3::bf16x8;
using x3::f32x4;

constexpr int DW = 8;        // waves per block
constexpr int DN = 2;        // 16-column tiles per block
constexpr int KB_MAX = 512;  // LDS: 3 planes x DN tiles x Kb x 2 B = 96 KiB at 512

enum : int { DF_RMS = 1, DF_RES = 2, DF_RELU = 4 };

struct DecArgs {
  const float* A;
  int64_t lda;
  const float* W;  // [N, K] fp32, row-major
  int64_t ldw;
  const float* R;  // residual (may alias C)
  int64_t ldr;
  float* C;
  int64_t ldc;
  const float* rms_w;
  float eps;
  int M, N, K, Kb, KS;
  float* part;     // [KS][M][N] (KS > 1)
  float* part_ss;  // [KS][M] partial sums of squares of the A rows (RMS, KS > 1)
};

// One (row tile i, the wave's column tiles) work unit: A fragments of the K slice straight into
// registers (a batch of loads issued first), then per 32-deep step the split and 6 MFMAs per
// column tile against the LDS planes.  *ss = the row's sum of squares over the slice (RMS).
template <int F, int NTW>
__device__ __forceinline__ void dec_unit(const DecArgs& a, const __bf16* wl, int nsb, int k0,
                                         int i, int j0, f32x4 (&acc)[NTW], float* ss) {
  constexpr bool RMS = (F & DF_RMS) != 0;
  const int lane = threadIdx.x & 63, li = lane & 15, lg = lane >> 4;
  const int row = i * 16 + li;
  const bool rok = row < a.M;
  const float* ar = a.A + (int64_t)min(row, a.M - 1) * a.lda + k0 + 8 * lg;
  const float* gr = RMS ? a.rms_w + k0 + 8 * lg : nullptr;
  const int PL = nsb * DN * 64;  // bf16x8 per plane
#pragma unroll
  for (int t = 0; t < NTW; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float s2 = 0.f;
  constexpr int PS = 4;  // k steps per batch of loads
  for (int s0 = 0; s0 < nsb; s0 += PS) {
    f32x4 va[PS][2], vg[PS][2];
#pragma unroll
    for (int u = 0; u < PS; ++u) {
      const int s = min(s0 + u, nsb - 1);
      va[u][0] = *reinterpret_cast<const f32x4*>(ar + s * 32);
      va[u][1] = *reinterpret_cast<const f32x4*>(ar + s * 32 + 4);
      if constexpr (RMS) {
        vg[u][0] = *reinterpret_cast<const f32x4*>(gr + s * 32);
        vg[u][1] = *reinterpret_cast<const f32x4*>(gr + s * 32 + 4);
      }
    }
#pragma unroll
    for (int u = 0; u < PS; ++u) {
      const int s = s0 + u;
      if (s >= nsb) break;
      f32x4 v0 = va[u][0], v1 = va[u][1];
      if (!rok) v0 = v1 = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (RMS) {
#pragma unroll
        for (int e = 0; e < 4; ++e) s2 += v0[e] * v0[e];
#pragma unroll
        for (int e = 0; e < 4; ++e) s2 += v1[e] * v1[e];
        v0 = vg[u][0] * v0;
        v1 = vg[u][1] * v1;
      }
      bf16x8 a0, a1, a2;
      x3::split8(v0, v1, a0, a1, a2);
#pragma unroll
      for (int t = 0; t < NTW; ++t) {
        // planes image in LDS: [plane][step][tile][lane] bf16x8
        const bf16x8* wp = reinterpret_cast<const bf16x8*>(wl) + ((s * DN + j0 + t) * 64 + lane);
        const bf16x8 w0 = wp[0], w1 = wp[PL], w2 = wp[2 * PL];
        f32x4 c = acc[t];
        // D[row = weight column n][col = activation row m]; terms in increasing magnitude
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2, a0, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1, a1, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0, a2, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1, a0, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0, a1, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0, a0, c, 0, 0, 0);
        acc[t] = c;
      }
    }
  }
  if constexpr (RMS) {
    s2 += __shfl_xor(s2, 16, 64);
    s2 += __shfl_xor(s2, 32, 64);
    *ss = s2;
  }
}

template <int F>
__device__ __forceinline__ void dec_store(const DecArgs& a, int ks, int i, int n0, f32x4 v,
                                          float ss, bool ss_writer) {
  constexpr bool RMS = (F & DF_RMS) != 0, RES = (F & DF_RES) != 0, RELU = (F & DF_RELU) != 0;
  const int lane = threadIdx.x & 63, li = lane & 15, lg = lane >> 4;
  const int m = i * 16 + li;
  if (m >= a.M || n0 >= a.N) return;
  const int n = n0 + 4 * lg;
  if (a.KS > 1) {
    *reinterpret_cast<f32x4*>(a.part + ((int64_t)ks * a.M + m) * a.N + n) = v;
    if (RMS && ss_writer && lg == 0) a.part_ss[(int64_t)ks * a.M + m] = ss;
    return;
  }
  if constexpr (RMS) v = v * (1.0f / sqrtf(ss / (float)a.K + a.eps));
  if constexpr (RELU) {
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : 0.f;
  }
  if constexpr (RES) v = *reinterpret_cast<const f32x4*>(a.R + (int64_t)m * a.ldr + n) + v;
  *reinterpret_cast<f32x4*>(a.C + (int64_t)m * a.ldc + n) = v;
}

template <int F>
__global__ __launch_bounds__(512) void dec_part_kernel(DecArgs a) {
  extern __shared__ __attribute__((aligned(16))) __bf16 dec_lds[];
  const int ncb = (a.N + 16 * DN - 1) / (16 * DN);
  // XCD-aware order: each XCD walks a contiguous run of (ks major, cb minor): its L2 holds the
  // A columns of about one K slice
  const int total = gridDim.x, hw = blockIdx.x;
  const int xcd = hw & 7, slot = hw >> 3, qq = total >> 3, rr = total & 7;
  const int t = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + slot;
  const int ks = t / ncb, cb = t - ks * ncb;
  const int k0 = ks * a.Kb, nsb = a.Kb >> 5;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  // stage the weight slice: 16 * DN rows x Kb fp32 -> three bf16 planes in fragment order
  {
    const int n0 = cb * 16 * DN;
    const int q4 = a.Kb >> 2;  // float4 per weight row
    const int nq = 16 * DN * q4;
    const int PL = nsb * DN * 512;  // bf16 per plane
    for (int q = tid; q < nq; q += DW * 64) {
      const int r = q / q4, k = (q - r * q4) * 4;
      const int n = min(n0 + r, a.N - 1);
      const f32x4 v = *reinterpret_cast<const f32x4*>(a.W + (int64_t)n * a.ldw + k0 + k);
      bf16x4 h0, h1, h2;
      x3::split3(v, h0, h1, h2);
      const int s = k >> 5, j = r >> 4;
      const int l = (r & 15) + 16 * ((k & 31) >> 3);
      __bf16* p = dec_lds + ((s * DN + j) * 64 + l) * 8 + (k & 7);
      *reinterpret_cast<bf16x4*>(p) = h0;
      *reinterpret_cast<bf16x4*>(p + PL) = h1;
      *reinterpret_cast<bf16x4*>(p + 2 * PL) = h2;
    }
  }
  __syncthreads();

  // work split: row tiles over waves; with fewer row tiles than waves, the waves of a row tile
  // split its DN column tiles (each output is still summed by one wave over the whole slice)
  const int nrt = (a.M + 15) >> 4;
  if (nrt > DW / DN) {
    for (int i = wave; i < nrt; i += DW) {
      f32x4 acc[DN];
      float ss = 0.f;
      dec_unit<F, DN>(a, dec_lds, nsb, k0, i, 0, acc, &ss);
#pragma unroll
      for (int j = 0; j < DN; ++j)
        dec_store<F>(a, ks, i, (cb * DN + j) * 16, acc[j], ss, cb == 0 && j == 0);
    }
  } else {  // <= 4 row tiles: one (row tile, column tile) pair per wave
    const int i = wave / DN, j = wave % DN;
    if (i < nrt) {
      f32x4 acc[1];
      float ss = 0.f;
      dec_unit<F, 1>(a, dec_lds, nsb, k0, i, j, acc, &ss);
      dec_store<F>(a, ks, i, (cb * DN + j) * 16, acc[0], ss, cb == 0 && j == 0);
    }
  }
}

// KS > 1: out[m, n] = epilogue(sum_ks part[ks][m][n]) in slice order; one block per row
template <int F>
__global__ __launch_bounds__(256) void dec_finish_kernel(DecArgs a) {
  constexpr bool RMS = (F & DF_RMS) != 0, RES = (F & DF_RES) != 0, RELU = (F & DF_RELU) != 0;
  const int m = blockIdx.x;
  float scale = 1.f;
  if constexpr (RMS) {
    float ss = 0.f;
    for (int ks = 0; ks < a.KS; ++ks) ss += a.part_ss[(int64_t)ks * a.M + m];
    scale = 1.0f / sqrtf(ss / (float)a.K + a.eps);
  }
  const int n4 = a.N >> 2;
  for (int q = threadIdx.x; q < n4; q += 256) {
    f32x4 v = *reinterpret_cast<const f32x4*>(a.part + (int64_t)m * a.N + 4 * q);
    for (int ks = 1; ks < a.KS; ++ks)
      v += *reinterpret_cast<const f32x4*>(a.part + ((int64_t)ks * a.M + m) * a.N + 4 * q);
    if constexpr (RMS) v = v * scale;
    if constexpr (RELU) {
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : 0.f;
    }
    if constexpr (RES) v = *reinterpret_cast<const f32x4*>(a.R + (int64_t)m * a.ldr + 4 * q) + v;
    *reinterpret_cast<f32x4*>(a.C + (int64_t)m * a.ldc + 4 * q) = v;
  }
}

struct DecPlan {
  int Kb, KS, ncb;
};

// The K partition of a launch: the fewest K slices (each <= KB_MAX deep, a divisor of the
// 32-deep steps) that give the launch >= MPR_DEC_BLOCKS blocks (default 192).  A function of
// (K, N) only, never of the row count.
DecPlan dec_plan(int N, int K) {
  static const int target = [] {
    const char* e = getenv("MPR_DEC_BLOCKS");
    return e ? std::max(1, atoi(e)) : 192;
  }();
  const int nks = K / 32;
  const int ncb = (N + 16 * DN - 1) / (16 * DN);
  int best = nks;
  for (int d = 1; d <= nks; ++d) {
    if (nks % d || K / d > KB_MAX) continue;
    best = d;
    if ((int64_t)ncb * d >= target) break;
  }
  return DecPlan{K / best, best, ncb};
}

template <int F>
int launch_dec(const DecArgs& a, const DecPlan& p, hipStream_t s) {
  static const hipError_t attr = hipFuncSetAttribute(
      reinterpret_cast<const void*>(dec_part_kernel<F>),
      hipFuncAttributeMaxDynamicSharedMemorySize, (int)(3 * DN * KB_MAX * 2));
  MPR_HIP(attr);
  const size_t lds = (size_t)3 * DN * p.Kb * 2;
  hipLaunchKernelGGL(dec_part_kernel<F>, dim3((unsigned)(p.ncb * p.KS)), dim3(DW * 64), lds, s,
                     a);
  MPR_LAUNCHED();
  if (p.KS > 1) {
    hipLaunchKernelGGL(dec_finish_kernel<F>, dim3((unsigned)a.M), dim3(256), 0, s, a);
    MPR_LAUNCHED();
  }
  return MPR_OK;
}

}  // namespace

bool gemm_dec_ok(int K, int N) { return K > 0 && K % 32 == 0 && N > 0 && N % 16 == 0; }

size_t gemm_dec_ws_floats(int M, int N, int K) {
  const DecPlan p = dec_plan(N, K);
  return p.KS > 1 ? (size_t)p.KS * M * (N + 1) : 0;
}

int gemm_dec(const SkinnyArgs& sa, float* ws, size_t ws_floats, hipStream_t s) {
  const GemmArgs& g = sa.g;
  MPR_REQUIRE(g.M >= 0 && g.M <= 256 && gemm_dec_ok(g.K, g.N),
              "gemm_dec: bad shape M=%d N=%d K=%d (M <= 256, K %% 32 == 0, N %% 16 == 0)", g.M,
              g.N, g.K);
  MPR_REQUIRE(g.W && aligned16(g.W) && g.ldw % 4 == 0 && g.lda % 4 == 0 && aligned16(g.A) &&
                  g.C && aligned16(g.C) && g.ldc % 4 == 0 &&
                  (!g.R || (aligned16(g.R) && g.ldr % 4 == 0)) &&
                  (!sa.rms_w || aligned16(sa.rms_w)),
              "gemm_dec: operands must be 16-byte aligned, leading dims multiples of 4");
  MPR_REQUIRE(!g.bias && (g.act == ACT_NONE || g.act == ACT_RELU) && !sa.amax_val &&
                  !sa.ssq_out && !sa.rs_part && !sa.relu_in && sa.a_scale == 1.f,
              "gemm_dec: the plain decode projections (RMSNorm prologue, ReLU, residual) only");
  if (g.M == 0 || g.N == 0) return MPR_OK;
  const DecPlan p = dec_plan(g.N, g.K);
  DecArgs a;
  a.A = g.A; a.lda = g.lda; a.W = g.W; a.ldw = g.ldw; a.R = g.R; a.ldr = g.ldr;
  a.C = g.C; a.ldc = g.ldc; a.rms_w = sa.rms_w; a.eps = sa.rms_eps;
  a.M = g.M; a.N = g.N; a.K = g.K; a.Kb = p.Kb; a.KS = p.KS;
  a.part = ws;
  a.part_ss = ws ? ws + (size_t)p.KS * g.M * g.N : nullptr;
  MPR_REQUIRE(p.KS == 1 || (ws && ws_floats >= gemm_dec_ws_floats(g.M, g.N, g.K) &&
                            aligned16(ws)),
              "gemm_dec: split-K workspace too small");
  const int F = (sa.rms_w ? DF_RMS : 0) | (g.R ? DF_RES : 0) | (g.act == ACT_RELU ? DF_RELU : 0);
  switch (F) {
    case 0: return launch_dec<0>(a, p, s);
    case DF_RELU: return launch_dec<DF_RELU>(a, p, s);
    case DF_RMS: return launch_dec<DF_RMS>(a, p, s);
    case DF_RMS | DF_RELU: return launch_dec<DF_RMS | DF_RELU>(a, p, s);
    case DF_RES: return launch_dec<DF_RES>(a, p, s);
    default: break;
  }
  set_error("gemm_dec: option set %d is not instantiated", F);
  return MPR_EINVAL;
}

}  // namespace mpr

// ---- C ABI (kernel-level tests and benchmarks of the decode projection) ----------------------
extern "C" {

int mpr_dec_gemm(const float* A, int64_t lda, const float* W, int64_t ldw, float* C, int64_t ldc,
                 int32_t M, int32_t N, int32_t K, const float* R, int64_t ldr, int32_t act,
                 const float* rms_w, float eps, void* stream) {
  try {
    using namespace mpr;
    MPR_REQUIRE(act == ACT_NONE || act == ACT_RELU, "dec_gemm: act %d", act);
    SkinnyArgs sa;
    sa.g.A = A; sa.g.lda = lda; sa.g.W = W; sa.g.ldw = ldw; sa.g.C = C; sa.g.ldc = ldc;
    sa.g.M = M; sa.g.N = N; sa.g.K = K; sa.g.R = R; sa.g.ldr = ldr; sa.g.act = act;
    sa.rms_w = rms_w; sa.rms_eps = eps;
    static DevBuf ws;  // the split-K partials of these calls (ordered on their stream)
    const size_t need = gemm_dec_ws_floats(M, N, K);
    if (need * 4 > ws.bytes) {
      MPR_HIP(hipDeviceSynchronize());
      MPR_TRY(ws.ensure(need * 4));
    }
    return gemm_dec(sa, ws.as<float>(), ws.bytes / 4, reinterpret_cast<hipStream_t>(stream));
  } catch (...) {
    mpr::set_error("dec_gemm: exception");
    return MPR_EINVAL;
  }
}

}  // extern "C"
