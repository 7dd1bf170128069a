// decode_gemm.hip — the decode-step projections of T5 greedy search at any row count (gfx950).
//
// Reference: the per-token decoder of transformers' T5 as driven by
// architectures/T5VisionModel.py:200-205 (generate, greedy, max_new_tokens=20): every step runs
// q|k|v, o, cross-q, cross-o, wi, wo of every decoder layer and the tied lm_head over the rows of
// the batch.  A 16-row predict() puts 16 rows through each projection; the serving loop's grouped
// decodes 128 (eight batches), config C5's 256-question batches 128-256.
//
// C[m, n] = R[m, n] + act(scale_m * sum_k A'[m, k] W[n, k])   on v_mfma_f32_16x16x32_bf16, fp32
// accurate: W arrives as three bf16 planes pre-split once at load (pack_planes, fragment order,
// one contiguous 1 KiB per plane and wave load), each A fragment is split into three planes in
// registers as it is loaded (x3.h), and the six cross products are accumulated in fp32 (x3.h).
//
// Block = 8 waves over one output tile of WM x WN 16x16 sub-tiles; wave w owns the contiguous
// k-step slice [w * nks / 8, (w + 1) * nks / 8) of the 32-deep k steps and keeps every sub-tile
// of the block in its accumulators, loading its operands straight into registers (no LDS
// staging: no operand is shared between the waves of a block).  The eight partial tiles are
// summed through LDS in wave order.  So every output element is summed in one order fixed by K
// alone — the block tile and the row count only decide which block computes it — and rows are
// independent: a batch's rows give the same bits alone or inside a grouped decode.
//
// The options are gemm_skinny's (kernels.h, SkinnyArgs), each a template flag:
//   RMS      A' = ln_w * A, scale_m = rsqrt(mean_k A[m,:]^2 + eps) (sums of squares of the loaded
//            A values: per lane, across the 4 lanes of a row, across waves in order)
//   RES      + R[m, n] (R may alias C)      RELU   max(., 0) before RES
//   AMAX     per (row, block) best column (lowest index on ties) instead of C: greedy head
//   RELU_IN  A' = max(A, 0)                  RSCALE scale_m from another launch's partial sums
//   SSQ      per (row, 16-column tile < ssq_cols) sums of squares of the output (folded chain)
#include <algorithm>
#include <cstdlib>

#include "kernels.h"
#include "x3.h"

namespace mpr {
namespace {

using x3::bf16x8;
using x3::f32x4;

constexpr int RW = 8;  // waves per block; the K range of every output splits into RW slices

enum : int { RF_RMS = 1, RF_RES = 2, RF_RELU = 4, RF_AMAX = 8, RF_RELU_IN = 16,
             RF_RSCALE = 32, RF_SSQ = 64 };

__global__ __launch_bounds__(256) void pack_planes_kernel(const float* __restrict__ W, int64_t N,
                                                          int64_t K, int64_t ldw, int64_t nks,
                                                          __bf16* __restrict__ out) {
  // one (16-column tile t, 32-deep step s, lane l) per thread: 8 values -> 3 planes
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = cdiv(N, 16) * nks * 64;
  if (q >= total) return;
  const int l = (int)(q & 63);
  const int64_t ts = q >> 6, t = ts / nks, s = ts % nks;
  const int64_t row = t * 16 + (l & 15), k0 = s * 32 + 8 * (l >> 4);
  f32x4 lo = {0.f, 0.f, 0.f, 0.f}, hi = lo;
  if (row < N) {
    lo = *reinterpret_cast<const f32x4*>(W + row * ldw + k0);
    hi = *reinterpret_cast<const f32x4*>(W + row * ldw + k0 + 4);
  }
  bf16x8 h0, h1, h2;
  x3::split8(lo, hi, h0, h1, h2);
  bf16x8* o = reinterpret_cast<bf16x8*>(out + (ts * 3) * 512) + l;
  o[0] = h0;
  o[64] = h1;
  o[128] = h2;
}

template <int WM, int WN, int F>
__global__ __launch_bounds__(512) void gemm_rows_kernel(SkinnyArgs sa, const __bf16* wpl) {
  constexpr bool RMS = (F & RF_RMS) != 0, RES = (F & RF_RES) != 0, RELU = (F & RF_RELU) != 0,
                 AMAX = (F & RF_AMAX) != 0, RELU_IN = (F & RF_RELU_IN) != 0,
                 RSCALE = (F & RF_RSCALE) != 0, SSQ = (F & RF_SSQ) != 0;
  static_assert(!(RMS && RSCALE), "one row-scale source");
  constexpr int ROWS = 16 * WM;
  // LDS: partial tiles [RW][WM][WN][64 lanes] f32x4 | row sums of squares [RW][ROWS] | row scales
  __shared__ __attribute__((aligned(16))) float smem[RW * WM * WN * 256 + RW * ROWS + ROWS];
  f32x4* red = reinterpret_cast<f32x4*>(smem);
  float* ssq_s = smem + RW * WM * WN * 256;
  float* rsc_s = ssq_s + RW * ROWS;

  const GemmArgs& a = sa.g;
  const int M = a.M, N = a.N, K = a.K;
  const int nks = K >> 5;
  const int ntiles = (N + 15) >> 4;
  const int nrb = (M + ROWS - 1) / ROWS;
  // XCD-aware order: blocks are dealt round-robin over the 8 XCDs; tile t (column block major,
  // row block minor) goes so that each XCD walks a contiguous run, i.e. the row blocks of one
  // column block (same weight columns) share an XCD's L2
  const int total = gridDim.x, hw = blockIdx.x;
  const int xcd = hw & 7, slot = hw >> 3, qq = total >> 3, rr = total & 7;
  const int t = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + slot;
  const int cb = t / nrb, rb = t - cb * nrb;
  const int m0 = rb * ROWS;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, lg = lane >> 4;
  const int s_lo = wave * nks / RW, s_hi = (wave + 1) * nks / RW;

  // RSCALE: the rows' partial sums of squares (<= 64 per row), lane = partial; wave w takes
  // rows w, w + 8, ... of the block; loaded first, summed after the main loop
  constexpr int RPW = (ROWS + RW - 1) / RW;
  float rsp[RSCALE ? RPW : 1];
  if constexpr (RSCALE) {
#pragma unroll
    for (int u = 0; u < RPW; ++u) {
      const int r = wave + u * RW, row = min(m0 + r, M - 1);
      rsp[u] = (r < ROWS && lane < sa.rs_nparts) ? sa.rs_part[(int64_t)row * sa.rs_nparts + lane]
                                                 : 0.f;
    }
  }

  const float* arow[WM];
  bool rok[WM];
#pragma unroll
  for (int i = 0; i < WM; ++i) {
    const int row = m0 + i * 16 + li;
    rok[i] = row < M;
    arow[i] = a.A + (int64_t)min(row, M - 1) * a.lda + 8 * lg;
  }
  const __bf16* wrow[WN];
#pragma unroll
  for (int j = 0; j < WN; ++j) {
    const int ct = min(cb * WN + j, ntiles - 1);  // a tile past N re-reads the last; not stored
    wrow[j] = wpl + (int64_t)ct * nks * 3 * 512 + lane * 8;
  }

  f32x4 acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ss[WM];
#pragma unroll
  for (int i = 0; i < WM; ++i) ss[i] = 0.f;

  // two k steps in flight: slot b holds step s's weight planes, A values (and RMS weights)
  bf16x8 rw[2][WN][3];
  f32x4 ra[2][WM][2];
  f32x4 rg[2][RMS ? 2 : 1];
  auto load = [&](int b, int s) {
#pragma unroll
    for (int j = 0; j < WN; ++j)
#pragma unroll
      for (int p = 0; p < 3; ++p)
        rw[b][j][p] = *reinterpret_cast<const bf16x8*>(wrow[j] + (int64_t)(s * 3 + p) * 512);
#pragma unroll
    for (int i = 0; i < WM; ++i) {
      ra[b][i][0] = *reinterpret_cast<const f32x4*>(arow[i] + s * 32);
      ra[b][i][1] = *reinterpret_cast<const f32x4*>(arow[i] + s * 32 + 4);
    }
    if constexpr (RMS) {
      rg[b][0] = *reinterpret_cast<const f32x4*>(sa.rms_w + s * 32 + 8 * lg);
      rg[b][1] = *reinterpret_cast<const f32x4*>(sa.rms_w + s * 32 + 8 * lg + 4);
    }
  };
  auto compute = [&](int b) {
#pragma unroll
    for (int i = 0; i < WM; ++i) {
      f32x4 v0 = ra[b][i][0], v1 = ra[b][i][1];
      if (!rok[i]) v0 = v1 = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (RELU_IN) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v0[e] = v0[e] > 0.f ? v0[e] : 0.f;
          v1[e] = v1[e] > 0.f ? v1[e] : 0.f;
        }
      }
      if constexpr (RMS) {
#pragma unroll
        for (int e = 0; e < 4; ++e) ss[i] += v0[e] * v0[e];
#pragma unroll
        for (int e = 0; e < 4; ++e) ss[i] += v1[e] * v1[e];
        v0 = rg[b][0] * v0;
        v1 = rg[b][1] * v1;
      }
      bf16x8 a0, a1, a2;
      x3::split8(v0, v1, a0, a1, a2);
#pragma unroll
      for (int j = 0; j < WN; ++j) {
        // D[row = weight column n][col = activation row m]; terms in increasing magnitude
        f32x4 c = acc[i][j];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rw[b][j][2], a0, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rw[b][j][1], a1, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rw[b][j][0], a2, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rw[b][j][1], a0, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rw[b][j][0], a1, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rw[b][j][0], a0, c, 0, 0, 0);
        acc[i][j] = c;
      }
    }
  };
  if (s_lo < s_hi) load(0, s_lo);
  for (int s = s_lo; s < s_hi; s += 2) {
    if (s + 1 < s_hi) load(1, s + 1);
    compute(0);
    if (s + 1 < s_hi) {
      if (s + 2 < s_hi) load(0, s + 2);
      compute(1);
    }
  }

  // partial tiles and row sums of squares to LDS, summed in wave order below
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) red[((wave * WM + i) * WN + j) * 64 + lane] = acc[i][j];
  if constexpr (RMS) {
#pragma unroll
    for (int i = 0; i < WM; ++i) {
      float v = ss[i];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (lane < 16) ssq_s[wave * ROWS + i * 16 + lane] = v;
    }
  }
  if constexpr (RSCALE) {
#pragma unroll
    for (int u = 0; u < RPW; ++u) {
      float v = rsp[u];
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
      const int r = wave + u * RW;
      if (lane == 0 && r < ROWS)
        rsc_s[r] = 1.0f / sqrtf(v / (float)sa.rs_n + sa.rms_eps);
    }
  }
  __syncthreads();

  // epilogue: wave q finishes sub-tiles q, q + 8, ... (argmax: row tiles, all WN column tiles)
  constexpr int NQ = AMAX ? WM : WM * WN;
  for (int q = wave; q < NQ; q += RW) {
    const int i = AMAX ? q : q / WN;
    const int m = m0 + i * 16 + li;  // the lane's row; its columns n0 + 4 lg .. + 3
    float scale = sa.a_scale;
    if constexpr (RMS) {
      float tt = 0.f;
#pragma unroll
      for (int w = 0; w < RW; ++w) tt += ssq_s[w * ROWS + i * 16 + li];
      scale = (1.0f / sqrtf(tt / (float)K + sa.rms_eps)) * sa.a_scale;
    }
    if constexpr (RSCALE) scale = rsc_s[i * 16 + li] * sa.a_scale;
    if constexpr (AMAX) {
      float bv = -INFINITY;
      int bi = 0x7fffffff;
#pragma unroll
      for (int j = 0; j < WN; ++j) {
        f32x4 sum = red[(i * WN + j) * 64 + lane];
#pragma unroll
        for (int w = 1; w < RW; ++w) sum += red[((w * WM + i) * WN + j) * 64 + lane];
        const int n0 = (cb * WN + j) * 16 + 4 * lg;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = sum[r] * scale;
          const int n = n0 + r;
          if (n < N && (v > bv || (v == bv && n < bi))) {
            bv = v;
            bi = n;
          }
        }
      }
#pragma unroll
      for (int off = 16; off <= 32; off <<= 1) {
        const float ov = __shfl_xor(bv, off, 64);
        const int oi = __shfl_xor(bi, off, 64);
        if (ov > bv || (ov == bv && oi < bi)) {
          bv = ov;
          bi = oi;
        }
      }
      const int nparts = (N + 16 * WN - 1) / (16 * WN);
      if (lane < 16 && m < M) {
        sa.amax_val[(int64_t)m * nparts + cb] = bv;
        sa.amax_idx[(int64_t)m * nparts + cb] = bi;
      }
    } else {
      const int j = q % WN;
      const int tile = cb * WN + j, n0 = tile * 16;
      f32x4 sum = red[(i * WN + j) * 64 + lane];
#pragma unroll
      for (int w = 1; w < RW; ++w) sum += red[((w * WM + i) * WN + j) * 64 + lane];
      f32x4 v = sum * scale;
      if constexpr (RELU) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : 0.f;
      }
      const bool ok = m < M && n0 < N;
      if constexpr (RES) {
        if (ok) v = *reinterpret_cast<const f32x4*>(a.R + (int64_t)m * a.ldr + n0 + 4 * lg) + v;
      }
      if (ok) *reinterpret_cast<f32x4*>(a.C + (int64_t)m * a.ldc + n0 + 4 * lg) = v;
      if constexpr (SSQ) {
        float sq = v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
        sq += __shfl_xor(sq, 16, 64);
        sq += __shfl_xor(sq, 32, 64);
        if (n0 < sa.ssq_cols && lane < 16 && m < M)
          sa.ssq_out[(int64_t)m * (sa.ssq_cols / 16) + tile] = sq;
      }
    }
  }
}

struct RowsTile {
  int wm, wn;
};

// The block tile of a launch: the largest of these (weight bytes per A byte, VALU of the A split
// per MFMA both fall with the tile) whose grid still puts a block on every CU; failing that the
// one with the most blocks.  MPR_ROWS_TILE=WMxWN forces one (measurements), MPR_ROWS_BLOCKS sets
// the target grid.
constexpr RowsTile kTiles[] = {{2, 4}, {4, 2}, {2, 2}, {1, 4}, {4, 1}, {1, 2}, {2, 1}, {1, 1}};

RowsTile pick_tile(int M, int N) {
  static const RowsTile forced = [] {
    const char* e = getenv("MPR_ROWS_TILE");
    RowsTile t{0, 0};
    if (e && sscanf(e, "%dx%d", &t.wm, &t.wn) == 2) {
      for (const RowsTile& c : kTiles)
        if (c.wm == t.wm && c.wn == t.wn) return t;
    }
    return RowsTile{0, 0};
  }();
  if (forced.wm) return forced;
  static const int target = [] {
    const char* e = getenv("MPR_ROWS_BLOCKS");
    return e ? std::max(1, atoi(e)) : 240;
  }();
  RowsTile best{1, 1};
  int64_t best_blocks = -1;
  for (const RowsTile& c : kTiles) {
    if (c.wm > 1 && 16 * c.wm > ((M + 15) / 16) * 16) continue;  // no mostly-empty row tiles
    const int64_t blocks = cdiv(M, 16 * c.wm) * cdiv(N, 16 * c.wn);
    if (blocks >= target) return c;
    if (blocks > best_blocks) {
      best_blocks = blocks;
      best = c;
    }
  }
  return best;
}

template <int WM, int WN>
int launch_rows(const SkinnyArgs& sa, const __bf16* wpl, int F, hipStream_t s) {
  const GemmArgs& a = sa.g;
  const unsigned blocks = (unsigned)(cdiv(a.M, 16 * WM) * cdiv(a.N, 16 * WN));
#define MPR_RK(f)                                                                        \
  case f:                                                                                \
    hipLaunchKernelGGL((gemm_rows_kernel<WM, WN, f>), dim3(blocks), dim3(512), 0, s, sa, \
                       wpl);                                                             \
    break;
  switch (F) {
    MPR_RK(RF_RMS)
    MPR_RK(RF_RES)
    MPR_RK(RF_RMS | RF_RELU)
    MPR_RK(RF_AMAX | RF_RMS)
    MPR_RK(RF_SSQ)
    MPR_RK(RF_RELU_IN | RF_RSCALE | RF_RES)
    default:
      set_error("gemm_rows: option set %d is not instantiated", F);
      return MPR_EINVAL;
  }
#undef MPR_RK
  MPR_LAUNCHED();
  return MPR_OK;
}

}  // namespace

bool gemm_rows_ok(int K) { return K > 0 && K % 32 == 0; }

int64_t packed_planes_elems(int64_t N, int64_t K) { return cdiv(N, 16) * (K / 32) * 3 * 512; }

int pack_planes(const float* W, int64_t N, int64_t K, int64_t ldw, void* out, hipStream_t s) {
  MPR_REQUIRE(N > 0 && K > 0 && K % 32 == 0 && ldw >= K && ldw % 4 == 0 && aligned16(W),
              "pack_planes: bad shape N=%lld K=%lld", (long long)N, (long long)K);
  const int64_t q = cdiv(N, 16) * (K / 32) * 64;
  hipLaunchKernelGGL(pack_planes_kernel, dim3((unsigned)cdiv(q, 256)), dim3(256), 0, s, W, N, K,
                     ldw, K / 32, reinterpret_cast<__bf16*>(out));
  MPR_LAUNCHED();
  return MPR_OK;
}

int gemm_rows(const SkinnyArgs& sa, const void* wpl, hipStream_t s, int* amax_nparts) {
  const GemmArgs& a = sa.g;
  MPR_REQUIRE(a.M >= 0 && a.N >= 0 && gemm_rows_ok(a.K), "gemm_rows: bad shape M=%d N=%d K=%d",
              a.M, a.N, a.K);
  MPR_REQUIRE(wpl && aligned16(wpl), "gemm_rows: needs the 16-byte aligned planes image");
  MPR_REQUIRE(a.lda % 4 == 0 && aligned16(a.A) && (!sa.rms_w || aligned16(sa.rms_w)),
              "gemm_rows: lda must be a multiple of 4, operands 16-byte aligned");
  MPR_REQUIRE(!a.bias && (a.act == ACT_NONE || a.act == ACT_RELU),
              "gemm_rows: no bias, activation none or relu (the T5 decoder's projections)");
  const bool amax = sa.amax_val != nullptr;
  MPR_REQUIRE(!amax || (sa.amax_idx && !a.R && !a.C && a.act == ACT_NONE),
              "gemm_rows: argmax mode takes plain logits and stores no C");
  MPR_REQUIRE(amax || (a.C && a.N % 16 == 0 && a.ldc % 4 == 0 && aligned16(a.C) &&
                       (!a.R || (a.ldr % 4 == 0 && aligned16(a.R)))),
              "gemm_rows: N must be a multiple of 16, C/R rows 16-byte aligned");
  MPR_REQUIRE(!sa.rs_part || (!sa.rms_w && !amax && sa.rs_n > 0 && sa.rs_nparts > 0 &&
                               sa.rs_nparts <= 64),
              "gemm_rows: an external row scale excludes the fused RMSNorm / argmax; at most "
              "64 partials per row");
  MPR_REQUIRE(!sa.ssq_out || (sa.ssq_cols % 16 == 0 && sa.ssq_cols <= a.N),
              "gemm_rows: ssq columns %d", sa.ssq_cols);
  const int F = (sa.rms_w ? RF_RMS : 0) | (a.R ? RF_RES : 0) | (a.act == ACT_RELU ? RF_RELU : 0) |
                (amax ? RF_AMAX : 0) | (sa.relu_in ? RF_RELU_IN : 0) |
                (sa.rs_part ? RF_RSCALE : 0) | (sa.ssq_out ? RF_SSQ : 0);
  const RowsTile tl = pick_tile(a.M, a.N);
  if (amax_nparts) *amax_nparts = (int)cdiv(a.N, 16 * tl.wn);
  if (a.M == 0 || a.N == 0) return MPR_OK;
  const __bf16* w = reinterpret_cast<const __bf16*>(wpl);
  switch (tl.wm * 8 + tl.wn) {
    case 1 * 8 + 1: return launch_rows<1, 1>(sa, w, F, s);
    case 1 * 8 + 2: return launch_rows<1, 2>(sa, w, F, s);
    case 1 * 8 + 4: return launch_rows<1, 4>(sa, w, F, s);
    case 2 * 8 + 1: return launch_rows<2, 1>(sa, w, F, s);
    case 2 * 8 + 2: return launch_rows<2, 2>(sa, w, F, s);
    case 2 * 8 + 4: return launch_rows<2, 4>(sa, w, F, s);
    case 4 * 8 + 1: return launch_rows<4, 1>(sa, w, F, s);
    default: return launch_rows<4, 2>(sa, w, F, s);
  }
}

}  // namespace mpr

// ---- C ABI (kernel-level tests and benchmarks of the decode projection) ----------------------
extern "C" {

int64_t mpr_planes_bytes(int64_t n, int32_t k) {
  return k > 0 && k % 32 == 0 && n > 0 ? mpr::packed_planes_elems(n, k) * 2 : 0;
}

int mpr_planes_pack(const float* W, int64_t n, int32_t k, void* planes, void* stream) {
  try {
    MPR_REQUIRE(planes && mpr::aligned16(planes), "planes_pack: output must be 16-byte aligned");
    return mpr::pack_planes(W, n, k, k, planes, reinterpret_cast<hipStream_t>(stream));
  } catch (...) {
    mpr::set_error("planes_pack: exception");
    return MPR_EINVAL;
  }
}

int mpr_rows_gemm(const float* A, int64_t lda, const void* planes, float* C, int64_t ldc,
                  int32_t M, int32_t N, int32_t K, const float* R, int64_t ldr, int32_t act,
                  const float* rms_w, float eps, float* amax_val, int32_t* amax_idx,
                  int32_t* nparts, void* stream) {
  try {
    MPR_REQUIRE(act == mpr::ACT_NONE || act == mpr::ACT_RELU, "rows_gemm: act %d", act);
    mpr::SkinnyArgs sa;
    sa.g.A = A; sa.g.lda = lda; sa.g.C = C; sa.g.ldc = ldc; sa.g.M = M; sa.g.N = N; sa.g.K = K;
    sa.g.R = R; sa.g.ldr = ldr; sa.g.act = act;
    sa.rms_w = rms_w; sa.rms_eps = eps;
    sa.amax_val = amax_val; sa.amax_idx = amax_idx;
    int np = 0;
    const int rc = mpr::gemm_rows(sa, planes, reinterpret_cast<hipStream_t>(stream), &np);
    if (nparts) *nparts = np;
    return rc;
  } catch (...) {
    mpr::set_error("rows_gemm: exception");
    return MPR_EINVAL;
  }
}

}  // extern "C"
