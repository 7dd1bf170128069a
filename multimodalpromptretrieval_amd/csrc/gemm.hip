// gemm.hip — fp32 GEMMs on gfx950 f32-input MFMA.
//
// Every dense projection of the three encoders (ViT-B/32, CLIP text, T5) is
//   C[m, n] = R[m, n] + act(sum_k A[m, k] * W[n, k] + bias[n])
// with W in torch nn.Linear layout [N, K].  Both operands are K-contiguous, so a block stages a
// BM x 32 slice of A and a BN x 32 slice of W into LDS and each wave feeds
// v_mfma_f32_32x32x2_f32 (exact f32 FMA chains, 64 FLOP/clk/SIMD — the fp32 peak of the chip).
// The contraction order inside a 32-wide K tile is permuted (lane half h owns k = 16h..16h+15) so
// that each lane reads 16 contiguous floats (4 x ds_read_b128) per operand and tile; the LDS rows
// are padded to 36 floats, which makes those 128-bit reads bank-conflict free.
//
// gemm_skinny() serves decoder steps (M = batch rows <= 16, or up to 64 when 2-4 batches share a
// decode loop): W streams straight from HBM/L2 into registers as the A operand of
// v_mfma_f32_16x16x4_f32 (16 output columns per block), each 16-row group of activations is a B
// operand for the same weight registers, K is split across the 8 waves of a block and reduced through
// LDS, and T5's RMSNorm of the activation rows is folded into the operand and the epilogue.
#include <algorithm>
#include <cstring>
#include <mutex>
#include <set>
#include <string>

#include "kernels.h"
#include "x3.h"

namespace mpr {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// Accurate QuickGELU (x * sigmoid(1.702 x)) — expf, not the fast exp: keeps parity with the
// fp32 CPU reference (torch.sigmoid) to a few ulp.
__device__ __forceinline__ float act_exact(float v, int act) {
  if (act == ACT_QUICKGELU) return v * (1.0f / (1.0f + expf(-1.702f * v)));
  if (act == ACT_RELU) return v > 0.f ? v : 0.f;
  return v;
}

// Tile configuration:
//   BM x BN output tile, waves of WM x WN 32x32 accumulators, BK-deep K tiles, KW wave groups
//   splitting each K tile (KW = 2: two waves per SIMD on the same output, summed through LDS at
//   the end), D = global-load prefetch depth in K tiles (tile t+2+D is requested while tile t is
//   multiplied and lands in LDS D iterations later).
// Two LDS stages: during iteration t the waves read tile t+1's fragments from one stage while
// tile t+2 is written into the other (tile t's stage, whose fragments were read in iteration t-1,
// before the barrier that closed it).  Fragments of tile t+1 are read under tile t's MFMAs.
//
// One BM x BN output tile of problem `a` (tile column bx, row by) with this block; `smem` is the
// kernel's single LDS object (>= 2 * (BM + BN) * (BK + 4) floats).
template <int BM, int BN, int WM, int WN, int BK, int D, int KW>
__device__ __forceinline__ void gemm_tile(const GemmArgs& a, int bx, int by, float* smem) {
  constexpr int WAVES_N = BN / (32 * WN);
  constexpr int WAVES_MN = (BM / (32 * WM)) * WAVES_N;
  constexpr int NT = 64 * WAVES_MN * KW;
  constexpr int LDK = BK + 4, KQ = BK / 4;  // LDS row stride (floats), float4 per tile row
  constexpr int LA = BM * KQ / NT, LB = BN * KQ / NT;
  constexpr int STAGE = (BM + BN) * LDK;  // floats per LDS stage (A rows then W rows)
  constexpr int KPW = BK / KW;            // k per tile and wave
  constexpr int NF = KPW / 8;             // float4 fragments per lane, operand and tile
  static_assert(LA * NT == BM * KQ && LB * NT == BN * KQ, "loader split");
  static_assert(NF >= 2 && KPW % 8 == 0, "k split");
  static_assert(KW == 1 || 2 * STAGE >= KW * BM * BN, "LDS reduction space");
  const int M = a.M, N = a.N, K = a.K;
  const int m0 = by * BM, n0 = bx * BN;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR)
  const int wmn = wave % WAVES_MN, kw = wave / WAVES_MN;
  const int wm = wmn / WAVES_N, wn = wmn % WAVES_N;

  // D register slots of in-flight global loads (slot j is indexed by compile-time constants
  // only: the k-loop is unrolled by D).
  f32x4 ra[D][LA], rb[D][LB];
  bool oka[D][LA], okb[D][LB];
  // Unconditional loads from clamped addresses, zeroed by a select only when written to LDS: an
  // exec-masked load makes hipcc branch around every load, and an early select makes it wait
  // for the data right after issuing the load.  Tiles past K load clamped, in-range data and
  // are written as zeros.
  auto gload = [&](int j, int k0) {
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int idx = tid + i * NT, r = idx / KQ, c = k0 + (idx % KQ) * 4, row = m0 + r;
      oka[j][i] = row < M && c < K;
      ra[j][i] = *reinterpret_cast<const f32x4*>(a.A + (int64_t)min(row, M - 1) * a.lda +
                                                 min(c, K - 4));
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int idx = tid + i * NT, r = idx / KQ, c = k0 + (idx % KQ) * 4, row = n0 + r;
      okb[j][i] = row < N && c < K;
      rb[j][i] = *reinterpret_cast<const f32x4*>(a.W + (int64_t)min(row, N - 1) * a.ldw +
                                                 min(c, K - 4));
    }
  };
  auto swrite = [&](int st, int j) {
    const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
    float* base = smem + st * STAGE;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int idx = tid + i * NT;
      *reinterpret_cast<f32x4*>(base + (idx / KQ) * LDK + (idx % KQ) * 4) =
          oka[j][i] ? ra[j][i] : zero;
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int idx = tid + i * NT;
      *reinterpret_cast<f32x4*>(base + (BM + idx / KQ) * LDK + (idx % KQ) * 4) =
          okb[j][i] ? rb[j][i] : zero;
    }
  };

  f32x16 acc[WM][WN];
#pragma unroll
  for (int mi = 0; mi < WM; ++mi)
#pragma unroll
    for (int ni = 0; ni < WN; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;

  // Operand fragments of one K tile: lane (li, lh) of wave group kw holds row li's
  // k = kw*KPW + lh*KPW/2 + [0, KPW/2) as NF float4 (the contraction order inside the tile is
  // permuted identically for A and W).  Row stride BK+4 floats: conflict-free ds_read_b128.
  const int li = lane & 31, lh = lane >> 5;
  const int kof = kw * KPW + lh * (KPW / 2);
  f32x4 fa[WM][NF], fb[WN][NF], na[WM][NF], nb[WN][NF];
  auto sread = [&](int st, f32x4(&xa)[WM][NF], f32x4(&xb)[WN][NF]) {
    const float* base = smem + st * STAGE;
#pragma unroll
    for (int s4 = 0; s4 < NF; ++s4) {
#pragma unroll
      for (int mi = 0; mi < WM; ++mi)
        xa[mi][s4] = *reinterpret_cast<const f32x4*>(
            base + (wm * 32 * WM + mi * 32 + li) * LDK + kof + s4 * 4);
#pragma unroll
      for (int ni = 0; ni < WN; ++ni)
        xb[ni][s4] = *reinterpret_cast<const f32x4*>(
            base + (BM + wn * 32 * WN + ni * 32 + li) * LDK + kof + s4 * 4);
    }
  };
  auto mfmas = [&](int s_lo, int s_hi) {
#pragma unroll
    for (int s4 = s_lo; s4 < s_hi; ++s4)
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int mi = 0; mi < WM; ++mi)
#pragma unroll
          for (int ni = 0; ni < WN; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[mi][s4][c], fb[ni][s4][c],
                                                               acc[mi][ni], 0, 0, 0);
  };
  auto advance = [&]() {
#pragma unroll
    for (int s4 = 0; s4 < NF; ++s4) {
#pragma unroll
      for (int mi = 0; mi < WM; ++mi) fa[mi][s4] = na[mi][s4];
#pragma unroll
      for (int ni = 0; ni < WN; ++ni) fb[ni][s4] = nb[ni][s4];
    }
  };

  // k-steps rounded up to a multiple of D (the extra steps multiply zero tiles: exact no-ops on
  // the accumulators; every projection of this path has K % (BK * D) == 0 anyway).
  const int nk = (K + BK - 1) / BK;
  const int nkr = (nk + D - 1) / D * D;

  gload(0, 0);
  swrite(0, 0);
  gload(0, BK);
  swrite(1, 0);
#pragma unroll
  for (int j = 0; j < D; ++j) gload(j, (2 + j) * BK);
  __syncthreads();
  sread(0, fa, fb);
  // Iteration 0 overwrites stage 0 (tile 2) while a slower wave may still be reading tile 0's
  // fragments from it here: every wave's reads must land first (this race made ~3% of grouped
  // launches nondeterministic before the barrier was added).
  __syncthreads();
  // Steady state, branch-free (the accumulators stay in AGPRs): iteration t multiplies tile t
  // (fragments already in registers), reads tile t+1's fragments after the first quarter of the
  // MFMAs, writes tile t+2 (register slot t % D) into tile t's stage and re-arms the slot with
  // tile t+2+D.
  for (int kt = 0; kt < nkr; kt += D) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const int st = (kt + j) & 1;
      __builtin_amdgcn_sched_barrier(0);
      mfmas(0, 1);
      __builtin_amdgcn_sched_barrier(0);
      sread(st ^ 1, na, nb);
      __builtin_amdgcn_sched_barrier(0);
      mfmas(1, NF);
      __builtin_amdgcn_sched_barrier(0);
      swrite(st, j);
      gload(j, (kt + j + 2 + D) * BK);
      __syncthreads();
      advance();
    }
  }

  if constexpr (KW > 1) {
    // wave groups 1.. park their partial accumulators in LDS (every stage read is complete: the
    // loop ended on a barrier), group 0 adds them in group order.
    f32x16* red = reinterpret_cast<f32x16*>(smem);
    if (kw > 0) {
#pragma unroll
      for (int mi = 0; mi < WM; ++mi)
#pragma unroll
        for (int ni = 0; ni < WN; ++ni)
          red[(((kw - 1) * WAVES_MN + wmn) * WM * WN + mi * WN + ni) * 64 + lane] = acc[mi][ni];
    }
    __syncthreads();
    if (kw > 0) return;
#pragma unroll
    for (int g = 1; g < KW; ++g)
#pragma unroll
      for (int mi = 0; mi < WM; ++mi)
#pragma unroll
        for (int ni = 0; ni < WN; ++ni)
          acc[mi][ni] += red[(((g - 1) * WAVES_MN + wmn) * WM * WN + mi * WN + ni) * 64 + lane];
  }

  // Epilogue: 32x32 accumulator, col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5).
  // Bias and residual values are all loaded (clamped addresses) before the first use: a load
  // behind a per-row bounds branch is waited for on its own, 16 dependent round trips.
#pragma unroll
  for (int mi = 0; mi < WM; ++mi)
#pragma unroll
    for (int ni = 0; ni < WN; ++ni) {
      const int col = n0 + wn * 32 * WN + ni * 32 + li, colc = min(col, N - 1);
      const int rbase = m0 + wm * 32 * WM + mi * 32 + 4 * lh;
      const float bv = a.bias ? a.bias[colc] : 0.f;
      float rv[16];
      if (a.R) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          rv[r] = a.R[(int64_t)min(rbase + (r & 3) + 8 * (r >> 2), M - 1) * a.ldr + colc];
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = rbase + (r & 3) + 8 * (r >> 2);
        float v = act_exact(acc[mi][ni][r] + bv, a.act);
        if (a.R) v = rv[r] + v;
        const int64_t coff = a.c_rpb ? (int64_t)(row / a.c_rpb) * a.c_bs +
                                           (int64_t)(row % a.c_rpb) * a.ldc
                                     : (int64_t)row * a.ldc;
        if (row < M && col < N) a.C[coff + col] = v;
      }
    }
}

// ---------------------------------------------------------------------------------------------
// fp32 GEMM on the bf16 matrix cores ("x3"): every fp32 operand is split into three bf16 terms
// with round-to-nearest residuals, a = a0 + a1 + a2 (|a - a0| <= 2^-8 |a|, |a - a0 - a1| <=
// 2^-16 |a|, the remainder <= 2^-24 |a|: fp32 input precision), and
//     a.b = a0.b0 + (a0.b1 + a1.b0) + (a0.b2 + a1.b1 + a2.b0)          (+ terms <= 2^-23 |a.b|)
// — six v_mfma_f32_32x32x16_bf16 per 16-deep k step, each product of two bf16 exact in fp32 and
// accumulated in fp32.  Six bf16 MFMAs cost 12 cycles per k per SIMD against 32 for one
// v_mfma_f32_32x32x2_f32 (bf16 runs at 16x the f32 MFMA rate): the same tile does 2.67x the
// arithmetic per cycle.  Error vs fp64 (round-1 lab tools/x3bench.hip, removed in round 5; git show 28e8ac6:tools/x3bench.hip): within a factor ~1.5 of the f32 MFMA
// kernel's (both ~1e-7 of sum|a.b| at K <= 3072), orders below every parity tolerance.
// Structure as gemm_tile: BM x BN block tile, WM x WN 32x32 accumulators per wave, BK-deep K
// tiles staged fp32 global -> registers (D tiles in flight) -> split -> 3 bf16 planes in LDS (two
// stages), KW wave groups splitting each K tile (partials summed through LDS).
using x3::bf16x4;
using x3::bf16x8;
using x3::split3;

template <int BM, int BN, int BK, int SB = 1>
constexpr int x3_lds_floats() {
  // per stage: 3 planes x (BM + BN) rows x (BK + 8) bf16 (16-byte row pad: conflict-free
  // ds_read_b128 of 32 rows), 2 SB stages, in floats
  return 2 * SB * 3 * (BM + BN) * (BK + 8) / 2;
}

// V (variants, the round-1 x3bench lab, git show 28e8ac6:tools/x3bench.hip): bit 0 interleaves the accumulators' MFMAs (term-major; the
// order of each accumulator's own terms is unchanged, results bit-identical) — neutral, unused;
// bit 1 raises the wave's issue priority over its MFMA run (s_setprio 1 .. 0): +0-4% on the
// 128x128 tiles (fc2 1600x768x3072 x4: 131.2 -> 126.9 us), neutral to slightly negative on 64x128.
// KT: some K is not a multiple of BK, or its tile count not a multiple of D (the loads past K
// are zeroed: the main loop runs whole groups of D tiles; otherwise no select touches a
// loaded value, so no load is waited for early).  Rows past M / N read a clamped in-range row;
// their results are not stored.  (Measured and dropped: W pre-split into three bf16 planes once
// per model, copied into LDS without conversion: +8% on 64x128 tiles, -11% on 128x128 — the
// planes' 32-byte row segments per k-tile coalesce worse than the 64-byte fp32 ones.)
// SB = 2: four stages and a block barrier every second K tile, as gemm_x3p_tile's SB.
template <int BM, int BN, int WM, int WN, int BK, int D, int KW, bool KT, int V = 0, int SB = 1>
__device__ __forceinline__ void gemm_x3_tile(const GemmArgs& a, int bx, int by, float* smem_f) {
  static_assert(SB == 1 || (SB == 2 && D % 2 == 0), "SB = 2 needs an even D");
  constexpr int NSTG = 2 * SB, AHEAD = SB + 1;
  constexpr int WAVES_N = BN / (32 * WN);
  constexpr int WAVES_MN = (BM / (32 * WM)) * WAVES_N;
  constexpr int NT = 64 * WAVES_MN * KW;
  constexpr int LDK = BK + 8, KQ = BK / 4;      // LDS row stride (bf16), float4 per tile row
  constexpr int LA = BM * KQ / NT, LB = BN * KQ / NT;
  constexpr int PLANE = (BM + BN) * LDK;        // bf16 per plane (A rows then W rows)
  constexpr int STAGE = 3 * PLANE;              // bf16 per stage
  constexpr int KPW = BK / KW;                  // k per tile and wave group
  constexpr int NS = KPW / 16;                  // 16-deep MFMA steps per tile and wave
  static_assert(LA * NT == BM * KQ && LB * NT == BN * KQ, "loader split");
  static_assert(NS >= 1 && KPW % 16 == 0, "k split");
  static_assert(KW == 1 || 2 * STAGE / 2 >= KW * BM * BN, "LDS reduction space");
  __bf16* smem = reinterpret_cast<__bf16*>(smem_f);
  const int M = a.M, N = a.N, K = a.K;
  const int m0 = by * BM, n0 = bx * BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wmn = wave % WAVES_MN, kw = wave / WAVES_MN;
  const int wm = wmn / WAVES_N, wn = wmn % WAVES_N;

  f32x4 ra[D][LA], rb[D][LB];
  bool oka[D][LA], okb[D][LB];
  auto gload = [&](int j, int k0) {
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int idx = tid + i * NT, r = idx / KQ, c = k0 + (idx % KQ) * 4, row = m0 + r;
      if constexpr (KT) oka[j][i] = c < K;
      ra[j][i] = *reinterpret_cast<const f32x4*>(a.A + (int64_t)min(row, M - 1) * a.lda +
                                                 min(c, K - 4));
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int idx = tid + i * NT, r = idx / KQ, c = k0 + (idx % KQ) * 4, row = n0 + r;
      if constexpr (KT) okb[j][i] = c < K;
      rb[j][i] = *reinterpret_cast<const f32x4*>(a.W + (int64_t)min(row, N - 1) * a.ldw +
                                                 min(c, K - 4));
    }
  };
  auto put = [&](__bf16* base, int row, int kc, const f32x4& v) {
    bf16x4 h0, h1, h2;
    split3(v, h0, h1, h2);
    __bf16* p = base + row * LDK + kc;
    *reinterpret_cast<bf16x4*>(p) = h0;
    *reinterpret_cast<bf16x4*>(p + PLANE) = h1;
    *reinterpret_cast<bf16x4*>(p + 2 * PLANE) = h2;
  };
  auto swrite = [&](int st, int j) {
    const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
    __bf16* base = smem + st * STAGE;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int idx = tid + i * NT;
      if constexpr (KT) put(base, idx / KQ, (idx % KQ) * 4, oka[j][i] ? ra[j][i] : zero);
      else put(base, idx / KQ, (idx % KQ) * 4, ra[j][i]);
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int idx = tid + i * NT;
      if constexpr (KT) put(base, BM + idx / KQ, (idx % KQ) * 4, okb[j][i] ? rb[j][i] : zero);
      else put(base, BM + idx / KQ, (idx % KQ) * 4, rb[j][i]);
    }
  };

  f32x16 acc[WM][WN];
#pragma unroll
  for (int mi = 0; mi < WM; ++mi)
#pragma unroll
    for (int ni = 0; ni < WN; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;

  // lane (li, lh) of a 32x32x16 step reads row li, k = 16 s + 8 lh .. +7 of every plane
  const int li = lane & 31, lh = lane >> 5;
  const int kof = kw * KPW + 8 * lh;
  bf16x8 fa[WM][NS][3], fb[WN][NS][3], na[WM][NS][3], nb[WN][NS][3];
  auto sread = [&](int st, bf16x8(&xa)[WM][NS][3], bf16x8(&xb)[WN][NS][3]) {
    const __bf16* base = smem + st * STAGE;
#pragma unroll
    for (int s4 = 0; s4 < NS; ++s4)
#pragma unroll
      for (int p = 0; p < 3; ++p) {
#pragma unroll
        for (int mi = 0; mi < WM; ++mi)
          xa[mi][s4][p] = *reinterpret_cast<const bf16x8*>(
              base + p * PLANE + (wm * 32 * WM + mi * 32 + li) * LDK + kof + 16 * s4);
#pragma unroll
        for (int ni = 0; ni < WN; ++ni)
          xb[ni][s4][p] = *reinterpret_cast<const bf16x8*>(
              base + p * PLANE + (BM + wn * 32 * WN + ni * 32 + li) * LDK + kof + 16 * s4);
      }
  };
  // MFMA u of the tile's NS * WM * WN * 6 (u = ((s4 * WM + mi) * WN + ni) * 6 + term); terms in
  // increasing magnitude: a2b0, a1b1, a0b2, a1b0, a0b1, a0b0
  constexpr int NMF = NS * WM * WN * 6;
  auto mfmas = [&](int u_lo, int u_hi) {
#pragma unroll
    for (int u = u_lo; u < u_hi; ++u) {
      int term, t;
      if constexpr (V & 1) {  // accumulators interleaved: term-major inside each 16-deep step
        constexpr int A = WM * WN;
        term = (u % (6 * A)) / A;
        t = (u / (6 * A)) * A + u % A;
      } else {
        term = u % 6;
        t = u / 6;
      }
      const int ni = t % WN, mi = (t / WN) % WM, s4 = t / (WN * WM);
      constexpr int PA[6] = {2, 1, 0, 1, 0, 0}, PB[6] = {0, 1, 2, 0, 1, 0};
      acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[mi][s4][PA[term]],
                                                            fb[ni][s4][PB[term]], acc[mi][ni],
                                                            0, 0, 0);
    }
  };
  auto advance = [&]() {
#pragma unroll
    for (int s4 = 0; s4 < NS; ++s4)
#pragma unroll
      for (int p = 0; p < 3; ++p) {
#pragma unroll
        for (int mi = 0; mi < WM; ++mi) fa[mi][s4][p] = na[mi][s4][p];
#pragma unroll
        for (int ni = 0; ni < WN; ++ni) fb[ni][s4][p] = nb[ni][s4][p];
      }
  };

  const int nk = (K + BK - 1) / BK;
  const int nkr = (nk + D - 1) / D * D;
#pragma unroll
  for (int t0 = 0; t0 < AHEAD; ++t0) {
    gload(0, t0 * BK);
    swrite(t0, 0);
  }
#pragma unroll
  for (int j = 0; j < D; ++j) gload(j, (AHEAD + j) * BK);
  __syncthreads();
  sread(0, fa, fb);
  __syncthreads();  // every wave's tile-0 reads land before iteration 0 rewrites stage 0
  // Iteration t: multiply tile t (fragments in registers), read tile t+1's fragments from its
  // stage under the first MFMAs, write tile t+AHEAD into the stage of tile t+AHEAD-NSTG (read by
  // every wave before the last barrier) and re-arm the register slot; a barrier every SB tiles.
  constexpr int U1 = NMF / 3 > 0 ? NMF / 3 : 1;
  for (int kt = 0; kt < nkr; kt += D) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const int t = kt + j;
      __builtin_amdgcn_sched_barrier(0);
      if constexpr ((V & 2) != 0) __builtin_amdgcn_s_setprio(1);
      mfmas(0, U1);
      __builtin_amdgcn_sched_barrier(0);
      sread((t + 1) % NSTG, na, nb);
      __builtin_amdgcn_sched_barrier(0);
      mfmas(U1, NMF);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr ((V & 2) != 0) __builtin_amdgcn_s_setprio(0);
      swrite((t + AHEAD) % NSTG, j);
      gload(j, (t + AHEAD + D) * BK);
      if (SB == 1 || (j & 1)) __syncthreads();
      advance();
    }
  }

  if constexpr (KW > 1) {
    f32x16* red = reinterpret_cast<f32x16*>(smem_f);
    if (kw > 0) {
#pragma unroll
      for (int mi = 0; mi < WM; ++mi)
#pragma unroll
        for (int ni = 0; ni < WN; ++ni)
          red[(((kw - 1) * WAVES_MN + wmn) * WM * WN + mi * WN + ni) * 64 + lane] = acc[mi][ni];
    }
    __syncthreads();
    if (kw > 0) return;
#pragma unroll
    for (int g = 1; g < KW; ++g)
#pragma unroll
      for (int mi = 0; mi < WM; ++mi)
#pragma unroll
        for (int ni = 0; ni < WN; ++ni)
          acc[mi][ni] += red[(((g - 1) * WAVES_MN + wmn) * WM * WN + mi * WN + ni) * 64 + lane];
  }

#pragma unroll
  for (int mi = 0; mi < WM; ++mi)
#pragma unroll
    for (int ni = 0; ni < WN; ++ni) {
      const int col = n0 + wn * 32 * WN + ni * 32 + li, colc = min(col, N - 1);
      const int rbase = m0 + wm * 32 * WM + mi * 32 + 4 * lh;
      const float bv = a.bias ? a.bias[colc] : 0.f;
      float rv[16];
      if (a.R) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          rv[r] = a.R[(int64_t)min(rbase + (r & 3) + 8 * (r >> 2), M - 1) * a.ldr + colc];
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = rbase + (r & 3) + 8 * (r >> 2);
        float v = act_exact(acc[mi][ni][r] + bv, a.act);
        if (a.R) v = rv[r] + v;
        const int64_t coff = a.c_rpb ? (int64_t)(row / a.c_rpb) * a.c_bs +
                                           (int64_t)(row % a.c_rpb) * a.ldc
                                     : (int64_t)row * a.ldc;
        if (row < M && col < N) a.C[coff + col] = v;
      }
    }
}

// XCD-aware tile order: blocks are dealt round-robin over the 8 XCDs (hardware id % 8), each
// with its own L2; remap so that every XCD walks a contiguous run of tiles in column-major
// order (all row tiles of a column tile before the next), i.e. an XCD reads its W columns once
// and shares the activation rows through its L2 (bijective for any grid size).
__device__ __forceinline__ void xcd_remap(int& z, int& bx, int& by) {
  const int gx = gridDim.x, gy = gridDim.y, total = gx * gy * gridDim.z;
  const int hw = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const int xcd = hw & 7, slot = hw >> 3, q = total >> 3, r = total & 7;
  const int t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  z = t / (gx * gy);
  const int rem = t - z * gx * gy;
  bx = rem / gy;
  by = rem - bx * gy;
}

// wave-uniform selection of problem z (no dynamic indexing of the kernarg struct: it spills)
__device__ __forceinline__ GemmArgs select_problem(const GemmGroup& grp, int z) {
#define MPR_SEL(f) (z == 0 ? grp.g[0].f : z == 1 ? grp.g[1].f : z == 2 ? grp.g[2].f : grp.g[3].f)
  GemmArgs a;
  a.A = MPR_SEL(A); a.lda = MPR_SEL(lda); a.W = MPR_SEL(W); a.ldw = MPR_SEL(ldw);
  a.bias = MPR_SEL(bias); a.R = MPR_SEL(R); a.ldr = MPR_SEL(ldr); a.C = MPR_SEL(C);
  a.ldc = MPR_SEL(ldc); a.M = MPR_SEL(M); a.N = MPR_SEL(N); a.K = MPR_SEL(K);
  a.act = MPR_SEL(act); a.c_rpb = MPR_SEL(c_rpb); a.c_bs = MPR_SEL(c_bs);
  a.batch = MPR_SEL(batch); a.a_bs = MPR_SEL(a_bs); a.w_bs = MPR_SEL(w_bs);
  a.cb_bs = MPR_SEL(cb_bs); a.wp = MPR_SEL(wp);
#undef MPR_SEL
  return a;
}

// Problems of one tile configuration; blockIdx.z picks the problem.  XR: XCD-aware order
// (measured 3-5% slower for the 32x32 K-split tiles; neutral in time for 64x64, where it cuts
// the L2-miss traffic).
template <int BM, int BN, int WM, int WN, int BK, int D, int KW, bool XR>
__global__ __launch_bounds__(64 * (BM / (32 * WM)) * (BN / (32 * WN)) * KW) void gemm_f32_kernel(
    const GemmGroup grp) {
  // ONE __shared__ object: a second LDS object makes hipcc drain vmcnt before every k-step's
  // first ds_read.
  __shared__ __attribute__((aligned(16))) float smem[2 * (BM + BN) * (BK + 4)];
  int z = blockIdx.z, bx = blockIdx.x, by = blockIdx.y;
  if constexpr (XR) xcd_remap(z, bx, by);
  const GemmArgs a = select_problem(grp, z);
  if (by * BM >= a.M || bx * BN >= a.N) return;  // grid sized for the largest problem
  gemm_tile<BM, BN, WM, WN, BK, D, KW>(a, bx, by, smem);
}

template <int BM, int BN, int WM, int WN, int BK, int D, int KW, bool XR = false>
int launch_gemm_group(const GemmGroup& g, hipStream_t s) {
  constexpr int NT = 64 * (BM / (32 * WM)) * (BN / (32 * WN)) * KW;
  int gx = 0, gy = 0;
  for (int i = 0; i < g.n; ++i) {
    gx = std::max(gx, (int)cdiv(g.g[i].N, BN));
    gy = std::max(gy, (int)cdiv(g.g[i].M, BM));
  }
  hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WM, WN, BK, D, KW, XR>), dim3(gx, gy, g.n), dim3(NT),
                     0, s, g);
  MPR_LAUNCHED();
  return MPR_OK;
}

// Grid = exactly the launch's tiles (every problem's own cdiv(M, BM) x cdiv(N, BN), problems in
// order), one dimension.  Blocks are dealt round-robin over the 8 XCDs; the index is remapped so
// each XCD walks a contiguous run of the concatenated tile list, column-major inside a problem
// (an XCD reads its W columns once and shares activation rows through its L2).  Sizing the grid
// by the largest problem instead (blockIdx.z per problem) leaves the small problems' slices
// mostly empty, and the remap then gives whole XCDs nothing to do (the tower launches' text
// problems: fc2 231 -> see DESIGN §3).
template <int BM, int BN, int WM, int WN, int BK, int D, int KW, bool KT, int V = 0, int SB = 1>
__global__ __launch_bounds__(64 * (BM / (32 * WM)) * (BN / (32 * WN)) * KW) void gemm_x3_kernel(
    const GemmGroup grp) {
  __shared__ __attribute__((aligned(16))) float smem[x3_lds_floats<BM, BN, BK, SB>()];
  const int total = gridDim.x, hw = blockIdx.x;
  const int xcd = hw & 7, slot = hw >> 3, q = total >> 3, r = total & 7;
  int t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  int z = 0, gy = 0;
#pragma unroll
  for (int i = 0; i < GEMM_GROUP; ++i) {
    if (i == z && i < grp.n) {
      const int gyi = (int)cdiv(i == 0 ? grp.g[0].M : i == 1 ? grp.g[1].M : i == 2 ? grp.g[2].M
                                                                                  : grp.g[3].M,
                                BM);
      const int gxi = (int)cdiv(i == 0 ? grp.g[0].N : i == 1 ? grp.g[1].N : i == 2 ? grp.g[2].N
                                                                                  : grp.g[3].N,
                                BN);
      const int nbi = i == 0 ? grp.g[0].batch : i == 1 ? grp.g[1].batch : i == 2 ? grp.g[2].batch
                                                                                 : grp.g[3].batch;
      if (t >= gxi * gyi * nbi) {
        t -= gxi * gyi * nbi;
        ++z;
      } else {
        gy = gyi;
      }
    }
  }
  GemmArgs a = select_problem(grp, z);
  // Inside a problem the tiles go in bands of G row tiles, column-major inside a band, so the
  // contiguous run of ~total/8 tiles an XCD gets is about sqrt(run) rows x sqrt(run) columns:
  // its L2 then fetches ~2 sqrt(run) operand panels instead of all gy row panels plus run/gy
  // column panels (plain column-major order).  The order changes which XCD computes a tile,
  // never how: results are bit-identical.
  const int gx = (int)cdiv(z == 0 ? grp.g[0].N : z == 1 ? grp.g[1].N : z == 2 ? grp.g[2].N
                                                                       : grp.g[3].N, BN);
  if (a.batch > 1) {  // batch copy b: the b-th run of gx * gy tiles
    const int b = t / (gx * gy);
    t -= b * gx * gy;
    a.A += b * a.a_bs;
    a.W += b * a.w_bs;
    a.C += b * a.cb_bs;
  }
  const int run = (total + 7) >> 3;
  int G = 1;
  while ((G + 1) * (G + 1) <= run) ++G;
  G = G < gy ? G : gy;
  const int full = gy / G * G, band = G * gx;
  int bx, by;
  if (t < (full / G) * band) {
    const int gb = t / band, tt = t - gb * band;
    bx = tt / G;
    by = gb * G + (tt - bx * G);
  } else {  // the last, shorter band
    const int rem = gy - full, tt = t - (full / G) * band;
    bx = tt / rem;
    by = full + (tt - bx * rem);
  }
  gemm_x3_tile<BM, BN, WM, WN, BK, D, KW, KT, V, SB>(a, bx, by, smem);
}

// KT when some K % BK != 0 or cdiv(K, BK) % D != 0
template <int BM, int BN, int WM, int WN, int BK, int D, int KW, int V = 0, int SB = 1>
int launch_gemm_x3_group(const GemmGroup& g, hipStream_t s) {
  constexpr int NT = 64 * (BM / (32 * WM)) * (BN / (32 * WN)) * KW;
  int64_t tiles = 0;
  bool kt = false;
  for (int i = 0; i < g.n; ++i) {
    tiles += cdiv(g.g[i].N, BN) * cdiv(g.g[i].M, BM) * g.g[i].batch;
    // masked K tail also when the tile count is not a multiple of D: the main loop multiplies
    // whole groups of D tiles, and an unmasked tile past K would add clamped (repeated) columns
    kt = kt || g.g[i].K % BK != 0 || cdiv(g.g[i].K, BK) % D != 0;
  }
  if (tiles == 0) return MPR_OK;
  if (kt)
    hipLaunchKernelGGL((gemm_x3_kernel<BM, BN, WM, WN, BK, D, KW, true, V, SB>),
                       dim3((unsigned)tiles), dim3(NT), 0, s, g);
  else
    hipLaunchKernelGGL((gemm_x3_kernel<BM, BN, WM, WN, BK, D, KW, false, V, SB>),
                       dim3((unsigned)tiles),
                       dim3(NT), 0, s, g);
  MPR_LAUNCHED();
  return MPR_OK;
}

// ---- split-bf16 GEMM with a packed W ("x3p") ------------------------------------------------
// The tower and T5-encoder weights are fixed for the life of a model, so their split is done
// once: pack_x3 writes W as the three bf16 planes in v_mfma_f32_32x32x16_bf16 operand order,
// [cdiv(N, 32) column tiles][cdiv(K, 16) k steps][3 planes][64 lanes][8 bf16] (lane (li, lh):
// column 32 t + li, k = 16 s + 8 lh .. +7; zero past N and K), and each wave loads its W
// fragments straight into registers — 1 KiB contiguous per wave load — D k steps ahead.  Only A
// goes through LDS.  Measured on the tower shapes with the LDS traffic of W removed from the
// 128x128 kernel (profiles/r04_x3_lds_diag.txt): 80.6 -> 56.5 us (qkv 1600x2304x768 x2), 109.7
// -> 77.4 (fc1): the LDS fragment traffic, not the MFMA issue, sets that kernel's pace.  Every
// output element is accumulated in the same order with the same split terms as gemm_x3_tile
// (W split by the same split3, per element): bit-identical results.  (Measured and dropped: W
// kept as fp32 in the same operand order — 4 bytes per element instead of 6 — and split in
// registers by each wave: 5-15 % slower than the planes, close to the LDS kernel again;
// profiles/r04_x3p_f32frag_ab.txt.)
__global__ __launch_bounds__(256) void pack_x3_kernel(const float* __restrict__ W, int N, int K,
                                                      int64_t ldw, int KS, bf16x8* __restrict__ out) {
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;  // one (column tile, k step, lane)
  const int64_t total = cdiv(N, 32) * (int64_t)KS * 64;
  if (q >= total) return;
  const int lane = (int)(q & 63);
  const int64_t t = q >> 6;
  const int ks = (int)(t % KS);
  const int n = (int)(t / KS) * 32 + (lane & 31), k0 = ks * 16 + 8 * (lane >> 5);
  f32x4 lo = {0.f, 0.f, 0.f, 0.f}, hi = {0.f, 0.f, 0.f, 0.f};
  if (n < N) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (k0 + e < K) lo[e] = W[(int64_t)n * ldw + k0 + e];
      if (k0 + 4 + e < K) hi[e] = W[(int64_t)n * ldw + k0 + 4 + e];
    }
  }
  bf16x8 h0, h1, h2;
  x3::split8(lo, hi, h0, h1, h2);
  out[(t * 3 + 0) * 64 + lane] = h0;
  out[(t * 3 + 1) * 64 + lane] = h1;
  out[(t * 3 + 2) * 64 + lane] = h2;
}

// SB = 2: four A stages and a block barrier every second K tile (tile t + 3 is written while
// tile t + 1 is read; each stage is rewritten two iterations after its last read, with a barrier
// in between), half the barriers of SB = 1 (two stages, one barrier per K tile).
template <int BM, int BN, int WM, int WN, int D, bool KT, int BK = 16, int SB = 1>
__device__ __forceinline__ void gemm_x3p_tile(const GemmArgs& a, int bx, int by, float* smem_f) {
  static_assert(SB == 1 || (SB == 2 && D % 2 == 0), "SB = 2 needs an even D");
  constexpr int NSTG = 2 * SB, AHEAD = SB + 1;  // A stages; tile written at iteration t: t + AHEAD
  constexpr int NS = BK / 16;  // 16-deep MFMA steps per K tile
  constexpr int WAVES_N = BN / (32 * WN);
  constexpr int WAVES_MN = (BM / (32 * WM)) * WAVES_N;
  constexpr int NT = 64 * WAVES_MN;
  constexpr int LDK = BK + 8, KQ = BK / 4;
  constexpr int LA = BM * KQ / NT;
  constexpr int PLANE = BM * LDK;   // bf16 per plane (A rows only)
  constexpr int STAGE = 3 * PLANE;
  static_assert(LA >= 1 && LA * NT == BM * KQ && NS * 16 == BK, "loader split");
  __bf16* smem = reinterpret_cast<__bf16*>(smem_f);
  const int M = a.M, N = a.N, K = a.K;
  const int m0 = by * BM, n0 = bx * BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wmn = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wmn / WAVES_N, wn = wmn % WAVES_N;
  const int KS = (K + 15) / 16, NTW = (N + 31) / 32;
  const bf16x8* wpk[WN];
#pragma unroll
  for (int ni = 0; ni < WN; ++ni)
    wpk[ni] = reinterpret_cast<const bf16x8*>(a.wp) +
              (int64_t)min(n0 / 32 + wn * WN + ni, NTW - 1) * KS * 3 * 64 + lane;

  f32x4 ra[D][LA];
  bool oka[D][LA];
  bf16x8 bq[D][NS][WN][3];
  auto aload = [&](int j, int kt) {
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int idx = tid + i * NT, r = idx / KQ, c = k0 + (idx % KQ) * 4, row = m0 + r;
      if constexpr (KT) oka[j][i] = c < K;
      ra[j][i] = *reinterpret_cast<const f32x4*>(a.A + (int64_t)min(row, M - 1) * a.lda +
                                                 min(c, K - 4));
    }
  };
  auto bload = [&](int j, int kt) {  // past the last k step: an in-range step (A is zero there)
#pragma unroll
    for (int s4 = 0; s4 < NS; ++s4) {
      const int ks = min(kt * NS + s4, KS - 1);
#pragma unroll
      for (int ni = 0; ni < WN; ++ni)
#pragma unroll
        for (int p = 0; p < 3; ++p) bq[j][s4][ni][p] = wpk[ni][((int64_t)ks * 3 + p) * 64];
    }
  };
  auto put = [&](__bf16* base, int row, int kc, const f32x4& v) {
    bf16x4 h0, h1, h2;
    split3(v, h0, h1, h2);
    __bf16* p = base + row * LDK + kc;
    *reinterpret_cast<bf16x4*>(p) = h0;
    *reinterpret_cast<bf16x4*>(p + PLANE) = h1;
    *reinterpret_cast<bf16x4*>(p + 2 * PLANE) = h2;
  };
  auto swrite = [&](int st, int j) {
    const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
    __bf16* base = smem + st * STAGE;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int idx = tid + i * NT;
      if constexpr (KT) put(base, idx / KQ, (idx % KQ) * 4, oka[j][i] ? ra[j][i] : zero);
      else put(base, idx / KQ, (idx % KQ) * 4, ra[j][i]);
    }
  };

  f32x16 acc[WM][WN];
#pragma unroll
  for (int mi = 0; mi < WM; ++mi)
#pragma unroll
    for (int ni = 0; ni < WN; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;

  const int li = lane & 31, lh = lane >> 5;
  bf16x8 fa[NS][WM][3], na[NS][WM][3];
  auto sread = [&](int st, bf16x8(&xa)[NS][WM][3]) {
    const __bf16* base = smem + st * STAGE;
#pragma unroll
    for (int s4 = 0; s4 < NS; ++s4)
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int mi = 0; mi < WM; ++mi)
          xa[s4][mi][p] = *reinterpret_cast<const bf16x8*>(
              base + p * PLANE + (wm * 32 * WM + mi * 32 + li) * LDK + 16 * s4 + 8 * lh);
  };
  // MFMA u of the tile's NS * WM * WN * 6 (u = ((s4 * WM + mi) * WN + ni) * 6 + term: every
  // accumulator takes its 16-deep steps in k order), terms in gemm_x3_tile's order: a2b0, a1b1,
  // a0b2, a1b0, a0b1, a0b0
  constexpr int NMF = NS * WM * WN * 6;
  auto mfmas = [&](int j, int u_lo, int u_hi) {
#pragma unroll
    for (int u = u_lo; u < u_hi; ++u) {
      const int term = u % 6, t = u / 6, ni = t % WN, mi = (t / WN) % WM, s4 = t / (WN * WM);
      constexpr int PA[6] = {2, 1, 0, 1, 0, 0}, PB[6] = {0, 1, 2, 0, 1, 0};
      acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
          fa[s4][mi][PA[term]], bq[j][s4][ni][PB[term]], acc[mi][ni], 0, 0, 0);
    }
  };

  const int nk = (K + BK - 1) / BK;
  const int nkr = (nk + D - 1) / D * D;
#pragma unroll
  for (int t0 = 0; t0 < AHEAD; ++t0) {
    aload(0, t0);
    swrite(t0, 0);
  }
#pragma unroll
  for (int j = 0; j < D; ++j) {
    aload(j, AHEAD + j);
    bload(j, j);
  }
  __syncthreads();
  sread(0, fa);
  __syncthreads();
  // Iteration t: multiply tile t (A fragments read the iteration before, W fragments loaded D
  // iterations before), read tile t+1's A fragments from its stage, write tile t+AHEAD's A into
  // the stage of tile t+AHEAD-NSTG (read by every wave before the last barrier), re-arm the
  // register slots with tile t+AHEAD+D's A and tile t+D's W.
  constexpr int U1 = NMF / 3 > 0 ? NMF / 3 : 1;
  for (int kt = 0; kt < nkr; kt += D) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const int t = kt + j;
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
      mfmas(j, 0, U1);
      __builtin_amdgcn_sched_barrier(0);
      sread((t + 1) % NSTG, na);
      __builtin_amdgcn_sched_barrier(0);
      mfmas(j, U1, NMF);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(0);
      swrite((t + AHEAD) % NSTG, j);
      aload(j, t + AHEAD + D);
      bload(j, t + D);
      if (SB == 1 || (j & 1)) __syncthreads();
#pragma unroll
      for (int s4 = 0; s4 < NS; ++s4)
#pragma unroll
        for (int mi = 0; mi < WM; ++mi)
#pragma unroll
          for (int p = 0; p < 3; ++p) fa[s4][mi][p] = na[s4][mi][p];
    }
  }

#pragma unroll
  for (int mi = 0; mi < WM; ++mi)
#pragma unroll
    for (int ni = 0; ni < WN; ++ni) {
      const int col = n0 + wn * 32 * WN + ni * 32 + li, colc = min(col, N - 1);
      const int rbase = m0 + wm * 32 * WM + mi * 32 + 4 * lh;
      const float bv = a.bias ? a.bias[colc] : 0.f;
      float rv[16];
      if (a.R) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          rv[r] = a.R[(int64_t)min(rbase + (r & 3) + 8 * (r >> 2), M - 1) * a.ldr + colc];
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = rbase + (r & 3) + 8 * (r >> 2);
        float v = act_exact(acc[mi][ni][r] + bv, a.act);
        if (a.R) v = rv[r] + v;
        const int64_t coff = a.c_rpb ? (int64_t)(row / a.c_rpb) * a.c_bs +
                                           (int64_t)(row % a.c_rpb) * a.ldc
                                     : (int64_t)row * a.ldc;
        if (row < M && col < N) a.C[coff + col] = v;
      }
    }
}

// gemm_x3_kernel's grid and tile order, the packed-W tile
template <int BM, int BN, int WM, int WN, int D, bool KT, int BK = 16, int SB = 1>
__global__ __launch_bounds__(64 * (BM / (32 * WM)) * (BN / (32 * WN))) void gemm_x3p_kernel(
    const GemmGroup grp) {
  __shared__ __attribute__((aligned(16))) float smem[2 * SB * 3 * BM * (BK + 8) / 2];
  const int total = gridDim.x, hw = blockIdx.x;
  const int xcd = hw & 7, slot = hw >> 3, q = total >> 3, r = total & 7;
  int t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  int z = 0, gy = 0;
#pragma unroll
  for (int i = 0; i < GEMM_GROUP; ++i) {
    if (i == z && i < grp.n) {
      const int gyi = (int)cdiv(i == 0 ? grp.g[0].M : i == 1 ? grp.g[1].M : i == 2 ? grp.g[2].M
                                                                                  : grp.g[3].M,
                                BM);
      const int gxi = (int)cdiv(i == 0 ? grp.g[0].N : i == 1 ? grp.g[1].N : i == 2 ? grp.g[2].N
                                                                                  : grp.g[3].N,
                                BN);
      if (t >= gxi * gyi) {
        t -= gxi * gyi;
        ++z;
      } else {
        gy = gyi;
      }
    }
  }
  const GemmArgs a = select_problem(grp, z);
  const int gx = (int)cdiv(a.N, BN);
  const int run = (total + 7) >> 3;
  int G = 1;
  while ((G + 1) * (G + 1) <= run) ++G;
  G = G < gy ? G : gy;
  const int full = gy / G * G, band = G * gx;
  int bx, by;
  if (t < (full / G) * band) {
    const int gb = t / band, tt = t - gb * band;
    bx = tt / G;
    by = gb * G + (tt - bx * G);
  } else {
    const int rem = gy - full, tt = t - (full / G) * band;
    bx = tt / rem;
    by = full + (tt - bx * rem);
  }
  gemm_x3p_tile<BM, BN, WM, WN, D, KT, BK, SB>(a, bx, by, smem);
}

template <int BM, int BN, int WM, int WN, int D, int BK = 16, int SB = 1>
int launch_gemm_x3p_group(const GemmGroup& g, hipStream_t s) {
  constexpr int NT = 64 * (BM / (32 * WM)) * (BN / (32 * WN));
  int64_t tiles = 0;
  bool kt = false;
  for (int i = 0; i < g.n; ++i) {
    tiles += cdiv(g.g[i].N, BN) * cdiv(g.g[i].M, BM);
    kt = kt || g.g[i].K % BK != 0 || cdiv(g.g[i].K, BK) % D != 0;
  }
  if (tiles == 0) return MPR_OK;
  if (kt)
    hipLaunchKernelGGL((gemm_x3p_kernel<BM, BN, WM, WN, D, true, BK, SB>), dim3((unsigned)tiles),
                       dim3(NT), 0, s, g);
  else
    hipLaunchKernelGGL((gemm_x3p_kernel<BM, BN, WM, WN, D, false, BK, SB>), dim3((unsigned)tiles),
                       dim3(NT), 0, s, g);
  MPR_LAUNCHED();
  return MPR_OK;
}

template <int BM, int BN, int WM, int WN, int BK = 32, int D = 2, int KW = 1>
int launch_gemm(const GemmArgs& a, hipStream_t s) {
  GemmGroup g;
  g.g[0] = a;
  g.n = 1;
  return launch_gemm_group<BM, BN, WM, WN, BK, D, KW>(g, s);
}

// ---------------------------------------------------------------------------------------------
// Skinny GEMM (M <= 16), optional fused RMSNorm of the A rows.
// A block = 8 waves = NT tiles of 16 output columns; wave w owns the K slice w of the rows.
// v_mfma_f32_16x16x4_f32 wants lane (i, h) to hold row i, k = 4h..4h+3 of a 16-column chunk, so
// adjacent lanes sit on different rows; loading that straight from row-major memory scatters
// every wave load over 16 rows (measured: ~0.85 us of a 3.5 us kernel).  Both operands therefore
// arrive lane-contiguous: W from its pack_rows16 image (1 KiB per wave load), A rows through a
// wave-private LDS slab filled with 256-byte row segments and read back as MFMA fragments
// (wave-private: no block barrier, the wave's own LDS ops stay in order).
// With RMSNorm fused, the operand is ln_w[k] * A[m,k] and the per-row 1/rms (from the squares of
// the same loaded A values, summed across the block) scales the accumulator in the epilogue.
constexpr int SK_WAVES = 8;

__global__ __launch_bounds__(256) void pack_rows16_kernel(const float* __restrict__ W, int64_t N,
                                                          int64_t K, int64_t ldw, int64_t nch,
                                                          float* __restrict__ out) {
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;  // one float4 of the image
  const int64_t total = cdiv(N, 16) * nch * 64;
  if (q >= total) return;
  const int l = (int)(q & 63);
  const int64_t tc = q >> 6, t = tc / nch, c = tc % nch;
  const int64_t row = t * 16 + (l & 15), k0 = c * 16 + (l >> 4) * 4;
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  if (row < N) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (k0 + e < K) v[e] = W[row * ldw + k0 + e];
  }
  reinterpret_cast<f32x4*>(out)[q] = v;
}

// Every option is a template flag: measured on MI355X, each runtime-optional part of this
// kernel (a residual/bias branch, an argmax branch, a K loop) added 0.4-0.6 us to a ~3 us
// launch, so each launch carries only the code its call needs, straight-line.
// SKF_RELU_IN: ReLU applied to the A operand as it is staged (relu commutes with the positive
// per-row scale of SKF_RSCALE); SKF_RSCALE: the epilogue scales row m by rsqrt(mean(src_m^2) +
// eps) of an external row (the decode chain's folded RMSNorm, t5.hip).
enum : int { SKF_RMS = 1, SKF_RES = 2, SKF_RELU = 4, SKF_AMAX = 8, SKF_RELU_IN = 16,
             SKF_RSCALE = 32, SKF_SSQ = 64 };

// NT 16-column tiles per block share the activation slab (NT > 1 for the 32k-column lm_head,
// which needs more bytes in flight per wave); two accumulator chains per tile halve the
// dependent-MFMA latency.  MAXC = chunks of 16 columns staged per pass; LOOP = more than one
// pass (K > 16 * 8 * MAXC).  (Issuing the next pass's loads before this pass's slab round trip,
// two register sets at half the MAXC, measured no faster: 32-row FFN-out 10.32 vs 10.24 us.)
template <int MAXC, int NT, int F, bool LOOP, int MR, int SK_WAVES = 8>
__global__ __launch_bounds__(64 * SK_WAVES) void gemm_skinny_kernel(SkinnyArgs sa) {
  constexpr bool RMS = (F & SKF_RMS) != 0, RES = (F & SKF_RES) != 0,
                 RELU = (F & SKF_RELU) != 0, AMAX = (F & SKF_AMAX) != 0,
                 RELU_IN = (F & SKF_RELU_IN) != 0, RSCALE = (F & SKF_RSCALE) != 0,
                 SSQ = (F & SKF_SSQ) != 0;
  static_assert(!(RMS && RSCALE), "one row-scale source");
  constexpr int MROWS = 16 * MR;      // activation rows: MR 16-row groups share each weight load
  const GemmArgs& a = sa.g;
  constexpr int XLD = MAXC * 16 + 4;  // slab row stride (floats): conflict-free fragment reads
  constexpr int XS = SK_WAVES * MROWS * XLD;
  // one LDS object: activation slabs | per-wave sums of squares.  After its K slice a wave
  // parks its NT * MR partial tiles in its own slab (wave-private until the block barrier), so
  // the partials cost no LDS of their own: more blocks stay resident per CU.
  static_assert(NT * MR * 256 <= MROWS * XLD, "partial tiles must fit the wave's slab");
  __shared__ __attribute__((aligned(16))) float smem[XS + SK_WAVES * MROWS +
                                                     (RSCALE ? MROWS : 0)];
  float(*xs)[MROWS][XLD] = reinterpret_cast<float(*)[MROWS][XLD]>(smem);
  auto red = [&](int slot, int w) -> f32x4* {  // partial tile `slot` of wave w, 64 lanes
    return reinterpret_cast<f32x4*>(smem + w * MROWS * XLD) + slot * 64;
  };
  float(*ssq_s)[MROWS] = reinterpret_cast<float(*)[MROWS]>(smem + XS);
  const int tid = threadIdx.x, lane = tid & 63;
  if (sa.poison) {  // debug: a read of LDS this block never wrote yields NaN
    for (int i = tid; i < (int)(sizeof(smem) / sizeof(float)); i += 64 * SK_WAVES)
      smem[i] = __builtin_nanf("");
    __syncthreads();
  }
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR)
  // blockIdx.y = a block of MROWS rows (a grouped decode's rows split over blocks); rows are
  // independent, so each row's sums keep their order whatever the split
  const int row0 = blockIdx.y * MROWS;
  const float* __restrict__ Ab = a.A + (int64_t)row0 * a.lda;
  const int M = min(a.M - row0, MROWS), N = a.N, K = a.K;
  const int i = lane & 15, h = lane >> 4;

  const int nchunk = (K + 15) / 16;
  const int ntiles = (N + 15) / 16;
  const int per = (nchunk + SK_WAVES - 1) / SK_WAVES;
  const int c_lo = wave * per, c_hi = min(nchunk, c_lo + per);
  const int c_safe = min(c_lo, nchunk - 1);  // an in-range chunk for padding reads
  // (a tile past N — the lm_head's last block — re-reads the last tile; never stored)
  const f32x4* wp[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
    wp[t] = reinterpret_cast<const f32x4*>(sa.wpk) +
            ((int64_t)min((int)blockIdx.x * NT + t, ntiles - 1) * nchunk) * 64 + lane;
  // Epilogue wave w finishes tile w % NT for row group w / NT.  The lane's 4 outputs are row
  // 16 * group + i, columns n0 + 4h .. +3 (16x16 D layout): its residual is one float4, fetched
  // before the main loads.
  const int et = wave % NT, er = wave / NT;
  f32x4 rres = {0.f, 0.f, 0.f, 0.f};
  if constexpr (RES) {
    if (wave < NT * MR)
      rres = *reinterpret_cast<const f32x4*>(a.R + (int64_t)(row0 + min(er * 16 + i, M - 1)) * a.ldr +
                                             min((int)blockIdx.x * NT + et, ntiles - 1) * 16 + h * 4);
  }
  // RSCALE: the rows' partial sums of squares (<= 64 per row): wave w loads those of rows w,
  // w + 8, ... (lane = partial), issued with the first loads, summed after the main loop
  constexpr int RPW = MROWS / SK_WAVES;  // rows per wave (1, 2 or 4)
  float rsp[RSCALE ? RPW : 1];
  if constexpr (RSCALE) {
#pragma unroll
    for (int u = 0; u < RPW; ++u)
      rsp[u] = lane < sa.rs_nparts
                   ? sa.rs_part[(int64_t)(row0 + min(wave + u * SK_WAVES, M - 1)) * sa.rs_nparts + lane]
                   : 0.f;
  }
  f32x4 acc[NT][MR][2];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < MR; ++r) acc[t][r][0] = acc[t][r][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ss[MR];
#pragma unroll
  for (int r = 0; r < MR; ++r) ss[r] = 0.f;
#pragma unroll 1
  for (int c0 = c_lo; LOOP ? c0 < c_hi : c0 == c_lo; c0 += MAXC) {
    // weights first (the long pole), then this pass's activation rows as 256-byte segments:
    // float4 q of the pass = row q / (4*MAXC), column (q % (4*MAXC)) * 4 of the pass
    f32x4 wv[NT][MAXC], xr[MR * MAXC], gv[MAXC];
#pragma unroll
    for (int u = 0; u < MAXC; ++u) {
      // a chunk past the wave's slice re-reads an in-range chunk; its activations are zero
      const int c = c0 + u, cc = c < c_hi ? c : c_safe;
#pragma unroll
      for (int t = 0; t < NT; ++t) wv[t][u] = wp[t][(int64_t)cc * 64];
      if constexpr (RMS) gv[u] = *reinterpret_cast<const f32x4*>(sa.rms_w + cc * 16 + h * 4);
    }
#pragma unroll
    for (int u = 0; u < MR * MAXC; ++u) {
      const int q = u * 64 + lane, row = q / (4 * MAXC), col = c0 * 16 + (q % (4 * MAXC)) * 4;
      const bool ok = row < M && col < c_hi * 16 && col < K;
      xr[u] = *reinterpret_cast<const f32x4*>(Ab + (int64_t)min(row, M - 1) * a.lda +
                                              min(col, K - 4));
      if (!ok) xr[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if constexpr (RELU_IN) {
#pragma unroll
      for (int u = 0; u < MR * MAXC; ++u)
#pragma unroll
        for (int e = 0; e < 4; ++e) xr[u][e] = xr[u][e] > 0.f ? xr[u][e] : 0.f;
    }
    // every load of the pass is in flight before the first wait (hipcc otherwise sinks the
    // weight loads next to their MFMAs, behind the activation round trip through LDS)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < MR * MAXC; ++u) {
      const int q = u * 64 + lane;
      *reinterpret_cast<f32x4*>(&xs[wave][q / (4 * MAXC)][(q % (4 * MAXC)) * 4]) = xr[u];
    }
#pragma unroll
    for (int u = 0; u < MAXC; ++u) {
      f32x4 xv[MR];
#pragma unroll
      for (int r = 0; r < MR; ++r) {
        xv[r] = *reinterpret_cast<const f32x4*>(&xs[wave][r * 16 + i][u * 16 + h * 4]);
        if constexpr (RMS) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            ss[r] += xv[r][e] * xv[r][e];
            xv[r][e] = gv[u][e] * xv[r][e];
          }
        }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int r = 0; r < MR; ++r)
            acc[t][r][u & 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[t][u][e], xv[r][e],
                                                                    acc[t][r][u & 1], 0, 0, 0);
    }
  }
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < MR; ++r) red(r * NT + t, wave)[lane] = acc[t][r][0] + acc[t][r][1];
  if constexpr (RMS) {
#pragma unroll
    for (int r = 0; r < MR; ++r) {
      float v = ss[r];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (lane < 16) ssq_s[wave][r * 16 + lane] = v;
    }
  }
  float* rsp_s = smem + XS + SK_WAVES * MROWS;  // RSCALE row sums of squares [MROWS]
  if constexpr (RSCALE) {
#pragma unroll
    for (int u = 0; u < RPW; ++u) {
      float v = rsp[u];
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
      if (lane == 0) rsp_s[wave + u * SK_WAVES] = v;
    }
  }
  __syncthreads();
  if (wave < NT * MR) {
    const int tile = blockIdx.x * NT + et;
    const int n0 = tile * 16, m = er * 16 + i;
    f32x4 sum = red(wave, 0)[lane];  // partial slot er * NT + et == wave
  #pragma unroll
    for (int w = 1; w < SK_WAVES; ++w) sum += red(wave, w)[lane];
    // D[row = W row (n), col = A row (m)]: col = lane&15, row = (lane>>4)*4 + r.
    float scale = sa.a_scale;
    if constexpr (RMS) {
      float t = 0.f;
  #pragma unroll
      for (int w = 0; w < SK_WAVES; ++w) t += ssq_s[w][m];
      scale = (1.0f / sqrtf(t / (float)K + sa.rms_eps)) * sa.a_scale;
    }
    if constexpr (RSCALE) {
      scale = (1.0f / sqrtf(rsp_s[m] / (float)sa.rs_n + sa.rms_eps)) * sa.a_scale;
    }
    if constexpr (AMAX) {
      // greedy head: per (row m, block) best column, lowest index on ties (torch.argmax)
      float bv = -INFINITY;
      int bi = 0x7fffffff;
  #pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + h * 4 + r;
        const float v = sum[r] * scale;
        if (n < N && (v > bv || (v == bv && n < bi))) {
          bv = v;
          bi = n;
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
      if (lane < 16 && n0 < N && m < M) {  // row-major [rows][ntiles]: greedy_step reads rows
        sa.amax_val[(int64_t)(row0 + m) * ntiles + tile] = bv;  // coalesced
        sa.amax_idx[(int64_t)(row0 + m) * ntiles + tile] = bi;
      }
    } else {
      f32x4 v = sum * scale;
      if constexpr (RELU) {
  #pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : 0.f;
      }
      if constexpr (RES) v = rres + v;
      if (m < M && n0 < N) *reinterpret_cast<f32x4*>(a.C + (int64_t)(row0 + m) * a.ldc + n0 + h * 4) = v;
      if constexpr (SSQ) {
        // the tile's 16 columns of row m: this lane's 4, then the 4 lane groups (h) of the row
        float q = v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
        q += __shfl_xor(q, 16, 64);
        q += __shfl_xor(q, 32, 64);
        if (n0 < sa.ssq_cols && lane < 16 && m < M)
          sa.ssq_out[(int64_t)(row0 + m) * (sa.ssq_cols / 16) + tile] = q;
      }
    }
  }
}


// ---- kernel probe: hipEvent pairs around every GEMM launch of the probed kind ----------------
struct ProbeRec {
  hipEvent_t a, b;
  double flops, bytes;
};
int g_probe_kind = 0;
std::vector<ProbeRec> g_recs;
std::vector<hipEvent_t> g_pool;

hipEvent_t pool_event() {
  if (!g_pool.empty()) {
    hipEvent_t e = g_pool.back();
    g_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

bool probing(int kind, hipStream_t s) {
  if (g_probe_kind != kind) return false;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &st) != hipSuccess || st != hipStreamCaptureStatusNone) return false;
  return true;
}

double gemm_bytes(const GemmArgs& a) {
  return 4.0 * ((double)a.M * a.K + (double)a.N * a.K + (double)a.M * a.N * (a.R ? 2 : 1) +
                (a.bias ? a.N : 0));
}

// PROBE_RECORD: every tiled-GEMM launch group (outside capture) is kept for probe_replay().
std::vector<GemmGroup> g_recorded;

template <class F>
int probed(int kind, double flops, double bytes, hipStream_t s, F&& launch) {
  if (!probing(kind, s)) return launch();
  ProbeRec r{pool_event(), pool_event(), flops, bytes};
  if (!r.a || !r.b) return launch();
  (void)hipEventRecord(r.a, s);
  const int rc = launch();
  (void)hipEventRecord(r.b, s);
  g_recs.push_back(r);
  return rc;
}

}  // namespace

int probe_kind() { return g_probe_kind; }

int probe_enable(int kind) {
  g_probe_kind = kind;
  return MPR_OK;
}

__global__ void probe_marker_kernel(int tag, int* sink) {
  if (tag < 0) sink[0] = tag;  // never true: the launch itself is the marker
}

int probe_replay(int iters, hipStream_t s, double* ms, int64_t* launches, double* flops,
                 double* bytes) {
  MPR_REQUIRE(iters >= 1, "probe_replay: iters=%d", iters);
  // Outputs go to a scratch buffer (the recorded C pointers may be tensors the caller freed);
  // inputs are read where they were (library workspaces, still mapped).
  size_t cmax = 0;
  for (const GemmGroup& g : g_recorded)
    for (int i = 0; i < g.n; ++i) {
      const GemmArgs& a = g.g[i];
      const int64_t r = a.M - 1;
      const int64_t last = (a.c_rpb ? (r / a.c_rpb) * a.c_bs + (r % a.c_rpb) * a.ldc + a.N
                                    : r * a.ldc + a.N) + (int64_t)(a.batch - 1) * a.cb_bs;
      cmax = std::max(cmax, (size_t)last * sizeof(float));
    }
  static DevBuf scratch;
  MPR_TRY(scratch.ensure(std::max<size_t>(cmax, 256)));
  // One event pair around the whole back-to-back replay (an event pair around every launch
  // added ~14 us of dispatch gap per launch: 96.5 vs rocprofv3's 82.2 us kernel average, r02_v9)
  hipLaunchKernelGGL(probe_marker_kernel, dim3(1), dim3(64), 0, s, 1, scratch.as<int>());
  hipEvent_t e0 = pool_event(), e1 = pool_event();
  MPR_REQUIRE(e0 && e1, "probe_replay: no events");
  MPR_HIP(hipEventRecord(e0, s));
  double f = 0, by = 0;
  int64_t n = 0;
  for (int it = 0; it < iters; ++it)
    for (const GemmGroup& g0 : g_recorded) {
      GemmGroup g = g0;
      for (int i = 0; i < g.n; ++i) {
        g.g[i].C = scratch.as<float>();
        if (g.g[i].R == g0.g[i].C) g.g[i].R = scratch.as<float>();  // in-place residual
        f += 2.0 * g.g[i].M * g.g[i].N * g.g[i].K * g.g[i].batch;
        by += gemm_bytes(g.g[i]) * g.g[i].batch;
      }
      const int saved = g_probe_kind;
      g_probe_kind = PROBE_OFF;
      const int rc = gemm_group(g, s);
      g_probe_kind = saved;
      MPR_TRY(rc);
      ++n;
    }
  MPR_HIP(hipEventRecord(e1, s));
  hipLaunchKernelGGL(probe_marker_kernel, dim3(1), dim3(64), 0, s, 2, scratch.as<int>());
  float e = 0.f;
  MPR_HIP(hipEventSynchronize(e1));
  MPR_HIP(hipEventElapsedTime(&e, e0, e1));
  g_pool.push_back(e0);
  g_pool.push_back(e1);
  if (ms) *ms = e;
  if (launches) *launches = n;
  if (flops) *flops = f;
  if (bytes) *bytes = by;
  return MPR_OK;
}

int probe_clear() {
  g_recorded.clear();
  return MPR_OK;
}

int probe_read(double* ms, int64_t* launches, double* flops, double* bytes) {
  double t = 0, f = 0, by = 0;
  for (auto& r : g_recs) {
    float e = 0.f;
    MPR_HIP(hipEventSynchronize(r.b));
    MPR_HIP(hipEventElapsedTime(&e, r.a, r.b));
    t += e;
    f += r.flops;
    by += r.bytes;
    g_pool.push_back(r.a);
    g_pool.push_back(r.b);
  }
  if (ms) *ms = t;
  if (launches) *launches = (int64_t)g_recs.size();
  if (flops) *flops = f;
  if (bytes) *bytes = by;
  g_recs.clear();
  return MPR_OK;
}

namespace {
// One launch of problems that share a tile configuration (probed / recorded as one launch).
// Kernel families of one launch.  F32_*: exact f32 MFMA (v_mfma_f32_32x32x2_f32), the round-1
// kernels, kept behind MPR_GEMM=f32.  X3_*: the split-bf16 kernels (default).  Within X3_WIDE /
// X3_TALL (16-deep k steps in order, KW = 1) every output element is accumulated in the same
// order whatever the block tile, so the tile may follow the launch (grouped or alone, one batch
// or two concatenated: bit-identical results).
enum GemmKind : int {
  F32_BIG = 0, F32_SMALL = 1, X3_WIDE = 2, X3_TALL = 3, X3_SMALL = 4, X3_WIDE32 = 5,
  X3P_WIDE = 6, X3P_SMALL = 7, X3P_SMALL3 = 8, X3_WIDE_SB2 = 9, X3_SMALL_SB2 = 10
};


const bool g_gemm_f32 = [] {
  const char* e = getenv("MPR_GEMM");
  return e && strcmp(e, "f32") == 0;
}();

const bool g_x3_sb1 = [] {
  const char* e = getenv("MPR_X3_SB");
  return e && e[0] == '1';
}();
const bool g_x3p_sb1 = [] {
  const char* e = getenv("MPR_X3P_SB");
  return !(e && e[0] == '2');
}();

const bool g_x3p_k32 = [] {
  const char* e = getenv("MPR_X3P_K32");
  return e && e[0] == '1';
}();

const bool g_x3p_longk_sb = [] {
  const char* e = getenv("MPR_X3P_LONGK_SB");
  return !(e && e[0] == '0');
}();

int gemm_launch(const GemmGroup& g, int kind, hipStream_t s) {
  double flops = 0, bytes = 0;
  for (int i = 0; i < g.n; ++i) {
    flops += 2.0 * g.g[i].M * g.g[i].N * g.g[i].K * g.g[i].batch;
    bytes += gemm_bytes(g.g[i]) * g.g[i].batch;
  }
  if (g_probe_kind == PROBE_RECORD) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &st) == hipSuccess && st == hipStreamCaptureStatusNone)
      g_recorded.push_back(g);
  }
  // F32_SMALL: 32x32 blocks, or 64x32 blocks (two 32x32 tiles sharing each W slice, 8 waves)
  // once the launch has >= 2048 32x32 blocks; every 32x32 sub-tile is summed by the same 4
  // K-slice waves in the same order in both (bit-identical: the round-1 gbench lab, git show a67dcca:tools/gbench.hip).
  int64_t blocks32 = 0;
  for (int i = 0; i < g.n; ++i) blocks32 += cdiv(g.g[i].M, 32) * cdiv(g.g[i].N, 32);
  return probed(PROBE_GEMM, flops, bytes, s, [&]() {
    switch (kind) {
      case F32_BIG: return launch_gemm_group<64, 64, 1, 1, 32, 2, 1, true>(g, s);
      case F32_SMALL:
        if (blocks32 >= 2048)
          return launch_gemm_group<64, 32, 1, 1, 64, 2, 4>(g, s);
        return launch_gemm_group<32, 32, 1, 1, 64, 2, 4>(g, s);
      case X3_WIDE: return launch_gemm_x3_group<128, 128, 2, 1, 16, 2, 1, 2>(g, s);
      case X3_WIDE32: return launch_gemm_x3_group<128, 128, 2, 1, 32, 2, 1, 2>(g, s);
      case X3_SMALL: return launch_gemm_x3_group<64, 64, 1, 1, 16, 2, 1>(g, s);
      case X3_WIDE_SB2: return launch_gemm_x3_group<128, 128, 2, 1, 16, 2, 1, 2, 2>(g, s);
      case X3_SMALL_SB2: return launch_gemm_x3_group<64, 64, 1, 1, 16, 2, 1, 0, 2>(g, s);
      // two A stages and a barrier every K tile (36.9 KB of LDS); MPR_X3P_SB=2: four stages, a
      // barrier every second tile (73.7 KB).  Replayed alone the four-stage form is ~1 % faster
      // (0.882 vs 0.874 of fp32 peak), but in the serving loop the two-stage blocks leave LDS for
      // the decode chain's blocks beside them: 4,156-4,195 vs 4,066-4,153 QA pairs/s over 5 / 4
      // alternating runs, in-loop GEMM frac 0.68 vs 0.66 (round 6, profiles/r06_loop_interference.txt)
      // Long-K launches of one round of blocks (<= 256: the ViT fc2 groups, 184) take the four
      // stages anyway: fc2 1600x768x3072 x2 107.7 -> 100.7 us (x3pbench, round 6); the K = 768
      // qkv / fc1 and the 368-block grouped T5 FFN-out are faster on two stages
      // (profiles/r06_x3p_small_ab.txt).  MPR_X3P_LONGK_SB=0: two stages there too.
      case X3P_WIDE: {
        int64_t b128 = 0;
        int max_k = 0;
        for (int i = 0; i < g.n; ++i) {
          b128 += cdiv(g.g[i].M, 128) * cdiv(g.g[i].N, 128);
          max_k = std::max(max_k, g.g[i].K);
        }
        const bool four = !g_x3p_sb1 || (g_x3p_longk_sb && max_k >= 2048 && b128 <= 256);
        return four ? launch_gemm_x3p_group<128, 128, 2, 1, 2, 16, 2>(g, s)
                    : launch_gemm_x3p_group<128, 128, 2, 1, 2>(g, s);
      }
      case X3P_SMALL: return launch_gemm_x3p_group<64, 64, 1, 1, 2>(g, s);
      // K >= 2048 on 64x64 blocks: 16-deep K tiles in four A stages, a barrier every second
      // tile (36.9 KB of LDS), not the 32-deep tiles of rounds 4-5: T5 wo 1536x512x2048 42.8 ->
      // 33.8 us, ViT fc2 1600x768x3072 x2 137.6 -> 113.4, 800 rows 68.5 -> 68.3 (x3pbench, round
      // 6, profiles/r06_x3p_small_ab.txt); same k order, bit-identical.  MPR_X3P_K32=1: 32-deep.
      case X3P_SMALL3:
        return g_x3p_k32 ? launch_gemm_x3p_group<64, 64, 1, 1, 2, 32>(g, s)
                         : launch_gemm_x3p_group<64, 64, 1, 1, 2, 16, 2>(g, s);
      default: return launch_gemm_x3_group<64, 128, 1, 1, 32, 2, 1>(g, s);
    }
  });
}
}  // namespace

bool gemm_uniform_order() { return !g_gemm_f32; }

int gemm_group(const GemmGroup& g, hipStream_t s) {
  MPR_REQUIRE(g.n >= 1 && g.n <= GEMM_GROUP, "gemm_group: %d problems", g.n);
  for (int i = 0; i < g.n; ++i) {
    const GemmArgs& a = g.g[i];
    MPR_REQUIRE(a.M >= 0 && a.N >= 0 && a.K > 0, "gemm: bad shape M=%d N=%d K=%d", a.M, a.N,
                a.K);
    MPR_REQUIRE(a.K % 4 == 0 && a.lda % 4 == 0 && a.ldw % 4 == 0 && aligned16(a.A) &&
                    aligned16(a.W),
                "gemm: K/lda/ldw must be multiples of 4 and A/W 16-byte aligned (K=%d)", a.K);
    MPR_REQUIRE(a.batch >= 1 && (a.batch == 1 || (!a.R && !a.c_rpb && a.a_bs % 4 == 0 &&
                                                   a.w_bs % 4 == 0)),
                "gemm: batch %d needs no residual / row batching and 16-byte batch strides",
                a.batch);
  }
  if (g_gemm_f32) {
    for (int i = 0; i < g.n; ++i)
      MPR_REQUIRE(g.g[i].batch == 1, "gemm: strided batches need the split-bf16 kernels");
    // Round-1 f32 MFMA tiles, per problem (round-1 gbench lab, a67dcca): 64x64 tiles (4 waves of 32x32,
    // BK 32) once the problem has >= 1.5 blocks per CU, else 32x32 tiles with the K tile split
    // over 4 waves.  A problem keeps its tile alone or grouped (bit-identical results).
    GemmGroup big, small;
    big.n = small.n = 0;
    for (int i = 0; i < g.n; ++i) {
      const GemmArgs& a = g.g[i];
      if (a.M == 0 || a.N == 0) continue;
      const int tm = a.tile_m > 0 ? a.tile_m : a.M;
      GemmGroup& dst = cdiv(tm, 64) * cdiv(a.N, 64) >= 384 ? big : small;
      dst.g[dst.n++] = a;
    }
    if (big.n) MPR_TRY(gemm_launch(big, F32_BIG, s));
    if (small.n) MPR_TRY(gemm_launch(small, F32_SMALL, s));
    return MPR_OK;
  }
  // Split-bf16 tiles (x3bench lab, 28e8ac6: the tower launches of two batches, each ViT problem plus
  // the text tower's problem of the same layer in one launch).  Every problem of a launch shares
  // one KW = 1 tile, so the choice may follow the launch: 128x128 blocks of 8 waves (2x1 32x32
  // accumulators each) once the launch has >= 160 of them — even below one block per CU they beat
  // smaller tiles (ViT out 1600x768x768 x2 + text: 41.3 us against 50.6 for 64x64 blocks and 60.6
  // for the f32 kernel; qkv 106 vs 158, fc1 140 vs 196, fc2 137 vs 178) — else 64x128 blocks of 8
  // waves of 32x32 (one-batch fc2 800x768x3072 x2 + text: 93.7 vs 114 us f32).
  // Below that, 64x64 blocks (4 waves) when the 64x128 grid would leave half the CUs idle or
  // every K is short (x3small_bench lab, git show 770f90b:tools/x3small_bench.hip, one-batch T5 encoder at M = 1440: qkv 37.2 ->
  // 25.8 us, o 18.0 -> 14.6, wo 52.1 -> 43.5; the one-batch ViT out / fc2, K >= 768 with 156+
  // 64x128 blocks, stay on 64x128).  Same k order in every tile: bit-identical results.
  GemmGroup fam;
  fam.n = 0;
  int64_t b128 = 0, b64x128 = 0;
  bool short_k = true, packed = true;
  int max_n = 0, max_k = 0;
  for (int i = 0; i < g.n; ++i) {
    const GemmArgs& a = g.g[i];
    if (a.M == 0 || a.N == 0) continue;
    fam.g[fam.n++] = a;
    b128 += cdiv(a.M, 128) * cdiv(a.N, 128) * a.batch;
    b64x128 += cdiv(a.M, 64) * cdiv(a.N, 128) * a.batch;
    short_k = short_k && a.K <= 512;
    packed = packed && a.wp && a.batch == 1;
    max_n = std::max(max_n, a.N);
    max_k = std::max(max_k, a.K);
  }
  // Every W of the launch packed (fixed model weights): W fragments straight from the packed
  // image (tools/x3pbench.hip over the tower / T5-encoder shapes, bit-identical to the kernels
  // below): 128x128 blocks of 8 waves for launches of > 160 of them with a wide N or a long K
  // (ViT qkv 1600x2304x768 x2: 80.9 -> 73.5 us, fc1 110.7 -> 102.1, qkv at 800 rows 46.0 ->
  // 41.4, fc2 1600x768x3072 x2 127.7 -> 116.2), else 64x64 blocks of 4 waves (ViT out
  // 1600x768x768 x2: 38.7 -> 33.6, T5 qkv 1536x1536x512 27.6 -> 24.3), at K >= 2048 four A
  // stages (round 6; rounds 4-5 took 32-deep K tiles there: T5 wo 1536x512x2048 44.2 -> 36.4,
  // ViT fc2 at 800 rows 76.5 -> 70.7 against the two-stage 16-deep tile; 32-deep tiles on the
  // 128x128 blocks measured 5-15 % slower, profiles/r04_x3p_k32_ab.txt).  (The 64x64 tiles on the ViT fc2,
  // 113.0 us alone, fetched 314 MB per launch from beyond L2 against ~120 MB for 128x128 tiles:
  // r04_v2 PMC.)
  if (getenv("MPR_GEMM_LOG")) {  // debug: each distinct launch shape once, to stderr
    static std::mutex mu;
    static std::set<std::string> seen;
    std::string key = packed ? "x3p" : "x3";
    for (int i = 0; i < fam.n; ++i)
      key += " " + std::to_string(fam.g[i].M) + "x" + std::to_string(fam.g[i].N) + "x" +
             std::to_string(fam.g[i].K) + (fam.g[i].batch > 1 ? "b" + std::to_string(fam.g[i].batch) : "");
    std::lock_guard<std::mutex> lk(mu);
    if (seen.insert(key).second)
      fprintf(stderr, "[gemm] %s  blocks of 128x128: %lld\n", key.c_str(), (long long)b128);
  }
  // (128x256 blocks of 8 waves of 4x1 accumulators — W fragments loaded once per block, half
  // the vector-memory bytes per MFMA of the 128x128 2x1 tile — ran the ViT qkv 1600x2304x768 x2
  // in 65.4 against 74.0 us (tools/x3pbench.hip), but 186 VGPRs hold one block per CU and no
  // serving-loop launch has 192-256 of them (the loop's qkv groups two ViT and two text problems:
  // 276).  As a rule on 192-256 such blocks it took only predict()'s 800-row fc1 groups (192-200
  // blocks), with no gain: 4057-4074 vs 4060-4092 QA pairs/s, sync 9.70-9.83 vs 9.65-9.76 ms,
  // profiles/r06_gemm_tiles.txt.)
  if (fam.n && packed)
    return gemm_launch(fam, b128 > 160 && (max_n >= 2048 || max_k >= 2048) ? X3P_WIDE
                            : max_k >= 2048                                 ? X3P_SMALL3
                                                                            : X3P_SMALL,
                       s);
  // A launch of <= 256 128x128 blocks (at most one per CU) takes 32-deep K tiles: 123 KB of LDS,
  // half the barriers per K, same k order (bit-identical).  Replayed alone equal (0.79-0.80 of
  // 157.3 either way); in the serving loop the GEMMs run 0.64 -> 0.68 (a CU holding one leaves no
  // LDS for decode blocks) and the loop 4157-4165 -> 4212-4309 QA pairs/s at 40 steps.  Every
  // 128x128 launch on 32-deep tiles halves the blocks per CU of the > 256-block launches
  // (4073-4127, r02); 16-deep only is slower in the loop.
  // K >= 1536 (the trainer's FFN-out and weight-gradient GEMMs): the 16-deep tiles take four
  // stages and one barrier per two K tiles (x3pbench, profiles/r05_x3_sb2.txt: T5 wo 1536x512x2048
  // 43.9 -> 40.4 us on 64x64, weight gradients 2048x512x1600 37.9 -> 35.1; shorter K loses, so
  // it stays on one barrier per tile).  Bit-identical either way.
  const bool sb2 = max_k >= 1536 && !g_x3_sb1;
  if (fam.n) {
    int kind = b128 >= 160 && b128 <= 256      ? X3_WIDE32
               : b128 >= 160                   ? X3_WIDE
               : (b64x128 < 128 || short_k)    ? X3_SMALL
                                               : X3_TALL;
    if (sb2 && kind == X3_WIDE) kind = X3_WIDE_SB2;
    if (sb2 && kind == X3_SMALL) kind = X3_SMALL_SB2;
    MPR_TRY(gemm_launch(fam, kind, s));
  }
  return MPR_OK;
}

int gemm(const GemmArgs& a, hipStream_t s) {
  if (a.M == 0 || a.N == 0) {
    MPR_REQUIRE(a.M >= 0 && a.N >= 0 && a.K > 0, "gemm: bad shape M=%d N=%d K=%d", a.M, a.N,
                a.K);
    return MPR_OK;
  }
  GemmGroup g;
  g.g[0] = a;
  g.n = 1;
  return gemm_group(g, s);
}

int64_t packed_x3_bytes(int64_t N, int64_t K) { return cdiv(N, 32) * cdiv(K, 16) * 3 * 64 * 16; }

int pack_x3(const float* W, int64_t N, int64_t K, int64_t ldw, void* out, hipStream_t s) {
  MPR_REQUIRE(N > 0 && K > 0 && ldw >= K && N < (1 << 30) && K < (1 << 30) && aligned16(out),
              "pack_x3: bad shape N=%lld K=%lld", (long long)N, (long long)K);
  const int64_t q = cdiv(N, 32) * cdiv(K, 16) * 64;
  hipLaunchKernelGGL(pack_x3_kernel, dim3((unsigned)cdiv(q, 256)), dim3(256), 0, s, W, (int)N,
                     (int)K, ldw, (int)cdiv(K, 16), reinterpret_cast<bf16x8*>(out));
  MPR_LAUNCHED();
  return MPR_OK;
}

int64_t packed_rows16_elems(int64_t N, int64_t K) { return cdiv(N, 16) * cdiv(K, 16) * 256; }

int pack_rows16(const float* W, int64_t N, int64_t K, int64_t ldw, float* out, hipStream_t s) {
  MPR_REQUIRE(N > 0 && K > 0 && ldw >= K, "pack_rows16: bad shape N=%lld K=%lld",
              (long long)N, (long long)K);
  const int64_t q = packed_rows16_elems(N, K) / 4;
  hipLaunchKernelGGL(pack_rows16_kernel, dim3((unsigned)cdiv(q, 256)), dim3(256), 0, s, W, N, K,
                     ldw, cdiv(K, 16), out);
  MPR_LAUNCHED();
  return MPR_OK;
}

template <int MAXC, int NT, bool LOOP, int MR = 1, int W = 8>
void launch_skinny(const SkinnyArgs& sa, int F, unsigned grid, hipStream_t s, unsigned gy = 1) {
#define MPR_SK(f)                                                                          \
  case f:                                                                                  \
    hipLaunchKernelGGL((gemm_skinny_kernel<MAXC, NT, f, LOOP, MR, W>), dim3(grid, gy),    \
                       dim3(64 * W), 0, s, sa);                                            \
    break;
  if constexpr (NT > 1) {
    switch (F) { MPR_SK(SKF_AMAX) MPR_SK(SKF_AMAX | SKF_RMS) default: break; }
  } else {
    switch (F) {
      MPR_SK(0) MPR_SK(1) MPR_SK(2) MPR_SK(3) MPR_SK(4) MPR_SK(5) MPR_SK(6) MPR_SK(7)
      MPR_SK(SKF_AMAX) MPR_SK(SKF_AMAX | SKF_RMS)
      MPR_SK(SKF_RELU_IN | SKF_RSCALE | SKF_RES) MPR_SK(SKF_SSQ)
      default: break;
    }
  }
#undef MPR_SK
}

// (Measured and dropped: capping encoder GEMM blocks at 2-3 per CU by LDS padding and running
// the K = 2048 GEMV in 43.5 KB passes, so a decode block always fits beside resident encoder
// blocks, made the two-decodes-in-flight serving loop 1-6% slower.)
// (Measured and dropped, round 6: the grouped-decode GEMVs in 2-chunk passes — 37 KB of LDS
// slabs instead of 70 KB, so a decode block sits beside more tower blocks — 3,899-4,163 vs
// 4,165-4,173 QA pairs/s, profiles/r06_loop_interference.txt.)
int gemm_skinny(const SkinnyArgs& sa, hipStream_t s) {
  const GemmArgs& a = sa.g;
  MPR_REQUIRE(a.M >= 0 && a.M <= 256 && a.N >= 0 && a.K > 0, "gemm_skinny: bad shape M=%d", a.M);
  if (a.M == 0 || a.N == 0) return MPR_OK;
  MPR_REQUIRE(sa.wpk && aligned16(sa.wpk), "gemm_skinny: needs the 16-byte aligned packed weight");
  MPR_REQUIRE(a.K % 4 == 0 && a.lda % 4 == 0 && aligned16(a.A) &&
                  (!sa.rms_w || aligned16(sa.rms_w)),
              "gemm_skinny: K/lda must be multiples of 4, operands 16-byte aligned");
  MPR_REQUIRE(!a.bias && (a.act == ACT_NONE || a.act == ACT_RELU),
              "gemm_skinny: no bias, activation none or relu (the T5 decoder's projections)");
  const bool amax = sa.amax_val != nullptr;
  MPR_REQUIRE(!amax || (sa.amax_idx && !a.R && !a.C && a.act == ACT_NONE),
              "gemm_skinny: argmax mode takes plain logits and stores no C");
  MPR_REQUIRE(amax || (a.C && a.N % 16 == 0 && a.ldc % 4 == 0 && aligned16(a.C) &&
                       (!a.R || (a.ldr % 4 == 0 && aligned16(a.R)))),
              "gemm_skinny: N must be a multiple of 16, C/R rows 16-byte aligned");
  MPR_REQUIRE(!sa.rs_part || (!sa.rms_w && !amax && sa.rs_n > 0 && sa.rs_nparts > 0 &&
                               sa.rs_nparts <= 64),
              "gemm_skinny: an external row scale excludes the fused RMSNorm / argmax; at most "
              "64 partials per row");
  MPR_REQUIRE(!sa.ssq_out || (sa.ssq_cols % 16 == 0 && sa.ssq_cols <= a.N),
              "gemm_skinny: ssq columns %d", sa.ssq_cols);
  const int F = (sa.rms_w ? SKF_RMS : 0) | (a.R ? SKF_RES : 0) |
                (a.act == ACT_RELU ? SKF_RELU : 0) | (amax ? SKF_AMAX : 0) |
                (sa.relu_in ? SKF_RELU_IN : 0) | (sa.rs_part ? SKF_RSCALE : 0) |
                (sa.ssq_out ? SKF_SSQ : 0);
  MPR_REQUIRE(!(F & (SKF_RELU_IN | SKF_RSCALE)) || F == (SKF_RELU_IN | SKF_RSCALE | SKF_RES),
              "gemm_skinny: relu_in / row scale only as the folded FFN-out (relu_in + scale + "
              "residual)");
  MPR_REQUIRE(!(F & SKF_SSQ) || F == SKF_SSQ, "gemm_skinny: ssq only on a plain projection");
  const int per = (int)cdiv(cdiv(a.K, 16), SK_WAVES);  // 16-column chunks per wave
  const int64_t tiles = cdiv(a.N, 16);
  // (16 waves splitting a long K — t5-small's K = 2048 FFN-out — chosen by K alone so every row
  // count sums alike: 218.5 -> 215.8 us per 16-row step but 433.9 -> 437.1 per 128-row step,
  // round 6, tools/decode_ab.py; not kept: the serving loop decodes 128-row groups.)
  if (debug_lds_poison() && !sa.poison) {
    SkinnyArgs p = sa;
    p.poison = 1;
    return gemm_skinny(p, s);
  }
  // Above 32 rows (grouped decodes on the skinny path: MPR_DECODE_GEMM=skinny) the rows split
  // over blocks of 32 (serving loop, 20 steps: 3783-3831 with one block column of up to 8 row
  // groups -> 3893-3908 QA pairs/s; 16-row blocks within 1 %).
  return probed(PROBE_SKINNY, 2.0 * a.M * a.N * a.K, gemm_bytes(a), s, [&]() {
    // (A K split of the K = 2048 GEMV over 4 blocks per tile, partials published with an
    // agent-scope fence and added by the last block, made a 16-row generate 5.49 -> 5.89 ms and
    // the serving loop 3050 -> 2830 QA pairs/s: the cross-XCD publish costs more than the
    // 32-block launch loses.)
    if (a.M > 32) {  // rows split over blocks of 32 rows (grouped decodes)
      const unsigned gy = (unsigned)cdiv(a.M, 32);
      // (Four 16-column tiles per block sharing each staged 32-row slab — the slab is staged
      // once per 16 columns — measured slower: C5's t5-base 128-row decodes 84.0 -> 96.3 ms
      // per batch, the serving loop 3.77-3.79 -> 3.86-3.88 ms per step.  Two tiles per 64-row
      // block above 128 rows, halving the rows' L2 reads: 146-164 VGPRs, one block per CU, C5
      // end to end 46.3-46.7 -> 50.5 ms per batch, round 5.)
      // 4-chunk passes above 4 chunks per wave, so the block's slabs take 70 KB of LDS instead
      // of 136 KB and two blocks fit per CU (the 8-chunk slab holds one: t5-base's 576-block
      // 128-row qkv ran in ~3 rounds of blocks).  Same chunk order per accumulator chain,
      // padding chunks add exact zeros: bit-identical.  C5 end to end 72.1-73.1 -> 68.4-69.3
      // ms per batch, the serving loop unchanged (3.69-3.71 ms per step either way).
      // Above 128 rows of a model with d >= 768 (C5's 256-row t5-base loop) the rows go in
      // blocks of 64 (MR = 4, 2-chunk passes: 74 KB of slabs), halving the weight re-reads per
      // step: t5-base 256 rows 1621 -> 1430 us per step, 192 rows 1490 -> 1331; at 128 rows
      // (1055 -> 1200) and for t5-small (256 rows 514 -> 586) the 32-row blocks stay; 128-row
      // blocks ran 2206 at 256, 48-row blocks 1712 vs 1479 (git show f10742c:tools/decode_rows.py,
      // profiles/r04_skinny_rows_ab.txt).  Rows
      // are independent and every chain keeps its chunk order: bit-identical.
      if (!amax && a.M > 128 && std::min(a.N, a.K) >= 768) {
        const unsigned g = (unsigned)cdiv(a.M, 64);
        if (per <= 2) launch_skinny<2, 1, false, 4>(sa, F, (unsigned)tiles, s, g);
        else launch_skinny<2, 1, true, 4>(sa, F, (unsigned)tiles, s, g);
      } else if (amax && tiles >= 1024 && per <= 4)  // (64-row blocks for the head, half its
        // weight re-reads: 429 -> 438 / 450 us per 128-row step, 2- / 4-chunk passes; round 6)
        launch_skinny<4, 2, false, 2>(sa, F, (unsigned)cdiv(tiles, 2), s, gy);
      else if (per <= 4)
        launch_skinny<4, 1, false, 2>(sa, F, (unsigned)tiles, s, gy);
      else
        launch_skinny<4, 1, true, 2>(sa, F, (unsigned)tiles, s, gy);
    } else if (a.M > 16) {  // two row groups per weight load (2 batches of <= 16 rows)
      if (amax && tiles >= 1024 && per <= 4)
        launch_skinny<4, 2, false, 2>(sa, F, (unsigned)cdiv(tiles, 2), s);
      else if (per <= 4)
        launch_skinny<4, 1, false, 2>(sa, F, (unsigned)tiles, s);
      else if (per <= 8)
        launch_skinny<8, 1, false, 2>(sa, F, (unsigned)tiles, s);
      else  // a 16-chunk slab for 32 rows would not fit the 160 KiB LDS
        launch_skinny<8, 1, true, 2>(sa, F, (unsigned)tiles, s);
    } else if (amax && tiles >= 1024 && per <= 4)  // lm_head: 2 tiles per block (NT 1/2/4/8
      launch_skinny<4, 2, false>(sa, F, (unsigned)cdiv(tiles, 2), s);  // 14.5/13.1/13.8/14.5 us)
    else if (per <= 4)
      launch_skinny<4, 1, false>(sa, F, (unsigned)tiles, s);
    else if (per <= 8)
      launch_skinny<8, 1, false>(sa, F, (unsigned)tiles, s);
    else if (per <= 16)
      launch_skinny<16, 1, false>(sa, F, (unsigned)tiles, s);
    else
      launch_skinny<16, 1, true>(sa, F, (unsigned)tiles, s);
    MPR_LAUNCHED();
    return MPR_OK;
  });
}

}  // namespace mpr
