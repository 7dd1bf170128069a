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
// gemm_skinny() serves decoder steps (M = batch <= 16): W streams straight from HBM/L2 into
// registers as the A operand of v_mfma_f32_16x16x4_f32 (16 output columns per block), the 16
// activation rows are the B operand, K is split across the 8 waves of a block and reduced through
// LDS, and T5's RMSNorm of the activation rows is folded into the operand and the epilogue.
#include "kernels.h"

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

template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(64 * (BM / (32 * WM)) * (BN / (32 * WN))) void gemm_f32_kernel(
    GemmArgs a) {
  constexpr int WAVES_N = BN / (32 * WN);
  constexpr int NT = 64 * (BM / (32 * WM)) * WAVES_N;
  constexpr int BK = 32, LDK = BK + 4, KQ = BK / 4;  // KQ float4 per row of a K tile
  constexpr int LA = BM * KQ / NT, LB = BN * KQ / NT;
  constexpr int STAGE = (BM + BN) * LDK;  // floats per LDS stage (A rows then W rows)
  static_assert(LA * NT == BM * KQ && LB * NT == BN * KQ, "loader split");

  // Three LDS stages: tile kt+1 is already visible while tile kt is multiplied, so its fragments
  // are read into registers under tile kt's MFMAs and the next k-step starts on the barrier
  // without waiting for LDS.  ONE __shared__ object holds the stages: a second LDS object
  // makes hipcc drain vmcnt before every k-step's first ds_read.
  __shared__ __attribute__((aligned(16))) float smem[3 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR)
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int M = a.M, N = a.N, K = a.K;

  f32x4 ra[LA], rb[LB];
  bool oka[LA], okb[LB];
  // Unconditional loads from clamped addresses, zeroed by a select only when written to LDS
  // (after the MFMAs of the current tile): an exec-masked load makes hipcc branch around every
  // load, and an early select makes it wait for the data right after issuing the load.
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int idx = tid + i * NT, r = idx / KQ, c = k0 + (idx % KQ) * 4, row = m0 + r;
      oka[i] = row < M && c < K;
      ra[i] = *reinterpret_cast<const f32x4*>(a.A + (int64_t)min(row, M - 1) * a.lda +
                                              min(c, K - 4));
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int idx = tid + i * NT, r = idx / KQ, c = k0 + (idx % KQ) * 4, row = n0 + r;
      okb[i] = row < N && c < K;
      rb[i] = *reinterpret_cast<const f32x4*>(a.W + (int64_t)min(row, N - 1) * a.ldw +
                                              min(c, K - 4));
    }
  };
  auto swrite = [&](int st) {
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
    float* base = smem + st * STAGE;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int idx = tid + i * NT;
      *reinterpret_cast<f32x4*>(base + (idx / KQ) * LDK + (idx % KQ) * 4) = oka[i] ? ra[i] : z;
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int idx = tid + i * NT;
      *reinterpret_cast<f32x4*>(base + (BM + idx / KQ) * LDK + (idx % KQ) * 4) =
          okb[i] ? rb[i] : z;
    }
  };

  f32x16 acc[WM][WN];
#pragma unroll
  for (int mi = 0; mi < WM; ++mi)
#pragma unroll
    for (int ni = 0; ni < WN; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;

  // Operand fragments of one K tile: lane (li, lh) holds row li's k = 16*lh .. 16*lh+15 as four
  // float4 (the contraction order inside the tile is permuted identically for A and W).
  const int li = lane & 31, lh = lane >> 5;
  f32x4 fa[WM][4], fb[WN][4], na[WM][4], nb[WN][4];
  auto sread = [&](int st, f32x4(&xa)[WM][4], f32x4(&xb)[WN][4]) {
    const float* base = smem + st * STAGE;
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
#pragma unroll
      for (int mi = 0; mi < WM; ++mi)
        xa[mi][s4] = *reinterpret_cast<const f32x4*>(
            base + (wm * 32 * WM + mi * 32 + li) * LDK + lh * 16 + s4 * 4);
#pragma unroll
      for (int ni = 0; ni < WN; ++ni)
        xb[ni][s4] = *reinterpret_cast<const f32x4*>(
            base + (BM + wn * 32 * WN + ni * 32 + li) * LDK + lh * 16 + s4 * 4);
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
    for (int s4 = 0; s4 < 4; ++s4) {
#pragma unroll
      for (int mi = 0; mi < WM; ++mi) fa[mi][s4] = na[mi][s4];
#pragma unroll
      for (int ni = 0; ni < WN; ++ni) fb[ni][s4] = nb[ni][s4];
    }
  };

  const int nk = (K + BK - 1) / BK;

  gload(0);
  swrite(0);
  gload(BK);  // clamped/zeroed when past K
  swrite(1);
  __syncthreads();
  sread(0, fa, fb);
  int kt = 0, st = 0;
  // Steady state, branch-free (the accumulators stay in AGPRs): global loads of tile kt+2 in
  // flight across tile kt's MFMAs, LDS reads of tile kt+1 issued after its first quarter.
  for (; kt + 2 < nk; ++kt) {
    const int st1 = st == 2 ? 0 : st + 1, st2 = st1 == 2 ? 0 : st1 + 1;
    gload((kt + 2) * BK);
    __builtin_amdgcn_sched_barrier(0);
    mfmas(0, 1);
    __builtin_amdgcn_sched_barrier(0);
    sread(st1, na, nb);
    __builtin_amdgcn_sched_barrier(0);
    mfmas(1, 4);
    __builtin_amdgcn_sched_barrier(0);
    swrite(st2);
    __syncthreads();
    advance();
    st = st1;
  }
  if (kt + 1 < nk) {  // second-to-last tile: its successor is already in LDS
    mfmas(0, 1);
    sread(st == 2 ? 0 : st + 1, na, nb);
    mfmas(1, 4);
    advance();
    ++kt;
  }
  if (kt < nk) mfmas(0, 4);

  // Epilogue: 32x32 accumulator, col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5).
#pragma unroll
  for (int mi = 0; mi < WM; ++mi)
#pragma unroll
    for (int ni = 0; ni < WN; ++ni) {
      const int col = n0 + wn * 32 * WN + ni * 32 + li;
      if (col >= N) continue;
      const float bv = a.bias ? a.bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 32 * WM + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (row >= M) continue;
        float v = act_exact(acc[mi][ni][r] + bv, a.act);
        if (a.R) v = a.R[(int64_t)row * a.ldr + col] + v;
        const int64_t coff = a.c_rpb ? (int64_t)(row / a.c_rpb) * a.c_bs +
                                           (int64_t)(row % a.c_rpb) * a.ldc
                                     : (int64_t)row * a.ldc;
        a.C[coff + col] = v;
      }
    }
}

template <int BM, int BN, int WM, int WN>
int launch_gemm(const GemmArgs& a, hipStream_t s) {
  constexpr int NT = 64 * (BM / (32 * WM)) * (BN / (32 * WN));
  dim3 grid((unsigned)cdiv(a.N, BN), (unsigned)cdiv(a.M, BM));
  hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WM, WN>), grid, dim3(NT), 0, s, a);
  MPR_LAUNCHED();
  return MPR_OK;
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
enum : int { SKF_RMS = 1, SKF_RES = 2, SKF_RELU = 4, SKF_AMAX = 8 };

// NT 16-column tiles per block share the activation slab (NT > 1 for the 32k-column lm_head,
// which needs more bytes in flight per wave); two accumulator chains per tile halve the
// dependent-MFMA latency.  MAXC = chunks of 16 columns staged per pass; LOOP = more than one
// pass (K > 16 * 8 * MAXC).
template <int MAXC, int NT, int F, bool LOOP>
__global__ __launch_bounds__(512) void gemm_skinny_kernel(SkinnyArgs sa) {
  constexpr bool RMS = (F & SKF_RMS) != 0, RES = (F & SKF_RES) != 0,
                 RELU = (F & SKF_RELU) != 0, AMAX = (F & SKF_AMAX) != 0;
  const GemmArgs& a = sa.g;
  constexpr int XLD = MAXC * 16 + 4;  // slab row stride (floats): conflict-free fragment reads
  constexpr int XS = SK_WAVES * 16 * XLD, RED = NT * SK_WAVES * 256;
  // one LDS object: activation slabs | partial tiles | per-wave sums of squares
  __shared__ __attribute__((aligned(16))) float smem[XS + RED + SK_WAVES * 16];
  float(*xs)[16][XLD] = reinterpret_cast<float(*)[16][XLD]>(smem);
  f32x4(*red)[SK_WAVES][64] = reinterpret_cast<f32x4(*)[SK_WAVES][64]>(smem + XS);
  float(*ssq_s)[16] = reinterpret_cast<float(*)[16]>(smem + XS + RED);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR)
  const int M = a.M, N = a.N, K = a.K;
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
  // The lane's 4 outputs are row i, columns n0 + 4h .. +3 (16x16 D layout): its residual is
  // one float4, fetched before the main loads.
  f32x4 rres = {0.f, 0.f, 0.f, 0.f};
  if constexpr (RES) {
    if (wave < NT)
      rres = *reinterpret_cast<const f32x4*>(a.R + (int64_t)min(i, M - 1) * a.ldr +
                                             (blockIdx.x * NT + wave) * 16 + h * 4);
  }
  f32x4 acc[NT][2];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t][0] = acc[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ss = 0.f;
#pragma unroll 1
  for (int c0 = c_lo; LOOP ? c0 < c_hi : c0 == c_lo; c0 += MAXC) {
    // weights first (the long pole), then this pass's activation rows as 256-byte segments:
    // float4 q of the pass = row q / (4*MAXC), column (q % (4*MAXC)) * 4 of the pass
    f32x4 wv[NT][MAXC], xr[MAXC], gv[MAXC];
#pragma unroll
    for (int u = 0; u < MAXC; ++u) {
      // a chunk past the wave's slice re-reads an in-range chunk; its activations are zero
      const int c = c0 + u, cc = c < c_hi ? c : c_safe;
#pragma unroll
      for (int t = 0; t < NT; ++t) wv[t][u] = wp[t][(int64_t)cc * 64];
      if constexpr (RMS) gv[u] = *reinterpret_cast<const f32x4*>(sa.rms_w + cc * 16 + h * 4);
    }
#pragma unroll
    for (int u = 0; u < MAXC; ++u) {
      const int q = u * 64 + lane, row = q / (4 * MAXC), col = c0 * 16 + (q % (4 * MAXC)) * 4;
      const bool ok = row < M && col < c_hi * 16 && col < K;
      xr[u] = *reinterpret_cast<const f32x4*>(a.A + (int64_t)min(row, M - 1) * a.lda +
                                              min(col, K - 4));
      if (!ok) xr[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    // every load of the pass is in flight before the first wait (hipcc otherwise sinks the
    // weight loads next to their MFMAs, behind the activation round trip through LDS)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < MAXC; ++u) {
      const int q = u * 64 + lane;
      *reinterpret_cast<f32x4*>(&xs[wave][q / (4 * MAXC)][(q % (4 * MAXC)) * 4]) = xr[u];
    }
#pragma unroll
    for (int u = 0; u < MAXC; ++u) {
      f32x4 xv = *reinterpret_cast<const f32x4*>(&xs[wave][i][u * 16 + h * 4]);
      if constexpr (RMS) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          ss += xv[e] * xv[e];
          xv[e] = gv[u][e] * xv[e];
        }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int t = 0; t < NT; ++t)
          acc[t][u & 1] =
              __builtin_amdgcn_mfma_f32_16x16x4f32(wv[t][u][e], xv[e], acc[t][u & 1], 0, 0, 0);
    }
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) red[t][wave][lane] = acc[t][0] + acc[t][1];
  if constexpr (RMS) {
    ss += __shfl_xor(ss, 16, 64);
    ss += __shfl_xor(ss, 32, 64);
    if (lane < 16) ssq_s[wave][lane] = ss;
  }
  __syncthreads();
  if (wave >= NT) return;
  const int tile = blockIdx.x * NT + wave;
  const int n0 = tile * 16;
  f32x4 sum = red[wave][0][lane];
#pragma unroll
  for (int w = 1; w < SK_WAVES; ++w) sum += red[wave][w][lane];
  // D[row = W row (n), col = A row (m)]: col = lane&15, row = (lane>>4)*4 + r.
  float scale = sa.a_scale;
  if constexpr (RMS) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < SK_WAVES; ++w) t += ssq_s[w][i];
    scale = (1.0f / sqrtf(t / (float)K + sa.rms_eps)) * sa.a_scale;
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
    if (lane < 16 && n0 < N) {  // row-major [16][ntiles]: greedy_step reads rows coalesced
      sa.amax_val[(int64_t)i * ntiles + tile] = bv;
      sa.amax_idx[(int64_t)i * ntiles + tile] = bi;
    }
  } else {
    f32x4 v = sum * scale;
    if constexpr (RELU) {
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : 0.f;
    }
    if constexpr (RES) v = rres + v;
    if (i < M) *reinterpret_cast<f32x4*>(a.C + (int64_t)i * a.ldc + n0 + h * 4) = v;
  }
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

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

template <class F>
int probed(int kind, const GemmArgs& a, hipStream_t s, F&& launch) {
  if (!probing(kind, s)) return launch();
  ProbeRec r{pool_event(), pool_event(), 2.0 * a.M * a.N * a.K, gemm_bytes(a)};
  if (!r.a || !r.b) return launch();
  (void)hipEventRecord(r.a, s);
  const int rc = launch();
  (void)hipEventRecord(r.b, s);
  g_recs.push_back(r);
  return rc;
}

}  // namespace

int probe_enable(int kind) {
  g_probe_kind = kind;
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

int gemm(const GemmArgs& a, hipStream_t s) {
  MPR_REQUIRE(a.M >= 0 && a.N >= 0 && a.K > 0, "gemm: bad shape M=%d N=%d K=%d", a.M, a.N, a.K);
  if (a.M == 0 || a.N == 0) return MPR_OK;
  MPR_REQUIRE(a.K % 4 == 0 && a.lda % 4 == 0 && a.ldw % 4 == 0 && aligned16(a.A) &&
                  aligned16(a.W),
              "gemm: K/lda/ldw must be multiples of 4 and A/W 16-byte aligned (K=%d)", a.K);
  // One tile shape: 64x64 (4 waves of 32x32, ~55 KB of LDS, 2 blocks per CU).  Measured on
  // MI355X over the ViT/T5 projection shapes (tools/gbench.hip): 128x64 and 128x128 tiles are
  // slower at every shape up to 2048^3 (fewer blocks, one per CU by LDS), 32x64 halves the
  // waves per block without adding SIMD work.  Split-K over blockIdx.z (in-launch agent-scope
  // combine) was slower at every shape too (800x768x768: 21.7 us plain, 30.6 at S=2, 47 at
  // S=4): the release fence writes back the XCD L2 and a 64x64 fp32 slab per slice costs more
  // than the idle CUs it fills.
  return probed(PROBE_GEMM, a, s, [&]() { return launch_gemm<64, 64, 1, 1>(a, s); });
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

template <int MAXC, int NT, bool LOOP>
void launch_skinny(const SkinnyArgs& sa, int F, unsigned grid, hipStream_t s) {
#define MPR_SK(f)                                                                          \
  case f:                                                                                  \
    hipLaunchKernelGGL((gemm_skinny_kernel<MAXC, NT, f, LOOP>), dim3(grid), dim3(512), 0, s, sa); \
    break;
  if constexpr (NT > 1) {
    switch (F) { MPR_SK(SKF_AMAX) MPR_SK(SKF_AMAX | SKF_RMS) default: break; }
  } else {
    switch (F) {
      MPR_SK(0) MPR_SK(1) MPR_SK(2) MPR_SK(3) MPR_SK(4) MPR_SK(5) MPR_SK(6) MPR_SK(7)
      MPR_SK(SKF_AMAX) MPR_SK(SKF_AMAX | SKF_RMS)
      default: break;
    }
  }
#undef MPR_SK
}

int gemm_skinny(const SkinnyArgs& sa, hipStream_t s) {
  const GemmArgs& a = sa.g;
  MPR_REQUIRE(a.M >= 0 && a.M <= 16 && a.N >= 0 && a.K > 0, "gemm_skinny: bad shape M=%d", a.M);
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
  const int F = (sa.rms_w ? SKF_RMS : 0) | (a.R ? SKF_RES : 0) |
                (a.act == ACT_RELU ? SKF_RELU : 0) | (amax ? SKF_AMAX : 0);
  const int per = (int)cdiv(cdiv(a.K, 16), SK_WAVES);  // 16-column chunks per wave
  const int64_t tiles = cdiv(a.N, 16);
  return probed(PROBE_SKINNY, a, s, [&]() {
    if (amax && tiles >= 1024 && per <= 4)  // lm_head: 2 tiles per block (NT 1/2/4/8 measured
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
