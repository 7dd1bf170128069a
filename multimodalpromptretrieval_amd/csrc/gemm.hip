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
// registers as the A operand of v_mfma_f32_16x16x4_f32 (16 output columns per wave), the 16
// activation rows are the B operand, K is split across the 4 waves of a block and reduced through
// LDS, and T5's RMSNorm of the activation rows can be fused into the operand load.
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
  constexpr int BK = 32, LDK = BK + 4;
  constexpr int LA = BM * (BK / 4) / NT, LB = BN * (BK / 4) / NT;
  static_assert(LA * NT == BM * (BK / 4) && LB * NT == BN * (BK / 4), "loader split");

  __shared__ __attribute__((aligned(16))) float As[2][BM][LDK];
  __shared__ __attribute__((aligned(16))) float Bs[2][BN][LDK];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int M = a.M, N = a.N, K = a.K;

  f32x4 ra[LA], rb[LB];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int idx = tid + i * NT, r = idx >> 3, c = k0 + (idx & 7) * 4, row = m0 + r;
      if (row < M && c < K)
        ra[i] = *reinterpret_cast<const f32x4*>(a.A + (int64_t)row * a.lda + c);
      else
        ra[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int idx = tid + i * NT, r = idx >> 3, c = k0 + (idx & 7) * 4, row = n0 + r;
      if (row < N && c < K)
        rb[i] = *reinterpret_cast<const f32x4*>(a.W + (int64_t)row * a.ldw + c);
      else
        rb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto swrite = [&](int buf) {
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int idx = tid + i * NT;
      *reinterpret_cast<f32x4*>(&As[buf][idx >> 3][(idx & 7) * 4]) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int idx = tid + i * NT;
      *reinterpret_cast<f32x4*>(&Bs[buf][idx >> 3][(idx & 7) * 4]) = rb[i];
    }
  };

  f32x16 acc[WM][WN];
#pragma unroll
  for (int mi = 0; mi < WM; ++mi)
#pragma unroll
    for (int ni = 0; ni < WN; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;

  const int nk = (K + BK - 1) / BK;
  gload(0);
  swrite(0);
  __syncthreads();

  const int li = lane & 31, lh = lane >> 5;
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * BK);
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      f32x4 af[WM], bf[WN];
#pragma unroll
      for (int mi = 0; mi < WM; ++mi)
        af[mi] = *reinterpret_cast<const f32x4*>(
            &As[buf][wm * 32 * WM + mi * 32 + li][lh * 16 + s4 * 4]);
#pragma unroll
      for (int ni = 0; ni < WN; ++ni)
        bf[ni] = *reinterpret_cast<const f32x4*>(
            &Bs[buf][wn * 32 * WN + ni * 32 + li][lh * 16 + s4 * 4]);
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int mi = 0; mi < WM; ++mi)
#pragma unroll
          for (int ni = 0; ni < WN; ++ni)
            acc[mi][ni] =
                __builtin_amdgcn_mfma_f32_32x32x2f32(af[mi][c], bf[ni][c], acc[mi][ni], 0, 0, 0);
    }
    if (kt + 1 < nk) {
      swrite(buf ^ 1);
      __syncthreads();
    }
  }

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
constexpr int SK_WAVES = 4;

__global__ __launch_bounds__(256) void gemm_skinny_kernel(SkinnyArgs sa) {
  const GemmArgs& a = sa.g;
  __shared__ float rstd_s[16];
  __shared__ __attribute__((aligned(16))) float red[SK_WAVES][64][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int M = a.M, N = a.N, K = a.K;
  const int n0 = blockIdx.x * 16;
  const int i = lane & 15, h = lane >> 4;

  if (sa.rms_w) {
    // 16 threads per row: sum of squares of A[row, :].
    const int row = tid >> 4, sub = tid & 15;
    float ss = 0.f;
    if (row < M) {
      const float* x = a.A + (int64_t)row * a.lda;
      for (int k = sub * 4; k < K; k += 64) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(x + k);
        ss += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
      }
    }
#pragma unroll
    for (int off = 8; off >= 1; off >>= 1) ss += __shfl_xor(ss, off, 64);
    if (sub == 0) rstd_s[row] = 1.0f / sqrtf(ss / (float)K + sa.rms_eps);
    __syncthreads();
  }

  // Each wave owns the K range [k_lo, k_hi) in 16-wide chunks.
  const int nchunk = (K + 15) / 16;
  const int per = (nchunk + SK_WAVES - 1) / SK_WAVES;
  const int c_lo = wave * per, c_hi = min(nchunk, c_lo + per);
  const int wrow = n0 + i;
  const bool wok = wrow < N, xok = i < M;
  const float* wp = a.W + (int64_t)(wok ? wrow : 0) * a.ldw + h * 4;
  const float* xp = a.A + (int64_t)(xok ? i : 0) * a.lda + h * 4;
  const float xr = sa.rms_w && xok ? rstd_s[i] : 1.f;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  constexpr int U = 4;
  const int c_full = min(c_hi, K / 16);
  int c = c_lo;
  for (; c + U <= c_full; c += U) {
    f32x4 wv[U], xv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = (c + u) * 16;
      wv[u] = wok ? *reinterpret_cast<const f32x4*>(wp + k) : f32x4{0.f, 0.f, 0.f, 0.f};
      xv[u] = xok ? *reinterpret_cast<const f32x4*>(xp + k) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (sa.rms_w) {
        const f32x4 g = *reinterpret_cast<const f32x4*>(sa.rms_w + (c + u) * 16 + h * 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) xv[u][e] = (g[e] * (xv[u][e] * xr)) * sa.a_scale;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e)
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[u][e], xv[u][e], acc, 0, 0, 0);
    }
  }
  for (; c < c_hi; ++c) {
    const int k = c * 16 + h * 4;
    f32x4 wv = {0.f, 0.f, 0.f, 0.f}, xv = {0.f, 0.f, 0.f, 0.f};
    if (k < K) {
      if (wok) wv = *reinterpret_cast<const f32x4*>(wp + c * 16);
      if (xok) xv = *reinterpret_cast<const f32x4*>(xp + c * 16);
      if (sa.rms_w) {
        const f32x4 g = *reinterpret_cast<const f32x4*>(sa.rms_w + k);
#pragma unroll
        for (int e = 0; e < 4; ++e) xv[e] = (g[e] * (xv[e] * xr)) * sa.a_scale;
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e)
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[e], xv[e], acc, 0, 0, 0);
  }
  *reinterpret_cast<f32x4*>(&red[wave][lane][0]) = acc;
  __syncthreads();
  if (wave != 0) return;
  f32x4 sum = *reinterpret_cast<const f32x4*>(&red[0][lane][0]);
#pragma unroll
  for (int w = 1; w < SK_WAVES; ++w) {
    const f32x4 p = *reinterpret_cast<const f32x4*>(&red[w][lane][0]);
    sum += p;
  }
  // D[row = W row (n), col = A row (m)]: col = lane&15, row = (lane>>4)*4 + r.
  const int m = lane & 15;
  if (m >= M) return;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int n = n0 + (lane >> 4) * 4 + r;
    if (n >= N) continue;
    float v = act_exact(sum[r] + (a.bias ? a.bias[n] : 0.f), a.act);
    if (a.R) v = a.R[(int64_t)m * a.ldr + n] + v;
    a.C[(int64_t)m * a.ldc + n] = v;
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
  const int64_t blocks128 = cdiv(a.M, 128) * cdiv(a.N, 64);
  // Larger tiles halve LDS traffic per FLOP but only pay while the grid still fills the chip.
  return probed(PROBE_GEMM, a, s, [&]() {
    if (blocks128 >= 512) return launch_gemm<128, 64, 2, 1>(a, s);
    return launch_gemm<64, 64, 1, 1>(a, s);
  });
}

int gemm_skinny(const SkinnyArgs& sa, hipStream_t s) {
  const GemmArgs& a = sa.g;
  MPR_REQUIRE(a.M >= 0 && a.M <= 16 && a.N >= 0 && a.K > 0, "gemm_skinny: bad shape M=%d", a.M);
  if (a.M == 0 || a.N == 0) return MPR_OK;
  MPR_REQUIRE(a.K % 4 == 0 && a.lda % 4 == 0 && a.ldw % 4 == 0 && aligned16(a.A) &&
                  aligned16(a.W) && (!sa.rms_w || aligned16(sa.rms_w)),
              "gemm_skinny: K/lda/ldw must be multiples of 4, operands 16-byte aligned");
  return probed(PROBE_SKINNY, a, s, [&]() {
    dim3 grid((unsigned)cdiv(a.N, 16));
    hipLaunchKernelGGL(gemm_skinny_kernel, grid, dim3(256), 0, s, sa);
    MPR_LAUNCHED();
    return MPR_OK;
  });
}

}  // namespace mpr
