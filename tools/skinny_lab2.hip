// skinny_lab2.hip — ablations of the library's decode GEMV (development aid): which part of
// gemm_skinny_kernel costs the microsecond the bare streaming GEMV does not pay?
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/skinny_lab2.hip -o tools/skinny_lab2
#include <hip/hip_runtime.h>

#include <cstdio>
#include <functional>

#include "../multimodalpromptretrieval_amd/csrc/api.hip"
#include "../multimodalpromptretrieval_amd/csrc/encoders.hip"
#include "../multimodalpromptretrieval_amd/csrc/gemm.hip"
#include "../multimodalpromptretrieval_amd/csrc/layers.hip"
#include "../multimodalpromptretrieval_amd/csrc/scan.hip"
#include "../multimodalpromptretrieval_amd/csrc/t5.hip"

typedef float f32x4 __attribute__((ext_vector_type(4)));

struct Args {
  const float* wpk;
  const float* A;
  float* C;
  const float* R;
  int M, N, K, lda, ldc, ldr;
  char pad[160];  // kernarg size of the library's SkinnyArgs
};

// STAGE: 1 = A rows through the wave's LDS slab (library), 0 = direct lane-contiguous loads
// (wrong math, cost reference).  EPI: 1 = library epilogue (residual prefetch, bounds), 0 = bare.
// RED: 1 = 8-wave LDS reduction + barrier, 0 = each wave stores its partial.
template <int STAGE, int EPI, int RED>
__global__ __launch_bounds__(512) void k(Args a) {
  constexpr int MAXC = 4, XLD = MAXC * 16 + 4, W8 = 8;
  __shared__ __attribute__((aligned(16))) float xs[W8][16][XLD];
  __shared__ __attribute__((aligned(16))) f32x4 red[W8][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int M = a.M, N = a.N, K = a.K;
  const int i = lane & 15, h = lane >> 4;
  const int nchunk = (K + 15) / 16, per = (nchunk + W8 - 1) / W8;
  const int c_lo = wave * per, c_hi = min(nchunk, c_lo + per);
  const f32x4* wp = reinterpret_cast<const f32x4*>(a.wpk) + (int64_t)blockIdx.x * nchunk * 64 + lane;
  float rres[4] = {0.f, 0.f, 0.f, 0.f};
  if (EPI && wave == 0 && a.R) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = min(blockIdx.x * 16 + (lane >> 4) * 4 + r, N - 1);
      rres[r] = a.R[(int64_t)min(i, M - 1) * a.ldr + n];
    }
  }
  f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  const int c0 = c_lo;
  f32x4 wv[MAXC], xr[MAXC];
#pragma unroll
  for (int u = 0; u < MAXC; ++u) wv[u] = wp[(int64_t)min(c0 + u, c_hi - 1) * 64];
  if (STAGE) {
#pragma unroll
    for (int u = 0; u < MAXC; ++u) {
      const int q = u * 64 + lane, row = q / (4 * MAXC), col = c0 * 16 + (q % (4 * MAXC)) * 4;
      const bool ok = row < M && col < c_hi * 16 && col < K;
      xr[u] = *reinterpret_cast<const f32x4*>(a.A + (int64_t)min(row, M - 1) * a.lda +
                                              min(col, K - 4));
      if (!ok) xr[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < MAXC; ++u) {
      const int q = u * 64 + lane;
      *reinterpret_cast<f32x4*>(&xs[wave][q / (4 * MAXC)][(q % (4 * MAXC)) * 4]) = xr[u];
    }
#pragma unroll
    for (int u = 0; u < MAXC; ++u) xr[u] = *reinterpret_cast<const f32x4*>(&xs[wave][i][u * 16 + h * 4]);
  } else {
#pragma unroll
    for (int u = 0; u < MAXC; ++u)
      xr[u] = *reinterpret_cast<const f32x4*>(a.A + c0 * 256 + u * 256 + lane * 4);
  }
#pragma unroll
  for (int u = 0; u < MAXC; ++u)
#pragma unroll
    for (int e = 0; e < 4; ++e)
      acc[u & 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[u][e], xr[u][e], acc[u & 1], 0, 0, 0);
  f32x4 sum = acc[0] + acc[1];
  if (RED) {
    red[wave][lane] = sum;
    __syncthreads();
    if (wave != 0) return;
#pragma unroll
    for (int w = 1; w < W8; ++w) sum += red[w][lane];
  }
  const int m = lane & 15;
  if (EPI) {
    if (m >= M) return;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = blockIdx.x * 16 + (lane >> 4) * 4 + r;
      if (n >= N) continue;
      float v = sum[r];
      if (a.R) v += rres[r];
      a.C[(int64_t)m * a.ldc + n] = v;
    }
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      a.C[(int64_t)m * a.ldc + blockIdx.x * 16 + (lane >> 4) * 4 + r + (RED ? 0 : wave * 0)] = sum[r];
  }
}

static double time_graph(hipStream_t s, const std::function<void(int)>& body, int n = 1000) {
  body(0);
  (void)hipStreamSynchronize(s);
  hipGraph_t g;
  hipGraphExec_t e;
  (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
  for (int i = 0; i < n; ++i) body(i);
  (void)hipStreamEndCapture(s, &g);
  (void)hipGraphInstantiate(&e, g, nullptr, nullptr, 0);
  (void)hipGraphLaunch(e, s);
  (void)hipStreamSynchronize(s);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a, s);
  (void)hipGraphLaunch(e, s);
  (void)hipEventRecord(b, s);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipGraphExecDestroy(e);
  (void)hipGraphDestroy(g);
  return ms * 1e3 / n;
}

int main() {
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  float *W, *x, *y;
  (void)hipMalloc(&W, 6 << 22);
  (void)hipMalloc(&x, 1 << 20);
  (void)hipMalloc(&y, 1 << 20);
  (void)hipMemset(W, 0, 6 << 22);
  (void)hipMemset(x, 0, 1 << 20);
  (void)hipMemset(y, 0, 1 << 20);
  auto args = [&](int i, bool res) {
    Args a{};
    a.wpk = W + (size_t)(i % 6) * (1 << 20);
    a.A = (i & 1) ? y : x;
    a.C = (i & 1) ? x : y;
    a.R = res ? a.C : nullptr;
    a.M = 16; a.N = 512; a.K = 512; a.lda = 512; a.ldc = 512; a.ldr = 512;
    return a;
  };
#define RUN(NAME, S, E, R, RES)                                                             \
  printf("%-34s %.3f us\n", NAME, time_graph(s, [&](int i) {                                 \
           hipLaunchKernelGGL((k<S, E, R>), dim3(32), dim3(512), 0, s, args(i, RES));        \
         }))
  RUN("bare (direct x, no epi, red)", 0, 0, 1, false);
  RUN("stage", 1, 0, 1, false);
  RUN("stage + epi", 1, 1, 1, false);
  RUN("stage + epi + residual", 1, 1, 1, true);
  RUN("direct + epi + residual", 0, 1, 1, true);
  RUN("stage, no red", 1, 0, 0, false);
  auto lib = [&](int i, bool res) {
    mpr::SkinnyArgs a;
    a.wpk = W + (size_t)(i % 6) * (1 << 20);
    a.g.A = (i & 1) ? y : x;
    a.g.C = (i & 1) ? x : y;
    if (res) { a.g.R = a.g.C; a.g.ldr = 512; }
    a.g.M = 16; a.g.N = 512; a.g.K = 512; a.g.lda = 512; a.g.ldc = 512;
    return a;
  };
  printf("%-34s %.3f us\n", "library gemm_skinny()", time_graph(s, [&](int i) {
           mpr::gemm_skinny(lib(i, false), s); }));
  printf("%-34s %.3f us\n", "library gemm_skinny() +res", time_graph(s, [&](int i) {
           mpr::gemm_skinny(lib(i, true), s); }));
  return 0;
}
