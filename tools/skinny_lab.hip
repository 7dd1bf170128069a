// skinny_lab.hip — where does a decode GEMV kernel's time go? (development aid)
// Chains of 1000 dependent launches in a hipGraph, 16 x 512 activations, 512 x 512 fp32 weights
// (1 MiB, six slices rotating so they stay in MALL like the T5 decode weights).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/skinny_lab.hip -o tools/skinny_lab
#include <hip/hip_runtime.h>

#include <cstdio>
#include <functional>

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Variant knobs: MF = use MFMA (else plain FMA), RED = LDS reduction over the 8 waves.
// Each block: 16 W rows, 8 waves split K (K = 512: 4 chunks of 16 per wave).
template <bool MF, bool RED, int WAVES, bool CW = false, int COAL = 0>
__global__ __launch_bounds__(64 * WAVES) void skinny(const float* __restrict__ W,
                                                     const float* __restrict__ x, float* y) {
  constexpr int K = 512, N = 512;
  __shared__ f32x4 red[WAVES][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 15, h = lane >> 4;
  const int n0 = blockIdx.x * 16;
  constexpr int PER = K / 16 / WAVES;
  // COAL bit 0: W read lane-contiguous (pre-packed tile layout); bit 1: x read lane-contiguous
  const float* wp = (COAL & 1) ? W + (size_t)n0 * K + lane * 4 - wave * 0 : W + (size_t)(n0 + i) * K + h * 4;
  const float* xp = (COAL & 2) ? x + lane * 4 : x + (size_t)i * K + h * 4;
  constexpr int WSTEP = (COAL & 1) ? 256 : 16, XSTEP = (COAL & 2) ? 256 : 16;
  f32x4 wv[PER], xv[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int c = wave * PER + u;
    wv[u] = *reinterpret_cast<const f32x4*>(wp + c * WSTEP);
    xv[u] = *reinterpret_cast<const f32x4*>(xp + c * XSTEP);
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < PER; ++u)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if constexpr (MF)
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[u][e], xv[u][e], acc, 0, 0, 0);
      else
        acc[e] += wv[u][e] * xv[u][e];
    }
  if constexpr (RED) {
    red[wave][lane] = acc;
    __syncthreads();
    if (wave != 0) return;
#pragma unroll
    for (int w = 1; w < WAVES; ++w) acc += red[w][lane];
  }
  const int m = lane & 15;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int n = n0 + (lane >> 4) * 4 + r;
    if constexpr (CW)  // contiguous 1 KiB per block instead of 16 rows x 64 B
      y[(size_t)blockIdx.x * 256 + lane * 4 + r] = acc[r];
    else
      y[(size_t)m * N + n] = acc[r];
  }
}

__global__ void trivial(float* y) {
  if (threadIdx.x == 0) y[blockIdx.x] = 1.f;
}

// chain_bench's streaming GEMV body for reference: thread reads 64 contiguous bytes of W
__global__ __launch_bounds__(512) void stream_gemv(const float* __restrict__ W, const float* x,
                                                   float* y) {
  const int t = blockIdx.x * 512 + threadIdx.x;
  const f32x4* w4 = reinterpret_cast<const f32x4*>(W) + (size_t)t * 4;
  const f32x4 xv = reinterpret_cast<const f32x4*>(x)[t & 2047];
  f32x4 wv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) wv[i] = w4[i];
  f32x4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 4; ++i) acc += wv[i] * xv;
  __shared__ float red[512];
  red[threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
  __syncthreads();
  if (threadIdx.x < 64) {
    float s = 0;
    for (int i = threadIdx.x; i < 512; i += 64) s += red[i];
    y[(blockIdx.x * 64 + threadIdx.x) & 8191] = s;
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
  auto wsl = [&](int i) { return W + (size_t)(i % 6) * (1 << 20); };
  auto X = [&](int i) { return (i & 1) ? y : x; };
  auto Y = [&](int i) { return (i & 1) ? x : y; };
  printf("trivial 32 blocks        %.3f us\n",
         time_graph(s, [&](int i) { hipLaunchKernelGGL(trivial, dim3(32), dim3(64), 0, s, Y(i)); }));
  printf("stream_gemv 32x512       %.3f us\n", time_graph(s, [&](int i) {
           hipLaunchKernelGGL(stream_gemv, dim3(32), dim3(512), 0, s, wsl(i), X(i), Y(i));
         }));
  printf("skinny mfma red 8w       %.3f us\n", time_graph(s, [&](int i) {
           hipLaunchKernelGGL((skinny<true, true, 8>), dim3(32), dim3(512), 0, s, wsl(i), X(i), Y(i));
         }));
  printf("skinny fma  red 8w       %.3f us\n", time_graph(s, [&](int i) {
           hipLaunchKernelGGL((skinny<false, true, 8>), dim3(32), dim3(512), 0, s, wsl(i), X(i), Y(i));
         }));
  printf("skinny mfma nored 8w     %.3f us\n", time_graph(s, [&](int i) {
           hipLaunchKernelGGL((skinny<true, false, 8>), dim3(32), dim3(512), 0, s, wsl(i), X(i), Y(i));
         }));
  printf("skinny mfma red 4w       %.3f us\n", time_graph(s, [&](int i) {
           hipLaunchKernelGGL((skinny<true, true, 4>), dim3(32), dim3(256), 0, s, wsl(i), X(i), Y(i));
         }));
  printf("skinny mfma red 2w       %.3f us\n", time_graph(s, [&](int i) {
           hipLaunchKernelGGL((skinny<true, true, 2>), dim3(32), dim3(128), 0, s, wsl(i), X(i), Y(i));
         }));
  printf("skinny mfma red 8w sameW %.3f us\n", time_graph(s, [&](int i) {
           hipLaunchKernelGGL((skinny<true, true, 8>), dim3(32), dim3(512), 0, s, W, X(i), Y(i));
         }));
  printf("skinny contiguous y      %.3f us\n", time_graph(s, [&](int i) {
           hipLaunchKernelGGL((skinny<true, true, 8, true>), dim3(32), dim3(512), 0, s, wsl(i), X(i), Y(i));
         }));
  printf("skinny fixed x, y        %.3f us\n", time_graph(s, [&](int i) {
           hipLaunchKernelGGL((skinny<true, true, 8>), dim3(32), dim3(512), 0, s, wsl(i), x, y);
         }));
  printf("skinny fixed x, cont y   %.3f us\n", time_graph(s, [&](int i) {
           hipLaunchKernelGGL((skinny<true, true, 8, true>), dim3(32), dim3(512), 0, s, wsl(i), x, y);
         }));
  printf("stream_gemv fixed x,y    %.3f us\n", time_graph(s, [&](int i) {
           hipLaunchKernelGGL(stream_gemv, dim3(32), dim3(512), 0, s, wsl(i), x, y);
         }));
  printf("skinny W packed          %.3f us\n", time_graph(s, [&](int i) {
           hipLaunchKernelGGL((skinny<true, true, 8, false, 1>), dim3(32), dim3(512), 0, s, wsl(i), X(i), Y(i));
         }));
  printf("skinny x coalesced       %.3f us\n", time_graph(s, [&](int i) {
           hipLaunchKernelGGL((skinny<true, true, 8, false, 2>), dim3(32), dim3(512), 0, s, wsl(i), X(i), Y(i));
         }));
  printf("skinny W+x coalesced     %.3f us\n", time_graph(s, [&](int i) {
           hipLaunchKernelGGL((skinny<true, true, 8, false, 3>), dim3(32), dim3(512), 0, s, wsl(i), X(i), Y(i));
         }));
  return 0;
}
