// small_scan_lab.hip — the C2 scan's floor (development aid): scan_small_kernel on a 6,500 x 1,024
// fp32 index and 16 queries against plain streaming reads of the same bytes (407 blocks of 256
// threads, float4 per lane, coalesced 1 KiB per wave instruction) and a row-tile read with the
// scan's lane mapping but no MFMA, each timed over a graph of 200 launches.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/small_scan_lab.hip -o tools/small_scan_lab
#include <cstdio>
#include <functional>
#include <vector>

#include "../multimodalpromptretrieval_amd/csrc/api.hip"
#include "../multimodalpromptretrieval_amd/csrc/encoders.hip"
#include "../multimodalpromptretrieval_amd/csrc/gemm.hip"
#include "../multimodalpromptretrieval_amd/csrc/layers.hip"
#include "../multimodalpromptretrieval_amd/csrc/scan.hip"
#include "../multimodalpromptretrieval_amd/csrc/t5.hip"

using namespace mpr;
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void stream_read(const f4* __restrict__ x, int64_t n4, float* out) {
  const int64_t per = (n4 + gridDim.x - 1) / gridDim.x;
  const int64_t lo = blockIdx.x * per, hi = lo + per < n4 ? lo + per : n4;
  f4 a = {0.f, 0.f, 0.f, 0.f};
  for (int64_t i = lo + threadIdx.x; i < hi; i += 256) a += x[i];
  if (a[0] + a[1] + a[2] + a[3] == 1.2345f) out[0] = a[0];
}

// the scan's mapping: lane (i = row of the 16-row tile, h), wave = quarter of d, 16 chunks
__global__ __launch_bounds__(256) void tile_read(const float* __restrict__ X, int64_t n, float* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, i = lane & 15, h = lane >> 4;
  const int64_t row = blockIdx.x * 16 + i;
  const float* xp = X + (row < n ? row : n - 1) * 1024 + wave * 256 + h * 4;
  f4 v[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) v[u] = *reinterpret_cast<const f4*>(xp + u * 16);
  f4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < 16; ++u) a += v[u];
  if (a[0] + a[1] + a[2] + a[3] == 1.2345f) out[0] = a[0];
}

// the same plus the 16 query rows' fragments (what scan_small_kernel also loads)
__global__ __launch_bounds__(256) void tileq_read(const float* __restrict__ X, int64_t n,
                                                  const float* __restrict__ Q, float* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, i = lane & 15, h = lane >> 4;
  const int64_t row = blockIdx.x * 16 + i;
  const float* xp = X + (row < n ? row : n - 1) * 1024 + wave * 256 + h * 4;
  const float* qp = Q + i * 1024 + wave * 256 + h * 4;
  f4 v[16], w[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    v[u] = *reinterpret_cast<const f4*>(xp + u * 16);
    w[u] = *reinterpret_cast<const f4*>(qp + u * 16);
  }
  f4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < 16; ++u) a += v[u] * w[u];
  if (a[0] + a[1] + a[2] + a[3] == 1.2345f) out[0] = a[0];
}

static double time_graph(hipStream_t s, const std::function<void()>& body, int n) {
  body();
  (void)hipStreamSynchronize(s);
  hipGraph_t g;
  hipGraphExec_t e;
  (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
  for (int i = 0; i < n; ++i) body();
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
  return ms * 1e3 / n;
}

int main() {
  const int64_t n = 6500, d = 1024;
  const int b = 16;
  float *X, *xn, *Q, *ck, *out, *big;
  int64_t* ci;
  (void)hipMalloc(&X, n * d * 4);
  (void)hipMalloc(&xn, n * 4);
  (void)hipMalloc(&Q, b * d * 4);
  (void)hipMalloc(&ck, (size_t)b * 512 * 4);
  (void)hipMalloc(&ci, (size_t)b * 512 * 8);
  (void)hipMalloc(&out, 64);
  (void)hipMalloc(&big, (size_t)512 << 20);
  (void)hipMemset(X, 0, n * d * 4);
  (void)hipMemset(xn, 0, n * 4);
  (void)hipMemset(Q, 0, b * d * 4);
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  const unsigned nb = (unsigned)((n + 16 * SS_TT - 1) / (16 * SS_TT));
  // L2/MALL-warm (the same 26.6 MB every launch) and cold (a 512 MiB sweep between launches)
  for (int cold = 0; cold < 1; ++cold) {
    auto flush = [&]() {
      if (cold) hipLaunchKernelGGL(stream_read, dim3(2048), dim3(256), 0, s,
                                   reinterpret_cast<const f4*>(big), (int64_t)(128 << 20), out);
    };
    const double tf = cold ? time_graph(s, flush, 50) : 0.0;
    printf("%s (flush %.1f us subtracted)\n", cold ? "cold" : "warm", tf);
    printf("  scan_small_kernel TT=1    %7.2f us\n", time_graph(s, [&]() {
      hipLaunchKernelGGL((scan_small_kernel<1, 16, 1>), dim3((unsigned)((n + 15) / 16), 1),
                         dim3(256), 0, s, X, xn, n, (int64_t)0, 0, Q, b, ck, ci);
    }, 50) - tf);
    printf("  scan_small_kernel TT=2    %7.2f us\n", time_graph(s, [&]() {
      hipLaunchKernelGGL((scan_small_kernel<1, 16, 2>), dim3((unsigned)((n + 31) / 32), 1),
                         dim3(256), 0, s, X, xn, n, (int64_t)0, 0, Q, b, ck, ci);
    }, 50) - tf);
    printf("  scan_small_kernel TT=4    %7.2f us\n", time_graph(s, [&]() {
      hipLaunchKernelGGL((scan_small_kernel<1, 16, 4>), dim3((unsigned)((n + 63) / 64), 1),
                         dim3(256), 0, s, X, xn, n, (int64_t)0, 0, Q, b, ck, ci);
    }, 50) - tf);
    printf("  tile_read (scan mapping)  %7.2f us\n", time_graph(s, [&]() {
      flush();
      hipLaunchKernelGGL(tile_read, dim3(nb), dim3(256), 0, s, X, n, out);
    }, 50) - tf);
    printf("  tile+query read           %7.2f us\n", time_graph(s, [&]() {
      flush();
      hipLaunchKernelGGL(tileq_read, dim3(nb), dim3(256), 0, s, X, n, Q, out);
    }, 50) - tf);
    for (unsigned g : {407u, 1024u, 2048u})
      printf("  stream_read %4u blocks   %7.2f us\n", g, time_graph(s, [&]() {
        flush();
        hipLaunchKernelGGL(stream_read, dim3(g), dim3(256), 0, s,
                           reinterpret_cast<const f4*>(X), n * d / 4, out);
      }, 50) - tf);
  }
  return 0;
}
