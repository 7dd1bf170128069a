// launch_floor.hip — the per-launch floor of a captured hipGraph chain on one stream: device time
// per launch of N back-to-back dependent launches (a graph of 200, replayed), for empty kernels
// of growing grid, block, kernel-argument size and register use, beside the decode chain's own
// kernel-argument sizes (development aid: what a decode step's 38 launches cost before any work).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/launch_floor.hip -o tools/launch_floor
#include <hip/hip_runtime.h>

#include <cstdio>
#include <functional>

struct Arg64 { int v[16]; };
struct Arg512 { int v[128]; };
struct Arg1k { int v[256]; };

__global__ void k_empty(int* sink) {
  if (sink && threadIdx.x == 1023) sink[0] = 1;
}
__global__ void k_arg512(Arg512 a, int* sink) {
  if (threadIdx.x == 0 && a.v[blockIdx.x & 127] == -7) sink[0] = 1;
}
__global__ void k_arg1k(Arg1k a, int* sink) {
  if (threadIdx.x == 0 && a.v[blockIdx.x & 255] == -7) sink[0] = 1;
}
__global__ void k_store(int* out) {  // every thread writes one int
  out[blockIdx.x * blockDim.x + threadIdx.x] = (int)threadIdx.x;
}
__global__ void k_load_store(const float* in, float* out) {  // one dependent global round trip
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  out[i] = in[i] * 2.f;
}
// a kernel that holds many VGPRs (the decode GEMV's footprint), doing almost nothing
__global__ __launch_bounds__(512) void k_fat(const float* in, float* out, int n) {
  float r[96];
#pragma unroll
  for (int i = 0; i < 96; ++i) r[i] = in[(threadIdx.x + i * 7) & 1023];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 96; ++i) s += r[i] * r[(i * 5) % 96];
  if (n < 0) out[threadIdx.x] = s;
}
__global__ void k_lds(float* out, int n) {  // a 64 KB static LDS object
  __shared__ float buf[16384];
  buf[threadIdx.x] = (float)threadIdx.x;
  __syncthreads();
  if (n < 0) out[threadIdx.x] = buf[(threadIdx.x + 1) & 255];
}

static double per_launch(hipStream_t s, const std::function<void()>& body, int n, bool graph) {
  body();
  (void)hipStreamSynchronize(s);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  float ms = 0;
  if (graph) {
    hipGraph_t g;
    hipGraphExec_t e;
    (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    for (int i = 0; i < n; ++i) body();
    (void)hipStreamEndCapture(s, &g);
    (void)hipGraphInstantiate(&e, g, nullptr, nullptr, 0);
    (void)hipGraphLaunch(e, s);
    (void)hipStreamSynchronize(s);
    double best = 1e30;
    for (int rep = 0; rep < 5; ++rep) {
      (void)hipEventRecord(a, s);
      (void)hipGraphLaunch(e, s);
      (void)hipEventRecord(b, s);
      (void)hipEventSynchronize(b);
      (void)hipEventElapsedTime(&ms, a, b);
      best = ms < best ? ms : best;
    }
    (void)hipGraphExecDestroy(e);
    (void)hipGraphDestroy(g);
    return best * 1e3 / n;
  }
  double best = 1e30;
  for (int rep = 0; rep < 5; ++rep) {
    (void)hipEventRecord(a, s);
    for (int i = 0; i < n; ++i) body();
    (void)hipEventRecord(b, s);
    (void)hipEventSynchronize(b);
    (void)hipEventElapsedTime(&ms, a, b);
    best = ms < best ? ms : best;
  }
  return best * 1e3 / n;
}

int main() {
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  int* sink;
  float *fin, *fout;
  (void)hipMalloc(&sink, 64 << 20);
  (void)hipMalloc(&fin, 64 << 20);
  (void)hipMalloc(&fout, 64 << 20);
  (void)hipMemset(fin, 0, 64 << 20);
  Arg512 a512{};
  Arg1k a1k{};
  struct Case { const char* name; std::function<void()> f; };
  const Case cases[] = {
      {"empty 1x64", [&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, nullptr); }},
      {"empty 128x64", [&] { hipLaunchKernelGGL(k_empty, dim3(128), dim3(64), 0, s, nullptr); }},
      {"empty 128x512", [&] { hipLaunchKernelGGL(k_empty, dim3(128), dim3(512), 0, s, nullptr); }},
      {"empty 1024x256", [&] { hipLaunchKernelGGL(k_empty, dim3(1024), dim3(256), 0, s, nullptr); }},
      {"arg 512 B 128x64", [&] { hipLaunchKernelGGL(k_arg512, dim3(128), dim3(64), 0, s, a512, sink); }},
      {"arg 1 KB 128x64", [&] { hipLaunchKernelGGL(k_arg1k, dim3(128), dim3(64), 0, s, a1k, sink); }},
      {"store 128x64", [&] { hipLaunchKernelGGL(k_store, dim3(128), dim3(64), 0, s, sink); }},
      {"load+store 128x64", [&] { hipLaunchKernelGGL(k_load_store, dim3(128), dim3(64), 0, s, fin, fout); }},
      {"load+store 1024x256", [&] { hipLaunchKernelGGL(k_load_store, dim3(1024), dim3(256), 0, s, fin, fout); }},
      {"fat 128x512 (96 regs live)", [&] { hipLaunchKernelGGL(k_fat, dim3(128), dim3(512), 0, s, fin, fout, 1); }},
      {"lds 64 KB 128x256", [&] { hipLaunchKernelGGL(k_lds, dim3(128), dim3(256), 0, s, fout, 1); }},
  };
  for (const Case& c : cases) {
    const double g = per_launch(s, c.f, 200, true);
    const double p = per_launch(s, c.f, 200, false);
    printf("%-30s graph %6.2f us/launch   stream %6.2f us/launch\n", c.name, g, p);
  }
  return 0;
}
