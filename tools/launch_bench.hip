// launch_bench.hip — per-kernel boundary cost on this box: null stream vs created stream,
// eager vs hipGraph replay (development aid).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

__global__ void tiny(float* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1.f;
}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int main() {
  float* p;
  (void)hipMalloc(&p, 1024);
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  const int N = 2000;
  for (int pass = 0; pass < 2; ++pass) {
    for (int which = 0; which < 2; ++which) {
      hipStream_t st = which ? s : nullptr;
      for (int w = 0; w < 100; ++w) hipLaunchKernelGGL(tiny, dim3(32), dim3(256), 0, st, p);
      (void)hipStreamSynchronize(st);
      double t = now_ms();
      for (int i = 0; i < N; ++i) hipLaunchKernelGGL(tiny, dim3(32), dim3(256), 0, st, p);
      (void)hipStreamSynchronize(st);
      printf("eager %s: %.3f us/kernel\n", which ? "stream" : "null  ", (now_ms() - t) * 1e3 / N);
    }
    hipGraph_t g;
    (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    for (int i = 0; i < N; ++i) hipLaunchKernelGGL(tiny, dim3(32), dim3(256), 0, s, p);
    (void)hipStreamEndCapture(s, &g);
    hipGraphExec_t e;
    (void)hipGraphInstantiate(&e, g, nullptr, nullptr, 0);
    for (int which = 0; which < 2; ++which) {
      hipStream_t st = which ? s : nullptr;
      (void)hipGraphLaunch(e, st);
      (void)hipStreamSynchronize(st);
      double t = now_ms();
      (void)hipGraphLaunch(e, st);
      (void)hipStreamSynchronize(st);
      printf("graph %s: %.3f us/kernel\n", which ? "stream" : "null  ", (now_ms() - t) * 1e3 / N);
    }
    (void)hipGraphExecDestroy(e);
    (void)hipGraphDestroy(g);
  }
  return 0;
}
