// chain_bench.hip — cost of a chain of dependent GEMV-like kernels (each reads a 1 MiB weight
// slice plus the 32 KiB vector the previous kernel wrote, writes 32 KiB), eager vs graph, to
// separate the platform's per-kernel floor from kernel design (development aid).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));

// grid = blocks x 512 threads; each thread reads `per` float4 of W and one float4 of x.
__global__ __launch_bounds__(512) void step(const float* __restrict__ W, const float* x, float* y,
                                            int per) {
  const int t = blockIdx.x * 512 + threadIdx.x;
  f4 acc = {0, 0, 0, 0};
  const f4* w4 = reinterpret_cast<const f4*>(W) + (size_t)t * per;
  const f4 xv = reinterpret_cast<const f4*>(x)[t & 2047];
  f4 wv[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) wv[i] = i < per ? w4[i] : f4{0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 16; ++i) acc += wv[i] * xv;
  __shared__ float red[512];
  red[threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
  __syncthreads();
  if (threadIdx.x < 64) {
    float s = 0;
    for (int i = threadIdx.x; i < 512; i += 64) s += red[i];
    y[(blockIdx.x * 64 + threadIdx.x) & 8191] = s;
  }
}

__global__ void empty_k() {}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int main() {
  float *W, *a, *b;
  (void)hipMalloc(&W, 64 << 20);
  (void)hipMalloc(&a, 1 << 20);
  (void)hipMalloc(&b, 1 << 20);
  (void)hipMemset(W, 0, 64 << 20);
  (void)hipMemset(a, 0, 1 << 20);
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  const int N = 1000;
  struct Cfg { int blocks, per; const char* name; } cfgs[] = {
      {32, 4, "32 blk x512, 1 MiB"}, {128, 1, "128 blk x512, 1 MiB"},
      {128, 4, "128 blk x512, 4 MiB"}, {8, 16, "8 blk x512, 1 MiB"}};
  for (auto& c : cfgs) {
    auto body = [&](hipStream_t st) {
      for (int i = 0; i < N; ++i)
        hipLaunchKernelGGL(step, dim3(c.blocks), dim3(512), 0, st,
                           W + (size_t)(i % 8) * (2 << 20), (i & 1) ? b : a, (i & 1) ? a : b,
                           c.per);
    };
    body(s);
    (void)hipStreamSynchronize(s);
    double t = now_ms();
    body(s);
    (void)hipStreamSynchronize(s);
    const double eager = (now_ms() - t) * 1e3 / N;
    hipGraph_t g;
    hipGraphExec_t e;
    (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    body(s);
    (void)hipStreamEndCapture(s, &g);
    (void)hipGraphInstantiate(&e, g, nullptr, nullptr, 0);
    (void)hipGraphLaunch(e, s);
    (void)hipStreamSynchronize(s);
    t = now_ms();
    (void)hipGraphLaunch(e, s);
    (void)hipStreamSynchronize(s);
    const double graph = (now_ms() - t) * 1e3 / N;
    printf("%-22s eager %.3f us/kernel  graph %.3f us/kernel\n", c.name, eager, graph);
    (void)hipGraphExecDestroy(e);
    (void)hipGraphDestroy(g);
  }
  {
    for (int i = 0; i < N; ++i) hipLaunchKernelGGL(empty_k, dim3(1), dim3(64), 0, s);
    (void)hipStreamSynchronize(s);
    double t = now_ms();
    for (int i = 0; i < N; ++i) hipLaunchKernelGGL(empty_k, dim3(1), dim3(64), 0, s);
    (void)hipStreamSynchronize(s);
    printf("empty kernel eager %.3f us\n", (now_ms() - t) * 1e3 / N);
  }
  return 0;
}
