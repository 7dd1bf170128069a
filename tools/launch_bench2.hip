// launch_bench2.hip — what a dependent decode-chain step costs on this box (development aid):
// per-kernel wall time of 1000-kernel chains (eager vs hipGraph; trivial bodies vs a GEMV-like
// body that reads the 32 KiB vector the previous kernel wrote; 256- vs 512-thread blocks; small vs
// 35 KiB static LDS; small vs 256-byte kernargs), and a persistent kernel doing the same chain
// with a counter grid barrier per step.
// build: hipcc -O3 --offload-arch=gfx950 tools/launch_bench2.hip -o tools/launch_bench2
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));

struct Big {
  const float* p[24];
  int n[16];
};

__global__ __launch_bounds__(256) void tiny256(float* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1.f;
}
__global__ __launch_bounds__(512) void tiny512_lds(float* p) {
  __shared__ float s[35 * 256];
  s[threadIdx.x] = p[threadIdx.x & 7];
  __syncthreads();
  if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += s[5];
}
__global__ __launch_bounds__(256) void tiny_bigarg(Big b) {
  if (threadIdx.x == 0 && blockIdx.x == 0) ((float*)b.p[0])[0] += (float)b.n[3];
}
// GEMV-like: 32 blocks x 512 threads; block reads a 32 KiB weight slice and the 32 KiB input
// vector x (written by the previous kernel), reduces, writes 16 floats of y.
__global__ __launch_bounds__(512) void gemv_like(const float* __restrict__ W, const float* x,
                                                 float* y) {
  const int t = threadIdx.x;
  const f4* w4 = reinterpret_cast<const f4*>(W) + (size_t)blockIdx.x * 2048;
  const f4* x4 = reinterpret_cast<const f4*>(x);
  f4 a = w4[t] * x4[t] + w4[t + 512] * x4[t + 512] + w4[t + 1024] * x4[t + 1024] +
         w4[t + 1536] * x4[t + 1536];
  __shared__ float red[512];
  red[t] = a[0] + a[1] + a[2] + a[3];
  __syncthreads();
  if (t < 64) {
    float s = 0.f;
    for (int i = t; i < 512; i += 64) s += red[i];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (t < 16) y[blockIdx.x * 16 + t] = s * 1e-3f + 1.f;
  }
}

// persistent: nsteps of gemv_like separated by a monotonic-counter grid barrier (relaxed agent
// atomics + release/acquire fences), nblk co-resident blocks (<= CUs, one per CU).
__global__ __launch_bounds__(512) void persistent(const float* __restrict__ W, float* xa,
                                                  float* xb, unsigned* ctr, int nsteps, int nblk) {
  const int t = threadIdx.x;
  __shared__ float red[512];
  for (int st = 0; st < nsteps; ++st) {
    const float* x = (st & 1) ? xb : xa;
    float* y = (st & 1) ? xa : xb;
    const f4* w4 = reinterpret_cast<const f4*>(W) + (size_t)(blockIdx.x & 31) * 2048;
    const f4* x4 = reinterpret_cast<const f4*>(x);
    f4 a = w4[t] * x4[t] + w4[t + 512] * x4[t + 512] + w4[t + 1024] * x4[t + 1024] +
           w4[t + 1536] * x4[t + 1536];
    red[t] = a[0] + a[1] + a[2] + a[3];
    __syncthreads();
    if (t < 64) {
      float s = 0.f;
      for (int i = t; i < 512; i += 64) s += red[i];
      for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
      if (t < 16 && blockIdx.x < 32) y[blockIdx.x * 16 + t] = s * 1e-3f + 1.f;
    }
    __syncthreads();
    if (t == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned want = (unsigned)(st + 1) * nblk;
      long spins = 0;
      while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want &&
             ++spins < 20000000)
        __builtin_amdgcn_s_sleep(1);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
  }
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

template <class L>
void bench(const char* name, hipStream_t s, int n, L&& launch) {
  for (int i = 0; i < 50; ++i) launch();
  (void)hipStreamSynchronize(s);
  double t = now_us();
  for (int i = 0; i < n; ++i) launch();
  (void)hipStreamSynchronize(s);
  const double eager = (now_us() - t) / n;
  hipGraph_t g;
  (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
  for (int i = 0; i < n; ++i) launch();
  (void)hipStreamEndCapture(s, &g);
  hipGraphExec_t e;
  (void)hipGraphInstantiate(&e, g, nullptr, nullptr, 0);
  (void)hipGraphLaunch(e, s);
  (void)hipStreamSynchronize(s);
  double best = 1e30;
  for (int r = 0; r < 3; ++r) {
    t = now_us();
    (void)hipGraphLaunch(e, s);
    (void)hipStreamSynchronize(s);
    best = std::min(best, (now_us() - t) / n);
  }
  printf("%-34s eager %6.2f us/kernel   graph %6.2f us/kernel\n", name, eager, best);
  (void)hipGraphExecDestroy(e);
  (void)hipGraphDestroy(g);
}

int main() {
  float *p, *W, *xa, *xb;
  unsigned* ctr;
  (void)hipMalloc(&p, 1 << 20);
  (void)hipMalloc(&W, 32 * 2048 * 16);
  (void)hipMalloc(&xa, 1 << 16);
  (void)hipMalloc(&xb, 1 << 16);
  (void)hipMalloc(&ctr, 256);
  (void)hipMemset(p, 0, 1 << 20);
  (void)hipMemset(W, 0, 32 * 2048 * 16);
  (void)hipMemset(xa, 0, 1 << 16);
  (void)hipMemset(xb, 0, 1 << 16);
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  const int N = 1000;
  Big big{};
  big.p[0] = p;
  bench("tiny 32x256", s, N, [&] { hipLaunchKernelGGL(tiny256, dim3(32), dim3(256), 0, s, p); });
  bench("tiny 256x256", s, N, [&] { hipLaunchKernelGGL(tiny256, dim3(256), dim3(256), 0, s, p); });
  bench("tiny 32x512 35KB LDS", s, N,
        [&] { hipLaunchKernelGGL(tiny512_lds, dim3(32), dim3(512), 0, s, p); });
  bench("tiny 32x256 256B kernarg", s, N,
        [&] { hipLaunchKernelGGL(tiny_bigarg, dim3(32), dim3(256), 0, s, big); });
  int i = 0;
  bench("gemv-like 32x512 (dependent x)", s, N, [&] {
    float* x = (i & 1) ? xb : xa;
    float* y = (i & 1) ? xa : xb;
    ++i;
    hipLaunchKernelGGL(gemv_like, dim3(32), dim3(512), 0, s, W, x, y);
  });
  for (int nb : {32, 128, 256}) {
    (void)hipMemset(ctr, 0, 256);
    (void)hipDeviceSynchronize();
    double t = now_us();
    hipLaunchKernelGGL(persistent, dim3(nb), dim3(512), 0, s, W, xa, xb, ctr, N, nb);
    (void)hipStreamSynchronize(s);
    printf("persistent %3d blocks, barrier/step: %6.2f us/step\n", nb, (now_us() - t) / N);
  }
  return 0;
}
