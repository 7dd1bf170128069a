// launch_bench3.hip — a decode-step-shaped chain (development aid): 1000 dependent GEMV-like
// launches, each 32 blocks x 512 threads reading its own 1 MiB weight slice of a 160 MiB set
// (cycled, as the T5 decode streams ~154 MB of weights per step) and the 32 KiB vector the
// previous launch wrote.  Variants: weights from the cycled set (MALL/HBM) vs one slice (L2);
// each launch also pulling the NEXT launch's slice toward the caches (plain loads whose result
// is kept alive by a never-taken store), by 32 or 256 blocks.
// build: hipcc -O3 --offload-arch=gfx950 tools/launch_bench3.hip -o tools/launch_bench3
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr size_t SLICE = 1 << 18;  // floats per launch (1 MiB)

// blocks [0, 32) compute; every block b also touches 1/nb of the next slice when pf != null
__global__ __launch_bounds__(512) void gemv(const float* __restrict__ W, const float* x, float* y,
                                            const float* __restrict__ pf, int flag) {
  const int t = threadIdx.x;
  __shared__ float red[512];
  float keep = 0.f;
  if (pf) {  // this block's share of the next slice: one float4 per thread per 8 KiB
    const int nb = gridDim.x;
    const f4* p = reinterpret_cast<const f4*>(pf);
    for (size_t i = (size_t)blockIdx.x * 512 + t; i < SLICE / 4; i += (size_t)nb * 512)
      keep += p[i][0];
  }
  if (blockIdx.x < 32) {
    const f4* w4 = reinterpret_cast<const f4*>(W) + (size_t)blockIdx.x * 2048;
    const f4* x4 = reinterpret_cast<const f4*>(x);
    f4 a = w4[t] * x4[t] + w4[t + 512] * x4[t + 512] + w4[t + 1024] * x4[t + 1024] +
           w4[t + 1536] * x4[t + 1536];
    red[t] = a[0] + a[1] + a[2] + a[3];
    __syncthreads();
    if (t < 64) {
      float s = 0.f;
      for (int i = t; i < 512; i += 64) s += red[i];
      for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
      if (t < 16) y[blockIdx.x * 16 + t] = s * 1e-3f + 1.f;
    }
  }
  if (flag == 12345 && keep == 1.2345f) y[0] = keep;  // never true: keeps the prefetch loads
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int main() {
  const int N = 1000, NS = 160;
  float *W, *xa, *xb;
  (void)hipMalloc(&W, (size_t)NS * SLICE * 4);
  (void)hipMalloc(&xa, 1 << 16);
  (void)hipMalloc(&xb, 1 << 16);
  (void)hipMemset(W, 0, (size_t)NS * SLICE * 4);
  (void)hipMemset(xa, 0, 1 << 16);
  (void)hipMemset(xb, 0, 1 << 16);
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  struct V { const char* name; bool cycle; int pf_blocks; };
  const V vs[] = {{"one slice (L2)", false, 0},
                  {"cycled 160 MiB", true, 0},
                  {"cycled + next slice by 32 blocks", true, 32},
                  {"cycled + next slice by 256 blocks", true, 256},
                  {"cycled + next slice by 1024 blocks", true, 1024}};
  for (const V& v : vs) {
    hipGraph_t g;
    (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    for (int i = 0; i < N; ++i) {
      const float* w = W + (v.cycle ? (size_t)(i % NS) * SLICE : 0);
      const float* nx = v.pf_blocks ? W + (size_t)((i + 1) % NS) * SLICE : nullptr;
      hipLaunchKernelGGL(gemv, dim3(v.pf_blocks ? v.pf_blocks : 32), dim3(512), 0, s, w,
                         (i & 1) ? xb : xa, (i & 1) ? xa : xb, nx, i);
    }
    (void)hipStreamEndCapture(s, &g);
    hipGraphExec_t e;
    (void)hipGraphInstantiate(&e, g, nullptr, nullptr, 0);
    (void)hipGraphLaunch(e, s);
    (void)hipStreamSynchronize(s);
    double best = 1e30;
    for (int r = 0; r < 3; ++r) {
      const double t = now_us();
      (void)hipGraphLaunch(e, s);
      (void)hipStreamSynchronize(s);
      best = std::min(best, (now_us() - t) / N);
    }
    printf("%-40s %6.2f us/launch\n", v.name, best);
    (void)hipGraphExecDestroy(e);
    (void)hipGraphDestroy(g);
  }
  return 0;
}
