// chain_fuse_lab.hip — can a dependent chain of decode GEMVs run faster inside one launch than as
// one launch per GEMV (development aid)?  P phases of a 16-row GEMV (K 512, N 512, 32 blocks of
// 16 output columns, 8 waves splitting K, v_mfma_f32_16x16x4_f32, packed weights, one distinct
// 1 MiB weight per phase), each phase reading the previous phase's output:
//   launches: one kernel per phase, captured in a hipGraph;
//   fused:    one kernel of 32 x P blocks; block b is phase b / 32.  Its weight loads are issued
//             first, then lane 0 polls the previous phase's arrival counter (sc1 loads, s_sleep);
//             producers store their tile with sc1 (write-through) stores, drain (vmcnt 0), join the
//             block barrier, and one lane adds 1 to the phase counter (agent scope).  Forward
//             progress rests on in-order workgroup dispatch: a block only waits for lower ones.
// Also prints the max |fused - launches| of the final output (must be 0: same arithmetic).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/chain_fuse_lab.hip -o tools/chain_fuse_lab
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int KD = 512, ND = 512, ROWS = 16, TILES = ND / 16, NCH = KD / 16, PER = NCH / 8;

__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// one 16-column tile of y = x W^T (+ small nonlinearity so the chain stays bounded)
template <bool FUSED>
__device__ __forceinline__ void gemv_tile(const float* __restrict__ wpk, const float* x, float* y,
                                          int tile, unsigned* wait_ctr, unsigned* arrive_ctr,
                                          float* smem) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i = lane & 15, h = lane >> 4;
  const f32x4* wp = reinterpret_cast<const f32x4*>(wpk) + ((int64_t)tile * NCH) * 64 + lane;
  f32x4 wv[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) wv[u] = wp[(int64_t)(wave * PER + u) * 64];
  if constexpr (FUSED) {
    if (wait_ctr) {
      if (tid == 0) {
        long spins = 0;
        while (__hip_atomic_load(wait_ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < TILES &&
               ++spins < (1L << 26))
          __builtin_amdgcn_s_sleep(1);
      }
      __syncthreads();
    }
  }
  // activations: row i, k = (wave*PER + u)*16 + 4h .. +3
  f32x4 xv[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const float* xp = x + i * KD + (wave * PER + u) * 16 + 4 * h;
    if constexpr (FUSED) {
#pragma unroll
      for (int e = 0; e < 4; ++e) xv[u][e] = ld_sc1(xp + e);
    } else {
      xv[u] = *reinterpret_cast<const f32x4*>(xp);
    }
  }
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
#pragma unroll
  for (int u = 0; u < PER; ++u)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (u & 1) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[u][e], xv[u][e], acc1, 0, 0, 0);
      else acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[u][e], xv[u][e], acc0, 0, 0, 0);
    }
  reinterpret_cast<f32x4*>(smem)[wave * 64 + lane] = acc0 + acc1;
  __syncthreads();
  if (wave == 0) {
    f32x4 s = reinterpret_cast<f32x4*>(smem)[lane];
#pragma unroll
    for (int w = 1; w < 8; ++w) s += reinterpret_cast<f32x4*>(smem)[w * 64 + lane];
    // D[row = W row n (4h + r), col = x row m (i)]
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float v = tanhf(s[r]) + 0.5f;
      float* yp = y + i * ND + tile * 16 + 4 * h + r;
      if constexpr (FUSED) st_sc1(yp, v);
      else *yp = v;
    }
    if constexpr (FUSED) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  if constexpr (FUSED) {
    __syncthreads();
    if (tid == 0) __hip_atomic_fetch_add(arrive_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ __launch_bounds__(512) void phase_kernel(const float* wpk, const float* x, float* y) {
  __shared__ __attribute__((aligned(16))) float smem[8 * 256];
  gemv_tile<false>(wpk, x, y, blockIdx.x, nullptr, nullptr, smem);
}

__global__ __launch_bounds__(512) void fused_kernel(const float* wpk, float* xa, float* xb,
                                                    unsigned* ctr) {
  __shared__ __attribute__((aligned(16))) float smem[8 * 256];
  const int p = blockIdx.x / TILES, tile = blockIdx.x % TILES;
  const float* x = (p & 1) ? xb : xa;
  float* y = (p & 1) ? xa : xb;
  gemv_tile<true>(wpk + (int64_t)p * TILES * NCH * 256, x, y, tile, p ? ctr + p - 1 : nullptr,
                  ctr + p, smem);
}

int main() {
  const int P = 48;
  float *W, *xa, *xb, *x0;
  unsigned* ctr;
  const size_t wel = (size_t)P * TILES * NCH * 256;
  (void)hipMalloc(&W, wel * 4);
  (void)hipMalloc(&xa, ROWS * KD * 4);
  (void)hipMalloc(&xb, ROWS * KD * 4);
  (void)hipMalloc(&x0, ROWS * KD * 4);
  (void)hipMalloc(&ctr, P * 4);
  {
    std::vector<float> h(wel);
    uint32_t s = 1;
    for (auto& v : h) {
      s = s * 1664525u + 1013904223u;
      v = ((s >> 9) * (1.0f / 8388608.0f) - 0.5f) * 0.1f;
    }
    (void)hipMemcpy(W, h.data(), wel * 4, hipMemcpyHostToDevice);
    std::vector<float> hx(ROWS * KD);
    for (auto& v : hx) {
      s = s * 1664525u + 1013904223u;
      v = (s >> 9) * (1.0f / 8388608.0f);
    }
    (void)hipMemcpy(x0, hx.data(), hx.size() * 4, hipMemcpyHostToDevice);
  }
  hipStream_t st;
  (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  auto launches = [&]() {
    (void)hipMemcpyAsync(xa, x0, ROWS * KD * 4, hipMemcpyDeviceToDevice, st);
    for (int p = 0; p < P; ++p)
      hipLaunchKernelGGL(phase_kernel, dim3(TILES), dim3(512), 0, st,
                         W + (size_t)p * TILES * NCH * 256, (p & 1) ? xb : xa, (p & 1) ? xa : xb);
  };
  auto fused = [&]() {
    (void)hipMemcpyAsync(xa, x0, ROWS * KD * 4, hipMemcpyDeviceToDevice, st);
    (void)hipMemsetAsync(ctr, 0, P * 4, st);
    hipLaunchKernelGGL(fused_kernel, dim3(TILES * P), dim3(512), 0, st, W, xa, xb, ctr);
  };
  auto timeit = [&](const char* name, auto&& body) {
    hipGraph_t g;
    hipGraphExec_t e;
    (void)hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal);
    for (int r = 0; r < 10; ++r) body();
    (void)hipStreamEndCapture(st, &g);
    (void)hipGraphInstantiate(&e, g, nullptr, nullptr, 0);
    (void)hipGraphLaunch(e, st);
    (void)hipStreamSynchronize(st);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      (void)hipEventRecord(a, st);
      (void)hipGraphLaunch(e, st);
      (void)hipEventRecord(b, st);
      (void)hipEventSynchronize(b);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, a, b);
      best = std::min(best, ms);
    }
    printf("%-10s %7.2f us per phase (%d phases x 10 chains)\n", name, best * 1e3 / (10 * P), P);
    std::vector<float> out(ROWS * KD);
    (void)hipMemcpy(out.data(), (P & 1) ? xb : xa, out.size() * 4, hipMemcpyDeviceToHost);
    return out;
  };
  auto r1 = timeit("launches", launches);
  auto r2 = timeit("fused", fused);
  double md = 0;
  for (size_t i = 0; i < r1.size(); ++i) md = std::max(md, (double)fabs(r1[i] - r2[i]));
  printf("max |fused - launches| = %g  (%s)\n", md, hipGetErrorString(hipGetLastError()));
  return 0;
}
