// mfma_rate.hip — sustained MFMA issue rate on the whole chip (development aid): every wave runs
// ITER x 4 independent accumulator chains of one MFMA shape, no memory traffic in the loop.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mfma_rate.hip -o tools/mfma_rate
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int ITER = 4096;

__global__ void k32x32x2(float* out, float seed) {
  f32x16 acc[4] = {};
  float a = seed * threadIdx.x, b = seed + threadIdx.x;
  for (int i = 0; i < ITER; ++i)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[c], 0, 0, 0);
  float s = 0;
  for (int c = 0; c < 4; ++c)
    for (int r = 0; r < 16; ++r) s += acc[c][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k16x16x4(float* out, float seed) {
  f32x4 acc[4] = {};
  float a = seed * threadIdx.x, b = seed + threadIdx.x;
  for (int i = 0; i < ITER; ++i)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[c], 0, 0, 0);
  float s = 0;
  for (int c = 0; c < 4; ++c)
    for (int r = 0; r < 4; ++r) s += acc[c][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void kbf16(float* out, float seed) {
  f32x16 acc[4] = {};
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (__bf16)(seed * (threadIdx.x + j));
    b[j] = (__bf16)(seed + threadIdx.x - j);
  }
  for (int i = 0; i < ITER; ++i)
#pragma unroll
    for (int c = 0; c < 4; ++c)
      acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[c], 0, 0, 0);
  float s = 0;
  for (int c = 0; c < 4; ++c)
    for (int r = 0; r < 16; ++r) s += acc[c][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename F>
static void run(const char* name, F kern, double flop_per_mfma, int waves_per_simd, float* out) {
  const int blocks = 256 * waves_per_simd;  // 256 threads = one wave per SIMD per block
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 1e-3f);
  (void)hipEventRecord(a, 0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 1e-3f);
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  const double mfmas = 5.0 * blocks * 4 * ITER * 4;  // launches x waves x ITER x chains
  const double ns_per = ms * 1e6 / (mfmas / (256.0 * 4));  // per SIMD
  printf("%-22s waves/SIMD %d  %8.3f ms  %7.1f TFLOP/s  %6.2f ns per MFMA per SIMD\n", name,
         waves_per_simd, ms / 5, mfmas * flop_per_mfma / (ms * 1e-3) * 1e-12, ns_per);
}

int main() {
  float* out;
  (void)hipMalloc(&out, 64 << 20);
  for (int w = 1; w <= 4; w *= 2) {
    run("mfma_f32_32x32x2f32", k32x32x2, 32.0 * 32 * 2 * 2, w, out);
    run("mfma_f32_16x16x4f32", k16x16x4, 16.0 * 16 * 4 * 2, w, out);
    run("mfma_f32_32x32x16_bf16", kbf16, 32.0 * 32 * 16 * 2, w, out);
  }
  return 0;
}
