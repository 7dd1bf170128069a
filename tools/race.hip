// race.hip — determinism stress of the encoder kernels: the same launch repeated, outputs compared
// bitwise against the first run (debugging aid).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/race.hip -o tools/race
#include <cstdio>
#include <cstring>
#include <functional>
#include <vector>

#include "../multimodalpromptretrieval_amd/csrc/api.hip"
#include "../multimodalpromptretrieval_amd/csrc/encoders.hip"
#include "../multimodalpromptretrieval_amd/csrc/gemm.hip"
#include "../multimodalpromptretrieval_amd/csrc/layers.hip"
#include "../multimodalpromptretrieval_amd/csrc/scan.hip"
#include "../multimodalpromptretrieval_amd/csrc/t5.hip"

using namespace mpr;

static float* dev_rand(size_t n, uint32_t seed, float scale = 1.f) {
  std::vector<float> h(n);
  for (auto& v : h) {
    seed = seed * 1664525u + 1013904223u;
    v = scale * (((seed >> 9) * (1.0f / 8388608.0f)) - 0.5f);
  }
  float* d;
  (void)hipMalloc(&d, n * 4);
  (void)hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice);
  return d;
}

static void stress(const char* name, const float* out, size_t n, int reps,
                   const std::function<void()>& f) {
  std::vector<float> ref(n), cur(n);
  f();
  (void)hipDeviceSynchronize();
  (void)hipMemcpy(ref.data(), out, n * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int r = 0; r < reps; ++r) {
    f();
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(cur.data(), out, n * 4, hipMemcpyDeviceToHost);
    if (memcmp(ref.data(), cur.data(), n * 4) != 0) ++bad;
  }
  printf("%-40s %4d / %d runs differ\n", name, bad, reps);
  fflush(stdout);
}

int main() {
  const int M = 800, W = 768, REPS = 300;
  float* A = dev_rand((size_t)M * 4 * W, 1);
  float* Wq = dev_rand((size_t)3 * W * W, 2, 0.07f);
  float* Wo = dev_rand((size_t)W * W, 3, 0.05f);
  float* W1 = dev_rand((size_t)4 * W * W, 4, 0.05f);
  float* W2 = dev_rand((size_t)4 * W * W, 5, 0.02f);
  float* bias = dev_rand(4 * W, 6, 0.1f);
  float* C = dev_rand((size_t)M * 4 * W, 7);
  float* C2 = dev_rand((size_t)M * 4 * W, 8);
  float* R = dev_rand((size_t)M * W, 9);
  auto mk = [&](const float* Wt, int N, int K, float* Cout, bool res) {
    GemmArgs g;
    g.A = A; g.lda = K; g.W = Wt; g.ldw = K; g.bias = bias; g.C = Cout; g.ldc = N;
    g.M = M; g.N = N; g.K = K;
    if (res) { g.R = R; g.ldr = N; }
    return g;
  };
  auto one = [&](GemmArgs g) { GemmGroup gg; gg.n = 1; gg.g[0] = g; return gg; };
  auto two = [&](GemmArgs g, GemmArgs h) { GemmGroup gg; gg.n = 2; gg.g[0] = g; gg.g[1] = h; return gg; };
  GemmArgs q = mk(Wq, 3 * W, W, C, false), q2 = mk(Wq, 3 * W, W, C2, false);
  GemmArgs o = mk(Wo, W, W, C, true), o2 = mk(Wo, W, W, C2, true);
  GemmArgs f1 = mk(W1, 4 * W, W, C, false), f1b = mk(W1, 4 * W, W, C2, false);
  f1.act = f1b.act = ACT_QUICKGELU;
  GemmArgs f2 = mk(W2, W, 4 * W, C, true), f2b = mk(W2, W, 4 * W, C2, true);
  stress("qkv single (64x64)", C, (size_t)M * 3 * W, REPS, [&] { gemm_group(one(q), nullptr); });
  stress("qkv pair (64x64)", C2, (size_t)M * 3 * W, REPS, [&] { gemm_group(two(q, q2), nullptr); });
  stress("qkv pair (64x64, no XCD remap)", C2, (size_t)M * 3 * W, REPS,
         [&] { launch_gemm_group<64, 64, 1, 1, 32, 2, 1, false>(two(q, q2), nullptr); });
  stress("qkv pair (64x64, remap)", C2, (size_t)M * 3 * W, REPS,
         [&] { launch_gemm_group<64, 64, 1, 1, 32, 2, 1, true>(two(q, q2), nullptr); });
  stress("qkv pair (64x64, remap) p0", C, (size_t)M * 3 * W, REPS,
         [&] { launch_gemm_group<64, 64, 1, 1, 32, 2, 1, true>(two(q, q2), nullptr); });
  stress("fc1 single (64x64 gelu)", C, (size_t)M * 4 * W, REPS, [&] { gemm_group(one(f1), nullptr); });
  stress("fc1 pair (64x64 gelu, no remap)", C2, (size_t)M * 4 * W, REPS,
         [&] { launch_gemm_group<64, 64, 1, 1, 32, 2, 1, false>(two(f1, f1b), nullptr); });
  stress("out single (32x32 W4)", C, (size_t)M * W, REPS, [&] { gemm_group(one(o), nullptr); });
  stress("out pair (32x32 W4)", C2, (size_t)M * W, REPS, [&] { gemm_group(two(o, o2), nullptr); });
  stress("fc1 pair (64x64 gelu)", C2, (size_t)M * 4 * W, REPS, [&] { gemm_group(two(f1, f1b), nullptr); });
  stress("fc2 single (32x32 W4, K3072)", C, (size_t)M * W, REPS, [&] { gemm_group(one(f2), nullptr); });
  stress("fc2 pair (32x32 W4, K3072)", C2, (size_t)M * W, REPS, [&] { gemm_group(two(f2, f2b), nullptr); });
  // attention (ViT shape) and LayerNorm
  float* qkv = dev_rand((size_t)M * 3 * W, 10, 2.f);
  float* ao = dev_rand((size_t)M * W, 11);
  AttnArgs at;
  at.q = qkv; at.q_bs = (int64_t)50 * 3 * W; at.q_rs = 3 * W;
  at.k = qkv + W; at.k_bs = at.q_bs; at.k_rs = 3 * W;
  at.v = qkv + 2 * W; at.v_bs = at.q_bs; at.v_rs = 3 * W;
  at.o = ao; at.o_bs = (int64_t)50 * W; at.o_rs = W;
  at.B = 16; at.H = 12; at.Lq = 50; at.Lk = 50; at.scale = 0.125f;
  stress("attention mfma (ViT)", ao, (size_t)M * W, REPS, [&] { attention(at, nullptr); });
  float* g = dev_rand(W, 12);
  float* lo = dev_rand((size_t)M * W, 13);
  stress("layernorm 800x768", lo, (size_t)M * W, REPS,
         [&] { layernorm(R, W, M, W, g, bias, 1e-5f, lo, W, nullptr); });
  return 0;
}
