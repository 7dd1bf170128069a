// gbench.hip — tile/variant sweep of libmpr's fp32 MFMA GEMM on the ViT/T5 projection shapes
// (development aid; includes the library sources so the kernel templates are visible).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/gbench.hip -o tools/gbench
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <functional>

#include "../multimodalpromptretrieval_amd/csrc/api.hip"
#include "../multimodalpromptretrieval_amd/csrc/encoders.hip"
#include "../multimodalpromptretrieval_amd/csrc/gemm.hip"
#include "../multimodalpromptretrieval_amd/csrc/layers.hip"
#include "../multimodalpromptretrieval_amd/csrc/scan.hip"
#include "../multimodalpromptretrieval_amd/csrc/t5.hip"

using namespace mpr;

// average device time per launch over a captured chain of n launches (graph removes CPU gaps)
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
  (void)hipGraphExecDestroy(e);
  (void)hipGraphDestroy(g);
  return ms * 1e3 / n;
}

// usage: gbench [shape variant groups]  (indices into the tables below; default: all)
int main(int argc, char** argv) {
  const int only_shape = argc > 1 ? atoi(argv[1]) : -1;
  const int only_var = argc > 2 ? atoi(argv[2]) : -1;
  const int only_grp = argc > 3 ? atoi(argv[3]) : -1;
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  float *A, *W, *C, *R;
  const size_t bytes = 128 << 20;
  (void)hipMalloc(&A, bytes);
  (void)hipMalloc(&W, bytes);
  (void)hipMalloc(&C, bytes);
  (void)hipMalloc(&R, bytes);
  {  // random operands (zero data runs at a higher clock and reads high)
    std::vector<float> h(bytes / 4);
    uint32_t x = 12345u;
    for (auto& v : h) {
      x = x * 1664525u + 1013904223u;
      v = ((x >> 9) * (1.0f / 8388608.0f)) - 0.5f;
    }
    (void)hipMemcpy(A, h.data(), bytes, hipMemcpyHostToDevice);
    (void)hipMemcpy(W, h.data() + 7, bytes - 64, hipMemcpyHostToDevice);
    (void)hipMemcpy(R, h.data() + 3, bytes - 64, hipMemcpyHostToDevice);
  }
  struct Shape { const char* name; int M, N, K; bool res; };
  const Shape shapes[] = {
      {"vit qkv  1600x2304x768", 1600, 2304, 768, false},
      {"vit out  1600x768x768 +R", 1600, 768, 768, true},
      {"vit fc1  1600x3072x768", 1600, 3072, 768, false},
      {"vit fc2  1600x768x3072 +R", 1600, 768, 3072, true},
      {"vit qkv   800x2304x768", 800, 2304, 768, false},
      {"vit fc1   800x3072x768", 800, 3072, 768, false},
      {"vit out   800x768x768 +R", 800, 768, 768, true},
      {"vit fc2   800x768x3072 +R", 800, 768, 3072, true},
      {"txt fc2   384x512x2048 +R", 384, 512, 2048, true},
  };
  using L = std::function<int(const GemmGroup&, hipStream_t)>;
  struct Var { const char* name; L fn; };
  const Var vars[] = {
      {"64x64 k32 D2 XR", launch_gemm_group<64, 64, 1, 1, 32, 2, 1, true>},
      {"32x32 k64 D2 W4", launch_gemm_group<32, 32, 1, 1, 64, 2, 4>},
      {"128x64 2x1/w k32 D2 XR", launch_gemm_group<128, 64, 2, 1, 32, 2, 1, true>},
      {"64x128 1x2/w k32 D2 XR", launch_gemm_group<64, 128, 1, 2, 32, 2, 1, true>},
      {"128x128 2x2/w k32 D2 XR", launch_gemm_group<128, 128, 2, 2, 32, 2, 1, true>},
      {"64x64 1x2/w k32 D2 W2 XR", launch_gemm_group<64, 64, 1, 2, 32, 2, 2, true>},
      {"32x64 k64 D2 W2", launch_gemm_group<32, 64, 1, 1, 64, 2, 2>},
      // bit-identical to "32x32 k64 D2 W4" (same per-wave K slices and reduction order)
      {"64x64 k64 D2 W4", launch_gemm_group<64, 64, 1, 1, 64, 2, 4>},
      {"64x64 k64 D2 W4 XR", launch_gemm_group<64, 64, 1, 1, 64, 2, 4, true>},
      {"64x32 k64 D2 W4", launch_gemm_group<64, 32, 1, 1, 64, 2, 4>},
      {"32x64 k64 D2 W4", launch_gemm_group<32, 64, 1, 1, 64, 2, 4>},
      {"32x32 k64 D2 W4 XR", launch_gemm_group<32, 32, 1, 1, 64, 2, 4, true>},
  };
  int si = -1;
  for (const Shape& sh : shapes) {
    if (++si, only_shape >= 0 && si != only_shape) continue;
    for (int grp = 1; grp <= 2; ++grp) {
      if (only_grp > 0 && grp != only_grp) continue;
      const double gf = grp * 2.0 * sh.M * sh.N * sh.K * 1e-9;
      printf("%s x%d (%.2f GFLOP)\n", sh.name, grp, gf);
      int vi = -1;
      for (const Var& v : vars) {
        if (++vi, only_var >= 0 && vi != only_var) continue;
        GemmGroup G;
        G.n = grp;
        for (int i = 0; i < grp; ++i) {
          GemmArgs& g = G.g[i];
          const size_t off = (size_t)i * (8 << 20);
          g.A = A + off; g.lda = sh.K; g.W = W + off; g.ldw = sh.K; g.C = C + off; g.ldc = sh.N;
          g.M = sh.M; g.N = sh.N; g.K = sh.K;
          if (sh.res) { g.R = R + off; g.ldr = sh.N; }
        }
        const double us = time_graph(s, [&]() { v.fn(G, s); }, 100);
        printf("   %-18s %8.2f us  %6.1f TF/s\n", v.name, us, gf / us * 1e3);
      }
    }
  }
  // bit-identity of the K-split-by-4 tiles (32x32 W4 vs the larger W4 blocks) on two shapes
  float* C2;
  (void)hipMalloc(&C2, bytes);
  const int same_a = 1, same_b[] = {7, 8, 9, 10, 11};
  for (int shi : {1, 3, 6, 7, 8}) {
    const Shape& sh = shapes[shi];
    GemmGroup G;
    G.n = 1;
    GemmArgs& g = G.g[0];
    g.A = A; g.lda = sh.K; g.W = W; g.ldw = sh.K; g.ldc = sh.N;
    g.M = sh.M; g.N = sh.N; g.K = sh.K;
    if (sh.res) { g.R = R; g.ldr = sh.N; }
    g.C = C;
    vars[same_a].fn(G, s);
    (void)hipStreamSynchronize(s);  // s is non-blocking: hipMemcpy would not wait for it
    std::vector<float> h1((size_t)sh.M * sh.N), h2(h1.size());
    (void)hipMemcpy(h1.data(), C, h1.size() * 4, hipMemcpyDeviceToHost);
    for (int vb : same_b) {
      g.C = C2;
      (void)hipMemsetAsync(C2, 0, h1.size() * 4, s);  // ordered before the kernel on s
      vars[vb].fn(G, s);
      (void)hipStreamSynchronize(s);
      (void)hipMemcpy(h2.data(), C2, h2.size() * 4, hipMemcpyDeviceToHost);
      printf("identity %s: %s vs %s: %s\n", sh.name, vars[same_a].name, vars[vb].name,
             memcmp(h1.data(), h2.data(), h1.size() * 4) == 0 ? "bit-identical" : "DIFFERENT");
    }
  }
  return 0;
}
