// gbench.hip — tile/variant sweep of libmpr's fp32 MFMA GEMM on the ViT/T5 projection shapes
// (development aid; includes the library sources so the kernel templates are visible).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/gbench.hip -o tools/gbench
#include <cstdio>
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

int main() {
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  float *A, *W, *C;
  (void)hipMalloc(&A, 64 << 20);
  (void)hipMalloc(&W, 64 << 20);
  (void)hipMalloc(&C, 64 << 20);
  (void)hipMemset(A, 0, 64 << 20);
  (void)hipMemset(W, 0, 64 << 20);
  struct Shape { const char* name; int M, N, K; };
  const Shape shapes[] = {
      {"vit qkv   800x2304x768", 800, 2304, 768},  {"vit out   800x768x768", 800, 768, 768},
      {"vit fc1   800x3072x768", 800, 3072, 768},  {"vit fc2   800x768x3072", 800, 768, 3072},
      {"t5e qkv  1136x1536x512", 1136, 1536, 512}, {"t5e wo   1136x512x2048", 1136, 512, 2048},
      {"sq 2048", 2048, 2048, 2048},
  };
  using L = std::function<int(const GemmArgs&, hipStream_t)>;
  struct Var { const char* name; L fn; int bm, bn; };
  const Var vars[] = {
      {"64x64 1x1", launch_gemm<64, 64, 1, 1>, 64, 64},
      {"32x64 1x1", launch_gemm<32, 64, 1, 1>, 32, 64},
      {"128x64 2x1", launch_gemm<128, 64, 2, 1>, 128, 64},
      {"128x128 2x2", launch_gemm<128, 128, 2, 2>, 128, 128},
  };
  for (const Shape& sh : shapes) {
    const double gf = 2.0 * sh.M * sh.N * sh.K * 1e-9;
    printf("%s  (%.2f GFLOP)\n", sh.name, gf);
    for (const Var& v : vars) {
      const int64_t tiles = cdiv(sh.M, v.bm) * cdiv(sh.N, v.bn);
      GemmArgs g;
      g.A = A; g.lda = sh.K; g.W = W; g.ldw = sh.K; g.C = C; g.ldc = sh.N;
      g.M = sh.M; g.N = sh.N; g.K = sh.K;
      const double us = time_graph(s, [&]() { v.fn(g, s); }, 200);
      printf("   %-22s blocks %5lld  %8.2f us  %6.1f TF/s\n", v.name, (long long)tiles, us,
             gf / us * 1e3);
    }
  }
  return 0;
}
