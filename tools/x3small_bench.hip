// x3small_bench.hip — split-bf16 GEMM tiles for under-filled launches (development aid): the
// one-batch T5 encoder projections (M = 16 x ~90 rows) and the one-batch ViT / text problems,
// 64x128 (the default below 160 128x128 blocks) against 64x64 tiles; device time per launch (graph
// of 100 launches) and a bitwise check that the outputs are identical (same k order per tile).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/x3small_bench.hip -o tools/x3small_bench \
//          -Lmultimodalpromptretrieval_amd -lmpr -Wl,-rpath,'$ORIGIN/../multimodalpromptretrieval_amd'
#include <cstdio>
#include <cstring>
#include <functional>
#include <vector>

#include "../multimodalpromptretrieval_amd/csrc/gemm.hip"  // the rest links from libmpr.so

using namespace mpr;

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
  return ms * 1e3 / n;
}

int main() {
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  float *A, *W, *C, *C2;
  const size_t bytes = 64 << 20;
  (void)hipMalloc(&A, bytes);
  (void)hipMalloc(&W, bytes);
  (void)hipMalloc(&C, bytes);
  (void)hipMalloc(&C2, bytes);
  {
    std::vector<float> h(bytes / 4);
    uint32_t x = 7u;
    for (auto& v : h) {
      x = x * 1664525u + 1013904223u;
      v = ((x >> 9) * (1.0f / 8388608.0f)) - 0.5f;
    }
    (void)hipMemcpy(A, h.data(), bytes, hipMemcpyHostToDevice);
    (void)hipMemcpy(W, h.data(), bytes, hipMemcpyHostToDevice);
  }
  struct Shape { const char* name; int M, N, K, n; };
  const Shape shapes[] = {
      {"t5 qkv 1440x1536x512", 1440, 1536, 512, 1}, {"t5 o 1440x512x512", 1440, 512, 512, 1},
      {"t5 wi 1440x2048x512", 1440, 2048, 512, 1},  {"t5 wo 1440x512x2048", 1440, 512, 2048, 1},
      {"t5 crosskv 1440x6144x512", 1440, 6144, 512, 1},
      {"vit out 800x768x768 x2", 800, 768, 768, 2},  {"vit fc2 800x768x3072 x2", 800, 768, 3072, 2},
      {"vit qkv 800x2304x768 x2", 800, 2304, 768, 2}, {"vit fc1 800x3072x768 x2", 800, 3072, 768, 2},
      {"vit qkv 1600x2304x768 x2", 1600, 2304, 768, 2},
      {"vit fc1 1600x3072x768 x2", 1600, 3072, 768, 2},
      {"t5 wi 5760x2048x512", 5760, 2048, 512, 1}, {"t5 qkv 5760x1536x512", 5760, 1536, 512, 1},
  };
  using L = std::function<int(const GemmGroup&, hipStream_t)>;
  struct Var { const char* name; L fn; };
  const Var vars[] = {
      {"64x128 k32 (TALL)", launch_gemm_x3_group<64, 128, 1, 1, 32, 2, 1>},
      {"128x128 2x1 k16 prio (WIDE)", launch_gemm_x3_group<128, 128, 2, 1, 16, 2, 1, 2>},
      {"64x64 k32", launch_gemm_x3_group<64, 64, 1, 1, 32, 2, 1>},
      {"64x64 k16", launch_gemm_x3_group<64, 64, 1, 1, 16, 2, 1>},
      {"32x64 k32", launch_gemm_x3_group<32, 64, 1, 1, 32, 2, 1>},
      {"64x32 k32", launch_gemm_x3_group<64, 32, 1, 1, 32, 2, 1>},
      {"128x128 2x2 4w k16", launch_gemm_x3_group<128, 128, 2, 2, 16, 2, 1>},
      {"128x128 2x2 4w k16 prio", launch_gemm_x3_group<128, 128, 2, 2, 16, 2, 1, 2>},
      {"128x128 2x2 4w k32 prio", launch_gemm_x3_group<128, 128, 2, 2, 32, 2, 1, 2>},
  };
  for (const Shape& sh : shapes) {
    GemmGroup G;
    G.n = sh.n;
    for (int i = 0; i < sh.n; ++i) {
      GemmArgs& g = G.g[i];
      const size_t off = (size_t)i * (6 << 20);
      g.A = A + off; g.lda = sh.K; g.W = W + off; g.ldw = sh.K; g.C = C + off; g.ldc = sh.N;
      g.M = sh.M; g.N = sh.N; g.K = sh.K;
    }
    const double gf = 2.0 * sh.n * sh.M * sh.N * sh.K * 1e-9;
    printf("%s (%.2f GFLOP)\n", sh.name, gf);
    std::vector<float> ref((size_t)sh.M * sh.N), out(ref.size());
    bool first = true;
    for (const Var& v : vars) {
      GemmGroup H = G;
      for (int i = 0; i < sh.n; ++i) H.g[i].C = (first ? C : C2) + (size_t)i * (6 << 20);
      const double us = time_graph(s, [&]() { v.fn(H, s); }, 100);
      (void)hipStreamSynchronize(s);
      (void)hipMemcpy(first ? ref.data() : out.data(), H.g[0].C, ref.size() * 4,
                      hipMemcpyDeviceToHost);
      const bool same = first || memcmp(ref.data(), out.data(), ref.size() * 4) == 0;
      printf("   %-30s %8.2f us  %6.1f TF/s  %s\n", v.name, us, gf / us * 1e3,
             same ? "" : "DIFFERS");
      first = false;
    }
  }
  return 0;
}
