// x3bench.hip — the split-bf16 ("x3") fp32 GEMM against the f32-MFMA GEMM on the tower shapes:
// device time per launch (graph of 100 launches) and max error against an fp64 host product,
// relative to sum_k |a_k b_k| of the element (development aid).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/x3bench.hip -o tools/x3bench \
//          -Lmultimodalpromptretrieval_amd -lmpr -Wl,-rpath,'$ORIGIN/../multimodalpromptretrieval_amd'
#include <cmath>
#include <cstdio>
#include <cstdlib>
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
  (void)hipGraphExecDestroy(e);
  (void)hipGraphDestroy(g);
  return ms * 1e3 / n;
}

int main(int argc, char** argv) {
  const int only_shape = argc > 1 ? atoi(argv[1]) : -1;
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  float *A, *W, *C, *R;
  const size_t bytes = 96 << 20;
  (void)hipMalloc(&A, bytes);
  (void)hipMalloc(&W, bytes);
  (void)hipMalloc(&C, bytes);
  (void)hipMalloc(&R, bytes);
  std::vector<float> hA(bytes / 4), hW(bytes / 4);
  {
    uint32_t x = 12345u;
    for (auto& v : hA) {
      x = x * 1664525u + 1013904223u;
      v = ((x >> 9) * (1.0f / 8388608.0f)) - 0.5f;
    }
    for (auto& v : hW) {
      x = x * 1664525u + 1013904223u;
      v = (((x >> 9) * (1.0f / 8388608.0f)) - 0.5f) * 0.05f;
    }
    (void)hipMemcpy(A, hA.data(), bytes, hipMemcpyHostToDevice);
    (void)hipMemcpy(W, hW.data(), bytes, hipMemcpyHostToDevice);
    (void)hipMemset(R, 0, bytes);
  }
  struct Shape { const char* name; int M, N, K; };
  const Shape shapes[] = {
      {"vit qkv  1600x2304x768", 1600, 2304, 768},
      {"vit out  1600x768x768", 1600, 768, 768},
      {"vit fc1  1600x3072x768", 1600, 3072, 768},
      {"vit fc2  1600x768x3072", 1600, 768, 3072},
      {"vit qkv   800x2304x768", 800, 2304, 768},
      {"vit fc2   800x768x3072", 800, 768, 3072},
  };
  using L = std::function<int(const GemmGroup&, hipStream_t)>;
  struct Var { const char* name; L fn; };
  const Var vars[] = {
      {"f32 64x64 k32 D2 XR", launch_gemm_group<64, 64, 1, 1, 32, 2, 1, true>},
      {"f32 64x32 k64 W4", launch_gemm_group<64, 32, 1, 1, 64, 2, 4>},
      {"x3 64x64 k16 D2", launch_gemm_x3_group<64, 64, 1, 1, 16, 2, 1>},
      {"x3 128x128 2x2 k16", launch_gemm_x3_group<128, 128, 2, 2, 16, 2, 1>},
      {"x3 128x128 2x1 8w k16 D2", launch_gemm_x3_group<128, 128, 2, 1, 16, 2, 1>},
      {"x3 128x128 2x1 8w k16 D3", launch_gemm_x3_group<128, 128, 2, 1, 16, 3, 1>},
      {"x3 128x128 2x1 k16 ilv", launch_gemm_x3_group<128, 128, 2, 1, 16, 2, 1, 1>},
      {"x3 128x128 2x1 k16 prio", launch_gemm_x3_group<128, 128, 2, 1, 16, 2, 1, 2>},
      {"x3 128x128 2x1 k16 ilv+prio", launch_gemm_x3_group<128, 128, 2, 1, 16, 2, 1, 3>},
      {"x3 64x128 k32 ilv", launch_gemm_x3_group<64, 128, 1, 1, 32, 2, 1, 1>},
      {"x3 64x128 k32 prio", launch_gemm_x3_group<64, 128, 1, 1, 32, 2, 1, 2>},
      {"x3 64x64 k16 prio", launch_gemm_x3_group<64, 64, 1, 1, 16, 2, 1, 2>},
      {"x3 128x64 1x1 8w k32 D2", launch_gemm_x3_group<128, 64, 1, 1, 32, 2, 1>},
      {"x3 64x128 1x1 8w k32 D2", launch_gemm_x3_group<64, 128, 1, 1, 32, 2, 1>},
      {"x3 128x64 2x1 4w k16 D2", launch_gemm_x3_group<128, 64, 2, 1, 16, 2, 1>},
      {"x3 128x128 2x1 8w k32 D2", launch_gemm_x3_group<128, 128, 2, 1, 32, 2, 1>},
      {"x3 128x128 2x2 4w k32 D2", launch_gemm_x3_group<128, 128, 2, 2, 32, 2, 1>},
      {"x3 128x256 2x2 8w k16 D2", launch_gemm_x3_group<128, 256, 2, 2, 16, 2, 1>},
  };
  int si = -1;
  for (const Shape& sh : shapes) {
    if (++si, only_shape >= 0 && si != only_shape) continue;
    for (int grp = 2; grp <= 4; grp += 2) {
      double gf = 2.0 * 2.0 * sh.M * sh.N * sh.K * 1e-9;
      if (grp == 4)
        gf += 2.0 * 704 * (sh.N == 768 ? 512 : sh.N == 2304 ? 1536 : 2048) *
              (sh.K == 768 ? 512 : 2048) * 1e-9;
      printf("%s x%d (%.2f GFLOP)\n", sh.name, grp, gf);
      for (const Var& v : vars) {
        GemmGroup G;
        G.n = grp;
        for (int i = 0; i < grp; ++i) {
          GemmArgs& g = G.g[i];
          const size_t off = (size_t)i * (6 << 20);
          g.A = A + off; g.lda = sh.K; g.W = W + off; g.ldw = sh.K; g.C = C + off; g.ldc = sh.N;
          g.M = sh.M; g.N = sh.N; g.K = sh.K; g.R = R + off; g.ldr = sh.N;
          if (i >= 2) {  // the text tower's problems of the same layer: 2 runs of 16 x 22 tokens
            g.M = 352; g.N = sh.N == 768 ? 512 : sh.N == 2304 ? 1536 : 2048;
            g.K = sh.K == 768 ? 512 : 2048; g.lda = g.K; g.ldw = g.K; g.ldc = g.N; g.ldr = g.N;
          }
        }
        const double us = time_graph(s, [&]() { v.fn(G, s); }, 100);
        // accuracy of problem 0 on sampled elements
        (void)hipStreamSynchronize(s);
        std::vector<float> hc((size_t)sh.M * sh.N);
        (void)hipMemcpy(hc.data(), C, hc.size() * 4, hipMemcpyDeviceToHost);
        double worst = 0;
        for (int t = 0; t < 4096; ++t) {
          const int m = (t * 7919) % sh.M, n = (t * 104729) % sh.N;
          double ref = 0, mag = 0;
          for (int k = 0; k < sh.K; ++k) {
            const double p = (double)hA[(size_t)m * sh.K + k] * hW[(size_t)n * sh.K + k];
            ref += p;
            mag += fabs(p);
          }
          worst = std::max(worst, fabs(hc[(size_t)m * sh.N + n] - ref) / mag);
        }
        printf("   %-24s %8.2f us  %6.1f TF/s   err %.2e\n", v.name, us, gf / us * 1e3, worst);
      }
    }
  }
  return 0;
}
