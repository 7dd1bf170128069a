// x3pbench.hip — the packed-W split-bf16 GEMM (gemm_x3p) against the LDS-staged one (gemm_x3) on
// the tower shapes: device time per launch (graph of 100 launches) and bitwise equality of the
// outputs (development aid).  usage: x3pbench [shape substring] [variant substring] [launches]
// (a filtered run of one shape / variant for PMC passes).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/x3pbench.hip -o tools/x3pbench \
//          -Lmultimodalpromptretrieval_amd -lmpr -Wl,-rpath,'$ORIGIN/../multimodalpromptretrieval_amd'
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
  const char* fshape = argc > 1 ? argv[1] : "";
  const char* fvar = argc > 2 ? argv[2] : "";
  const int nl = argc > 3 ? atoi(argv[3]) : 100;
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  const size_t bytes = 96 << 20;
  float *A, *W, *C, *C2, *R;
  void* P;
  (void)hipMalloc(&A, bytes);
  (void)hipMalloc(&W, bytes);
  (void)hipMalloc(&C, bytes);
  (void)hipMalloc(&C2, bytes);
  (void)hipMalloc(&R, bytes);
  (void)hipMalloc(&P, 2 * bytes);
  {
    std::vector<float> h(bytes / 4);
    uint32_t x = 12345u;
    for (auto& v : h) {
      x = x * 1664525u + 1013904223u;
      v = ((x >> 9) * (1.0f / 8388608.0f)) - 0.5f;
    }
    (void)hipMemcpy(A, h.data(), bytes, hipMemcpyHostToDevice);
    for (auto& v : h) {
      x = x * 1664525u + 1013904223u;
      v = (((x >> 9) * (1.0f / 8388608.0f)) - 0.5f) * 0.05f;
    }
    (void)hipMemcpy(W, h.data(), bytes, hipMemcpyHostToDevice);
    (void)hipMemset(R, 0, bytes);
  }
  struct Shape { const char* name; int M, N, K, grp; };
  const Shape shapes[] = {
      {"vit qkv 1600x2304x768", 1600, 2304, 768, 2}, {"vit out 1600x768x768", 1600, 768, 768, 2},
      {"vit fc1 1600x3072x768", 1600, 3072, 768, 2}, {"vit fc2 1600x768x3072", 1600, 768, 3072, 2},
      {"vit qkv 800x2304x768", 800, 2304, 768, 2},   {"vit fc2 800x768x3072", 800, 768, 3072, 2},
      {"t5 qkv 1536x1536x512", 1536, 1536, 512, 1},  {"t5 wo 1536x512x2048", 1536, 512, 2048, 1},
      {"odd 1000x1000x1000", 1000, 1000, 1000, 1},   {"odd 77x200x52", 77, 200, 52, 1},
      {"train dW ff 2048x512x1600", 2048, 512, 1600, 1}, {"train dW qkv 1536x512x1600", 1536, 512, 1600, 1},
      {"train qkv 1600x1536x512", 1600, 1536, 512, 1},
      {"tr o 1440x512x512", 1440, 512, 512, 1},
      {"tr wo 1440x512x2048", 1440, 512, 2048, 1},
      {"tr qkv 1440x1536x512", 1440, 1536, 512, 1},
      {"tr wi 1440x2048x512", 1440, 2048, 512, 1},
      {"tr dckv 1440x512x6144", 1440, 512, 6144, 1},
      {"tr dWckv 6144x512x1440", 6144, 512, 1440, 1},
      {"tr dWwi 2048x512x1440", 2048, 512, 1440, 1},
      {"tr dWo 512x512x1440", 512, 512, 1440, 1},
      {"tr dxqkv 1440x512x1536", 1440, 512, 1536, 1},
      {"loop t5 qkv 11776x1536x512", 11776, 1536, 512, 1},
      {"loop t5 o 11776x512x512", 11776, 512, 512, 1},
      {"loop t5 wi 11776x2048x512", 11776, 2048, 512, 1},
      {"loop t5 wo 11776x512x2048", 11776, 512, 2048, 1},
      {"c5 t5b qkv 10240x2304x768", 10240, 2304, 768, 1},
  };
  using L = std::function<int(const GemmGroup&, hipStream_t)>;
  struct Var { const char* name; L fn; bool packed; };
  const Var vars[] = {
      {"x3  128x128 2x1 k16 prio", launch_gemm_x3_group<128, 128, 2, 1, 16, 2, 1, 2>, false},
      {"x3  64x128 k32", launch_gemm_x3_group<64, 128, 1, 1, 32, 2, 1>, false},
      {"x3  64x64 k16", launch_gemm_x3_group<64, 64, 1, 1, 16, 2, 1>, false},
      {"x3  128x128 2x1 k16 prio SB2", launch_gemm_x3_group<128, 128, 2, 1, 16, 2, 1, 2, 2>, false},
      {"x3  64x64 k16 SB2", launch_gemm_x3_group<64, 64, 1, 1, 16, 2, 1, 0, 2>, false},
      {"x3  32x64 k16", launch_gemm_x3_group<32, 64, 1, 1, 16, 2, 1>, false},
      {"x3  64x32 k16", launch_gemm_x3_group<64, 32, 1, 1, 16, 2, 1>, false},
      {"x3  32x32 k16", launch_gemm_x3_group<32, 32, 1, 1, 16, 2, 1>, false},
      {"x3  32x64 k16 SB2", launch_gemm_x3_group<32, 64, 1, 1, 16, 2, 1, 0, 2>, false},
      {"x3p 128x128 4x1 D3", launch_gemm_x3p_group<128, 128, 4, 1, 3>, true},
      {"x3p 128x128 2x1 D2 (8w)", launch_gemm_x3p_group<128, 128, 2, 1, 2>, true},
      {"x3p 128x128 2x1 D3 (8w)", launch_gemm_x3p_group<128, 128, 2, 1, 3>, true},
      {"x3p 128x128 2x1 D2 SB2", launch_gemm_x3p_group<128, 128, 2, 1, 2, 16, 2>, true},
      {"x3p 128x128 2x1 D4 SB2", launch_gemm_x3p_group<128, 128, 2, 1, 4, 16, 2>, true},
      {"x3p 64x64 1x1 D2 SB2", launch_gemm_x3p_group<64, 64, 1, 1, 2, 16, 2>, true},
      {"x3p 64x64 1x1 D2 k32", launch_gemm_x3p_group<64, 64, 1, 1, 2, 32>, true},
      {"x3p 64x64 1x1 D2 k32 SB2", launch_gemm_x3p_group<64, 64, 1, 1, 2, 32, 2>, true},
      {"x3p 64x128 1x2 D2", launch_gemm_x3p_group<64, 128, 1, 2, 2>, true},
      {"x3p 64x128 1x2 D3", launch_gemm_x3p_group<64, 128, 1, 2, 3>, true},
      {"x3p 128x64 1x1 D2 (8w)", launch_gemm_x3p_group<128, 64, 1, 1, 2>, true},
      {"x3p 128x64 2x1 D2", launch_gemm_x3p_group<128, 64, 2, 1, 2>, true},
      {"x3p 64x64 1x1 D2", launch_gemm_x3p_group<64, 64, 1, 1, 2>, true},
      {"x3p 64x64 1x1 D3", launch_gemm_x3p_group<64, 64, 1, 1, 3>, true},
      {"x3p 32x64 1x1 D2", launch_gemm_x3p_group<32, 64, 1, 1, 2>, true},
      {"x3p 64x32 1x1 D2", launch_gemm_x3p_group<64, 32, 1, 1, 2>, true},
      {"x3p 128x128 4x1 D2 SB2 (4w)", launch_gemm_x3p_group<128, 128, 4, 1, 2, 16, 2>, true},
      {"x3p 128x128 2x2 D2 SB2 (4w)", launch_gemm_x3p_group<128, 128, 2, 2, 2, 16, 2>, true},
      {"x3p 128x256 2x2 D2 SB2 (8w)", launch_gemm_x3p_group<128, 256, 2, 2, 2, 16, 2>, true},
      {"x3p 256x128 4x1 D2 SB2 (8w)", launch_gemm_x3p_group<256, 128, 4, 1, 2, 16, 2>, true},
      {"x3p 128x256 4x1 D2 SB2 (8w)", launch_gemm_x3p_group<128, 256, 4, 1, 2, 16, 2>, true},
  };

  for (const Shape& sh : shapes) {
    if (!strstr(sh.name, fshape)) continue;
    double gf = 2.0 * sh.grp * sh.M * sh.N * sh.K * 1e-9;
    printf("%s x%d (%.2f GFLOP)\n", sh.name, sh.grp, gf);
    const size_t off = 6 << 20;
    for (int i = 0; i < sh.grp; ++i)
      (void)pack_x3(W + i * off, sh.N, sh.K, sh.K, (char*)P + i * (size_t)(24 << 20), s);
    (void)hipStreamSynchronize(s);
    std::vector<float> ref((size_t)sh.M * sh.N), got(ref.size());
    bool have_ref = false;
    for (const Var& v : vars) {
      if (have_ref && !strstr(v.name, fvar)) continue;
      GemmGroup G;
      G.n = sh.grp;
      for (int i = 0; i < sh.grp; ++i) {
        GemmArgs& g = G.g[i];
        g.A = A + i * off; g.lda = sh.K; g.W = W + i * off; g.ldw = sh.K;
        g.C = C + i * off; g.ldc = sh.N; g.M = sh.M; g.N = sh.N; g.K = sh.K;
        g.R = R + i * off; g.ldr = sh.N;
        g.wp = v.packed ? (char*)P + i * (size_t)(24 << 20) : nullptr;
      }
      (void)hipMemset(C, 0, bytes);
      const double us = time_graph(s, [&]() { v.fn(G, s); }, nl);
      (void)hipStreamSynchronize(s);
      (void)hipMemcpy(got.data(), C, got.size() * 4, hipMemcpyDeviceToHost);
      const char* eq = "ref";
      if (!have_ref) {
        ref = got;
        have_ref = true;
      } else {
        eq = memcmp(ref.data(), got.data(), ref.size() * 4) == 0 ? "bit-identical" : "DIFFERS";
      }
      printf("   %-26s %8.2f us  %6.1f TF/s  %s\n", v.name, us, gf / us * 1e3, eq);
    }
  }
  return 0;
}
