// kbench.hip — per-kernel cost of libmpr's decode kernels in a captured chain of 1000 launches
// (development aid; compiles the library sources directly so internal launchers are visible).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/kbench.hip -o tools/kbench
#include <chrono>
#include <cstdio>
#include <functional>

#include "../multimodalpromptretrieval_amd/csrc/api.hip"
#include "../multimodalpromptretrieval_amd/csrc/encoders.hip"
#include "../multimodalpromptretrieval_amd/csrc/gemm.hip"
#include "../multimodalpromptretrieval_amd/csrc/layers.hip"
#include "../multimodalpromptretrieval_amd/csrc/scan.hip"
#include "../multimodalpromptretrieval_amd/csrc/t5.hip"

using namespace mpr;

static double now_ms() {
  return std::chrono::duration<double, std::milli>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

static void time_chain(const char* name, hipStream_t s, const std::function<void(int)>& body,
                       int n = 1000) {
  body(0);
  (void)hipStreamSynchronize(s);
  double t = now_ms();
  for (int i = 0; i < n; ++i) body(i);
  (void)hipStreamSynchronize(s);
  const double eager = (now_ms() - t) * 1e3 / n;
  hipGraph_t g;
  hipGraphExec_t e;
  (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
  for (int i = 0; i < n; ++i) body(i);
  (void)hipStreamEndCapture(s, &g);
  (void)hipGraphInstantiate(&e, g, nullptr, nullptr, 0);
  (void)hipGraphLaunch(e, s);
  (void)hipStreamSynchronize(s);
  t = now_ms();
  (void)hipGraphLaunch(e, s);
  (void)hipStreamSynchronize(s);
  printf("%-40s eager %7.3f us   graph %7.3f us\n", name, eager, (now_ms() - t) * 1e3 / n);
  (void)hipGraphExecDestroy(e);
  (void)hipGraphDestroy(g);
}

int main() {
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  float *W, *x, *y, *g, *kv, *mask, *tab, *pv;
  int32_t *pi, *unf, *tok;
  (void)hipMalloc(&W, 160 << 20);
  (void)hipMalloc(&x, 4 << 20);
  (void)hipMalloc(&y, 4 << 20);
  (void)hipMalloc(&g, 1 << 20);
  (void)hipMalloc(&kv, 64 << 20);
  (void)hipMalloc(&mask, 1 << 20);
  (void)hipMalloc(&tab, 1 << 20);
  (void)hipMalloc(&pv, 1 << 20);
  (void)hipMalloc(&pi, 1 << 20);
  (void)hipMalloc(&unf, 4096);
  (void)hipMalloc(&tok, 1 << 16);
  (void)hipMemset(W, 0, 160 << 20);
  (void)hipMemset(x, 0, 4 << 20);
  (void)hipMemset(y, 0, 4 << 20);
  (void)hipMemset(g, 0, 1 << 20);
  (void)hipMemset(kv, 0, 64 << 20);
  (void)hipMemset(tab, 0, 1 << 20);
  (void)hipMemset(unf, 0, 4096);
  std::vector<float> ones(1 << 18, 1.f);
  (void)hipMemcpy(mask, ones.data(), 1 << 20, hipMemcpyHostToDevice);

  time_chain("fill_i32 (1 block)", s, [&](int) { fill_i32(unf, 1, 16, s); });
  size_t wstride = 4 << 20;
  auto skinny = [&](int N, int K, bool rms, bool res, int i) {
    SkinnyArgs a;
    a.g.A = (i & 1) ? y : x;
    a.g.lda = K;
    a.wpk = W + (size_t)(i % 6) * wstride;
    a.g.C = (i & 1) ? x : y;
    a.g.ldc = N;
    a.g.M = 16;
    a.g.N = N;
    a.g.K = K;
    if (res) {
      a.g.R = a.g.C;
      a.g.ldr = N;
    }
    if (rms) a.rms_w = g;
    gemm_skinny(a, s);
  };
  time_chain("skinny N512 K512 plain", s, [&](int i) { skinny(512, 512, false, false, i); });
  wstride = 1 << 20;
  time_chain("skinny N512 K512 plain, 4MB stride", s, [&](int i) { skinny(512, 512, false, false, i); });
  time_chain("skinny N512 K512 +res, 4MB stride", s, [&](int i) { skinny(512, 512, false, true, i); });
  wstride = 4 << 20;
  time_chain("skinny N512 K512 rms", s, [&](int i) { skinny(512, 512, true, false, i); });
  time_chain("skinny N512 K512 +res", s, [&](int i) { skinny(512, 512, false, true, i); });
  time_chain("skinny N1536 K512 rms", s, [&](int i) { skinny(1536, 512, true, false, i); });
  time_chain("skinny N2048 K512 rms", s, [&](int i) { skinny(2048, 512, true, false, i); });
  time_chain("skinny N512 K2048 +res", s, [&](int i) { skinny(512, 2048, false, true, i); });
  time_chain("lm_head N32101 K512 argmax", s, [&](int i) {
    SkinnyArgs a;
    a.g.A = x; a.g.lda = 512; a.wpk = W; a.g.C = nullptr; a.g.M = 16;
    a.g.N = 32101; a.g.K = 512; a.rms_w = g; a.amax_val = pv; a.amax_idx = pi;
    gemm_skinny(a, s);
  }, 200);
  for (int nt : {1, 2, 4, 8}) {
    char name[64];
    snprintf(name, sizeof name, "lm_head argmax NT=%d", nt);
    time_chain(name, s, [&](int i) {
      SkinnyArgs a;
      a.g.A = x; a.g.lda = 512; a.wpk = W; a.g.C = nullptr; a.g.M = 16;
      a.g.N = 32101; a.g.K = 512; a.rms_w = g; a.amax_val = pv; a.amax_idx = pi;
      const int F = SKF_AMAX | SKF_RMS;
      const unsigned tiles = (unsigned)cdiv(32101, 16);
      if (nt == 1) launch_skinny<4, 1, false>(a, F, tiles, s);
      if (nt == 2) launch_skinny<4, 2, false>(a, F, (unsigned)cdiv(tiles, 2), s);
      if (nt == 4) launch_skinny<4, 4, false>(a, F, (unsigned)cdiv(tiles, 4), s);
      if (nt == 8) launch_skinny<4, 8, false>(a, F, (unsigned)cdiv(tiles, 8), s);
    }, 200);
  }
  time_chain("greedy_step", s, [&](int i) {
    greedy_step(pv, pi, 2007, 16, unf, tok, 21, 1 + (i % 20), 1, 0, W, 512, x, s);
  });
  auto dec_attn = [&](int Lk, bool bias, int i) {
    AttnArgs a;
    a.q = kv; a.q_bs = 3 * 512 * 20; a.q_rs = 1536;
    a.k = kv + 512; a.k_bs = a.q_bs; a.k_rs = 1536;
    a.v = kv + 1024; a.v_bs = a.q_bs; a.v_rs = 1536;
    a.o = (i & 1) ? x : y; a.o_bs = 512; a.o_rs = 512;
    a.B = 16; a.H = 8; a.Lq = 1; a.Lk = Lk; a.scale = 1.f;
    if (bias) {
      a.causal = 1; a.q_pos0 = Lk - 1; a.rel_tab = tab; a.lut_radius = 1024;
    } else {
      a.q_bs = 512; a.q_rs = 512; a.k_bs = (int64_t)Lk * 6144; a.k_rs = 6144;
      a.v_bs = a.k_bs; a.v_rs = 6144; a.key_mask = mask; a.mask_bs = Lk;
    }
    attention(a, s);
  };
  time_chain("decode self-attn Lk=20", s, [&](int i) { dec_attn(20, true, i); });
  time_chain("decode cross-attn Lk=71", s, [&](int i) { dec_attn(71, false, i); });
  return 0;
}
