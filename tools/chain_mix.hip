// chain_mix.hip — where a decode step's ~4.7 us per kernel goes (development aid): graphs of 240
// dependent launches of (a) one skinny GEMV shape repeated, (b) attention_decode repeated, (c) the
// 8-kernel decoder-layer sequence of t5.hip (distinct kernels in turn), (d) an empty kernel, with
// the T5 decode shapes (16 rows, d 512, inner 512, dff 2048, 20 cached keys).  Weights cycle over
// 24 layer copies (the decode's MALL-resident working set) or stay on one copy (L2).
// build (links the library's internal entry points from libmpr.so):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/chain_mix.hip -o tools/chain_mix \
//     -Lmultimodalpromptretrieval_amd -lmpr -Wl,-rpath,'$ORIGIN/../multimodalpromptretrieval_amd'
#include <cstdio>
#include <functional>
#include <vector>

#include "../multimodalpromptretrieval_amd/csrc/kernels.h"

using namespace mpr;

__global__ void empty_kernel(float* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && p[0] == 12345.f) p[1] = 1.f;
}

static double time_graph(hipStream_t s, const std::function<void(int)>& body, int n) {
  body(0);
  (void)hipStreamSynchronize(s);
  hipGraph_t g;
  hipGraphExec_t e;
  (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
  for (int i = 0; i < n; ++i) body(i);
  (void)hipStreamEndCapture(s, &g);
  (void)hipGraphInstantiate(&e, g, nullptr, nullptr, 0);
  (void)hipGraphLaunch(e, s);
  (void)hipStreamSynchronize(s);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  float best = 1e30f;
  for (int r = 0; r < 3; ++r) {
    (void)hipEventRecord(a, s);
    (void)hipGraphLaunch(e, s);
    (void)hipEventRecord(b, s);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    best = std::min(best, ms);
  }
  (void)hipGraphExecDestroy(e);
  (void)hipGraphDestroy(g);
  return best * 1e3 / n;
}

int main() {
  const int B = 16, d = 512, inner = 512, dff = 2048, H = 8, T = 20, NL = 24;
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  auto alloc = [](size_t n) {
    float* p;
    (void)hipMalloc(&p, n * 4);
    (void)hipMemset(p, 0, n * 4);
    return p;
  };
  // packed weights per layer copy
  const int64_t e_qkv = packed_rows16_elems(3 * inner, d), e_o = packed_rows16_elems(d, inner),
                e_wi = packed_rows16_elems(dff, d), e_wo = packed_rows16_elems(d, dff);
  std::vector<float*> qkv(NL), wo_(NL), wi(NL), wo2(NL), cq(NL), co(NL);
  for (int l = 0; l < NL; ++l) {
    qkv[l] = alloc(e_qkv); wo_[l] = alloc(e_o); cq[l] = alloc(e_o); co[l] = alloc(e_o);
    wi[l] = alloc(e_wi); wo2[l] = alloc(e_wo);
  }
  float* ln = alloc(d);
  float* x = alloc(B * d);
  float* cache = alloc((size_t)B * T * 3 * inner);
  float* ao = alloc(B * dff);
  float* qp = alloc(B * inner);
  float* ff = alloc(B * dff);
  float* ckv = alloc((size_t)B * 64 * 2 * inner);
  float* mask = alloc(B * 64);
  float* rel = alloc((2 * 1024 + 1) * H);
  float* flag = alloc(16);
  const int t = T - 1;
  auto sk = [&](const float* A, int lda, float* C, int ldc, int N, int K, const float* wpk,
                const float* rms, const float* R) {
    SkinnyArgs a;
    a.g.A = A; a.g.lda = lda; a.g.C = C; a.g.ldc = ldc; a.g.M = B; a.g.N = N; a.g.K = K;
    a.g.R = R; a.g.ldr = R ? d : 0;
    a.rms_w = rms; a.wpk = wpk;
    (void)gemm_skinny(a, s);
  };
  auto self_attn = [&]() {
    AttnArgs at;
    at.q = cache + (int64_t)t * 3 * inner; at.q_bs = (int64_t)T * 3 * inner; at.q_rs = 3 * inner;
    at.k = cache + inner; at.k_bs = at.q_bs; at.k_rs = 3 * inner;
    at.v = cache + 2 * inner; at.v_bs = at.q_bs; at.v_rs = 3 * inner;
    at.o = ao; at.o_bs = inner; at.o_rs = inner;
    at.B = B; at.H = H; at.Lq = 1; at.Lk = t + 1; at.causal = 1; at.q_pos0 = t;
    at.rel_tab = rel; at.lut_radius = 1024;
    (void)attention(at, s);
  };
  auto cross_attn = [&]() {
    AttnArgs ca;
    const int64_t ld = 2 * inner;
    ca.q = qp; ca.q_bs = inner; ca.q_rs = inner;
    ca.k = ckv; ca.k_bs = 64 * ld; ca.k_rs = ld;
    ca.v = ckv + inner; ca.v_bs = ca.k_bs; ca.v_rs = ld;
    ca.o = ao; ca.o_bs = inner; ca.o_rs = inner;
    ca.B = B; ca.H = H; ca.Lq = 1; ca.Lk = 64;
    ca.key_mask = mask; ca.mask_bs = 64;
    (void)attention(ca, s);
  };
  const int N = 240;
  for (int cyc = 0; cyc < 2; ++cyc) {
    auto L = [&](int i) { return cyc ? (i / 8) % NL : 0; };
    printf("%s\n", cyc ? "weights cycled over 24 layer copies" : "one weight copy (L2)");
    printf("  empty kernel                 %6.2f us\n", time_graph(s, [&](int) {
      hipLaunchKernelGGL(empty_kernel, dim3(64), dim3(256), 0, s, flag);
    }, N));
    printf("  qkv skinny (rms) repeated    %6.2f us\n", time_graph(s, [&](int i) {
      sk(x, d, cache, 3 * inner, 3 * inner, d, qkv[L(i * 8)], ln, nullptr);
    }, N));
    printf("  o skinny (+res) repeated     %6.2f us\n", time_graph(s, [&](int i) {
      sk(ao, inner, x, d, d, inner, wo_[L(i * 8)], nullptr, x);
    }, N));
    printf("  wi skinny (rms,relu) rep.    %6.2f us\n", time_graph(s, [&](int i) {
      SkinnyArgs a;
      a.g.A = x; a.g.lda = d; a.g.C = ff; a.g.ldc = dff; a.g.M = B; a.g.N = dff; a.g.K = d;
      a.g.act = ACT_RELU; a.rms_w = ln; a.wpk = wi[L(i * 8)];
      (void)gemm_skinny(a, s);
    }, N));
    printf("  wo skinny K=2048 repeated    %6.2f us\n", time_graph(s, [&](int i) {
      sk(ff, dff, x, d, d, dff, wo2[L(i * 8)], nullptr, x);
    }, N));
    printf("  self attention repeated      %6.2f us\n", time_graph(s, [&](int) { self_attn(); }, N));
    printf("  cross attention repeated     %6.2f us\n", time_graph(s, [&](int) { cross_attn(); }, N));
    float* x2 = x + 0;  // ping-pong partner below
    static float* xb = nullptr;
    if (!xb) xb = alloc(B * d);
    printf("  o skinny, reads prev output  %6.2f us\n", time_graph(s, [&](int i) {
      // A = the previous launch's C (a real read-after-write dependency), residual none
      sk((i & 1) ? xb : x2, d, (i & 1) ? x2 : xb, d, d, inner, wo_[L(i * 8)], nullptr, nullptr);
    }, N));
    printf("  o / cq alternating, no dep   %6.2f us\n", time_graph(s, [&](int i) {
      if (i & 1) sk(ao, inner, ff, d, d, inner, wo_[L(i * 8)], nullptr, nullptr);
      else sk(x, d, qp, inner, inner, d, cq[L(i * 8)], ln, nullptr);
    }, N));
    printf("  o / cq alternating, dep      %6.2f us\n", time_graph(s, [&](int i) {
      if (i & 1) sk(qp, inner, x, d, d, inner, wo_[L(i * 8)], nullptr, nullptr);
      else sk(x, d, qp, inner, inner, d, cq[L(i * 8)], ln, nullptr);
    }, N));
    printf("  decoder-layer sequence (8)   %6.2f us\n", time_graph(s, [&](int i) {
      const int l = L(i);
      switch (i % 8) {
        case 0: sk(x, d, cache + (int64_t)t * 3 * inner, T * 3 * inner, 3 * inner, d, qkv[l], ln, nullptr); break;
        case 1: self_attn(); break;
        case 2: sk(ao, inner, x, d, d, inner, wo_[l], nullptr, x); break;
        case 3: sk(x, d, qp, inner, inner, d, cq[l], ln, nullptr); break;
        case 4: cross_attn(); break;
        case 5: sk(ao, inner, x, d, d, inner, co[l], nullptr, x); break;
        case 6: {
          SkinnyArgs a;
          a.g.A = x; a.g.lda = d; a.g.C = ff; a.g.ldc = dff; a.g.M = B; a.g.N = dff; a.g.K = d;
          a.g.act = ACT_RELU; a.rms_w = ln; a.wpk = wi[l];
          (void)gemm_skinny(a, s);
          break;
        }
        default: sk(ff, dff, x, d, d, dff, wo2[l], nullptr, x); break;
      }
    }, N));
  }
  return 0;
}
