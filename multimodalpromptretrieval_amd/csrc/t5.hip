// t5.hip — T5 encoder, greedy decoder and teacher-forced logits on the gfx950 kernels.
//
// Reference semantics: transformers T5ForConditionalGeneration as driven by
// architectures/T5VisionModel.py:200-205 (generate(inputs_embeds, attention_mask, do_sample=False,
// max_new_tokens=20)) and :233 (teacher-forced loss):
//   T5LayerNorm = RMSNorm (no mean, no bias, eps 1e-6);  attention without 1/sqrt(d) scaling,
//   relative position bias from layer 0 (bidirectional buckets in the encoder, causal in the
//   decoder) shared by every layer, padding mask on encoder keys; ReLU FFN; final RMSNorm, then
//   * d_model^-0.5 before the tied lm_head (scale_decoder_outputs).
// Decoder steps run M = batch rows: every projection is a skinny GEMM with the preceding RMSNorm
// fused (operand ln_w*x, 1/rms applied in the epilogue); K/V of the self-attention live in a
// per-layer cache laid out [B][max_new][3*inner] (the fused q|k|v row of each generated position);
// the cross-attention K/V of every decoder layer come from one GEMM over the encoder output; the
// lm_head never materialises logits: each block emits its per-row best column and greedy_step
// reduces those and gathers the next input embedding.  generate() is captured once per shape into
// two hipGraphs (private capture stream): the encoder + cross K/V projection, replayed on the
// caller's stream, and the decode loop (~50 launches per step), replayed on the decode stream when
// one is set (a CU partition of its own) or else on the caller's stream.
#include <chrono>
#include <cstdlib>

#include "models.h"

namespace mpr {

namespace {
constexpr float T5_EPS = 1e-6f;
// per workspace slot: an eval run meets a handful of bucketed source lengths, each with an encoder
// graph, a decode graph and (early-stop generate) max_new / chunk decode-chunk graphs
constexpr size_t MAX_GRAPHS = 256;

bool graphs_enabled() {
  const char* e = getenv("MPR_GRAPHS");
  return !(e && e[0] == '0');
}

// Weight refresh after an optimizer step (mpr_t5_update_async): ~130 tensor copies and ~37
// lane-order packs as hipMemcpyAsync / pack_rows16 launches cost ~5 us each of launch-bound GPU
// time (0.75 + 0.26 ms per training step); these take up to 32 / 16 of them per launch, each
// segment a row of blocks walking it grid-stride (float4 when aligned).
__global__ __launch_bounds__(256) void copy_segments_kernel(const CopySegs segs) {
  const CopySeg sg = segs.s[blockIdx.y];
  const int64_t stride = (int64_t)gridDim.x * 256;
  const int64_t t0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (((reinterpret_cast<uintptr_t>(sg.src) | reinterpret_cast<uintptr_t>(sg.dst)) & 15) == 0) {
    const int64_t n4 = sg.n >> 2;
    const float4* s4 = reinterpret_cast<const float4*>(sg.src);
    float4* d4 = reinterpret_cast<float4*>(sg.dst);
    for (int64_t i = t0; i < n4; i += stride) d4[i] = s4[i];
    for (int64_t i = (n4 << 2) + t0; i < sg.n; i += stride) sg.dst[i] = sg.src[i];
  } else {
    for (int64_t i = t0; i < sg.n; i += stride) sg.dst[i] = sg.src[i];
  }
}

__global__ __launch_bounds__(256) void pack_many_kernel(const PackJobs jobs) {
  const PackJob jb = jobs.j[blockIdx.y];
  const int64_t nch = (jb.K + 15) / 16;
  const int64_t total = (jb.N + 15) / 16 * nch * 64;  // float4s of the image
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < total;
       q += (int64_t)gridDim.x * 256) {
    const int l = (int)(q & 63);
    const int64_t tc = q >> 6, t = tc / nch, c = tc % nch;
    const int64_t row = t * 16 + (l & 15), k0 = c * 16 + (l >> 4) * 4;
    float4 v = {0.f, 0.f, 0.f, 0.f};
    if (row < jb.N) {
      if (k0 + 0 < jb.K) v.x = jb.src[row * jb.K + k0 + 0];
      if (k0 + 1 < jb.K) v.y = jb.src[row * jb.K + k0 + 1];
      if (k0 + 2 < jb.K) v.z = jb.src[row * jb.K + k0 + 2];
      if (k0 + 3 < jb.K) v.w = jb.src[row * jb.K + k0 + 3];
    }
    reinterpret_cast<float4*>(jb.dst)[q] = v;
  }
}

// One folded decode-chain weight [d + N2, inner + d]:
//   rows n < d:       [top[n, :] | e_n]                      (top: [d, inner], the o / co weight)
//   rows d + j < N2:  [sum_k bot[j, k] w[k] top[k, :] | bot[j, :] * w]
// (bot: [N2, d], the cq / wi weight; w the RMSNorm weight between them), written straight into
// its pack_rows16 lane-order image (the decode GEMV's weight layout; d + N2 and inner + d are
// multiples of 16, so there is no padding).  The product is summed in double and rounded once.
// Every fold of the model goes in two launches (fold_copy_kernel: the copied / scaled parts;
// fold_product_kernel: the product blocks as double-precision tiles through LDS, the next k
// step's operands prefetched into registers): one
// thread per element with a column of top re-read per output took 264 us per fold of t5-small's
// 2048-row wi, 12 folds after every optimizer step.
struct FoldJob {
  const float* top;
  const float* bot;
  const float* w;
  float* out;
  int N2;
};
constexpr int FOLD_JOBS = 32;
struct FoldJobs {
  FoldJob j[FOLD_JOBS];
};

__device__ __forceinline__ int64_t packed16(int row, int col, int kc16) {
  return ((int64_t)(row >> 4) * kc16 + (col >> 4)) * 256 + ((row & 15) + 16 * ((col & 15) >> 2)) * 4 +
         (col & 3);
}

__global__ void fold_copy_kernel(const FoldJobs jobs, int d, int inner) {
  const FoldJob jb = jobs.j[blockIdx.y];
  const int K = inner + d;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)(d + jb.N2) * K) return;
  const int row = (int)(e / K), col = (int)(e % K);
  float v;
  if (row < d)
    v = col < inner ? jb.top[(int64_t)row * inner + col] : (col - inner == row ? 1.f : 0.f);
  else if (col >= inner)
    v = jb.bot[(int64_t)(row - d) * d + (col - inner)] * jb.w[col - inner];
  else
    return;  // fold_product_kernel
  jb.out[packed16(row, col, K >> 4)] = v;
}

// 128 x 128 product tile per block, 8 x 8 per thread (rows ty + 16 r, columns tx + 16 q): 16 LDS
// reads per 64 FMAs keeps the fp64 FMA pipe, not LDS, the limit (2 x 2 per thread: 690 us for
// t5-small's 12 folds, LDS-bound).  k in ascending order per output: the same sum as one thread
// looping over k.
constexpr int FOLD_T = 128, FOLD_K = 8;
__global__ __launch_bounds__(256) void fold_product_kernel(const FoldJobs jobs, int d, int inner) {
  __shared__ double sb[FOLD_K][FOLD_T];  // bot[j0 + j, k0 + k] * w[k0 + k] at [k][j]
  __shared__ double st[FOLD_K][FOLD_T];  // top[k0 + k, c0 + c] at [k][c]
  const FoldJob jb = jobs.j[blockIdx.z];
  const int N2 = jb.N2, K = inner + d;
  const int j0 = blockIdx.y * FOLD_T, c0 = blockIdx.x * FOLD_T;
  if (j0 >= N2) return;
  const int t = threadIdx.x, tx = t & 15, ty = t >> 4;
  constexpr int PER = FOLD_K * FOLD_T / 256;  // operand elements each thread stages per k step
  double pb[PER], pt[PER];
  auto load = [&](int k0) {
#pragma unroll
    for (int h = 0; h < PER; ++h) {
      const int i = t + 256 * h;
      const int kb = i % FOLD_K, jr = i / FOLD_K;
      const int j = j0 + jr, k = k0 + kb;
      pb[h] = (j < N2 && k < d) ? (double)jb.bot[(int64_t)j * d + k] * (double)jb.w[k] : 0.0;
      const int ct = i % FOLD_T, kt = i / FOLD_T;
      const int c = c0 + ct, k2 = k0 + kt;
      pt[h] = (c < inner && k2 < d) ? (double)jb.top[(int64_t)k2 * inner + c] : 0.0;
    }
  };
  double acc[8][8];
#pragma unroll
  for (int r = 0; r < 8; ++r)
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[r][q] = 0.0;
  load(0);
  for (int k0 = 0; k0 < d; k0 += FOLD_K) {
#pragma unroll
    for (int h = 0; h < PER; ++h) {
      const int i = t + 256 * h;
      sb[i % FOLD_K][i / FOLD_K] = pb[h];
      st[i / FOLD_T][i % FOLD_T] = pt[h];
    }
    __syncthreads();
    if (k0 + FOLD_K < d) load(k0 + FOLD_K);
#pragma unroll
    for (int kk = 0; kk < FOLD_K; ++kk) {
      double a[8], b[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) a[r] = sb[kk][ty + 16 * r];
#pragma unroll
      for (int q = 0; q < 8; ++q) b[q] = st[kk][tx + 16 * q];
#pragma unroll
      for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[r][q] += a[r] * b[q];
    }
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const int j = j0 + ty + 16 * r;
    if (j >= N2) continue;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = c0 + tx + 16 * q;
      if (c < inner) jb.out[packed16(d + j, c, K >> 4)] = (float)acc[r][q];
    }
  }
}
}  // namespace

// The folded decode chain.  T5's decoder layer is
//   x1 = x + a Wo^T;  q = rms(x1) ln1 Wcq^T;  x2 = x1 + c Wco^T;  f = relu(rms(x2) ln2 Wi^T);
//   x3 = x2 + f Wwo^T
// and rms(v) = v / sqrt(mean(v^2) + eps) is a positive per-row scale, so with
// M1 = Wcq diag(ln1), M3 = Wi diag(ln2):
//   [x1 | u] = [a | x] [[Wo | I], [M1 Wo | M1]]^T,  q = u / rms_scale(x1)
//   [x2 | z] = [c | x1] [[Wco | I], [M3 Wco | M3]]^T,  f Wwo^T = (relu(z) Wwo^T) / rms_scale(x2)
// (relu commutes with the positive scale): the two RMSNorm launches fold into the o and co
// projections, the cross-attention applies its query's scale from the x1 row it reads, and the
// FFN-out GEMM applies relu on load and the x2 scale in its epilogue.  8 -> 6 dependent launches
// per layer, at a different fp32 rounding order than the reference's.
//
// One decode chain per model at every row count, so a batch decoded alone (predict(), <= 16 rows)
// and inside a serving loop's grouped decode (128 rows) gets the same bits: rows are independent
// in every kernel of a chain, whatever the row blocking.  t5-small (d < 768) takes the folded
// chain with the skinny argmax head at every row count (its 128-row groups cost nothing
// measurable folded: 3,934 against 3,938 QA pairs/s, profiles/r06_chain_ab.txt); d >= 768
// (t5-base) takes the 8-launch chain with the tiled argmax head at every row count (folded, two of
// a layer's three GEMV pairs read twice the weights, which C5's 256-row decodes pay for; the
// skinny head stages the rows once per 16 columns: 201 against 55 us for 128 rows).
// MPR_DECODE_FOLD_ROWS (fold only up to that many rows) / MPR_TILED_HEAD are A/B switches: a
// chain that changes with the row count no longer matches predict() bit for bit.
bool T5Model::fold_rows(int B) const {
  static const int max_rows = [] {
    const char* e = getenv("MPR_DECODE_FOLD_ROWS");
    return e ? atoi(e) : -1;
  }();
  return fold && (max_rows < 0 || B <= max_rows);
}

int T5Model::dec_gemm(const SkinnyArgs& a, const DevBuf& pk, hipStream_t s,
                      int* amax_nparts) const {
  SkinnyArgs b = a;
  b.wpk = pk.as<float>();
  if (amax_nparts) *amax_nparts = (int)cdiv(a.g.N, 16);
  return gemm_skinny(b, s);
}

// The argmax head as RMSNorm + the tiled split-bf16 GEMM into a logits buffer + a row argmax,
// instead of the skinny GEMV (which stages the rows once per 16 columns: 8,032 blocks re-reading
// 96 KB of rows for t5-base's 128-row head, 201 us).  Default for d >= 768 (t5-base and up) at
// every row count (fold_rows); MPR_TILED_HEAD=0 / 1 forces it off / on (read per call; a captured
// decode graph keeps the head it was captured with).
bool T5Model::tiled_head(int B) const {
  const char* e = getenv("MPR_TILED_HEAD");
  const bool on = e ? e[0] == '1' : d >= 768;
  return on && !fold_rows(B);
}

int T5Model::build_folded(hipStream_t s) {
  const int K = inner + d;
  MPR_REQUIRE(d % 16 == 0 && inner % 16 == 0 && dff % 16 == 0, "fold: d=%d inner=%d dff=%d", d,
              inner, dff);
  std::vector<FoldJob> all;
  for (auto& lp : dec) {
    T5Layer& ly = *lp;
    MPR_TRY(ly.pk_ocq.ensure((size_t)packed_rows16_elems(d + inner, K) * 4));
    MPR_TRY(ly.pk_cowi.ensure((size_t)packed_rows16_elems(d + dff, K) * 4));
    all.push_back({ly.o.as<float>(), ly.cq.as<float>(), ly.ln1.as<float>(), ly.pk_ocq.as<float>(),
                   inner});
    all.push_back({ly.co.as<float>(), ly.wi.as<float>(), ly.ln2.as<float>(),
                   ly.pk_cowi.as<float>(), dff});
  }
  for (size_t j0 = 0; j0 < all.size(); j0 += FOLD_JOBS) {
    FoldJobs jobs;
    const int n = (int)std::min<size_t>(FOLD_JOBS, all.size() - j0);
    int max_n2 = 0;
    for (int j = 0; j < n; ++j) {
      jobs.j[j] = all[j0 + j];
      max_n2 = std::max(max_n2, jobs.j[j].N2);
    }
    const int64_t elems = (int64_t)(d + max_n2) * K;
    hipLaunchKernelGGL(fold_copy_kernel, dim3((unsigned)cdiv(elems, 256), (unsigned)n), dim3(256),
                       0, s, jobs, d, inner);
    MPR_LAUNCHED();
    hipLaunchKernelGGL(fold_product_kernel,
                       dim3((unsigned)cdiv(inner, FOLD_T), (unsigned)cdiv(max_n2, FOLD_T), (unsigned)n),
                       dim3(256), 0, s, jobs, d, inner);
    MPR_LAUNCHED();
  }
  return MPR_OK;
}

int copy_segments(const std::vector<CopySeg>& segs, hipStream_t s) {
  for (size_t i0 = 0; i0 < segs.size(); i0 += COPY_SEGS) {
    CopySegs cs;
    const int n = (int)std::min<size_t>(COPY_SEGS, segs.size() - i0);
    int64_t mx = 1;
    for (int i = 0; i < n; ++i) {
      cs.s[i] = segs[i0 + i];
      mx = std::max(mx, cs.s[i].n);
    }
    hipLaunchKernelGGL(copy_segments_kernel,
                       dim3((unsigned)std::min<int64_t>(cdiv(cdiv(mx, 4), 256), 1024), (unsigned)n),
                       dim3(256), 0, s, cs);
    MPR_LAUNCHED();
  }
  return MPR_OK;
}

int pack_many(const std::vector<PackJob>& jobs, hipStream_t s) {
  for (size_t i0 = 0; i0 < jobs.size(); i0 += PACK_JOBS) {
    PackJobs pj;
    const int n = (int)std::min<size_t>(PACK_JOBS, jobs.size() - i0);
    int64_t mx = 1;
    for (int i = 0; i < n; ++i) {
      pj.j[i] = jobs[i0 + i];
      mx = std::max(mx, packed_rows16_elems(pj.j[i].N, pj.j[i].K) / 4);
    }
    hipLaunchKernelGGL(pack_many_kernel, dim3((unsigned)std::min<int64_t>(cdiv(mx, 256), 1024),
                                              (unsigned)n),
                       dim3(256), 0, s, pj);
    MPR_LAUNCHED();
  }
  return MPR_OK;
}

T5Work::~T5Work() {
  for (auto& kv : graphs) (void)hipGraphExecDestroy(kv.second.exec);
  for (hipEvent_t e : ev_chunk) (void)hipEventDestroy(e);
  if (h_unf) (void)hipHostFree(h_unf);
  if (cap_stream) (void)hipStreamDestroy(cap_stream);
  if (ev_fork) (void)hipEventDestroy(ev_fork);
  if (ev_join) (void)hipEventDestroy(ev_join);
}

int T5Model::grow(DevBuf& b, size_t bytes) {
  void* before = b.ptr;
  MPR_TRY(b.ensure(bytes));
  if (b.ptr != before) ++ws->gen;
  return MPR_OK;
}

int T5Model::use_slot(int slot) {
  MPR_REQUIRE(slot >= 0 && slot < MAX_SLOTS, "t5: workspace slot %d outside [0, %d)", slot,
              MAX_SLOTS);
  while ((int)work.size() <= slot) work.push_back(std::make_unique<T5Work>());
  ws = work[slot].get();
  return MPR_OK;
}

int T5Model::embed(const int32_t* ids, int B, int len, float* out, int64_t out_bs, int row0,
                   hipStream_t s) {
  return embed_gather(shared.as<float>(), ids, len, B, len, d, nullptr, out, out_bs, row0, s);
}

int T5Model::encode(const float* embeds, const float* mask, int B, int L, float* out,
                    hipStream_t s) {
  return encode_multi(1, &B, &L, embeds, mask, out, s);
}

// The T5 encoder over n <= MAX_GROUPS batches at once: batch g's rows (B[g] x L[g]) follow
// batch g-1's in `embeds`, `mask` and `out`.  Row-wise ops run once over all rows; every projection
// is ONE problem over all the batches' stacked rows when every tiled-GEMM configuration sums an
// output in the same order (the split-bf16 kernels: gemm_uniform_order) — a 16-batch C5 group's
// q|k|v is one 8,000-row launch that fills the chip instead of four 4-problem launches of ~500-row
// problems — else one problem per batch (each keeps the tile it gets alone, GEMM_GROUP per
// launch); the attentions go ATTN_GROUP batches per launch.  Each batch's result is bit-identical
// to encoding it alone.
int T5Model::encode_multi(int n, const int* Bs, const int* Ls, const float* embeds,
                          const float* mask, float* out, hipStream_t s) {
  MPR_REQUIRE(n >= 1 && n <= MAX_GROUPS, "t5 encode: %d batches", n);
  int64_t row0[MAX_GROUPS + 1];
  row0[0] = 0;
  for (int g = 0; g < n; ++g) {
    MPR_REQUIRE(Ls[g] >= 1, "t5 encode: L=%d", Ls[g]);
    MPR_REQUIRE(Ls[g] - 1 <= lut_radius, "t5 encode: L=%d exceeds the bucket lut radius %d + 1",
                Ls[g], lut_radius);
    row0[g + 1] = row0[g] + (int64_t)Bs[g] * Ls[g];
  }
  const int64_t M = row0[n];
  if (M == 0) return MPR_OK;
  MPR_REQUIRE(M < (int64_t)1 << 31, "t5 encode: %lld rows", (long long)M);
  MPR_TRY(grow(ws->x, (size_t)M * d * 4));
  MPR_TRY(grow(ws->h, (size_t)M * d * 4));
  MPR_TRY(grow(ws->qkv, (size_t)M * 3 * inner * 4));
  MPR_TRY(grow(ws->ao, (size_t)M * inner * 4));
  MPR_TRY(grow(ws->ff, (size_t)M * dff * 4));
  float* xp = ws->x.as<float>();
  float* hp = ws->h.as<float>();
  float* qp = ws->qkv.as<float>();
  float* ap = ws->ao.as<float>();
  float* fp = ws->ff.as<float>();
  const bool merged = gemm_uniform_order();
  // one projection over rows [r0, r1) of the stacked batches
  auto proj = [&](int64_t r0, int64_t r1, const float* A, int64_t lda, const DevBuf& Wb,
                  const DevBuf& Wp, int N, int K, const float* R, float* C, int act) {
    GemmArgs g;
    g.A = A + r0 * lda; g.lda = lda; g.W = Wb.as<float>(); g.ldw = K; g.wp = Wp.ptr;
    g.R = R ? R + r0 * N : nullptr; g.ldr = N; g.C = C + r0 * N; g.ldc = N;
    g.M = (int)(r1 - r0); g.N = N; g.K = K; g.act = act;
    return g;
  };
  auto run = [&](const float* A, int64_t lda, const DevBuf& W, const DevBuf& Wp, int N, int K,
                 const float* R, float* C, int act) -> int {
    if (merged) return gemm(proj(0, M, A, lda, W, Wp, N, K, R, C, act), s);
    for (int g0 = 0; g0 < n; g0 += GEMM_GROUP) {
      GemmGroup gg;
      gg.n = 0;
      for (int g = g0; g < std::min(n, g0 + GEMM_GROUP); ++g)
        if (row0[g + 1] > row0[g])
          gg.g[gg.n++] = proj(row0[g], row0[g + 1], A, lda, W, Wp, N, K, R, C, act);
      if (gg.n) MPR_TRY(gemm_group(gg, s));
    }
    return MPR_OK;
  };
  MPR_HIP(hipMemcpyAsync(xp, embeds, (size_t)M * d * 4, hipMemcpyDeviceToDevice, s));
  for (auto& lp : enc) {
    const T5Layer& ly = *lp;
    MPR_TRY(rmsnorm(xp, d, (int)M, d, ly.ln0.as<float>(), T5_EPS, hp, d, s));
    MPR_TRY(run(hp, d, ly.qkv, ly.xp_qkv, 3 * inner, d, nullptr, qp, ACT_NONE));
    for (int g0 = 0; g0 < n; g0 += ATTN_GROUP) {
      AttnGroup at;
      at.n = 0;
      for (int g = g0; g < std::min(n, g0 + ATTN_GROUP); ++g) {
        const int B = Bs[g], L = Ls[g];
        if (B * L == 0) continue;
        const int64_t r = row0[g];
        AttnArgs& a = at.a[at.n++];
        const float* qb = qp + r * 3 * inner;
        a.q = qb; a.q_bs = (int64_t)L * 3 * inner; a.q_rs = 3 * inner;
        a.k = qb + inner; a.k_bs = a.q_bs; a.k_rs = 3 * inner;
        a.v = qb + 2 * inner; a.v_bs = a.q_bs; a.v_rs = 3 * inner;
        a.o = ap + r * inner; a.o_bs = (int64_t)L * inner; a.o_rs = inner;
        a.B = B; a.H = H; a.Lq = L; a.Lk = L; a.scale = 1.f;
        a.key_mask = mask + r; a.mask_bs = L;
        a.rel_tab = enc_tab.as<float>();
        a.lut_radius = lut_radius;
      }
      if (at.n) MPR_TRY(attention_group(at, s));
    }
    MPR_TRY(run(ap, inner, ly.o, ly.xp_o, d, inner, xp, xp, ACT_NONE));
    MPR_TRY(rmsnorm(xp, d, (int)M, d, ly.ln1.as<float>(), T5_EPS, hp, d, s));
    MPR_TRY(run(hp, d, ly.wi, ly.xp_wi, dff, d, nullptr, fp, ACT_RELU));
    MPR_TRY(run(fp, dff, ly.wo, ly.xp_wo, d, dff, xp, xp, ACT_NONE));
  }
  MPR_TRY(rmsnorm(xp, d, (int)M, d, enc_final.as<float>(), T5_EPS, out, d, s));
  return MPR_OK;
}

int T5Model::cross_kv_project(int B, int L, hipStream_t s) {
  const int M = B * L, N = Ld * 2 * inner;
  GemmArgs g;
  g.A = ws->enc_out.as<float>(); g.lda = d; g.W = cross_kv_w.as<float>(); g.ldw = d;
  g.wp = xp_cross_kv.ptr;
  g.C = ws->cross_kv.as<float>(); g.ldc = N; g.M = M; g.N = N; g.K = d;
  return gemm(g, s);
}

// Everything generate() enqueues after its inputs sit in enc_in / mask_in, in two parts: the
// encoder (+ cross-attention K/V of every decoder layer, + the decode state reset) and the greedy
// decode loop.  Only model-owned buffers are touched, so each part is captured into a graph and
// replayed; the decode part can run on its own stream (mpr_t5_set_decode_stream).
int T5Model::encode_body(int B, int L, int max_new, int start, hipStream_t s) {
  MPR_TRY(encode(ws->enc_in.as<float>(), ws->mask_in.as<float>(), B, L, ws->enc_out.as<float>(),
                 s));
  return init_body(B, L, max_new, start, s);
}

// Cross-attention K/V over enc_out [B, L] and the decode state reset.
int T5Model::init_body(int B, int L, int max_new, int start, hipStream_t s) {
  const int T1 = max_new + 1;
  MPR_TRY(cross_kv_project(B, L, s));
  if (debug_decode_trace()) {  // a new trace: the decode's inputs first
    ws->trace_off = 0;
    ws->segs.clear();
    MPR_TRY(trace(TR_ENC_OUT, -1, -1, ws->enc_out.ptr, (int64_t)B * L, d, d, s));
    MPR_TRY(trace(TR_CROSS_KV, -1, -1, ws->cross_kv.ptr, (int64_t)B * L, (int64_t)Ld * 2 * inner,
                  (int64_t)Ld * 2 * inner, s));
  }
  MPR_TRY(fill_i32(ws->unfinished.as<int32_t>(), 1, B, s));
  MPR_TRY(fill_i32(ws->cur_tok.as<int32_t>(), start, B, s));
  MPR_TRY(fill_i32(ws->tok_buf.as<int32_t>(), start, (int64_t)B * T1, s));  // column 0 = start
  if (fold_rows(B))  // the residual stream lives in the x half of the [a | x] rows
    MPR_TRY(embed_gather(shared.as<float>(), ws->cur_tok.as<int32_t>(), 1, B, 1, d, nullptr,
                         ws->ax.as<float>() + inner, inner + d, 0, s));
  else
    MPR_TRY(embed_gather(shared.as<float>(), ws->cur_tok.as<int32_t>(), 1, B, 1, d, nullptr,
                         ws->dx.as<float>(), d, 0, s));
  return MPR_OK;
}

// Decode steps [t0, t1) of a max_new-step greedy loop (t1 < 0: to the end).
int T5Model::decode_body(int B, int L, int max_new, int eos, int pad, hipStream_t s, int t0,
                         int t1) {
  if (t1 < 0 || t1 > max_new) t1 = max_new;
  const int T1 = max_new + 1, Tc = max_new > 0 ? max_new : 1;
  const int64_t cache_layer = (int64_t)B * Tc * 3 * inner;
  const float* maskp = ws->mask_in.as<float>();
  float* xp = ws->dx.as<float>();
  float* qp = ws->dq.as<float>();
  float* ap = ws->ao.as<float>();
  float* fp = ws->ff.as<float>();
  int32_t* unf = ws->unfinished.as<int32_t>();
  int32_t* toks = ws->tok_buf.as<int32_t>();
  const float* ckv = ws->cross_kv.as<float>();
  const int64_t ckv_ld = (int64_t)Ld * 2 * inner;

  const float out_scale = scale_out ? 1.0f / sqrtf((float)d) : 1.0f;
  if (fold_rows(B)) return decode_body_folded(B, L, max_new, eos, pad, s, t0, t1);
  for (int t = t0; t < t1; ++t) {
    for (int l = 0; l < Ld; ++l) {
      const T5Layer& ly = *dec[l];
      float* cl = ws->cache.as<float>() + l * cache_layer;
      SkinnyArgs sq;
      sq.g.A = xp; sq.g.lda = d;
      sq.g.C = cl + (int64_t)t * 3 * inner; sq.g.ldc = (int64_t)Tc * 3 * inner;
      sq.g.M = B; sq.g.N = 3 * inner; sq.g.K = d; sq.rms_w = ly.ln0.as<float>(); sq.rms_eps = T5_EPS;
      MPR_TRY(dec_gemm(sq, ly.pk_qkv, s));
      MPR_TRY(trace(TR_QKV, t, l, sq.g.C, B, 3 * inner, sq.g.ldc, s));
      AttnArgs at;
      at.q = cl + (int64_t)t * 3 * inner; at.q_bs = (int64_t)Tc * 3 * inner; at.q_rs = 3 * inner;
      at.k = cl + inner; at.k_bs = at.q_bs; at.k_rs = 3 * inner;
      at.v = cl + 2 * inner; at.v_bs = at.q_bs; at.v_rs = 3 * inner;
      at.o = ap; at.o_bs = inner; at.o_rs = inner;
      at.B = B; at.H = H; at.Lq = 1; at.Lk = t + 1; at.scale = 1.f; at.causal = 1; at.q_pos0 = t;
      at.rel_tab = dec_tab.as<float>();
      at.lut_radius = lut_radius;
      MPR_TRY(attention(at, s));
      MPR_TRY(trace(TR_SELF_ATT, t, l, ap, B, inner, inner, s));
      SkinnyArgs so;
      so.g.A = ap; so.g.lda = inner; so.g.R = xp;
      so.g.ldr = d; so.g.C = xp; so.g.ldc = d; so.g.M = B; so.g.N = d; so.g.K = inner;
      MPR_TRY(dec_gemm(so, ly.pk_o, s));
      MPR_TRY(trace(TR_O, t, l, xp, B, d, d, s));
      SkinnyArgs cq;
      cq.g.A = xp; cq.g.lda = d; cq.g.C = qp;
      cq.g.ldc = inner; cq.g.M = B; cq.g.N = inner; cq.g.K = d; cq.rms_w = ly.ln1.as<float>();
      cq.rms_eps = T5_EPS;
      MPR_TRY(dec_gemm(cq, ly.pk_cq, s));
      MPR_TRY(trace(TR_CQ, t, l, qp, B, inner, inner, s));
      AttnArgs ca;
      ca.q = qp; ca.q_bs = inner; ca.q_rs = inner;
      ca.k = ckv + (int64_t)l * 2 * inner; ca.k_bs = (int64_t)L * ckv_ld; ca.k_rs = ckv_ld;
      ca.v = ckv + (int64_t)l * 2 * inner + inner; ca.v_bs = ca.k_bs; ca.v_rs = ckv_ld;
      ca.o = ap; ca.o_bs = inner; ca.o_rs = inner;
      ca.B = B; ca.H = H; ca.Lq = 1; ca.Lk = L; ca.scale = 1.f;
      ca.key_mask = maskp; ca.mask_bs = L;
      MPR_TRY(attention(ca, s));
      MPR_TRY(trace(TR_CROSS_ATT, t, l, ap, B, inner, inner, s));
      SkinnyArgs co;
      co.g.A = ap; co.g.lda = inner; co.g.R = xp;
      co.g.ldr = d; co.g.C = xp; co.g.ldc = d; co.g.M = B; co.g.N = d; co.g.K = inner;
      MPR_TRY(dec_gemm(co, ly.pk_co, s));
      MPR_TRY(trace(TR_CO, t, l, xp, B, d, d, s));
      SkinnyArgs fi;
      fi.g.A = xp; fi.g.lda = d; fi.g.C = fp;
      fi.g.ldc = dff; fi.g.M = B; fi.g.N = dff; fi.g.K = d; fi.g.act = ACT_RELU;
      fi.rms_w = ly.ln2.as<float>(); fi.rms_eps = T5_EPS;
      MPR_TRY(dec_gemm(fi, ly.pk_wi, s));
      MPR_TRY(trace(TR_WI, t, l, fp, B, dff, dff, s));
      SkinnyArgs fo;
      fo.g.A = fp; fo.g.lda = dff; fo.g.R = xp;
      fo.g.ldr = d; fo.g.C = xp; fo.g.ldc = d; fo.g.M = B; fo.g.N = d; fo.g.K = dff;
      MPR_TRY(dec_gemm(fo, ly.pk_wo, s));
      MPR_TRY(trace(TR_WO, t, l, xp, B, d, d, s));
    }
    if (tiled_head(B)) {
      // logits = rms(x) . lm_head^T on the tiled GEMM, then the row argmax in 16 parts per row
      // (out_scale > 0 multiplies every logit of a row alike: the argmax does not need it)
      constexpr int HP = 16;
      float* hb = ws->h.as<float>();
      float* lg = ws->logits.as<float>();
      MPR_TRY(rmsnorm(xp, d, B, d, dec_final.as<float>(), T5_EPS, hb, d, s));
      MPR_TRY(trace(TR_HEAD_RMS, t, -1, hb, B, d, d, s));
      GemmArgs g;
      g.A = hb; g.lda = d; g.W = lm_head.as<float>(); g.ldw = d;
      g.C = lg; g.ldc = V; g.M = B; g.N = V; g.K = d;
      MPR_TRY(gemm(g, s));
      MPR_TRY(trace(TR_LOGITS, t, -1, lg, B, V, V, s));
      MPR_TRY(argmax_parts(lg, V, B, V, HP, ws->part_val.as<float>(), ws->part_idx.as<int32_t>(),
                           s));
      MPR_TRY(trace(TR_HEAD_VAL, t, -1, ws->part_val.ptr, B, HP, HP, s));
      MPR_TRY(trace(TR_HEAD_IDX, t, -1, ws->part_idx.ptr, B, HP, HP, s));
      MPR_TRY(greedy_step(ws->part_val.as<float>(), ws->part_idx.as<int32_t>(), HP, B, unf, toks,
                          T1, t + 1, eos, pad, shared.as<float>(), d,
                          t + 1 < max_new ? xp : nullptr, s));
      MPR_TRY(trace(TR_TOKEN, t, -1, toks + t + 1, B, 1, T1, s));
      if (t + 1 < max_new) MPR_TRY(trace(TR_X_NEXT, t, -1, xp, B, d, d, s));
      continue;
    }
    // The argmax head, one launch for all rows (gemm_skinny splits more than 32 rows over blocks
    // of 16; as two 64-row launches it cost 2 x 42 us against 80.8 us per 128-row step).
    SkinnyArgs hd;
    hd.g.A = xp; hd.g.lda = d; hd.g.C = nullptr; hd.g.M = B; hd.g.N = V; hd.g.K = d;
    hd.rms_w = dec_final.as<float>(); hd.rms_eps = T5_EPS; hd.a_scale = out_scale;
    hd.amax_val = ws->part_val.as<float>();
    hd.amax_idx = ws->part_idx.as<int32_t>();
    int np = 0;
    MPR_TRY(dec_gemm(hd, pk_lm_head, s, &np));
    MPR_TRY(trace(TR_HEAD_VAL, t, -1, ws->part_val.ptr, B, np, np, s));
    MPR_TRY(trace(TR_HEAD_IDX, t, -1, ws->part_idx.ptr, B, np, np, s));
    MPR_TRY(greedy_step(ws->part_val.as<float>(), ws->part_idx.as<int32_t>(), np, B, unf, toks, T1,
                        t + 1, eos, pad, shared.as<float>(), d, t + 1 < max_new ? xp : nullptr,
                        s));
    MPR_TRY(trace(TR_TOKEN, t, -1, toks + t + 1, B, 1, T1, s));
    if (t + 1 < max_new) MPR_TRY(trace(TR_X_NEXT, t, -1, xp, B, d, d, s));
  }
  return MPR_OK;
}

// decode_body with the folded chain (build_folded): per layer qkv (RMS fused), self-attention into
// the a half of [a | x], [x1 | u] (one GEMM over [a | x]), cross-attention (query scaled by
// x1's RMS) into the c half of [c | x1 | u], [x2 | z] (one GEMM over [c | x1]), FFN-out (relu on
// load, x2's RMS scale, + x2) into the x half of [a | x].
// Timing bisection (tools/decode_ab.py): MPR_DEBUG_CHAIN_SKIP = a bit mask of the folded chain's
// launch kinds a decode step leaves out (its tokens are then wrong): 1 q|k|v GEMVs, 2 self-
// attentions, 4 o|cq GEMVs, 8 cross-attentions, 16 co|wi GEMVs, 32 FFN-out GEMVs, 64 the argmax
// head, 128 the greedy step.
static int chain_skip() {
  static const int m = [] {
    const char* e = getenv("MPR_DEBUG_CHAIN_SKIP");
    return e ? atoi(e) : 0;
  }();
  return m;
}

int T5Model::decode_body_folded(int B, int L, int max_new, int eos, int pad, hipStream_t s,
                                int t0, int t1) {
  const int skip = chain_skip();
  const int T1 = max_new + 1, Tc = max_new > 0 ? max_new : 1;
  const int64_t cache_layer = (int64_t)B * Tc * 3 * inner;
  const float* maskp = ws->mask_in.as<float>();
  const int64_t ldA = inner + d, ldY = 2 * inner + d, ldZ = d + dff;
  float* ax = ws->ax.as<float>();  // [a | x]
  float* yq = ws->yq.as<float>();  // [c | x1 | u]
  float* hz = ws->hz.as<float>();  // [x2 | z]
  float* x1ss = ws->x1ss.as<float>();  // [B, d / 16] per-tile sums of squares of x1 / x2
  float* x2ss = ws->x2ss.as<float>();
  float* xp = ax + inner;
  int32_t* unf = ws->unfinished.as<int32_t>();
  int32_t* toks = ws->tok_buf.as<int32_t>();
  const float* ckv = ws->cross_kv.as<float>();
  const int64_t ckv_ld = (int64_t)Ld * 2 * inner;
  const float out_scale = scale_out ? 1.0f / sqrtf((float)d) : 1.0f;
  for (int t = t0; t < t1; ++t) {
    for (int l = 0; l < Ld; ++l) {
      const T5Layer& ly = *dec[l];
      float* cl = ws->cache.as<float>() + l * cache_layer;
      AttnArgs at;
      at.q = cl + (int64_t)t * 3 * inner; at.q_bs = (int64_t)Tc * 3 * inner; at.q_rs = 3 * inner;
      at.k = cl + inner; at.k_bs = at.q_bs; at.k_rs = 3 * inner;
      at.v = cl + 2 * inner; at.v_bs = at.q_bs; at.v_rs = 3 * inner;
      at.o = ax; at.o_bs = ldA; at.o_rs = ldA;
      at.B = B; at.H = H; at.Lq = 1; at.Lk = t + 1; at.scale = 1.f; at.causal = 1; at.q_pos0 = t;
      at.rel_tab = dec_tab.as<float>();
      at.lut_radius = lut_radius;
      SkinnyArgs sq;  // q | k | v of this position = rms(x) ln0 Wqkv^T
      sq.g.A = xp; sq.g.lda = ldA;
      sq.g.C = cl + (int64_t)t * 3 * inner; sq.g.ldc = (int64_t)Tc * 3 * inner;
      sq.g.M = B; sq.g.N = 3 * inner; sq.g.K = d; sq.rms_w = ly.ln0.as<float>(); sq.rms_eps = T5_EPS;
      if (!(skip & 1)) MPR_TRY(dec_gemm(sq, ly.pk_qkv, s));
      MPR_TRY(trace(TR_QKV, t, l, sq.g.C, B, 3 * inner, sq.g.ldc, s));
      if (!(skip & 2)) MPR_TRY(attention(at, s));
      MPR_TRY(trace(TR_SELF_ATT, t, l, ax, B, inner, ldA, s));
      SkinnyArgs so;  // [x1 | u] = [a | x] W_ocq^T
      so.g.A = ax; so.g.lda = ldA; so.g.C = yq + inner; so.g.ldc = ldY;
      so.g.M = B; so.g.N = d + inner; so.g.K = inner + d;
      so.ssq_out = x1ss; so.ssq_cols = d;  // x1's per-tile sums of squares (its RMS)
      if (!(skip & 4)) MPR_TRY(dec_gemm(so, ly.pk_ocq, s));
      MPR_TRY(trace(TR_OCQ, t, l, yq + inner, B, d + inner, ldY, s));
      MPR_TRY(trace(TR_X1SS, t, l, x1ss, B, d / 16, d / 16, s));
      AttnArgs ca;  // c = attention(u / rms_scale(x1), K_enc, V_enc)
      ca.q = yq + inner + d; ca.q_bs = ldY; ca.q_rs = ldY;
      ca.k = ckv + (int64_t)l * 2 * inner; ca.k_bs = (int64_t)L * ckv_ld; ca.k_rs = ckv_ld;
      ca.v = ckv + (int64_t)l * 2 * inner + inner; ca.v_bs = ca.k_bs; ca.v_rs = ckv_ld;
      ca.o = yq; ca.o_bs = ldY; ca.o_rs = ldY;
      ca.B = B; ca.H = H; ca.Lq = 1; ca.Lk = L; ca.scale = 1.f;
      ca.key_mask = maskp; ca.mask_bs = L;
      ca.q_rms_part = x1ss; ca.q_rms_nparts = d / 16; ca.q_rms_n = d; ca.q_rms_eps = T5_EPS;
      if (!(skip & 8)) MPR_TRY(attention(ca, s));
      MPR_TRY(trace(TR_CROSS_ATT, t, l, yq, B, inner, ldY, s));
      SkinnyArgs cw;  // [x2 | z] = [c | x1] W_cowi^T
      cw.g.A = yq; cw.g.lda = ldY; cw.g.C = hz; cw.g.ldc = ldZ;
      cw.g.M = B; cw.g.N = d + dff; cw.g.K = inner + d;
      cw.ssq_out = x2ss; cw.ssq_cols = d;
      if (!(skip & 16)) MPR_TRY(dec_gemm(cw, ly.pk_cowi, s));
      MPR_TRY(trace(TR_COWI, t, l, hz, B, d + dff, ldZ, s));
      MPR_TRY(trace(TR_X2SS, t, l, x2ss, B, d / 16, d / 16, s));
      // (Measured and dropped, round 6: the FFN-out with K split over twice the blocks, its two
      // partials summed into the residual stream by the next reader (the next layer's q|k|v, which
      // stored x3, or the head) — tokens unchanged, 16-row step 207-215 vs 211-216 us, but the
      // serving loop's 128-row step 487 vs 434 us: the readers' extra partial loads cost more
      // than the split saves; profiles/r06_decode_chain_parts.txt.)
      SkinnyArgs fo;  // x3 = x2 + (relu(z) Wwo^T) / rms_scale(x2), into the x half of [a | x]
      fo.g.A = hz + d; fo.g.lda = ldZ; fo.g.R = hz; fo.g.ldr = ldZ;
      fo.g.C = xp; fo.g.ldc = ldA; fo.g.M = B; fo.g.N = d; fo.g.K = dff;
      fo.relu_in = true; fo.rs_part = x2ss; fo.rs_nparts = d / 16; fo.rs_n = d;
      fo.rms_eps = T5_EPS;
      if (!(skip & 32)) MPR_TRY(dec_gemm(fo, ly.pk_wo, s));
      MPR_TRY(trace(TR_FO, t, l, xp, B, d, ldA, s));
    }
    SkinnyArgs hd;
    hd.g.A = xp; hd.g.lda = ldA; hd.g.C = nullptr; hd.g.M = B; hd.g.N = V; hd.g.K = d;
    hd.rms_w = dec_final.as<float>(); hd.rms_eps = T5_EPS; hd.a_scale = out_scale;
    hd.amax_val = ws->part_val.as<float>();
    hd.amax_idx = ws->part_idx.as<int32_t>();
    int np = (int)cdiv(V, 16);
    if (!(skip & 64)) MPR_TRY(dec_gemm(hd, pk_lm_head, s, &np));
    MPR_TRY(trace(TR_HEAD_VAL, t, -1, ws->part_val.ptr, B, np, np, s));
    MPR_TRY(trace(TR_HEAD_IDX, t, -1, ws->part_idx.ptr, B, np, np, s));
    if (!(skip & 128))
      MPR_TRY(greedy_step(ws->part_val.as<float>(), ws->part_idx.as<int32_t>(), np, B, unf, toks,
                          T1, t + 1, eos, pad, shared.as<float>(), d,
                          t + 1 < max_new ? xp : nullptr, s, ldA));
    MPR_TRY(trace(TR_TOKEN, t, -1, toks + t + 1, B, 1, T1, s));
    if (t + 1 < max_new) MPR_TRY(trace(TR_X_NEXT, t, -1, xp, B, d, ldA, s));
  }
  return MPR_OK;
}

int T5Model::generate(const float* embeds, const float* mask, int B, int L, int max_new,
                      int start, int eos, int pad, int32_t* out_tokens, hipStream_t s,
                      int slot) {
  return generate_groups(1, &embeds, &mask, &B, &L, max_new, start, eos, pad, &out_tokens, s,
                         slot);
}

namespace {
// [B, Lsrc] rows (row length `w` floats per position) into [B, Ldst] rows, zero beyond Lsrc.
int stage_rows(float* dst, const float* src, int B, int Lsrc, int Ldst, int64_t w,
               hipStream_t s) {
  const size_t row = (size_t)w * 4;
  if (Lsrc == Ldst)
    MPR_HIP(hipMemcpyAsync(dst, src, (size_t)B * Lsrc * row, hipMemcpyDeviceToDevice, s));
  else {
    MPR_HIP(hipMemsetAsync(dst, 0, (size_t)B * Ldst * row, s));
    MPR_HIP(hipMemcpy2DAsync(dst, (size_t)Ldst * row, src, (size_t)Lsrc * row, (size_t)Lsrc * row,
                             B, hipMemcpyDeviceToDevice, s));
  }
  return MPR_OK;
}
}  // namespace

int T5Model::generate_groups(int ng, const float* const* embeds, const float* const* masks,
                             const int* Bs, const int* Ls, int max_new, int start, int eos,
                             int pad, int32_t* const* outs, hipStream_t s, int slot,
                             int stop_chunk, int* steps_run) {
  if (steps_run) *steps_run = 0;
  MPR_TRY(gen_begin(ng, embeds, masks, Bs, Ls, max_new, start, eos, pad, outs, s, slot,
                    stop_chunk, 2));
  int done = 0;
  return gen_poll(slot, true, &done, steps_run, s);
}

int T5Model::gen_begin(int ng, const float* const* embeds, const float* const* masks,
                       const int* Bs, const int* Ls, int max_new, int start, int eos, int pad,
                       int32_t* const* outs, hipStream_t s, int slot, int stop_chunk,
                       int ahead) {
  MPR_TRY(use_slot(slot));
  MPR_REQUIRE(!ws->pend.active,
              "t5 generate: slot %d still has a decode in flight (poll it to the end first)",
              slot);
  MPR_REQUIRE(ahead >= 1 && ahead <= 16, "t5 generate: ahead=%d", ahead);
  MPR_REQUIRE(ng >= 1 && ng <= MAX_GROUPS, "t5 generate: %d batch groups (1 to %d)", ng,
              MAX_GROUPS);
  MPR_REQUIRE(max_new >= 0 && max_new <= 512, "t5 generate: max_new=%d", max_new);
  MPR_REQUIRE(max_new + 1 <= lut_radius, "t5 generate: max_new exceeds lut radius");
  // The source length is bucketed to a multiple of 8 (zero rows, mask 0) so a serving loop
  // with varying prompt lengths replays a few captured graphs instead of capturing one per
  // length.  Masked keys add exact zeros to every softmax sum and rows are independent in
  // every other op, so the real rows' results are bit-identical.  Groups sharing a decode are
  // each encoded at their own bucket (the same launches as a generate() of their own) and
  // then padded the same way to the longest one.
  struct Grp {
    const float *e, *m;
    int B, L, Lb, row0;
    int32_t* out;
  } gr[MAX_GROUPS];
  int n = 0, Btot = 0, Lp = 0;
  int64_t Mg = 0;
  for (int g = 0; g < ng; ++g) {
    MPR_REQUIRE(Bs[g] >= 0 && Bs[g] <= 16, "t5 generate: batch %d > 16 unsupported by the decode path", Bs[g]);
    if (Bs[g] == 0) continue;
    // every key/query offset of the (bucketed) source must have a bias-table entry
    const int Lb = (int)cdiv(Ls[g], 8) * 8;
    MPR_REQUIRE(Ls[g] >= 1 && Lb - 1 <= lut_radius,
                "t5 generate: L=%d (bucketed %d) exceeds the bucket lut radius %d + 1", Ls[g], Lb,
                lut_radius);
    gr[n++] = Grp{embeds[g], masks[g], Bs[g], Ls[g], Lb, Btot, outs[g]};
    Btot += Bs[g];
    Lp = std::max(Lp, Lb);
    Mg += (int64_t)Bs[g] * Lb;  // the batches' encoder rows, stacked
  }
  if (n == 0) {
    ws->pend = T5Work::Pending();  // nothing to decode: polls report done
    return MPR_OK;
  }
  const int L = Lp, B = Btot;
  const int T1 = max_new + 1, Tc = max_new > 0 ? max_new : 1;
  const int64_t M = (int64_t)B * L, Mx = std::max(M, Mg);
  const int nparts = (int)cdiv(V, 16);
  // Every buffer the bodies touch is sized before capture (no allocation inside a graph).
  MPR_TRY(grow(ws->enc_in, (size_t)Mx * d * 4));
  MPR_TRY(grow(ws->mask_in, (size_t)M * 4));
  MPR_TRY(grow(ws->enc_out, (size_t)M * d * 4));
  MPR_TRY(grow(ws->cross_kv, (size_t)M * Ld * 2 * inner * 4));
  MPR_TRY(grow(ws->x, (size_t)Mx * d * 4));
  MPR_TRY(grow(ws->h, (size_t)Mx * d * 4));
  MPR_TRY(grow(ws->qkv, (size_t)Mx * 3 * inner * 4));
  MPR_TRY(grow(ws->ao, (size_t)Mx * (inner > dff ? inner : dff) * 4));
  MPR_TRY(grow(ws->ff, (size_t)Mx * dff * 4));
  MPR_TRY(grow(ws->cache, (size_t)Ld * B * Tc * 3 * inner * 4));
  MPR_TRY(grow(ws->dx, (size_t)B * d * 4));
  MPR_TRY(grow(ws->dq, (size_t)B * inner * 4));
  if (fold_rows(B)) {
    MPR_TRY(grow(ws->ax, (size_t)B * (inner + d) * 4));
    MPR_TRY(grow(ws->yq, (size_t)B * (2 * inner + d) * 4));
    MPR_TRY(grow(ws->hz, (size_t)B * (d + dff) * 4));
    MPR_TRY(grow(ws->x1ss, (size_t)B * (d / 16) * 4));
    MPR_TRY(grow(ws->x2ss, (size_t)B * (d / 16) * 4));
  }
  MPR_TRY(grow(ws->part_val, (size_t)nparts * 16 * MAX_GROUPS * 4));
  MPR_TRY(grow(ws->part_idx, (size_t)nparts * 16 * MAX_GROUPS * 4));
  MPR_TRY(grow(ws->unfinished, (size_t)16 * MAX_GROUPS * 4));
  MPR_TRY(grow(ws->cur_tok, (size_t)16 * MAX_GROUPS * 4));
  MPR_TRY(grow(ws->tok_buf, (size_t)B * T1 * 4));
  if (tiled_head(B)) MPR_TRY(grow(ws->logits, (size_t)B * V * 4));
  if (debug_decode_trace()) {  // every traced output of the call (T5Model::trace)
    const int64_t per_step = (int64_t)B * ((int64_t)Ld * (6 * inner + 6 * d + 2 * dff + d / 8) +
                                           2 * nparts + (tiled_head(B) ? V : 0) + 2 * d + 40);
    MPR_TRY(grow(ws->trace, (size_t)(M * d + M * Ld * 2 * inner + Tc * per_step) * 4));
  }
  if (n > 1) {
    MPR_TRY(grow(ws->mask_enc, (size_t)Mg * 4));
    MPR_TRY(grow(ws->enc_tmp, (size_t)Mg * d * 4));
  }
  auto run = [&](const GraphKey& key, hipStream_t st, auto&& body) -> int {
    return run_graph(key, st, body);
  };
  if (n == 1) {
    const Grp& g = gr[0];
    MPR_TRY(stage_rows(ws->enc_in.as<float>(), g.e, B, g.L, L, d, s));
    MPR_TRY(stage_rows(ws->mask_in.as<float>(), g.m, B, g.L, L, 1, s));
    MPR_TRY(run(GraphKey{0, B, L, max_new, start, 0}, s,
                [&](hipStream_t c) { return encode_body(B, L, max_new, start, c); }));
  } else {
    float* eo = ws->enc_out.as<float>();
    MPR_HIP(hipMemsetAsync(ws->mask_in.ptr, 0, (size_t)M * 4, s));
    bool ragged = false;
    for (int k = 1; k < n; ++k) ragged |= gr[k].Lb != gr[0].Lb;
    if (ragged) MPR_HIP(hipMemsetAsync(eo, 0, (size_t)M * d * 4, s));
    // every batch's inputs at its own bucket, back to back; one grouped encoder pass
    int bs[MAX_GROUPS], lbs[MAX_GROUPS], pack[MAX_GROUPS / 2] = {};
    int64_t r = 0;
    for (int k = 0; k < n; ++k) {
      const Grp& g = gr[k];
      MPR_TRY(stage_rows(ws->enc_in.as<float>() + r * d, g.e, g.B, g.L, g.Lb, d, s));
      MPR_TRY(stage_rows(ws->mask_enc.as<float>() + r, g.m, g.B, g.L, g.Lb, 1, s));
      MPR_HIP(hipMemcpy2DAsync(ws->mask_in.as<float>() + (int64_t)g.row0 * L, (size_t)L * 4, g.m,
                               (size_t)g.L * 4, (size_t)g.L * 4, g.B, hipMemcpyDeviceToDevice,
                               s));
      bs[k] = g.B;
      lbs[k] = g.Lb;
      pack[k / 2] |= (g.B | (g.Lb << 5)) << (16 * (k % 2));  // B <= 16, Lb <= 1024
      r += (int64_t)g.B * g.Lb;
    }
    GraphKey key{2, n};
    for (int k = 0; k < (n + 1) / 2; ++k) key.push_back(pack[k]);
    MPR_TRY(run(key, s,
                [&](hipStream_t c) {
                  // one grouped pass over every batch's stacked rows
                  return encode_multi(n, bs, lbs, ws->enc_in.as<float>(),
                                      ws->mask_enc.as<float>(), ws->enc_tmp.as<float>(), c);
                }));
    r = 0;
    for (int k = 0; k < n; ++k) {
      const Grp& g = gr[k];
      MPR_HIP(hipMemcpy2DAsync(eo + (int64_t)g.row0 * L * d, (size_t)L * d * 4,
                               ws->enc_tmp.as<float>() + r * d, (size_t)g.Lb * d * 4,
                               (size_t)g.Lb * d * 4, g.B, hipMemcpyDeviceToDevice, s));
      r += (int64_t)g.B * g.Lb;
    }
    MPR_TRY(run(GraphKey{3, B, L, max_new, start, 0}, s,
                [&](hipStream_t c) { return init_body(B, L, max_new, start, c); }));
  }
  hipStream_t ds = ws->dec_stream ? ws->dec_stream : s;
  if (ds != s) {
    MPR_HIP(hipEventRecord(ws->ev_fork, s));
    MPR_HIP(hipStreamWaitEvent(ds, ws->ev_fork, 0));
  }
  T5Work::Pending& P = ws->pend;
  P = T5Work::Pending();
  P.B = B; P.L = L; P.max_new = max_new; P.eos = eos; P.pad = pad; P.ds = ds; P.n = n;
  P.ahead = ahead;
  for (int k = 0; k < n; ++k) {
    P.outs[k] = gr[k].out;
    P.row0[k] = gr[k].row0;
    P.rows[k] = gr[k].B;
  }
  if (stop_chunk <= 0 || max_new <= stop_chunk) {
    // one graph of all max_new steps: nothing to poll
    MPR_TRY(run_graph(GraphKey{1, B, L, max_new, eos, pad}, ds,
                      [&](hipStream_t c) { return decode_body(B, L, max_new, eos, pad, c); }));
    P.chunk = 0;
    P.nch = P.launched = 1;
    P.active = true;
    return MPR_OK;
  }
  // Chunks of stop_chunk steps, each a graph of its own, and after each an async copy of the
  // rows' unfinished flags; gen_poll reads them in order and keeps `ahead` chunks unread.
  P.chunk = stop_chunk;
  P.nch = (int)cdiv(max_new, stop_chunk);
  if (ws->h_unf_n < (size_t)P.nch * B) {
    if (ws->h_unf) MPR_HIP(hipHostFree(ws->h_unf));
    ws->h_unf = nullptr;
    ws->h_unf_n = 0;
    MPR_HIP(hipHostMalloc(reinterpret_cast<void**>(&ws->h_unf), (size_t)P.nch * B * 4, 0));
    ws->h_unf_n = (size_t)P.nch * B;
  }
  while ((int)ws->ev_chunk.size() < P.nch) {
    hipEvent_t e;
    MPR_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    ws->ev_chunk.push_back(e);
  }
  P.active = true;
  for (int c = 0; c < std::min(ahead, P.nch); ++c) MPR_TRY(launch_chunk(c));
  return MPR_OK;
}

int T5Model::launch_chunk(int c) {
  T5Work::Pending& P = ws->pend;
  const int t0 = c * P.chunk, t1 = std::min(P.max_new, t0 + P.chunk);
  const int B = P.B, L = P.L, max_new = P.max_new, eos = P.eos, pad = P.pad;
  MPR_TRY(run_graph(GraphKey{100 + c, B, L, max_new * 1024 + P.chunk, eos, pad}, P.ds,
                    [&](hipStream_t cs) {
                      return decode_body(B, L, max_new, eos, pad, cs, t0, t1);
                    }));
  MPR_HIP(hipMemcpyAsync(ws->h_unf + (size_t)c * B, ws->unfinished.ptr, (size_t)B * 4,
                         hipMemcpyDeviceToHost, P.ds));
  MPR_HIP(hipEventRecord(ws->ev_chunk[c], P.ds));
  P.launched = c + 1;
  return MPR_OK;
}

int T5Model::finish_pending(hipStream_t s) {
  T5Work::Pending& P = ws->pend;
  const int T1 = P.max_new + 1;
  for (int k = 0; k < P.n; ++k)
    MPR_HIP(hipMemcpyAsync(P.outs[k], ws->tok_buf.as<int32_t>() + (int64_t)P.row0[k] * T1,
                           (size_t)P.rows[k] * T1 * 4, hipMemcpyDeviceToDevice, P.ds));
  if (P.ds != s) {  // the caller's stream sees the tokens (and may reuse the buffers) after this
    MPR_HIP(hipEventRecord(ws->ev_join, P.ds));
    MPR_HIP(hipStreamWaitEvent(s, ws->ev_join, 0));
  }
  P.steps = P.chunk == 0 ? P.max_new : std::min(P.max_new, P.launched * P.chunk);
  P.active = false;
  return MPR_OK;
}

int T5Model::gen_poll(int slot, bool wait, int* done, int* steps_run, hipStream_t s) {
  MPR_TRY(use_slot(slot));
  T5Work::Pending& P = ws->pend;
  *done = 0;
  if (!P.active) {
    *done = 1;
    if (steps_run) *steps_run = P.steps;
    return MPR_OK;
  }
  for (;;) {
    // read the flags of every completed chunk, oldest first
    while (P.chunk > 0 && !P.stop && P.checked < P.launched) {
      hipEvent_t e = ws->ev_chunk[P.checked];
      if (wait) {
        MPR_HIP(hipEventSynchronize(e));
      } else {
        const hipError_t r = hipEventQuery(e);
        if (r == hipErrorNotReady) break;
        MPR_HIP(r);
      }
      const int32_t* f = ws->h_unf + (size_t)P.checked * P.B;
      bool any = false;
      for (int r = 0; r < P.B && !any; ++r) any = f[r] != 0;
      ++P.checked;
      if (!any) P.stop = true;  // greedy search is over for every row
    }
    if (P.stop || P.launched == P.nch) {
      MPR_TRY(finish_pending(s));
      *done = 1;
      if (steps_run) *steps_run = P.steps;
      return MPR_OK;
    }
    if (P.launched - P.checked < P.ahead) {
      MPR_TRY(launch_chunk(P.launched));
      continue;
    }
    if (!wait) return MPR_OK;
  }
}

int T5Model::set_decode_stream(int slot, hipStream_t ds) {
  MPR_TRY(use_slot(slot));
  if (ds && !ws->ev_fork) {
    MPR_HIP(hipEventCreateWithFlags(&ws->ev_fork, hipEventDisableTiming));
    MPR_HIP(hipEventCreateWithFlags(&ws->ev_join, hipEventDisableTiming));
  }
  ws->dec_stream = ds;
  return MPR_OK;
}

template <class F>
int T5Model::graph_for(const GraphKey& key, hipGraphExec_t* out, F&& body) {
  auto& graphs = ws->graphs;
  auto it = graphs.find(key);
  if (it != graphs.end() && it->second.gen != ws->gen) {
    for (auto& kv : graphs) (void)hipGraphExecDestroy(kv.second.exec);
    graphs.clear();
    it = graphs.end();
  }
  if (it == graphs.end()) {
    if (graphs.size() >= MAX_GRAPHS) {
      for (auto& kv : graphs) (void)hipGraphExecDestroy(kv.second.exec);
      graphs.clear();
    }
    if (!ws->cap_stream)
      MPR_HIP(hipStreamCreateWithFlags(&ws->cap_stream, hipStreamNonBlocking));
    hipGraph_t graph = nullptr;
    const auto t_cap0 = std::chrono::steady_clock::now();
    MPR_HIP(hipStreamBeginCapture(ws->cap_stream, hipStreamCaptureModeThreadLocal));
    const int rc = body(ws->cap_stream);
    const hipError_t ec = hipStreamEndCapture(ws->cap_stream, &graph);
    const auto t_cap1 = std::chrono::steady_clock::now();
    if (rc != MPR_OK) {
      if (graph) (void)hipGraphDestroy(graph);
      return rc;
    }
    MPR_HIP(ec);
    hipGraphExec_t exec = nullptr;
    const hipError_t ei = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    MPR_HIP(ei);
    if (getenv("MPR_GRAPH_LOG")) {  // host cost of each capture
      const auto t_ins = std::chrono::steady_clock::now();
      fprintf(stderr, "[graph] key");
      for (int v : key) fprintf(stderr, " %d", v);
      fprintf(stderr, ": capture %.3f ms, instantiate %.3f ms\n",
              std::chrono::duration<double, std::milli>(t_cap1 - t_cap0).count(),
              std::chrono::duration<double, std::milli>(t_ins - t_cap1).count());
    }
    it = graphs.emplace(key, T5Work::GraphEnt{exec, ws->gen}).first;
  }
  *out = it->second.exec;
  return MPR_OK;
}

template <class F>
int T5Model::run_graph(const GraphKey& key, hipStream_t st, F&& body) {
  if (!graphs_enabled()) return body(st);
  hipGraphExec_t exec = nullptr;
  MPR_TRY(graph_for(key, &exec, body));
  MPR_HIP(hipGraphLaunch(exec, st));
  return MPR_OK;
}

int T5Model::logits_tf(const float* embeds, const float* mask, int B, int L,
                       const int32_t* dec_in, int T, float* logits_out, hipStream_t s) {
  MPR_REQUIRE(T >= 1 && T <= lut_radius, "t5 logits: T=%d", T);
  if (B == 0) return MPR_OK;
  MPR_TRY(grow(ws->enc_out, (size_t)B * L * d * 4));
  MPR_TRY(grow(ws->cross_kv, (size_t)B * L * Ld * 2 * inner * 4));
  MPR_TRY(encode(embeds, mask, B, L, ws->enc_out.as<float>(), s));
  MPR_TRY(cross_kv_project(B, L, s));
  const int M = B * T;
  MPR_TRY(grow(ws->x, (size_t)M * d * 4));
  MPR_TRY(grow(ws->h, (size_t)M * d * 4));
  MPR_TRY(grow(ws->qkv, (size_t)M * 3 * inner * 4));
  MPR_TRY(grow(ws->ao, (size_t)M * inner * 4));
  MPR_TRY(grow(ws->dq, (size_t)M * inner * 4));
  MPR_TRY(grow(ws->ff, (size_t)M * dff * 4));
  float* xp = ws->x.as<float>();
  float* hp = ws->h.as<float>();
  float* qp = ws->qkv.as<float>();
  float* ap = ws->ao.as<float>();
  float* cqp = ws->dq.as<float>();
  float* fp = ws->ff.as<float>();
  const float* ckv = ws->cross_kv.as<float>();
  const int64_t ckv_ld = (int64_t)Ld * 2 * inner;
  MPR_TRY(embed_gather(shared.as<float>(), dec_in, T, B, T, d, nullptr, xp, (int64_t)T * d, 0, s));
  for (int l = 0; l < Ld; ++l) {
    const T5Layer& ly = *dec[l];
    MPR_TRY(rmsnorm(xp, d, M, d, ly.ln0.as<float>(), T5_EPS, hp, d, s));
    GemmArgs g;
    g.A = hp; g.lda = d; g.W = ly.qkv.as<float>(); g.ldw = d; g.C = qp; g.ldc = 3 * inner;
    g.M = M; g.N = 3 * inner; g.K = d;
    MPR_TRY(gemm(g, s));
    AttnArgs at;
    at.q = qp; at.q_bs = (int64_t)T * 3 * inner; at.q_rs = 3 * inner;
    at.k = qp + inner; at.k_bs = at.q_bs; at.k_rs = 3 * inner;
    at.v = qp + 2 * inner; at.v_bs = at.q_bs; at.v_rs = 3 * inner;
    at.o = ap; at.o_bs = (int64_t)T * inner; at.o_rs = inner;
    at.B = B; at.H = H; at.Lq = T; at.Lk = T; at.scale = 1.f; at.causal = 1;
    at.rel_tab = dec_tab.as<float>();
    at.lut_radius = lut_radius;
    MPR_TRY(attention(at, s));
    GemmArgs o;
    o.A = ap; o.lda = inner; o.W = ly.o.as<float>(); o.ldw = inner; o.R = xp; o.ldr = d;
    o.C = xp; o.ldc = d; o.M = M; o.N = d; o.K = inner;
    MPR_TRY(gemm(o, s));
    MPR_TRY(rmsnorm(xp, d, M, d, ly.ln1.as<float>(), T5_EPS, hp, d, s));
    GemmArgs cq;
    cq.A = hp; cq.lda = d; cq.W = ly.cq.as<float>(); cq.ldw = d; cq.C = cqp; cq.ldc = inner;
    cq.M = M; cq.N = inner; cq.K = d;
    MPR_TRY(gemm(cq, s));
    AttnArgs ca;
    ca.q = cqp; ca.q_bs = (int64_t)T * inner; ca.q_rs = inner;
    ca.k = ckv + (int64_t)l * 2 * inner; ca.k_bs = (int64_t)L * ckv_ld; ca.k_rs = ckv_ld;
    ca.v = ckv + (int64_t)l * 2 * inner + inner; ca.v_bs = ca.k_bs; ca.v_rs = ckv_ld;
    ca.o = ap; ca.o_bs = (int64_t)T * inner; ca.o_rs = inner;
    ca.B = B; ca.H = H; ca.Lq = T; ca.Lk = L; ca.scale = 1.f;
    ca.key_mask = mask; ca.mask_bs = L;
    MPR_TRY(attention(ca, s));
    GemmArgs co;
    co.A = ap; co.lda = inner; co.W = ly.co.as<float>(); co.ldw = inner; co.R = xp; co.ldr = d;
    co.C = xp; co.ldc = d; co.M = M; co.N = d; co.K = inner;
    MPR_TRY(gemm(co, s));
    MPR_TRY(rmsnorm(xp, d, M, d, ly.ln2.as<float>(), T5_EPS, hp, d, s));
    GemmArgs f;
    f.A = hp; f.lda = d; f.W = ly.wi.as<float>(); f.ldw = d; f.C = fp; f.ldc = dff;
    f.M = M; f.N = dff; f.K = d; f.act = ACT_RELU;
    MPR_TRY(gemm(f, s));
    GemmArgs w;
    w.A = fp; w.lda = dff; w.W = ly.wo.as<float>(); w.ldw = dff; w.R = xp; w.ldr = d;
    w.C = xp; w.ldc = d; w.M = M; w.N = d; w.K = dff;
    MPR_TRY(gemm(w, s));
  }
  // final norm, then * d^-0.5 (the reference's op order, modeling_t5.py scale_decoder_outputs)
  MPR_TRY(rmsnorm(xp, d, M, d, dec_final.as<float>(), T5_EPS, hp, d, s));
  if (scale_out) MPR_TRY(scale_inplace(hp, (int64_t)M * d, 1.0f / sqrtf((float)d), s));
  GemmArgs hd;
  hd.A = hp; hd.lda = d; hd.W = lm_head.as<float>(); hd.ldw = d; hd.C = logits_out; hd.ldc = V;
  hd.M = M; hd.N = V; hd.K = d;
  MPR_TRY(gemm(hd, s));
  return MPR_OK;
}

}  // namespace mpr
