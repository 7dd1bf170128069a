// trainer.hip — the T5 training step issued natively (main.py:177-188,
// ``loss = model(batch); loss.backward()`` on architectures/T5VisionModel.py:219-234, i.e.
// transformers' T5ForConditionalGeneration(inputs_embeds, attention_mask, labels).loss and the
// autograd backward of it).
//
// train.py composed the same forward / backward from Python, one ctypes call per kernel: ~450
// launches a step at ~12-15 us of host time each left the GPU waiting on the host through the
// decoder (M = B*T rows: kernels of a few us).  Here one call runs the whole forward (activations
// into a tape arena) and one the whole backward (temporaries in a per-layer scratch arena,
// parameter gradients written straight into the caller's buffers), on the kernels of train.hip
// and the tiled split-bf16 GEMM — the same launches in the same order as train.py's, so the
// results are the same bits.
//
// Layout per forward (the tape): the input dropout of inputs_embeds, per encoder layer the
// residual stream, RMSNorm outputs and 1/rms, the stacked q|k|v weight and its packed projection
// [B*L, 3 inner], attention probabilities [B, H, L, L], attention output, FFN activation; the
// encoder output, every decoder layer's cross k|v of it in one packed [B*L, 2 Ld inner] buffer,
// the decoder's per-layer tensors likewise, the logits [B*T, V].
#include <cmath>
#include <cstring>
#include <vector>

#include "models.h"

extern "C" {
int mpr_gemm_f32(const float* A, int64_t lda, const float* W, int64_t ldw, float* C, int64_t ldc,
                 int32_t M, int32_t N, int32_t K, const float* R, int64_t ldr, int32_t act,
                 void* stream);
int mpr_gemm_f32_splitk(const float* A, int64_t lda, const float* W, int64_t ldw, float* C,
                        int64_t ldc, int32_t M, int32_t N, int32_t K, const float* R, int64_t ldr,
                        int32_t act, int32_t splits, float* partial, void* stream);
int mpr_transpose(const float* in, int64_t rows, int64_t cols, int64_t ld_in, float* out,
                  int64_t ld_out, void* stream);
int mpr_rmsnorm_fwd(const float* x, int32_t M, int32_t D, const float* w, float eps, float scale,
                    float* y, float* rstd, void* stream);
int mpr_rmsnorm_bwd(const float* x, int32_t M, int32_t D, const float* w, const float* rstd,
                    const float* dy, float scale, float* dx, int32_t accumulate, float* dw,
                    float* dw_partial, void* stream);
int mpr_attn_train_fwd(const float* q, int64_t q_bs, int64_t q_rs, const float* k, int64_t k_bs,
                       int64_t k_rs, const float* v, int64_t v_bs, int64_t v_rs, int32_t B,
                       int32_t H, int32_t Lq, int32_t Lk, int32_t causal, const float* key_mask,
                       const float* rel, int32_t R, float* o, int64_t o_bs, int64_t o_rs, float* P,
                       uint64_t drop_seed, uint32_t drop_site, uint32_t drop_thresh,
                       float drop_scale, void* stream);
int mpr_attn_train_bwd(const float* q, int64_t q_bs, int64_t q_rs, const float* k, int64_t k_bs,
                       int64_t k_rs, const float* v, int64_t v_bs, int64_t v_rs, int32_t B,
                       int32_t H, int32_t Lq, int32_t Lk, const float* P, const float* dO,
                       int64_t do_bs, int64_t do_rs, float* dS, float* dq, int64_t dq_bs,
                       int64_t dq_rs, float* dk, int64_t dk_bs, int64_t dk_rs, float* dv,
                       int64_t dv_bs, int64_t dv_rs, float* drel, int32_t R, uint64_t drop_seed,
                       uint32_t drop_site, uint32_t drop_thresh, float drop_scale, void* stream);
int mpr_dropout(const float* x, int64_t n, uint64_t seed, uint32_t site, uint32_t thresh,
                float scale, const float* residual, float* y, void* stream);
int mpr_rel_gather(const float* table, const int32_t* lut, int32_t R, int32_t H, float* rel,
                   void* stream);
int mpr_rel_scatter(const float* drel, const int32_t* lut, int32_t R, int32_t num_buckets,
                    int32_t H, float* dtable, void* stream);
int mpr_relu_bwd(const float* y, const float* dy, int64_t n, float* dx, void* stream);
int mpr_ce_train(const float* logits, int64_t n, int32_t V, const int32_t* labels,
                 float loss_scale, float grad_scale, const float* grad_mult, float* row_loss,
                 float* loss, float* dlogits, int64_t ld_dlogits, void* stream);
int mpr_gather_rows(const float* table, const int32_t* ids, int64_t n, int32_t d, float* out,
                    void* stream);
int mpr_embed_bwd(const float* dY, int32_t d, const int32_t* uniq, const int32_t* offs,
                  const int32_t* pos, int32_t n_uniq, float* dW, void* stream);
}

namespace mpr {
namespace {

constexpr float T5_TRAIN_EPS = 1e-6f;
constexpr int ACT_RELU_T = 2;
// dropout sites (train.py dropout_site): ((stack * 256 + layer) * 8 + kind), layer 255 for the
// stack-level sites
enum { D_IN = 0, D_FINAL, D_SELF_P, D_SELF_OUT, D_CROSS_P, D_CROSS_OUT, D_FFN_ACT, D_FFN_OUT };
inline uint32_t site(int stack, int layer, int kind) {
  return (uint32_t)((stack * 256 + layer) * 8 + kind);
}

// Bump allocator over device chunks: reset per use, chunks kept (stream-ordered reuse: the calls
// that use an arena are serialized on one stream).  mark / rewind free a layer's temporaries.
struct Arena {
  std::vector<std::unique_ptr<DevBuf>> chunks;
  size_t ci = 0, off = 0;
  void reset() { ci = 0; off = 0; }
  std::pair<size_t, size_t> mark() const { return {ci, off}; }
  void rewind(std::pair<size_t, size_t> m) { ci = m.first; off = m.second; }
  float* get(int64_t n) {
    const size_t bytes = ((size_t)std::max<int64_t>(n, 1) * 4 + 255) / 256 * 256;
    while (ci < chunks.size()) {
      if (off + bytes <= chunks[ci]->bytes) {
        float* p = reinterpret_cast<float*>(static_cast<char*>(chunks[ci]->ptr) + off);
        off += bytes;
        return p;
      }
      ++ci;
      off = 0;
    }
    auto c = std::make_unique<DevBuf>();
    if (c->ensure(std::max<size_t>(bytes, (size_t)64 << 20)) != MPR_OK) return nullptr;
    chunks.push_back(std::move(c));
    ci = chunks.size() - 1;
    off = bytes;
    return chunks[ci]->as<float>();
  }
};

struct Drop {
  uint64_t seed = 0;
  uint32_t thresh = 0;
  float scale = 1.f;
  bool on() const { return thresh != 0; }
};

struct EncTape {
  float *x0, *n1, *r1, *Wqkv, *qkv, *a, *P, *x1, *n2, *r2, *f;
};
struct DecTape {
  float *g0, *n1, *r1, *Wqkv, *qkv, *a, *P, *g1, *n2, *r2, *cq, *ca, *cP, *g2, *n3, *r3, *f;
};
struct Tape {
  bool busy = false;
  Arena ar;
  int B = 0, L = 0, T = 0, Re = 0, Rd = 0;
  Drop dr;
  const int32_t* labels = nullptr;  // the caller keeps these alive until the backward
  std::vector<EncTape> enc;
  std::vector<DecTape> dec;
  float *enc_in, *enc_r, *enc_out, *Wckv, *ckv, *dec_in, *dec_r, *hs, *logits;
};

}  // namespace

struct T5Trainer : mpr_model {
  T5Trainer() : mpr_model(T5_TRAIN) {}
  int d = 0, dkv = 0, H = 0, dff = 0, Le = 0, Ld = 0, V = 0, nb = 0, scale_out = 1, inner = 0;
  int radius = 0;
  DevBuf enc_lut, dec_lut;  // bucket of offset r - radius, r in [0, 2 radius]
  std::vector<int32_t> enc_lut_h, dec_lut_h;  // host copies (grown on demand, grow_luts)
  std::vector<std::unique_ptr<Tape>> tapes;
  Arena scratch;  // the backward's temporaries
  hipStream_t s = nullptr;

  // Relative positions beyond the LUT radius: T5's buckets saturate past max_distance (every
  // |offset| >= max_distance of one sign shares the last bucket of that sign,
  // modeling_t5.py _relative_position_bucket), so the tables extend exactly by repeating their
  // end entries (checked at create: radius >= max_distance there).  Tapes recorded before a
  // growth stay valid: both tables stay centred on offset 0.
  int grow_luts(int R) {
    const int R2 = std::max(R, 2 * radius);
    const size_t nr = 2 * (size_t)R2 + 1, pad = (size_t)(R2 - radius);
    for (auto* h : {&enc_lut_h, &dec_lut_h}) {
      std::vector<int32_t> g(nr);
      for (size_t i = 0; i < nr; ++i) {
        const size_t j = i < pad ? 0 : std::min(i - pad, h->size() - 1);
        g[i] = (*h)[j];
      }
      h->swap(g);
    }
    MPR_HIP(hipStreamSynchronize(s));  // the old tables may be read by queued work
    enc_lut.release();
    dec_lut.release();
    MPR_TRY(enc_lut.ensure(nr * 4));
    MPR_TRY(dec_lut.ensure(nr * 4));
    MPR_HIP(hipMemcpy(enc_lut.ptr, enc_lut_h.data(), nr * 4, hipMemcpyHostToDevice));
    MPR_HIP(hipMemcpy(dec_lut.ptr, dec_lut_h.data(), nr * 4, hipMemcpyHostToDevice));
    radius = R2;
    return MPR_OK;
  }
  int nparams() const { return 5 + 8 * Le + 13 * Ld; }

  // parameter order of train.py t5_param_names
  const float* const* P = nullptr;
  const float* shared() const { return P[0]; }
  const float* enc_rel() const { return P[1]; }
  const float* dec_rel() const { return P[2]; }
  const float* enc_final() const { return P[3]; }
  const float* dec_final() const { return P[4]; }
  int ep(int l, int j) const { return 5 + 8 * l + j; }            // ln0 q k v o ln1 wi wo
  int dp(int l, int j) const { return 5 + 8 * Le + 13 * l + j; }  // ln0 q k v o ln1 cq ck cv co
                                                                   // ln2 wi wo

  // ---- the train.py helpers, on this stream ----------------------------------------------------
  static int splits(int M, int N, int K) {
    const int64_t tiles = cdiv(M, 64) * cdiv(N, 64);
    if (tiles >= 128 || K < 1024) return 1;
    return (int)std::max<int64_t>(1, std::min<int64_t>({16, cdiv(256, tiles), K / 256}));
  }
  // C [M, N] = act(A [M, K] (row stride lda) W [N, K]^T (row stride ldw)) + R (row stride N)
  int gemm(Arena& ar, const float* A, int64_t lda, const float* W, int64_t ldw, float* C, int M,
           int N, int K, const float* R = nullptr, int act = 0) {
    const int sp = splits(M, N, K);
    if (sp > 1) {
      float* part = ar.get((int64_t)sp * M * N);
      MPR_REQUIRE(part, "trainer: out of device memory");
      return mpr_gemm_f32_splitk(A, lda, W, ldw, C, N, M, N, K, R, R ? N : 0, act, sp, part, s);
    }
    return mpr_gemm_f32(A, lda, W, ldw, C, N, M, N, K, R, R ? N : 0, act, s);
  }
  static int64_t r4(int64_t n) { return (n + 3) / 4 * 4; }
  // x [r, c] (row stride ld) -> [c, r4]
  float* transpose(Arena& ar, const float* x, int64_t r, int64_t c, int64_t ld) {
    float* out = ar.get(c * r4(r));
    if (!out || mpr_transpose(x, r, c, ld, out, r4(r), s) != MPR_OK) return nullptr;
    return out;
  }
  // y = x W^T (x [M, K] row stride ldx, W [N, K]): dx (+)= dy W, dW = dy^T x (dy row stride ldy)
  // (Measured and reverted, round 6: the split-bf16 tiles reading dy / x / W K-major in place —
  // bit-identical, no transpose launches — as four scalar loads per float4 or as 4 x 4 blocks
  // scattered into LDS: the GEMMs' own time rose 0.85-1.6 ms per step against ~0.3 ms of
  // transposes saved; git show 49e0c84, profiles/r06_train_kmajor_ab.txt.)
  int linear_bwd(Arena& ar, const float* x, int64_t ldx, const float* W, int N, int K, int M,
                 const float* dy, int64_t ldy, float* dx, bool dx_acc, float* dW,
                 const float* xt = nullptr) {
    if (dW) {
      const float* dyt = transpose(ar, dy, M, N, ldy);
      const float* xT = xt ? xt : transpose(ar, x, M, K, ldx);
      MPR_REQUIRE(dyt && xT, "trainer: out of device memory");
      MPR_TRY(gemm(ar, dyt, r4(M), xT, r4(M), dW, N, K, (int)r4(M)));
    }
    if (dx) {
      const float* Wt = transpose(ar, W, N, K, K);
      MPR_REQUIRE(Wt, "trainer: out of device memory");
      MPR_TRY(gemm(ar, dy, ldy, Wt, r4(N), dx, M, K, (int)r4(N), dx_acc ? dx : nullptr));
    }
    return MPR_OK;
  }
  float* drop(Arena& ar, const float* x, int64_t n, const Drop& dr, uint32_t st,
              const float* residual = nullptr) {
    float* y = ar.get(n);
    if (!y || mpr_dropout(x, n, dr.seed, st, dr.thresh, dr.scale, residual, y, s) != MPR_OK)
      return nullptr;
    return y;
  }
  // gradient through a dropout site (g itself without dropout)
  const float* dmask(Arena& ar, const float* g, int64_t n, const Drop& dr, uint32_t st) {
    return dr.on() ? drop(ar, g, n, dr, st) : g;
  }
  int rms_fwd(const float* x, int M, const float* w, float scale, float* y, float* r) {
    return mpr_rmsnorm_fwd(x, M, d, w, T5_TRAIN_EPS, scale, y, r, s);
  }
  int rms_bwd(Arena& ar, const float* x, int M, const float* w, const float* rstd,
              const float* dy, float* dx, bool acc, float* dw, float scale = 1.f) {
    float* part = ar.get(cdiv(M, 64) * d);
    float* dwt = dw ? dw : ar.get(d);
    MPR_REQUIRE(part && dwt, "trainer: out of device memory");
    return mpr_rmsnorm_bwd(x, M, d, w, rstd, dy, scale, dx, acc ? 1 : 0, dwt, part, s);
  }
  // R + dropout(a W^T) / R + a W^T
  int proj_res(Arena& ar, const float* a, int64_t lda, const float* W, int N, int K, int M,
               const float* R, const Drop& dr, uint32_t st, float* out) {
    if (!dr.on()) return gemm(ar, a, lda, W, K, out, M, N, K, R);
    float* y = ar.get((int64_t)M * N);
    MPR_REQUIRE(y, "trainer: out of device memory");
    MPR_TRY(gemm(ar, a, lda, W, K, y, M, N, K));
    return mpr_dropout(y, (int64_t)M * N, dr.seed, st, dr.thresh, dr.scale, R, out, s);
  }
  int attn_fwd(const float* q, int64_t qs, const float* k, int64_t ks, const float* v, int64_t vs,
               int B, int Lq, int Lk, bool causal, const float* mask, const float* rel, int R,
               const Drop& dr, uint32_t st, float* o, float* Pm) {
    return mpr_attn_train_fwd(q, Lq * qs, qs, k, Lk * ks, ks, v, Lk * vs, vs, B, H, Lq, Lk,
                              causal ? 1 : 0, mask, rel, R, o, (int64_t)Lq * inner, inner, Pm,
                              dr.seed, dr.on() ? st : 0, dr.thresh, dr.scale, s);
  }
  int attn_bwd(Arena& ar, const float* q, int64_t qs, const float* k, int64_t ks, const float* v,
               int64_t vs, const float* Pm, const float* dO, int B, int Lq, int Lk, float* drel,
               int R, const Drop& dr, uint32_t st, float* dq, int64_t dqs, float* dk, int64_t dks,
               float* dv, int64_t dvs) {
    float* dS = ar.get((int64_t)B * H * Lq * Lk);
    MPR_REQUIRE(dS, "trainer: out of device memory");
    return mpr_attn_train_bwd(q, Lq * qs, qs, k, Lk * ks, ks, v, Lk * vs, vs, B, H, Lq, Lk, Pm,
                              dO, (int64_t)Lq * inner, inner, dS, dq, Lq * dqs, dqs, dk,
                              Lk * dks, dks, dv, Lk * dvs, dvs, drel, R, dr.seed,
                              dr.on() ? st : 0, dr.thresh, dr.scale, s);
  }
  // the [n, K] parameters ids... stacked row-wise into out
  int stack(const std::vector<int>& ids, int n, int K, float* out) {
    for (size_t j = 0; j < ids.size(); ++j)
      MPR_HIP(hipMemcpyAsync(out + j * (int64_t)n * K, P[ids[j]], (size_t)n * K * 4,
                             hipMemcpyDeviceToDevice, s));
    return MPR_OK;
  }

  int forward(Tape& tp, const float* emb, const float* mask, const int32_t* dec_ids,
              const int32_t* labels, float loss_scale, float* loss);
  int backward(Tape& tp, const float* dloss, float grad_scale, const int32_t* uniq,
               const int32_t* offs, const int32_t* pos, int n_uniq, float* const* grads,
               float* d_emb);
};

#define TR_GET(var, n)                                                  \
  float* var = ar.get(n);                                               \
  MPR_REQUIRE(var, "trainer: out of device memory (%lld floats)", (long long)(n))

int T5Trainer::forward(Tape& tp, const float* emb, const float* mask, const int32_t* dec_ids,
                       const int32_t* labels, float loss_scale, float* loss) {
  Arena& ar = tp.ar;
  ar.reset();
  const int B = tp.B, L = tp.L, T = tp.T, I = inner;
  const int Me = B * L, Md = B * T;
  const Drop& dr = tp.dr;
  tp.labels = labels;
  tp.Re = std::max(L, 1);
  tp.Rd = std::max(T, 1);
  if (std::max(tp.Re, tp.Rd) > radius) MPR_TRY(grow_luts(std::max(tp.Re, tp.Rd)));
  TR_GET(rel_e, (int64_t)(2 * tp.Re + 1) * H);
  TR_GET(rel_d, (int64_t)(2 * tp.Rd + 1) * H);
  MPR_TRY(mpr_rel_gather(enc_rel(), enc_lut.as<int32_t>() + (radius - tp.Re), tp.Re, H, rel_e, s));
  MPR_TRY(mpr_rel_gather(dec_rel(), dec_lut.as<int32_t>() + (radius - tp.Rd), tp.Rd, H, rel_d, s));
  // encoder
  TR_GET(x, (int64_t)Me * d);
  if (dr.on())
    MPR_TRY(mpr_dropout(emb, (int64_t)Me * d, dr.seed, site(0, 255, D_IN), dr.thresh, dr.scale,
                        nullptr, x, s));
  else
    MPR_HIP(hipMemcpyAsync(x, emb, (size_t)Me * d * 4, hipMemcpyDeviceToDevice, s));
  tp.enc.assign(Le, EncTape{});
  for (int l = 0; l < Le; ++l) {
    EncTape& t = tp.enc[l];
    t.x0 = x;
    TR_GET(n1, (int64_t)Me * d);
    TR_GET(r1, Me);
    MPR_TRY(rms_fwd(x, Me, P[ep(l, 0)], 1.f, n1, r1));
    TR_GET(Wqkv, (int64_t)3 * I * d);
    MPR_TRY(stack({ep(l, 1), ep(l, 2), ep(l, 3)}, I, d, Wqkv));
    TR_GET(qkv, (int64_t)Me * 3 * I);
    MPR_TRY(gemm(ar, n1, d, Wqkv, d, qkv, Me, 3 * I, d));
    TR_GET(a, (int64_t)Me * I);
    TR_GET(Pm, (int64_t)B * H * L * L);
    MPR_TRY(attn_fwd(qkv, 3 * I, qkv + I, 3 * I, qkv + 2 * I, 3 * I, B, L, L, false, mask, rel_e,
                     tp.Re, dr, site(0, l, D_SELF_P), a, Pm));
    TR_GET(x1, (int64_t)Me * d);
    MPR_TRY(proj_res(ar, a, I, P[ep(l, 4)], d, I, Me, x, dr, site(0, l, D_SELF_OUT), x1));
    TR_GET(n2, (int64_t)Me * d);
    TR_GET(r2, Me);
    MPR_TRY(rms_fwd(x1, Me, P[ep(l, 5)], 1.f, n2, r2));
    TR_GET(f, (int64_t)Me * dff);
    MPR_TRY(gemm(ar, n2, d, P[ep(l, 6)], d, f, Me, dff, d, nullptr, ACT_RELU_T));
    const float* fd = dr.on() ? drop(ar, f, (int64_t)Me * dff, dr, site(0, l, D_FFN_ACT)) : f;
    MPR_REQUIRE(fd, "trainer: out of device memory");
    TR_GET(xn, (int64_t)Me * d);
    MPR_TRY(proj_res(ar, fd, dff, P[ep(l, 7)], d, dff, Me, x1, dr, site(0, l, D_FFN_OUT), xn));
    t.n1 = n1; t.r1 = r1; t.Wqkv = Wqkv; t.qkv = qkv; t.a = a; t.P = Pm; t.x1 = x1; t.n2 = n2;
    t.r2 = r2; t.f = f;
    x = xn;
  }
  tp.enc_in = x;
  TR_GET(encn, (int64_t)Me * d);
  TR_GET(enc_r, Me);
  MPR_TRY(rms_fwd(x, Me, enc_final(), 1.f, encn, enc_r));
  tp.enc_r = enc_r;
  float* enc = encn;
  if (dr.on()) {
    enc = drop(ar, encn, (int64_t)Me * d, dr, site(0, 255, D_FINAL));
    MPR_REQUIRE(enc, "trainer: out of device memory");
  }
  tp.enc_out = enc;
  // every decoder layer's cross k | v of the encoder output in one GEMM
  tp.Wckv = tp.ckv = nullptr;
  if (Ld) {
    TR_GET(Wckv, (int64_t)2 * Ld * I * d);
    std::vector<int> ids;
    for (int l = 0; l < Ld; ++l) {
      ids.push_back(dp(l, 7));
      ids.push_back(dp(l, 8));
    }
    MPR_TRY(stack(ids, I, d, Wckv));
    TR_GET(ckv, (int64_t)Me * 2 * Ld * I);
    MPR_TRY(gemm(ar, enc, d, Wckv, d, ckv, Me, 2 * Ld * I, d));
    tp.Wckv = Wckv;
    tp.ckv = ckv;
  }
  // decoder
  TR_GET(g0e, (int64_t)Md * d);
  MPR_TRY(mpr_gather_rows(shared(), dec_ids, Md, d, g0e, s));
  float* g = g0e;
  if (dr.on()) {
    g = drop(ar, g0e, (int64_t)Md * d, dr, site(1, 255, D_IN));
    MPR_REQUIRE(g, "trainer: out of device memory");
  }
  const int64_t ckv_ld = (int64_t)2 * Ld * I;
  tp.dec.assign(Ld, DecTape{});
  for (int l = 0; l < Ld; ++l) {
    DecTape& t = tp.dec[l];
    t.g0 = g;
    TR_GET(n1, (int64_t)Md * d);
    TR_GET(r1, Md);
    MPR_TRY(rms_fwd(g, Md, P[dp(l, 0)], 1.f, n1, r1));
    TR_GET(Wqkv, (int64_t)3 * I * d);
    MPR_TRY(stack({dp(l, 1), dp(l, 2), dp(l, 3)}, I, d, Wqkv));
    TR_GET(qkv, (int64_t)Md * 3 * I);
    MPR_TRY(gemm(ar, n1, d, Wqkv, d, qkv, Md, 3 * I, d));
    TR_GET(a, (int64_t)Md * I);
    TR_GET(Pm, (int64_t)B * H * T * T);
    MPR_TRY(attn_fwd(qkv, 3 * I, qkv + I, 3 * I, qkv + 2 * I, 3 * I, B, T, T, true, nullptr,
                     rel_d, tp.Rd, dr, site(1, l, D_SELF_P), a, Pm));
    TR_GET(g1, (int64_t)Md * d);
    MPR_TRY(proj_res(ar, a, I, P[dp(l, 4)], d, I, Md, g, dr, site(1, l, D_SELF_OUT), g1));
    TR_GET(n2, (int64_t)Md * d);
    TR_GET(r2, Md);
    MPR_TRY(rms_fwd(g1, Md, P[dp(l, 5)], 1.f, n2, r2));
    TR_GET(cq, (int64_t)Md * I);
    MPR_TRY(gemm(ar, n2, d, P[dp(l, 6)], d, cq, Md, I, d));
    TR_GET(ca, (int64_t)Md * I);
    TR_GET(cP, (int64_t)B * H * T * L);
    MPR_TRY(attn_fwd(cq, I, tp.ckv + 2 * l * I, ckv_ld, tp.ckv + (2 * l + 1) * I, ckv_ld, B, T, L,
                     false, mask, nullptr, 0, dr, site(1, l, D_CROSS_P), ca, cP));
    TR_GET(g2, (int64_t)Md * d);
    MPR_TRY(proj_res(ar, ca, I, P[dp(l, 9)], d, I, Md, g1, dr, site(1, l, D_CROSS_OUT), g2));
    TR_GET(n3, (int64_t)Md * d);
    TR_GET(r3, Md);
    MPR_TRY(rms_fwd(g2, Md, P[dp(l, 10)], 1.f, n3, r3));
    TR_GET(f, (int64_t)Md * dff);
    MPR_TRY(gemm(ar, n3, d, P[dp(l, 11)], d, f, Md, dff, d, nullptr, ACT_RELU_T));
    const float* fd = dr.on() ? drop(ar, f, (int64_t)Md * dff, dr, site(1, l, D_FFN_ACT)) : f;
    MPR_REQUIRE(fd, "trainer: out of device memory");
    TR_GET(gn, (int64_t)Md * d);
    MPR_TRY(proj_res(ar, fd, dff, P[dp(l, 12)], d, dff, Md, g2, dr, site(1, l, D_FFN_OUT), gn));
    t.n1 = n1; t.r1 = r1; t.Wqkv = Wqkv; t.qkv = qkv; t.a = a; t.P = Pm; t.g1 = g1; t.n2 = n2;
    t.r2 = r2; t.cq = cq; t.ca = ca; t.cP = cP; t.g2 = g2; t.n3 = n3; t.r3 = r3; t.f = f;
    g = gn;
  }
  tp.dec_in = g;
  const float sc = scale_out ? (float)(1.0 / std::sqrt((double)d)) : 1.f;
  TR_GET(hsn, (int64_t)Md * d);
  TR_GET(dec_r, Md);
  MPR_TRY(rms_fwd(g, Md, dec_final(), sc, hsn, dec_r));
  tp.dec_r = dec_r;
  float* hs = hsn;
  if (dr.on()) {
    hs = drop(ar, hsn, (int64_t)Md * d, dr, site(1, 255, D_FINAL));
    MPR_REQUIRE(hs, "trainer: out of device memory");
  }
  tp.hs = hs;
  TR_GET(logits, (int64_t)Md * V);
  MPR_TRY(gemm(ar, hs, d, shared(), d, logits, Md, V, d));
  tp.logits = logits;
  TR_GET(row_loss, Md);
  return mpr_ce_train(logits, Md, V, labels, loss_scale, 0.f, nullptr, row_loss, loss, nullptr, 0,
                      s);
}

// grads[i] of parameter i (nullptr: not wanted) — the row blocks of a stacked weight's gradient
// C [sum rows, K] of one GEMM land in their parameters' buffers: straight when they are adjacent
// in memory, else through a scratch result and one batched copy.
int T5Trainer::backward(Tape& tp, const float* dloss, float grad_scale, const int32_t* uniq,
                        const int32_t* offs, const int32_t* pos, int n_uniq, float* const* grads,
                        float* d_emb) {
  Arena& ar = scratch;
  ar.reset();
  const int B = tp.B, L = tp.L, T = tp.T, I = inner;
  const int Me = B * L, Md = B * T;
  const Drop& dr = tp.dr;
  const int64_t V4 = r4(V);
  auto want = [&](int i) { return grads[i] != nullptr; };
  // stacked-weight gradient: rows j * n .. of C [ids.size() * n, K] -> grads[ids[j]]
  auto stacked_dw = [&](const std::vector<int>& ids, int n, const float* At, const float* Wt,
                        int K, int Kc) -> int {
    bool any = false, adjacent = true;
    for (size_t j = 0; j < ids.size(); ++j) {
      any = any || want(ids[j]);
      adjacent = adjacent && want(ids[j]) && grads[ids[j]] == grads[ids[0]] + j * (int64_t)n * K;
    }
    if (!any) return MPR_OK;
    const int M = (int)ids.size() * n;
    if (adjacent) return gemm(ar, At, r4(Kc), Wt, r4(Kc), grads[ids[0]], M, K, (int)r4(Kc));
    TR_GET(C, (int64_t)M * K);
    MPR_TRY(gemm(ar, At, r4(Kc), Wt, r4(Kc), C, M, K, (int)r4(Kc)));
    std::vector<CopySeg> segs;
    for (size_t j = 0; j < ids.size(); ++j)
      if (want(ids[j])) segs.push_back({C + j * (int64_t)n * K, grads[ids[j]], (int64_t)n * K});
    return copy_segments(segs, s);
  };
  // self-attention block: dqkv from da, dn (the q|k|v input's gradient), the stacked weight
  // gradient
  auto self_attn_bwd = [&](const float* qkv, const float* Pm, const float* Wqkv, const float* n1,
                           const float* da, int Lx, float* drel, int R, uint32_t st,
                           const std::vector<int>& ids, float* dn) -> int {
    const int M = B * Lx;
    TR_GET(dqkv, (int64_t)M * 3 * I);
    MPR_TRY(attn_bwd(ar, qkv, 3 * I, qkv + I, 3 * I, qkv + 2 * I, 3 * I, Pm, da, B, Lx, Lx, drel,
                     R, dr, st, dqkv, 3 * I, dqkv + I, 3 * I, dqkv + 2 * I, 3 * I));
    const bool wdw = want(ids[0]) || want(ids[1]) || want(ids[2]);
    const float* WqkvT = transpose(ar, Wqkv, 3 * I, d, d);
    const float* dT = wdw ? transpose(ar, dqkv, M, 3 * I, 3 * I) : nullptr;
    const float* xT = wdw ? transpose(ar, n1, M, d, d) : nullptr;
    MPR_REQUIRE(WqkvT && (!wdw || (dT && xT)), "trainer: out of device memory");
    MPR_TRY(gemm(ar, dqkv, 3 * I, WqkvT, 3 * I, dn, M, d, 3 * I));
    if (wdw) MPR_TRY(stacked_dw(ids, I, dT, xT, d, M));
    return MPR_OK;
  };
  // loss -> logits
  TR_GET(dlogits, Md * V4);
  TR_GET(row_loss, Md);
  TR_GET(scal, 1);
  MPR_TRY(mpr_ce_train(tp.logits, Md, V, tp.labels, grad_scale, grad_scale, dloss, row_loss, scal,
                       dlogits, V4, s));
  // lm_head (tied): logits = hs shared^T; its weight gradient opens the tied gradient
  float* d_shared = grads[0];
  TR_GET(dhs, (int64_t)Md * d);
  MPR_TRY(linear_bwd(ar, tp.hs, d, shared(), V, d, Md, dlogits, V4, dhs, false, d_shared));
  TR_GET(dg, (int64_t)Md * d);  // the decoder's gradient chain, updated in place layer by layer
  {
    const float* g = dmask(ar, dhs, (int64_t)Md * d, dr, site(1, 255, D_FINAL));
    MPR_REQUIRE(g, "trainer: out of device memory");
    MPR_TRY(rms_bwd(ar, tp.dec_in, Md, dec_final(), tp.dec_r, g, dg, false, grads[4],
                    scale_out ? (float)(1.0 / std::sqrt((double)d)) : 1.f));
  }
  TR_GET(drel_d, (int64_t)(2 * tp.Rd + 1) * H);
  MPR_HIP(hipMemsetAsync(drel_d, 0, (size_t)(2 * tp.Rd + 1) * H * 4, s));
  const int64_t ckv_ld = (int64_t)2 * Ld * I;
  float* dckv = nullptr;
  if (Ld) {
    dckv = ar.get((int64_t)Me * ckv_ld);
    MPR_REQUIRE(dckv, "trainer: out of device memory");
  }
  for (int l = Ld - 1; l >= 0; --l) {
    const DecTape& t = tp.dec[l];
    const auto m = ar.mark();
    // FFN: g = g2 + drop(drop(relu(n3 Wi^T)) Wo^T)
    const float* fd = dmask(ar, t.f, (int64_t)Md * dff, dr, site(1, l, D_FFN_ACT));
    const float* dy = dmask(ar, dg, (int64_t)Md * d, dr, site(1, l, D_FFN_OUT));
    TR_GET(df, (int64_t)Md * dff);
    MPR_REQUIRE(fd && dy, "trainer: out of device memory");
    MPR_TRY(linear_bwd(ar, fd, dff, P[dp(l, 12)], d, dff, Md, dy, d, df, false, grads[dp(l, 12)]));
    float* dfm = dr.on() ? drop(ar, df, (int64_t)Md * dff, dr, site(1, l, D_FFN_ACT)) : df;
    MPR_REQUIRE(dfm, "trainer: out of device memory");
    MPR_TRY(mpr_relu_bwd(t.f, dfm, (int64_t)Md * dff, dfm, s));
    TR_GET(dn3, (int64_t)Md * d);
    MPR_TRY(linear_bwd(ar, t.n3, d, P[dp(l, 11)], dff, d, Md, dfm, dff, dn3, false,
                       grads[dp(l, 11)]));
    MPR_TRY(rms_bwd(ar, t.g2, Md, P[dp(l, 10)], t.r3, dn3, dg, true, grads[dp(l, 10)]));
    // cross-attention: g2 = g1 + drop(attn(n2 Wq^T, enc Wk^T, enc Wv^T) Wo^T)
    dy = dmask(ar, dg, (int64_t)Md * d, dr, site(1, l, D_CROSS_OUT));
    TR_GET(dca, (int64_t)Md * I);
    MPR_REQUIRE(dy, "trainer: out of device memory");
    MPR_TRY(linear_bwd(ar, t.ca, I, P[dp(l, 9)], d, I, Md, dy, d, dca, false, grads[dp(l, 9)]));
    TR_GET(dcq, (int64_t)Md * I);
    MPR_TRY(attn_bwd(ar, t.cq, I, tp.ckv + 2 * l * I, ckv_ld, tp.ckv + (2 * l + 1) * I, ckv_ld,
                     t.cP, dca, B, T, L, nullptr, 0, dr, site(1, l, D_CROSS_P), dcq, I,
                     dckv + 2 * l * I, ckv_ld, dckv + (2 * l + 1) * I, ckv_ld));
    TR_GET(dn2, (int64_t)Md * d);
    MPR_TRY(linear_bwd(ar, t.n2, d, P[dp(l, 6)], I, d, Md, dcq, I, dn2, false, grads[dp(l, 6)]));
    MPR_TRY(rms_bwd(ar, t.g1, Md, P[dp(l, 5)], t.r2, dn2, dg, true, grads[dp(l, 5)]));
    // self-attention: g1 = g0 + drop(attn(n1 Wq^T, n1 Wk^T, n1 Wv^T; causal, bias) Wo^T)
    dy = dmask(ar, dg, (int64_t)Md * d, dr, site(1, l, D_SELF_OUT));
    TR_GET(da, (int64_t)Md * I);
    MPR_REQUIRE(dy, "trainer: out of device memory");
    MPR_TRY(linear_bwd(ar, t.a, I, P[dp(l, 4)], d, I, Md, dy, d, da, false, grads[dp(l, 4)]));
    TR_GET(dn1, (int64_t)Md * d);
    MPR_TRY(self_attn_bwd(t.qkv, t.P, t.Wqkv, t.n1, da, T, drel_d, tp.Rd, site(1, l, D_SELF_P),
                          {dp(l, 1), dp(l, 2), dp(l, 3)}, dn1));
    MPR_TRY(rms_bwd(ar, t.g0, Md, P[dp(l, 0)], t.r1, dn1, dg, true, grads[dp(l, 0)]));
    ar.rewind(m);
  }
  // decoder input embedding (tied), through its dropout
  if (d_shared) {
    const float* g = dmask(ar, dg, (int64_t)Md * d, dr, site(1, 255, D_IN));
    MPR_REQUIRE(g, "trainer: out of device memory");
    MPR_TRY(mpr_embed_bwd(g, d, uniq, offs, pos, n_uniq, d_shared, s));
  }
  if (want(2)) {
    MPR_HIP(hipMemsetAsync(grads[2], 0, (size_t)nb * H * 4, s));
    MPR_TRY(mpr_rel_scatter(drel_d, dec_lut.as<int32_t>() + (radius - tp.Rd), tp.Rd, nb, H,
                            grads[2], s));
  }
  // the cross k | v projections of every layer: the encoder output's gradient and the stacked
  // weight gradient
  float* d_enc = nullptr;
  if (Ld) {
    std::vector<int> ids;
    bool any = false;
    for (int l = 0; l < Ld; ++l) {
      ids.push_back(dp(l, 7));
      ids.push_back(dp(l, 8));
      any = any || want(dp(l, 7)) || want(dp(l, 8));
    }
    d_enc = ar.get((int64_t)Me * d);
    const float* WckvT = transpose(ar, tp.Wckv, ckv_ld, d, d);
    const float* dT = any ? transpose(ar, dckv, Me, ckv_ld, ckv_ld) : nullptr;
    const float* xT = any ? transpose(ar, tp.enc_out, Me, d, d) : nullptr;
    MPR_REQUIRE(d_enc && WckvT && (!any || (dT && xT)), "trainer: out of device memory");
    MPR_TRY(gemm(ar, dckv, ckv_ld, WckvT, ckv_ld, d_enc, Me, d, (int)ckv_ld));
    if (any) MPR_TRY(stacked_dw(ids, I, dT, xT, d, Me));
  } else {
    d_enc = ar.get((int64_t)Me * d);
    MPR_REQUIRE(d_enc, "trainer: out of device memory");
    MPR_HIP(hipMemsetAsync(d_enc, 0, (size_t)Me * d * 4, s));
  }
  // encoder
  TR_GET(dx, (int64_t)Me * d);  // the encoder's gradient chain
  {
    const float* g = dmask(ar, d_enc, (int64_t)Me * d, dr, site(0, 255, D_FINAL));
    MPR_REQUIRE(g, "trainer: out of device memory");
    MPR_TRY(rms_bwd(ar, tp.enc_in, Me, enc_final(), tp.enc_r, g, dx, false, grads[3]));
  }
  TR_GET(drel_e, (int64_t)(2 * tp.Re + 1) * H);
  MPR_HIP(hipMemsetAsync(drel_e, 0, (size_t)(2 * tp.Re + 1) * H * 4, s));
  for (int l = Le - 1; l >= 0; --l) {
    const EncTape& t = tp.enc[l];
    const auto m = ar.mark();
    const float* fd = dmask(ar, t.f, (int64_t)Me * dff, dr, site(0, l, D_FFN_ACT));
    const float* dy = dmask(ar, dx, (int64_t)Me * d, dr, site(0, l, D_FFN_OUT));
    TR_GET(df, (int64_t)Me * dff);
    MPR_REQUIRE(fd && dy, "trainer: out of device memory");
    MPR_TRY(linear_bwd(ar, fd, dff, P[ep(l, 7)], d, dff, Me, dy, d, df, false, grads[ep(l, 7)]));
    float* dfm = dr.on() ? drop(ar, df, (int64_t)Me * dff, dr, site(0, l, D_FFN_ACT)) : df;
    MPR_REQUIRE(dfm, "trainer: out of device memory");
    MPR_TRY(mpr_relu_bwd(t.f, dfm, (int64_t)Me * dff, dfm, s));
    TR_GET(dn2, (int64_t)Me * d);
    MPR_TRY(linear_bwd(ar, t.n2, d, P[ep(l, 6)], dff, d, Me, dfm, dff, dn2, false,
                       grads[ep(l, 6)]));
    MPR_TRY(rms_bwd(ar, t.x1, Me, P[ep(l, 5)], t.r2, dn2, dx, true, grads[ep(l, 5)]));
    dy = dmask(ar, dx, (int64_t)Me * d, dr, site(0, l, D_SELF_OUT));
    TR_GET(da, (int64_t)Me * I);
    MPR_REQUIRE(dy, "trainer: out of device memory");
    MPR_TRY(linear_bwd(ar, t.a, I, P[ep(l, 4)], d, I, Me, dy, d, da, false, grads[ep(l, 4)]));
    TR_GET(dn1, (int64_t)Me * d);
    MPR_TRY(self_attn_bwd(t.qkv, t.P, t.Wqkv, t.n1, da, L, drel_e, tp.Re, site(0, l, D_SELF_P),
                          {ep(l, 1), ep(l, 2), ep(l, 3)}, dn1));
    MPR_TRY(rms_bwd(ar, t.x0, Me, P[ep(l, 0)], t.r1, dn1, dx, true, grads[ep(l, 0)]));
    ar.rewind(m);
  }
  if (want(1)) {
    MPR_HIP(hipMemsetAsync(grads[1], 0, (size_t)nb * H * 4, s));
    MPR_TRY(mpr_rel_scatter(drel_e, enc_lut.as<int32_t>() + (radius - tp.Re), tp.Re, nb, H,
                            grads[1], s));
  }
  if (d_emb) {
    if (dr.on())
      MPR_TRY(mpr_dropout(dx, (int64_t)Me * d, dr.seed, site(0, 255, D_IN), dr.thresh, dr.scale,
                          nullptr, d_emb, s));
    else
      MPR_HIP(hipMemcpyAsync(d_emb, dx, (size_t)Me * d * 4, hipMemcpyDeviceToDevice, s));
  }
  return MPR_OK;
}

}  // namespace mpr

using namespace mpr;

namespace {
template <class F>
int tr_guarded(F&& f) {
  try {
    return f();
  } catch (const std::exception& e) {
    set_error("exception: %s", e.what());
    return MPR_ENOMEM;
  } catch (...) {
    set_error("unknown exception");
    return MPR_EINVAL;
  }
}
#define TRAINER(m)                                                                    \
  MPR_REQUIRE((m) && (m)->kind == mpr_model::T5_TRAIN, "trainer: not a T5 trainer"); \
  T5Trainer* tr = static_cast<T5Trainer*>(m)
}  // namespace

extern "C" {

int mpr_t5_trainer_create(const int32_t* cfg, int32_t n_cfg, const int32_t* enc_lut,
                          const int32_t* dec_lut, int32_t radius, mpr_model** out) {
  return tr_guarded([&]() -> int {
    MPR_REQUIRE(cfg && n_cfg >= 9 && enc_lut && dec_lut && out && radius >= 1,
                "trainer_create: bad arguments");
    auto t = std::make_unique<T5Trainer>();
    t->d = cfg[0]; t->dkv = cfg[1]; t->H = cfg[2]; t->dff = cfg[3]; t->Le = cfg[4];
    t->Ld = cfg[5]; t->V = cfg[6]; t->nb = cfg[7]; t->scale_out = cfg[8];
    t->inner = t->H * t->dkv;
    t->radius = radius;
    MPR_REQUIRE(t->dkv == 64 && t->d % 4 == 0 && t->dff % 4 == 0,
                "trainer_create: d_kv=%d d=%d d_ff=%d", t->dkv, t->d, t->dff);
    const size_t nr = 2 * (size_t)radius + 1;
    for (const int32_t* lut : {enc_lut, dec_lut})
      for (size_t r = 0; r < nr; ++r)
        MPR_REQUIRE(lut[r] >= 0 && lut[r] < t->nb, "trainer_create: lut bucket %d", lut[r]);
    // the tables must have reached their saturated buckets at both ends (grow_luts extends them
    // by repetition): true whenever radius >= max_distance
    for (const int32_t* lut : {enc_lut, dec_lut})
      MPR_REQUIRE(radius < 2 || (lut[0] == lut[1] && lut[nr - 1] == lut[nr - 2]),
                  "trainer_create: the lut of radius %d does not saturate at its ends", radius);
    t->enc_lut_h.assign(enc_lut, enc_lut + nr);
    t->dec_lut_h.assign(dec_lut, dec_lut + nr);
    MPR_TRY(t->enc_lut.ensure(nr * 4));
    MPR_TRY(t->dec_lut.ensure(nr * 4));
    MPR_HIP(hipMemcpy(t->enc_lut.ptr, enc_lut, nr * 4, hipMemcpyHostToDevice));
    MPR_HIP(hipMemcpy(t->dec_lut.ptr, dec_lut, nr * 4, hipMemcpyHostToDevice));
    *out = t.release();
    return MPR_OK;
  });
}

int mpr_t5_train_forward(mpr_model* m, const float* const* params, int32_t n_params,
                         const float* emb, const float* mask, int32_t B, int32_t L,
                         const int32_t* dec_ids, const int32_t* labels, int32_t T,
                         float loss_scale, uint64_t drop_seed, uint32_t drop_thresh,
                         float drop_scale, float* loss, int32_t* tape_out, void* stream) {
  return tr_guarded([&]() -> int {
    TRAINER(m);
    MPR_REQUIRE(params && n_params == tr->nparams() && emb && mask && dec_ids && labels && loss &&
                    tape_out && B >= 1 && L >= 1 && T >= 1,
                "train_forward: bad arguments (%d params, expected %d)", n_params, tr->nparams());
    int id = -1;
    for (size_t i = 0; i < tr->tapes.size(); ++i)
      if (!tr->tapes[i]->busy) {
        id = (int)i;
        break;
      }
    if (id < 0) {
      MPR_REQUIRE(tr->tapes.size() < 64, "train_forward: 64 tapes alive (backward never run?)");
      tr->tapes.push_back(std::make_unique<Tape>());
      id = (int)tr->tapes.size() - 1;
    }
    Tape& tp = *tr->tapes[id];
    tp.B = B; tp.L = L; tp.T = T;
    tp.dr = Drop{drop_seed, drop_thresh, drop_scale};
    tr->P = params;
    tr->s = reinterpret_cast<hipStream_t>(stream);
    const int rc = tr->forward(tp, emb, mask, dec_ids, labels, loss_scale, loss);
    tr->P = nullptr;
    if (rc != MPR_OK) return rc;
    tp.busy = true;
    *tape_out = id;
    return MPR_OK;
  });
}

int mpr_t5_train_backward(mpr_model* m, int32_t tape, const float* const* params,
                          int32_t n_params, const float* dloss, float grad_scale,
                          const int32_t* emb_uniq, const int32_t* emb_offs,
                          const int32_t* emb_pos, int32_t n_uniq, float* const* grads,
                          float* d_emb, void* stream) {
  return tr_guarded([&]() -> int {
    TRAINER(m);
    MPR_REQUIRE(tape >= 0 && tape < (int)tr->tapes.size() && tr->tapes[tape]->busy,
                "train_backward: tape %d is not alive", tape);
    MPR_REQUIRE(params && n_params == tr->nparams() && dloss && grads,
                "train_backward: bad arguments");
    MPR_REQUIRE(!grads[0] || (emb_uniq && emb_offs && emb_pos && n_uniq >= 0),
                "train_backward: the tied embedding's gradient needs the decoder ids grouped");
    tr->P = params;
    tr->s = reinterpret_cast<hipStream_t>(stream);
    const int rc = tr->backward(*tr->tapes[tape], dloss, grad_scale, emb_uniq, emb_offs, emb_pos,
                                n_uniq, grads, d_emb);
    tr->P = nullptr;
    return rc;
  });
}

int mpr_t5_train_release(mpr_model* m, int32_t tape) {
  return tr_guarded([&]() -> int {
    TRAINER(m);
    MPR_REQUIRE(tape >= 0 && tape < (int)tr->tapes.size(), "train_release: tape %d", tape);
    tr->tapes[tape]->busy = false;
    return MPR_OK;
  });
}

int mpr_t5_trainer_trim(mpr_model* m, int32_t keep_idle, void* stream) {
  return tr_guarded([&]() -> int {
    TRAINER(m);
    MPR_REQUIRE(keep_idle >= 0, "trainer_trim: keep_idle %d", keep_idle);
    // queued forwards / backwards on `stream` may still read the arenas
    MPR_HIP(hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream)));
    int idle = 0;
    for (auto& t : tr->tapes)
      if (!t->busy && idle++ >= keep_idle) {  // a released tape past the first keep_idle: free
        t->ar.chunks.clear();
        t->ar.reset();
      }
    if (keep_idle == 0) {
      tr->scratch.chunks.clear();
      tr->scratch.reset();
    }
    return MPR_OK;
  });
}

}  // extern "C"
