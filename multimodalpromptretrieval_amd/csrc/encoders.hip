// encoders.hip — CLIP ViT-B/32 image tower and CLIP text tower on the gfx950 kernels.
//
// Reference semantics (openai CLIP model.py, called from the reference at
// dataset/VQAFeatureDataset.py:189-190 and architectures/T5VisionModel.py:112-139):
//   image: conv1 (patch 32, stride 32, no bias) -> [CLS; patches] + positional -> ln_pre ->
//          12 x ResidualAttentionBlock -> ln_post -> @ proj      (CLS row only for encode_image,
//          every token for get_image_token_features)
//   text:  token_embedding + positional -> 12 x causal ResidualAttentionBlock -> ln_final ->
//          row at argmax(token id) (EOT) -> @ text_projection
//   ResidualAttentionBlock: x = x + out_proj(MHA(ln_1(x)));  x = x + c_proj(QuickGELU(c_fc(ln_2(x))))
// Data layout in HBM: activations [B*L, width] fp32 row-major; QKV [B*L, 3*width] with head h
// of q/k/v at columns h*64, width + h*64, 2*width + h*64 (nn.MultiheadAttention in_proj order).
#include <map>
#include <vector>

#include "models.h"

namespace mpr {

namespace {
constexpr float CLIP_LN_EPS = 1e-5f;
// MPR_POOL_LAST=0: the last block of pooled towers over every row (A/B; TowerRun::pool)
bool pool_last() {
  static const bool on = [] {
    const char* e = getenv("MPR_POOL_LAST");
    return !(e && e[0] == '0');
  }();
  return on;
}
// Debug bisection (tools/decode_race.py): MPR_DEBUG_TOWER_SKIP = a bit mask of launch kinds a
// tower pass leaves out (its outputs are then wrong): 1 LayerNorms, 2 q|k|v GEMMs, 4 attentions,
// 8 out-projection GEMMs, 16 c_fc GEMMs, 32 c_proj GEMMs, 64 embedding / EOT gathers.
int tower_skip() {
  static const int m = [] {
    const char* e = getenv("MPR_DEBUG_TOWER_SKIP");
    return e ? atoi(e) : 0;
  }();
  return m;
}
}

int ClipTower::load_blocks(const float* const* t, int w, int nl) {
  width = w;
  layers = nl;
  heads = w / 64;
  blocks.clear();
  for (int l = 0; l < nl; ++l) {
    auto b = std::make_unique<ClipBlock>();
    const float* const* p = t + 12 * l;
    MPR_TRY(upload(b->ln1_w, p[0], w));
    MPR_TRY(upload(b->ln1_b, p[1], w));
    MPR_TRY(upload(b->in_w, p[2], (size_t)3 * w * w));
    MPR_TRY(upload(b->in_b, p[3], (size_t)3 * w));
    MPR_TRY(upload(b->out_w, p[4], (size_t)w * w));
    MPR_TRY(upload(b->out_b, p[5], w));
    MPR_TRY(upload(b->ln2_w, p[6], w));
    MPR_TRY(upload(b->ln2_b, p[7], w));
    MPR_TRY(upload(b->fc_w, p[8], (size_t)4 * w * w));
    MPR_TRY(upload(b->fc_b, p[9], (size_t)4 * w));
    MPR_TRY(upload(b->pj_w, p[10], (size_t)4 * w * w));
    MPR_TRY(upload(b->pj_b, p[11], w));
    MPR_TRY(pack_weight(b->pk_in, b->in_w, 3 * w, w));
    MPR_TRY(pack_weight(b->pk_out, b->out_w, w, w));
    MPR_TRY(pack_weight(b->pk_fc, b->fc_w, 4 * w, w));
    MPR_TRY(pack_weight(b->pk_pj, b->pj_w, w, 4 * w));
    blocks.push_back(std::move(b));
  }
  MPR_HIP(hipStreamSynchronize(nullptr));
  return MPR_OK;
}

int pack_weight(DevBuf& dst, const DevBuf& w, int64_t N, int64_t K) {
  MPR_REQUIRE(w.bytes >= (size_t)N * K * sizeof(float), "pack_weight: %lld x %lld of %zu bytes",
              (long long)N, (long long)K, w.bytes);
  MPR_TRY(dst.ensure((size_t)packed_x3_bytes(N, K)));
  return pack_x3(w.as<float>(), N, K, K, dst.ptr, nullptr);
}

// n CLIP transformers with the same layer count stepped in lockstep (the retrieval ViT, the
// token-feature ViT and the CLIP text tower of a batch): every projection of layer l is one
// grouped GEMM launch over the towers (split by tile choice, gemm_group); per tower its own
// width, batch, sequence length and causality.
int ClipTower::run_group(const TowerRun* r, int n, hipStream_t s) {
  MPR_REQUIRE(n >= 1 && n <= ATTN_GROUP && n <= LN_GROUP, "clip tower group: n=%d", n);
  for (int i = 0; i < n; ++i) {
    ClipTower& t = *r[i].t;
    TowerWs& w = *r[i].w;
    MPR_REQUIRE(t.layers == r[0].t->layers, "clip tower group: towers differ in depth");
    const size_t M = (size_t)r[i].B * r[i].L, W = t.width;
    MPR_TRY(w.h.ensure(M * W * 4));
    MPR_TRY(w.qkv.ensure(M * 3 * W * 4));
    MPR_TRY(w.ao.ensure(M * W * 4));
    MPR_TRY(w.mlp.ensure(M * 4 * W * 4));
  }
  const int nl = r[0].t->layers;
  for (int l = 0; l < nl; ++l) {
    GemmGroup gq, go, gf, gp;
    gq.n = go.n = gf.n = gp.n = n;
    for (int i = 0; i < n; ++i) {
      ClipTower& t = *r[i].t;
      const ClipBlock& b = *t.blocks[l];
      const int W = t.width, M = r[i].B * r[i].L, TM = M / r[i].tile_div;
      float* x = r[i].x;
      float* hp = r[i].w->h.as<float>();
      float* qp = r[i].w->qkv.as<float>();
      float* ap = r[i].w->ao.as<float>();
      float* mp = r[i].w->mlp.as<float>();
      GemmArgs& g = gq.g[i];
      g.A = hp; g.lda = W; g.W = b.in_w.as<float>(); g.ldw = W; g.bias = b.in_b.as<float>();
      g.wp = b.pk_in.ptr;
      g.C = qp; g.ldc = 3 * W; g.M = M; g.N = 3 * W; g.K = W;
      GemmArgs& o = go.g[i];
      o.A = ap; o.lda = W; o.W = b.out_w.as<float>(); o.ldw = W; o.bias = b.out_b.as<float>();
      o.wp = b.pk_out.ptr;
      o.R = x; o.ldr = W; o.C = x; o.ldc = W; o.M = M; o.N = W; o.K = W;
      GemmArgs& f = gf.g[i];
      f.A = hp; f.lda = W; f.W = b.fc_w.as<float>(); f.ldw = W; f.bias = b.fc_b.as<float>();
      f.wp = b.pk_fc.ptr;
      f.C = mp; f.ldc = 4 * W; f.M = M; f.N = 4 * W; f.K = W; f.act = ACT_QUICKGELU;
      GemmArgs& pj = gp.g[i];
      pj.A = mp; pj.lda = 4 * W; pj.W = b.pj_w.as<float>(); pj.ldw = 4 * W;
      pj.wp = b.pk_pj.ptr;
      pj.bias = b.pj_b.as<float>(); pj.R = x; pj.ldr = W; pj.C = x; pj.ldc = W; pj.M = M;
      pj.N = W; pj.K = 4 * W;
      g.tile_m = o.tile_m = f.tile_m = pj.tile_m = TM;
      if (l == nl - 1 && r[i].pool != POOL_NONE) {  // the pooled rows only (TowerRun::pool)
        const int B = r[i].B;
        const int64_t ld = r[i].pool == POOL_CLS ? (int64_t)r[i].L * W : W;
        float* xr = r[i].pool == POOL_CLS ? x : r[i].w->pooled.as<float>();
        o.A = r[i].pool == POOL_CLS ? ap : hp; o.lda = ld;  // EOT: gathered attention rows in h
        o.R = o.C = xr; o.ldr = o.ldc = ld; o.M = B;
        f.M = B;
        pj.R = pj.C = xr; pj.ldr = pj.ldc = ld; pj.M = B;
        o.tile_m = f.tile_m = pj.tile_m = B / r[i].tile_div;
      }
    }
    // the towers' LayerNorms and attentions are grouped launches too (one kernel each)
    LnGroup n1, n2;
    AttnGroup ag;
    n1.n = n2.n = ag.n = n;
    for (int i = 0; i < n; ++i) {
      ClipTower& t = *r[i].t;
      const ClipBlock& b = *t.blocks[l];
      const int W = t.width, L = r[i].L, M = r[i].B * L;
      n1.p[i] = LnArgs{r[i].x, W, M, W, b.ln1_w.as<float>(), b.ln1_b.as<float>(),
                       r[i].w->h.as<float>(), W};
      n2.p[i] = LnArgs{r[i].x, W, M, W, b.ln2_w.as<float>(), b.ln2_b.as<float>(),
                       r[i].w->h.as<float>(), W};
      if (l == nl - 1 && r[i].pool == POOL_CLS)
        n2.p[i] = LnArgs{r[i].x, (int64_t)L * W, r[i].B, W, b.ln2_w.as<float>(),
                         b.ln2_b.as<float>(), r[i].w->h.as<float>(), W};
      else if (l == nl - 1 && r[i].pool == POOL_EOT)
        n2.p[i] = LnArgs{r[i].w->pooled.as<float>(), W, r[i].B, W, b.ln2_w.as<float>(),
                         b.ln2_b.as<float>(), r[i].w->h.as<float>(), W};
      float* qp = r[i].w->qkv.as<float>();
      AttnArgs& at = ag.a[i];
      at.q = qp; at.q_bs = (int64_t)L * 3 * W; at.q_rs = 3 * W;
      at.k = qp + W; at.k_bs = at.q_bs; at.k_rs = 3 * W;
      at.v = qp + 2 * W; at.v_bs = at.q_bs; at.v_rs = 3 * W;
      at.o = r[i].w->ao.as<float>(); at.o_bs = (int64_t)L * W; at.o_rs = W;
      at.B = r[i].B; at.H = t.heads; at.Lq = L; at.Lk = L;
      at.scale = 0.125f;  // 64 ** -0.5, exact power of two
      at.causal = r[i].causal ? 1 : 0;
    }
    const int skip = tower_skip();
    if (!(skip & 1)) MPR_TRY(layernorm_group(n1, CLIP_LN_EPS, s));
    if (!(skip & 2)) MPR_TRY(gemm_group(gq, s));
    if (!(skip & 4)) MPR_TRY(attention_group(ag, s));
    for (int i = 0; l == nl - 1 && i < n && !(skip & 64); ++i)
      if (r[i].pool == POOL_EOT) {  // the EOT rows of the residual stream and of attention
        const int W = r[i].t->width;
        MPR_TRY(eot_gather(r[i].x, r[i].tok, r[i].B, r[i].L, r[i].ctx, W,
                           r[i].w->pooled.as<float>(), s));
        MPR_TRY(eot_gather(r[i].w->ao.as<float>(), r[i].tok, r[i].B, r[i].L, r[i].ctx, W,
                           r[i].w->h.as<float>(), s));
      }
    if (!(skip & 8)) MPR_TRY(gemm_group(go, s));
    if (!(skip & 1)) MPR_TRY(layernorm_group(n2, CLIP_LN_EPS, s));
    if (!(skip & 16)) MPR_TRY(gemm_group(gf, s));
    if (!(skip & 32)) MPR_TRY(gemm_group(gp, s));
  }
  return MPR_OK;
}

int VitModel::forward(const float* img, int B, int mode, float* out, int64_t out_bs,
                      hipStream_t s) {
  VitModel* m = this;
  return encode_towers(&m, &mode, &out, &out_bs, 1, img, B, nullptr, nullptr, 0, 0, nullptr, 0,
                       s);
}

int TextModel::forward(const int32_t* tok, int B, int L, float* out, int64_t out_bs,
                       hipStream_t s) {
  return encode_towers(nullptr, nullptr, nullptr, nullptr, 0, nullptr, 0, this, tok, B, L, out,
                       out_bs, s);
}

// The CLIP towers of one batch in lockstep: nv (0..2) ViTs of one geometry over the same images
// (im2col once) and optionally the text tower over the batch's tokens.  Results are identical to
// separate calls (every GEMM keeps its own tile choice, every other kernel is per tower).
int encode_towers(VitModel* const* v, const int* modes, float* const* outs,
                  const int64_t* out_bs, int nv, const float* img, int B, TextModel* tm,
                  const int32_t* tok, int Bt, int Lt, float* out_t, int64_t out_t_bs,
                  hipStream_t s, int slot) {
  return encode_towers_multi(v, modes, outs, out_bs, nv, img, B, tm, tm ? 1 : 0, &tok, &Bt, &Lt,
                             &out_t, &out_t_bs, s, slot);
}

namespace {
int encode_towers_eager(VitModel* const* v, const int* modes, float* const* outs,
                        const int64_t* out_bs, int nv, const float* img, int B, TextModel* tm,
                        int nt, const int32_t* const* toks, const int* Bts, const int* Lts,
                        float* const* out_ts, const int64_t* out_t_bss, hipStream_t s,
                        int slot) {
  MPR_REQUIRE(nv >= 0 && nv <= 2, "encode_towers: %d ViTs", nv);
  MPR_REQUIRE(nt >= 0 && nt <= MAX_TEXT_RUNS && (tm || nt == 0),
              "encode_towers: %d text runs (at most %d)", nt, MAX_TEXT_RUNS);
  MPR_REQUIRE(slot >= 0 && slot < TOWER_SLOTS, "encode_towers: slot %d outside [0, %d)", slot,
              TOWER_SLOTS);
  for (int i = 0; i < nv; ++i) {
    MPR_REQUIRE(modes[i] == 0 || modes[i] == 1, "vit: mode must be 0 (CLS) or 1 (tokens)");
    MPR_REQUIRE(v[i]->width == v[0]->width && v[i]->patch == v[0]->patch &&
                    v[i]->image == v[0]->image && v[i]->tower.layers == v[0]->tower.layers,
                "vit group: towers differ in geometry");
  }
  // the text runs that have rows
  const int32_t* tok[MAX_TEXT_RUNS];
  int Btv[MAX_TEXT_RUNS], Ltv[MAX_TEXT_RUNS], tslot[MAX_TEXT_RUNS];
  float* out_t[MAX_TEXT_RUNS];
  int64_t out_t_bs[MAX_TEXT_RUNS];
  int ntr = 0;
  for (int j = 0; j < nt; ++j) {
    MPR_REQUIRE(Lts[j] >= 1 && Lts[j] <= tm->ctx, "clip text: seq_len %d outside [1, %d]",
                Lts[j], tm->ctx);
    MPR_REQUIRE(nv == 0 || tm->tower.layers == v[0]->tower.layers,
                "encode_towers: text and image towers differ in depth");
    if (Bts[j] == 0) continue;
    tok[ntr] = toks[j];
    Btv[ntr] = Bts[j];
    Ltv[ntr] = Lts[j];
    tslot[ntr] = (slot + j) % TOWER_SLOTS;
    out_t[ntr] = out_ts[j];
    out_t_bs[ntr] = out_t_bss[j];
    ++ntr;
  }
  // the images are `ig` equal serving batches: ViT GEMMs choose tiles for one batch's rows
  const int ig = (nv > 0 && nt > 1) ? nt : 1;
  MPR_REQUIRE(B % ig == 0, "encode_towers: %d images are not %d equal batches", B, ig);
  if (B == 0) nv = 0;
  if (ntr == 0) tm = nullptr;
  if (nv == 0 && !tm) return MPR_OK;
  TowerRun runs[2 + MAX_TEXT_RUNS];
  int nr = 0;
  if (nv > 0) {
    VitModel& a0 = *v[0];
    const int W = a0.width, g2 = a0.grid * a0.grid, T = g2 + 1, P = 3 * a0.patch * a0.patch;
    DevBuf& cols = a0.ws[slot].cols;
    MPR_TRY(cols.ensure((size_t)B * g2 * P * 4));
    for (int i = 0; i < nv; ++i) {
      TowerWs& w = v[i]->ws[slot];
      MPR_TRY(w.patches.ensure((size_t)B * g2 * W * 4));
      MPR_TRY(w.x.ensure((size_t)B * T * W * 4));
      MPR_TRY(w.tmp.ensure((size_t)B * T * W * 4));
    }
    MPR_TRY(im2col_patches(img, B, a0.image, a0.patch, cols.as<float>(), s));
    GemmGroup pe;
    pe.n = nv;
    for (int i = 0; i < nv; ++i) {
      GemmArgs& g = pe.g[i];
      g.A = cols.as<float>(); g.lda = P; g.W = v[i]->conv_w.as<float>(); g.ldw = P;
      g.wp = v[i]->pk_conv.ptr;
      g.C = v[i]->ws[slot].patches.as<float>(); g.ldc = W; g.M = B * g2; g.N = W; g.K = P;
      g.tile_m = B / ig * g2;
    }
    MPR_TRY(gemm_group(pe, s));
    for (int i = 0; i < nv; ++i) {
      VitModel& m = *v[i];
      TowerWs& w = m.ws[slot];
      float* xp = w.x.as<float>();
      MPR_TRY(vit_assemble(w.patches.as<float>(), m.cls.as<float>(), m.pos.as<float>(), B, g2,
                           W, xp, s));
      MPR_TRY(layernorm(xp, W, B * T, W, m.lnpre_w.as<float>(), m.lnpre_b.as<float>(),
                        CLIP_LN_EPS, xp, W, s));
      runs[nr++] = TowerRun{&m.tower, &w, xp, B, T, false, ig,
                            modes[i] == 0 && pool_last() ? POOL_CLS : POOL_NONE};
    }
  }
  for (int j = 0; tm && j < ntr; ++j) {
    const int W = tm->width, Bt = Btv[j], Lt = Ltv[j];
    TowerWs& w = tm->ws[tslot[j]];
    MPR_TRY(w.x.ensure((size_t)Bt * Lt * W * 4));
    MPR_TRY(w.pooled.ensure((size_t)Bt * W * 4));
    if (!(tower_skip() & 64))
      MPR_TRY(embed_gather(tm->tok_emb.as<float>(), tok[j], tm->ctx, Bt, Lt, W,
                           tm->pos.as<float>(), w.x.as<float>(), (int64_t)Lt * W, 0, s));
    runs[nr++] = TowerRun{&tm->tower, &w, w.x.as<float>(), Bt, Lt, true, 1,
                          pool_last() ? POOL_EOT : POOL_NONE, tok[j], tm->ctx};
  }
  MPR_TRY(ClipTower::run_group(runs, nr, s));
  GemmGroup pg;
  pg.n = 0;
  for (int i = 0; i < nv; ++i) {
    VitModel& m = *v[i];
    const int W = m.width, T = m.grid * m.grid + 1;
    float* xp = m.ws[slot].x.as<float>();
    float* tp = m.ws[slot].tmp.as<float>();
    GemmArgs& pj = pg.g[pg.n++];
    pj.W = m.projT.as<float>(); pj.ldw = W; pj.N = m.out_dim; pj.K = W; pj.A = tp; pj.lda = W;
    pj.wp = m.pk_projT.ptr;
    if (modes[i] == 0) {
      // ln_post on the CLS rows only (x[b*T]), then @ proj
      MPR_TRY(layernorm(xp, (int64_t)T * W, B, W, m.lnpost_w.as<float>(),
                        m.lnpost_b.as<float>(), CLIP_LN_EPS, tp, W, s));
      pj.M = B; pj.C = outs[i]; pj.ldc = out_bs[i]; pj.tile_m = B / ig;
    } else {
      MPR_TRY(layernorm(xp, W, B * T, W, m.lnpost_w.as<float>(), m.lnpost_b.as<float>(),
                        CLIP_LN_EPS, tp, W, s));
      pj.M = B * T; pj.C = outs[i]; pj.ldc = m.out_dim; pj.c_rpb = T; pj.c_bs = out_bs[i];
      pj.tile_m = B / ig * T;
    }
  }
  for (int j = 0; tm && j < ntr; ++j) {
    const int W = tm->width, Bt = Btv[j], Lt = Ltv[j];
    TowerWs& w = tm->ws[tslot[j]];
    float* pp = w.pooled.as<float>();
    if (!pool_last()) MPR_TRY(eot_gather(w.x.as<float>(), tok[j], Bt, Lt, tm->ctx, W, pp, s));
    MPR_TRY(layernorm(pp, W, Bt, W, tm->lnf_w.as<float>(), tm->lnf_b.as<float>(), CLIP_LN_EPS,
                      pp, W, s));
    GemmArgs& pj = pg.g[pg.n++];
    pj.A = pp; pj.lda = W; pj.W = tm->projT.as<float>(); pj.ldw = W; pj.M = Bt;
    pj.wp = tm->pk_projT.ptr;
    pj.N = tm->out_dim; pj.K = W; pj.C = out_t[j]; pj.ldc = out_t_bs[j];
  }
  MPR_TRY(gemm_group(pg, s));
  return MPR_OK;
}

// A tower pass launches ~200 kernels (two ViTs and the text tower, 12 blocks each): ~1 ms of
// host time per pass, which a serving loop feeding the GPU from one host thread cannot spare.
// With MPR_TOWER_GRAPHS=1 the pass is captured once per shape into a hipGraph over staged
// inputs and outputs (library-owned buffers: the images, the token ids and the outputs are
// copied in and out around the replay, device to device) and replayed with one launch.  The
// same kernels with the same arguments run: outputs are bit-identical to the eager pass.  Not
// while a GEMM probe records launches (the bench roofline), not for the batches of the first
// sighting of a shape (run eagerly, which also sizes every workspace before the capture).
struct TowerGraph {
  hipGraphExec_t exec;
  uint64_t gen;
};
std::map<std::vector<int64_t>, TowerGraph> g_tower_graphs;
hipStream_t g_tower_cap = nullptr;
constexpr size_t MAX_TOWER_GRAPHS = 64;

bool tower_graphs_on() {
  const char* e = getenv("MPR_TOWER_GRAPHS");
  return e && e[0] == '1' && probe_kind() == 0;
}
}  // namespace

int encode_towers_multi(VitModel* const* v, const int* modes, float* const* outs,
                        const int64_t* out_bs, int nv, const float* img, int B, TextModel* tm,
                        int nt, const int32_t* const* toks, const int* Bts, const int* Lts,
                        float* const* out_ts, const int64_t* out_t_bss, hipStream_t s,
                        int slot) {
  if (!tower_graphs_on() || nv < 0 || nv > 2 || nt < 0 || nt > MAX_TEXT_RUNS || slot < 0 ||
      slot >= TOWER_SLOTS || (nv > 0 && B == 0) || (nt > 0 && !tm))  // (errors: the eager path)
    return encode_towers_eager(v, modes, outs, out_bs, nv, img, B, tm, nt, toks, Bts, Lts, out_ts,
                               out_t_bss, s, slot);
  // the staged operands: images and outputs in ViT 0's / each model's workspace of this slot,
  // every text run's tokens and output in the text workspace of its slot (as the eager pass)
  const int ctx = tm ? tm->ctx : 0;
  std::vector<int64_t> key = {nv, B, nt, slot, (int64_t)(intptr_t)tm};
  for (int i = 0; i < nv; ++i) {
    key.push_back((int64_t)(intptr_t)v[i]);
    key.push_back(modes[i]);
  }
  for (int j = 0; j < nt; ++j) {
    key.push_back(Bts[j]);
    key.push_back(Lts[j]);
  }
  const float* s_img = img;
  float* s_out[2] = {nullptr, nullptr};
  int64_t s_bs[2] = {0, 0};
  const int32_t* s_tok[MAX_TEXT_RUNS];
  float* s_outt[MAX_TEXT_RUNS];
  int64_t s_tbs[MAX_TEXT_RUNS];
  if (nv > 0) {
    VitModel& a0 = *v[0];
    const size_t img_elems = (size_t)B * 3 * a0.image * a0.image;
    MPR_TRY(a0.ws[slot].img_in.ensure(img_elems * 4));
    s_img = a0.ws[slot].img_in.as<float>();
    for (int i = 0; i < nv; ++i) {
      const int T = v[i]->grid * v[i]->grid + 1;
      s_bs[i] = modes[i] == 0 ? v[i]->out_dim : (int64_t)T * v[i]->out_dim;
      MPR_TRY(v[i]->ws[slot].out_st.ensure((size_t)B * s_bs[i] * 4));
      s_out[i] = v[i]->ws[slot].out_st.as<float>();
    }
  }
  for (int j = 0; j < nt; ++j) {
    TowerWs& w = tm->ws[(slot + j) % TOWER_SLOTS];
    MPR_TRY(w.tok_in.ensure((size_t)std::max(Bts[j], 1) * ctx * 4));
    MPR_TRY(w.out_st.ensure((size_t)std::max(Bts[j], 1) * tm->out_dim * 4));
    s_tok[j] = w.tok_in.as<int32_t>();
    s_outt[j] = w.out_st.as<float>();
    s_tbs[j] = tm->out_dim;
  }
  auto body = [&](hipStream_t c) {
    return encode_towers_eager(v, modes, s_out, s_bs, nv, s_img, B, tm, nt, s_tok, Bts, Lts,
                               s_outt, s_tbs, c, slot);
  };
  // stage the inputs
  if (nv > 0)
    MPR_HIP(hipMemcpyAsync(const_cast<float*>(s_img), img,
                           (size_t)B * 3 * v[0]->image * v[0]->image * 4,
                           hipMemcpyDeviceToDevice, s));
  for (int j = 0; j < nt; ++j)
    if (Bts[j] > 0)
      MPR_HIP(hipMemcpyAsync(const_cast<int32_t*>(s_tok[j]), toks[j],
                             (size_t)Bts[j] * ctx * 4, hipMemcpyDeviceToDevice, s));
  auto it = g_tower_graphs.find(key);
  if (it != g_tower_graphs.end() && it->second.gen != alloc_generation()) {
    (void)hipGraphExecDestroy(it->second.exec);
    g_tower_graphs.erase(it);
    it = g_tower_graphs.end();
  }
  if (it != g_tower_graphs.end()) {
    MPR_HIP(hipGraphLaunch(it->second.exec, s));
  } else {
    // first sighting of this shape: run eagerly (sizes every workspace), then capture
    MPR_TRY(body(s));
    if (g_tower_graphs.size() >= MAX_TOWER_GRAPHS) {
      for (auto& kv : g_tower_graphs) (void)hipGraphExecDestroy(kv.second.exec);
      g_tower_graphs.clear();
    }
    if (!g_tower_cap) MPR_HIP(hipStreamCreateWithFlags(&g_tower_cap, hipStreamNonBlocking));
    const uint64_t gen = alloc_generation();
    hipGraph_t graph = nullptr;
    MPR_HIP(hipStreamBeginCapture(g_tower_cap, hipStreamCaptureModeThreadLocal));
    const int rc = body(g_tower_cap);
    const hipError_t ec = hipStreamEndCapture(g_tower_cap, &graph);
    if (rc != MPR_OK || ec != hipSuccess || alloc_generation() != gen) {
      if (graph) (void)hipGraphDestroy(graph);  // not cached: the eager run already computed
    } else {
      hipGraphExec_t exec = nullptr;
      const hipError_t ei = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
      (void)hipGraphDestroy(graph);
      if (ei == hipSuccess) g_tower_graphs.emplace(key, TowerGraph{exec, gen});
    }
  }
  // copy the outputs out to the caller's strided rows
  for (int i = 0; i < nv; ++i)
    MPR_HIP(hipMemcpy2DAsync(outs[i], (size_t)out_bs[i] * 4, s_out[i], (size_t)s_bs[i] * 4,
                             (size_t)s_bs[i] * 4, B, hipMemcpyDeviceToDevice, s));
  for (int j = 0; j < nt; ++j)
    if (Bts[j] > 0)
      MPR_HIP(hipMemcpy2DAsync(out_ts[j], (size_t)out_t_bss[j] * 4, s_outt[j],
                               (size_t)s_tbs[j] * 4, (size_t)tm->out_dim * 4, Bts[j],
                               hipMemcpyDeviceToDevice, s));
  return MPR_OK;
}

}  // namespace mpr
