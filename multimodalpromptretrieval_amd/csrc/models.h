// models.h — device-resident model handles behind the opaque mpr_model of the C ABI.
#pragma once

#include <array>
#include <map>
#include <memory>
#include <tuple>

#include "kernels.h"

struct mpr_model {
  enum Kind { VIT = 1, CLIP_TEXT = 2, T5 = 3, T5_TRAIN = 4 };
  explicit mpr_model(int k) : kind(k) {}
  virtual ~mpr_model() = default;
  int kind;
};

struct mpr_index {
  mpr::DevBuf rows;   // [n, d] fp32
  mpr::DevBuf norms;  // [n] squared L2 norms
  mpr::DevBuf rows_bf16, xmax;  // coarse-scan copy of the rows, max squared norm (built on demand)
  // search workspace per stream: searches enqueued on different streams (a prefetched search on
  // the tower stream beside an analytics search on the caller's) never share candidate buffers
  std::map<void*, std::unique_ptr<mpr::DevBuf>> ws;
  std::map<void*, int> last_coarse_b;  // batch of the last coarse search per stream (0: none)
  // mpr_sharded_search_all: the local top-k per stream before it is packed for the exchange
  std::map<void*, std::unique_ptr<mpr::DevBuf>> xch;
  int64_t n = 0;
  int d = 0;
  int metric = 0;
  int64_t row_offset = 0;
};

namespace mpr {

// One pre-LN residual attention block of the CLIP transformers (openai CLIP ResidualAttentionBlock).
struct ClipBlock {
  DevBuf ln1_w, ln1_b, in_w, in_b, out_w, out_b, ln2_w, ln2_b, fc_w, fc_b, pj_w, pj_b;
  DevBuf pk_in, pk_out, pk_fc, pk_pj;  // their pack_x3 images (the towers' weights are fixed)
};

// dst = the pack_x3 image of the fixed weight w [N, K] (legacy stream; the creating call syncs).
int pack_weight(DevBuf& dst, const DevBuf& w, int64_t N, int64_t K);

// Per-call scratch of one CLIP model (activations of its tower, patch/pooling buffers).  A model
// holds TOWER_SLOTS of them: passes on different slots may be in flight at once (two batches'
// towers of a serving loop on two streams), sharing the weights.
constexpr int TOWER_SLOTS = 4;
struct TowerWs {
  DevBuf h, qkv, ao, mlp;             // transformer layer activations
  DevBuf cols, patches, x, tmp, pooled;  // ViT im2col / patch embeddings / residual stream;
                                         // text residual stream / pooled EOT rows
  DevBuf img_in, tok_in, out_st;         // graph-captured passes: staged inputs and outputs
};

struct ClipTower;
struct TowerRun {
  ClipTower* t;
  TowerWs* w;
  float* x;  // [B*L, width], updated in place
  int B, L;
  bool causal;
  int tile_div = 1;  // the B rows are tile_div equal batches (GemmArgs::tile_m = M / tile_div)
  // Pooled towers need one row per sequence after the last block (encode_image: the CLS row;
  // encode_text: the EOT row; causal attention already made every other row irrelevant), so the
  // last block's out_proj / ln_2 / MLP run on those rows only: POOL_CLS updates row 0 of every
  // sequence of x in place, POOL_EOT gathers the EOT rows (argmax of tok, ctx ids a row) into
  // w->pooled and updates them there.  Each pooled row is bit-identical to the full block's.
  int pool = 0;
  const int32_t* tok = nullptr;
  int ctx = 0;
};
enum : int { POOL_NONE = 0, POOL_CLS = 1, POOL_EOT = 2 };

struct ClipTower {
  int width = 0, layers = 0, heads = 0;
  std::vector<std::unique_ptr<ClipBlock>> blocks;
  int load_blocks(const float* const* t, int width, int layers);
  static int run_group(const TowerRun* r, int n, hipStream_t s);
};

struct VitModel : mpr_model {
  VitModel() : mpr_model(VIT) {}
  int width = 0, patch = 0, image = 0, out_dim = 0, grid = 0;
  DevBuf conv_w, cls, pos, lnpre_w, lnpre_b, lnpost_w, lnpost_b, projT;
  DevBuf pk_conv, pk_projT;
  ClipTower tower;
  TowerWs ws[TOWER_SLOTS];
  int forward(const float* img, int B, int mode, float* out, int64_t out_bs, hipStream_t s);
};

struct TextModel : mpr_model {
  TextModel() : mpr_model(CLIP_TEXT) {}
  int width = 0, ctx = 0, vocab = 0, out_dim = 0;
  DevBuf tok_emb, pos, lnf_w, lnf_b, projT;
  DevBuf pk_projT;
  ClipTower tower;
  TowerWs ws[TOWER_SLOTS];
  int forward(const int32_t* tok, int B, int L, float* out, int64_t out_bs, hipStream_t s);
};

// The CLIP towers of one batch in lockstep (encoders.hip): nv <= 2 ViTs over the same images,
// optionally the text tower; identical results to separate calls.  `slot` picks every model's
// workspace (calls on different slots may run concurrently; calls on one slot must be ordered).
int encode_towers(VitModel* const* v, const int* modes, float* const* outs,
                  const int64_t* out_bs, int nv, const float* img, int B, TextModel* tm,
                  const int32_t* tok, int Bt, int Lt, float* out_t, int64_t out_t_bs,
                  hipStream_t s, int slot = 0);
// Same with up to MAX_TEXT_RUNS separate text batches (their own lengths) in the pass: several
// serving batches' towers at once.  With ViTs and nt >= 1 text runs the B images are nt equal
// batches concatenated (B % nt == 0): every ViT GEMM makes its tile choice for one batch's rows,
// so each batch's outputs are bit-identical to its own pass.  Text run j uses the text model's
// workspace slot (slot + j) % TOWER_SLOTS.
constexpr int MAX_TEXT_RUNS = 2;
int encode_towers_multi(VitModel* const* v, const int* modes, float* const* outs,
                        const int64_t* out_bs, int nv, const float* img, int B, TextModel* tm,
                        int nt, const int32_t* const* tok, const int* Bt, const int* Lt,
                        float* const* out_t, const int64_t* out_t_bs, hipStream_t s,
                        int slot = 0);

struct T5Layer {
  DevBuf ln0, qkv, o, ln1, wi, wo;         // encoder layer / decoder self-attn + ffn
  DevBuf cq, co, ln2;                      // decoder only: cross-attn q/o, ffn norm
  // decoder only: pack_rows16 images of qkv, o, cq, co, wi, wo for the decode-step GEMMs
  DevBuf pk_qkv, pk_o, pk_cq, pk_co, pk_wi, pk_wo;
  // decoder only, folded decode chain (T5Model::fold): images of
  //   W_ocq  = [[o | I_d], [cq diag(ln1) o | cq diag(ln1)]]     [d + inner, inner + d]
  //   W_cowi = [[co | I_d], [wi diag(ln2) co | wi diag(ln2)]]   [d + d_ff, inner + d]
  DevBuf pk_ocq, pk_cowi;
  DevBuf xp_qkv, xp_o, xp_wi, xp_wo;       // encoder only: pack_x3 images (tiled GEMMs)
};

// Per-call workspace of generate(): activations, decode caches, captured graphs and the decode
// stream.  A model holds MAX_SLOTS of them so independent generate calls (two batches of a
// serving loop) can be in flight on the device at once, sharing the weights.
struct T5Work {
  ~T5Work();
  DevBuf x, h, qkv, ao, ff, enc_out, cross_kv, cache, dx, dq, unfinished, cur_tok;
  DevBuf enc_in, mask_in, part_val, part_idx, tok_buf;
  DevBuf logits;  // [B, V] of the tiled decode head (T5Model::tiled_head)
  DevBuf mask_enc, enc_tmp;  // a group's encoder mask / output when several groups share a decode
  DevBuf ax, yq, hz;  // folded decode chain rows: [a | x], [c | h | u], [h2 | z]
  DevBuf x1ss, x2ss;  // their residual rows' per-16-column sums of squares
  // MPR_DECODE_TRACE=1: every decode-chain kernel's output of the last generate, back to back;
  // segs[i] = {kind, step, layer, rows, cols, float offset} (T5Model::trace, TraceKind)
  DevBuf trace;
  std::vector<std::array<int64_t, 6>> segs;
  int64_t trace_off = 0;
  uint64_t gen = 0;  // bumped by every buffer growth: invalidates captured graphs
  hipStream_t cap_stream = nullptr;
  struct GraphEnt {
    hipGraphExec_t exec;
    uint64_t gen;
  };
  using GraphKey = std::vector<int>;  // (part, B, L, max_new, ...)
  std::map<GraphKey, GraphEnt> graphs;
  hipStream_t dec_stream = nullptr;  // not owned
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  // early stop (generate_groups stop_chunk): per-chunk copies of the unfinished flags
  int32_t* h_unf = nullptr;  // pinned host
  size_t h_unf_n = 0;
  std::vector<hipEvent_t> ev_chunk;
  // the generate call in flight on this slot (gen_begin .. gen_poll finalising it)
  struct Pending {
    bool active = false;
    int B = 0, L = 0, max_new = 0, eos = 0, pad = 0, chunk = 0, nch = 0;
    int launched = 0, checked = 0;  // decode chunks enqueued / whose flags were read
    bool stop = false;              // every row had emitted eos after chunk `checked - 1`
    int ahead = 2;                  // chunks kept launched but unread
    int steps = 0;                  // decode steps launched by the last finished call
    int n = 0;
    int32_t* outs[16] = {};
    int row0[16] = {}, rows[16] = {};
    hipStream_t ds = nullptr;
  } pend;
};

// Batched device copies / lane-order packs (the weight refresh of mpr_t5_update_async)
struct CopySeg {
  const float* src;
  float* dst;
  int64_t n;  // floats
};
constexpr int COPY_SEGS = 32;
struct CopySegs {
  CopySeg s[COPY_SEGS];
};
int copy_segments(const std::vector<CopySeg>& segs, hipStream_t s);
struct PackJob {
  const float* src;  // [N, K] row-major
  float* dst;        // pack_rows16 image
  int64_t N, K;
};
constexpr int PACK_JOBS = 16;
struct PackJobs {
  PackJob j[PACK_JOBS];
};
int pack_many(const std::vector<PackJob>& jobs, hipStream_t s);

struct T5Model : mpr_model {
  // slots 0..3: serving-loop calls in flight; 4 (and 5 for > 128 rows): predict()'s own
  static constexpr int MAX_SLOTS = 6;
  static constexpr int MAX_GROUPS = 16;  // batches (<= 16 rows each) sharing one decode loop
  T5Model() : mpr_model(T5) { use_slot(0); }
  int d = 0, dkv = 0, H = 0, dff = 0, Le = 0, Ld = 0, V = 0, nb = 0, scale_out = 1;
  int inner = 0, lut_radius = 0;
  // The decode chain with its RMSNorms folded into the preceding projections (6 launches per
  // layer instead of 8; MPR_DECODE_FOLD=0 keeps the 8-launch chain): see decode_body.
  bool fold = false;
  bool fold_rows(int B) const;  // the folded chain for a B-row decode
  // A decode projection: the skinny GEMV on the packed weight (gemm_skinny)
  int dec_gemm(const SkinnyArgs& a, const DevBuf& pk, hipStream_t s,
               int* amax_nparts = nullptr) const;
  bool tiled_head(int B) const;  // the grouped decode's argmax head on the tiled GEMM
  // (Measured and dropped: decodes of > 128 rows with their projections on the packed-W
  // split-bf16 tiles, RMSNorm fused, git show e050f85: each tile's serial K loop made the
  // 256-row t5-base projections 27-41 us against 14-21 for the skinny GEMVs' K split over 8
  // waves; C5 end to end 45 -> 56-64 ms per batch, profiles/r05_decode_x3_ab.txt.)
  int build_folded(hipStream_t s);  // stream-ordered
  DevBuf rel_tmp;  // update scratch: a bias table
  DevBuf shared, enc_final, dec_final, lm_head, cross_kv_w;
  DevBuf xp_cross_kv;  // pack_x3 image of cross_kv_w
  DevBuf pk_lm_head;  // pack_rows16 image of lm_head (decode argmax head)
  // relative position bias by offset: tab[(key - query + lut_radius) * H + h]
  DevBuf enc_tab, dec_tab;
  DevBuf enc_lut, dec_lut;  // the bucket LUTs (2 lut_radius + 1 int32 each): device-side updates
  std::vector<std::unique_ptr<T5Layer>> enc, dec;
  std::vector<std::unique_ptr<T5Work>> work;
  T5Work* ws = nullptr;  // workspace of the call being enqueued

  // encode / logits / embed use workspace slot 0; generate the given slot.
  int encode(const float* embeds, const float* mask, int B, int L, float* out, hipStream_t s);
  // the encoder over n batches stacked row-wise (batch g: Bs[g] x Ls[g] rows) in one pass of
  // grouped launches; each batch bit-identical to encode() alone
  int encode_multi(int n, const int* Bs, const int* Ls, const float* embeds, const float* mask,
                   float* out, hipStream_t s);
  int generate(const float* embeds, const float* mask, int B, int L, int max_new, int start,
               int eos, int pad, int32_t* out_tokens, hipStream_t s, int slot = 0);
  // generate() of ng <= MAX_GROUPS independent batches (<= 16 rows each) with one shared
  // decode loop of up to 128 rows: each batch is encoded on its own (as generate() would), the
  // decode runs over all; every batch's tokens are bit-identical to its own generate() call.
  // stop_chunk > 0: the decode runs as graphs of stop_chunk steps and no further chunk is
  // launched once every row has emitted eos (GenerationMixin's stop; the host blocks on the
  // chunk two behind the one it launches).  The skipped steps' columns stay pad, so the tokens
  // equal the full loop's.  *steps_run (optional) = decode steps launched.
  int generate_groups(int ng, const float* const* embeds, const float* const* masks,
                      const int* Bs, const int* Ls, int max_new, int start, int eos, int pad,
                      int32_t* const* outs, hipStream_t s, int slot = 0, int stop_chunk = 0,
                      int* steps_run = nullptr);
  // generate_groups split for a host that must not block: gen_begin enqueues the encoders and,
  // with stop_chunk > 0, the first decode chunks (their unfinished flags copied to pinned host
  // memory after each), then returns; gen_poll(wait = false) reads the flags of every chunk that
  // has completed, launches the next chunk while fewer than `ahead` are unread, and once every row
  // has emitted eos (or every chunk is launched) enqueues the token copies on `s` and reports
  // *done = 1.  wait = true blocks until then.  One call per slot in flight.
  int gen_begin(int ng, const float* const* embeds, const float* const* masks, const int* Bs,
                const int* Ls, int max_new, int start, int eos, int pad, int32_t* const* outs,
                hipStream_t s, int slot, int stop_chunk, int ahead);
  int gen_poll(int slot, bool wait, int* done, int* steps_run, hipStream_t s);
  int logits_tf(const float* embeds, const float* mask, int B, int L, const int32_t* dec_in,
                int T, float* logits_out, hipStream_t s);
  int embed(const int32_t* ids, int B, int len, float* out, int64_t out_bs, int row0,
            hipStream_t s);
  // Stream for the greedy decode loop of generate() in a slot (null: the caller's stream).
  int set_decode_stream(int slot, hipStream_t ds);
  int use_slot(int slot);
  // MPR_DECODE_TRACE: copy rows x cols floats (row stride ld) of a kernel's output into the slot's
  // trace as one segment (debug.hip); a no-op otherwise
  enum TraceKind : int {
    TR_ENC_OUT = 0, TR_CROSS_KV, TR_QKV, TR_SELF_ATT, TR_O, TR_CQ, TR_CROSS_ATT, TR_CO, TR_WI,
    TR_WO, TR_HEAD_VAL, TR_HEAD_IDX, TR_TOKEN, TR_X_NEXT, TR_OCQ, TR_X1SS, TR_COWI, TR_X2SS,
    TR_FO, TR_HEAD_RMS, TR_LOGITS
  };
  int trace(int kind, int t, int l, const void* p, int64_t rows, int64_t cols, int64_t ld,
            hipStream_t s);

 private:
  using GraphKey = T5Work::GraphKey;
  int grow(DevBuf& b, size_t bytes);
  int cross_kv_project(int B, int L, hipStream_t s);
  int encode_body(int B, int L, int max_new, int start, hipStream_t s);
  int init_body(int B, int L, int max_new, int start, hipStream_t s);
  int decode_body(int B, int L, int max_new, int eos, int pad, hipStream_t s, int t0 = 0,
                  int t1 = -1);
  int decode_body_folded(int B, int L, int max_new, int eos, int pad, hipStream_t s, int t0,
                         int t1);
  int launch_chunk(int c);          // decode chunk c of the pending call + its flag copy
  int finish_pending(hipStream_t s);  // token copies, join onto s, slot free
  template <class F>
  int graph_for(const GraphKey& key, hipGraphExec_t* out, F&& body);
  template <class F>
  int run_graph(const GraphKey& key, hipStream_t st, F&& body);
};

}  // namespace mpr
