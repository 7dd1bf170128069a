// kernels.h — launchers for the gfx950 kernels used by the model runners (csrc/*.hip).
#pragma once

#include "common.h"

namespace mpr {

enum Act : int { ACT_NONE = 0, ACT_QUICKGELU = 1, ACT_RELU = 2 };

// C[m, n] = R[m, n] + act(sum_k A[m, k] * W[n, k] + bias[n])      (R, bias optional)
// fp32 in / fp32 accumulate on v_mfma_f32_32x32x2_f32 (exact f32 FMA chains).
struct GemmArgs {
  const float* A = nullptr;
  int64_t lda = 0;
  const float* W = nullptr;  // [N, K] row-major (torch nn.Linear layout)
  int64_t ldw = 0;
  const float* bias = nullptr;
  const float* R = nullptr;  // residual, may alias C
  int64_t ldr = 0;
  float* C = nullptr;
  int64_t ldc = 0;
  int M = 0, N = 0, K = 0;
  int act = ACT_NONE;
  // Optional batched C rows: row r is stored at C + (r / c_rpb) * c_bs + (r % c_rpb) * ldc.
  int c_rpb = 0;
  int64_t c_bs = 0;
  // Rows the tile choice is made for (0: M).  A problem whose rows are several equal serving
  // batches concatenated sets one batch's rows, so it gets the tile (summation order) each batch
  // gets alone: bit-identical results.
  int tile_m = 0;
  // Strided batch (split-bf16 kernels only): `batch` copies of the problem, copy b reading
  // A + b a_bs, W + b w_bs and writing C + b cb_bs (no residual) — e.g. the K chunks of a split-K
  // GEMM side by side in one launch.
  int batch = 1;
  int64_t a_bs = 0, w_bs = 0, cb_bs = 0;
  // Optional packed split image of W (pack_x3): the split-bf16 kernel then loads its W operand
  // fragments straight into registers instead of staging W through LDS (results identical).
  const void* wp = nullptr;
};

int gemm(const GemmArgs& a, hipStream_t s);

// The packed split image of a fixed W [N, K] for GemmArgs::wp (bytes, and the pack itself).
int64_t packed_x3_bytes(int64_t N, int64_t K);
int pack_x3(const float* W, int64_t N, int64_t K, int64_t ldw, void* out, hipStream_t s);

// Up to GEMM_GROUP independent problems in one launch (blockIdx.z picks the problem): the two
// ViT-B/32 towers of a batch run their layer-l projections together, which doubles the blocks
// of the 768-column GEMMs that alone fill only 156 of the 256 CUs.
constexpr int GEMM_GROUP = 4;
struct GemmGroup {
  GemmArgs g[GEMM_GROUP];
  int n = 1;
};
int gemm_group(const GemmGroup& g, hipStream_t s);
// Every tiled-GEMM configuration sums each output element in the same order (the default
// split-bf16 kernels; not MPR_GEMM=f32): rows may then be merged into one problem or split over
// launches without changing any bit of the results.
bool gemm_uniform_order();

// Skinny GEMM for M <= 16 rows (decode steps): same contract as gemm() plus an optional fused
// T5 RMSNorm of the A rows: A'[m,k] = ln_w[k] * (A[m,k] * rsqrt(mean_k A[m,:]^2 + eps)).
// Skinny GEMM weights live in a lane-order image of W (pack_rows16): for 16-row tile t and
// 16-column chunk c, the 256 floats sit in the order the MFMA lanes consume them, so a wave's
// weight load is one contiguous 1 KiB (W row-major would put adjacent lanes 2 KiB apart).
//   Wp[(t * cdiv(K,16) + c) * 256 + l * 4 + e] = W[16t + (l & 15)][16c + 4(l >> 4) + e]  (0 outside)
int64_t packed_rows16_elems(int64_t N, int64_t K);
int pack_rows16(const float* W, int64_t N, int64_t K, int64_t ldw, float* out, hipStream_t s);

struct AttnArgs {
  const float* q = nullptr;
  int64_t q_bs = 0, q_rs = 0;
  const float* k = nullptr;
  int64_t k_bs = 0, k_rs = 0;
  const float* v = nullptr;
  int64_t v_bs = 0, v_rs = 0;
  float* o = nullptr;
  int64_t o_bs = 0, o_rs = 0;
  int B = 0, H = 0, Lq = 0, Lk = 0;
  float scale = 1.f;
  int causal = 0;   // key j visible iff j <= i + q_pos0
  int q_pos0 = 0;   // absolute position of query row 0
  const float* key_mask = nullptr;  // [B, mask_bs] 1/0 (0 = padded key), optional
  int64_t mask_bs = 0;
  // T5 relative position bias by offset: rel_tab[(j - (i + q_pos0) + lut_radius) * H + h]
  // (the layer-0 bias table gathered through the bucket LUT once at model load), optional.
  const float* rel_tab = nullptr;
  int lut_radius = 0;
  // one-query decode only: q row b is scaled by rsqrt(sum_t q_rms_part[b * q_rms_nparts + t] /
  // q_rms_n + eps) — the decode chain's folded RMSNorm ahead of the cross-attention query, from
  // the per-tile partial sums of squares the producing GEMM wrote (t5.hip)
  const float* q_rms_part = nullptr;
  int q_rms_nparts = 0;
  int q_rms_n = 0;
  float q_rms_eps = 1e-6f;
  int poison = 0;  // MPR_DEBUG_LDS_POISON: LDS filled with NaN at kernel entry (set by attention())
};

struct SkinnyArgs {
  GemmArgs g;                    // g.W / g.ldw unused: the weights come from wpk
  const float* wpk = nullptr;    // pack_rows16 image of the [N, K] weight
  const float* rms_w = nullptr;  // fuse RMSNorm prologue when non-null
  float rms_eps = 1e-6f;
  float a_scale = 1.f;           // A' = (ln_w * (A * rstd)) * a_scale (T5 tied-head d^-0.5)
  // Greedy head: per (16-column tile, row) best column -> amax_val/idx[row * cdiv(N,16) + tile]
  // (C must be null).
  float* amax_val = nullptr;
  int32_t* amax_idx = nullptr;
  // Folded RMSNorm of the decode chain (t5.hip).  ssq_out: for the output columns < ssq_cols,
  // each 16-column tile also stores its rows' partial sums of squares,
  // ssq_out[row * (ssq_cols / 16) + tile].  relu_in: ReLU applied to A as it is staged.
  // rs_part: row m of the result is scaled by rsqrt(sum_t rs_part[m * rs_nparts + t] / rs_n +
  // rms_eps) (the partials another launch's ssq_out wrote, summed in tile order).
  float* ssq_out = nullptr;
  int ssq_cols = 0;
  bool relu_in = false;
  const float* rs_part = nullptr;
  int rs_nparts = 0;
  int rs_n = 0;
  int poison = 0;  // MPR_DEBUG_LDS_POISON: LDS filled with NaN at kernel entry (set by gemm_skinny)
};
int gemm_skinny(const SkinnyArgs& a, hipStream_t s);

// Kernel probe (bench roofline): hipEvent pairs around every launch of one GEMM kind.
enum ProbeKind : int { PROBE_OFF = 0, PROBE_GEMM = 1, PROBE_SKINNY = 2, PROBE_RECORD = 3 };
int probe_enable(int kind);
int probe_kind();  // the probed GEMM kind (0: off)
int probe_read(double* ms, int64_t* launches, double* flops, double* bytes);
// Re-launch the tiled-GEMM groups recorded under PROBE_RECORD back to back on one stream
// (outputs to a scratch buffer), hipEvents around each; marker kernels bracket the replay.
int probe_replay(int iters, hipStream_t s, double* ms, int64_t* launches, double* flops,
                 double* bytes);
int probe_clear();

// LayerNorm over rows of width D (eps, affine), out may alias x.  ld in floats.
// Up to LN_GROUP LayerNorms (one per tower of a lockstep pass) in one launch; identical results.
constexpr int LN_GROUP = 4;
struct LnArgs {
  const float* x = nullptr;
  int64_t ldx = 0;
  int M = 0, D = 0;
  const float *g = nullptr, *b = nullptr;
  float* out = nullptr;
  int64_t ldo = 0;
};
struct LnGroup {
  LnArgs p[LN_GROUP];
  int n = 0;
};
int layernorm_group(const LnGroup& g, float eps, hipStream_t s);
int layernorm(const float* x, int64_t ldx, int M, int D, const float* gamma, const float* beta,
              float eps, float* out, int64_t ldo, hipStream_t s);
// T5LayerNorm (RMSNorm, weight only).
int rmsnorm(const float* x, int64_t ldx, int M, int D, const float* w, float eps, float* out,
            int64_t ldo, hipStream_t s);

// Multi-head attention with head_dim 64 for short sequences.
// q(b,i,h,:) at q + b*q_bs + i*q_rs + h*64  (same for k, v, o).
int attention(const AttnArgs& a, hipStream_t s);
// The attentions of up to ATTN_GROUP towers of a lockstep pass (or batches of a T5 encoder
// group) in one launch (when all take the
// MFMA prefill path; otherwise one attention() each).  Identical results to separate calls.
constexpr int ATTN_GROUP = 4;
struct AttnGroup {
  AttnArgs a[ATTN_GROUP];
  int n = 0;
};
int attention_group(const AttnGroup& g, hipStream_t s);

// ViT patch extraction: img [B,3,S,S] -> cols [B*g*g, 3*p*p] in (c, kh, kw) order (conv1 weight
// flattening).
int im2col_patches(const float* img, int B, int S, int p, float* cols, hipStream_t s);
// x[b,0,:] = cls + pos[0]; x[b,1+t,:] = patch[b*g2+t,:] + pos[1+t]   (x: [B, g2+1, W])
int vit_assemble(const float* patches, const float* cls, const float* pos, int B, int g2, int W,
                 float* x, hipStream_t s);
// Embedding gather: out[b*obs + (row0+t)*D + c] = table[ids[b*len+t]*D + c] (+ pos[t*D + c])
int embed_gather(const float* table, const int32_t* ids, int64_t ids_bs, int B, int len, int D,
                 const float* pos, float* out, int64_t obs, int row0, hipStream_t s);
// CLIP text pooling: for each b, row e = argmax_t tok[b,t] (first max); out_rows[b,:] = x[b*L+e,:]
int eot_gather(const float* x, const int32_t* tok, int B, int L, int ctx, int D, float* out,
               hipStream_t s);
// Row argmax (first maximal index, torch.argmax semantics).
int argmax_rows(const float* logits, int M, int V, int64_t ld, int32_t* out, hipStream_t s);
// Greedy-search step (GenerationMixin._sample, do_sample=False): next = argmax over the
// lm_head's per-tile partials part_*[b*nparts + p] (first maximal index); finished rows emit pad;
// tokens[b*tok_ld + col] = next; unfinished[b] &= next != eos;
// x[b, :] = table[next, :] (decoder input embedding of the next step, may be null).
// (x: the next step's input rows, row stride x_ld)
// Row argmax of logits [M, N] (row stride ld) in P parts per row: pv/pi[row * P + part], the
// part's largest value and its lowest column (greedy_step's partials layout).
int argmax_parts(const float* L, int64_t ld, int M, int N, int P, float* pv, int32_t* pi,
                 hipStream_t s);
int greedy_step(const float* part_val, const int32_t* part_idx, int nparts, int M,
                int32_t* unfinished, int32_t* tokens, int64_t tok_ld, int col, int eos, int pad,
                const float* table, int D, float* x, hipStream_t s, int64_t x_ld = -1);

// Generic device helpers.
int fill_i32(int32_t* p, int32_t v, int64_t n, hipStream_t s);
int scale_inplace(float* p, int64_t n, float scale, hipStream_t s);

// Retrieval scan (scan.hip).
// Xb / xmax (optional): the index as bf16 rows and {max_i |x_i|^2, max_i |bf16(x_i) - x_i|^2} —
// enable the coarse bf16 scan +
// exact re-rank for large batches (scan_coarse_eligible).
// select.hip: per query the best k of n_cand (key, id) candidates ((key, id) ascending; ids < 0
// are empty slots); keys_are_values && metric 1: the keys are similarities (negated inside);
// gate (optional, per query): 0 skips the query.
int merge_lists(const float* ck, const int64_t* ci, int b, int64_t n_cand, int k,
                int keys_are_values, int metric, float* od, int64_t* oi, hipStream_t s,
                const int* gate, double* pack_out = nullptr);
// the sharded search's exchange (select.hip): (dist, id) -> float64 pairs; merge of packed
// [W][Bp][kc][2] candidate lists for query slots < b (keys are values)
// (rows of kk pairs padded to k with (NaN, -1) when kk < k; n = rows * k)
int topk_pack(const float* d, const int64_t* ids, int64_t n, double* out, hipStream_t s,
              int kk = 1, int k = 1);
int merge_packed(const double* packed, int W, int Bp, int b, int kc, int k, int metric,
                 float* od, int64_t* oi, hipStream_t s);
// k > 64: per row the k smallest (sign * key, id) of n (ids null: id = column + id_offset),
// ascending, ties to the lowest id; values written as given (sign undone).
constexpr int SELECT_MAX_K = 16384;
int select_large(const float* keys, const int64_t* ids, int b, int64_t n, int k, float sign,
                 int64_t id_offset, float* od, int64_t* oi, hipStream_t s);
// pack_out (optional): the results also as float64 (dist, id) pairs [b][k][2] when the search
// can write them on the way (the coarse path's gated merge); *packed tells whether it did
int scan_topk(const float* X, const float* xnorm, int64_t n, int d, int64_t row_offset,
              int metric, const float* Q, int b, int k, float* ws, size_t ws_bytes,
              float* out_dist, int64_t* out_ids, hipStream_t s, const void* Xb = nullptr,
              const float* xmax = nullptr, double* pack_out = nullptr, bool* packed = nullptr);
size_t scan_topk_workspace(int64_t n, int b, int k);
bool scan_coarse_eligible(int64_t n, int d, int b, int k, int metric);
// queries of the last coarse search on workspace `ws` that needed the exact fallback (host sync)
int coarse_flag_count(const void* ws, int64_t n, int d, int b, int* count);
int index_to_bf16(const float* X, int64_t count, void* out, hipStream_t s);
// |bf16(x_i) - x_i|^2 per row
int bf16_residuals(const float* X, int64_t n, int d, float* out, hipStream_t s);
int max_of(const float* x, int64_t n, float* out, hipStream_t s);
int scan_scores(const float* X, const float* xnorm, int64_t n, int d, int metric, const float* Q,
                int b, float* out, hipStream_t s);
int row_sqnorms(const float* X, int64_t n, int d, float* out, hipStream_t s);
int topk_merge(const float* cand_d, const int64_t* cand_i, int b, int64_t n_cand, int k,
               int metric, float* out_d, int64_t* out_i, hipStream_t s);
int cosine_rows(const float* x1, const float* x2, int64_t m, int d, float eps, float* out,
                hipStream_t s);
int cross_entropy(const float* logits, const int32_t* labels, int64_t n, int V, float* ws,
                  float* out, hipStream_t s);

}  // namespace mpr
