/*
 * mpr.h — C ABI of libmpr.so, the MI355X (gfx950) hot path of multimodal prompt-retrieval VQA.
 *
 * The reference (tossowski/MultimodalPromptRetrieval) is pure Python with no native layer; every
 * entry point below replaces a Python call site on its encode -> retrieve -> prompt -> T5-generate
 * path.  The reference call each function stands in for is cited next to it (paths relative to
 * the reference repository root).  The Python host (multimodalpromptretrieval_amd/_lib.py) binds
 * these symbols with ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions
 *   - Every function returns 0 on success, a negative MPR_E* code on failure; the message is in
 *     mpr_last_error() (thread-local).  No C++ exception crosses the boundary.
 *   - Pointers named *_dev are device pointers (e.g. torch tensor .data_ptr() on cuda).  Weight
 *     tensors passed to *_create may be host or device pointers (copied with hipMemcpyDefault);
 *     the library owns its copies until *_destroy.  The caller owns every I/O buffer.
 *   - `stream` is a hipStream_t (NULL = the legacy default stream).  Work is enqueued on it; the
 *     functions do not synchronise the host unless stated.
 *   - Floating-point arithmetic is fp32-accurate, like the reference's CPU path, but not
 *     IEEE-fp32 bitwise: the tiled GEMMs form each fp32 product from six bf16 MFMA partial
 *     products of a 3-way bf16 split (max error ~1.6e-7 of sum |a*b|, the f32 MFMA's ~2e-7;
 *     MPR_GEMM=f32 selects the f32-input MFMA kernel); everything else is fp32 VALU / f32 MFMA.
 */
#ifndef MPR_H_
#define MPR_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPR_OK 0
#define MPR_EINVAL (-1)   /* bad argument / shape */
#define MPR_EHIP (-2)     /* HIP runtime error */
#define MPR_ENOMEM (-3)   /* device allocation failed */
#define MPR_EUNSUP (-4)   /* unsupported configuration */

typedef struct mpr_index mpr_index;
typedef struct mpr_model mpr_model;

/* ---- runtime ----------------------------------------------------------------------------- */
int mpr_init(int32_t device);
const char* mpr_last_error(void);
int32_t mpr_abi_version(void);
/* Waits for all work on `stream` (host sync).  Used by the Python host only where the
 * reference itself syncs (D2H of retrieved ids, generated tokens). */
int mpr_stream_sync(void* stream);
/* A stream of the current device: with mask_words > 0 restricted to the CUs whose bits are set in
 * cu_mask (hipExtStreamCreateWithCUMask; bit i of word w = CU 32*w + i in the driver's CU order,
 * which deals consecutive bits round-robin over the 8 XCDs), else a non-blocking stream of the
 * given priority (lower = higher, hipDeviceGetStreamPriorityRange).  Used to give the
 * latency-bound decode chain CUs of its own beside the encoders of the next batch. */
int mpr_stream_create(int32_t priority, const uint32_t* cu_mask, int32_t mask_words, void** out);
int mpr_stream_destroy(void* stream);

/* ---- retrieval index: dataset/VQAFeatureDataset.py:192-197 (torch.cdist + torch.argsort) ----
 * rows: [n, d] fp32 row-major (host or device).  metric 0 = L2 (cdist, ascending distance),
 * 1 = cosine (utils.py:57-62 cosine_similarity, descending similarity).  row_offset is added to
 * every returned id (global id of row 0 of this shard, §8(e) index sharding). */
int mpr_index_create(const float* rows, int64_t n, int32_t d, int32_t metric, int64_t row_offset,
                     mpr_index** out);
int mpr_index_destroy(mpr_index* index);
int64_t mpr_index_rows(const mpr_index* index);
/* Top-k nearest rows for each of b queries q_dev [b, d] (fp32, device).  ids_dev [b, k] int64,
 * dist_dev [b, k] fp32: L2 distance (sqrt(max(|q|^2+|x|^2-2q.x, 0)), cdist mm-path) or cosine
 * similarity.  Order: best first; exact ties broken by lowest id.  1 <= k <= 16384, k <= n
 * (k > 64: the full score rows, then a per-query radix select). */
int mpr_index_search(mpr_index* index, const float* q_dev, int32_t b, int32_t k, int64_t* ids_dev,
                     float* dist_dev, void* stream);
/* Queries of the last search on `stream` that took the exact fallback of the coarse large-batch
 * path (bf16 scan + exact re-rank; see scan.hip): -1 when that search was not a coarse one.
 * Synchronises the stream (measurement / tests; no reference counterpart). */
int mpr_index_coarse_fallbacks(mpr_index* index, void* stream, int32_t* count);
/* Full score matrix out_dev [b, n] (L2 distance or cosine similarity), the torch.cdist output
 * (dataset/VQAFeatureDataset.py:192) / pairwise cosine_similarity (utils.py:57-62). */
int mpr_index_scores(mpr_index* index, const float* q_dev, int32_t b, float* out_dev, void* stream);
/* Merge per-shard candidates: cand_* [b, n_cand] (e.g. the RCCL all-gather of W shards' local
 * top-k) -> best k per query with the same order/tie rule.  metric as above. */
int mpr_topk_merge(const float* cand_dist_dev, const int64_t* cand_ids_dev, int32_t b,
                   int32_t n_cand, int32_t k, int32_t metric, float* out_dist_dev,
                   int64_t* out_ids_dev, void* stream);
/* The sharded search's candidate exchange without host-side reshaping (distributed.py):
 * mpr_topk_pack writes n (dist, id) pairs as float64 [n][2] (ids < 2^53 and fp32 values are
 * exact), the tensor the RCCL all_gather / all_to_all moves; mpr_topk_merge_packed merges what
 * arrives, packed [W shards][Bp query slots][kc][2], for query slots 0 .. b-1 (each query's
 * candidates shard-major): the same outputs as mpr_topk_merge over the unpacked [b, W kc] lists.
 * k <= 64, W kc <= 512. */
int mpr_topk_pack(const float* dist_dev, const int64_t* ids_dev, int64_t n, double* packed_dev,
                  void* stream);
int mpr_topk_merge_packed(const double* packed_dev, int32_t W, int32_t Bp, int32_t b, int32_t kc,
                          int32_t k, int32_t metric, float* out_dist_dev, int64_t* out_ids_dev,
                          void* stream);
/* One search of a row-sharded index with the query batch replicated on every rank (config C5;
 * north_star's "RCCL all-gather over xGMI of per-shard local top-k"), in one call on `stream`:
 * this rank's local search (index rows carry their global ids through row_offset), its top-k
 * packed into block `rank` of recv ((NaN, -1) past a tiny shard's rows), ncclAllGather in place
 * on `comm` (an RCCL communicator of `world` ranks: PyTorch's, ProcessGroupNCCL._comm_ptr(); the
 * RCCL library already loaded in the process is used; none at world 1), then the merge of recv's
 * n_blocks >= world
 * blocks [n_blocks][b][k][2] (blocks past world: candidates the caller placed there) into
 * out_dist / out_ids [b, k].  Replaces dataset/VQAFeatureDataset.py:192-197 over a sharded index;
 * the same results as mpr_index_search over the whole index up to fp32 rounding ties (exact ties
 * to the lowest global id).  k <= 64, n_blocks * k <= 512. */
/* 1 in *ok when the process has RCCL loaded with ncclAllGather and ncclCommGetAsyncError (the
 * symbols mpr_sharded_search_all calls; the Python host falls back to torch.distributed's
 * all_gather otherwise). */
int mpr_rccl_available(int32_t* ok);
int mpr_sharded_search_all(mpr_index* index, void* comm, int32_t world, int32_t rank,
                           const float* q_dev, int32_t b, int32_t k, double* recv_dev,
                           int32_t n_blocks, float* out_dist_dev, int64_t* out_ids_dev,
                           void* stream);
/* Row-wise cosine similarity (utils.py:57-62 with aligned rows): out[i] =
 * sum(x1[i]*x2[i]) / max(|x1[i]|*|x2[i]|, eps), x1/x2 [m, d]. */
int mpr_cosine_rows(const float* x1_dev, const float* x2_dev, int64_t m, int32_t d, float eps,
                    float* out_dev, void* stream);

/* ---- CLIP ViT-B/32 image encoder ------------------------------------------------------------
 * openai CLIP VisionTransformer; called at dataset/VQAFeatureDataset.py:189 (encode_image, CLS)
 * and architectures/T5VisionModel.py:112-139 (get_image_token_features, all tokens).
 * cfg = {width, layers, heads, patch, image_size, out_dim}.  tensors (fp32), in order:
 *   conv1.weight [w,3,p,p], class_embedding [w], positional_embedding [g*g+1, w],
 *   ln_pre.weight [w], ln_pre.bias [w],
 *   per layer: ln_1.weight, ln_1.bias, attn.in_proj_weight [3w,w], attn.in_proj_bias [3w],
 *              attn.out_proj.weight [w,w], attn.out_proj.bias [w], ln_2.weight, ln_2.bias,
 *              mlp.c_fc.weight [4w,w], mlp.c_fc.bias [4w], mlp.c_proj.weight [w,4w], mlp.c_proj.bias [w]
 *   ln_post.weight, ln_post.bias, proj [w, out_dim]                      (5 + 12*layers + 3) */
int mpr_vit_create(const int32_t* cfg, int32_t n_cfg, const float* const* tensors,
                   int32_t n_tensors, mpr_model** out);
/* img_dev [b,3,S,S] fp32 NCHW.  mode 0: CLS path (encode_image) -> out[b*out_bstride + c],
 * mode 1: token path (ln_post on all tokens, @proj) -> out[b*out_bstride + t*out_dim + c]. */
int mpr_vit_forward(mpr_model* m, const float* img_dev, int32_t b, int32_t mode, float* out_dev,
                    int64_t out_bstride, void* stream);
/* Two ViTs of the same geometry over the same images in one pass (the reference runs the
 * retrieval encode_image, dataset/VQAFeatureDataset.py:189, and get_image_token_features,
 * architectures/T5VisionModel.py:112-139, on every batch): results identical to two
 * mpr_vit_forward calls; the towers' projections share launches.  a != b. */
int mpr_vit_forward_pair(mpr_model* a, int32_t mode_a, float* out_a_dev, int64_t out_a_bstride,
                         mpr_model* b, int32_t mode_b, float* out_b_dev, int64_t out_b_bstride,
                         const float* img_dev, int32_t b_images, void* stream);
/* All CLIP towers of a batch in one lockstep pass: up to two ViTs over the same images
 * (vit_b may be null; both null = text only) and the CLIP text tower over tok_dev [n_texts, ctx]
 * (text may be null), as mpr_vit_forward_pair + mpr_clip_text_forward — the reference's
 * encode_image / get_image_token_features / encode_text of one batch
 * (dataset/VQAFeatureDataset.py:189-190, architectures/T5VisionModel.py:112-139).  Results are
 * bit-identical to the separate calls; each layer's projections share launches.  `slot`
 * (0 <= slot < 4; the single-model calls use 0) picks each model's activation workspace: passes
 * on different slots may be in flight at once (two batches' towers on two streams); passes on
 * one slot must be ordered by their streams. */
int mpr_encode_towers(mpr_model* vit_a, int32_t mode_a, float* out_a_dev, int64_t out_a_bstride,
                      mpr_model* vit_b, int32_t mode_b, float* out_b_dev, int64_t out_b_bstride,
                      const float* img_dev, int32_t n_images, mpr_model* text,
                      const int32_t* tok_dev, int32_t n_texts, int32_t seq_len, float* out_t_dev,
                      int64_t out_t_bstride, int32_t slot, void* stream);

/* mpr_encode_towers with n_text_runs (0..2) separate text batches in the same pass: the towers of
 * two serving batches at once (their images concatenated in img_dev for the ViTs, each batch's
 * tokens / length / output as its own text run).  Every output is bit-identical to the
 * single-batch calls.  Text run j uses the text model's workspace slot (slot + j) % 4. */
int mpr_encode_towers_multi(mpr_model* vit_a, int32_t mode_a, float* out_a_dev,
                            int64_t out_a_bstride, mpr_model* vit_b, int32_t mode_b,
                            float* out_b_dev, int64_t out_b_bstride, const float* img_dev,
                            int32_t n_images, mpr_model* text, int32_t n_text_runs,
                            const int32_t* const* tok_dev, const int32_t* n_texts,
                            const int32_t* seq_lens, float* const* out_t_dev,
                            const int64_t* out_t_bstride, int32_t slot, void* stream);

/* ---- CLIP text encoder: dataset/VQAFeatureDataset.py:190 (clip_model.encode_text) -----------
 * cfg = {width, layers, heads, context_length, vocab, out_dim}.  tensors: token_embedding
 * [vocab,w], positional_embedding [ctx,w], 12 per layer (as ViT), ln_final.weight,
 * ln_final.bias, text_projection [w,out_dim]                                (2 + 12*layers + 3) */
int mpr_clip_text_create(const int32_t* cfg, int32_t n_cfg, const float* const* tensors,
                         int32_t n_tensors, mpr_model** out);
/* tok_dev [b, ctx] int32 (clip.tokenize ids).  Pools at argmax(token id) (the EOT token).
 * seq_len (<= ctx) = number of leading positions to run; the attention is causal, so any
 * seq_len > max_b argmax_t tok[b, t] gives bit-identical pooled outputs (pass ctx if unknown). */
int mpr_clip_text_forward(mpr_model* m, const int32_t* tok_dev, int32_t b, int32_t seq_len,
                          float* out_dev, int64_t out_bstride, void* stream);

/* ---- T5 encoder/decoder: architectures/T5VisionModel.py:169,200-205,233 -----------------------
 * (transformers T5ForConditionalGeneration: encoder, greedy generate, teacher-forced logits)
 * cfg = {d_model, d_kv, n_heads, d_ff, n_enc_layers, n_dec_layers, vocab, num_buckets,
 *        scale_decoder_outputs}.
 * tensors: shared [vocab,d], enc relative_attention_bias [nb,H],
 *   per enc layer: ln0 [d], q [H*dkv,d], k, v, o [d,H*dkv], ln1 [d], wi [dff,d], wo [d,dff]
 *   enc final_layer_norm [d], dec relative_attention_bias [nb,H],
 *   per dec layer: ln0, q, k, v, o, ln1, cq, ck, cv, co, ln2, wi, wo
 *   dec final_layer_norm [d], lm_head [vocab,d]            (2 + 8*Le + 1 + 1 + 13*Ld + 2)
 * bucket luts: relative-position bucket of (key_pos - query_pos) for rel in [-radius, radius],
 * index rel + radius (encoder: bidirectional, decoder: causal), as computed by
 * T5Attention._relative_position_bucket. */
int mpr_t5_create(const int32_t* cfg, int32_t n_cfg, const float* const* tensors, int32_t n_tensors,
                  const int32_t* enc_lut, const int32_t* dec_lut, int32_t lut_radius,
                  mpr_model** out);
/* New weights for an existing T5 handle (same configuration and tensor list as mpr_t5_create):
 * copied into the handle's own buffers, so its captured generate graphs stay valid (an optimizer
 * step between training-mode predict() calls, main.py:179-187).  Waits for the device first. */
int mpr_t5_update(mpr_model* m, const float* const* tensors, int32_t n_tensors,
                  const int32_t* enc_lut, const int32_t* dec_lut);
/* mpr_t5_update without a host wait: every copy (device tensors: device to device), bias-table
 * gather, pack and fold is enqueued on `stream` (the bucket luts of mpr_t5_create are kept).
 * The caller orders `stream` after every call still reading this handle's weights and later
 * calls after `stream`, and keeps the tensors alive until it completes. */
int mpr_t5_update_async(mpr_model* m, const float* const* tensors, int32_t n_tensors,
                        void* stream);
/* Gather shared[ids] into out[b*out_bstride + (row0+t)*d + c] (T5VisionModel.py:169). */
int mpr_t5_embed(mpr_model* m, const int32_t* ids_dev, int32_t b, int32_t len, float* out_dev,
                 int64_t out_bstride, int32_t row0, void* stream);
/* Encoder stack over inputs_embeds [b,L,d] with attention mask [b,L] (1/0 fp32) -> out [b,L,d]. */
int mpr_t5_encode(mpr_model* m, const float* embeds_dev, const float* mask_dev, int32_t b,
                  int32_t L, float* out_dev, void* stream);
/* Greedy generation (GenerationMixin greedy search, do_sample=False): encoder once, then
 * max_new decoder steps with KV cache; rows that emitted eos keep emitting pad.
 * out_tokens_dev [b, max_new+1] int32 (column 0 = decoder_start).  No host sync. */
int mpr_t5_generate(mpr_model* m, const float* embeds_dev, const float* mask_dev, int32_t b,
                    int32_t L, int32_t max_new, int32_t decoder_start, int32_t eos, int32_t pad,
                    int32_t* out_tokens_dev, void* stream);
/* Teacher-forced decoder logits: dec_in_dev [b,T] int32 decoder input ids -> logits [b,T,vocab]. */
/* mpr_t5_generate on workspace slot `slot` (0 <= slot < 6; mpr_t5_generate uses slot 0).  Each
 * slot has its own activations, decode caches and captured graphs, so calls on different slots
 * may be in flight on the device at the same time (a serving loop decoding two batches at once);
 * calls on one slot must be ordered by their streams. */
int mpr_t5_generate_slot(mpr_model* m, int32_t slot, const float* embeds_dev,
                         const float* mask_dev, int32_t b, int32_t L, int32_t max_new,
                         int32_t decoder_start, int32_t eos, int32_t pad, int32_t* out_tokens_dev,
                         void* stream);
/* mpr_t5_generate_slot that stops where GenerationMixin's greedy search stops: the decode loop
 * runs as graphs of stop_chunk steps, and once every row has emitted eos no further chunk is
 * launched (the columns of the steps not run stay pad, so out_tokens equals the full loop's).
 * BLOCKS the host: before launching chunk c it waits for chunk c-2's flags.  *steps_run
 * (optional) = decode steps launched (a multiple of stop_chunk, at most max_new).  Serves the
 * one-batch predict() (architectures/T5VisionModel.py:200-205); serving loops keep the
 * asynchronous calls. */
int mpr_t5_generate_stop(mpr_model* m, int32_t slot, const float* embeds_dev,
                         const float* mask_dev, int32_t b, int32_t L, int32_t max_new,
                         int32_t decoder_start, int32_t eos, int32_t pad, int32_t stop_chunk,
                         int32_t* out_tokens_dev, int32_t* steps_run, void* stream);
/* Two batches (b_a, b_b <= 16 rows, own source lengths) generated with one shared decode loop of
 * b_a + b_b rows on workspace slot `slot`: each batch is encoded as mpr_t5_generate_slot would,
 * the greedy steps run once for both (every decode-step weight is read once per step for 32 rows
 * instead of twice for 16).  out_a [b_a, 1+max_new] / out_b [b_b, 1+max_new] are bit-identical
 * to two mpr_t5_generate_slot calls.  b_b = 0 is a plain generate of batch a. */
int mpr_t5_generate_pair(mpr_model* m, int32_t slot, const float* embeds_a_dev,
                         const float* mask_a_dev, int32_t b_a, int32_t L_a,
                         const float* embeds_b_dev, const float* mask_b_dev, int32_t b_b,
                         int32_t L_b, int32_t max_new, int32_t decoder_start, int32_t eos,
                         int32_t pad, int32_t* out_a_dev, int32_t* out_b_dev, void* stream);
/* n (1..8) batches (b[i] <= 16 rows each, own source lengths L[i]) generated with one shared
 * decode loop of sum(b) <= 128 rows on workspace slot `slot` (the general form of
 * mpr_t5_generate_pair; arrays of n device pointers / sizes).  out[i] [b[i], 1+max_new] is
 * bit-identical to mpr_t5_generate_slot on batch i. */
int mpr_t5_generate_batches(mpr_model* m, int32_t slot, int32_t n,
                            const float* const* embeds_dev, const float* const* masks_dev,
                            const int32_t* b, const int32_t* L, int32_t max_new,
                            int32_t decoder_start, int32_t eos, int32_t pad,
                            int32_t* const* out_dev, void* stream);
/* mpr_t5_generate_batches for a host that must not block (a serving loop; GenerationMixin's
 * stop of greedy search, architectures/T5VisionModel.py:200-205): enqueues the n batches'
 * encoders and, with stop_chunk > 0, the first `ahead` decode chunks of stop_chunk steps (each
 * followed by an async copy of the rows' unfinished flags), and returns without waiting.
 * stop_chunk = 0: the whole max_new-step loop as one graph (nothing to poll but the finish).
 * mpr_t5_generate_poll then advances the call: it reads the flags of every chunk that has
 * completed (oldest first; wait = 0 never blocks), launches the next chunk while fewer than
 * `ahead` are unread, and once every row has emitted eos — or every chunk is launched — enqueues
 * the token copies into out[i] ordered before later work on `stream` and sets *done = 1,
 * *steps_run = decode steps launched.  Columns of steps not run stay pad, so out[i] equals
 * mpr_t5_generate_batches's.  wait = 1 blocks until done.  One call per slot in flight: a
 * begin on a slot whose call is not done fails. */
int mpr_t5_generate_begin(mpr_model* m, int32_t slot, int32_t n,
                          const float* const* embeds_dev, const float* const* masks_dev,
                          const int32_t* b, const int32_t* L, int32_t max_new,
                          int32_t decoder_start, int32_t eos, int32_t pad, int32_t stop_chunk,
                          int32_t ahead, int32_t* const* out_dev, void* stream);
int mpr_t5_generate_poll(mpr_model* m, int32_t slot, int32_t wait, int32_t* done,
                         int32_t* steps_run, void* stream);
/* Run the greedy decode loop of later generate calls on a slot on decode_stream (null = the
 * call's own stream).  The call's stream still orders everything: the loop starts after the
 * encoder enqueued on it and the call's stream waits for the tokens. */
int mpr_t5_set_decode_stream(mpr_model* m, int32_t slot, void* decode_stream);
int mpr_t5_logits(mpr_model* m, const float* embeds_dev, const float* mask_dev, int32_t b,
                  int32_t L, const int32_t* dec_in_dev, int32_t T, float* logits_dev,
                  void* stream);
/* Mean token cross-entropy of logits [n, vocab] against labels [n] (label -100 ignored),
 * torch.nn.CrossEntropyLoss semantics (T5ForConditionalGeneration loss). out_dev: 1 float. */
int mpr_cross_entropy(const float* logits_dev, const int32_t* labels_dev, int64_t n, int32_t vocab,
                      float* out_dev, void* stream);

int mpr_model_destroy(mpr_model* m);

/* ---- training step (replaces the autograd backward of T5ForConditionalGeneration's loss that
 * main.py:186 calls through architectures/T5VisionModel.py:219-234) ----
 * Building blocks of the teacher-forced T5 forward + backward (multimodalpromptretrieval_amd/
 * train.py orchestrates them).  All pointers are device pointers, row-major fp32 unless noted;
 * every gradient is computed in a fixed order (deterministic).
 *   mpr_gemm_f32: C[M,N] = act(A[M,K] W[N,K]^T) + R (R optional, may alias C; act 0 none, 2 relu)
 *   on the fp32-accurate tiled GEMM of the encoders.
 *   mpr_transpose: out[cols, ld_out] = in[rows, cols] (row stride ld_in; columns rows..ld_out of
 *   out are zero: a GEMM's K padded to a multiple of 4).
 *   mpr_rmsnorm_fwd/bwd: T5LayerNorm y = x * rsqrt(mean(x^2) + eps) * w * scale; rstd[M] saved;
 *   bwd writes (accumulate = 0) or adds to dx, writes dw[D].
 *   mpr_attn_train_fwd/bwd: head dim 64, q/k/v/o rows at base + b*bs + i*rs + h*64; optional
 *   key mask [B, Lk] (0 = padded), causal, per-offset bias rel[(j - i + R) * H + h]; P [B,H,Lq,Lk]
 *   saved (before dropout); bwd uses a dS scratch [B,H,Lq,Lk] and adds the bias gradient by
 *   offset to drel.  drop_*: dropout of the probabilities in train mode (T5Attention's
 *   functional dropout; drop_thresh 0 = off), the mask regenerated in the backward.
 *   mpr_dropout: y = residual + x * mask (residual optional; y may alias x or residual), mask
 *   element e of (seed, site) kept iff the top 24 bits of splitmix64(seed ^ site * 0x9E37..,
 *   + e * 0xD1B5..) are >= thresh (thresh = p * 2^24), kept elements * scale (1 / (1 - p)):
 *   T5's nn.Dropout sites in train mode (main.py:170 model.train()), counter-based so the
 *   backward applies the same mask without storing it.
 *   mpr_rel_gather / mpr_rel_scatter: per-offset bias from / gradient onto the [buckets, H] table
 *   through lut[2R + 1] (bucket of offset off - R).
 *   mpr_ce_train: per-row loss of logits [n, V] against labels [n] (-100 ignored) into row_loss,
 *   loss = sum * loss_scale; dlogits (optional, row stride ld_dlogits >= V, zero padded) =
 *   (softmax - onehot) * (grad_scale * grad_mult[0]) (grad_mult: an optional device scalar, the
 *   incoming gradient of the loss, read on the device: no host wait for it).
 *   mpr_gemm_f32_splitk: mpr_gemm_f32 with K cut into `splits` chunks (multiples of 32) computed
 *   side by side into partial [splits, M, N] and summed in chunk order (for few output tiles
 *   over a long K, e.g. the tied lm_head's input gradient: K = vocab).
 *   mpr_rmsnorm_bwd: dw_partial (optional, cdiv(M, 64) x D floats) sums dw over 64-row chunks
 *   side by side first.
 *   mpr_gemm_f32_many: n mpr_gemm_f32 problems, desc[12 i ..] = {A, lda, W, ldw, C, ldc, M, N, K,
 *   R, ldr, act} (pointers as int64), GEMM_GROUP (4) per launch; each problem's result is
 *   bit-identical to its own mpr_gemm_f32 (every tile sums in the same order).
 *   mpr_gather_rows / mpr_embed_bwd: embedding rows and the gradient of the gather (positions
 *   grouped per unique id: pos[offs[u] .. offs[u+1]) hold uniq[u]), added into dW. */
int mpr_gemm_f32(const float* A, int64_t lda, const float* W, int64_t ldw, float* C, int64_t ldc,
                 int32_t M, int32_t N, int32_t K, const float* R, int64_t ldr, int32_t act,
                 void* stream);
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
int mpr_add(const float* a, const float* b, int64_t n, float* out, void* stream);
int mpr_ce_train(const float* logits, int64_t n, int32_t V, const int32_t* labels,
                 float loss_scale, float grad_scale, const float* grad_mult, float* row_loss,
                 float* loss, float* dlogits, int64_t ld_dlogits, void* stream);
int mpr_gemm_f32_many(int32_t n, const int64_t* desc, void* stream);

/* Native T5 trainer (csrc/trainer.hip): the whole teacher-forced forward and its backward
 * (T5ForConditionalGeneration(inputs_embeds, attention_mask, labels).loss, loss.backward() at
 * main.py:177-186) as one call each on the kernels above.  cfg as mpr_t5_create; the bucket luts
 * of radius lut_radius as mpr_t5_create's.  params: the 5 + 8 Le + 13 Ld fp32 device tensors in
 * train.py t5_param_names order (shared, enc / dec relative_attention_bias, enc / dec
 * final_layer_norm, per encoder layer ln0 q k v o ln1 wi wo, per decoder layer ln0 q k v o ln1
 * cq ck cv co ln2 wi wo).
 *   mpr_t5_train_forward: emb [B, L, d], mask [B, L] (1/0), dec_ids / labels [B, T] int32 (-100
 *   ignored) on the device; loss = sum of the per-token cross-entropies * loss_scale; dropout
 *   (thresh 0: off) as mpr_dropout, one seed per forward.  The activations go to a tape of the
 *   trainer (*tape_out), which reads emb-derived copies only but keeps pointers to dec_ids /
 *   labels / params: the caller keeps them alive until the backward.
 *   mpr_t5_train_backward: dloss (device scalar) * grad_scale per token; the decoder input ids
 *   grouped per unique id (mpr_embed_bwd) for the tied embedding's gradient; grads[i] (nullptr:
 *   not wanted) written, not accumulated; d_emb (optional) the gradient of emb.
 *   mpr_t5_train_release: the tape's buffers back to the trainer (after the backward, or when
 *   the forward's graph is dropped).  One stream at a time per trainer. */
int mpr_t5_trainer_create(const int32_t* cfg, int32_t n_cfg, const int32_t* enc_lut,
                          const int32_t* dec_lut, int32_t lut_radius, mpr_model** out);
int mpr_t5_train_forward(mpr_model* trainer, const float* const* params, int32_t n_params,
                         const float* emb, const float* mask, int32_t B, int32_t L,
                         const int32_t* dec_ids, const int32_t* labels, int32_t T,
                         float loss_scale, uint64_t drop_seed, uint32_t drop_thresh,
                         float drop_scale, float* loss, int32_t* tape_out, void* stream);
int mpr_t5_train_backward(mpr_model* trainer, int32_t tape, const float* const* params,
                          int32_t n_params, const float* dloss, float grad_scale,
                          const int32_t* emb_uniq, const int32_t* emb_offs,
                          const int32_t* emb_pos, int32_t n_uniq, float* const* grads,
                          float* d_emb, void* stream);
int mpr_t5_train_release(mpr_model* trainer, int32_t tape);
/* Give device memory back: after the work queued on `stream` completes, the arenas of released
 * tapes past the first `keep_idle` are freed (and the backward's scratch when keep_idle == 0);
 * later forwards re-grow them.  train.trim_trainers() calls it (e.g. after a large validation
 * batch).  The trainer itself goes with mpr_model_destroy. */
int mpr_t5_trainer_trim(mpr_model* trainer, int32_t keep_idle, void* stream);
int mpr_gemm_f32_splitk(const float* A, int64_t lda, const float* W, int64_t ldw, float* C,
                        int64_t ldc, int32_t M, int32_t N, int32_t K, const float* R, int64_t ldr,
                        int32_t act, int32_t splits, float* partial, void* stream);
/* Fixed weights (the CLIP towers', the T5 encoder's and its cross-attention K/V projection) are
 * split once: mpr_pack_x3 writes W [N, K] (row stride ldw) as its three bf16 planes in the
 * matrix-core operand order (mpr_pack_x3_bytes bytes), and a GEMM handed that image loads its W
 * fragments from it instead of staging W through LDS.  mpr_gemm_f32_packed: mpr_gemm_f32 with
 * the packed image of W — bit-identical results (same split, same summation order). */
int mpr_pack_x3_bytes(int64_t N, int64_t K, int64_t* bytes);
int mpr_pack_x3(const float* W, int64_t N, int64_t K, int64_t ldw, void* out, int64_t out_bytes,
                void* stream);
int mpr_gemm_f32_packed(const float* A, int64_t lda, const float* W, int64_t ldw, const void* wp,
                        float* C, int64_t ldc, int32_t M, int32_t N, int32_t K, const float* R,
                        int64_t ldr, int32_t act, void* stream);
int mpr_gather_rows(const float* table, const int32_t* ids, int64_t n, int32_t d, float* out,
                    void* stream);
int mpr_embed_bwd(const float* dY, int32_t d, const int32_t* uniq, const int32_t* offs,
                  const int32_t* pos, int32_t n_uniq, float* dW, void* stream);

/* ---- cosine_similarity with broadcasting (utils.py:57-62, every layout the reference takes;
 * the aligned-rows and [B,1,D] x [1,N,D] forms run mpr_cosine_rows / the index scan) ----
 *   mpr_dot_reduce: out[o] = sum_t a[off_a(o) + t * a_axis_stride] * b[off_b(o) + t *
 *   b_axis_stride], t < axis_len (sqrt of it with take_sqrt), for every o of the row-major
 *   out_shape [nd], off_x(o) = sum_d o_d * x_strides[d] (element strides, 0 = broadcast).
 *   mpr_cos_combine: out[o] = w12[.] / max(n1[.] * n2[.], eps) over out_shape, each operand by
 *   its own strides (the broadcasting of the three reductions). */
int mpr_dot_reduce(const float* a, const float* b, int32_t nd, const int64_t* out_shape,
                   const int64_t* a_strides, const int64_t* b_strides, int64_t axis_len,
                   int64_t a_axis_stride, int64_t b_axis_stride, int32_t take_sqrt, float* out,
                   void* stream);
int mpr_cos_combine(const float* w12, const float* n1, const float* n2, int32_t nd,
                    const int64_t* out_shape, const int64_t* w12_strides,
                    const int64_t* n1_strides, const int64_t* n2_strides, float eps, float* out,
                    void* stream);

/* ---- measurement (bench.py roofline; no reference counterpart) --------------------------------
 * kind 1 = tiled f32-MFMA GEMM, 2 = skinny (decode) GEMM, 0 = off.  While enabled, every launch
 * of that kernel (outside graph capture) is bracketed by hipEvents on its own stream.
 * mpr_probe_read waits for the recorded events and returns the summed kernel time (ms), the
 * launch count and the summed algorithmic FLOPs and bytes of those launches, then resets.
 * kind 3 = record: every tiled-GEMM launch (outside capture) is kept; mpr_probe_replay launches
 * the recorded problems again `iters` times back to back on `stream` (outputs to a scratch
 * buffer), hipEvents around each launch, bracketed by two launches of probe_marker_kernel (so a
 * rocprofv3 kernel trace of the same process can be windowed to the replay), and returns the
 * same totals; mpr_probe_clear drops the recording. */
int mpr_probe_enable(int32_t kind);
int mpr_probe_read(double* total_ms, int64_t* launches, double* flops, double* bytes);
int mpr_probe_replay(int32_t iters, void* stream, double* total_ms, int64_t* launches,
                     double* flops, double* bytes);
int mpr_probe_clear(void);

/* ---- debug detectors (no reference counterpart; off unless switched on before the library
 * loads: MPR_DEBUG_GUARD=1, MPR_DEBUG_LDS_POISON=1, MPR_DECODE_TRACE=1) --------------------------
 * mpr_debug_flags: bit 0 guard bands, bit 1 LDS poison, bit 2 decode trace.
 * mpr_debug_check_guards: after a device sync, counts the library buffers whose 64 KiB guard
 * bands (0xFF on both sides of every allocation) were written and describes up to a few in report.
 * mpr_debug_hash_buffers: after a device sync, a 64-bit FNV-1a hash of every live library buffer
 * (with its device address and size, in address order); *n = the number of buffers.
 * mpr_debug_t5_workspace: the addresses and sizes of one generate workspace slot's buffers (the
 * order of T5Work's fields; tools/decode_race.py names them).
 * mpr_debug_t5_trace: the decode trace of the slot's last generate (every decode-chain kernel's
 * output, MPR_DECODE_TRACE=1): copies its *n_floats floats to dst (device, cap_floats at least)
 * on stream and its segments {kind, step, layer, rows, cols, float offset} into segs (host,
 * 6 int64 each). */
int mpr_debug_flags(int32_t* flags);
int mpr_debug_check_guards(int32_t* n_bad, char* report, int32_t report_len);
int mpr_debug_hash_buffers(uint64_t* hashes, uint64_t* ptrs, int64_t* sizes, int32_t cap,
                           int32_t* n);
int mpr_debug_t5_workspace(mpr_model* m, int32_t slot, uint64_t* ptrs, int64_t* sizes,
                           int32_t cap, int32_t* n);
int mpr_debug_t5_trace(mpr_model* m, int32_t slot, float* dst, int64_t cap_floats,
                       int64_t* n_floats, int64_t* segs, int32_t seg_cap, int32_t* n_segs,
                       void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MPR_H_ */
