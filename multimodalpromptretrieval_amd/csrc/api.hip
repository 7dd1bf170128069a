// api.hip — the extern "C" boundary of libmpr.so (declared in include/mpr.h).
#include <dlfcn.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "models.h"

namespace mpr {

namespace {
thread_local char g_err[1024] = "";
}

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int upload(DevBuf& dst, const float* src, size_t count) {
  MPR_REQUIRE(src != nullptr, "upload: null tensor pointer");
  MPR_TRY(dst.ensure(count * sizeof(float)));
  MPR_HIP(hipMemcpy(dst.ptr, src, count * sizeof(float), hipMemcpyDefault));
  return MPR_OK;
}

namespace {

// Copy `count` floats into dst at float offset `off` (dst already sized).
int upload_at(DevBuf& dst, size_t off, const float* src, size_t count) {
  MPR_REQUIRE(src != nullptr, "upload: null tensor pointer");
  MPR_REQUIRE((off + count) * sizeof(float) <= dst.bytes, "upload: overflow");
  MPR_HIP(hipMemcpy(dst.as<float>() + off, src, count * sizeof(float), hipMemcpyDefault));
  return MPR_OK;
}

// dst = src^T for src [rows, cols] given on host or device.
int upload_t(DevBuf& dst, const float* src, int64_t rows, int64_t cols) {
  std::vector<float> h((size_t)rows * cols), t((size_t)rows * cols);
  MPR_HIP(hipMemcpy(h.data(), src, h.size() * sizeof(float), hipMemcpyDefault));
  for (int64_t r = 0; r < rows; ++r)
    for (int64_t c = 0; c < cols; ++c) t[(size_t)c * rows + r] = h[(size_t)r * cols + c];
  MPR_TRY(dst.ensure(t.size() * sizeof(float)));
  MPR_HIP(hipMemcpy(dst.ptr, t.data(), t.size() * sizeof(float), hipMemcpyHostToDevice));
  return MPR_OK;
}

template <class F>
int guarded(F&& f) {
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

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace
}  // namespace mpr

using namespace mpr;

extern "C" {

int32_t mpr_abi_version(void) { return 1; }

const char* mpr_last_error(void) { return mpr::g_err; }

int mpr_init(int32_t device) {
  int n = 0;
  MPR_HIP(hipGetDeviceCount(&n));
  MPR_REQUIRE(device >= 0 && device < n, "mpr_init: device %d of %d", device, n);
  MPR_HIP(hipSetDevice(device));
  return MPR_OK;
}

int mpr_stream_sync(void* stream) {
  MPR_HIP(hipStreamSynchronize(S(stream)));
  return MPR_OK;
}

int mpr_stream_create(int32_t priority, const uint32_t* cu_mask, int32_t mask_words,
                      void** out) {
  MPR_REQUIRE(out != nullptr, "stream_create: out is null");
  MPR_REQUIRE(mask_words >= 0 && (mask_words == 0 || cu_mask), "stream_create: bad mask");
  hipStream_t s = nullptr;
  if (mask_words > 0) {
    MPR_REQUIRE(priority == 0, "stream_create: a CU-masked stream has the default priority");
    MPR_HIP(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask_words, cu_mask));
  } else {
    MPR_HIP(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority));
  }
  *out = s;
  return MPR_OK;
}

int mpr_stream_destroy(void* stream) {
  if (stream) MPR_HIP(hipStreamDestroy(S(stream)));
  return MPR_OK;
}

// ---- index -------------------------------------------------------------------------------------
int mpr_index_create(const float* rows, int64_t n, int32_t d, int32_t metric, int64_t row_offset,
                     mpr_index** out) {
  return guarded([&]() -> int {
    MPR_REQUIRE(out != nullptr, "index_create: out is null");
    MPR_REQUIRE(n >= 1 && rows != nullptr, "index_create: empty index");
    MPR_REQUIRE(d >= 16 && d % 16 == 0, "index_create: d=%d must be a positive multiple of 16", d);
    MPR_REQUIRE(metric == 0 || metric == 1, "index_create: metric %d (0=L2, 1=cosine)", metric);
    MPR_REQUIRE(n < (int64_t)0x7fffffff, "index_create: n=%lld rows exceeds int32 row ids per shard",
                (long long)n);
    auto ix = std::make_unique<mpr_index>();
    ix->n = n;
    ix->d = d;
    ix->metric = metric;
    ix->row_offset = row_offset;
    MPR_TRY(upload(ix->rows, rows, (size_t)n * d));
    MPR_TRY(ix->norms.ensure((size_t)n * sizeof(float)));
    MPR_TRY(row_sqnorms(ix->rows.as<float>(), n, d, ix->norms.as<float>(), nullptr));
    MPR_HIP(hipStreamSynchronize(nullptr));
    *out = ix.release();
    return MPR_OK;
  });
}

int mpr_index_destroy(mpr_index* index) {
  delete index;
  return MPR_OK;
}

int64_t mpr_index_rows(const mpr_index* index) { return index ? index->n : -1; }

namespace {
int index_search(mpr_index* ix, const float* q, int32_t b, int32_t k, int64_t* ids, float* dist,
                 void* stream, double* pack_out = nullptr, bool* packed = nullptr) {
  {
    MPR_REQUIRE(ix != nullptr, "search: null index");
    MPR_REQUIRE(b == 0 || (q && ids && dist), "search: null buffer");
    if (b == 0) return MPR_OK;
    MPR_REQUIRE(k >= 1 && k <= SELECT_MAX_K && k <= ix->n, "search: k=%d (1..%d, <= %lld rows)",
                k, SELECT_MAX_K, (long long)ix->n);
    auto& slot = ix->ws[stream];
    if (!slot) slot = std::make_unique<DevBuf>();
    // a growth frees the old buffer: hipFree waits for the device, so work of earlier searches
    // on this stream that still reads it completes first
    MPR_TRY(slot->ensure(scan_topk_workspace(ix->n, b, k)));
    const void* xb = nullptr;
    const float* xmax = nullptr;
    if (scan_coarse_eligible(ix->n, ix->d, b, k, ix->metric)) {
      if (!ix->rows_bf16.ptr) {  // first large-batch search: the bf16 rows and the norm bound
        MPR_TRY(ix->rows_bf16.ensure((size_t)ix->n * ix->d * 2));
        MPR_TRY(ix->xmax.ensure(2 * sizeof(float)));
        MPR_TRY(index_to_bf16(ix->rows.as<float>(), ix->n * ix->d, ix->rows_bf16.ptr, S(stream)));
        MPR_TRY(max_of(ix->norms.as<float>(), ix->n, ix->xmax.as<float>(), S(stream)));
        DevBuf res;  // per-row rounding residuals, reduced to their max (freed after the sync)
        MPR_TRY(res.ensure((size_t)ix->n * sizeof(float)));
        MPR_TRY(bf16_residuals(ix->rows.as<float>(), ix->n, ix->d, res.as<float>(), S(stream)));
        MPR_TRY(max_of(res.as<float>(), ix->n, ix->xmax.as<float>() + 1, S(stream)));
        MPR_HIP(hipStreamSynchronize(S(stream)));
      }
      xb = ix->rows_bf16.ptr;
      xmax = ix->xmax.as<float>();
    }
    ix->last_coarse_b[stream] = xb ? b : 0;
    return scan_topk(ix->rows.as<float>(), ix->norms.as<float>(), ix->n, ix->d, ix->row_offset,
                     ix->metric, q, b, k, slot->as<float>(), slot->bytes, dist, ids, S(stream),
                     xb, xmax, pack_out, packed);
  }
}
}  // namespace

int mpr_index_search(mpr_index* ix, const float* q, int32_t b, int32_t k, int64_t* ids,
                     float* dist, void* stream) {
  return guarded([&]() -> int { return index_search(ix, q, b, k, ids, dist, stream); });
}

int mpr_index_coarse_fallbacks(mpr_index* ix, void* stream, int32_t* count) {
  return guarded([&]() -> int {
    MPR_REQUIRE(ix != nullptr && count != nullptr, "coarse_fallbacks: null argument");
    *count = -1;
    auto it = ix->last_coarse_b.find(stream);
    if (it == ix->last_coarse_b.end() || it->second == 0) return MPR_OK;
    MPR_HIP(hipStreamSynchronize(S(stream)));
    int c = 0;
    MPR_TRY(coarse_flag_count(ix->ws[stream]->ptr, ix->n, ix->d, it->second, &c));
    *count = c;
    return MPR_OK;
  });
}

int mpr_index_scores(mpr_index* ix, const float* q, int32_t b, float* out, void* stream) {
  return guarded([&]() -> int {
    MPR_REQUIRE(ix != nullptr, "scores: null index");
    return scan_scores(ix->rows.as<float>(), ix->norms.as<float>(), ix->n, ix->d, ix->metric, q,
                       b, out, S(stream));
  });
}

int mpr_topk_merge(const float* cand_dist, const int64_t* cand_ids, int32_t b, int32_t n_cand,
                   int32_t k, int32_t metric, float* out_dist, int64_t* out_ids, void* stream) {
  return guarded([&]() -> int {
    MPR_REQUIRE(metric == 0 || metric == 1, "merge: metric %d", metric);
    return topk_merge(cand_dist, cand_ids, b, n_cand, k, metric, out_dist, out_ids, S(stream));
  });
}

int mpr_topk_pack(const float* dist, const int64_t* ids, int64_t n, double* packed, void* stream) {
  return guarded([&]() -> int {
    MPR_REQUIRE(n >= 0 && (n == 0 || (dist && ids && packed)), "topk_pack: null buffer");
    return topk_pack(dist, ids, n, packed, S(stream), 1, 1);
  });
}

// ---- the sharded search in one call: local scan -> pack -> RCCL all_gather -> merge ----------
// ncclAllGather is taken from the RCCL library already loaded in the process (PyTorch's, whose
// communicator the caller passes: ProcessGroupNCCL._comm_ptr()), found by its soname without
// loading another copy; libmpr.so itself does not link RCCL.
// The collective is issued outside ProcessGroupNCCL, so the process group's watchdog and error
// handling do not cover it: a failed or hung all_gather surfaces here (an error code) or at the
// next synchronisation, not as a PG timeout.
namespace {
using AllGatherFn = int (*)(const void*, void*, size_t, int, void*, hipStream_t);
using AsyncErrFn = int (*)(void*, int*);
void* rccl_handle() {
  static void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
  return h;
}
AllGatherFn rccl_allgather() {
  static AllGatherFn fn = rccl_handle() ? reinterpret_cast<AllGatherFn>(
                                              dlsym(rccl_handle(), "ncclAllGather"))
                                        : nullptr;
  return fn;
}
AsyncErrFn rccl_async_error() {
  static AsyncErrFn fn = rccl_handle() ? reinterpret_cast<AsyncErrFn>(
                                             dlsym(rccl_handle(), "ncclCommGetAsyncError"))
                                       : nullptr;
  return fn;
}
constexpr int NCCL_FLOAT64 = 8;      // ncclFloat64 (rccl.h)
constexpr int NCCL_IN_PROGRESS = 7;  // ncclInProgress: a nonblocking communicator's enqueue
}  // namespace

int mpr_rccl_available(int32_t* ok) {
  MPR_REQUIRE(ok != nullptr, "rccl_available: null");
  *ok = rccl_allgather() != nullptr && rccl_async_error() != nullptr;
  return MPR_OK;
}

int mpr_sharded_search_all(mpr_index* ix, void* comm, int32_t world, int32_t rank,
                           const float* q, int32_t b, int32_t k, double* recv, int32_t n_blocks,
                           float* out_dist, int64_t* out_ids, void* stream) {
  return guarded([&]() -> int {
    MPR_REQUIRE(ix != nullptr && comm != nullptr && recv != nullptr, "sharded_search: null argument");
    MPR_REQUIRE(world >= 1 && rank >= 0 && rank < world && n_blocks >= world,
                "sharded_search: world %d rank %d n_blocks %d", world, rank, n_blocks);
    MPR_REQUIRE(k >= 1 && k <= 64 && (int64_t)n_blocks * k <= 512,
                "sharded_search: k=%d (<= 64, n_blocks * k <= 512)", k);
    if (b == 0) return MPR_OK;
    MPR_REQUIRE(q && out_dist && out_ids, "sharded_search: null buffer");
    AllGatherFn ag = rccl_allgather();
    MPR_REQUIRE(ag != nullptr, "sharded_search: RCCL (librccl.so.1) is not loaded in this process");
    const int kk = (int)std::min<int64_t>(k, ix->n);
    auto& slot = ix->xch[stream];
    if (!slot) slot = std::make_unique<DevBuf>();
    MPR_TRY(slot->ensure((size_t)b * kk * 12 + 256));
    float* ld = slot->as<float>();
    int64_t* li = reinterpret_cast<int64_t*>(ld + ((size_t)b * kk + 63) / 64 * 64);
    const size_t count = (size_t)b * k * 2;  // this rank's block, float64 words
    double* mine = recv + (size_t)rank * count;
    bool packed = false;  // the coarse path packs on the way (its gated merge)
    MPR_TRY(index_search(ix, q, b, kk, li, ld, stream, kk == k ? mine : nullptr, &packed));
    if (!packed) MPR_TRY(topk_pack(ld, li, (int64_t)b * k, mine, S(stream), kk, k));
    // (one rank: its block is the whole exchange; MPR_SHARDED_FORCE_COLLECTIVE=1 keeps the call,
    // so a one-GPU test exercises the RCCL path)
    const bool force = getenv("MPR_SHARDED_FORCE_COLLECTIVE") != nullptr;
    if (world > 1 || force) {
      int rc = ag(mine, recv, count, NCCL_FLOAT64, comm, S(stream));  // in place
      if (rc == NCCL_IN_PROGRESS) {  // a nonblocking communicator: wait for the enqueue
        AsyncErrFn ae = rccl_async_error();
        MPR_REQUIRE(ae != nullptr, "sharded_search: nonblocking communicator without "
                                   "ncclCommGetAsyncError");
        for (long spin = 0; rc == NCCL_IN_PROGRESS && spin < 100000000L; ++spin) {
          int st = 0;
          const int e = ae(comm, &st);
          rc = e != 0 ? e : st;
        }
      }
      MPR_REQUIRE(rc == 0, "sharded_search: ncclAllGather returned %d", rc);
    }
    return merge_packed(recv, n_blocks, b, b, k, k, ix->metric, out_dist, out_ids, S(stream));
  });
}

int mpr_topk_merge_packed(const double* packed, int32_t W, int32_t Bp, int32_t b, int32_t kc,
                          int32_t k, int32_t metric, float* out_dist, int64_t* out_ids,
                          void* stream) {
  return guarded([&]() -> int {
    MPR_REQUIRE(metric == 0 || metric == 1, "merge_packed: metric %d", metric);
    MPR_REQUIRE(b == 0 || (packed && out_dist && out_ids), "merge_packed: null buffer");
    return merge_packed(packed, W, Bp, b, kc, k, metric, out_dist, out_ids, S(stream));
  });
}

int mpr_cosine_rows(const float* x1, const float* x2, int64_t m, int32_t d, float eps, float* out,
                    void* stream) {
  return guarded([&]() -> int {
    MPR_REQUIRE(d >= 1, "cosine_rows: d=%d", d);
    return cosine_rows(x1, x2, m, d, eps, out, S(stream));
  });
}

// ---- CLIP ViT -------------------------------------------------------------------------------------
int mpr_vit_create(const int32_t* cfg, int32_t n_cfg, const float* const* t, int32_t nt,
                   mpr_model** out) {
  return guarded([&]() -> int {
    MPR_REQUIRE(cfg && n_cfg >= 6 && t && out, "vit_create: bad arguments");
    const int W = cfg[0], layers = cfg[1], heads = cfg[2], patch = cfg[3], image = cfg[4],
              out_dim = cfg[5];
    MPR_REQUIRE(W % 64 == 0 && heads * 64 == W, "vit_create: width %d / heads %d (head dim 64)", W,
                heads);
    MPR_REQUIRE(image % patch == 0 && patch % 4 == 0 && W <= 1024, "vit_create: geometry");
    MPR_REQUIRE(nt == 5 + 12 * layers + 3, "vit_create: expected %d tensors, got %d",
                5 + 12 * layers + 3, nt);
    auto m = std::make_unique<VitModel>();
    m->width = W;
    m->patch = patch;
    m->image = image;
    m->out_dim = out_dim;
    m->grid = image / patch;
    const int g2 = m->grid * m->grid;
    MPR_TRY(upload(m->conv_w, t[0], (size_t)W * 3 * patch * patch));
    MPR_TRY(upload(m->cls, t[1], W));
    MPR_TRY(upload(m->pos, t[2], (size_t)(g2 + 1) * W));
    MPR_TRY(upload(m->lnpre_w, t[3], W));
    MPR_TRY(upload(m->lnpre_b, t[4], W));
    MPR_TRY(m->tower.load_blocks(t + 5, W, layers));
    const float* const* tail = t + 5 + 12 * layers;
    MPR_TRY(upload(m->lnpost_w, tail[0], W));
    MPR_TRY(upload(m->lnpost_b, tail[1], W));
    MPR_TRY(upload_t(m->projT, tail[2], W, out_dim));
    MPR_TRY(pack_weight(m->pk_conv, m->conv_w, W, (int64_t)3 * patch * patch));
    MPR_TRY(pack_weight(m->pk_projT, m->projT, out_dim, W));
    MPR_HIP(hipStreamSynchronize(nullptr));
    *out = m.release();
    return MPR_OK;
  });
}

int mpr_vit_forward(mpr_model* m, const float* img, int32_t b, int32_t mode, float* out,
                    int64_t out_bs, void* stream) {
  return guarded([&]() -> int {
    MPR_REQUIRE(m && m->kind == mpr_model::VIT, "vit_forward: not a ViT handle");
    return static_cast<VitModel*>(m)->forward(img, b, mode, out, out_bs, S(stream));
  });
}

int mpr_vit_forward_pair(mpr_model* a, int32_t mode_a, float* out_a, int64_t out_a_bs,
                         mpr_model* b, int32_t mode_b, float* out_b, int64_t out_b_bs,
                         const float* img, int32_t batch, void* stream) {
  return mpr_encode_towers(a, mode_a, out_a, out_a_bs, b, mode_b, out_b, out_b_bs, img, batch,
                           nullptr, nullptr, 0, 0, nullptr, 0, 0, stream);
}

int mpr_encode_towers(mpr_model* vit_a, int32_t mode_a, float* out_a, int64_t out_a_bs,
                      mpr_model* vit_b, int32_t mode_b, float* out_b, int64_t out_b_bs,
                      const float* img, int32_t n_images, mpr_model* text, const int32_t* tok,
                      int32_t n_texts, int32_t seq_len, float* out_t, int64_t out_t_bs,
                      int32_t slot, void* stream) {
  return guarded([&]() -> int {
    MPR_REQUIRE(!vit_a || vit_a->kind == mpr_model::VIT, "encode_towers: vit_a not a ViT");
    MPR_REQUIRE(!vit_b || vit_b->kind == mpr_model::VIT, "encode_towers: vit_b not a ViT");
    MPR_REQUIRE(!vit_b || vit_a, "encode_towers: vit_b without vit_a");
    MPR_REQUIRE(!vit_b || vit_a != vit_b, "encode_towers: the two ViT handles must differ");
    MPR_REQUIRE(!text || text->kind == mpr_model::CLIP_TEXT, "encode_towers: not a text handle");
    VitModel* v[2] = {static_cast<VitModel*>(vit_a), static_cast<VitModel*>(vit_b)};
    const int modes[2] = {mode_a, mode_b};
    float* outs[2] = {out_a, out_b};
    const int64_t bs[2] = {out_a_bs, out_b_bs};
    const int nv = vit_b ? 2 : (vit_a ? 1 : 0);
    return encode_towers(v, modes, outs, bs, nv, img, n_images, static_cast<TextModel*>(text),
                         tok, n_texts, seq_len, out_t, out_t_bs, S(stream), slot);
  });
}

int mpr_encode_towers_multi(mpr_model* vit_a, int32_t mode_a, float* out_a, int64_t out_a_bs,
                            mpr_model* vit_b, int32_t mode_b, float* out_b, int64_t out_b_bs,
                            const float* img, int32_t n_images, mpr_model* text,
                            int32_t n_text_runs, const int32_t* const* tok,
                            const int32_t* n_texts, const int32_t* seq_lens,
                            float* const* out_t, const int64_t* out_t_bs, int32_t slot,
                            void* stream) {
  return guarded([&]() -> int {
    MPR_REQUIRE(!vit_a || vit_a->kind == mpr_model::VIT, "encode_towers: vit_a not a ViT");
    MPR_REQUIRE(!vit_b || vit_b->kind == mpr_model::VIT, "encode_towers: vit_b not a ViT");
    MPR_REQUIRE(!vit_b || vit_a, "encode_towers: vit_b without vit_a");
    MPR_REQUIRE(!vit_b || vit_a != vit_b, "encode_towers: the two ViT handles must differ");
    MPR_REQUIRE(!text || text->kind == mpr_model::CLIP_TEXT, "encode_towers: not a text handle");
    MPR_REQUIRE(n_text_runs >= 0 && n_text_runs <= MAX_TEXT_RUNS && (text || n_text_runs == 0),
                "encode_towers: %d text runs", n_text_runs);
    MPR_REQUIRE(n_text_runs == 0 || (tok && n_texts && seq_lens && out_t && out_t_bs),
                "encode_towers: text run arrays missing");
    VitModel* v[2] = {static_cast<VitModel*>(vit_a), static_cast<VitModel*>(vit_b)};
    const int modes[2] = {mode_a, mode_b};
    float* outs[2] = {out_a, out_b};
    const int64_t bs[2] = {out_a_bs, out_b_bs};
    const int nv = vit_b ? 2 : (vit_a ? 1 : 0);
    int bt[MAX_TEXT_RUNS] = {0, 0}, lt[MAX_TEXT_RUNS] = {1, 1};
    for (int j = 0; j < n_text_runs; ++j) {
      bt[j] = n_texts[j];
      lt[j] = seq_lens[j];
    }
    return encode_towers_multi(v, modes, outs, bs, nv, img, n_images,
                               static_cast<TextModel*>(text), n_text_runs, tok, bt, lt, out_t,
                               out_t_bs, S(stream), slot);
  });
}

// ---- CLIP text ------------------------------------------------------------------------------------
int mpr_clip_text_create(const int32_t* cfg, int32_t n_cfg, const float* const* t, int32_t nt,
                         mpr_model** out) {
  return guarded([&]() -> int {
    MPR_REQUIRE(cfg && n_cfg >= 6 && t && out, "text_create: bad arguments");
    const int W = cfg[0], layers = cfg[1], heads = cfg[2], ctx = cfg[3], vocab = cfg[4],
              out_dim = cfg[5];
    MPR_REQUIRE(heads * 64 == W && W <= 1024, "text_create: width %d / heads %d", W, heads);
    MPR_REQUIRE(nt == 2 + 12 * layers + 3, "text_create: expected %d tensors, got %d",
                2 + 12 * layers + 3, nt);
    auto m = std::make_unique<TextModel>();
    m->width = W;
    m->ctx = ctx;
    m->vocab = vocab;
    m->out_dim = out_dim;
    MPR_TRY(upload(m->tok_emb, t[0], (size_t)vocab * W));
    MPR_TRY(upload(m->pos, t[1], (size_t)ctx * W));
    MPR_TRY(m->tower.load_blocks(t + 2, W, layers));
    const float* const* tail = t + 2 + 12 * layers;
    MPR_TRY(upload(m->lnf_w, tail[0], W));
    MPR_TRY(upload(m->lnf_b, tail[1], W));
    MPR_TRY(upload_t(m->projT, tail[2], W, out_dim));
    MPR_TRY(pack_weight(m->pk_projT, m->projT, out_dim, W));
    MPR_HIP(hipStreamSynchronize(nullptr));
    *out = m.release();
    return MPR_OK;
  });
}

int mpr_clip_text_forward(mpr_model* m, const int32_t* tok, int32_t b, int32_t seq_len, float* out,
                          int64_t out_bs, void* stream) {
  return guarded([&]() -> int {
    MPR_REQUIRE(m && m->kind == mpr_model::CLIP_TEXT, "text_forward: not a CLIP text handle");
    return static_cast<TextModel*>(m)->forward(tok, b, seq_len, out, out_bs, S(stream));
  });
}

// ---- T5 -------------------------------------------------------------------------------------------
namespace {
// Weights of a T5 handle from the tensor list of mpr_t5_create (fresh: allocate the layers) or
// into the same device buffers (an update: every pointer a captured graph holds stays valid).
// Every copy, bias-table gather, pack and fold is enqueued on s; luts (host, 2 radius + 1 each)
// are validated and uploaded when given, else the handle's device copies are used.  device_src:
// every tensor is device memory — the copies and packs then go as batched kernels (copy_segments,
// pack_many: ~10 launches instead of ~170).
int t5_load(T5Model* m, const float* const* t, const int32_t* enc_lut, const int32_t* dec_lut,
            bool fresh, hipStream_t s, bool device_src = false) {
  const int d = m->d, inner = m->inner, dff = m->dff, Le = m->Le, Ld = m->Ld;
  const int64_t nr = 2 * (int64_t)m->lut_radius + 1;
  if (enc_lut || dec_lut) {
    MPR_REQUIRE(enc_lut && dec_lut, "t5_load: both bucket luts needed");
    for (const int32_t* lut : {enc_lut, dec_lut})
      for (int64_t r = 0; r < nr; ++r)
        MPR_REQUIRE(lut[r] >= 0 && lut[r] < m->nb, "t5_load: lut bucket %d out of range", lut[r]);
    MPR_TRY(m->enc_lut.ensure(nr * 4));
    MPR_TRY(m->dec_lut.ensure(nr * 4));
    MPR_HIP(hipMemcpy(m->enc_lut.ptr, enc_lut, nr * 4, hipMemcpyHostToDevice));
    MPR_HIP(hipMemcpy(m->dec_lut.ptr, dec_lut, nr * 4, hipMemcpyHostToDevice));
  }
  MPR_REQUIRE(m->enc_lut.bytes >= (size_t)nr * 4, "t5_load: no bucket luts");
  // count floats of src at float offset off of dst (a buffer of several tensors is sized first)
  std::vector<CopySeg> segs;
  std::vector<PackJob> packs;
  auto put = [&](DevBuf& dst, size_t off, const float* src, size_t count) -> int {
    MPR_REQUIRE(src != nullptr, "t5_load: null tensor pointer");
    MPR_TRY(dst.ensure((off + count) * 4));
    MPR_REQUIRE((off + count) * 4 <= dst.bytes, "t5_load: overflow");
    if (device_src)
      segs.push_back({src, dst.as<float>() + off, (int64_t)count});
    else
      MPR_HIP(hipMemcpyAsync(dst.as<float>() + off, src, count * 4, hipMemcpyDefault, s));
    return MPR_OK;
  };
  // Relative position bias by offset r = key - query: tab[(r + radius) * H + h] =
  // rel_bias[lut[r + radius], h] (the bucket gather done once here, not per score).
  auto bias_table = [&](DevBuf& dst, const float* rel, const DevBuf& lut) -> int {
    MPR_REQUIRE(rel != nullptr, "t5_load: null tensor pointer");
    MPR_TRY(dst.ensure((size_t)nr * m->H * 4));
    if (device_src)  // gathered straight from the tensor
      return mpr_rel_gather(rel, lut.as<int32_t>(), m->lut_radius, m->H, dst.as<float>(), s);
    if (m->nb * m->H > 0) MPR_TRY(m->rel_tmp.ensure((size_t)m->nb * m->H * 4));
    MPR_HIP(hipMemcpyAsync(m->rel_tmp.ptr, rel, (size_t)m->nb * m->H * 4, hipMemcpyDefault, s));
    return mpr_rel_gather(m->rel_tmp.as<float>(), lut.as<int32_t>(), m->lut_radius, m->H,
                          dst.as<float>(), s);
  };
  int p = 0;
  MPR_TRY(put(m->shared, 0, t[p++], (size_t)m->V * d));
  MPR_TRY(bias_table(m->enc_tab, t[p++], m->enc_lut));
  for (int l = 0; l < Le; ++l) {
    if (fresh) m->enc.push_back(std::make_unique<T5Layer>());
    T5Layer& ly = *m->enc[l];
    MPR_TRY(put(ly.ln0, 0, t[p++], d));
    MPR_TRY(ly.qkv.ensure((size_t)3 * inner * d * 4));
    for (int j = 0; j < 3; ++j) MPR_TRY(put(ly.qkv, (size_t)j * inner * d, t[p++], (size_t)inner * d));
    MPR_TRY(put(ly.o, 0, t[p++], (size_t)d * inner));
    MPR_TRY(put(ly.ln1, 0, t[p++], d));
    MPR_TRY(put(ly.wi, 0, t[p++], (size_t)dff * d));
    MPR_TRY(put(ly.wo, 0, t[p++], (size_t)d * dff));
  }
  MPR_TRY(put(m->enc_final, 0, t[p++], d));
  MPR_TRY(bias_table(m->dec_tab, t[p++], m->dec_lut));
  MPR_TRY(m->cross_kv_w.ensure((size_t)Ld * 2 * inner * d * 4));
  for (int l = 0; l < Ld; ++l) {
    if (fresh) m->dec.push_back(std::make_unique<T5Layer>());
    T5Layer& ly = *m->dec[l];
    MPR_TRY(put(ly.ln0, 0, t[p++], d));
    MPR_TRY(ly.qkv.ensure((size_t)3 * inner * d * 4));
    for (int j = 0; j < 3; ++j) MPR_TRY(put(ly.qkv, (size_t)j * inner * d, t[p++], (size_t)inner * d));
    MPR_TRY(put(ly.o, 0, t[p++], (size_t)d * inner));
    MPR_TRY(put(ly.ln1, 0, t[p++], d));
    MPR_TRY(put(ly.cq, 0, t[p++], (size_t)inner * d));
    MPR_TRY(put(m->cross_kv_w, (size_t)(2 * l) * inner * d, t[p++], (size_t)inner * d));
    MPR_TRY(put(m->cross_kv_w, (size_t)(2 * l + 1) * inner * d, t[p++], (size_t)inner * d));
    MPR_TRY(put(ly.co, 0, t[p++], (size_t)d * inner));
    MPR_TRY(put(ly.ln2, 0, t[p++], d));
    MPR_TRY(put(ly.wi, 0, t[p++], (size_t)dff * d));
    MPR_TRY(put(ly.wo, 0, t[p++], (size_t)d * dff));
  }
  MPR_TRY(put(m->dec_final, 0, t[p++], d));
  MPR_TRY(put(m->lm_head, 0, t[p++], (size_t)m->V * d));
  // lane-order images of the decoder projections for the decode-step GEMMs
  auto pack = [&](DevBuf& dst, const DevBuf& src, int64_t n, int64_t k) -> int {
    MPR_TRY(dst.ensure((size_t)packed_rows16_elems(n, k) * 4));
    packs.push_back({src.as<float>(), dst.as<float>(), n, k});
    return MPR_OK;
  };
  MPR_TRY(copy_segments(segs, s));  // device_src: every tensor copy so far, batched
  for (auto& ly : m->dec) {
    MPR_TRY(pack(ly->pk_qkv, ly->qkv, 3 * inner, d));
    MPR_TRY(pack(ly->pk_o, ly->o, d, inner));
    MPR_TRY(pack(ly->pk_cq, ly->cq, inner, d));
    MPR_TRY(pack(ly->pk_co, ly->co, d, inner));
    MPR_TRY(pack(ly->pk_wi, ly->wi, dff, d));
    MPR_TRY(pack(ly->pk_wo, ly->wo, d, dff));
  }
  MPR_TRY(pack(m->pk_lm_head, m->lm_head, m->V, d));
  MPR_TRY(pack_many(packs, s));
  // split images of the encoder projections and the cross-attention K/V weight (tiled GEMMs)
  auto pack3 = [&](DevBuf& dst, const DevBuf& src, int64_t n, int64_t k) -> int {
    MPR_TRY(dst.ensure((size_t)packed_x3_bytes(n, k)));
    return pack_x3(src.as<float>(), n, k, k, dst.ptr, s);
  };
  for (auto& ly : m->enc) {
    MPR_TRY(pack3(ly->xp_qkv, ly->qkv, 3 * inner, d));
    MPR_TRY(pack3(ly->xp_o, ly->o, d, inner));
    MPR_TRY(pack3(ly->xp_wi, ly->wi, dff, d));
    MPR_TRY(pack3(ly->xp_wo, ly->wo, d, dff));
  }
  MPR_TRY(pack3(m->xp_cross_kv, m->cross_kv_w, (int64_t)Ld * 2 * inner, d));
  if (m->fold) MPR_TRY(m->build_folded(s));
  return MPR_OK;
}
}  // namespace

int mpr_t5_create(const int32_t* cfg, int32_t n_cfg, const float* const* t, int32_t nt,
                  const int32_t* enc_lut, const int32_t* dec_lut, int32_t radius,
                  mpr_model** out) {
  return guarded([&]() -> int {
    MPR_REQUIRE(cfg && n_cfg >= 9 && t && out && enc_lut && dec_lut, "t5_create: bad arguments");
    auto m = std::make_unique<T5Model>();
    m->d = cfg[0];
    m->dkv = cfg[1];
    m->H = cfg[2];
    m->dff = cfg[3];
    m->Le = cfg[4];
    m->Ld = cfg[5];
    m->V = cfg[6];
    m->nb = cfg[7];
    m->scale_out = cfg[8];
    m->inner = m->H * m->dkv;
    m->lut_radius = radius;
    const int d = m->d, dff = m->dff, Le = m->Le, Ld = m->Ld;
    MPR_REQUIRE(m->dkv == 64, "t5_create: d_kv=%d (head dim 64 supported)", m->dkv);
    MPR_REQUIRE(d % 16 == 0 && d <= 1024 && dff % 16 == 0, "t5_create: d_model=%d d_ff=%d", d, dff);
    MPR_REQUIRE(radius >= 64, "t5_create: lut radius %d too small", radius);
    const int expect = 2 + 8 * Le + 1 + 1 + 13 * Ld + 2;
    MPR_REQUIRE(nt == expect, "t5_create: expected %d tensors, got %d", expect, nt);
    {
      // the folded decode chain for models below d = 768 (T5Model::fold_rows); MPR_DECODE_FOLD
      // = 0 / 1 forces it off / on
      const char* e = getenv("MPR_DECODE_FOLD");
      m->fold = e ? e[0] != '0' : d < 768;
    }
    MPR_TRY(t5_load(m.get(), t, enc_lut, dec_lut, /*fresh=*/true, nullptr));
    MPR_HIP(hipDeviceSynchronize());
    *out = m.release();
    return MPR_OK;
  });
}

int mpr_t5_update(mpr_model* mm, const float* const* t, int32_t nt, const int32_t* enc_lut,
                  const int32_t* dec_lut) {
  return guarded([&]() -> int {
    MPR_REQUIRE(mm && mm->kind == mpr_model::T5 && t && enc_lut && dec_lut,
                "t5_update: bad arguments");
    T5Model* m = static_cast<T5Model*>(mm);
    const int expect = 2 + 8 * m->Le + 1 + 1 + 13 * m->Ld + 2;
    MPR_REQUIRE(nt == expect, "t5_update: expected %d tensors, got %d", expect, nt);
    MPR_HIP(hipDeviceSynchronize());  // no work in flight reads the weights being replaced
    MPR_TRY(t5_load(m, t, enc_lut, dec_lut, /*fresh=*/false, nullptr));
    MPR_HIP(hipDeviceSynchronize());
    return MPR_OK;
  });
}

int mpr_t5_update_async(mpr_model* mm, const float* const* t, int32_t nt, void* stream) {
  return guarded([&]() -> int {
    MPR_REQUIRE(mm && mm->kind == mpr_model::T5 && t, "t5_update_async: bad arguments");
    T5Model* m = static_cast<T5Model*>(mm);
    const int expect = 2 + 8 * m->Le + 1 + 1 + 13 * m->Ld + 2;
    MPR_REQUIRE(nt == expect, "t5_update_async: expected %d tensors, got %d", expect, nt);
    for (int i = 0; i < nt; ++i) {  // device memory only: the copies are kernels
      hipPointerAttribute_t at;
      MPR_REQUIRE(t[i] && hipPointerGetAttributes(&at, t[i]) == hipSuccess &&
                      at.type == hipMemoryTypeDevice,
                  "t5_update_async: tensor %d is not device memory", i);
    }
    return t5_load(m, t, nullptr, nullptr, /*fresh=*/false, S(stream), /*device_src=*/true);
  });
}

#define T5_HANDLE(m)                                                            \
  MPR_REQUIRE((m) && (m)->kind == mpr_model::T5, "t5: not a T5 handle");        \
  T5Model* t5 = static_cast<T5Model*>(m)

int mpr_t5_embed(mpr_model* m, const int32_t* ids, int32_t b, int32_t len, float* out,
                 int64_t out_bs, int32_t row0, void* stream) {
  return guarded([&]() -> int {
    T5_HANDLE(m);
    MPR_TRY(t5->use_slot(0));
    return t5->embed(ids, b, len, out, out_bs, row0, S(stream));
  });
}

int mpr_t5_encode(mpr_model* m, const float* embeds, const float* mask, int32_t b, int32_t L,
                  float* out, void* stream) {
  return guarded([&]() -> int {
    T5_HANDLE(m);
    MPR_TRY(t5->use_slot(0));
    return t5->encode(embeds, mask, b, L, out, S(stream));
  });
}

int mpr_t5_generate(mpr_model* m, const float* embeds, const float* mask, int32_t b, int32_t L,
                    int32_t max_new, int32_t start, int32_t eos, int32_t pad, int32_t* out_tokens,
                    void* stream) {
  return mpr_t5_generate_slot(m, 0, embeds, mask, b, L, max_new, start, eos, pad, out_tokens,
                              stream);
}

int mpr_t5_generate_slot(mpr_model* m, int32_t slot, const float* embeds, const float* mask,
                         int32_t b, int32_t L, int32_t max_new, int32_t start, int32_t eos,
                         int32_t pad, int32_t* out_tokens, void* stream) {
  return guarded([&]() -> int {
    T5_HANDLE(m);
    return t5->generate(embeds, mask, b, L, max_new, start, eos, pad, out_tokens, S(stream),
                        slot);
  });
}

int mpr_t5_generate_stop(mpr_model* m, int32_t slot, const float* embeds, const float* mask,
                         int32_t b, int32_t L, int32_t max_new, int32_t start, int32_t eos,
                         int32_t pad, int32_t stop_chunk, int32_t* out_tokens,
                         int32_t* steps_run, void* stream) {
  return guarded([&]() -> int {
    T5_HANDLE(m);
    MPR_REQUIRE(stop_chunk >= 1 && stop_chunk <= 512, "generate_stop: chunk %d", stop_chunk);
    int steps = 0;
    MPR_TRY(t5->generate_groups(1, &embeds, &mask, &b, &L, max_new, start, eos, pad, &out_tokens,
                                S(stream), slot, stop_chunk, &steps));
    if (steps_run) *steps_run = steps;
    return MPR_OK;
  });
}

int mpr_t5_generate_pair(mpr_model* m, int32_t slot, const float* embeds_a, const float* mask_a,
                         int32_t b_a, int32_t L_a, const float* embeds_b, const float* mask_b,
                         int32_t b_b, int32_t L_b, int32_t max_new, int32_t start, int32_t eos,
                         int32_t pad, int32_t* out_a, int32_t* out_b, void* stream) {
  return guarded([&]() -> int {
    T5_HANDLE(m);
    const float* e[2] = {embeds_a, embeds_b};
    const float* k[2] = {mask_a, mask_b};
    const int bs[2] = {b_a, b_b}, ls[2] = {L_a, L_b};
    int32_t* o[2] = {out_a, out_b};
    return t5->generate_groups(2, e, k, bs, ls, max_new, start, eos, pad, o, S(stream), slot);
  });
}

int mpr_t5_generate_batches(mpr_model* m, int32_t slot, int32_t n,
                            const float* const* embeds, const float* const* masks,
                            const int32_t* b, const int32_t* L, int32_t max_new, int32_t start,
                            int32_t eos, int32_t pad, int32_t* const* outs, void* stream) {
  return guarded([&]() -> int {
    T5_HANDLE(m);
    MPR_REQUIRE(n >= 1 && n <= T5Model::MAX_GROUPS && embeds && masks && b && L && outs,
                "t5 generate_batches: n=%d (1 to %d) and every array", n, T5Model::MAX_GROUPS);
    int bs[T5Model::MAX_GROUPS], ls[T5Model::MAX_GROUPS];
    for (int i = 0; i < n; ++i) {
      bs[i] = b[i];
      ls[i] = L[i];
    }
    return t5->generate_groups(n, embeds, masks, bs, ls, max_new, start, eos, pad, outs,
                               S(stream), slot);
  });
}

int mpr_t5_generate_begin(mpr_model* m, int32_t slot, int32_t n, const float* const* embeds,
                          const float* const* masks, const int32_t* b, const int32_t* L,
                          int32_t max_new, int32_t start, int32_t eos, int32_t pad,
                          int32_t stop_chunk, int32_t ahead, int32_t* const* outs,
                          void* stream) {
  return guarded([&]() -> int {
    T5_HANDLE(m);
    MPR_REQUIRE(n >= 1 && n <= T5Model::MAX_GROUPS && embeds && masks && b && L && outs,
                "t5 generate_begin: n=%d (1 to %d) and every array", n, T5Model::MAX_GROUPS);
    MPR_REQUIRE(stop_chunk >= 0 && stop_chunk <= 512, "generate_begin: chunk %d", stop_chunk);
    int bs[T5Model::MAX_GROUPS], ls[T5Model::MAX_GROUPS];
    for (int i = 0; i < n; ++i) {
      bs[i] = b[i];
      ls[i] = L[i];
    }
    return t5->gen_begin(n, embeds, masks, bs, ls, max_new, start, eos, pad, outs, S(stream),
                         slot, stop_chunk, ahead);
  });
}

int mpr_t5_generate_poll(mpr_model* m, int32_t slot, int32_t wait, int32_t* done,
                         int32_t* steps_run, void* stream) {
  return guarded([&]() -> int {
    T5_HANDLE(m);
    MPR_REQUIRE(done != nullptr, "generate_poll: done is required");
    int d = 0, st = 0;
    MPR_TRY(t5->gen_poll(slot, wait != 0, &d, &st, S(stream)));
    *done = d;
    if (steps_run) *steps_run = st;
    return MPR_OK;
  });
}

int mpr_t5_set_decode_stream(mpr_model* m, int32_t slot, void* decode_stream) {
  return guarded([&]() -> int {
    T5_HANDLE(m);
    return t5->set_decode_stream(slot, S(decode_stream));
  });
}

int mpr_t5_logits(mpr_model* m, const float* embeds, const float* mask, int32_t b, int32_t L,
                  const int32_t* dec_in, int32_t T, float* logits, void* stream) {
  return guarded([&]() -> int {
    T5_HANDLE(m);
    MPR_TRY(t5->use_slot(0));
    return t5->logits_tf(embeds, mask, b, L, dec_in, T, logits, S(stream));
  });
}

int mpr_cross_entropy(const float* logits, const int32_t* labels, int64_t n, int32_t vocab,
                      float* out, void* stream) {
  return guarded([&]() -> int {
    // 2n floats of per-row partials, one buffer per stream (calls on different streams may be
    // in flight together)
    static std::map<void*, std::unique_ptr<DevBuf>> by_stream;
    auto& ws = by_stream[stream];
    if (!ws) ws = std::make_unique<DevBuf>();
    MPR_TRY(ws->ensure((size_t)n * 2 * sizeof(float)));
    return cross_entropy(logits, labels, n, vocab, ws->as<float>(), out, S(stream));
  });
}

int mpr_model_destroy(mpr_model* m) {
  delete m;
  return MPR_OK;
}

int mpr_probe_enable(int32_t kind) {
  MPR_REQUIRE(kind >= 0 && kind <= 3, "probe: kind %d", kind);
  return probe_enable(kind);
}

int mpr_probe_read(double* ms, int64_t* launches, double* flops, double* bytes) {
  return guarded([&]() -> int { return probe_read(ms, launches, flops, bytes); });
}

int mpr_probe_replay(int32_t iters, void* stream, double* ms, int64_t* launches, double* flops,
                     double* bytes) {
  return guarded([&]() -> int {
    return probe_replay(iters, S(stream), ms, launches, flops, bytes);
  });
}

int mpr_probe_clear(void) {
  return guarded([&]() -> int { return probe_clear(); });
}

}  // extern "C"
