// debug.hip — deterministic detectors for cross-kernel memory hazards (common.h "Debug switches"):
// the registry of live device buffers, their guard bands, content hashes of every buffer, and the
// decode-chain trace of T5Model::generate.  None of this runs unless a debug switch is set or an
// mpr_debug_* entry point is called; the product path only pays one registry insert per buffer
// allocation.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <unordered_set>

#include "models.h"

namespace mpr {

namespace {
bool env_on(const char* name) {
  const char* e = getenv(name);
  return e && e[0] == '1';
}

std::mutex& reg_mu() {
  static std::mutex m;
  return m;
}
std::unordered_set<DevBuf*>& registry() {
  static std::unordered_set<DevBuf*>* r = new std::unordered_set<DevBuf*>();  // outlives statics
  return *r;
}

// every live buffer, by address (a stable order for reports)
std::vector<DevBuf*> live_buffers() {
  std::lock_guard<std::mutex> lk(reg_mu());
  std::vector<DevBuf*> v(registry().begin(), registry().end());
  std::sort(v.begin(), v.end(), [](const DevBuf* a, const DevBuf* b) { return a->ptr < b->ptr; });
  return v;
}

uint64_t fnv1a(const uint8_t* p, size_t n, uint64_t h) {
  for (size_t i = 0; i < n; ++i) {
    h ^= p[i];
    h *= 1099511628211ull;
  }
  return h;
}
}  // namespace

bool debug_guard() {
  static const bool on = env_on("MPR_DEBUG_GUARD");
  return on;
}
bool debug_lds_poison() {
  static const bool on = env_on("MPR_DEBUG_LDS_POISON");
  return on;
}
bool debug_decode_trace() {
  static const bool on = env_on("MPR_DECODE_TRACE");
  return on;
}

void devbuf_track(DevBuf* b, bool live) {
  std::lock_guard<std::mutex> lk(reg_mu());
  if (live)
    registry().insert(b);
  else
    registry().erase(b);
}

// T5Model's decode trace (t5.hip): one segment per traced kernel output
int T5Model::trace(int kind, int t, int l, const void* p, int64_t rows, int64_t cols, int64_t ld,
                   hipStream_t s) {
  if (!debug_decode_trace() || rows <= 0 || cols <= 0) return MPR_OK;
  const int64_t n = rows * cols;
  MPR_REQUIRE((size_t)(ws->trace_off + n) * 4 <= ws->trace.bytes,
              "decode trace: %lld floats past the %zu-byte trace", (long long)(ws->trace_off + n),
              ws->trace.bytes);
  MPR_HIP(hipMemcpy2DAsync(ws->trace.as<float>() + ws->trace_off, (size_t)cols * 4, p,
                           (size_t)ld * 4, (size_t)cols * 4, (size_t)rows,
                           hipMemcpyDeviceToDevice, s));
  ws->segs.push_back({kind, t, l, rows, cols, ws->trace_off});
  ws->trace_off += n;
  return MPR_OK;
}

}  // namespace mpr

using namespace mpr;

extern "C" {

int mpr_debug_flags(int32_t* flags) {
  MPR_REQUIRE(flags != nullptr, "debug_flags: null");
  *flags = (debug_guard() ? 1 : 0) | (debug_lds_poison() ? 2 : 0) | (debug_decode_trace() ? 4 : 0);
  return MPR_OK;
}

int mpr_debug_check_guards(int32_t* n_bad, char* report, int32_t report_len) {
  MPR_REQUIRE(n_bad != nullptr, "check_guards: n_bad is null");
  *n_bad = 0;
  if (report && report_len > 0) report[0] = 0;
  MPR_REQUIRE(debug_guard(), "check_guards: set MPR_DEBUG_GUARD=1 before the library loads");
  MPR_HIP(hipDeviceSynchronize());
  std::string rep;
  std::vector<uint8_t> band(GUARD_BYTES);
  for (DevBuf* b : live_buffers()) {
    if (!b->guard) continue;
    for (int side = 0; side < 2; ++side) {
      const char* src = side == 0 ? static_cast<const char*>(b->base)
                                  : static_cast<const char*>(b->ptr) + b->bytes;
      MPR_HIP(hipMemcpy(band.data(), src, b->guard, hipMemcpyDeviceToHost));
      size_t first = b->guard, last = 0, count = 0;
      for (size_t i = 0; i < b->guard; ++i)
        if (band[i] != 0xFF) {
          first = std::min(first, i);
          last = i;
          ++count;
        }
      if (!count) continue;
      ++*n_bad;
      if (rep.size() < 4096) {
        char line[512];
        // offsets relative to the buffer: negative below it, past its end above it
        const long long f = side == 0 ? (long long)first - (long long)b->guard
                                      : (long long)(b->bytes + first);
        const long long l = side == 0 ? (long long)last - (long long)b->guard
                                      : (long long)(b->bytes + last);
        uint32_t w = 0;
        memcpy(&w, band.data() + (first & ~(size_t)3), 4);
        float fv;
        memcpy(&fv, &w, 4);
        snprintf(line, sizeof(line),
                 "buffer %p (%zu B): %s band, %zu bytes changed at offsets [%lld, %lld], first "
                 "word 0x%08x (%g)\n",
                 b->ptr, b->bytes, side == 0 ? "lower" : "upper", count, f, l, w, fv);
        rep += line;
      }
    }
  }
  if (report && report_len > 0) {
    strncpy(report, rep.c_str(), (size_t)report_len - 1);
    report[report_len - 1] = 0;
  }
  return MPR_OK;
}

int mpr_debug_hash_buffers(uint64_t* hashes, uint64_t* ptrs, int64_t* sizes, int32_t cap,
                           int32_t* n) {
  MPR_REQUIRE(n != nullptr && cap >= 0, "hash_buffers: bad arguments");
  MPR_HIP(hipDeviceSynchronize());
  const std::vector<DevBuf*> bufs = live_buffers();
  *n = (int32_t)bufs.size();
  std::vector<uint8_t> host;
  for (size_t i = 0; i < bufs.size() && (int32_t)i < cap; ++i) {
    const DevBuf* b = bufs[i];
    uint64_t h = 1469598103934665603ull;
    const size_t chunk = 64 << 20;
    host.resize(std::min(chunk, b->bytes));
    for (size_t off = 0; off < b->bytes; off += chunk) {
      const size_t m = std::min(chunk, b->bytes - off);
      MPR_HIP(hipMemcpy(host.data(), static_cast<const char*>(b->ptr) + off, m,
                        hipMemcpyDeviceToHost));
      h = fnv1a(host.data(), m, h);
    }
    if (hashes) hashes[i] = h;
    if (ptrs) ptrs[i] = reinterpret_cast<uint64_t>(b->ptr);
    if (sizes) sizes[i] = (int64_t)b->bytes;
  }
  return MPR_OK;
}

// The pointers and sizes of a T5 handle's workspace slot buffers, in T5Work's field order (the
// Python side names them), so a hash report can say which workspace a changed buffer belongs to.
int mpr_debug_t5_workspace(mpr_model* m, int32_t slot, uint64_t* ptrs, int64_t* sizes,
                           int32_t cap, int32_t* n) {
  MPR_REQUIRE(m && m->kind == mpr_model::T5 && n, "t5_workspace: not a T5 handle");
  T5Model* t5 = static_cast<T5Model*>(m);
  MPR_TRY(t5->use_slot(slot));
  T5Work& w = *t5->work[slot];
  const DevBuf* f[] = {&w.x,        &w.h,        &w.qkv,      &w.ao,       &w.ff,
                       &w.enc_out,  &w.cross_kv, &w.cache,    &w.dx,       &w.dq,
                       &w.unfinished, &w.cur_tok, &w.enc_in,  &w.mask_in,  &w.part_val,
                       &w.part_idx, &w.tok_buf,  &w.logits,   &w.mask_enc, &w.enc_tmp,
                       &w.ax,       &w.yq,       &w.hz,       &w.x1ss,     &w.x2ss};
  *n = (int32_t)(sizeof(f) / sizeof(f[0]));
  for (int i = 0; i < *n && i < cap; ++i) {
    if (ptrs) ptrs[i] = reinterpret_cast<uint64_t>(f[i]->ptr);
    if (sizes) sizes[i] = (int64_t)f[i]->bytes;
  }
  return MPR_OK;
}

int mpr_debug_t5_trace(mpr_model* m, int32_t slot, float* dst, int64_t cap_floats,
                       int64_t* n_floats, int64_t* segs, int32_t seg_cap, int32_t* n_segs,
                       void* stream) {
  MPR_REQUIRE(m && m->kind == mpr_model::T5 && n_floats && n_segs, "t5_trace: bad arguments");
  MPR_REQUIRE(debug_decode_trace(), "t5_trace: set MPR_DECODE_TRACE=1 before the library loads");
  T5Model* t5 = static_cast<T5Model*>(m);
  MPR_TRY(t5->use_slot(slot));
  T5Work& w = *t5->work[slot];
  *n_floats = w.trace_off;
  *n_segs = (int32_t)w.segs.size();
  if (dst && w.trace_off > 0) {
    MPR_REQUIRE(cap_floats >= w.trace_off, "t5_trace: %lld floats do not fit %lld",
                (long long)w.trace_off, (long long)cap_floats);
    MPR_HIP(hipMemcpyAsync(dst, w.trace.ptr, (size_t)w.trace_off * 4, hipMemcpyDeviceToDevice,
                           reinterpret_cast<hipStream_t>(stream)));
  }
  for (int i = 0; segs && i < (int)w.segs.size() && i < seg_cap; ++i)
    for (int j = 0; j < 6; ++j) segs[(int64_t)i * 6 + j] = w.segs[i][j];
  return MPR_OK;
}

}  // extern "C"
