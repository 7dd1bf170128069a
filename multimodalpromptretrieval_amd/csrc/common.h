// common.h — shared runtime helpers for libmpr (error state, device buffers, small utilities).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdarg>
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/mpr.h"

namespace mpr {

void set_error(const char* fmt, ...);

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

#define MPR_HIP(expr)                                                                      \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    if (_e != hipSuccess) {                                                                \
      ::mpr::set_error("%s:%d: %s failed: %s", __FILE__, __LINE__, #expr,                  \
                       hipGetErrorString(_e));                                             \
      return MPR_EHIP;                                                                     \
    }                                                                                      \
  } while (0)

#define MPR_REQUIRE(cond, ...)              \
  do {                                      \
    if (!(cond)) {                          \
      ::mpr::set_error(__VA_ARGS__);        \
      return MPR_EINVAL;                    \
    }                                       \
  } while (0)

#define MPR_TRY(expr)            \
  do {                           \
    int _rc = (expr);            \
    if (_rc != MPR_OK) return _rc; \
  } while (0)

// Kernel launch error check (launch config errors surface through hipGetLastError).
#define MPR_LAUNCHED()                                                                    \
  do {                                                                                    \
    hipError_t _e = hipGetLastError();                                                    \
    if (_e != hipSuccess) {                                                               \
      ::mpr::set_error("%s:%d: kernel launch failed: %s", __FILE__, __LINE__,             \
                       hipGetErrorString(_e));                                            \
      return MPR_EHIP;                                                                    \
    }                                                                                     \
  } while (0)

// Owning device buffer (hipMalloc'd).  Grows, never shrinks; not copyable.
// Bumped by every device buffer (re)allocation: a captured graph bakes buffer addresses in, so
// one captured at an older generation may point at freed memory and is re-captured.
inline uint64_t& alloc_generation() {
  static uint64_t g = 0;
  return g;
}

// Debug switches (debug.hip; read once per process, off unless set):
//   MPR_DEBUG_GUARD=1       every DevBuf gets GUARD_BYTES of 0xFF (a float NaN, an int -1) on both
//                           sides; mpr_debug_check_guards reports any band that changed (an
//                           out-of-bounds store) and an out-of-bounds load that matters reads NaN
//   MPR_DEBUG_LDS_POISON=1  the decode chain's kernels fill their LDS with NaN at entry (a read
//                           of LDS the kernel never wrote turns into a NaN in its output)
//   MPR_DECODE_TRACE=1      generate() copies every decode-chain kernel's output into a per-slot
//                           trace (mpr_debug_t5_trace), for run-to-run comparison
bool debug_guard();
bool debug_lds_poison();
bool debug_decode_trace();
constexpr size_t GUARD_BYTES = 64 << 10;
struct DevBuf;
void devbuf_track(DevBuf* b, bool live);  // the registry of live buffers (mpr_debug_*)

struct DevBuf {
  void* ptr = nullptr;
  size_t bytes = 0;
  void* base = nullptr;  // the allocation: ptr - guard
  size_t guard = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  void release() {
    if (base) {
      devbuf_track(this, false);
      (void)hipFree(base);
    }
    ptr = base = nullptr;
    bytes = guard = 0;
  }
  int ensure(size_t want) {
    if (want <= bytes) return MPR_OK;
    release();
    if (want == 0) return MPR_OK;
    ++alloc_generation();
    const size_t g = debug_guard() ? GUARD_BYTES : 0;
    hipError_t e = hipMalloc(&base, want + 2 * g);
    if (e != hipSuccess) {
      base = nullptr;
      set_error("hipMalloc(%zu) failed: %s", want, hipGetErrorString(e));
      return MPR_ENOMEM;
    }
    ptr = static_cast<char*>(base) + g;
    bytes = want;
    guard = g;
    if (g) {
      e = hipMemset(base, 0xFF, g);
      if (e == hipSuccess) e = hipMemset(static_cast<char*>(ptr) + want, 0xFF, g);
      if (e != hipSuccess) {
        set_error("guard fill failed: %s", hipGetErrorString(e));
        return MPR_EHIP;
      }
    }
    devbuf_track(this, true);
    return MPR_OK;
  }
  template <class T>
  T* as() const { return reinterpret_cast<T*>(ptr); }
};

__host__ __device__ inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Copies `count` floats from a host-or-device pointer into a fresh device buffer.
int upload(DevBuf& dst, const float* src, size_t count);

}  // namespace mpr
