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

struct DevBuf {
  void* ptr = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  void release() {
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    bytes = 0;
  }
  int ensure(size_t want) {
    if (want <= bytes) return MPR_OK;
    release();
    if (want == 0) return MPR_OK;
    ++alloc_generation();
    hipError_t e = hipMalloc(&ptr, want);
    if (e != hipSuccess) {
      ptr = nullptr;
      set_error("hipMalloc(%zu) failed: %s", want, hipGetErrorString(e));
      return MPR_ENOMEM;
    }
    bytes = want;
    return MPR_OK;
  }
  template <class T>
  T* as() const { return reinterpret_cast<T*>(ptr); }
};

__host__ __device__ inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Copies `count` floats from a host-or-device pointer into a fresh device buffer.
int upload(DevBuf& dst, const float* src, size_t count);

}  // namespace mpr
