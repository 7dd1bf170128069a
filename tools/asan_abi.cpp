// asan_abi.cpp — host AddressSanitizer check of the C ABI's argument handling (development aid):
// built by `make -C multimodalpromptretrieval_amd/csrc asan` against the library compiled with
// host-side ASan (`-Xarch_host -fsanitize=address`; device code is not instrumented), it calls
// every entry point that validates its arguments on the host with bad / null / oversized
// arguments and checks each is refused with an error code and message — no GPU needed, and any
// host out-of-bounds access or leak in those paths aborts the run.
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "../include/mpr.h"

static int fails = 0;
static void expect_error(int rc, const char* what) {
  if (rc == 0) {
    std::printf("FAIL %s: accepted\n", what);
    ++fails;
    return;
  }
  const char* msg = mpr_last_error();
  if (!msg || !*msg) {
    std::printf("FAIL %s: rc %d with no message\n", what, rc);
    ++fails;
    return;
  }
  std::printf("ok   %s: rc %d (%s)\n", what, rc, msg);
}

int main() {
  int64_t bytes = 0;
  if (mpr_pack_x3_bytes(100, 52, &bytes) != 0 || bytes != 4 * 4 * 3 * 64 * 16) {
    std::printf("FAIL pack_x3_bytes: %lld\n", (long long)bytes);
    ++fails;
  }
  expect_error(mpr_pack_x3_bytes(0, 52, &bytes), "pack_x3_bytes N=0");
  expect_error(mpr_pack_x3_bytes(16, 16, nullptr), "pack_x3_bytes null out");
  expect_error(mpr_pack_x3(nullptr, 16, 16, 16, nullptr, 0, nullptr), "pack_x3 null");
  mpr_index* ix = nullptr;
  expect_error(mpr_index_create(nullptr, 0, 16, 0, 0, &ix), "index_create n=0");
  expect_error(mpr_index_search(nullptr, nullptr, 1, 1, nullptr, nullptr, nullptr),
               "index_search null index");
  float dummy[16] = {0};
  expect_error(mpr_gemm_f32_packed(dummy, 4, dummy, 4, nullptr, dummy, 4, 1, 1, 4, nullptr, 0, 0,
                                   nullptr),
               "gemm_f32_packed without image");
  expect_error(mpr_gemm_f32(dummy, 4, dummy, 4, dummy, 4, 1, 1, 4, nullptr, 0, 7, nullptr),
               "gemm_f32 act 7");
  const int32_t cfg[6] = {0, 0, 0, 0, 0, 0};
  mpr_model* m = nullptr;
  expect_error(mpr_vit_create(cfg, 6, nullptr, 0, &m), "vit_create bad");
  expect_error(mpr_t5_trainer_create(nullptr, 0, nullptr, nullptr, 0, &m), "trainer_create null");
  std::printf(fails ? "%d FAILED\n" : "all refused cleanly\n", fails);
  return fails ? 1 : 0;
}
