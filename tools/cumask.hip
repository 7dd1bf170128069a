// cumask.hip — which CUs (XCC, SE, CU) run the blocks of a stream created with a CU mask
// (development aid for the decode / encoder CU partition).
// build: hipcc --offload-arch=gfx950 -O3 tools/cumask.hip -o tools/cumask
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <set>
#include <vector>

__global__ void where(unsigned* out) {
  if (threadIdx.x == 0) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc;
    // keep the block resident a little so the dispatcher spreads the grid
    long long t0 = clock64();
    while (clock64() - t0 < 200000) {
    }
  }
}

int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  printf("CUs %d\n", p.multiProcessorCount);
  const int nb = 2048;
  unsigned* d;
  (void)hipMalloc(&d, nb * 8);
  std::vector<unsigned> h(nb * 2);
  const char* names[] = {"bits 0-31", "bits 0-63", "every 4th bit", "bits 224-255"};
  for (int v = 0; v < 4; ++v) {
    std::vector<uint32_t> m(8, 0);
    for (int i = 0; i < 256; ++i) {
      bool on = v == 0 ? i < 32 : v == 1 ? i < 64 : v == 2 ? i % 4 == 0 : i >= 224;
      if (on) m[i / 32] |= 1u << (i % 32);
    }
    hipStream_t s;
    if (hipExtStreamCreateWithCUMask(&s, 8, m.data()) != hipSuccess) {
      printf("mask create failed\n");
      return 1;
    }
    hipLaunchKernelGGL(where, dim3(nb), dim3(64), 0, s, d);
    (void)hipStreamSynchronize(s);
    (void)hipMemcpy(h.data(), d, nb * 8, hipMemcpyDeviceToHost);
    std::set<std::tuple<unsigned, unsigned, unsigned>> cus;
    std::set<unsigned> xccs;
    for (int b = 0; b < nb; ++b) {
      const unsigned hw = h[2 * b], xcc = h[2 * b + 1] & 0xf;
      const unsigned cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 0x7;
      cus.insert({xcc, se * 2 + sh, cu});
      xccs.insert(xcc);
    }
    printf("%-14s: %zu distinct CUs on %zu XCCs:", names[v], cus.size(), xccs.size());
    std::vector<int> per(8, 0);
    for (auto& c : cus) per[std::get<0>(c)]++;
    for (int x = 0; x < 8; ++x) printf(" %d", per[x]);
    printf("\n");
    (void)hipStreamDestroy(s);
  }
  return 0;
}
