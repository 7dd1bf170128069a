// similarity.hip — the general (broadcasting) form of the reference's cosine_similarity
// (utils.py:57-62):  (sum(x1 * x2, dim) / clamp(norm(x1, 2, dim) * norm(x2, 2, dim), eps))
// for any pair of broadcastable operands.  Two strided device kernels: a reduction of a . b along
// one axis for every element of the remaining (broadcast) shape — one wave per output, lanes over
// the axis, shuffle tree (the three reductions of the formula: x1 . x2 over the broadcast axis,
// x1 . x1 and x2 . x2 over each operand's own axis) — and the final division, broadcasting the
// three results.  The aligned-rows and [B,1,D] x [1,N,D] forms keep their fused kernels
// (cosine_rows, the index scan in cosine mode); this serves every other layout.
#include "kernels.h"

namespace mpr {
namespace {

constexpr int SV_MAX = 8;
struct StridedView {
  int nd = 0;
  int64_t shape[SV_MAX] = {};
  int64_t st[3][SV_MAX] = {};  // element strides of up to three operands (0: broadcast)
};

__device__ __forceinline__ void sv_offsets(const StridedView& v, int64_t o, int nops,
                                           int64_t* off) {
  for (int p = 0; p < 3; ++p) off[p] = 0;
  for (int d = v.nd - 1; d >= 0; --d) {
    const int64_t i = o % v.shape[d];
    o /= v.shape[d];
    for (int p = 0; p < nops; ++p) off[p] += i * v.st[p][d];
  }
}

__global__ __launch_bounds__(256) void dot_reduce_kernel(const float* a, const float* b,
                                                         StridedView v, int64_t D, int64_t ta,
                                                         int64_t tb, int64_t n_out, int take_sqrt,
                                                         float* out) {
  const int64_t o = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (o >= n_out) return;
  int64_t off[3];
  sv_offsets(v, o, 2, off);
  float acc = 0.f;
  for (int64_t t = lane; t < D; t += 64) acc += a[off[0] + t * ta] * b[off[1] + t * tb];
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) acc += __shfl_xor(acc, s, 64);
  if (lane == 0) out[o] = take_sqrt ? sqrtf(acc) : acc;
}

__global__ __launch_bounds__(256) void cos_combine_kernel(const float* w12, const float* n1,
                                                          const float* n2, StridedView v,
                                                          int64_t n_out, float eps, float* out) {
  const int64_t o = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (o >= n_out) return;
  int64_t off[3];
  sv_offsets(v, o, 3, off);
  out[o] = w12[off[0]] / fmaxf(n1[off[1]] * n2[off[2]], eps);
}

int make_view(int nd, const int64_t* shape, const int64_t* const* strides, int nops,
              StridedView* v, int64_t* n_out) {
  MPR_REQUIRE(nd >= 0 && nd <= SV_MAX, "similarity: %d output dims (at most %d)", nd, SV_MAX);
  v->nd = nd;
  int64_t n = 1;
  for (int d = 0; d < nd; ++d) {
    MPR_REQUIRE(shape[d] >= 0, "similarity: negative extent");
    v->shape[d] = shape[d];
    n *= shape[d];
    for (int p = 0; p < nops; ++p) v->st[p][d] = strides[p][d];
  }
  *n_out = n;
  return MPR_OK;
}

}  // namespace
}  // namespace mpr

extern "C" {

int mpr_dot_reduce(const float* a, const float* b, int32_t nd, const int64_t* out_shape,
                   const int64_t* a_strides, const int64_t* b_strides, int64_t axis_len,
                   int64_t a_axis_stride, int64_t b_axis_stride, int32_t take_sqrt, float* out,
                   void* stream) {
  try {
    using namespace mpr;
    MPR_REQUIRE(a && b && out && axis_len >= 0, "dot_reduce: bad arguments");
    StridedView v;
    int64_t n = 0;
    const int64_t* st[2] = {a_strides, b_strides};
    MPR_TRY(make_view(nd, out_shape, st, 2, &v, &n));
    if (n == 0) return MPR_OK;
    hipLaunchKernelGGL(dot_reduce_kernel, dim3((unsigned)cdiv(n, 4)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), a, b, v, axis_len, a_axis_stride,
                       b_axis_stride, n, take_sqrt ? 1 : 0, out);
    MPR_LAUNCHED();
    return MPR_OK;
  } catch (...) {
    mpr::set_error("dot_reduce: exception");
    return MPR_EINVAL;
  }
}

int mpr_cos_combine(const float* w12, const float* n1, const float* n2, int32_t nd,
                    const int64_t* out_shape, const int64_t* w12_strides,
                    const int64_t* n1_strides, const int64_t* n2_strides, float eps, float* out,
                    void* stream) {
  try {
    using namespace mpr;
    MPR_REQUIRE(w12 && n1 && n2 && out, "cos_combine: bad arguments");
    StridedView v;
    int64_t n = 0;
    const int64_t* st[3] = {w12_strides, n1_strides, n2_strides};
    MPR_TRY(make_view(nd, out_shape, st, 3, &v, &n));
    if (n == 0) return MPR_OK;
    hipLaunchKernelGGL(cos_combine_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), w12, n1, n2, v, n, eps, out);
    MPR_LAUNCHED();
    return MPR_OK;
  } catch (...) {
    mpr::set_error("cos_combine: exception");
    return MPR_EINVAL;
  }
}

}  // extern "C"
