// decode_attn.h — one-query decode attention of one (batch, head) pair by one wave, with few keys
// (Lk <= 128): the body of layers.hip's attention_decode_wave_kernel (bit-identical to
// attention_decode_kernel: see layers.hip), as a device function a kernel can call per pair.
// (Round 5 used it for a q|k|v GEMV with the step's self-attention fused in by the last-arriving
// tile block of each head: bit-identical tokens, but 225 -> 298 us per 16-row t5-small step and
// 631 -> 824 for t5-base, profiles/r05_decode_fuse_ab.txt; removed, git show fe367d2.)
#pragma once

#include "kernels.h"

namespace mpr {
namespace dattn {

constexpr int D = 64;  // head dim

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
__device__ __forceinline__ float wmax(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}

// Pair (b, h) of `a` by the calling wave (all 64 lanes): Ps = 128 floats and Os = 8 x 64 floats
// of wave-private LDS.  Lane i scores keys i and 64 + i; softmax max / sum and the P.V partials
// combine in attention_decode_kernel's order (its waves 2-3, and key groups past Lk, contribute
// exact zeros).
// TWO = false: the caller guarantees Lk <= 64 (after the causal clamp), so the second key half
// is dead code and its K / V registers are never allocated (256 -> ~130 VGPRs, 1 -> 3 waves per
// SIMD); every arithmetic expression is the one the runtime test would take: same bits.
template <bool TWO = true>
__device__ __forceinline__ void pair(const AttnArgs& a, int b, int h, float* Ps,
                                     float (*Os)[D]) {
  const int lane = threadIdx.x & 63;
  const float* qp = a.q + (int64_t)b * a.q_bs + h * D;
  const int qpos = a.q_pos0;
  const float* maskb = a.key_mask ? a.key_mask + (int64_t)b * a.mask_bs : nullptr;
  const float* kb = a.k + (int64_t)b * a.k_bs + h * D;
  const float* vb = a.v + (int64_t)b * a.v_bs + h * D;
  int lk_end = a.Lk;
  if (a.causal) lk_end = min(lk_end, qpos + 1);
  const bool two = TWO && lk_end > 64;  // wave-uniform
  float qscale = a.scale, qpart = 0.f;
  if (a.q_rms_part && lane < a.q_rms_nparts) qpart = a.q_rms_part[(int64_t)b * a.q_rms_nparts + lane];
  // scores of keys lane and 64 + lane (clamped rows / words as the block kernel's)
  f32x4 qv[D / 4], kr[2][D / 4];
  float mraw[2], braw[2];
#pragma unroll
  for (int d = 0; d < D / 4; ++d) qv[d] = *reinterpret_cast<const f32x4*>(qp + 4 * d);
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
    if (hf == 1 && !two) break;
    const int j = hf * 64 + lane;
    const int jc = j < lk_end ? j : 0;
    const float* kp = kb + (int64_t)jc * a.k_rs;
#pragma unroll
    for (int d = 0; d < D / 4; ++d) kr[hf][d] = *reinterpret_cast<const f32x4*>(kp + 4 * d);
    const float* mp = maskb ? maskb + jc : kp;
    const float* bp = a.rel_tab ? a.rel_tab + (int64_t)(jc - qpos + a.lut_radius) * a.H + h : kp;
    mraw[hf] = *mp;
    braw[hf] = *bp;
  }
  // the P.V operands too, before any arithmetic: lane (dg, kq) reads dims 4 dg .. +3 of keys
  // (hf * 4 + kq) * 16 .. +15, so every load of the pair is in flight at once (one memory round
  // trip instead of two; the arithmetic is unchanged)
  const int dg = lane & 15, kq = lane >> 4;
  f32x4 vr[2][16];
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
    if (hf == 1 && !two) break;
    const int jv0 = (hf * 4 + kq) * 16;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int jv = jv0 + u < lk_end ? jv0 + u : 0;
      vr[hf][u] = *reinterpret_cast<const f32x4*>(vb + (int64_t)jv * a.v_rs + 4 * dg);
    }
  }
  if (a.q_rms_part)
    qscale = a.scale * (1.0f / sqrtf(wsum(qpart) / (float)a.q_rms_n + a.q_rms_eps));
  float sc[2] = {-INFINITY, -INFINITY};
  bool valid[2] = {false, false};
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
    if (hf == 1 && !two) break;
    const int j = hf * 64 + lane;
    const float mk = maskb ? mraw[hf] : 1.f, rb = a.rel_tab ? braw[hf] : 0.f;
    float s = 0.f;
#pragma unroll
    for (int d = 0; d < D / 4; ++d)
      s += qv[d][0] * kr[hf][d][0] + qv[d][1] * kr[hf][d][1] + qv[d][2] * kr[hf][d][2] +
           qv[d][3] * kr[hf][d][3];
    valid[hf] = j < lk_end && mk != 0.f;
    sc[hf] = valid[hf] ? s * qscale + rb : -INFINITY;
  }
  const float mnew = fmaxf(wmax(sc[0]), wmax(sc[1]));
  float p[2];
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) p[hf] = valid[hf] ? expf(sc[hf] - mnew) : 0.f;
  // the block kernel: l = 0 * alpha + ((w0 + w1) + (w2 + w3)), waves 2-3 (and 1 when Lk <= 64)
  // summing zeros
  const float l = (wsum(p[0]) + wsum(p[1])) + (0.f + 0.f);
  Ps[lane] = p[0];
  Ps[64 + lane] = p[1];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // P.V: lane (dg, kq) sums dims 4 dg .. +3 over key group kq (and 4 + kq), 16 keys each, as the
  // block kernel's thread (dg, kg) does (o starts at 0 * alpha = 0)
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
    if (hf == 1 && !two) break;
    const int g = hf * 4 + kq;
    f32x4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 16; ++u) o += Ps[g * 16 + u] * vr[hf][u];
    *reinterpret_cast<f32x4*>(&Os[g][4 * dg]) = o;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // the block kernel's sum over its 16 key groups in order (groups past Lk add exact zeros)
  float acc = 0.f;
  const int ng = two ? 8 : 4;
  for (int g = 0; g < ng; ++g) acc += Os[g][lane];
  a.o[(int64_t)b * a.o_bs + h * D + lane] = acc / l;
}

}  // namespace dattn
}  // namespace mpr
