// layers.hip — normalisation, attention and data-movement kernels of the encoders.
//
// Row reductions (LayerNorm / T5 RMSNorm) run one 64-lane wave per row with __shfl_xor
// butterflies; attention for the short sequences of this path (ViT 50 tokens, CLIP text <= 77,
// T5 <= 562, decoder steps of 1 query) keeps a 64-key chunk of K and V of one (batch, head) in
// LDS and runs an online softmax per query row, one key per lane.
#include <algorithm>
#include <cfloat>
#include <cstdlib>

#include "decode_attn.h"
#include "kernels.h"

namespace mpr {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}

// ---- LayerNorm / RMSNorm: 32 lanes per row (2 rows per wave), float4 accesses -----------------
// The row, gamma and beta are all requested before the first reduction (one memory round trip);
// rows of width D <= 128 * V4 stay in registers.  Out-of-range slots load clamped, in-range data
// and are zeroed by a select (a guarded load makes hipcc wait for each load separately).
__device__ __forceinline__ float half_sum(float v) {  // over the 32 lanes of a half-wave
#pragma unroll
  for (int off = 16; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

template <int V4>
__device__ __forceinline__ void layernorm_rows(const float* x, int64_t ldx, int M, int D,
                                               const float* g, const float* b, float eps,
                                               float* out, int64_t ldo) {
  const int row = blockIdx.x * 8 + (threadIdx.x >> 5), l32 = threadIdx.x & 31;
  const float* xr = x + (int64_t)min(row, M - 1) * ldx;
  const int D4 = D >> 2;
  f32x4 v[V4], gv[V4], bv[V4];
#pragma unroll
  for (int j = 0; j < V4; ++j) {
    const int c4 = min(l32 + 32 * j, D4 - 1);
    v[j] = reinterpret_cast<const f32x4*>(xr)[c4];
    gv[j] = reinterpret_cast<const f32x4*>(g)[c4];
    bv[j] = reinterpret_cast<const f32x4*>(b)[c4];
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < V4; ++j) {
    if (l32 + 32 * j >= D4) v[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    s += (v[j][0] + v[j][1]) + (v[j][2] + v[j][3]);
  }
  const float mean = half_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < V4; ++j) {
    if (l32 + 32 * j < D4) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = v[j][e] - mean;
        q += d * d;
      }
    }
  }
  const float rstd = 1.0f / sqrtf(half_sum(q) / (float)D + eps);
  if (row >= M) return;
  float* orow = out + (int64_t)row * ldo;
#pragma unroll
  for (int j = 0; j < V4; ++j) {
    const int c4 = l32 + 32 * j;
    if (c4 < D4) {
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (v[j][e] - mean) * rstd * gv[j][e] + bv[j][e];
      reinterpret_cast<f32x4*>(orow)[c4] = o;
    }
  }
}

template <int V4>
__global__ __launch_bounds__(256) void layernorm_kernel(const float* x, int64_t ldx, int M, int D,
                                                        const float* g, const float* b, float eps,
                                                        float* out, int64_t ldo) {
  layernorm_rows<V4>(x, ldx, M, D, g, b, eps, out, ldo);
}

// Up to LN_GROUP LayerNorms in one launch (blockIdx.y picks the problem).  A row's arithmetic
// does not depend on V4 (slots past D are exact zeros), so results equal the single launches.
template <int V4>
__global__ __launch_bounds__(256) void layernorm_group_kernel(LnGroup grp, float eps) {
  const int z = blockIdx.y;
#define MPR_SEL(f) (z == 0 ? grp.p[0].f : z == 1 ? grp.p[1].f : z == 2 ? grp.p[2].f : grp.p[3].f)
  const int M = MPR_SEL(M);
  if ((int)blockIdx.x * 8 >= M) return;
  layernorm_rows<V4>(MPR_SEL(x), MPR_SEL(ldx), M, MPR_SEL(D), MPR_SEL(g), MPR_SEL(b), eps,
                     MPR_SEL(out), MPR_SEL(ldo));
#undef MPR_SEL
}

template <int V4>
__global__ __launch_bounds__(256) void rmsnorm_kernel(const float* x, int64_t ldx, int M, int D,
                                                      const float* w, float eps, float* out,
                                                      int64_t ldo) {
  const int row = blockIdx.x * 8 + (threadIdx.x >> 5), l32 = threadIdx.x & 31;
  const float* xr = x + (int64_t)min(row, M - 1) * ldx;
  const int D4 = D >> 2;
  f32x4 v[V4], wv[V4];
#pragma unroll
  for (int j = 0; j < V4; ++j) {
    const int c4 = min(l32 + 32 * j, D4 - 1);
    v[j] = reinterpret_cast<const f32x4*>(xr)[c4];
    wv[j] = reinterpret_cast<const f32x4*>(w)[c4];
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < V4; ++j) {
    if (l32 + 32 * j >= D4) v[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    s += (v[j][0] * v[j][0] + v[j][1] * v[j][1]) + (v[j][2] * v[j][2] + v[j][3] * v[j][3]);
  }
  const float rstd = 1.0f / sqrtf(half_sum(s) / (float)D + eps);
  if (row >= M) return;
  float* orow = out + (int64_t)row * ldo;
#pragma unroll
  for (int j = 0; j < V4; ++j) {
    const int c4 = l32 + 32 * j;
    if (c4 < D4) {
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = wv[j][e] * (v[j][e] * rstd);
      reinterpret_cast<f32x4*>(orow)[c4] = o;
    }
  }
}

// ---- attention -------------------------------------------------------------------------------
constexpr int ATT_QR = 16;      // query rows per block (4 per wave)
constexpr int ATT_KC = 64;      // keys per LDS chunk (one per lane)
constexpr int ATT_D = 64;       // head dim

__global__ __launch_bounds__(256) void attention_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) float Ks[ATT_KC][ATT_D + 4];
  __shared__ __attribute__((aligned(16))) float Vs[ATT_KC][ATT_D];
  __shared__ __attribute__((aligned(16))) float Qs[ATT_QR][ATT_D];
  __shared__ __attribute__((aligned(16))) float Ps[4][4][ATT_KC];

  const int b = blockIdx.z, h = blockIdx.y, q0 = blockIdx.x * ATT_QR;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR)
  {
    const int r = tid >> 4, c4 = (tid & 15) * 4, i = q0 + r;
    f32x4 qv = {0.f, 0.f, 0.f, 0.f};
    if (i < a.Lq)
      qv = *reinterpret_cast<const f32x4*>(a.q + (int64_t)b * a.q_bs + (int64_t)i * a.q_rs +
                                            h * ATT_D + c4);
    *reinterpret_cast<f32x4*>(&Qs[r][c4]) = qv;
  }
  float m[4], l[4], o[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    m[r] = -INFINITY;
    l[r] = 0.f;
    o[r] = 0.f;
  }
  const int row0 = q0 + wave * 4;
  const float* maskb = a.key_mask ? a.key_mask + (int64_t)b * a.mask_bs : nullptr;
  int lk_end = a.Lk;
  if (a.causal) lk_end = min(lk_end, q0 + ATT_QR - 1 + a.q_pos0 + 1);

  for (int kc = 0; kc < lk_end; kc += ATT_KC) {
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int idx = tid + u * 256, r = idx >> 4, c4 = (idx & 15) * 4, j = kc + r;
      f32x4 kv = {0.f, 0.f, 0.f, 0.f}, vv = {0.f, 0.f, 0.f, 0.f};
      if (j < a.Lk) {
        kv = *reinterpret_cast<const f32x4*>(a.k + (int64_t)b * a.k_bs + (int64_t)j * a.k_rs +
                                              h * ATT_D + c4);
        vv = *reinterpret_cast<const f32x4*>(a.v + (int64_t)b * a.v_bs + (int64_t)j * a.v_rs +
                                              h * ATT_D + c4);
      }
      *reinterpret_cast<f32x4*>(&Ks[r][c4]) = kv;
      *reinterpret_cast<f32x4*>(&Vs[r][c4]) = vv;
    }
    __syncthreads();
    if (row0 >= a.Lq) continue;  // wave-uniform; keeps participating in the barriers

    const int j = kc + lane;
    float s[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int d = 0; d < ATT_D; d += 4) {
      const f32x4 kv = *reinterpret_cast<const f32x4*>(&Ks[lane][d]);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const f32x4 qv = *reinterpret_cast<const f32x4*>(&Qs[wave * 4 + r][d]);
        s[r] += qv[0] * kv[0] + qv[1] * kv[1] + qv[2] * kv[2] + qv[3] * kv[3];
      }
    }
    bool kvalid = j < a.Lk;
    if (maskb && kvalid) kvalid = maskb[j] != 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = row0 + r;
      if (i >= a.Lq) break;  // wave-uniform
      const int qpos = i + a.q_pos0;
      bool valid = kvalid && (!a.causal || j <= qpos);
      float sc = s[r] * a.scale;
      if (a.rel_tab && valid) sc += a.rel_tab[(int64_t)(j - qpos + a.lut_radius) * a.H + h];
      sc = valid ? sc : -INFINITY;
      const float mnew = fmaxf(m[r], wave_max(sc));
      float p = 0.f, alpha = 1.f;
      if (mnew != -INFINITY) {
        p = valid ? expf(sc - mnew) : 0.f;
        alpha = m[r] == -INFINITY ? 0.f : expf(m[r] - mnew);
        m[r] = mnew;
      }
      l[r] = l[r] * alpha + wave_sum(p);
      o[r] *= alpha;
      Ps[wave][r][lane] = p;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int kn = min(ATT_KC, a.Lk - kc);
    for (int jj = 0; jj < kn; jj += 4) {
      const float v0 = Vs[jj][lane], v1 = Vs[jj + 1][lane], v2 = Vs[jj + 2][lane],
                  v3 = Vs[jj + 3][lane];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const f32x4 p = *reinterpret_cast<const f32x4*>(&Ps[wave][r][jj]);
        o[r] += p[0] * v0 + p[1] * v1 + p[2] * v2 + p[3] * v3;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = row0 + r;
    if (i < a.Lq)
      a.o[(int64_t)b * a.o_bs + (int64_t)i * a.o_rs + h * ATT_D + lane] = o[r] / l[r];
  }
}

// Single query row (decoder step): one 256-thread block per (batch, head), up to 256 keys per
// pass.  Every global load of a pass — q (broadcast), the thread's key row (16 x 16 B), the
// thread's value slice (4 dims x 16 keys as 16 x 16 B; a wave-instruction covers 4 whole 256 B
// value rows), the mask word and the bias-by-offset word — is independent of the others and
// issued up front, so a pass costs one memory round trip; max / sum / P go through LDS.
constexpr int DEC_KC = 256;

// debug (MPR_DEBUG_LDS_POISON): NaN into n floats of LDS, then a block barrier
__device__ __forceinline__ void poison_lds(float* p, int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) p[i] = __builtin_nanf("");
  __syncthreads();
}

__global__ __launch_bounds__(256) void attention_decode_kernel(AttnArgs a) {
  __shared__ float red[2][4];
  __shared__ float Ps[DEC_KC];
  __shared__ __attribute__((aligned(16))) float Os[16][ATT_D];
  if (a.poison) {
    poison_lds(&red[0][0], 8);
    poison_lds(Ps, DEC_KC);
    poison_lds(&Os[0][0], 16 * ATT_D);
  }
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR)
  const int b = blockIdx.x / a.H, h = blockIdx.x % a.H;
  const float* qp = a.q + (int64_t)b * a.q_bs + h * ATT_D;
  const int qpos = a.q_pos0;
  const float* maskb = a.key_mask ? a.key_mask + (int64_t)b * a.mask_bs : nullptr;
  const float* kb = a.k + (int64_t)b * a.k_bs + h * ATT_D;
  const float* vb = a.v + (int64_t)b * a.v_bs + h * ATT_D;
  int lk_end = a.Lk;
  if (a.causal) lk_end = min(lk_end, qpos + 1);
  const int dg = tid & 15, kg = tid >> 4;  // PV: dims 4*dg..4*dg+3, keys kg*16..kg*16+15
  // folded RMSNorm of the query's source row (t5.hip decode chain): the producing GEMM's per-tile
  // partial sums of squares (<= 64), loaded now and reduced once the first pass's loads are out
  float qscale = a.scale, qpart = 0.f;
  if (a.q_rms_part && lane < a.q_rms_nparts) qpart = a.q_rms_part[(int64_t)b * a.q_rms_nparts + lane];
  float m = -INFINITY, l = 0.f;
  f32x4 o = {0.f, 0.f, 0.f, 0.f};
  for (int kc = 0; kc < lk_end; kc += DEC_KC) {
    const int j = kc + tid;
    const bool in = j < lk_end;
    const float* kp = kb + (int64_t)(in ? j : kc) * a.k_rs;
    f32x4 kr[ATT_D / 4], qv[ATT_D / 4], vr[16];
#pragma unroll
    for (int d = 0; d < ATT_D / 4; ++d) {
      kr[d] = *reinterpret_cast<const f32x4*>(kp + 4 * d);
      qv[d] = *reinterpret_cast<const f32x4*>(qp + 4 * d);
    }
    const int jv0 = kc + kg * 16;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int jv = jv0 + u < lk_end ? jv0 + u : kc;
      vr[u] = *reinterpret_cast<const f32x4*>(vb + (int64_t)jv * a.v_rs + 4 * dg);
    }
    // mask / bias words from a clamped, in-range key: unconditional loads (a load under a
    // per-lane condition is waited for on its own, a second round trip)
    const int jc = in ? j : kc;
    const float* mp = maskb ? maskb + jc : kp;  // any valid address when there is no mask
    const float* bp = a.rel_tab ? a.rel_tab + (int64_t)(jc - qpos + a.lut_radius) * a.H + h : kp;
    const float mraw = *mp, braw = *bp;
    const float mk = maskb ? mraw : 1.f, rb = a.rel_tab ? braw : 0.f;
    if (a.q_rms_part && kc == 0)  // every wave sums the partials in the same fixed order
      qscale = a.scale * (1.0f / sqrtf(wave_sum(qpart) / (float)a.q_rms_n + a.q_rms_eps));
    float s = 0.f;
#pragma unroll
    for (int d = 0; d < ATT_D / 4; ++d)
      s += qv[d][0] * kr[d][0] + qv[d][1] * kr[d][1] + qv[d][2] * kr[d][2] + qv[d][3] * kr[d][3];
    const bool valid = in && mk != 0.f;
    const float sc = valid ? s * qscale + rb : -INFINITY;  // rb is 0 without a bias table
    float wm = wave_max(sc);
    if (lane == 0) red[0][wave] = wm;
    __syncthreads();
    const float cmax = fmaxf(fmaxf(red[0][0], red[0][1]), fmaxf(red[0][2], red[0][3]));
    const float mnew = fmaxf(m, cmax);
    const float p = valid ? expf(sc - mnew) : 0.f;
    const float alpha = (m == -INFINITY) ? (mnew == -INFINITY ? 1.f : 0.f) : expf(m - mnew);
    Ps[tid] = p;
    const float ws = wave_sum(p);
    if (lane == 0) red[1][wave] = ws;
    __syncthreads();
    l = l * alpha + ((red[1][0] + red[1][1]) + (red[1][2] + red[1][3]));
    m = mnew;
    o *= alpha;
#pragma unroll
    for (int u = 0; u < 16; ++u) o += Ps[kg * 16 + u] * vr[u];
    __syncthreads();  // Ps / red reused by the next pass
  }
  *reinterpret_cast<f32x4*>(&Os[kg][4 * dg]) = o;
  __syncthreads();
  if (wave == 0) {
    float s = 0.f;
#pragma unroll
    for (int g = 0; g < 16; ++g) s += Os[g][lane];
    a.o[(int64_t)b * a.o_bs + h * ATT_D + lane] = s / l;
  }
}

// attention_decode_kernel's arithmetic for many (batch, head) pairs with few keys (Lk <= 128,
// grouped decodes of 64-128 rows): one wave per pair, 4 pairs per block, no block barrier.  Lane
// i scores keys i and 64 + i with the same expression; the softmax max / sum and the P.V partials
// combine in the block kernel's order (its waves 2-3, and waves / key groups past Lk, contribute
// exact zeros), so outputs are bit-identical to attention_decode_kernel's.  The block kernel
// issues 48 clamped 16-byte loads per thread for every key slot of its 256 whatever Lk: at 128
// rows x 12 heads that load issue, not the bytes, was its 13.6 us.
template <bool TWO>
__global__ __launch_bounds__(256) void attention_decode_wave_kernel(AttnArgs a) {
  __shared__ float Ps[4][128];
  __shared__ __attribute__((aligned(16))) float Os[4][8][ATT_D];
  if (a.poison) {
    poison_lds(&Ps[0][0], 4 * 128);
    poison_lds(&Os[0][0][0], 4 * 8 * ATT_D);
  }
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int pr = blockIdx.x * 4 + wave;
  if (pr >= a.B * a.H) return;  // wave-uniform; no block barrier below
  dattn::pair<TWO>(a, pr / a.H, pr % a.H, Ps[wave], Os[wave]);  // decode_attn.h
}

// The same pair per 64-thread block (one wave): the few-pair decodes (a 16-row batch: 128 pairs)
// get a block per pair, spread over 128 CUs, instead of 32 four-pair blocks.
__global__ __launch_bounds__(64) void attention_decode_wave1_kernel(AttnArgs a) {
  __shared__ float Ps[128];
  __shared__ __attribute__((aligned(16))) float Os[8][ATT_D];
  if (a.poison) {
    poison_lds(Ps, 128);
    poison_lds(&Os[0][0], 8 * ATT_D);
  }
  dattn::pair(a, blockIdx.x / a.H, blockIdx.x % a.H, Ps, Os);  // decode_attn.h
}

// attention_decode_wave_kernel's pairs with 65..128 keys (a grouped decode's cross-attention over
// its encoder rows) as two waves per pair, one per 64-key half, so twice the loads of a pair are
// in flight per CU.  The halves' maxima, sums and P.V groups meet in LDS and combine in the same
// expressions and order as the one-wave form (fmaxf(max0, max1), (sum0 + sum1) + (0 + 0), the
// groups 0..7 summed in order): bit-identical outputs.  4 pairs per block, 8 waves.
__global__ __launch_bounds__(512) void attention_decode_wave2_kernel(AttnArgs a) {
  using dattn::D;
  __shared__ float Ps[4][128];
  __shared__ __attribute__((aligned(16))) float Os[4][8][D];
  __shared__ float mx[4][2], sm[4][2];
  if (a.poison) {
    poison_lds(&Ps[0][0], 4 * 128);
    poison_lds(&Os[0][0][0], 4 * 8 * D);
    poison_lds(&mx[0][0], 8);
    poison_lds(&sm[0][0], 8);
  }
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ps = wave >> 1, hf = wave & 1;  // pair slot, key half
  const int pr = blockIdx.x * 4 + ps;
  const bool live = pr < a.B * a.H;  // wave-uniform; dead waves still meet the barriers
  const int b = live ? pr / a.H : 0, h = live ? pr % a.H : 0;
  const float* qp = a.q + (int64_t)b * a.q_bs + h * D;
  const int qpos = a.q_pos0;
  const float* maskb = a.key_mask ? a.key_mask + (int64_t)b * a.mask_bs : nullptr;
  const float* kb = a.k + (int64_t)b * a.k_bs + h * D;
  const float* vb = a.v + (int64_t)b * a.v_bs + h * D;
  int lk_end = a.Lk;
  if (a.causal) lk_end = min(lk_end, qpos + 1);
  float qscale = a.scale, qpart = 0.f;
  if (a.q_rms_part && lane < a.q_rms_nparts) qpart = a.q_rms_part[(int64_t)b * a.q_rms_nparts + lane];
  f32x4 qv[D / 4], kr[D / 4];
#pragma unroll
  for (int d = 0; d < D / 4; ++d) qv[d] = *reinterpret_cast<const f32x4*>(qp + 4 * d);
  const int j = hf * 64 + lane;
  const int jc = j < lk_end ? j : 0;
  const float* kp = kb + (int64_t)jc * a.k_rs;
#pragma unroll
  for (int d = 0; d < D / 4; ++d) kr[d] = *reinterpret_cast<const f32x4*>(kp + 4 * d);
  const float* mp = maskb ? maskb + jc : kp;
  const float* bp = a.rel_tab ? a.rel_tab + (int64_t)(jc - qpos + a.lut_radius) * a.H + h : kp;
  const float mraw = *mp, braw = *bp;
  // this half's P.V operands, issued with the key loads
  const int dg = lane & 15, kq = lane >> 4;
  f32x4 vr[16];
  {
    const int jv0 = (hf * 4 + kq) * 16;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int jv = jv0 + u < lk_end ? jv0 + u : 0;
      vr[u] = *reinterpret_cast<const f32x4*>(vb + (int64_t)jv * a.v_rs + 4 * dg);
    }
  }
  if (a.q_rms_part)
    qscale = a.scale * (1.0f / sqrtf(dattn::wsum(qpart) / (float)a.q_rms_n + a.q_rms_eps));
  const float mk = maskb ? mraw : 1.f, rb = a.rel_tab ? braw : 0.f;
  float sd = 0.f;
#pragma unroll
  for (int d = 0; d < D / 4; ++d)
    sd += qv[d][0] * kr[d][0] + qv[d][1] * kr[d][1] + qv[d][2] * kr[d][2] + qv[d][3] * kr[d][3];
  const bool valid = j < lk_end && mk != 0.f;
  const float sc = valid ? sd * qscale + rb : -INFINITY;
  const float hmax = dattn::wmax(sc);
  if (lane == 0) mx[ps][hf] = hmax;
  __syncthreads();
  const float mnew = fmaxf(mx[ps][0], mx[ps][1]);
  const float p = valid ? expf(sc - mnew) : 0.f;
  const float hsum = dattn::wsum(p);
  if (lane == 0) sm[ps][hf] = hsum;
  Ps[ps][hf * 64 + lane] = p;
  __syncthreads();
  const float l = (sm[ps][0] + sm[ps][1]) + (0.f + 0.f);
  const int g = hf * 4 + kq;
  f32x4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < 16; ++u) o += Ps[ps][g * 16 + u] * vr[u];
  *reinterpret_cast<f32x4*>(&Os[ps][g][4 * dg]) = o;
  __syncthreads();
  if (hf == 0 && live) {
    float acc = 0.f;
    for (int gg = 0; gg < 8; ++gg) acc += Os[ps][gg][lane];
    a.o[(int64_t)b * a.o_bs + h * D + lane] = acc / l;
  }
}

// ---- short-sequence attention on MFMA ----------------------------------------------------------
// Block = one (batch, head) and up to 64 queries (4 waves x 16-query tiles), Lk <= ATT_MFMA_MAXK,
// head dim 64, on v_mfma_f32_16x16x4_f32 (exact f32 products, 4-deep k steps).  The block stages
// the (b, h) K and V rows into LDS with every load in flight at once (one memory round trip),
// then each wave computes
//   S^T = K Q^T  — key tiles of 16 as the A operand, the query tile as B; the accumulator gives
//                  lane (query j = lane&15, group g = lane>>4) the scores of keys 16t + 4g + r,
//                  so the softmax over keys is in-lane plus two xor-shuffles (16, 32);
//   O   = P V    — P is used straight from those accumulators as the A operand (k step (t, r):
//                  lane group g supplies key 16t + 4g + r), V rows as B, four 16-wide d tiles.
// The contraction order over the head dim inside a step is permuted identically for K and Q
// (lane group g holds d = 16g .. 16g+15).  Softmax follows torch: p = exp(s - max) / sum, then
// P @ V.
// (Measured and dropped, round 6: an instantiation for <= 128 keys — staging registers and score
// tiles sized for 128, 98 VGPRs and 4 waves per SIMD instead of 168 and 2 — ran the serving loop
// 3,888-4,069 vs 3,891-4,033 QA pairs/s and the index build 10.4k vs 10.4-10.8k rows/s: the
// towers' attentions, ~4 % of kernel time, are not occupancy-bound.)
constexpr int ATT_MFMA_MAXK = 256;
constexpr int ATT_MFMA_KT = ATT_MFMA_MAXK / 16;
constexpr int ATT_MFMA_LD = 68;  // LDS row stride (floats)

__device__ __forceinline__ void attention_mfma_body(const AttnArgs& a, int nqt, float* kv_s) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bh = blockIdx.x, h = bh % a.H, b = bh / a.H;
  const int qt = blockIdx.y * 4 + wave;
  const int li = lane & 15, g = lane >> 4;
  const int q0 = qt * 16;
  const int qi = q0 + li;  // this lane's query (scores layout)
  const int qpos = qi + a.q_pos0;
  int lkb = a.Lk;          // keys any query of the block can see
  if (a.causal) lkb = min(lkb, min(a.Lq, blockIdx.y * 64 + 64) - 1 + a.q_pos0 + 1);
  const int nkb = (lkb + 15) / 16;
  float* Ks = kv_s;
  float* Vs = kv_s + nkb * 16 * ATT_MFMA_LD;

  // this wave's query fragments, then the block's K / V rows (keys past lkb are zero rows)
  const float* qp = a.q + (int64_t)b * a.q_bs + (int64_t)min(qi, a.Lq - 1) * a.q_rs + h * 64 +
                    16 * g;
  f32x4 qf[4];
#pragma unroll
  for (int s4 = 0; s4 < 4; ++s4) qf[s4] = *reinterpret_cast<const f32x4*>(qp + 4 * s4);
  {
    const float* kb = a.k + (int64_t)b * a.k_bs + h * 64;
    const float* vb = a.v + (int64_t)b * a.v_bs + h * 64;
    const int n4 = nkb * 16 * 16;  // float4 per operand
    constexpr int PER = ATT_MFMA_MAXK * 16 / 256;
    f32x4 kr[PER], vr[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int idx = tid + u * 256;
      if (idx < n4) {
        const int key = min(idx >> 4, a.Lk - 1), c4 = (idx & 15) * 4;
        kr[u] = *reinterpret_cast<const f32x4*>(kb + (int64_t)key * a.k_rs + c4);
        vr[u] = *reinterpret_cast<const f32x4*>(vb + (int64_t)key * a.v_rs + c4);
      }
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int idx = tid + u * 256;
      if (idx < n4) {
        const int key = idx >> 4, c4 = (idx & 15) * 4;
        *reinterpret_cast<f32x4*>(Ks + key * ATT_MFMA_LD + c4) = kr[u];
        *reinterpret_cast<f32x4*>(Vs + key * ATT_MFMA_LD + c4) = vr[u];
      }
    }
  }
  __syncthreads();
  if (qt >= nqt) return;  // wave-uniform; no barrier follows

  int lk = lkb;  // keys this wave's queries can see
  if (a.causal) lk = min(lk, q0 + 15 + a.q_pos0 + 1);
  const int nkt = (lk + 15) / 16;
  const float* maskb = a.key_mask ? a.key_mask + (int64_t)b * a.mask_bs : nullptr;
  f32x4 S[ATT_MFMA_KT];
  float m = -INFINITY;
#pragma unroll
  for (int t = 0; t < ATT_MFMA_KT; ++t) {
    if (t < nkt) {  // wave-uniform
      const float* kp = Ks + (16 * t + li) * ATT_MFMA_LD + 16 * g;
      f32x4 kf[4];
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) kf[s4] = *reinterpret_cast<const f32x4*>(kp + 4 * s4);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(kf[s4][e], qf[s4][e], acc, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = 16 * t + 4 * g + r;
        bool valid = key < lk && (!a.causal || key <= qpos);
        if (maskb && valid) valid = maskb[key] != 0.f;
        float sc = acc[r] * a.scale;
        if (a.rel_tab && valid) sc += a.rel_tab[(int64_t)(key - qpos + a.lut_radius) * a.H + h];
        sc = valid ? sc : -INFINITY;
        acc[r] = sc;
        m = fmaxf(m, sc);
      }
      S[t] = acc;
    }
  }
  m = fmaxf(m, __shfl_xor(m, 16, 64));
  m = fmaxf(m, __shfl_xor(m, 32, 64));
  float l = 0.f;
#pragma unroll
  for (int t = 0; t < ATT_MFMA_KT; ++t) {
    if (t < nkt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = S[t][r] == -INFINITY ? 0.f : expf(S[t][r] - m);
        S[t][r] = p;
        l += p;
      }
    }
  }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  const float lok = l > 0.f ? 1.f : 0.f;  // a query with no visible key gets zeros
  const float ld = l > 0.f ? l : 1.f;
  f32x4 O[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) O[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < ATT_MFMA_KT; ++t) {
    if (t < nkt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = (S[t][r] / ld) * lok;
        const float* vp = Vs + (16 * t + 4 * g + r) * ATT_MFMA_LD + li;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
          O[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(p, vp[16 * dt], O[dt], 0, 0, 0);
      }
    }
  }
  // O[dt]: lane (d = 16 dt + li, group g) holds queries q0 + 4g + r
  float* ob = a.o + (int64_t)b * a.o_bs + h * 64 + li;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int q = q0 + 4 * g + r;
    if (q < a.Lq) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) ob[(int64_t)q * a.o_rs + 16 * dt] = O[dt][r];
    }
  }
}

__global__ __launch_bounds__(256) void attention_mfma_kernel(AttnArgs a, int nqt) {
  extern __shared__ __attribute__((aligned(16))) float kv_s[];  // K rows | V rows
  attention_mfma_body(a, nqt, kv_s);
}

// The attentions of up to ATTN_GROUP towers / batches in one launch (blockIdx.z picks the problem; the
// grid covers the largest, blocks past a problem's heads / query tiles exit).  Per block the same
// code and data as attention_mfma_kernel: identical results.
__global__ __launch_bounds__(256) void attention_mfma_group_kernel(AttnGroup grp) {
  extern __shared__ __attribute__((aligned(16))) float kv_s[];
  const int z = blockIdx.z;
  // field-wise wave-uniform selection (dynamic indexing of the kernarg struct spills to scratch)
#define MPR_SEL(f) (z == 0 ? grp.a[0].f : z == 1 ? grp.a[1].f : z == 2 ? grp.a[2].f : grp.a[3].f)
  AttnArgs a;
  a.q = MPR_SEL(q); a.q_bs = MPR_SEL(q_bs); a.q_rs = MPR_SEL(q_rs);
  a.k = MPR_SEL(k); a.k_bs = MPR_SEL(k_bs); a.k_rs = MPR_SEL(k_rs);
  a.v = MPR_SEL(v); a.v_bs = MPR_SEL(v_bs); a.v_rs = MPR_SEL(v_rs);
  a.o = MPR_SEL(o); a.o_bs = MPR_SEL(o_bs); a.o_rs = MPR_SEL(o_rs);
  a.B = MPR_SEL(B); a.H = MPR_SEL(H); a.Lq = MPR_SEL(Lq); a.Lk = MPR_SEL(Lk);
  a.scale = MPR_SEL(scale); a.causal = MPR_SEL(causal); a.q_pos0 = MPR_SEL(q_pos0);
  a.key_mask = MPR_SEL(key_mask); a.mask_bs = MPR_SEL(mask_bs);
  a.rel_tab = MPR_SEL(rel_tab); a.lut_radius = MPR_SEL(lut_radius);
#undef MPR_SEL
  const int nqt = (a.Lq + 15) / 16;
  if ((int)blockIdx.x >= a.B * a.H || (int)blockIdx.y * 4 >= nqt) return;  // whole block
  attention_mfma_body(a, nqt, kv_s);
}

// ---- data movement ----------------------------------------------------------------------------
__global__ void im2col_kernel(const float* img, int B, int S, int p, float* cols) {
  // one thread per float4 of a patch row (kx contiguous)
  const int g = S / p, g2 = g * g, P4 = 3 * p * p / 4;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)B * g2 * P4) return;
  const int e4 = (int)(idx % P4);
  const int64_t pr = idx / P4;
  const int b = (int)(pr / g2), t = (int)(pr % g2), py = t / g, px = t % g;
  const int e = e4 * 4, c = e / (p * p), rem = e % (p * p), ky = rem / p, kx = rem % p;
  const float* src = img + (((int64_t)b * 3 + c) * S + (py * p + ky)) * S + px * p + kx;
  *reinterpret_cast<f32x4*>(cols + pr * (3 * p * p) + e) = *reinterpret_cast<const f32x4*>(src);
}

__global__ void vit_assemble_kernel(const float* patches, const float* cls, const float* pos,
                                    int B, int g2, int W, float* x) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int T = g2 + 1;
  if (idx >= (int64_t)B * T * W) return;
  const int c = (int)(idx % W);
  const int64_t bt = idx / W;
  const int t = (int)(bt % T), b = (int)(bt / T);
  const float base = t == 0 ? cls[c] : patches[((int64_t)b * g2 + t - 1) * W + c];
  x[idx] = base + pos[(int64_t)t * W + c];
}

__global__ void embed_gather_kernel(const float* table, const int32_t* ids, int64_t ids_bs, int B,
                                    int len, int D, const float* pos, float* out, int64_t obs,
                                    int row0) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)B * len * D) return;
  const int c = (int)(idx % D);
  const int64_t bt = idx / D;
  const int t = (int)(bt % len), b = (int)(bt / len);
  float v = table[(int64_t)ids[(int64_t)b * ids_bs + t] * D + c];
  if (pos) v = v + pos[(int64_t)t * D + c];
  out[(int64_t)b * obs + (int64_t)(row0 + t) * D + c] = v;
}

__global__ void eot_gather_kernel(const float* x, const int32_t* tok, int L, int ctx, int D,
                                  float* out) {
  const int b = blockIdx.x;
  __shared__ int e_s;
  if (threadIdx.x == 0) {
    int best = tok[(int64_t)b * ctx], e = 0;
    for (int t = 1; t < ctx; ++t) {
      const int v = tok[(int64_t)b * ctx + t];
      if (v > best) {
        best = v;
        e = t;
      }
    }
    e_s = e < L ? e : L - 1;
  }
  __syncthreads();
  const float* src = x + ((int64_t)b * L + e_s) * D;
  for (int c = threadIdx.x; c < D; c += blockDim.x) out[(int64_t)b * D + c] = src[c];
}

__global__ __launch_bounds__(256) void argmax_rows_kernel(const float* logits, int V, int64_t ld,
                                                          int32_t* out) {
  const int row = blockIdx.x;
  const float* x = logits + (int64_t)row * ld;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int c = threadIdx.x; c < V; c += 256) {
    const float v = x[c];
    if (v > best || (v == best && c < bi)) {
      best = v;
      bi = c;
    }
  }
  __shared__ float bv[256];
  __shared__ int bix[256];
  bv[threadIdx.x] = best;
  bix[threadIdx.x] = bi;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      const float ov = bv[threadIdx.x + s];
      const int oi = bix[threadIdx.x + s];
      if (ov > bv[threadIdx.x] || (ov == bv[threadIdx.x] && oi < bix[threadIdx.x])) {
        bv[threadIdx.x] = ov;
        bix[threadIdx.x] = oi;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) out[row] = bix[0] == 0x7fffffff ? 0 : bix[0];
}

// One block per row: argmax over the vocabulary, then the greedy-search bookkeeping and the
// embedding gather of the chosen token for the next decoder step.
__global__ __launch_bounds__(256) void greedy_step_kernel(const float* part_val,
                                                          const int32_t* part_idx, int nparts,
                                                          int32_t* unfinished, int32_t* tokens,
                                                          int64_t tok_ld, int col, int eos,
                                                          int pad, const float* table, int D,
                                                          float* x, int64_t x_ld, int poison) {
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int unf = unfinished[row];  // issued with the partial loads, not after the argmax
  const float* pv = part_val + (int64_t)row * nparts;
  const int32_t* pi = part_idx + (int64_t)row * nparts;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int p0 = 0; p0 < nparts; p0 += 256 * 8) {
    float v[8];
    int c[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {  // all loads first, lane-contiguous
      const int p = p0 + u * 256 + tid;
      const int pc = p < nparts ? p : 0;
      v[u] = pv[pc];
      c[u] = pi[pc];
      if (p >= nparts) v[u] = -INFINITY;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (v[u] > best || (v[u] == best && c[u] < bi)) {
        best = v[u];
        bi = c[u];
      }
    }
  }
  // wave argmax by shuffles, then the 4 wave results through LDS (one barrier)
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float ov = __shfl_xor(best, off, 64);
    const int oi = __shfl_xor(bi, off, 64);
    if (ov > best || (ov == best && oi < bi)) {
      best = ov;
      bi = oi;
    }
  }
  __shared__ float wb[4];
  __shared__ int wi[4];
  if (poison) {
    poison_lds(wb, 4);
    poison_lds(reinterpret_cast<float*>(wi), 4);
  }
  if (lane == 0) {
    wb[wave] = best;
    wi[wave] = bi;
  }
  __syncthreads();
  best = wb[0];
  bi = wi[0];
#pragma unroll
  for (int w = 1; w < 4; ++w)
    if (wb[w] > best || (wb[w] == best && wi[w] < bi)) {
      best = wb[w];
      bi = wi[w];
    }
  int next = bi == 0x7fffffff ? 0 : bi;
  next = unf ? next : pad;
  if (tid == 0) {
    tokens[(int64_t)row * tok_ld + col] = next;
    unfinished[row] = (unf && next != eos) ? 1 : 0;
  }
  if (x) {
    const float* src = table + (int64_t)next * D;
    for (int c = tid; c < D; c += 256) x[(int64_t)row * x_ld + c] = src[c];
  }
}

__global__ void fill_i32_kernel(int32_t* p, int32_t v, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

__global__ void scale_kernel(float* p, int64_t n, float sc) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = p[i] * sc;
}

// Cross entropy, stage 1: per-row loss (logsumexp - logit[label]) and validity.
__global__ __launch_bounds__(256) void ce_rows_kernel(const float* logits, const int32_t* labels,
                                                      int V, float* loss, float* valid) {
  const int row = blockIdx.x;
  const int lab = labels[row];
  const float* x = logits + (int64_t)row * V;
  float mx = -INFINITY;
  for (int c = threadIdx.x; c < V; c += 256) mx = fmaxf(mx, x[c]);
  __shared__ float red[4];
  mx = wave_max(mx);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float s = 0.f;
  for (int c = threadIdx.x; c < V; c += 256) s += expf(x[c] - mx);
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float tot = red[0] + red[1] + red[2] + red[3];
    const bool ok = lab >= 0 && lab < V;
    loss[row] = ok ? (logf(tot) + mx - x[lab]) : 0.f;
    valid[row] = ok ? 1.f : 0.f;
  }
}

__global__ __launch_bounds__(256) void ce_reduce_kernel(const float* loss, const float* valid,
                                                        int64_t n, float* out) {
  float s = 0.f, c = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += 256) {
    s += loss[i];
    c += valid[i];
  }
  __shared__ float rs[4], rc[4];
  s = wave_sum(s);
  c = wave_sum(c);
  if ((threadIdx.x & 63) == 0) {
    rs[threadIdx.x >> 6] = s;
    rc[threadIdx.x >> 6] = c;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float ts = rs[0] + rs[1] + rs[2] + rs[3], tc = rc[0] + rc[1] + rc[2] + rc[3];
    out[0] = ts / tc;  // NaN when every label is ignored, as torch
  }
}

}  // namespace

int layernorm(const float* x, int64_t ldx, int M, int D, const float* gamma, const float* beta,
              float eps, float* out, int64_t ldo, hipStream_t s) {
  MPR_REQUIRE(D > 0 && D <= 1024 && D % 4 == 0 && ldx % 4 == 0 && ldo % 4 == 0,
              "layernorm: D=%d / strides unsupported (D <= 1024, multiples of 4)", D);
  MPR_REQUIRE(aligned16(x) && aligned16(out) && aligned16(gamma) && aligned16(beta),
              "layernorm: operands must be 16-byte aligned");
  if (M <= 0) return MPR_OK;
  dim3 grid((unsigned)cdiv(M, 8));
  if (D <= 512)
    hipLaunchKernelGGL(layernorm_kernel<4>, grid, dim3(256), 0, s, x, ldx, M, D, gamma, beta, eps,
                       out, ldo);
  else
    hipLaunchKernelGGL(layernorm_kernel<8>, grid, dim3(256), 0, s, x, ldx, M, D, gamma, beta,
                       eps, out, ldo);
  MPR_LAUNCHED();
  return MPR_OK;
}

int layernorm_group(const LnGroup& g, float eps, hipStream_t s) {
  MPR_REQUIRE(g.n >= 1 && g.n <= LN_GROUP, "layernorm_group: %d problems", g.n);
  int64_t blocks = 0;
  int dmax = 0;
  for (int i = 0; i < g.n; ++i) {
    const LnArgs& p = g.p[i];
    MPR_REQUIRE(p.D > 0 && p.D <= 1024 && p.D % 4 == 0 && p.ldx % 4 == 0 && p.ldo % 4 == 0,
                "layernorm: D=%d / strides unsupported (D <= 1024, multiples of 4)", p.D);
    MPR_REQUIRE(aligned16(p.x) && aligned16(p.out) && aligned16(p.g) && aligned16(p.b),
                "layernorm: operands must be 16-byte aligned");
    blocks = std::max<int64_t>(blocks, cdiv(p.M, 8));
    dmax = std::max(dmax, p.D);
  }
  if (blocks == 0) return MPR_OK;
  dim3 grid((unsigned)blocks, (unsigned)g.n);
  if (dmax <= 512)
    hipLaunchKernelGGL(layernorm_group_kernel<4>, grid, dim3(256), 0, s, g, eps);
  else
    hipLaunchKernelGGL(layernorm_group_kernel<8>, grid, dim3(256), 0, s, g, eps);
  MPR_LAUNCHED();
  return MPR_OK;
}

int rmsnorm(const float* x, int64_t ldx, int M, int D, const float* w, float eps, float* out,
            int64_t ldo, hipStream_t s) {
  MPR_REQUIRE(D > 0 && D <= 1024 && D % 4 == 0 && ldx % 4 == 0 && ldo % 4 == 0,
              "rmsnorm: D=%d / strides unsupported (D <= 1024, multiples of 4)", D);
  MPR_REQUIRE(aligned16(x) && aligned16(out) && aligned16(w),
              "rmsnorm: operands must be 16-byte aligned");
  if (M <= 0) return MPR_OK;
  dim3 grid((unsigned)cdiv(M, 8));
  if (D <= 512)
    hipLaunchKernelGGL(rmsnorm_kernel<4>, grid, dim3(256), 0, s, x, ldx, M, D, w, eps, out, ldo);
  else
    hipLaunchKernelGGL(rmsnorm_kernel<8>, grid, dim3(256), 0, s, x, ldx, M, D, w, eps, out, ldo);
  MPR_LAUNCHED();
  return MPR_OK;
}

bool mfma_attention_disabled() {
  static const bool off = [] {
    const char* e = getenv("MPR_MFMA_ATTN");
    return e && e[0] == '0';
  }();
  return off;
}

// MPR_ATT_KEYS64=0 (read per call, as MPR_ATT_WAVE): the grouped decodes' four-pair wave form
// keeps the two-half code for <= 64 keys too (A/B of its TWO = false instantiation, 149 instead of
// 256 VGPRs, 3 waves per SIMD instead of 1; same bits either way).  C5's 256-row t5-base generate
// 44.6 -> 43.9 ms, C5 end to end 44.4-45.9 -> 43.7-43.8 ms per batch (round 6,
// profiles/r06_attn_keys64_ab.txt).
static bool small_keys_off() {
  const char* e = getenv("MPR_ATT_KEYS64");
  return e && e[0] == '0';
}

int attention(const AttnArgs& a, hipStream_t s) {
  MPR_REQUIRE(a.B >= 0 && a.H > 0 && a.Lq >= 0 && a.Lk > 0, "attention: bad shape");
  if (a.B == 0 || a.Lq == 0) return MPR_OK;
  if (a.rel_tab)  // offsets key - query span [-(q_pos0 + Lq - 1), Lk - 1 - q_pos0]
    MPR_REQUIRE(std::max(a.q_pos0 + a.Lq, a.Lk) - 1 <= a.lut_radius,
                "attention: bias table radius %d too small (Lq %d, Lk %d)", a.lut_radius, a.Lq,
                a.Lk);
  MPR_REQUIRE(!a.q_rms_part || (a.Lq == 1 && a.q_rms_n > 0 && a.q_rms_nparts > 0 &&
                                a.q_rms_nparts <= 64),
              "attention: a query row scale only on the one-query decode path");
  if (a.Lq == 1 && debug_lds_poison() && !a.poison) {
    AttnArgs p = a;
    p.poison = 1;
    return attention(p, s);
  }
  if (a.Lq == 1) {
    // Every form below sums in the block kernel's order: outputs bit-identical (tested).  Many
    // pairs with few keys (grouped decodes): four pairs per block, a wave each (two per pair
    // past 64 keys); few pairs: a block per pair (below); > 128 keys: the block kernel.
    const char* we = getenv("MPR_ATT_WAVE");  // read per call (a captured graph keeps its form)
    const bool wave_ok = !(we && we[0] == '0');
    const int lk_end = a.causal ? std::min(a.Lk, a.q_pos0 + 1) : a.Lk;
    if (wave_ok && lk_end <= 128 && (int64_t)a.B * a.H >= 512) {
      const char* w2 = getenv("MPR_ATT_WAVE2");  // read per call (as MPR_ATT_WAVE)
      if (lk_end > 64 && !(w2 && w2[0] == '0'))  // two 64-key halves: a wave each
        hipLaunchKernelGGL(attention_decode_wave2_kernel,
                           dim3((unsigned)cdiv((int64_t)a.B * a.H, 4)), dim3(512), 0, s, a);
      else if (lk_end <= 64 && !small_keys_off())
        hipLaunchKernelGGL(attention_decode_wave_kernel<false>,
                           dim3((unsigned)cdiv((int64_t)a.B * a.H, 4)), dim3(256), 0, s, a);
      else
        hipLaunchKernelGGL(attention_decode_wave_kernel<true>,
                           dim3((unsigned)cdiv((int64_t)a.B * a.H, 4)), dim3(256), 0, s, a);
      MPR_LAUNCHED();
      return MPR_OK;
    }
    // Few pairs (one batch's decode: 16 rows x 8 heads): one wave per block, a block per pair
    // spread over as many CUs (16-row t5-small decode 227.9 -> 215.7 us per step against the
    // 256-thread block kernel, same tokens: profiles/r06_decode_attn_ab.txt).  MPR_ATT_SMALL
    // (read per call; a captured graph keeps its form): "block" = the block kernel, "wave2" =
    // two waves per pair for 65..128 keys.
    const char* sm = getenv("MPR_ATT_SMALL");
    if (wave_ok && lk_end <= 128 && !(sm && sm[0] == 'b')) {
      if (sm && sm[0] == 'w' && sm[4] == '2' && lk_end > 64)
        hipLaunchKernelGGL(attention_decode_wave2_kernel,
                           dim3((unsigned)cdiv((int64_t)a.B * a.H, 4)), dim3(512), 0, s, a);
      else  // (the single-half instantiation for the <= 64-key self-attentions measured no
            // faster here: 16-row step 216.9-221.7 vs 218.7-220.2 us over 4 + 4 alternating
            // tools/decode_ab.py runs — one wave per CU gains nothing from freed registers)
        hipLaunchKernelGGL(attention_decode_wave1_kernel, dim3((unsigned)((int64_t)a.B * a.H)),
                           dim3(64), 0, s, a);
      MPR_LAUNCHED();
      return MPR_OK;
    }
    hipLaunchKernelGGL(attention_decode_kernel, dim3((unsigned)((int64_t)a.B * a.H)), dim3(256),
                       0, s, a);
    MPR_LAUNCHED();
    return MPR_OK;
  }
  int lk = a.Lk;
  if (a.causal) lk = std::min(lk, a.Lq + a.q_pos0);
  if (lk <= ATT_MFMA_MAXK && !mfma_attention_disabled()) {
    const int nqt = (int)cdiv(a.Lq, 16);
    const size_t lds = (size_t)2 * cdiv(lk, 16) * 16 * ATT_MFMA_LD * sizeof(float);
    hipLaunchKernelGGL(attention_mfma_kernel, dim3((unsigned)((int64_t)a.B * a.H),
                                                   (unsigned)cdiv(nqt, 4)),
                       dim3(256), lds, s, a, nqt);
    MPR_LAUNCHED();
    return MPR_OK;
  }
  dim3 grid((unsigned)cdiv(a.Lq, ATT_QR), (unsigned)a.H, (unsigned)a.B);
  hipLaunchKernelGGL(attention_kernel, grid, dim3(256), 0, s, a);
  MPR_LAUNCHED();
  return MPR_OK;
}

int attention_group(const AttnGroup& g, hipStream_t s) {
  MPR_REQUIRE(g.n >= 1 && g.n <= ATTN_GROUP, "attention_group: %d problems", g.n);
  // one launch when every problem takes the MFMA path (prefill, keys <= ATT_MFMA_MAXK)
  bool mfma = !mfma_attention_disabled();
  unsigned gx = 0, gy = 0;
  size_t lds = 0;
  for (int i = 0; i < g.n && mfma; ++i) {
    const AttnArgs& a = g.a[i];
    MPR_REQUIRE(a.B >= 0 && a.H > 0 && a.Lq >= 0 && a.Lk > 0, "attention: bad shape");
    if (a.rel_tab)
      MPR_REQUIRE(std::max(a.q_pos0 + a.Lq, a.Lk) - 1 <= a.lut_radius,
                  "attention: bias table radius %d too small (Lq %d, Lk %d)", a.lut_radius, a.Lq,
                  a.Lk);
    int lk = a.Lk;
    if (a.causal) lk = std::min(lk, a.Lq + a.q_pos0);
    mfma = a.Lq > 1 && lk <= ATT_MFMA_MAXK;
    gx = std::max(gx, (unsigned)((int64_t)a.B * a.H));
    gy = std::max(gy, (unsigned)cdiv(cdiv(a.Lq, 16), 4));
    lds = std::max(lds, (size_t)2 * cdiv(a.Lk, 16) * 16 * ATT_MFMA_LD * sizeof(float));
  }
  if (!mfma) {
    for (int i = 0; i < g.n; ++i) MPR_TRY(attention(g.a[i], s));
    return MPR_OK;
  }
  if (gx == 0 || gy == 0) return MPR_OK;
  hipLaunchKernelGGL(attention_mfma_group_kernel, dim3(gx, gy, (unsigned)g.n), dim3(256), lds, s,
                     g);
  MPR_LAUNCHED();
  return MPR_OK;
}

int im2col_patches(const float* img, int B, int S, int p, float* cols, hipStream_t s) {
  MPR_REQUIRE(S % p == 0 && p % 4 == 0, "im2col: S=%d p=%d", S, p);
  const int g = S / p;
  const int64_t n = (int64_t)B * g * g * (3 * p * p / 4);
  if (n == 0) return MPR_OK;
  hipLaunchKernelGGL(im2col_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, s, img, B, S, p,
                     cols);
  MPR_LAUNCHED();
  return MPR_OK;
}

int vit_assemble(const float* patches, const float* cls, const float* pos, int B, int g2, int W,
                 float* x, hipStream_t s) {
  const int64_t n = (int64_t)B * (g2 + 1) * W;
  if (n == 0) return MPR_OK;
  hipLaunchKernelGGL(vit_assemble_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, s, patches,
                     cls, pos, B, g2, W, x);
  MPR_LAUNCHED();
  return MPR_OK;
}

int embed_gather(const float* table, const int32_t* ids, int64_t ids_bs, int B, int len, int D,
                 const float* pos, float* out, int64_t obs, int row0, hipStream_t s) {
  const int64_t n = (int64_t)B * len * D;
  if (n == 0) return MPR_OK;
  hipLaunchKernelGGL(embed_gather_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, s, table,
                     ids, ids_bs, B, len, D, pos, out, obs, row0);
  MPR_LAUNCHED();
  return MPR_OK;
}

int eot_gather(const float* x, const int32_t* tok, int B, int L, int ctx, int D, float* out,
               hipStream_t s) {
  if (B == 0) return MPR_OK;
  hipLaunchKernelGGL(eot_gather_kernel, dim3(B), dim3(256), 0, s, x, tok, L, ctx, D, out);
  MPR_LAUNCHED();
  return MPR_OK;
}

int argmax_rows(const float* logits, int M, int V, int64_t ld, int32_t* out, hipStream_t s) {
  if (M == 0) return MPR_OK;
  hipLaunchKernelGGL(argmax_rows_kernel, dim3(M), dim3(256), 0, s, logits, V, ld, out);
  MPR_LAUNCHED();
  return MPR_OK;
}

// Row argmax of a logits matrix in P parts per row (the tiled decode head, t5.hip): part p of
// row r covers columns [p * seg, min(N, (p + 1) * seg)); its largest value, ties to the lowest
// column (greedy_step's rule, which then reduces the P parts of each row).
__global__ __launch_bounds__(256) void argmax_parts_kernel(const float* __restrict__ L,
                                                           int64_t ld, int N, int seg,
                                                           float* __restrict__ pv,
                                                           int32_t* __restrict__ pi) {
  const int p = blockIdx.x, row = blockIdx.y, tid = threadIdx.x, lane = tid & 63;
  const int wave = tid >> 6;
  const float* lr = L + (int64_t)row * ld;
  const int c0 = p * seg, c1 = min(N, c0 + seg);
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int b0 = c0; b0 < c1; b0 += 256 * 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {  // all loads first, lane-contiguous
      const int c = b0 + u * 256 + tid;
      v[u] = c < c1 ? lr[c] : -INFINITY;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int c = b0 + u * 256 + tid;
      if (c < c1 && (v[u] > best || (v[u] == best && c < bi))) {
        best = v[u];
        bi = c;
      }
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float ov = __shfl_xor(best, off, 64);
    const int oi = __shfl_xor(bi, off, 64);
    if (ov > best || (ov == best && oi < bi)) {
      best = ov;
      bi = oi;
    }
  }
  __shared__ float wv[4];
  __shared__ int wi[4];
  if (lane == 0) {
    wv[wave] = best;
    wi[wave] = bi;
  }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < 4; ++w)
      if (wv[w] > best || (wv[w] == best && wi[w] < bi)) {
        best = wv[w];
        bi = wi[w];
      }
    const int64_t o = (int64_t)row * gridDim.x + p;
    pv[o] = best;
    pi[o] = bi == 0x7fffffff ? c0 : bi;
  }
}

int argmax_parts(const float* L, int64_t ld, int M, int N, int P, float* pv, int32_t* pi,
                 hipStream_t s) {
  MPR_REQUIRE(M >= 0 && N > 0 && P >= 1 && P <= N, "argmax_parts: M=%d N=%d P=%d", M, N, P);
  if (M == 0) return MPR_OK;
  hipLaunchKernelGGL(argmax_parts_kernel, dim3((unsigned)P, (unsigned)M), dim3(256), 0, s, L, ld,
                     N, (int)cdiv(N, P), pv, pi);
  MPR_LAUNCHED();
  return MPR_OK;
}

int greedy_step(const float* part_val, const int32_t* part_idx, int nparts, int M,
                int32_t* unfinished, int32_t* tokens, int64_t tok_ld, int col, int eos, int pad,
                const float* table, int D, float* x, hipStream_t s, int64_t x_ld) {
  if (M == 0) return MPR_OK;
  MPR_REQUIRE(M <= 256, "greedy_step: %d rows > 256", M);
  hipLaunchKernelGGL(greedy_step_kernel, dim3(M), dim3(256), 0, s, part_val, part_idx, nparts,
                     unfinished, tokens, tok_ld, col, eos, pad, table, D, x,
                     x_ld < 0 ? (int64_t)D : x_ld, debug_lds_poison() ? 1 : 0);
  MPR_LAUNCHED();
  return MPR_OK;
}

int scale_inplace(float* p, int64_t n, float sc, hipStream_t s) {
  if (n == 0) return MPR_OK;
  hipLaunchKernelGGL(scale_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, s, p, n, sc);
  MPR_LAUNCHED();
  return MPR_OK;
}

int fill_i32(int32_t* p, int32_t v, int64_t n, hipStream_t s) {
  if (n == 0) return MPR_OK;
  hipLaunchKernelGGL(fill_i32_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, s, p, v, n);
  MPR_LAUNCHED();
  return MPR_OK;
}

int cross_entropy(const float* logits, const int32_t* labels, int64_t n, int V, float* ws,
                  float* out, hipStream_t s) {
  MPR_REQUIRE(n > 0 && V > 0, "cross_entropy: bad shape");
  hipLaunchKernelGGL(ce_rows_kernel, dim3((unsigned)n), dim3(256), 0, s, logits, labels, V, ws,
                     ws + n);
  MPR_LAUNCHED();
  hipLaunchKernelGGL(ce_reduce_kernel, dim3(1), dim3(256), 0, s, ws, ws + n, n, out);
  MPR_LAUNCHED();
  return MPR_OK;
}

}  // namespace mpr
