// Partial-label soft Dice + per-class BCE (EDiceLoss_partial, reference loss_partial.py:59-99 with
// DiceLoss :10-57) and the hard Dice metric of evaluate_amos.py:92-154, on NDHWC fp32 logits.
//
// Forward is one pass over the logits producing per-class sums (sum p*t, sum p^2, sum t, sum BCE) for
// the whole batch (the reference sums every sample together, :24-36), combined in fp64; the scalar loss
// is formed on the device (no host sync: the reference's per-class .item() at :55 is dropped).
// Backward is one elementwise pass: dL/dp from the sums, then the softmax (or sigmoid) Jacobian.
// Class counts the models use (2, 8, 14, 16) are compile-time so every per-voxel array stays in registers.
#include "common.h"
#include "loss_grad.h"

namespace u3d {

constexpr int LT = 256;
constexpr int CMAX = 32;

// softmax == 1: softmax, 0: sigmoid, 2: identity (inputs are probabilities)
template <int NC>
__device__ __forceinline__ void probs(const float* __restrict__ lg, int C, int softmax, float (&p)[NC]) {
  if constexpr (NC % 4 == 0 && NC <= 16) {
#pragma unroll
    for (int c = 0; c < NC; c += 4) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(lg + c);
      p[c] = v[0]; p[c + 1] = v[1]; p[c + 2] = v[2]; p[c + 3] = v[3];
    }
  } else {
#pragma unroll
    for (int c = 0; c < NC; ++c) p[c] = c < C ? lg[c] : 0.f;
  }
  if (softmax == 1) {
    float m = -INFINITY;
#pragma unroll
    for (int c = 0; c < NC; ++c)
      if (c < C) m = fmaxf(m, p[c]);
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c)
      if (c < C) {
        p[c] = expf(p[c] - m);
        s += p[c];
      }
#pragma unroll
    for (int c = 0; c < NC; ++c)
      if (c < C) p[c] = p[c] / s;
  } else if (softmax == 0) {
#pragma unroll
    for (int c = 0; c < NC; ++c)
      if (c < C) p[c] = 1.f / (1.f + expf(-p[c]));
  }
}

// torch BCELoss element: (t - 1) * max(log1p(-p), -100) - t * max(log(p), -100)
__device__ __forceinline__ float bce_elem(float p, float t) {
  return (t - 1.f) * fmaxf(log1pf(-p), -100.f) - t * fmaxf(logf(p), -100.f);
}

constexpr float LOG2E = 1.4426950408889634f, LN2 = 0.6931471805599453f;

// Softmax path on the hardware transcendentals (v_exp_f32 / v_log_f32 / v_rcp_f32, ~1 ulp): e_c = 2^((x_c-m)
// log2 e), p_c = e_c / s, and the two logs BCE needs are exact identities of the softmax instead of log(p):
//   log p_c = (x_c - m) - ln s,   log(1 - p_c) = ln(s - e_c) - ln s.
// The loss was transcendental-bound with libm expf/logf/log1pf (48 calls per voxel at C = 16).
template <int NC>
__device__ __forceinline__ void softmax_fast(const float* __restrict__ lg, int C, float (&x)[NC], float (&e)[NC],
                                             float& s, float& inv) {
  if constexpr (NC % 4 == 0 && NC <= 16) {
#pragma unroll
    for (int c = 0; c < NC; c += 4) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(lg + c);
      x[c] = v[0]; x[c + 1] = v[1]; x[c + 2] = v[2]; x[c + 3] = v[3];
    }
  } else {
#pragma unroll
    for (int c = 0; c < NC; ++c) x[c] = c < C ? lg[c] : 0.f;
  }
  float m = -INFINITY;
#pragma unroll
  for (int c = 0; c < NC; ++c)
    if (c < C) m = fmaxf(m, x[c]);
  s = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    x[c] -= m;
    e[c] = c < C ? __builtin_amdgcn_exp2f(x[c] * LOG2E) : 0.f;
    s += e[c];
  }
  inv = __builtin_amdgcn_rcpf(s);
}

template <int NC>
__global__ __launch_bounds__(LT) void loss_partial_kernel(const float* __restrict__ lg, const float* __restrict__ lab,
                                                         long long nvox, int C, int softmax, int uce,
                                                         float* __restrict__ ws) {
  __shared__ float red[LT / 64][4 * NC];
  float acc[4][NC];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[k][c] = 0.f;
  const long long stride = (long long)gridDim.x * LT;
  if constexpr (NC % 4 == 0 && NC <= 16) {
    if (softmax == 1 && uce != 2 && C == NC) {
      // software-pipelined softmax path: the next voxel's logits and label are loaded before this voxel's math
      // (one voxel per thread in flight otherwise: the pass waited on every load at 3 waves per SIMD)
      long long v = blockIdx.x * (long long)LT + threadIdx.x;
      f32x4 cur[NC / 4], nxt[NC / 4];
      float tcur = 0.f, tnxt = 0.f;
      // (clamped index, no branch around the loads: a divergent branch makes the wait for the prefetch land at
      // the branch merge, right after it is issued)
      auto load = [&](long long vv, f32x4 (&q)[NC / 4], float& t) {
        vv = vv < nvox ? vv : nvox - 1;
#pragma unroll
        for (int k = 0; k < NC / 4; ++k) q[k] = *reinterpret_cast<const f32x4*>(lg + vv * NC + 4 * k);
        t = lab[vv];
      };
      load(v, cur, tcur);
      for (; v < nvox; v += stride) {
        load(v + stride, nxt, tnxt);
        float x[NC], e[NC];
#pragma unroll
        for (int k = 0; k < NC / 4; ++k)
#pragma unroll
          for (int j = 0; j < 4; ++j) x[4 * k + j] = cur[k][j];
        float m = x[0];
#pragma unroll
        for (int c = 1; c < NC; ++c) m = fmaxf(m, x[c]);
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          x[c] -= m;
          e[c] = __builtin_amdgcn_exp2f(x[c] * LOG2E);
          s += e[c];
        }
        const float inv = __builtin_amdgcn_rcpf(s), ls = __builtin_amdgcn_logf(s) * LN2;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const bool hit = tcur == (float)c;
          const float tc = hit ? 1.f : 0.f, p = e[c] * inv;
          acc[0][c] = fmaf(p, tc, acc[0][c]);
          acc[1][c] = fmaf(p, p, acc[1][c]);
          acc[2][c] += tc;
          if (uce == 1) {
            const float lq = hit ? x[c] - ls : __builtin_amdgcn_logf(s - e[c]) * LN2 - ls;
            acc[3][c] -= fmaxf(lq, -100.f);
          }
        }
#pragma unroll
        for (int k = 0; k < NC / 4; ++k) cur[k] = nxt[k];
        tcur = tnxt;
      }
      goto reduce;
    }
  }
  for (long long v = blockIdx.x * (long long)LT + threadIdx.x; v < nvox; v += stride) {
    const float t = lab[v];
    if (softmax == 1) {
      float x[NC], e[NC], s, inv;
      softmax_fast<NC>(lg + v * C, C, x, e, s, inv);
      const float ls = __builtin_amdgcn_logf(s) * LN2;
#pragma unroll
      for (int c = 0; c < NC; ++c)
        if (c < C) {
          const bool hit = t == (float)c;
          const float tc = hit ? 1.f : 0.f, p = e[c] * inv;
          acc[0][c] = fmaf(p, tc, acc[0][c]);
          acc[1][c] = fmaf(p, p, acc[1][c]);
          acc[2][c] += tc;
          if (uce == 1) {
            const float lq = hit ? x[c] - ls : __builtin_amdgcn_logf(s - e[c]) * LN2 - ls;
            acc[3][c] -= fmaxf(lq, -100.f);
          } else if (uce == 2 && hit) {
            acc[3][c] -= x[c] - ls;  // cross entropy: -log_softmax(x)[t] (nn.CrossEntropyLoss, no clamp)
          }
        }
    } else {
      float p[NC];
      probs<NC>(lg + v * C, C, softmax, p);
#pragma unroll
      for (int c = 0; c < NC; ++c)
        if (c < C) {
          const float tc = (t == (float)c) ? 1.f : 0.f;
          acc[0][c] = fmaf(p[c], tc, acc[0][c]);
          acc[1][c] = fmaf(p[c], p[c], acc[1][c]);
          acc[2][c] += tc;
          if (uce == 1) acc[3][c] += bce_elem(p[c], tc);
        }
    }
  }
reduce:
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int c = 0; c < NC; ++c)
      if (c < C) {
        float s = wave_sum(acc[k][c]);
        if (lane == 0) red[wave][k * NC + c] = s;
      }
  __syncthreads();
  for (int i = threadIdx.x; i < 4 * C; i += LT) {
    const int k = i / C, c = i % C;
    float s = 0.f;
    for (int w = 0; w < LT / 64; ++w) s += red[w][k * NC + c];
    ws[(long long)blockIdx.x * 4 * C + k * C + c] = s;
  }
}

// The 16-class softmax + per-class BCE forward (the bench's loss) with each voxel's classes split over a lane pair
// (lanes i, i + 32 hold classes 0-7 / 8-15; the max and the softmax sum exchanged once each, as the backward's
// dice_bce_softmax_grad8): 4 x 8 accumulators per lane instead of 4 x 16, so the grid can keep three times the waves in
// flight (the one-lane form held 161 VGPRs and ran at 3.2 TB/s, latency-bound). Per-block partials in
// loss_partial_kernel's layout ([block][k * 16 + c]), summed by loss_combine_kernel.
constexpr int LP_NB = 1280;  // blocks: five 4-wave blocks per CU resident at once (90 VGPRs)
__global__ __launch_bounds__(LT) void loss_partial16_pair_kernel(const float* __restrict__ lg,
                                                                const float* __restrict__ lab, long long nvox,
                                                                float* __restrict__ ws) {
  __shared__ float red[LT / 64][64];
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5, wave = threadIdx.x >> 6;
  float acc[4][8];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[k][c] = 0.f;
  const long long stride = (long long)gridDim.x * (LT / 2);
  long long v = (long long)blockIdx.x * (LT / 2) + wave * 32 + r;  // lanes r and r + 32: the same voxel
  auto load = [&](long long vv, f32x4 (&q)[2], float& t) {  // clamped index, no branch around the loads
    vv = vv < nvox ? vv : nvox - 1;
#pragma unroll
    for (int k = 0; k < 2; ++k) q[k] = *reinterpret_cast<const f32x4*>(lg + vv * 16 + 8 * h + 4 * k);
    t = lab[vv];
  };
  f32x4 cur[2], nxt[2];
  float tcur = 0.f, tnxt = 0.f;
  load(v, cur, tcur);
  for (; v < nvox; v += stride) {  // both lanes of a pair take the same trips (the exchanges need both)
    load(v + stride, nxt, tnxt);
    float x[8], e[8];
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) x[4 * k + j] = cur[k][j];
    float m = x[0];
#pragma unroll
    for (int c = 1; c < 8; ++c) m = fmaxf(m, x[c]);
    m = fmaxf(m, __shfl_xor(m, 32));
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      x[c] -= m;
      e[c] = __builtin_amdgcn_exp2f(x[c] * LOG2E);
      s += e[c];
    }
    s += __shfl_xor(s, 32);
    const float inv = __builtin_amdgcn_rcpf(s), ls = __builtin_amdgcn_logf(s) * LN2;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const bool hit = tcur == (float)(8 * h + c);
      const float tc = hit ? 1.f : 0.f, p = e[c] * inv;
      acc[0][c] = fmaf(p, tc, acc[0][c]);
      acc[1][c] = fmaf(p, p, acc[1][c]);
      acc[2][c] += tc;
      const float lq = hit ? x[c] - ls : __builtin_amdgcn_logf(s - e[c]) * LN2 - ls;
      acc[3][c] -= fmaxf(lq, -100.f);
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) cur[k] = nxt[k];
    tcur = tnxt;
  }
  // per class over the wave's 32 voxels (lanes with equal h), then the block's waves in order
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      float t = acc[k][c];
#pragma unroll
      for (int o = 1; o < 32; o <<= 1) t += __shfl_xor(t, o, 32);
      if (r == 0) red[wave][k * 16 + 8 * h + c] = t;
    }
  __syncthreads();
  if (threadIdx.x < 64) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < LT / 64; ++w) t += red[w][threadIdx.x];
    ws[(long long)blockIdx.x * 64 + threadIdx.x] = t;
  }
}

// one block per (k, c): s = sum over the per-block partials, fixed order (fp64)
__global__ __launch_bounds__(LT) void loss_combine_kernel(const float* __restrict__ ws, int nblk, int C,
                                                         double* __restrict__ sums) {
  __shared__ double red[LT / 64];
  const int i = blockIdx.x;  // = k*C + c
  double a = 0;
  for (int b = threadIdx.x; b < nblk; b += LT) a += ws[(long long)b * 4 * C + i];
  a = wave_sum(a);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int k = i / C, c = i % C;
    sums[c * 4 + k] = red[0] + red[1] + red[2] + red[3];
  }
}

__global__ void loss_final_kernel(int C, const float* __restrict__ wt, int uce, double count,
                                  const double* __restrict__ sums, float* __restrict__ loss) {
  if (threadIdx.x == 0) {
    double dice = 0, ce = 0;
    for (int c = 0; c < C; ++c) {
      const double I = sums[c * 4 + 0], Z = sums[c * 4 + 1], Y = sums[c * 4 + 2], B = sums[c * 4 + 3];
      const float d = 1.f - (float)((2.0 * I + 1e-5) / (Z + Y + 1e-5));
      dice += (double)d * wt[c];
      ce += uce == 2 ? B / count : (double)(float)(B / count) * wt[c];
    }
    double l = dice / C;
    if (uce) l += ce;
    loss[0] = (float)l;
  }
}

template <int NC, typename TO>
__global__ __launch_bounds__(LT) void loss_bwd_kernel(const float* __restrict__ lg, const float* __restrict__ lab,
                                                     long long nvox, int C, int softmax, int uce,
                                                     const float* __restrict__ wt, const double* __restrict__ sums,
                                                     const float* __restrict__ gout, double count, TO* __restrict__ dl) {
  __shared__ float kd_a[NC], kd_b[NC], kb[NC];
  if (threadIdx.x < NC) {
    const int c = threadIdx.x;
    float a, b, e;
    dice_bce_coefs(c, C, sums, wt, gout, uce, count, a, b, e);
    kd_a[c] = a;
    kd_b[c] = b;
    kb[c] = e;
  }
  __syncthreads();
  if constexpr (NC == 16 && sizeof(TO) == 4) {
    if (softmax == 1 && uce == 1 && C == NC) {
      // software-pipelined softmax + BCE path (the bench's loss): the next voxel's logits and label are loaded
      // before this voxel's math; same arithmetic as the generic loop below
      const long long stride = (long long)gridDim.x * LT;
      long long v = blockIdx.x * (long long)LT + threadIdx.x;
      f32x4 cur[4], nxt[4];
      float tcur = 0.f, tnxt = 0.f;
      auto load = [&](long long vv, f32x4 (&q)[4], float& t) {  // clamped index, no branch (see the forward)
        vv = vv < nvox ? vv : nvox - 1;
#pragma unroll
        for (int k = 0; k < 4; ++k) q[k] = *reinterpret_cast<const f32x4*>(lg + vv * 16 + 4 * k);
        t = lab[vv];
      };
      load(v, cur, tcur);
      for (; v < nvox; v += stride) {
        load(v + stride, nxt, tnxt);
        float r[16];
        dice_bce_softmax_grad16(cur, tcur, kd_a, kd_b, kb, r);
#pragma unroll
        for (int c = 0; c < 16; c += 4)
          *reinterpret_cast<f32x4*>(dl + v * 16 + c) = f32x4{r[c], r[c + 1], r[c + 2], r[c + 3]};
#pragma unroll
        for (int k = 0; k < 4; ++k) cur[k] = nxt[k];
        tcur = tnxt;
      }
      return;
    }
  }
  for (long long v = blockIdx.x * (long long)LT + threadIdx.x; v < nvox; v += (long long)gridDim.x * LT) {
    float p[NC], g[NC];
    if (softmax == 1) {
      float x[NC], s, inv;
      softmax_fast<NC>(lg + v * C, C, x, p, s, inv);
#pragma unroll
      for (int c = 0; c < NC; ++c) p[c] *= inv;
    } else {
      probs<NC>(lg + v * C, C, softmax, p);
    }
    const float t = lab[v];
    float dot = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      g[c] = 0.f;
      if (c < C) {
        const float tc = (t == (float)c) ? 1.f : 0.f;
        float gc = fmaf(tc, kd_a[c], p[c] * kd_b[c]);
        if (uce == 1) gc += kb[c] * (p[c] - tc) * __builtin_amdgcn_rcpf(fmaxf((1.f - p[c]) * p[c], 1e-12f));
        g[c] = gc;
        dot = fmaf(gc, p[c], dot);
      }
    }
    float r[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c)
      r[c] = softmax == 1 ? p[c] * (g[c] - dot) : softmax == 0 ? g[c] * (1.f - p[c]) * p[c] : g[c];
    if (uce == 2) {  // cross entropy, in logit space: (softmax - onehot) / count
#pragma unroll
      for (int c = 0; c < NC; ++c)
        if (c < C) r[c] += kb[c] * (p[c] - ((t == (float)c) ? 1.f : 0.f));
    }
    if constexpr (NC == 16 && sizeof(TO) == 4) {
#pragma unroll
      for (int c = 0; c < 16; c += 4)
        *reinterpret_cast<f32x4*>(dl + v * 16 + c) = f32x4{r[c], r[c + 1], r[c + 2], r[c + 3]};
    } else {
#pragma unroll
      for (int c = 0; c < NC; ++c)
        if (c < C) dl[v * C + c] = from_f<TO>(r[c]);
    }
  }
}

// ---------------------------------------------------------------------------- partial-label target
// cmask = labels with every organ the sample's dataset does not annotate set to background
// (train_amos_atlas_final.py:252-255: for l in 1..13, if not mask[l]: cmask[cmask == l] = 0).
__global__ __launch_bounds__(LT) void partial_target_kernel(const float* __restrict__ lab, long long V, int S,
                                                           const long long* __restrict__ mask, int mstride, int M,
                                                           int lmin, int lmax, float* __restrict__ out) {
  const long long total = (long long)S * V;
  for (long long i = blockIdx.x * (long long)LT + threadIdx.x; i < total; i += (long long)gridDim.x * LT) {
    const float t = lab[i];
    const long long* m = mask + (i / V) * mstride;
    bool drop = false;
    for (int l = lmin; l <= lmax && l < M; ++l) drop |= (t == (float)l) && m[l] == 0;
    out[i] = drop ? 0.f : t;
  }
}

// ------------------------------------------------------------------------------------- Dice metric
template <int NC>
__global__ __launch_bounds__(LT) void dice_count_kernel(const float* __restrict__ lg, const float* __restrict__ lab,
                                                       long long V, int C, int ncls,
                                                       unsigned long long* __restrict__ cnt,
                                                       long long* __restrict__ amap) {
  __shared__ unsigned int h[3 * CMAX];
  for (int i = threadIdx.x; i < 3 * CMAX; i += LT) h[i] = 0;
  __syncthreads();
  const int s = blockIdx.y;
  const float* base = lg + (long long)s * V * C;
  for (long long v = blockIdx.x * (long long)LT + threadIdx.x; v < V; v += (long long)gridDim.x * LT) {
    float p[NC];
    probs<NC>(base + v * C, C, 1, p);
    int am = 0;
    float best = p[0];
#pragma unroll
    for (int c = 1; c < NC; ++c)
      if (c < C && p[c] > best) {
        best = p[c];
        am = c;
      }
    if (amap) amap[(long long)s * V + v] = am;
    const float t = lab[(long long)s * V + v];
    const int ti = (t >= 1.f && t <= (float)ncls && t == floorf(t)) ? (int)t : 0;
    if (am >= 1 && am <= ncls) atomicAdd(&h[(am - 1) * 3 + 1], 1u);
    if (ti >= 1) atomicAdd(&h[(ti - 1) * 3 + 2], 1u);
    if (am >= 1 && am <= ncls && am == ti) atomicAdd(&h[(am - 1) * 3 + 0], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 3 * ncls; i += LT)
    if (h[i]) atomicAdd(&cnt[(long long)s * 3 * ncls + i], (unsigned long long)h[i]);
}

__global__ void dice_final_kernel(const unsigned long long* __restrict__ cnt, int S, int ncls, float* __restrict__ m) {
  const int l = threadIdx.x;
  if (l >= ncls) return;
  float sd = 0.f, ss = 0.f, sp = 0.f;
  for (int s = 0; s < S; ++s) {
    const unsigned long long* c = cnt + ((long long)s * ncls + l) * 3;
    const float num = (float)c[0];
    sd += (float)(2 * c[0]) / (float)(c[1] + c[2] + 1);
    ss += num / (float)(c[2] + 1);
    sp += num / (float)(c[1] + 1);
  }
  m[l * 3 + 0] = sd / (float)S;
  m[l * 3 + 1] = ss / (float)S;
  m[l * 3 + 2] = sp / (float)S;
}

// get_dice2 (evaluate_amos.py:156-182, atlas=None): the refiner's output holds one 2-class prediction per organ
// (sample l = organ l); per organ the binary prediction argmax(softmax(ref[l])) == 1 is scored against the shared
// label volume == l+1. Element strides for the refiner layout (organ rsn, class rsc, voxel rsv).
__global__ __launch_bounds__(LT) void dice_binary_count_kernel(const float* __restrict__ ref, long long rsn,
                                                              long long rsc, long long rsv,
                                                              const float* __restrict__ lab, long long V,
                                                              unsigned long long* __restrict__ cnt,
                                                              long long* __restrict__ amap) {
  __shared__ unsigned int h[3];
  if (threadIdx.x < 3) h[threadIdx.x] = 0;
  __syncthreads();
  const int l = blockIdx.y;
  unsigned int a = 0, b = 0, c = 0;
  for (long long v = blockIdx.x * (long long)LT + threadIdx.x; v < V; v += (long long)gridDim.x * LT) {
    const float r0 = ref[l * rsn + v * rsv], r1 = ref[l * rsn + rsc + v * rsv];
    const float m = fmaxf(r0, r1);
    const float e0 = expf(r0 - m), e1 = expf(r1 - m), inv = 1.f / (e0 + e1);
    const int am = e1 * inv > e0 * inv ? 1 : 0;  // torch.argmax: the first maximum on ties
    if (amap) amap[(long long)l * V + v] = am;
    const int t = lab[v] == (float)(l + 1);
    a += am & t;
    b += am;
    c += t;
  }
  atomicAdd(&h[0], a);  // integer: order-independent
  atomicAdd(&h[1], b);
  atomicAdd(&h[2], c);
  __syncthreads();
  if (threadIdx.x < 3 && h[threadIdx.x]) atomicAdd(&cnt[l * 3 + threadIdx.x], (unsigned long long)h[threadIdx.x]);
}

// Forward grid: at most 512 blocks = two per CU, all resident at once (the softmax path holds 161 VGPRs: 3 waves per
// SIMD, so 1024 blocks ran as a full and a one-third round). 2 x 96^3 x 16 (tools/kbench.py loss96, gpurun_out/r04_u):
// 1024 / 768 / 512 / 384 / 256 blocks -> 63.6 / 48.6 / 45.8 / 51.0 / 51.7 us
#ifndef U3D_LOSS_NB
#define U3D_LOSS_NB 512
#endif
static int loss_blocks(long long nvox) {
  return (int)std::min<long long>(U3D_LOSS_NB, std::max<long long>(1, (nvox + LT - 1) / LT));
}

// dispatch on the class count: exact instantiations for the model heads, a guarded 32-wide fallback
#define U3D_NC_DISPATCH(C, F)        \
  switch (C) {                       \
    case 2: F(2); break;             \
    case 8: F(8); break;             \
    case 14: F(14); break;           \
    case 16: F(16); break;           \
    default: F(32); break;           \
  }

}  // namespace u3d

using namespace u3d;

static int loss_pair_blocks(long long nvox) {
  return (int)std::min<long long>(LP_NB, std::max<long long>(1, (nvox + LT / 2 - 1) / (LT / 2)));
}

extern "C" long long u3d_loss_workspace_bytes(int S, long long V, int C) {
  const long long nvox = (long long)S * V;
  return (long long)std::max(loss_blocks(nvox), C == 16 ? loss_pair_blocks(nvox) : 0) * 4 * C * 4;
}

extern "C" int u3d_partial_loss_fwd(const float* logits, const float* labels, int S, long long V, int C, int softmax,
                                    const float* weights, int uce, double* sums, float* loss, float* ws,
                                    u3d_stream_t stream) {
  U3D_REQUIRE(logits && labels && weights && sums && loss && ws, "partial_loss_fwd: null pointer");
  U3D_REQUIRE(C >= 1 && C <= CMAX && S >= 1 && V >= 1, "partial_loss_fwd: C=%d unsupported (max %d)", C, CMAX);
  U3D_REQUIRE(uce >= 0 && uce <= 2 && (uce != 2 || softmax == 1), "partial_loss_fwd: uce=%d (2 = cross entropy, "
              "softmax logits only)", uce);
  hipStream_t s = (hipStream_t)stream;
  const long long nvox = (long long)S * V;
  int nb = loss_blocks(nvox);
  if (C == 16 && softmax == 1 && uce == 1 && opt(OPT_LOSS_PAIR) != 0) {
    nb = loss_pair_blocks(nvox);
    hipLaunchKernelGGL(loss_partial16_pair_kernel, dim3(nb), dim3(LT), 0, s, logits, labels, nvox, ws);
  } else {
#define LAUNCH(NCV) \
  hipLaunchKernelGGL(loss_partial_kernel<NCV>, dim3(nb), dim3(LT), 0, s, logits, labels, nvox, C, softmax, uce, ws)
    U3D_NC_DISPATCH(C, LAUNCH)
#undef LAUNCH
  }
  hipLaunchKernelGGL(loss_combine_kernel, dim3(4 * C), dim3(LT), 0, s, ws, nb, C, sums);
  hipLaunchKernelGGL(loss_final_kernel, dim3(1), dim3(64), 0, s, C, weights, uce, (double)nvox, sums, loss);
  return check_launch("partial_loss_fwd");
}

extern "C" int u3d_partial_loss_bwd(int dtype_out, const float* logits, const float* labels, int S, long long V, int C,
                                    int softmax, const float* weights, int uce, const double* sums,
                                    const float* grad_out, void* dlogits, u3d_stream_t stream) {
  U3D_REQUIRE(logits && labels && weights && sums && grad_out && dlogits, "partial_loss_bwd: null pointer");
  U3D_REQUIRE(C >= 1 && C <= CMAX, "partial_loss_bwd: C=%d unsupported", C);
  U3D_REQUIRE(uce >= 0 && uce <= 2 && (uce != 2 || softmax == 1), "partial_loss_bwd: bad uce=%d", uce);
  hipStream_t s = (hipStream_t)stream;
  const long long nvox = (long long)S * V;
  const int nb = (int)std::min<long long>(8192, (nvox + LT - 1) / LT);
  if (dtype_out == U3D_BF16) {
#define LAUNCH(NCV)                                                                                                   \
  hipLaunchKernelGGL((loss_bwd_kernel<NCV, bf16>), dim3(nb), dim3(LT), 0, s, logits, labels, nvox, C, softmax, uce, \
                     weights, sums, grad_out, (double)nvox, (bf16*)dlogits)
    U3D_NC_DISPATCH(C, LAUNCH)
#undef LAUNCH
  } else {
#define LAUNCH(NCV)                                                                                                    \
  hipLaunchKernelGGL((loss_bwd_kernel<NCV, float>), dim3(nb), dim3(LT), 0, s, logits, labels, nvox, C, softmax, uce, \
                     weights, sums, grad_out, (double)nvox, (float*)dlogits)
    U3D_NC_DISPATCH(C, LAUNCH)
#undef LAUNCH
  }
  return check_launch("partial_loss_bwd");
}

extern "C" int u3d_dice_metric(const float* logits, const float* labels, int S, long long V, int C, int num_class,
                               long long* counts, float* metrics, long long* argmax, u3d_stream_t stream) {
  U3D_REQUIRE(logits && labels && counts && metrics, "dice_metric: null pointer");
  U3D_REQUIRE(C >= 1 && C <= CMAX && num_class >= 1 && num_class <= CMAX && S >= 1, "dice_metric: bad sizes");
  hipStream_t s = (hipStream_t)stream;
  U3D_HIP(hipMemsetAsync(counts, 0, (size_t)S * num_class * 3 * 8, s));
  const int nb = (int)std::min<long long>(1024, (V + LT - 1) / LT);
#define LAUNCH(NCV)                                                                                         \
  hipLaunchKernelGGL(dice_count_kernel<NCV>, dim3(nb, S), dim3(LT), 0, s, logits, labels, V, C, num_class, \
                     (unsigned long long*)counts, argmax)
  U3D_NC_DISPATCH(C, LAUNCH)
#undef LAUNCH
  hipLaunchKernelGGL(dice_final_kernel, dim3(1), dim3(64), 0, s, (const unsigned long long*)counts, S, num_class,
                     metrics);
  return check_launch("dice_metric");
}

extern "C" int u3d_partial_target(const float* labels, int S, long long V, const long long* mask, int mask_stride,
                                  int M, int lmin, int lmax, float* out, u3d_stream_t stream) {
  U3D_REQUIRE(labels && mask && out && S >= 1 && V >= 1 && M >= 1 && mask_stride >= 0, "partial_target: bad args");
  const long long total = (long long)S * V;
  const int nb = (int)std::min<long long>(4096, (total + LT - 1) / LT);
  hipLaunchKernelGGL(partial_target_kernel, dim3(nb), dim3(LT), 0, (hipStream_t)stream, labels, V, S, mask,
                     mask_stride, M, lmin, lmax, out);
  return check_launch("partial_target_kernel");
}

extern "C" int u3d_dice_metric_binary(const float* refine, int nt, long long V, long long rsn, long long rsc,
                                      long long rsv, const float* labels, long long* counts, float* metrics,
                                      long long* argmax, u3d_stream_t stream) {
  U3D_REQUIRE(refine && labels && counts && metrics && nt >= 1 && nt <= 64 && V >= 1, "dice_metric_binary: bad args");
  hipStream_t s = (hipStream_t)stream;
  U3D_HIP(hipMemsetAsync(counts, 0, (size_t)nt * 3 * 8, s));
  const int nb = (int)std::min<long long>(1024, (V + LT - 1) / LT);
  hipLaunchKernelGGL(dice_binary_count_kernel, dim3(nb, nt), dim3(LT), 0, s, refine, rsn, rsc, rsv, labels, V,
                     (unsigned long long*)counts, argmax);
  // per organ (a batch of one each): the reference's ratios from the integer counts = dice_final_kernel with one
  // sample and nt "classes"
  hipLaunchKernelGGL(dice_final_kernel, dim3(1), dim3(64), 0, s, (const unsigned long long*)counts, 1, nt, metrics);
  return check_launch("dice_metric_binary");
}
