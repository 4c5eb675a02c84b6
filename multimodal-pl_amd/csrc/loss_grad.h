// The per-voxel gradient of the partial-label soft Dice + per-class BCE on softmax probabilities (reference
// loss_partial.py:59-99, DiceLoss :10-57), shared by loss_bwd_kernel (loss.hip) and the head backward that forms it in
// registers (head_loss_bwd_kernel, head.hip): one definition, so both produce the same bits.
#pragma once
#include "common.h"

namespace u3d {

// per-class coefficients: dL/dp_c = t_c * a + p_c * b (+ the BCE term e * (p_c - t_c) / ((1 - p_c) p_c))
//   d(1 - num/den)/dp = -(2 t den - num * 2 p) / den^2, num = 2 I + 1e-5, den = Z + Y + 1e-5 (per class sums)
__device__ __forceinline__ void dice_bce_coefs(int c, int C, const double* __restrict__ sums,
                                               const float* __restrict__ wt, const float* __restrict__ gout, int uce,
                                               double count, float& a, float& b, float& e) {
  a = b = e = 0.f;
  if (c < C) {
    const double I = sums[c * 4], Z = sums[c * 4 + 1], Y = sums[c * 4 + 2];
    const double num = 2.0 * I + 1e-5, den = Z + Y + 1e-5;
    const double scale = (double)wt[c] / C * gout[0];
    a = (float)(-2.0 / den * scale);
    b = (float)(2.0 * num / (den * den) * scale);
    e = uce == 1 ? (float)((double)wt[c] / count * gout[0]) : uce == 2 ? (float)(1.0 / count * gout[0]) : 0.f;
  }
}

// dL/dlogits of one voxel, 16 classes, softmax + per-class BCE (uce 1): the logits in x4 (4 x 16 B), its label t,
// the coefficient tables (LDS) -> r[16]. Softmax on the hardware exp2 / rcp (~1 ulp), as the forward. The sums over
// the classes run as two halves (classes 0-7, 8-15) added at the end — the order dice_bce_softmax_grad8 reproduces
// with each half in one lane of a lane pair (fp addition commutes, max is exact).
__device__ __forceinline__ void dice_bce_softmax_grad16(const f32x4 (&x4)[4], float t, const float* kd_a,
                                                        const float* kd_b, const float* kb, float (&r)[16]) {
  constexpr float kLog2e = 1.4426950408889634f;
  float x[16], p[16];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) x[4 * k + j] = x4[k][j];
  float m = x[0];
#pragma unroll
  for (int c = 1; c < 16; ++c) m = fmaxf(m, x[c]);
  float sh[2] = {0.f, 0.f};
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    p[c] = __builtin_amdgcn_exp2f((x[c] - m) * kLog2e);
    sh[c >> 3] += p[c];
  }
  const float inv = __builtin_amdgcn_rcpf(sh[0] + sh[1]);
#pragma unroll
  for (int c = 0; c < 16; ++c) p[c] *= inv;
  float g[16], dh[2] = {0.f, 0.f};
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const float tc = (t == (float)c) ? 1.f : 0.f;
    float gc = fmaf(tc, kd_a[c], p[c] * kd_b[c]);
    gc += kb[c] * (p[c] - tc) * __builtin_amdgcn_rcpf(fmaxf((1.f - p[c]) * p[c], 1e-12f));
    g[c] = gc;
    dh[c >> 3] = fmaf(gc, p[c], dh[c >> 3]);
  }
  const float dot = dh[0] + dh[1];
#pragma unroll
  for (int c = 0; c < 16; ++c) r[c] = p[c] * (g[c] - dot);
}

// The same gradient with the voxel's classes split over a lane pair (lanes i, i ^ 32 of a wave): this lane holds
// classes 8h .. 8h+7 in x4 and gets r for them; the max, the softmax sum and the dot product are exchanged once each.
// Bitwise dice_bce_softmax_grad16's values for those classes.
__device__ __forceinline__ void dice_bce_softmax_grad8(const f32x4 (&x4)[2], float t, int h, const float* kd_a,
                                                       const float* kd_b, const float* kb, float (&r)[8]) {
  constexpr float kLog2e = 1.4426950408889634f;
  float x[8], p[8];
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) x[4 * k + j] = x4[k][j];
  float m = x[0];
#pragma unroll
  for (int c = 1; c < 8; ++c) m = fmaxf(m, x[c]);
  m = fmaxf(m, __shfl_xor(m, 32));
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    p[c] = __builtin_amdgcn_exp2f((x[c] - m) * kLog2e);
    s += p[c];
  }
  const float inv = __builtin_amdgcn_rcpf(s + __shfl_xor(s, 32));
#pragma unroll
  for (int c = 0; c < 8; ++c) p[c] *= inv;
  float g[8], d = 0.f;
  const int c0 = 8 * h;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const float tc = (t == (float)(c0 + c)) ? 1.f : 0.f;
    float gc = fmaf(tc, kd_a[c0 + c], p[c] * kd_b[c0 + c]);
    gc += kb[c0 + c] * (p[c] - tc) * __builtin_amdgcn_rcpf(fmaxf((1.f - p[c]) * p[c], 1e-12f));
    g[c] = gc;
    d = fmaf(gc, p[c], d);
  }
  const float dot = d + __shfl_xor(d, 32);
#pragma unroll
  for (int c = 0; c < 8; ++c) r[c] = p[c] * (g[c] - dot);
}

}  // namespace u3d
