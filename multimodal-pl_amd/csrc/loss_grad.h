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
// the coefficient tables (LDS) -> r[16]. Softmax on the hardware exp2 / rcp (~1 ulp), as the forward.
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
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    p[c] = __builtin_amdgcn_exp2f((x[c] - m) * kLog2e);
    s += p[c];
  }
  const float inv = __builtin_amdgcn_rcpf(s);
#pragma unroll
  for (int c = 0; c < 16; ++c) p[c] *= inv;
  float g[16], dot = 0.f;
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const float tc = (t == (float)c) ? 1.f : 0.f;
    float gc = fmaf(tc, kd_a[c], p[c] * kd_b[c]);
    gc += kb[c] * (p[c] - tc) * __builtin_amdgcn_rcpf(fmaxf((1.f - p[c]) * p[c], 1e-12f));
    g[c] = gc;
    dot = fmaf(gc, p[c], dot);
  }
#pragma unroll
  for (int c = 0; c < 16; ++c) r[c] = p[c] * (g[c] - dot);
}

}  // namespace u3d
