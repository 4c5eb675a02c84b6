// Fused SGD step (momentum, dampening, weight decay, nesterov, maximize) over a batch of parameter tensors in
// one launch: each element reads p, g, buf once and writes p, buf once (20 B/element fp32) — torch's foreach
// SGD runs it as 3-5 passes of separate kernels.
// Reference: torch.optim.SGD(model.parameters(), lr, momentum=0.9, weight_decay=1e-4) built in
// train_amos_atlas_final.py:132-135 and stepped at :378 (the poly LR of utils.py:53-60 edits param_groups[0]).
// The learning rate is read from device memory so a captured hipGraph picks up LR changes.
#include "common.h"

namespace u3d {

struct SgdBatch {
  int count;
  u3d_sgd_desc d[U3D_SGD_BATCH_MAX];
  long long b0[U3D_SGD_BATCH_MAX];  // first block of each tensor
};

constexpr int SG_T = 256, SG_PER = SG_T * 4 * 4;  // elements per block: 4 float4 per thread

__global__ __launch_bounds__(SG_T) void sgd_kernel(SgdBatch bt, const float* __restrict__ lr_dev, float momentum,
                                                   float dampening, float wd, int nesterov, int maximize, int init) {
  int i = 0;
  while (i + 1 < bt.count && bt.b0[i + 1] <= (long long)blockIdx.x) ++i;
  const u3d_sgd_desc& D = bt.d[i];
  const float lr = *lr_dev;
  const long long e0 = ((long long)blockIdx.x - bt.b0[i]) * SG_PER;
  auto upd = [&](float p, float g, float& b) {
    if (maximize) g = -g;
    float d = wd != 0.f ? fmaf(wd, p, g) : g;  // d_p = g + wd * p
    if (momentum != 0.f) {
      b = init ? d : fmaf(momentum, b, (1.f - dampening) * d);
      d = nesterov ? fmaf(momentum, b, d) : b;
    }
    return fmaf(-lr, d, p);
  };
  for (int k = 0; k < 4; ++k) {
    const long long e = e0 + ((long long)k * SG_T + threadIdx.x) * 4;
    if (e >= D.n) break;
    if (e + 4 <= D.n && ((uintptr_t)(D.p + e) & 15) == 0 && ((uintptr_t)(D.g + e) & 15) == 0 &&
        (!D.buf || ((uintptr_t)(D.buf + e) & 15) == 0)) {
      f32x4 p = *reinterpret_cast<const f32x4*>(D.p + e);
      const f32x4 g = *reinterpret_cast<const f32x4*>(D.g + e);
      f32x4 b = {0.f, 0.f, 0.f, 0.f};
      if (D.buf && !init) b = *reinterpret_cast<const f32x4*>(D.buf + e);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float bq = b[q];
        p[q] = upd(p[q], g[q], bq);
        b[q] = bq;
      }
      *reinterpret_cast<f32x4*>(D.p + e) = p;
      if (D.buf) *reinterpret_cast<f32x4*>(D.buf + e) = b;
    } else {
      for (long long q = e; q < e + 4 && q < D.n; ++q) {
        float b = (D.buf && !init) ? D.buf[q] : 0.f;
        D.p[q] = upd(D.p[q], D.g[q], b);
        if (D.buf) D.buf[q] = b;
      }
    }
  }
}

}  // namespace u3d

using namespace u3d;

extern "C" int u3d_sgd_step(const u3d_sgd_desc* descs, int count, const float* lr, float momentum, float dampening,
                            float weight_decay, int nesterov, int maximize, int init, u3d_stream_t stream) {
  U3D_REQUIRE(descs && lr && count >= 0 && count <= U3D_SGD_BATCH_MAX, "sgd_step: count must be <= %d",
              U3D_SGD_BATCH_MAX);
  if (count == 0) return U3D_OK;
  SgdBatch bt{};
  long long blocks = 0;
  for (int i = 0; i < count; ++i) {
    U3D_REQUIRE(descs[i].p && descs[i].g && descs[i].n >= 0, "sgd_step: bad descriptor %d", i);
    U3D_REQUIRE(momentum == 0.f || descs[i].buf, "sgd_step: descriptor %d needs a momentum buffer", i);
    bt.d[bt.count] = descs[i];
    bt.b0[bt.count++] = blocks;
    blocks += (descs[i].n + SG_PER - 1) / SG_PER;
  }
  if (blocks == 0) return U3D_OK;
  U3D_REQUIRE(blocks < (1LL << 31), "sgd_step: too many elements");
  hipLaunchKernelGGL(sgd_kernel, dim3((unsigned)blocks), dim3(SG_T), 0, (hipStream_t)stream, bt, lr, momentum, dampening,
                     weight_decay, nesterov, maximize, init);
  return check_launch("sgd_kernel");
}
