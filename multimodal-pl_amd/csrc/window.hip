// Sliding-window inference accumulation (reference evaluate_amos.py:198-279 predict_sliding + _get_gaussian
// :184-197), on the device instead of the reference's per-tile device->host copies and float64 host arrays.
//
//   full[n][c][d][h][w] += scale * pred[n][a][b][e][c] * g(a, b, e)      (pred NDHWC fp32 logits of one tile)
//   count[n][d][h][w]   += g(a, b, e)                                     (once per tile position)
//   g(a, b, e) = gd[a] * gh[b] * gw[e]  (separable Gaussian importance map, each profile scaled to max 1),
//                zeros replaced by gmin (the reference replaces zeros of the map by its minimum non-zero value)
// Output flips (test-time augmentation, :244-251) are read as mirrored tile indices. The final division
// full /= count is a second kernel. Accumulation is fp32 (the reference accumulates in float64 on the host).
#include "common.h"

namespace u3d {

// grid (w chunks, tile rows td*th, n): one output voxel per thread along w, no 64-bit div/mod; the prediction row
// (C contiguous fp32 per voxel) is read as 16-B vectors when C % 4 == 0
__global__ __launch_bounds__(256) void window_acc_kernel(const float* __restrict__ pred, int C, int td, int th, int tw,
                                                        const float* __restrict__ gd, const float* __restrict__ gh,
                                                        const float* __restrict__ gw, float gmin, float scale,
                                                        float* __restrict__ full, float* __restrict__ count, int D,
                                                        int H, int W, int d1, int y1, int x1, int flips,
                                                        int add_count) {
  const int n = blockIdx.z, row = blockIdx.y;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= tw) return;
  const int a = row / th, b = row - a * th;
  const long long DHW = (long long)D * H * W;
  float g = gd[a] * gh[b] * gw[e];
  if (g == 0.f) g = gmin;
  const long long vox = ((long long)(d1 + a) * H + (y1 + b)) * W + (x1 + e);
  if (add_count) count[n * DHW + vox] += g;
  // the prediction of the flipped input is flipped back: read the mirrored tile voxel
  const int pa = (flips & 1) ? td - 1 - a : a, pb = (flips & 2) ? th - 1 - b : b, pe = (flips & 4) ? tw - 1 - e : e;
  const float* pv = pred + ((((long long)n * td + pa) * th + pb) * tw + pe) * C;
  const float gs = g * scale;
  float* fo = full + (long long)n * C * DHW + vox;
  if ((C & 3) == 0) {
    for (int c = 0; c < C; c += 4) {
      const f32x4 q = *reinterpret_cast<const f32x4*>(pv + c);
#pragma unroll
      for (int k = 0; k < 4; ++k) fo[(long long)(c + k) * DHW] += q[k] * gs;
    }
  } else {
    for (int c = 0; c < C; ++c) fo[(long long)c * DHW] += pv[c] * gs;
  }
}

__global__ __launch_bounds__(256) void window_norm_kernel(float* __restrict__ full, const float* __restrict__ count,
                                                         int C, long long DHW) {
  const int n = blockIdx.z, c = blockIdx.y;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < DHW; i += (long long)gridDim.x * 256)
    full[((long long)n * C + c) * DHW + i] /= count[n * DHW + i];
}

}  // namespace u3d

using namespace u3d;

extern "C" int u3d_window_accumulate(const float* pred, int n, int C, int td, int th, int tw, const float* gd,
                                     const float* gh, const float* gw, float gmin, float scale, float* full,
                                     float* count, int D, int H, int W, int d1, int y1, int x1, int flips,
                                     int add_count, u3d_stream_t stream) {
  U3D_REQUIRE(pred && gd && gh && gw && full && count && n >= 1 && C >= 1, "window_accumulate: bad args");
  U3D_REQUIRE(d1 >= 0 && y1 >= 0 && x1 >= 0 && d1 + td <= D && y1 + th <= H && x1 + tw <= W,
              "window_accumulate: tile [%d+%d, %d+%d, %d+%d] outside the volume %dx%dx%d", d1, td, y1, th, x1, tw, D,
              H, W);
  U3D_REQUIRE((long long)td * th <= 65535 && n <= 65535, "window_accumulate: tile rows %d x %d beyond the grid", td, th);
  hipLaunchKernelGGL(window_acc_kernel, dim3(cdiv(tw, 256), td * th, n), dim3(256), 0, (hipStream_t)stream, pred, C,
                     td, th, tw, gd, gh, gw, gmin, scale, full, count, D, H, W, d1, y1, x1, flips, add_count);
  return check_launch("window_acc_kernel");
}

extern "C" int u3d_window_normalize(float* full, const float* count, int n, int C, long long dhw, u3d_stream_t stream) {
  U3D_REQUIRE(full && count && n >= 1 && C >= 1 && dhw >= 1, "window_normalize: bad args");
  const int nb = (int)std::min<long long>(4096, (dhw + 255) / 256);
  hipLaunchKernelGGL(window_norm_kernel, dim3(nb, C, n), dim3(256), 0, (hipStream_t)stream, full, count, C, dhw);
  return check_launch("window_norm_kernel");
}
