// Training data path on the device: AMOSDataSet_newatlas.__getitem__ (MOTSDataset.py:299-
// 384: truncate :171-186, random crop :364-371, transpose :376-378) and the batchgenerators intensity transforms of
// my_collate (get_train_transform, MOTSDataset.py:33-52): Gaussian noise, Gaussian blur, multiplicative and additive
// brightness, contrast. The random decisions / parameters are drawn on the host (numpy, as the reference does);
// the kernels apply them. Volumes are fp32.
#include "common.h"

namespace u3d {

constexpr int DT = 256;
constexpr int DS_BLOCKS = 512;

// sum, sum of squares (fp64 block partials), min, max of x[0..V) -> part[block][4]
__global__ __launch_bounds__(DT) void vol_stats_kernel(const float* __restrict__ x, long long V,
                                                      double* __restrict__ part) {
  double s = 0, q = 0;
  float mn = INFINITY, mx = -INFINITY;
  for (long long i = blockIdx.x * (long long)DT + threadIdx.x; i < V; i += (long long)gridDim.x * DT) {
    const float v = x[i];
    s += v;
    q += (double)v * v;
    mn = fminf(mn, v);
    mx = fmaxf(mx, v);
  }
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o);
    q += __shfl_xor(q, o);
    mn = fminf(mn, __shfl_xor(mn, o));
    mx = fmaxf(mx, __shfl_xor(mx, o));
  }
  __shared__ double r[4][4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    r[wave][0] = s;
    r[wave][1] = q;
    r[wave][2] = mn;
    r[wave][3] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0, b = 0, c = INFINITY, d = -INFINITY;
    for (int w = 0; w < DT / 64; ++w) {
      a += r[w][0];
      b += r[w][1];
      c = fmin(c, r[w][2]);
      d = fmax(d, r[w][3]);
    }
    double* o = part + blockIdx.x * 4;
    o[0] = a;
    o[1] = b;
    o[2] = c;
    o[3] = d;
  }
}

// out[0..3] = mean, population std, min, max (fixed-order combine) of x extended by (count - V) zeros (pad_image)
__global__ void vol_stats_final_kernel(const double* __restrict__ part, int nb, long long count,
                                       float* __restrict__ out, int padded) {
  if (threadIdx.x != 0) return;
  double a = 0, b = 0, c = INFINITY, d = -INFINITY;
  for (int k = 0; k < nb; ++k) {
    a += part[k * 4];
    b += part[k * 4 + 1];
    c = fmin(c, part[k * 4 + 2]);
    d = fmax(d, part[k * 4 + 3]);
  }
  if (padded) {
    c = fmin(c, 0.0);
    d = fmax(d, 0.0);
  }
  const double mean = a / count;
  double var = b / count - mean * mean;
  if (var < 0) var = 0;
  out[0] = (float)mean;
  out[1] = (float)sqrt(var);
  out[2] = (float)c;
  out[3] = (float)d;
}

// out[c][dd][hh][ww] = f(src[c][b0 + hh][c0 + ww][a0 + dd]) — the crop of the padded (H, W, D) array followed by
// the reference's transpose to (D, H, W); outside the source = the zero padding of pad_image (:269-282).
// mode 0: copy; 1: CT truncate (clip to [-325, 325], / 325); 2: MRI (x - mean) / std with stats[0..1].
__global__ __launch_bounds__(DT) void crop_kernel(const float* __restrict__ src, int C, int sh, int sw, int sd,
                                                 int b0, int c0, int a0, int ch, int cw, int cd, int mode,
                                                 const float* __restrict__ stats, float* __restrict__ out) {
  const long long total = (long long)C * cd * ch * cw;
  for (long long i = blockIdx.x * (long long)DT + threadIdx.x; i < total; i += (long long)gridDim.x * DT) {
    long long r = i;
    const int ww = (int)(r % cw); r /= cw;
    const int hh = (int)(r % ch); r /= ch;
    const int dd = (int)(r % cd);
    const int cc = (int)(r / cd);
    const int y = b0 + hh, x = c0 + ww, z = a0 + dd;
    float v = 0.f;
    if (y < sh && x < sw && z < sd) v = src[(((long long)cc * sh + y) * sw + x) * sd + z];
    if (mode == 1) v = fminf(fmaxf(v, -325.f), 325.f) / 325.f;
    else if (mode == 2) v = (v - stats[0]) / stats[1];
    out[i] = v;
  }
}

// counter-based normal samples (splitmix64 hash + Box-Muller): x += N(0, sigma) per element
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(DT) void noise_kernel(float* __restrict__ x, long long V, float sigma,
                                                  unsigned long long seed) {
  for (long long i = blockIdx.x * (long long)DT + threadIdx.x; i < V; i += (long long)gridDim.x * DT) {
    const unsigned long long h = mix64(seed ^ mix64((unsigned long long)i));
    const float u1 = ((h >> 40) + 1) * (1.0f / 16777217.0f), u2 = (float)((h >> 16) & 0xFFFFFF) * (1.0f / 16777216.0f);
    x[i] += sigma * sqrtf(-2.f * logf(u1)) * cosf(6.283185307f * u2);
  }
}

// one separable pass of scipy.ndimage.gaussian_filter (mode 'reflect' = half-sample symmetric, truncate 4.0)
// along the middle axis of [outer][L][inner]; w[0..2r] the normalised 1-D kernel
__global__ __launch_bounds__(DT) void blur_axis_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                      long long outer, int L, long long inner,
                                                      const float* __restrict__ w, int r) {
  const long long total = outer * L * inner;
  for (long long i = blockIdx.x * (long long)DT + threadIdx.x; i < total; i += (long long)gridDim.x * DT) {
    const long long in_ = i % inner;
    const long long t = i / inner;
    const int l = (int)(t % L);
    const long long o = t / L;
    const float* row = x + o * L * inner + in_;
    double acc = 0;  // scipy accumulates in double
    for (int k = -r; k <= r; ++k) {
      int j = l + k;
      // reflect: ... b a | a b c ... (period 2L)
      if (L == 1) j = 0;
      else {
        const int p = 2 * L;
        j %= p;
        if (j < 0) j += p;
        if (j >= L) j = p - 1 - j;
      }
      acc += (double)w[k + r] * row[(long long)j * inner];
    }
    y[i] = (float)acc;
  }
}

// x = x * mul + add; contrast: (x - mean) * factor + mean, clipped to [min, max] when preserve (stats = mean, std,
// min, max of the channel before the transform)
__global__ __launch_bounds__(DT) void affine_kernel(float* __restrict__ x, long long V, float mul, float add) {
  for (long long i = blockIdx.x * (long long)DT + threadIdx.x; i < V; i += (long long)gridDim.x * DT)
    x[i] = x[i] * mul + add;
}

__global__ __launch_bounds__(DT) void contrast_kernel(float* __restrict__ x, long long V, float factor,
                                                     const float* __restrict__ stats, int preserve) {
  const float mn = stats[0], lo = stats[2], hi = stats[3];
  for (long long i = blockIdx.x * (long long)DT + threadIdx.x; i < V; i += (long long)gridDim.x * DT) {
    float v = (x[i] - mn) * factor + mn;
    if (preserve) v = fminf(fmaxf(v, lo), hi);
    x[i] = v;
  }
}

static int blocks(long long n) { return (int)std::min<long long>(4096, std::max<long long>(1, (n + DT - 1) / DT)); }

}  // namespace u3d

using namespace u3d;

extern "C" long long u3d_volume_stats_ws_bytes(void) { return (long long)DS_BLOCKS * 4 * 8; }

extern "C" int u3d_volume_stats(const float* x, long long V, long long count, float* out4, void* ws,
                                u3d_stream_t stream) {
  U3D_REQUIRE(x && out4 && ws && V > 0 && count >= V, "volume_stats: bad args");
  hipStream_t s = (hipStream_t)stream;
  const int nb = (int)std::min<long long>(DS_BLOCKS, (V + DT - 1) / DT);
  hipLaunchKernelGGL(vol_stats_kernel, dim3(nb), dim3(DT), 0, s, x, V, (double*)ws);
  hipLaunchKernelGGL(vol_stats_final_kernel, dim3(1), dim3(64), 0, s, (const double*)ws, nb, count, out4,
                     count > V ? 1 : 0);
  return check_launch("volume_stats");
}

extern "C" int u3d_crop_transpose(const float* src, int C, int sh, int sw, int sd, int b0, int c0, int a0, int ch,
                                  int cw, int cd, int mode, const float* stats, float* out, u3d_stream_t stream) {
  U3D_REQUIRE(src && out && C >= 1 && ch >= 1 && cw >= 1 && cd >= 1 && b0 >= 0 && c0 >= 0 && a0 >= 0,
              "crop_transpose: bad args");
  U3D_REQUIRE(mode >= 0 && mode <= 2 && (mode != 2 || stats), "crop_transpose: mode %d", mode);
  hipLaunchKernelGGL(crop_kernel, dim3(blocks((long long)C * ch * cw * cd)), dim3(DT), 0, (hipStream_t)stream, src, C,
                     sh, sw, sd, b0, c0, a0, ch, cw, cd, mode, stats, out);
  return check_launch("crop_kernel");
}

extern "C" int u3d_aug_noise(float* x, long long V, float sigma, unsigned long long seed, u3d_stream_t stream) {
  U3D_REQUIRE(x && V > 0, "aug_noise: bad args");
  hipLaunchKernelGGL(noise_kernel, dim3(blocks(V)), dim3(DT), 0, (hipStream_t)stream, x, V, sigma, seed);
  return check_launch("noise_kernel");
}

extern "C" int u3d_aug_blur_axis(const float* x, float* y, long long outer, int L, long long inner, const float* w,
                                 int radius, u3d_stream_t stream) {
  U3D_REQUIRE(x && y && w && outer >= 1 && L >= 1 && inner >= 1 && radius >= 0, "aug_blur_axis: bad args");
  hipLaunchKernelGGL(blur_axis_kernel, dim3(blocks(outer * L * inner)), dim3(DT), 0, (hipStream_t)stream, x, y, outer,
                     L, inner, w, radius);
  return check_launch("blur_axis_kernel");
}

extern "C" int u3d_aug_affine(float* x, long long V, float mul, float add, u3d_stream_t stream) {
  U3D_REQUIRE(x && V > 0, "aug_affine: bad args");
  hipLaunchKernelGGL(affine_kernel, dim3(blocks(V)), dim3(DT), 0, (hipStream_t)stream, x, V, mul, add);
  return check_launch("affine_kernel");
}

extern "C" int u3d_aug_contrast(float* x, long long V, float factor, const float* stats, int preserve_range,
                                u3d_stream_t stream) {
  U3D_REQUIRE(x && stats && V > 0, "aug_contrast: bad args");
  hipLaunchKernelGGL(contrast_kernel, dim3(blocks(V)), dim3(DT), 0, (hipStream_t)stream, x, V, factor, stats,
                     preserve_range);
  return check_launch("contrast_kernel");
}
