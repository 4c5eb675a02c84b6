// DynConv "8,8,2" head of UNet3D (reference unet3D.py:1659-1664, 1688-1732, 1753-1804):
//   GAP  = mean_v relu(GroupNorm(16,256)(bottleneck))            -> feat [n][256]
//   params = controller(cat(feat, onehot(task, 7)))  (1^3 conv 263->162 with bias) -> [n][162]
//   per sample n: h1 = relu(W1 h + b1), h2 = relu(W2 h1 + b2), logits = W3 h2 + b3   (8 -> 8 -> 8 -> 2)
// with W1 = params[n, 0:64] as [out 8][in 8], W2 = [64:128], W3 = [128:144] as [2][8], b1 = [144:152],
// b2 = [152:160], b3 = [160:162] (parse_dynamic_params :1695-1718).
#include "common.h"

namespace u3d {

// feat[n][c] = mean_v relu(x * sc + sh); one block per (n, channel chunk of 64)
template <typename T>
__global__ __launch_bounds__(256) void gn_relu_mean_kernel(const T* __restrict__ x, int c, long long v, int groups,
                                                          const float* __restrict__ st, const float* __restrict__ ga,
                                                          const float* __restrict__ be, float* __restrict__ out) {
  __shared__ double red[4][64];
  const int n = blockIdx.y, c0 = blockIdx.x * 64;
  const int lane = threadIdx.x & 63, vl = threadIdx.x >> 6;
  const int ch = c0 + lane;
  double s = 0;
  if (ch < c) {
    const int cpg = c / groups, g = ch / cpg;
    const float mean = st[(n * groups + g) * 2], rstd = st[(n * groups + g) * 2 + 1];
    const float sc = rstd * ga[ch], sh = be[ch] - mean * sc;
    for (long long i = vl; i < v; i += 4) s += fmaxf(0.f, fmaf(to_f(x[((long long)n * v + i) * c + ch]), sc, sh));
  }
  red[vl][lane] = s;
  __syncthreads();
  if (vl == 0 && ch < c) out[n * c + ch] = (float)((red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane]) / v);
}

// y[n][m] = sum_k w[m][k] x[n][k] + b[m], x = cat(feat[n][0:kf], onehot(task[n], kt))
__global__ void controller_kernel(const float* __restrict__ feat, int kf, const long long* __restrict__ task, int kt,
                                  const float* __restrict__ w, const float* __restrict__ b, int m,
                                  float* __restrict__ y) {
  const int n = blockIdx.x;
  for (int o = threadIdx.x; o < m; o += blockDim.x) {
    const float* wr = w + (long long)o * (kf + kt);
    float s = b[o];
    for (int k = 0; k < kf; ++k) s = fmaf(wr[k], feat[n * kf + k], s);
    const long long t = task[n];
    if (t >= 0 && t < kt) s += wr[kf + t];
    y[n * m + o] = s;
  }
}

__global__ __launch_bounds__(256) void dynhead_fwd_kernel(const float* __restrict__ h, const float* __restrict__ prm,
                                                         long long v, float* __restrict__ out) {
  __shared__ float p[162];
  const int n = blockIdx.y;
  for (int i = threadIdx.x; i < 162; i += 256) p[i] = prm[n * 162 + i];
  __syncthreads();
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < v; i += (long long)gridDim.x * 256) {
    const float* hv = h + ((long long)n * v + i) * 8;
    float a[8], b[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = hv[k];
#pragma unroll
    for (int o = 0; o < 8; ++o) {
      float s = p[144 + o];
#pragma unroll
      for (int k = 0; k < 8; ++k) s = fmaf(p[o * 8 + k], a[k], s);
      b[o] = fmaxf(s, 0.f);
    }
#pragma unroll
    for (int o = 0; o < 8; ++o) {
      float s = p[152 + o];
#pragma unroll
      for (int k = 0; k < 8; ++k) s = fmaf(p[64 + o * 8 + k], b[k], s);
      a[o] = fmaxf(s, 0.f);
    }
    float* ov = out + ((long long)n * v + i) * 2;
#pragma unroll
    for (int o = 0; o < 2; ++o) {
      float s = p[160 + o];
#pragma unroll
      for (int k = 0; k < 8; ++k) s = fmaf(p[128 + o * 8 + k], a[k], s);
      ov[o] = s;
    }
  }
}

}  // namespace u3d

using namespace u3d;

extern "C" int u3d_gn_relu_mean(int dtype, const void* x, int n, int c, long long v, int groups, const float* stats,
                                const float* gamma, const float* beta, float* out, u3d_stream_t stream) {
  U3D_REQUIRE(dtype == U3D_F32 || dtype == U3D_BF16, "gn_relu_mean: bad dtype");
  U3D_REQUIRE(x && stats && gamma && beta && out && groups > 0 && c % groups == 0, "gn_relu_mean: bad args");
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((c + 63) / 64, n);
  if (dtype == U3D_BF16)
    hipLaunchKernelGGL(gn_relu_mean_kernel<bf16>, grid, dim3(256), 0, s, (const bf16*)x, c, v, groups, stats, gamma,
                       beta, out);
  else
    hipLaunchKernelGGL(gn_relu_mean_kernel<float>, grid, dim3(256), 0, s, (const float*)x, c, v, groups, stats, gamma,
                       beta, out);
  return check_launch("gn_relu_mean_kernel");
}

extern "C" int u3d_dyn_controller(const float* feat, int n, int kf, const long long* task, int kt, const float* w,
                                  const float* b, int m, float* params, u3d_stream_t stream) {
  U3D_REQUIRE(feat && task && w && b && params && n > 0, "dyn_controller: bad args");
  hipLaunchKernelGGL(controller_kernel, dim3(n), dim3(256), 0, (hipStream_t)stream, feat, kf, task, kt, w, b, m, params);
  return check_launch("controller_kernel");
}

extern "C" int u3d_dynhead_fwd(const float* h, const float* params, int n, long long v, float* out,
                               u3d_stream_t stream) {
  U3D_REQUIRE(h && params && out && n > 0 && v > 0, "dynhead_fwd: bad args");
  const int nb = (int)std::min<long long>(2048, (v + 255) / 256);
  hipLaunchKernelGGL(dynhead_fwd_kernel, dim3(nb, n), dim3(256), 0, (hipStream_t)stream, h, params, v, out);
  return check_launch("dynhead_fwd_kernel");
}
