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

// ---------------------------------------------------------------------------------------------- backward
// Per voxel: recompute the 8-8-2 MLP (h -> a1 -> r1 -> a2 -> r2 -> out), back-propagate dlogits, write dh and
// accumulate the 162 parameter gradients (same layout as params) per thread; block partials are reduced by
// wave shuffles + LDS in fixed order into part[n][block][162].
__global__ __launch_bounds__(256) void dynhead_bwd_kernel(const float* __restrict__ h, const float* __restrict__ prm,
                                                         const float* __restrict__ dout, long long v,
                                                         float* __restrict__ dh, float* __restrict__ part) {
  __shared__ float p[162];
  __shared__ float red[4][162];
  const int n = blockIdx.y;
  for (int i = threadIdx.x; i < 162; i += 256) p[i] = prm[n * 162 + i];
  __syncthreads();
  float g[162];
#pragma unroll
  for (int k = 0; k < 162; ++k) g[k] = 0.f;
#pragma unroll 1
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < v; i += (long long)gridDim.x * 256) {
    // the 162 parameters are re-read from the LDS each voxel (broadcast reads), not hoisted into registers next to
    // the 162 gradient accumulators
    asm volatile("" ::: "memory");
    const float* hv = h + ((long long)n * v + i) * 8;
    float x0[8], a1[8], r1[8], a2[8], r2[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) x0[k] = hv[k];
#pragma unroll
    for (int o = 0; o < 8; ++o) {
      float s = p[144 + o];
#pragma unroll
      for (int k = 0; k < 8; ++k) s = fmaf(p[o * 8 + k], x0[k], s);
      a1[o] = s;
      r1[o] = fmaxf(s, 0.f);
    }
#pragma unroll
    for (int o = 0; o < 8; ++o) {
      float s = p[152 + o];
#pragma unroll
      for (int k = 0; k < 8; ++k) s = fmaf(p[64 + o * 8 + k], r1[k], s);
      a2[o] = s;
      r2[o] = fmaxf(s, 0.f);
    }
    const float* dv = dout + ((long long)n * v + i) * 2;
    const float d0 = dv[0], d1 = dv[1];
    // layer 3: out = W3 r2 + b3
    float dr2[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      g[128 + k] = fmaf(d0, r2[k], g[128 + k]);
      g[136 + k] = fmaf(d1, r2[k], g[136 + k]);
      dr2[k] = fmaf(p[128 + k], d0, p[136 + k] * d1);
    }
    g[160] += d0;
    g[161] += d1;
    // layer 2: a2 = W2 r1 + b2, r2 = relu(a2)
    float da2[8], dr1[8];
#pragma unroll
    for (int o = 0; o < 8; ++o) da2[o] = a2[o] > 0.f ? dr2[o] : 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) dr1[k] = 0.f;
#pragma unroll
    for (int o = 0; o < 8; ++o) {
      g[152 + o] += da2[o];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        g[64 + o * 8 + k] = fmaf(da2[o], r1[k], g[64 + o * 8 + k]);
        dr1[k] = fmaf(p[64 + o * 8 + k], da2[o], dr1[k]);
      }
    }
    // layer 1: a1 = W1 x0 + b1, r1 = relu(a1)
    float da1[8], dx0[8];
#pragma unroll
    for (int o = 0; o < 8; ++o) da1[o] = a1[o] > 0.f ? dr1[o] : 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) dx0[k] = 0.f;
#pragma unroll
    for (int o = 0; o < 8; ++o) {
      g[144 + o] += da1[o];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        g[o * 8 + k] = fmaf(da1[o], x0[k], g[o * 8 + k]);
        dx0[k] = fmaf(p[o * 8 + k], da1[o], dx0[k]);
      }
    }
    float* dhv = dh + ((long long)n * v + i) * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) dhv[k] = dx0[k];
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 162; ++k) {  // one scheduling region per accumulator: the 162 reductions are not interleaved
    const float t = wave_sum(g[k]);
    if (lane == 0) red[wave][k] = t;
    __builtin_amdgcn_sched_barrier(0);
  }
  __syncthreads();
  for (int k = threadIdx.x; k < 162; k += 256)
    part[((long long)n * gridDim.x + blockIdx.x) * 162 + k] = red[0][k] + red[1][k] + red[2][k] + red[3][k];
}

// dparams[n][k] = sum_b part[n][b][k] (fp64, fixed order)
__global__ void dyn_param_reduce_kernel(const float* __restrict__ part, int nblk, float* __restrict__ dparams) {
  const int n = blockIdx.x;
  for (int k = threadIdx.x; k < 162; k += blockDim.x) {
    double s = 0;
    for (int b = 0; b < nblk; ++b) s += part[((long long)n * nblk + b) * 162 + k];
    dparams[n * 162 + k] = (float)s;
  }
}

// Controller backward (1^3 conv 263 -> m with bias on x = cat(feat, onehot(task))):
//   blocks 0..m-1: dW[o][k] (+)= sum_n dy[n][o] x[n][k], db[o] (+)= sum_n dy[n][o]
//   blocks m..m+n-1: dfeat[n][k] = sum_o W[o][k] dy[n][o] (k < kf), written as the GAP's dA broadcast over the
//   v bottleneck voxels: dA[n][v][k] = dfeat[n][k] / v   (AdaptiveAvgPool3d backward; NDHWC, dtype T)
template <typename T>
__global__ void controller_bwd_kernel(const float* __restrict__ feat, int n, int kf, const long long* __restrict__ task,
                                      int kt, const float* __restrict__ w, const float* __restrict__ dy, int m,
                                      float* __restrict__ dw, float* __restrict__ db, int accp, long long v,
                                      T* __restrict__ dA) {
  const int kx = kf + kt;
  if ((int)blockIdx.x < m) {
    const int o = blockIdx.x;
    for (int k = threadIdx.x; k < kx; k += blockDim.x) {
      float s = 0.f;
      for (int i = 0; i < n; ++i) {
        const long long t = task[i];
        const float xv = k < kf ? feat[i * kf + k] : (t == k - kf ? 1.f : 0.f);
        s = fmaf(dy[i * m + o], xv, s);
      }
      dw[(long long)o * kx + k] = (accp ? dw[(long long)o * kx + k] : 0.f) + s;
    }
    if (threadIdx.x == 0) {
      float s = 0.f;
      for (int i = 0; i < n; ++i) s += dy[i * m + o];
      db[o] = (accp ? db[o] : 0.f) + s;
    }
    return;
  }
  extern __shared__ float df[];
  const int i = blockIdx.x - m;
  for (int k = threadIdx.x; k < kf; k += blockDim.x) {
    float s = 0.f;
    for (int o = 0; o < m; ++o) s = fmaf(w[(long long)o * kx + k], dy[i * m + o], s);
    df[k] = s / (float)v;
  }
  __syncthreads();
  for (long long e = threadIdx.x; e < v * kf; e += blockDim.x) dA[(long long)i * v * kf + e] = from_f<T>(df[e % kf]);
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

extern "C" int u3d_dynhead_bwd_blocks(long long v) { return (int)std::min<long long>(512, (v + 255) / 256); }

extern "C" int u3d_dynhead_bwd(const float* h, const float* params, const float* dlogits, int n, long long v, float* dh,
                               float* part, float* dparams, u3d_stream_t stream) {
  U3D_REQUIRE(h && params && dlogits && dh && part && dparams && n > 0 && v > 0, "dynhead_bwd: bad args");
  const int nb = u3d_dynhead_bwd_blocks(v);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(dynhead_bwd_kernel, dim3(nb, n), dim3(256), 0, s, h, params, dlogits, v, dh, part);
  hipLaunchKernelGGL(dyn_param_reduce_kernel, dim3(n), dim3(192), 0, s, part, nb, dparams);
  return check_launch("dynhead_bwd");
}

extern "C" int u3d_dyn_controller_bwd(int dtype, const float* feat, int n, int kf, const long long* task, int kt,
                                      const float* w, const float* dparams, int m, float* dw, float* db, int accumulate,
                                      long long v, void* dA, u3d_stream_t stream) {
  U3D_REQUIRE(dtype == U3D_F32 || dtype == U3D_BF16, "dyn_controller_bwd: bad dtype");
  U3D_REQUIRE(feat && task && w && dparams && dw && db && dA && n > 0 && v > 0 && kf <= 1024,
              "dyn_controller_bwd: bad args");
  hipStream_t s = (hipStream_t)stream;
  if (dtype == U3D_BF16)
    hipLaunchKernelGGL(controller_bwd_kernel<bf16>, dim3(m + n), dim3(256), kf * 4, s, feat, n, kf, task, kt, w,
                       dparams, m, dw, db, accumulate, v, (bf16*)dA);
  else
    hipLaunchKernelGGL(controller_bwd_kernel<float>, dim3(m + n), dim3(256), kf * 4, s, feat, n, kf, task, kt, w,
                       dparams, m, dw, db, accumulate, v, (float*)dA);
  return check_launch("controller_bwd_kernel");
}
