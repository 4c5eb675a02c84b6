// GroupNorm statistics and the backward of relu(group_norm(x)) on NDHWC tensors.
// Reference: nn.GroupNorm(G, C) + nn.ReLU in NoBottleneck (unet3D.py:44-53), fusionConv (:1640-1642),
// precls_conv (:1653-1655), GAP (:1659-1661). The forward apply is fused into the consumer conv's
// prologue (conv.hip), so only statistics are produced here.
//
// Determinism: each block reduces a fixed voxel range into per-channel fp32 partials (of values shifted
// by a per-group constant, so the sum of squares does not cancel), and a finalize pass combines blocks
// and channels in fp64 in a fixed order. No float atomics.
#include "common.h"

namespace u3d {

constexpr int GT = 256;

struct RedGeom {
  int n, c, groups, cpg, nblk, vpb, chn, vlanes;  // chn = 16-B chunks per voxel, vlanes = voxels per pass
  long long v;
};

static RedGeom make_geom(int n, int c, long long v, int groups, int vec) {
  RedGeom g{};
  g.n = n;
  g.c = c;
  g.v = v;
  g.groups = groups;
  g.cpg = groups > 0 ? c / groups : 0;
  g.chn = c / vec;
  g.vlanes = std::max(1, GT / g.chn);
  long long want = std::max<long long>(g.vlanes, (v * n + 2047) / 2048);
  g.vpb = (int)((want + g.vlanes - 1) / g.vlanes * g.vlanes);
  g.nblk = (int)((v + g.vpb - 1) / g.vpb);
  return g;
}

// Block-level per-channel reduction of VEC-wide per-thread partials into out[c] for c < C.
template <int VEC, int NV>
__device__ __forceinline__ void block_channel_reduce(float (&acc)[NV][VEC], float* lds, const RedGeom& g,
                                                     float* out /*[NV][C]*/) {
  const int tid = threadIdx.x;
  const int active = g.vlanes * g.chn;
  for (int k = 0; k < NV; ++k) {
    __syncthreads();
    if (tid < active)
      for (int e = 0; e < VEC; ++e) lds[tid * VEC + e] = acc[k][e];
    __syncthreads();
    for (int c = tid; c < g.c; c += GT) {
      const int j = c / VEC, e = c % VEC;
      float s = 0.f;
      for (int l = 0; l < g.vlanes; ++l) s += lds[(l * g.chn + j) * VEC + e];
      out[k * g.c + c] = s;
    }
  }
}

template <typename T>
__global__ __launch_bounds__(GT) void gn_stats_partial(const T* __restrict__ x, RedGeom g, float* __restrict__ ws) {
  constexpr int VEC = 16 / sizeof(T);
  __shared__ float lds[GT * VEC];
  const int n = blockIdx.y, blk = blockIdx.x, tid = threadIdx.x;
  const T* xn = x + (long long)n * g.v * g.c;
  const int j = tid % g.chn, vl = tid / g.chn;
  float acc[2][VEC];
  for (int e = 0; e < VEC; ++e) acc[0][e] = acc[1][e] = 0.f;
  if (vl < g.vlanes) {
    float shift[VEC];
    for (int e = 0; e < VEC; ++e) shift[e] = to_f(xn[((j * VEC + e) / g.cpg) * g.cpg]);  // x[n, voxel 0, first ch of group]
    const long long v0 = (long long)blk * g.vpb, v1 = std::min<long long>(g.v, v0 + g.vpb);
    for (long long v = v0 + vl; v < v1; v += g.vlanes) {
      float xv[VEC];
      load16<T>(xn + v * g.c + j * VEC, xv);
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        float d = xv[e] - shift[e];
        acc[0][e] += d;
        acc[1][e] = fmaf(d, d, acc[1][e]);
      }
    }
  }
  block_channel_reduce<VEC, 2>(acc, lds, g, ws + ((long long)n * g.nblk + blk) * 2 * g.c);
}

// one block per (n, group)
template <typename T>
__global__ __launch_bounds__(GT) void gn_stats_final(const T* __restrict__ x, RedGeom g, const float* __restrict__ ws,
                                                    float* __restrict__ stats) {
  __shared__ double red[2][GT / 64];
  const int n = blockIdx.x / g.groups, gr = blockIdx.x % g.groups;
  double s1 = 0, s2 = 0;
  const int items = g.nblk * g.cpg;
  for (int it = threadIdx.x; it < items; it += GT) {
    const int b = it / g.cpg, c = gr * g.cpg + it % g.cpg;
    const float* p = ws + ((long long)n * g.nblk + b) * 2 * g.c;
    s1 += p[c];
    s2 += p[g.c + c];
  }
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = s1;
    red[1][threadIdx.x >> 6] = s2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0, b = 0;
    for (int i = 0; i < GT / 64; ++i) {
      a += red[0][i];
      b += red[1][i];
    }
    const double M = (double)g.v * g.cpg;
    const double shift = to_f(x[(long long)n * g.v * g.c + gr * g.cpg]);
    const double dm = a / M;
    double var = b / M - dm * dm;
    if (var < 0) var = 0;
    stats[(n * g.groups + gr) * 2] = (float)(shift + dm);
    stats[(n * g.groups + gr) * 2 + 1] = (float)(1.0 / sqrt(var + 1e-5));
  }
}

// backward partial: per channel s1 = sum dA*m, s2 = sum dA*m*xhat, m = [gamma*xhat + beta > 0]
template <typename T>
__global__ __launch_bounds__(GT) void gn_bwd_partial(const T* __restrict__ da, const T* __restrict__ x, RedGeom g,
                                                    const float* __restrict__ stats, const float* __restrict__ gamma,
                                                    const float* __restrict__ beta, float* __restrict__ ws) {
  constexpr int VEC = 16 / sizeof(T);
  __shared__ float lds[GT * VEC];
  const int n = blockIdx.y, blk = blockIdx.x, tid = threadIdx.x;
  const long long base = (long long)n * g.v * g.c;
  const int j = tid % g.chn, vl = tid / g.chn;
  float acc[2][VEC];
  for (int e = 0; e < VEC; ++e) acc[0][e] = acc[1][e] = 0.f;
  if (vl < g.vlanes) {
    float mu[VEC], rs[VEC], ga[VEC], be[VEC];
    for (int e = 0; e < VEC; ++e) {
      const int c = j * VEC + e, gr = c / g.cpg;
      mu[e] = stats[(n * g.groups + gr) * 2];
      rs[e] = stats[(n * g.groups + gr) * 2 + 1];
      ga[e] = gamma[c];
      be[e] = beta[c];
    }
    const long long v0 = (long long)blk * g.vpb, v1 = std::min<long long>(g.v, v0 + g.vpb);
    for (long long v = v0 + vl; v < v1; v += g.vlanes) {
      float xv[VEC], dv[VEC];
      load16<T>(x + base + v * g.c + j * VEC, xv);
      load16<T>(da + base + v * g.c + j * VEC, dv);
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        const float xh = (xv[e] - mu[e]) * rs[e];
        const float gd = fmaf(ga[e], xh, be[e]) > 0.f ? dv[e] : 0.f;
        acc[0][e] += gd;
        acc[1][e] = fmaf(gd, xh, acc[1][e]);
      }
    }
  }
  block_channel_reduce<VEC, 2>(acc, lds, g, ws + ((long long)n * g.nblk + blk) * 2 * g.c);
}

// one block per channel: csum[n][c] = (s1, s2) in fp64; dgamma/dbeta
__global__ __launch_bounds__(GT) void gn_bwd_final(RedGeom g, const float* __restrict__ ws, double* __restrict__ csum,
                                                  float* __restrict__ dgamma, float* __restrict__ dbeta, int accp) {
  __shared__ double red[2][GT / 64];
  const int c = blockIdx.x;
  double tg = 0, tb = 0;
  for (int n = 0; n < g.n; ++n) {
    double s1 = 0, s2 = 0;
    for (int b = threadIdx.x; b < g.nblk; b += GT) {
      const float* p = ws + ((long long)n * g.nblk + b) * 2 * g.c;
      s1 += p[c];
      s2 += p[g.c + c];
    }
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
      red[0][threadIdx.x >> 6] = s1;
      red[1][threadIdx.x >> 6] = s2;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      double a = 0, b = 0;
      for (int i = 0; i < GT / 64; ++i) {
        a += red[0][i];
        b += red[1][i];
      }
      csum[(n * g.c + c) * 2] = a;
      csum[(n * g.c + c) * 2 + 1] = b;
      tb += a;
      tg += b;
    }
  }
  if (threadIdx.x == 0) {
    if (dgamma) dgamma[c] = (accp ? dgamma[c] : 0.f) + (float)tg;
    if (dbeta) dbeta[c] = (accp ? dbeta[c] : 0.f) + (float)tb;
  }
}

// dx (+)= rstd * (gamma*m*dA - (a_g + xhat*b_g)/M),  a_g = sum_{c in g} gamma_c s1, b_g = sum gamma_c s2
template <typename T>
__global__ __launch_bounds__(GT) void gn_bwd_apply(const T* __restrict__ da, const T* __restrict__ x, RedGeom g,
                                                  const float* __restrict__ stats, const float* __restrict__ gamma,
                                                  const float* __restrict__ beta, const double* __restrict__ csum,
                                                  T* __restrict__ dx, int accum) {
  constexpr int VEC = 16 / sizeof(T);
  __shared__ float coef[2][2 * 256];  // per (n, group): a/M, b/M  (n <= 2 cached; else recomputed)
  const int tid = threadIdx.x;
  const double M = (double)g.v * g.cpg;
  const int ncache = std::min(g.n, 2);
  for (int i = tid; i < ncache * g.groups; i += GT) {
    const int n = i / g.groups, gr = i % g.groups;
    double a = 0, b = 0;
    for (int k = 0; k < g.cpg; ++k) {
      const int c = gr * g.cpg + k;
      a += gamma[c] * csum[(n * g.c + c) * 2];
      b += gamma[c] * csum[(n * g.c + c) * 2 + 1];
    }
    coef[n][2 * gr] = (float)(a / M);
    coef[n][2 * gr + 1] = (float)(b / M);
  }
  __syncthreads();
  const long long nvec = (long long)g.n * g.v * g.chn;
  for (long long i = blockIdx.x * (long long)GT + tid; i < nvec; i += (long long)gridDim.x * GT) {
    const int j = (int)(i % g.chn);
    const long long vv = i / g.chn;
    const int n = (int)(vv / g.v);
    const long long off = vv * g.c + j * VEC;
    float xv[VEC], dv[VEC], o[VEC];
    load16<T>(x + off, xv);
    load16<T>(da + off, dv);
    if (accum) load16<T>(dx + off, o);
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      const int c = j * VEC + e, gr = c / g.cpg;
      const float mu = stats[(n * g.groups + gr) * 2], rs = stats[(n * g.groups + gr) * 2 + 1];
      float ca, cb;
      if (n < 2) {
        ca = coef[n][2 * gr];
        cb = coef[n][2 * gr + 1];
      } else {
        double a = 0, b = 0;
        for (int k = 0; k < g.cpg; ++k) {
          const int cc = gr * g.cpg + k;
          a += gamma[cc] * csum[(n * g.c + cc) * 2];
          b += gamma[cc] * csum[(n * g.c + cc) * 2 + 1];
        }
        ca = (float)(a / M);
        cb = (float)(b / M);
      }
      const float xh = (xv[e] - mu) * rs;
      const float gd = fmaf(gamma[c], xh, beta[c]) > 0.f ? dv[e] : 0.f;
      const float r = rs * (gamma[c] * gd - ca - xh * cb);
      o[e] = accum ? o[e] + r : r;
    }
    store16<T>(dx + off, o);
  }
}


// y = relu(x * scale[n,c] + shift[n,c]) materialised (8 channels per thread): used ahead of the implicit
// GEMM on the small deep-layer activations so its K loop carries no GroupNorm arithmetic.
template <typename T>
__global__ __launch_bounds__(256) void gn_apply_kernel(const T* __restrict__ x, T* __restrict__ y, int n, int c,
                                                       long long v, int groups, const float* __restrict__ st,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta) {
  constexpr int VEC = 8;
  const int c8 = c / VEC;
  const long long per = v * c8, total = per * n;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int nn = (int)(i / per), cc = (int)(i % c8) * VEC;
    f32x2 sc[4], sh[4];
    gn_coef8(st, gamma, beta, groups, c, nn, cc, sc, sh);
    float a[VEC];
    loadv<T, VEC>(x + i * VEC, a);
#pragma unroll
    for (int e = 0; e < VEC; ++e) a[e] = fmaxf(0.f, fmaf(a[e], sc[e >> 1][e & 1], sh[e >> 1][e & 1]));
    storev<T, VEC>(y + i * VEC, a);
  }
}
}  // namespace u3d

using namespace u3d;

extern "C" long long u3d_gn_workspace_bytes(int n, int c, long long v) {
  RedGeom g = make_geom(n, c, v, 1, 4);  // f32 VEC gives the larger block count
  RedGeom g2 = make_geom(n, c, v, 1, 8);
  long long nb = std::max(g.nblk, g2.nblk);
  // partials [n][nblk][2][c] floats + channel sums [n][c][2] doubles
  return (long long)n * nb * 2 * c * 4 + (long long)n * c * 2 * 8 + 256;
}

extern "C" int u3d_gn_stats(int dtype, const void* x, int n, int c, long long v, int groups, float* stats, float* ws,
                            u3d_stream_t stream) {
  U3D_REQUIRE(dtype == U3D_F32 || dtype == U3D_BF16, "gn_stats: bad dtype");
  U3D_REQUIRE(x && stats && ws && n > 0 && v > 0 && groups > 0 && c % groups == 0, "gn_stats: bad args");
  const int vec = dtype == U3D_BF16 ? 8 : 4;
  U3D_REQUIRE(c % vec == 0 && c / vec <= GT, "gn_stats: channels %d unsupported", c);
  RedGeom g = make_geom(n, c, v, groups, vec);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == U3D_BF16) {
    hipLaunchKernelGGL(gn_stats_partial<bf16>, dim3(g.nblk, n), dim3(GT), 0, s, (const bf16*)x, g, ws);
    hipLaunchKernelGGL(gn_stats_final<bf16>, dim3(n * groups), dim3(GT), 0, s, (const bf16*)x, g, ws, stats);
  } else {
    hipLaunchKernelGGL(gn_stats_partial<float>, dim3(g.nblk, n), dim3(GT), 0, s, (const float*)x, g, ws);
    hipLaunchKernelGGL(gn_stats_final<float>, dim3(n * groups), dim3(GT), 0, s, (const float*)x, g, ws, stats);
  }
  return check_launch("gn_stats");
}

extern "C" int u3d_gn_bwd(int dtype, const void* da, const void* x, int n, int c, long long v, int groups,
                          const float* stats, const float* gamma, const float* beta, void* dx, int accumulate,
                          float* dgamma, float* dbeta, int accumulate_params, float* ws, u3d_stream_t stream) {
  U3D_REQUIRE(dtype == U3D_F32 || dtype == U3D_BF16, "gn_bwd: bad dtype");
  U3D_REQUIRE(da && x && stats && gamma && beta && dx && ws && groups > 0 && c % groups == 0, "gn_bwd: bad args");
  const int vec = dtype == U3D_BF16 ? 8 : 4;
  U3D_REQUIRE(c % vec == 0 && c <= 256, "gn_bwd: channels %d unsupported", c);
  RedGeom g = make_geom(n, c, v, groups, vec);
  hipStream_t s = (hipStream_t)stream;
  double* csum = reinterpret_cast<double*>(
      reinterpret_cast<char*>(ws) + (((long long)n * g.nblk * 2 * c * 4 + 255) / 256) * 256);
  const long long nvec = (long long)n * v * g.chn;
  const int ablk = (int)std::min<long long>(4096, (nvec + GT - 1) / GT);
  if (dtype == U3D_BF16) {
    hipLaunchKernelGGL(gn_bwd_partial<bf16>, dim3(g.nblk, n), dim3(GT), 0, s, (const bf16*)da, (const bf16*)x, g, stats,
                       gamma, beta, ws);
    hipLaunchKernelGGL(gn_bwd_final, dim3(c), dim3(GT), 0, s, g, ws, csum, dgamma, dbeta, accumulate_params);
    hipLaunchKernelGGL(gn_bwd_apply<bf16>, dim3(ablk), dim3(GT), 0, s, (const bf16*)da, (const bf16*)x, g, stats, gamma,
                       beta, csum, (bf16*)dx, accumulate);
  } else {
    hipLaunchKernelGGL(gn_bwd_partial<float>, dim3(g.nblk, n), dim3(GT), 0, s, (const float*)da, (const float*)x, g,
                       stats, gamma, beta, ws);
    hipLaunchKernelGGL(gn_bwd_final, dim3(c), dim3(GT), 0, s, g, ws, csum, dgamma, dbeta, accumulate_params);
    hipLaunchKernelGGL(gn_bwd_apply<float>, dim3(ablk), dim3(GT), 0, s, (const float*)da, (const float*)x, g, stats,
                       gamma, beta, csum, (float*)dx, accumulate);
  }
  return check_launch("gn_bwd");
}

extern "C" int u3d_gn_apply(int dtype, const void* x, int n, int c, long long v, int groups, const float* stats,
                            const float* gamma, const float* beta, void* y, u3d_stream_t stream) {
  U3D_REQUIRE(dtype == U3D_F32 || dtype == U3D_BF16, "gn_apply: bad dtype");
  U3D_REQUIRE(x && y && stats && gamma && beta && n >= 1 && c % 8 == 0 && groups > 0 && c % groups == 0,
              "gn_apply: bad args (c %% 8 == 0)");
  const long long total = (long long)n * v * (c / 8);
  const int grid = (int)std::min<long long>(4096, (total + 255) / 256);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == U3D_BF16)
    hipLaunchKernelGGL(gn_apply_kernel<bf16>, dim3(grid), dim3(256), 0, s, (const bf16*)x, (bf16*)y, n, c, v, groups,
                       stats, gamma, beta);
  else
    hipLaunchKernelGGL(gn_apply_kernel<float>, dim3(grid), dim3(256), 0, s, (const float*)x, (float*)y, n, c, v,
                       groups, stats, gamma, beta);
  return check_launch("gn_apply_kernel");
}
