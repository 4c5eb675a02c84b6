// Weight standardisation (reference Conv3d.forward, unet3D.py:21-26) fused with the weight packing the
// implicit-GEMM kernels read, and its backward (summing the wgrad split slabs on the way).
#include "common.h"

namespace u3d {

constexpr int WT = 256;

template <typename T>
__global__ __launch_bounds__(WT) void wstd_fwd_kernel(const float* __restrict__ w, int cout, int cin, int k3, int std_,
                                                     T* __restrict__ pf, T* __restrict__ pd, float* __restrict__ st,
                                                     int cout_p, int cin_p) {
  __shared__ double red[WT / 64];
  __shared__ float s_mean, s_std;
  const int co = blockIdx.x, K = cin * k3;
  const float* wr = w + (long long)co * K;
  float mean = 0.f, sd = 1.f;
  if (std_) {
    double s = 0.0;
    for (int i = threadIdx.x; i < K; i += WT) s += wr[i];
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
      double t = 0.0;
      for (int i = 0; i < WT / 64; ++i) t += red[i];
      s_mean = (float)(t / K);
    }
    __syncthreads();
    mean = s_mean;
    double v = 0.0;
    for (int i = threadIdx.x; i < K; i += WT) {
      float c = wr[i] - mean;
      v += (double)c * c;
    }
    v = wave_sum(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
      double t = 0.0;
      for (int i = 0; i < WT / 64; ++i) t += red[i];
      float var = (float)(t / (K > 1 ? K - 1 : 1));  // torch.var: unbiased
      s_std = sqrtf(var + 1e-12f);
      st[co * 2] = s_mean;
      st[co * 2 + 1] = s_std;
    }
    __syncthreads();
    sd = s_std;
  }
  for (int i = threadIdx.x; i < K; i += WT) {
    const int ci = i / k3, t = i - ci * k3;
    const float v = std_ ? (wr[i] - mean) / sd : wr[i];
    const T tv = from_f<T>(v);
    pf[((long long)t * cout_p + co) * cin_p + ci] = tv;
    if (pd) pd[((long long)t * cin_p + ci) * cout_p + co] = tv;
  }
}

// slab 0 <- sum of slabs (in place)
__global__ void sum_slabs_kernel(float* __restrict__ p, long long per, int ns) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < per; i += (long long)gridDim.x * blockDim.x) {
    float s = p[i];
    for (int k = 1; k < ns; ++k) s += p[k * per + i];
    p[i] = s;
  }
}

__global__ __launch_bounds__(WT) void wstd_bwd_kernel(const float* __restrict__ g, const float* __restrict__ w,
                                                     const float* __restrict__ st, int cout, int cin, int k3, int std_,
                                                     int cout_p, int cin_p, float* __restrict__ dw, int accum) {
  __shared__ double red[2][WT / 64];
  __shared__ double s_m1, s_m2;
  const int co = blockIdx.x, K = cin * k3;
  const float* wr = w + (long long)co * K;
  float* dr = dw + (long long)co * K;
  auto gval = [&](int i) {
    const int ci = i / k3, t = i - ci * k3;
    return g[((long long)t * cout_p + co) * cin_p + ci];
  };
  if (!std_) {
    for (int i = threadIdx.x; i < K; i += WT) dr[i] = (accum ? dr[i] : 0.f) + gval(i);
    return;
  }
  const float mean = st[co * 2], sd = st[co * 2 + 1];
  double m1 = 0.0, m2 = 0.0;
  for (int i = threadIdx.x; i < K; i += WT) {
    const float gv = gval(i);
    const float wh = (wr[i] - mean) / sd;
    m1 += gv;
    m2 += (double)gv * wh;
  }
  m1 = wave_sum(m1);
  m2 = wave_sum(m2);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = m1;
    red[1][threadIdx.x >> 6] = m2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0, b = 0;
    for (int i = 0; i < WT / 64; ++i) {
      a += red[0][i];
      b += red[1][i];
    }
    s_m1 = a / K;
    s_m2 = b / (K > 1 ? K - 1 : 1);
  }
  __syncthreads();
  const float fm1 = (float)s_m1, fm2 = (float)s_m2;
  for (int i = threadIdx.x; i < K; i += WT) {
    const float wh = (wr[i] - mean) / sd;
    const float v = (gval(i) - fm1 - wh * fm2) / sd;
    dr[i] = (accum ? dr[i] : 0.f) + v;
  }
}

}  // namespace u3d

using namespace u3d;

extern "C" int u3d_wstd_fwd(int dtype, const float* w, int cout, int cin, int ksize, int standardize, void* wpk_fwd,
                            void* wpk_dgrad, float* wstats, u3d_stream_t stream) {
  U3D_REQUIRE(dtype == U3D_F32 || dtype == U3D_BF16, "wstd_fwd: bad dtype %d", dtype);
  U3D_REQUIRE(w && wpk_fwd && cout > 0 && cin > 0 && (ksize == 1 || ksize == 3), "wstd_fwd: bad args");
  U3D_REQUIRE(!standardize || wstats, "wstd_fwd: wstats required when standardizing");
  hipStream_t s = (hipStream_t)stream;
  const int k3 = ksize * ksize * ksize, cout_p = round_up(cout, 32), cin_p = round_up(cin, 32);
  const size_t esz = dtype == U3D_BF16 ? 2 : 4, bytes = (size_t)k3 * cout_p * cin_p * esz;
  if (cout_p != cout || cin_p != cin) {
    U3D_HIP(hipMemsetAsync(wpk_fwd, 0, bytes, s));
    if (wpk_dgrad) U3D_HIP(hipMemsetAsync(wpk_dgrad, 0, bytes, s));
  }
  if (dtype == U3D_BF16)
    hipLaunchKernelGGL(wstd_fwd_kernel<bf16>, dim3(cout), dim3(WT), 0, s, w, cout, cin, k3, standardize,
                       (bf16*)wpk_fwd, (bf16*)wpk_dgrad, wstats, cout_p, cin_p);
  else
    hipLaunchKernelGGL(wstd_fwd_kernel<float>, dim3(cout), dim3(WT), 0, s, w, cout, cin, k3, standardize,
                       (float*)wpk_fwd, (float*)wpk_dgrad, wstats, cout_p, cin_p);
  return check_launch("wstd_fwd_kernel");
}

extern "C" int u3d_wstd_bwd(float* part, int nsplit, const float* w, const float* wstats, int cout, int cin, int ksize,
                            int standardize, float* dw, int accumulate, u3d_stream_t stream) {
  U3D_REQUIRE(part && w && dw && nsplit >= 1 && (ksize == 1 || ksize == 3), "wstd_bwd: bad args");
  U3D_REQUIRE(!standardize || wstats, "wstd_bwd: wstats required");
  hipStream_t s = (hipStream_t)stream;
  const int k3 = ksize * ksize * ksize, cout_p = round_up(cout, 32), cin_p = round_up(cin, 32);
  const long long per = (long long)k3 * cout_p * cin_p;
  if (nsplit > 1) {
    int blocks = (int)std::min<long long>(2048, cdiv(per, 256));
    hipLaunchKernelGGL(sum_slabs_kernel, dim3(blocks), dim3(256), 0, s, part, per, nsplit);
    int rc = check_launch("sum_slabs_kernel");
    if (rc) return rc;
  }
  hipLaunchKernelGGL(wstd_bwd_kernel, dim3(cout), dim3(WT), 0, s, part, w, wstats, cout, cin, k3, standardize, cout_p,
                     cin_p, dw, accumulate);
  return check_launch("wstd_bwd_kernel");
}
