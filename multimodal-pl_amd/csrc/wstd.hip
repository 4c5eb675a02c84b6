// Weight standardisation (reference Conv3d.forward, unet3D.py:21-26) fused with the weight packing the
// implicit-GEMM kernels read, and its backward (summing the wgrad split slabs on the way).
// Packs: forward [k^3][cout_p][cin_p], data-grad [k^3][cin_p][cout_p] (a tiled LDS transpose of the first).
#include "common.h"

namespace u3d {

constexpr int WT = 256;

__device__ __forceinline__ double block_sum(double v, double* red) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double t = 0.0;
  for (int i = 0; i < WT / 64; ++i) t += red[i];
  return t;
}

// one block per output channel; iteration j -> (tap t = j / cin, ci = j % cin) so the pack write is
// contiguous along ci; w[co][ci][t] is read from the (cached) row.
template <typename T>
__global__ __launch_bounds__(WT) void wstd_fwd_kernel(const float* __restrict__ w, int cout, int cin, int k3, int std_,
                                                     T* __restrict__ pf, float* __restrict__ st, int cout_p,
                                                     int cin_p) {
  __shared__ double red[WT / 64];
  const int co = blockIdx.x, K = cin * k3;
  const float* wr = w + (long long)co * K;
  float mean = 0.f, sd = 1.f;
  if (std_) {
    double s = 0.0;
    for (int i = threadIdx.x; i < K; i += WT) s += wr[i];
    mean = (float)(block_sum(s, red) / K);
    double v = 0.0;
    for (int i = threadIdx.x; i < K; i += WT) {
      const float c = wr[i] - mean;
      v += (double)c * c;
    }
    const float var = (float)(block_sum(v, red) / (K > 1 ? K - 1 : 1));  // torch.var: unbiased
    sd = sqrtf(var + 1e-12f);
    if (threadIdx.x == 0) {
      st[co * 2] = mean;
      st[co * 2 + 1] = sd;
    }
  }
  for (int j = threadIdx.x; j < K; j += WT) {
    const int t = j / cin, ci = j - t * cin;
    const float x = wr[ci * k3 + t];
    pf[((long long)t * cout_p + co) * cin_p + ci] = from_f<T>(std_ ? (x - mean) / sd : x);
  }
}

// pd[t][ci][co] = pf[t][co][ci], 32x32 tiles through LDS (both sides coalesced)
template <typename T>
__global__ __launch_bounds__(256) void pack_transpose_kernel(const T* __restrict__ pf, T* __restrict__ pd, int cout_p,
                                                            int cin_p) {
  __shared__ T tile[32][33];
  const int t = blockIdx.z, co0 = blockIdx.y * 32, ci0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  const T* src = pf + (long long)t * cout_p * cin_p;
  T* dst = pd + (long long)t * cout_p * cin_p;
  for (int r = ty; r < 32; r += 8) tile[r][tx] = src[(long long)(co0 + r) * cin_p + ci0 + tx];
  __syncthreads();
  for (int r = ty; r < 32; r += 8) dst[(long long)(ci0 + r) * cout_p + co0 + tx] = tile[tx][r];
}

// One level of the in-place slab tree: block (x, y) sums slabs stride*(32y + j), j < 32, into slab stride*32y.
// Each block only touches its own group of slabs, so levels are race-free and the order is fixed.
__global__ __launch_bounds__(256) void sum_slabs_kernel(float* __restrict__ p, long long per, int ns, int stride) {
  const long long i = blockIdx.x * 256LL + threadIdx.x;
  if (i >= per) return;
  const int first = blockIdx.y * 32;
  float s = 0.f;
  for (int j = 0; j < 32; ++j) {
    const int k = first + j;
    if ((long long)k * stride >= ns) break;
    s += p[(long long)k * stride * per + i];
  }
  p[(long long)first * stride * per + i] = s;
}

// dW = (g - mean(g) - W_hat * sum(g * W_hat)/(K-1)) / std per output channel (autograd of unet3D.py:22-26)
__global__ __launch_bounds__(WT) void wstd_bwd_kernel(const float* __restrict__ g, const float* __restrict__ w,
                                                     const float* __restrict__ st, int cout, int cin, int k3, int std_,
                                                     int cout_p, int cin_p, float* __restrict__ dw, int accum) {
  __shared__ double red[WT / 64];
  const int co = blockIdx.x, K = cin * k3;
  const float* wr = w + (long long)co * K;
  float* dr = dw + (long long)co * K;
  auto gval = [&](int t, int ci) { return g[((long long)t * cout_p + co) * cin_p + ci]; };
  if (!std_) {
    for (int j = threadIdx.x; j < K; j += WT) {
      const int t = j / cin, ci = j - t * cin, i = ci * k3 + t;
      dr[i] = (accum ? dr[i] : 0.f) + gval(t, ci);
    }
    return;
  }
  const float mean = st[co * 2], sd = st[co * 2 + 1];
  double m1 = 0.0, m2 = 0.0;
  for (int j = threadIdx.x; j < K; j += WT) {
    const int t = j / cin, ci = j - t * cin;
    const float gv = gval(t, ci);
    const float wh = (wr[ci * k3 + t] - mean) / sd;
    m1 += gv;
    m2 += (double)gv * wh;
  }
  const float fm1 = (float)(block_sum(m1, red) / K);
  const float fm2 = (float)(block_sum(m2, red) / (K > 1 ? K - 1 : 1));
  for (int j = threadIdx.x; j < K; j += WT) {
    const int t = j / cin, ci = j - t * cin, i = ci * k3 + t;
    const float wh = (wr[i] - mean) / sd;
    const float v = (gval(t, ci) - fm1 - wh * fm2) / sd;
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
  if (cout_p != cout || cin_p != cin) U3D_HIP(hipMemsetAsync(wpk_fwd, 0, bytes, s));
  const dim3 tg(cin_p / 32, cout_p / 32, k3);
  if (dtype == U3D_BF16) {
    hipLaunchKernelGGL(wstd_fwd_kernel<bf16>, dim3(cout), dim3(WT), 0, s, w, cout, cin, k3, standardize,
                       (bf16*)wpk_fwd, wstats, cout_p, cin_p);
    if (wpk_dgrad)
      hipLaunchKernelGGL(pack_transpose_kernel<bf16>, tg, dim3(256), 0, s, (const bf16*)wpk_fwd, (bf16*)wpk_dgrad,
                         cout_p, cin_p);
  } else {
    hipLaunchKernelGGL(wstd_fwd_kernel<float>, dim3(cout), dim3(WT), 0, s, w, cout, cin, k3, standardize,
                       (float*)wpk_fwd, wstats, cout_p, cin_p);
    if (wpk_dgrad)
      hipLaunchKernelGGL(pack_transpose_kernel<float>, tg, dim3(256), 0, s, (const float*)wpk_fwd, (float*)wpk_dgrad,
                         cout_p, cin_p);
  }
  return check_launch("wstd_fwd_kernel");
}

extern "C" int u3d_wstd_bwd(float* part, int nsplit, const float* w, const float* wstats, int cout, int cin, int ksize,
                            int standardize, float* dw, int accumulate, u3d_stream_t stream) {
  U3D_REQUIRE(part && w && dw && nsplit >= 1 && (ksize == 1 || ksize == 3), "wstd_bwd: bad args");
  U3D_REQUIRE(!standardize || wstats, "wstd_bwd: wstats required");
  hipStream_t s = (hipStream_t)stream;
  const int k3 = ksize * ksize * ksize, cout_p = round_up(cout, 32), cin_p = round_up(cin, 32);
  const long long per = (long long)k3 * cout_p * cin_p;
  for (int stride = 1; stride < nsplit; stride *= 32) {
    const int groups = cdiv(cdiv(nsplit, stride), 32);
    hipLaunchKernelGGL(sum_slabs_kernel, dim3(cdiv(per, 256), groups), dim3(256), 0, s, part, per, nsplit, stride);
    int rc = check_launch("sum_slabs_kernel");
    if (rc) return rc;
  }
  hipLaunchKernelGGL(wstd_bwd_kernel, dim3(cout), dim3(WT), 0, s, part, w, wstats, cout, cin, k3, standardize, cout_p,
                     cin_p, dw, accumulate);
  return check_launch("wstd_bwd_kernel");
}
