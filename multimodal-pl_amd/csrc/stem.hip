// Stem convolutions with 1-2 input channels: conv1 1->32 (reference unet3D.py:1632, :602) and the
// stride-2 conv0 of unet3D_g (in_channel -> init_filter, :1514). K = 27*cin is far below one MFMA
// K-block, so this is a direct VALU conv: one thread per output voxel keeps all cout accumulators in
// registers; the standardised weights sit in LDS as fp32. Input is the model's fp32 NCDHW volume.
#include "common.h"

namespace u3d {

constexpr int ST = 256;
constexpr int SCO = 32;  // max cout handled by one thread (register accumulators)

template <typename T>
__global__ __launch_bounds__(ST) void stem_fwd_kernel(const float* __restrict__ x, const T* __restrict__ wpk,
                                                     T* __restrict__ y, int n, int cin, int d, int h, int w,
                                                     int cout, int cout_p, int cin_p, int stride, int od, int oh,
                                                     int ow, int co0) {
  __shared__ float wl[27 * 4 * SCO];  // [t][ci][co]
  const int ncol = min(SCO, cout - co0);
  for (int i = threadIdx.x; i < 27 * cin * SCO; i += ST) {
    const int co = i % SCO, tc = i / SCO, ci = tc % cin, t = tc / cin;
    wl[i] = co < ncol ? to_f(wpk[((long long)t * cout_p + co0 + co) * cin_p + ci]) : 0.f;
  }
  __syncthreads();
  const long long Vo = (long long)od * oh * ow, total = (long long)n * Vo;
  for (long long i = blockIdx.x * (long long)ST + threadIdx.x; i < total; i += (long long)gridDim.x * ST) {
    const int nn = (int)(i / Vo);
    long long q = i - (long long)nn * Vo;
    const int qw = (int)(q % ow);
    q /= ow;
    const int qh = (int)(q % oh), qd = (int)(q / oh);
    float acc[SCO];
#pragma unroll
    for (int c = 0; c < SCO; ++c) acc[c] = 0.f;
    for (int ci = 0; ci < cin; ++ci) {
      const float* xc = x + ((long long)nn * cin + ci) * d * h * w;
      for (int t = 0; t < 27; ++t) {
        const int zd = qd * stride + t / 9 - 1, zh = qh * stride + (t / 3) % 3 - 1, zw = qw * stride + t % 3 - 1;
        if ((unsigned)zd >= (unsigned)d || (unsigned)zh >= (unsigned)h || (unsigned)zw >= (unsigned)w) continue;
        const float xv = xc[((long long)zd * h + zh) * w + zw];
        const float* wr = wl + (t * cin + ci) * SCO;
#pragma unroll
        for (int c = 0; c < SCO; ++c) acc[c] = fmaf(xv, wr[c], acc[c]);
      }
    }
    T* yr = y + i * cout + co0;
    if (ncol == SCO && (cout % (16 / (int)sizeof(T))) == 0) {
      constexpr int VEC = 16 / sizeof(T);
#pragma unroll
      for (int c = 0; c < SCO; c += VEC) {
        float v[VEC];
#pragma unroll
        for (int e = 0; e < VEC; ++e) v[e] = acc[c + e];
        store16<T>(yr + c, v);
      }
    } else {
      for (int c = 0; c < ncol; ++c) yr[c] = from_f<T>(acc[c]);
    }
  }
}

// dW[t][co][ci] partial over a voxel split: thread per (t, ci, co) output, loop over the split's voxels.
template <typename T>
__global__ __launch_bounds__(ST) void stem_wgrad_kernel(const T* __restrict__ dy, const float* __restrict__ x,
                                                       float* __restrict__ part, int n, int cin, int d, int h, int w,
                                                       int cout, int cout_p, int cin_p, int stride, int od, int oh,
                                                       int ow, long long vps) {
  constexpr int CH = 64;  // voxels staged per step
  __shared__ float sdy[CH][SCO + 1];
  __shared__ float sx[4][27][CH];
  const int split = blockIdx.x;
  const long long Vo = (long long)od * oh * ow, total = (long long)n * Vo;
  const long long v0 = split * vps, v1 = min(total, v0 + vps);
  const int nout = 27 * cin * cout;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // up to 8 outputs per thread
  for (long long vb = v0; vb < v1; vb += CH) {
    __syncthreads();
    for (int i = threadIdx.x; i < CH * SCO; i += ST) {
      const int vv = i / SCO, co = i % SCO;
      const long long v = vb + vv;
      sdy[vv][co] = (v < v1 && co < cout) ? to_f(dy[v * cout + co]) : 0.f;
    }
    for (int i = threadIdx.x; i < CH * 27 * cin; i += ST) {
      const int vv = i % CH, tc = i / CH, t = tc % 27, ci = tc / 27;
      const long long v = vb + vv;
      float xv = 0.f;
      if (v < v1) {
        const int nn = (int)(v / Vo);
        long long q = v - (long long)nn * Vo;
        const int qw = (int)(q % ow);
        q /= ow;
        const int qh = (int)(q % oh), qd = (int)(q / oh);
        const int zd = qd * stride + t / 9 - 1, zh = qh * stride + (t / 3) % 3 - 1, zw = qw * stride + t % 3 - 1;
        if ((unsigned)zd < (unsigned)d && (unsigned)zh < (unsigned)h && (unsigned)zw < (unsigned)w)
          xv = x[(((long long)nn * cin + ci) * d + zd) * h * w + (long long)zh * w + zw];
      }
      sx[ci][t][vv] = xv;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int o = threadIdx.x + k * ST;
      if (o < nout) {
        const int co = o % cout, tc = o / cout, ci = tc % cin, t = tc / cin;
        float a = acc[k];
        for (int vv = 0; vv < CH; ++vv) a = fmaf(sdy[vv][co], sx[ci][t][vv], a);
        acc[k] = a;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int o = threadIdx.x + k * ST;
    if (o < nout) {
      const int co = o % cout, tc = o / cout, ci = tc % cin, t = tc / cin;
      part[(((long long)split * 27 + t) * cout_p + co) * cin_p + ci] = acc[k];
    }
  }
}

}  // namespace u3d

using namespace u3d;

static int sdim(int d, int s) { return (d - 1) / s + 1; }  // k3 pad1: (d + 2 - 3)/s + 1

extern "C" int u3d_stem_fwd(int dtype, const float* x, int n, int cin, int d, int h, int w, const void* wpk, int cout,
                            int stride, void* y, u3d_stream_t stream) {
  U3D_REQUIRE(dtype == U3D_F32 || dtype == U3D_BF16, "stem_fwd: bad dtype");
  U3D_REQUIRE(x && wpk && y && cin >= 1 && cin <= 4 && cout >= 1 && (stride == 1 || stride == 2), "stem_fwd: bad args");
  hipStream_t s = (hipStream_t)stream;
  const int od = sdim(d, stride), oh = sdim(h, stride), ow = sdim(w, stride);
  const long long total = (long long)n * od * oh * ow;
  const int nb = (int)std::min<long long>(8192, (total + ST - 1) / ST);
  for (int co0 = 0; co0 < cout; co0 += SCO) {
    if (dtype == U3D_BF16)
      hipLaunchKernelGGL(stem_fwd_kernel<bf16>, dim3(nb), dim3(ST), 0, s, x, (const bf16*)wpk, (bf16*)y, n, cin, d, h, w,
                         cout, round_up(cout, 32), round_up(cin, 32), stride, od, oh, ow, co0);
    else
      hipLaunchKernelGGL(stem_fwd_kernel<float>, dim3(nb), dim3(ST), 0, s, x, (const float*)wpk, (float*)y, n, cin, d, h,
                         w, cout, round_up(cout, 32), round_up(cin, 32), stride, od, oh, ow, co0);
  }
  return check_launch("stem_fwd_kernel");
}

extern "C" int u3d_stem_wgrad_splits(int n, int d, int h, int w, int stride) {
  const long long total = (long long)n * sdim(d, stride) * sdim(h, stride) * sdim(w, stride);
  return (int)std::max<long long>(1, std::min<long long>(1024, total / 2048));
}

extern "C" int u3d_stem_wgrad(int dtype, const void* dy, const float* x, int n, int cin, int d, int h, int w, int cout,
                              int stride, float* partials, int nsplit, u3d_stream_t stream) {
  U3D_REQUIRE(dtype == U3D_F32 || dtype == U3D_BF16, "stem_wgrad: bad dtype");
  U3D_REQUIRE(dy && x && partials && cin >= 1 && cin <= 4 && cout >= 1 && cout <= SCO && nsplit >= 1,
              "stem_wgrad: bad args");
  U3D_REQUIRE(27 * cin * cout <= 8 * ST, "stem_wgrad: 27*cin*cout > %d", 8 * ST);
  hipStream_t s = (hipStream_t)stream;
  const int od = sdim(d, stride), oh = sdim(h, stride), ow = sdim(w, stride);
  const long long total = (long long)n * od * oh * ow;
  const long long vps = (total + nsplit - 1) / nsplit;
  const int cout_p = round_up(cout, 32), cin_p = round_up(cin, 32);
  U3D_HIP(hipMemsetAsync(partials, 0, (size_t)nsplit * 27 * cout_p * cin_p * 4, s));
  if (dtype == U3D_BF16)
    hipLaunchKernelGGL(stem_wgrad_kernel<bf16>, dim3(nsplit), dim3(ST), 0, s, (const bf16*)dy, x, partials, n, cin, d, h,
                       w, cout, cout_p, cin_p, stride, od, oh, ow, vps);
  else
    hipLaunchKernelGGL(stem_wgrad_kernel<float>, dim3(nsplit), dim3(ST), 0, s, (const float*)dy, x, partials, n, cin, d,
                       h, w, cout, cout_p, cin_p, stride, od, oh, ow, vps);
  return check_launch("stem_wgrad_kernel");
}
