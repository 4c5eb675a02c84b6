// Consistency branch of get_loss (reference loss_functions/losses.py:131-178) and EDiceLoss_full2
// (loss_partial.py:137-170).
//
// For every unsupervised organ g (label_t[g] == 0) and every map k (the three EAM attention maps through a sigmoid,
// then softmax(output)[:, g+1] as is), a soft Dice between s = map value and t = softmax(refine[g])[1] over the
// voxels where the refiner is confident (t > 1 - confi or t < confi):
//   d_kg = 1 - (2 I + 1e-5) / (Z + Y + 1e-5),  I = sum s t, Z = sum s^2, Y = sum t^2
//   aux  = sum_{k,g} d_kg * w_k * weight_feature / (num_classes - supcount),  w = [0.125, 0.25, 0.5, 1]
// Forward: one pass per organ (grid.y) over the voxels -> fixed-order fp64 block partials -> a finalize kernel
// forming aux and the per-(g,k) gradient coefficients A = 2/(Z+Y+eps), B = 2(2I+eps)/(Z+Y+eps)^2.
// Backward: one elementwise pass: d map_k = c_k m (-A t + B s) s(1-s) (sigmoid maps), and the softmax map's
// gradient folded through the softmax of the output logits. Layouts are given as element strides so the native
// NDHWC logits / refiner output and NCDHW attention maps are read in place.
#include "common.h"

namespace u3d {

constexpr int CS_MAPS = 4;     // 3 attention maps + softmax(output)
constexpr int CS_CMAX = 16;    // output classes
constexpr int CS_BLOCKS = 128; // voxel blocks per organ

struct ConsistArgs {
  const float* att[3];
  long long att_sc, att_sv;  // attention map strides: organ, voxel
  int natt;
  const float* logits;       // output logits: voxel stride lsv, class stride lsc
  long long lsv, lsc;
  int C;
  const float* refine;       // refiner logits: organ stride rsn, class stride rsc, voxel stride rsv
  long long rsn, rsc, rsv;
  const float* label_t;
  int nt;
  long long V;
  float hi, lo;              // confidence thresholds (1 - confi, confi) as float32
};

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

__device__ __forceinline__ void softmax_row(const ConsistArgs& a, long long v, float* p) {
  float m = -INFINITY;
  for (int k = 0; k < a.C; ++k) {
    p[k] = a.logits[v * a.lsv + k * a.lsc];
    m = fmaxf(m, p[k]);
  }
  float s = 0.f;
  for (int k = 0; k < a.C; ++k) {
    p[k] = expf(p[k] - m);
    s += p[k];
  }
  const float inv = 1.f / s;
  for (int k = 0; k < a.C; ++k) p[k] *= inv;
}

// refiner foreground probability (2-class softmax, channel 1) and the confidence mask
__device__ __forceinline__ float refine_p1(const ConsistArgs& a, int g, long long v, bool& conf) {
  const float r0 = a.refine[g * a.rsn + v * a.rsv], r1 = a.refine[g * a.rsn + a.rsc + v * a.rsv];
  const float m = fmaxf(r0, r1);
  const float e0 = expf(r0 - m), e1 = expf(r1 - m);
  const float p = e1 / (e0 + e1);
  conf = p > a.hi || p < a.lo;
  return p;
}

// part [nt][CS_BLOCKS][1 + 2*CS_MAPS] doubles: Y, then (I, Z) per map
__global__ __launch_bounds__(256) void consist_fwd_kernel(ConsistArgs a, double* __restrict__ part) {
  const int g = blockIdx.y;
  constexpr int NS = 1 + 2 * CS_MAPS;
  double* out = part + ((long long)g * gridDim.x + blockIdx.x) * NS;
  if (a.label_t[g] != 0.f) {
    if (threadIdx.x < NS) out[threadIdx.x] = 0.0;
    return;
  }
  float acc[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) acc[i] = 0.f;
  float p[CS_CMAX];
  for (long long v = blockIdx.x * 256LL + threadIdx.x; v < a.V; v += (long long)gridDim.x * 256) {
    bool conf;
    const float t = refine_p1(a, g, v, conf);
    if (!conf) continue;
    acc[0] = fmaf(t, t, acc[0]);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      if (k < a.natt) {
        const float s = sigm(a.att[k][g * a.att_sc + v * a.att_sv]);
        acc[1 + 2 * k] = fmaf(s, t, acc[1 + 2 * k]);
        acc[2 + 2 * k] = fmaf(s, s, acc[2 + 2 * k]);
      }
    }
    softmax_row(a, v, p);
    const float s = p[g + 1];
    acc[7] = fmaf(s, t, acc[7]);
    acc[8] = fmaf(s, s, acc[8]);
  }
  __shared__ double red[4][NS];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    double x = acc[i];
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    if (lane == 0) red[wave][i] = x;
  }
  __syncthreads();
  if (threadIdx.x < NS) out[threadIdx.x] = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] +
                                           red[3][threadIdx.x];
}

// one thread per organ: fixed-order sum of the partials; coef [nt][CS_MAPS][2] = (c*A, c*B) with c the term's
// weight (0 for supervised organs / absent maps); aux[0] = the weighted dice sum; dice [nt][CS_MAPS] per term
__global__ void consist_finalize_kernel(const double* __restrict__ part, int nblk, int nt, int natt,
                                        const float* __restrict__ label_t, float weight_feature,
                                        float* __restrict__ coef, float* __restrict__ dice, float* __restrict__ aux) {
  __shared__ float terms[32];
  const int g = threadIdx.x;
  constexpr int NS = 1 + 2 * CS_MAPS;
  const float wk[CS_MAPS] = {0.125f, 0.25f, 0.5f, 1.f};
  int sup = 0;
  for (int i = 0; i < nt; ++i) sup += label_t[i] != 0.f;
  float tsum = 0.f;
  if (g < nt) {
    double s[NS];
    for (int i = 0; i < NS; ++i) s[i] = 0.0;
    for (int b = 0; b < nblk; ++b)
      for (int i = 0; i < NS; ++i) s[i] += part[((long long)g * nblk + b) * NS + i];
    const bool active = label_t[g] == 0.f;
    for (int k = 0; k < CS_MAPS; ++k) {
      const bool present = active && (k == 3 || k < natt);
      const float I = (float)s[1 + 2 * k], Z = (float)s[2 + 2 * k], Y = (float)s[0];
      const float den = Z + Y + 1e-5f;
      const float d = 1.f - (2.f * I + 1e-5f) / den;
      const float c = present ? wk[k] * weight_feature / (float)(nt - sup) : 0.f;
      dice[g * CS_MAPS + k] = present ? d : 0.f;
      coef[(g * CS_MAPS + k) * 2] = c * 2.f / den;
      coef[(g * CS_MAPS + k) * 2 + 1] = c * 2.f * (2.f * I + 1e-5f) / (den * den);
      if (present) tsum += d * c;
    }
  }
  if (g < 32) terms[g] = tsum;
  __syncthreads();
  if (g == 0) {
    float t = 0.f;
    for (int i = 0; i < nt; ++i) t += terms[i];  // organ order: as the reference's loop
    aux[0] = t;
  }
}

// backward: grad_out scales everything. datt_k [nt][V] (NCDHW, contiguous), dlogits [V][C] (NDHWC, contiguous)
__global__ __launch_bounds__(256) void consist_bwd_kernel(ConsistArgs a, const float* __restrict__ coef,
                                                         const float* __restrict__ grad_out, float* datt0,
                                                         float* datt1, float* datt2, float* __restrict__ dlogits) {
  const float go = grad_out[0];
  float* datt[3] = {datt0, datt1, datt2};
  float p[CS_CMAX], gp[CS_CMAX];
  for (long long v = blockIdx.x * 256LL + threadIdx.x; v < a.V; v += (long long)gridDim.x * 256) {
    softmax_row(a, v, p);
#pragma unroll
    for (int k = 0; k < CS_CMAX; ++k) gp[k] = 0.f;
    for (int g = 0; g < a.nt; ++g) {
      const bool active = a.label_t[g] == 0.f;
      bool conf = false;
      const float t = active ? refine_p1(a, g, v, conf) : 0.f;
      const bool on = active && conf;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        if (k < a.natt) {
          float d = 0.f;
          if (on) {
            const float s = sigm(a.att[k][g * a.att_sc + v * a.att_sv]);
            const float cA = coef[(g * CS_MAPS + k) * 2], cB = coef[(g * CS_MAPS + k) * 2 + 1];
            d = go * (cB * s - cA * t) * s * (1.f - s);
          }
          datt[k][(long long)g * a.V + v] = d;
        }
      }
      if (on && g + 1 < a.C) {
        const float s = p[g + 1];
        const float cA = coef[(g * CS_MAPS + 3) * 2], cB = coef[(g * CS_MAPS + 3) * 2 + 1];
        gp[g + 1] = go * (cB * s - cA * t);
      }
    }
    float dot = 0.f;
    for (int k = 0; k < a.C; ++k) dot = fmaf(gp[k], p[k], dot);
    for (int k = 0; k < a.C; ++k) dlogits[v * a.C + k] = p[k] * (gp[k] - dot);
  }
}

// ------------------------------------------------------------------------------------------ EDiceLoss_full2
// x [V] (inputs; sigmoid applied when sig), t [V] soft target, m [V] mask (nullable = all ones), uce: + mean
// BCEWithLogits(x, t) over all V. part [nblk][4] doubles: I, Z, Y, bce
__global__ __launch_bounds__(256) void full2_fwd_kernel(const float* __restrict__ x, const float* __restrict__ t,
                                                       const float* __restrict__ m, long long V, int sig, int uce,
                                                       double* __restrict__ part) {
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (long long v = blockIdx.x * 256LL + threadIdx.x; v < V; v += (long long)gridDim.x * 256) {
    const float xv = x[v], tv = t[v];
    if (uce) acc[3] += fmaxf(xv, 0.f) - xv * tv + log1pf(expf(-fabsf(xv)));
    if (m && m[v] == 0.f) continue;
    const float s = sig ? sigm(xv) : xv;
    acc[0] = fmaf(s, tv, acc[0]);
    acc[1] = fmaf(s, s, acc[1]);
    acc[2] = fmaf(tv, tv, acc[2]);
  }
  __shared__ double red[4][4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    double y = acc[i];
    for (int o = 32; o > 0; o >>= 1) y += __shfl_xor(y, o);
    if (lane == 0) red[wave][i] = y;
  }
  __syncthreads();
  if (threadIdx.x < 4)
    part[blockIdx.x * 4 + threadIdx.x] = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] +
                                         red[3][threadIdx.x];
}

// loss[0] = value; coef[0..2] = A, B, bce scale (1/V) for the backward
__global__ void full2_finalize_kernel(const double* __restrict__ part, int nblk, long long V, int uce,
                                      float* __restrict__ loss, float* __restrict__ coef) {
  if (threadIdx.x != 0) return;
  double s[4] = {0, 0, 0, 0};
  for (int b = 0; b < nblk; ++b)
    for (int i = 0; i < 4; ++i) s[i] += part[b * 4 + i];
  const float I = (float)s[0], Z = (float)s[1], Y = (float)s[2];
  const float den = Z + Y + 1e-5f;
  float l = 1.f - (2.f * I + 1e-5f) / den;
  if (uce) l += (float)(s[3] / (double)V);
  loss[0] = l;
  coef[0] = 2.f / den;
  coef[1] = 2.f * (2.f * I + 1e-5f) / (den * den);
  coef[2] = uce ? 1.f / (float)V : 0.f;
}

__global__ __launch_bounds__(256) void full2_bwd_kernel(const float* __restrict__ x, const float* __restrict__ t,
                                                       const float* __restrict__ m, long long V, int sig,
                                                       const float* __restrict__ coef,
                                                       const float* __restrict__ grad_out, float* __restrict__ dx) {
  const float go = grad_out[0], A = coef[0], B = coef[1], cb = coef[2];
  for (long long v = blockIdx.x * 256LL + threadIdx.x; v < V; v += (long long)gridDim.x * 256) {
    const float xv = x[v], tv = t[v];
    const float sg = sigm(xv);
    float d = cb * (sg - tv);
    if (!(m && m[v] == 0.f)) {
      const float s = sig ? sg : xv;
      const float ds = B * s - A * tv;
      d += sig ? ds * s * (1.f - s) : ds;
    }
    dx[v] = go * d;
  }
}

}  // namespace u3d

using namespace u3d;

static int consist_args(ConsistArgs& a, const float* att0, const float* att1, const float* att2, int natt,
                        long long att_sc, long long att_sv, const float* logits, long long lsv, long long lsc, int C,
                        const float* refine, long long rsn, long long rsc, long long rsv, const float* label_t, int nt,
                        long long V, float confi) {
  U3D_REQUIRE(natt >= 0 && natt <= 3 && logits && refine && label_t && V > 0, "consistency: bad args");
  U3D_REQUIRE(C >= 2 && C <= CS_CMAX && nt >= 1 && nt <= C - 1 && nt <= 32, "consistency: C %d, nt %d", C, nt);
  a.att[0] = att0;
  a.att[1] = att1;
  a.att[2] = att2;
  for (int k = 0; k < natt; ++k) U3D_REQUIRE(a.att[k], "consistency: attention map %d is null", k);
  a.att_sc = att_sc;
  a.att_sv = att_sv;
  a.natt = natt;
  a.logits = logits;
  a.lsv = lsv;
  a.lsc = lsc;
  a.C = C;
  a.refine = refine;
  a.rsn = rsn;
  a.rsc = rsc;
  a.rsv = rsv;
  a.label_t = label_t;
  a.nt = nt;
  a.V = V;
  a.hi = (float)(1.0 - (double)confi);
  a.lo = confi;
  return 0;
}

extern "C" long long u3d_consistency_ws_bytes(int nt) {
  return (long long)nt * CS_BLOCKS * (1 + 2 * CS_MAPS) * 8 + (long long)nt * CS_MAPS * 3 * 4 + 256;
}

extern "C" int u3d_consistency_fwd(const float* att0, const float* att1, const float* att2, int natt, long long att_sc,
                                   long long att_sv, const float* logits, long long lsv, long long lsc, int C,
                                   const float* refine, long long rsn, long long rsc, long long rsv,
                                   const float* label_t, int nt, long long V, float confi, float weight_feature,
                                   float* aux, float* dice, float* coef, void* ws, u3d_stream_t stream) {
  ConsistArgs a;
  int rc = consist_args(a, att0, att1, att2, natt, att_sc, att_sv, logits, lsv, lsc, C, refine, rsn, rsc, rsv, label_t,
                        nt, V, confi);
  if (rc) return rc;
  U3D_REQUIRE(aux && dice && coef && ws, "consistency_fwd: null output");
  hipStream_t s = (hipStream_t)stream;
  double* part = (double*)ws;
  hipLaunchKernelGGL(consist_fwd_kernel, dim3(CS_BLOCKS, nt), dim3(256), 0, s, a, part);
  hipLaunchKernelGGL(consist_finalize_kernel, dim3(1), dim3(32), 0, s, part, CS_BLOCKS, nt, natt, label_t,
                     weight_feature, coef, dice, aux);
  return check_launch("consistency_fwd");
}

extern "C" int u3d_consistency_bwd(const float* att0, const float* att1, const float* att2, int natt, long long att_sc,
                                   long long att_sv, const float* logits, long long lsv, long long lsc, int C,
                                   const float* refine, long long rsn, long long rsc, long long rsv,
                                   const float* label_t, int nt, long long V, float confi, const float* coef,
                                   const float* grad_out, float* datt0, float* datt1, float* datt2, float* dlogits,
                                   u3d_stream_t stream) {
  ConsistArgs a;
  int rc = consist_args(a, att0, att1, att2, natt, att_sc, att_sv, logits, lsv, lsc, C, refine, rsn, rsc, rsv, label_t,
                        nt, V, confi);
  if (rc) return rc;
  U3D_REQUIRE(coef && grad_out && dlogits, "consistency_bwd: null output");
  float* d[3] = {datt0, datt1, datt2};
  for (int k = 0; k < natt; ++k) U3D_REQUIRE(d[k], "consistency_bwd: datt%d is null", k);
  const int nb = (int)std::min<long long>(2048, (V + 255) / 256);
  hipLaunchKernelGGL(consist_bwd_kernel, dim3(nb), dim3(256), 0, (hipStream_t)stream, a, coef, grad_out, datt0, datt1,
                     datt2, dlogits);
  return check_launch("consist_bwd_kernel");
}

extern "C" int u3d_edice_full2_fwd(const float* x, const float* t, const float* m, long long V, int sigmoid, int uce,
                                   float* loss, float* coef, void* ws, u3d_stream_t stream) {
  U3D_REQUIRE(x && t && loss && coef && ws && V > 0, "edice_full2_fwd: bad args");
  hipStream_t s = (hipStream_t)stream;
  const int nb = (int)std::min<long long>(CS_BLOCKS, (V + 255) / 256);
  hipLaunchKernelGGL(full2_fwd_kernel, dim3(nb), dim3(256), 0, s, x, t, m, V, sigmoid, uce, (double*)ws);
  hipLaunchKernelGGL(full2_finalize_kernel, dim3(1), dim3(64), 0, s, (const double*)ws, nb, V, uce, loss, coef);
  return check_launch("edice_full2_fwd");
}

extern "C" int u3d_edice_full2_bwd(const float* x, const float* t, const float* m, long long V, int sigmoid,
                                   const float* coef, const float* grad_out, float* dx, u3d_stream_t stream) {
  U3D_REQUIRE(x && t && coef && grad_out && dx && V > 0, "edice_full2_bwd: bad args");
  const int nb = (int)std::min<long long>(2048, (V + 255) / 256);
  hipLaunchKernelGGL(full2_bwd_kernel, dim3(nb), dim3(256), 0, (hipStream_t)stream, x, t, m, V, sigmoid, coef,
                     grad_out, dx);
  return check_launch("full2_bwd_kernel");
}
