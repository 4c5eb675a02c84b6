// unet3D_with_feam3 attention branch (reference unet3D.py:142-212 EAM, :1051-1068 renew_token, :1131-1175 forward).
//
// The model keeps only EAM's `attn` output, averaged over the heads (cattn.mean(1), :1136): with k = Wk LN2(x_n)
// (Wk = rows 0..C-1 of kv.weight, :198-199) and q = Wq LN3(token) (:200),
//     att[t][n] = 1/h sum_h sum_d q[t][h,d] k[n][h,d] = sum_c M[t][c] LN2(x_n)[c],   M = (1/h) q Wk   [Nt][C],
// so the forward is one HBM pass over the feature (per-voxel LayerNorm + an Nt x C GEMV) writing Nt maps, and the
// backward one pass writing dx plus fixed-order block partials of dM, dgamma2, dbeta2; the token-side algebra
// (LN3, q, Wq, Wk) is Nt x C x C work in two tiny kernels. The EAM's `x` output (proj/norm2 of the attention
// result) is discarded by the model (:1134), so it is not computed and proj gets no gradient, as in the reference.
#include "common.h"

namespace u3d {

constexpr int EAM_NT = 16;  // max tokens (num_classes - 1)

__device__ __forceinline__ float ln_eps() { return 1e-5f; }

// ------------------------------------------------------------------------------------------ token side
// one block per token t: zhat = (tok - mean) * rstd (LayerNorm norm3, eps 1e-5, biased var), z = zhat g3 + b3,
// q[t] = Wq z, M[t] = inv_h * q[t] Wk
__global__ __launch_bounds__(256) void eam_prep_kernel(const float* __restrict__ tok, int c, const float* __restrict__ g3,
                                                      const float* __restrict__ b3, const float* __restrict__ wq,
                                                      const float* __restrict__ wk, float inv_h,
                                                      float* __restrict__ zhat, float* __restrict__ q,
                                                      float* __restrict__ m) {
  __shared__ float z[256], qs[256], red[256];
  const int t = blockIdx.x, i = threadIdx.x;
  const float xv = i < c ? tok[t * c + i] : 0.f;
  red[i] = xv;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (i < s) red[i] += red[i + s];
    __syncthreads();
  }
  const float mean = red[0] / c;
  __syncthreads();
  const float dv = i < c ? xv - mean : 0.f;
  red[i] = dv * dv;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (i < s) red[i] += red[i + s];
    __syncthreads();
  }
  const float rstd = rsqrtf(red[0] / c + ln_eps());
  if (i < c) {
    const float zh = dv * rstd;
    zhat[t * c + i] = zh;
    z[i] = fmaf(zh, g3[i], b3[i]);
  }
  __syncthreads();
  if (i < c) {
    float s = 0.f;
    for (int k = 0; k < c; ++k) s = fmaf(wq[(long long)i * c + k], z[k], s);
    qs[i] = s;
    q[t * c + i] = s;
  }
  __syncthreads();
  if (i < c) {
    float s = 0.f;
    for (int o = 0; o < c; ++o) s = fmaf(qs[o], wk[(long long)o * c + i], s);
    m[t * c + i] = s * inv_h;
  }
}

// ------------------------------------------------------------------------------------------ forward
// One thread per voxel: mean (pass 1), then sum (x-mean)^2 and sum_c A[t][c] (x_c - mean) (pass 2, cache hits),
// att = rstd * acc[t] + a0[t] with A = M * g2 and a0 = M b2. Output NCDHW [n][nt][v] (coalesced over v).
template <typename T>
__global__ __launch_bounds__(256) void eam_attn_fwd_kernel(const T* __restrict__ x, int n, long long v, int c,
                                                          const float* __restrict__ g2, const float* __restrict__ b2,
                                                          const float* __restrict__ m, int nt,
                                                          float* __restrict__ out) {
  extern __shared__ float sm[];
  float* A = sm;              // [nt][c]
  float* a0 = sm + nt * c;    // [nt]
  for (int e = threadIdx.x; e < nt * c; e += blockDim.x) A[e] = m[e] * g2[e % c];
  for (int t = threadIdx.x; t < nt; t += blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < c; ++k) s = fmaf(m[t * c + k], b2[k], s);
    a0[t] = s;
  }
  __syncthreads();
  constexpr int VN = Vec16<T>::N;
  const long long total = (long long)n * v;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const T* row = x + i * c;
    float s = 0.f;
    for (int k = 0; k < c; k += VN) {
      float f[VN];
      load16(row + k, f);
#pragma unroll
      for (int j = 0; j < VN; ++j) s += f[j];
    }
    const float mean = s / c;
    float var = 0.f, acc[EAM_NT];
#pragma unroll
    for (int t = 0; t < EAM_NT; ++t) acc[t] = 0.f;
    for (int k = 0; k < c; k += VN) {
      float f[VN];
      load16(row + k, f);
#pragma unroll
      for (int j = 0; j < VN; ++j) {
        const float d = f[j] - mean;
        var = fmaf(d, d, var);
#pragma unroll
        for (int t = 0; t < EAM_NT; ++t)
          if (t < nt) acc[t] = fmaf(A[t * c + k + j], d, acc[t]);
      }
    }
    const float rstd = rsqrtf(var / c + ln_eps());
    const long long b = i / v, vox = i - b * v;
#pragma unroll
    for (int t = 0; t < EAM_NT; ++t)
      if (t < nt) out[(b * nt + t) * v + vox] = fmaf(rstd, acc[t], a0[t]);
  }
}

// ------------------------------------------------------------------------------------------ backward
// Tiles of 64 voxels, 4 lanes per voxel (C/4 channels each). Per voxel: xhat, dLN = sum_t g[t] M[t], dxhat = dLN g2,
// dx = rstd (dxhat - mean(dxhat) - xhat mean(dxhat xhat)). Block partials (registers across tiles, fixed order):
//   P[t][c] = sum g[t] xhat[c], Gs[t] = sum g[t], dg2[c] = sum dLN xhat, db2[c] = sum dLN;
// dM[t][c] = g2[c] P[t][c] + b2[c] Gs[t] (LN2 output = xhat g2 + b2) is formed by the reduce kernel.
constexpr int EAM_TV = 64;

template <typename T, int C>
__global__ __launch_bounds__(256) void eam_attn_bwd_kernel(const T* __restrict__ x, int n, long long v,
                                                          const float* __restrict__ g2, const float* __restrict__ m,
                                                          int nt, const float* __restrict__ gout, T* __restrict__ dx,
                                                          int accumulate, float* __restrict__ part) {
  constexpr int CS = C / 4;             // channels per lane
  constexpr int VN = Vec16<T>::N;
  constexpr int CP = C + 1;
  constexpr int NPAIR = (EAM_NT * C + 255) / 256;
  __shared__ float XH[EAM_TV * CP], DL[EAM_TV * CP], GL[EAM_NT * EAM_TV], Ms[EAM_NT * C], G2[C];
  const int tid = threadIdx.x, sub = tid & 3, vl = tid >> 2;
  for (int e = tid; e < nt * C; e += 256) Ms[e] = m[e];
  for (int e = tid; e < C; e += 256) G2[e] = g2[e];
  float accP[NPAIR], accG = 0.f, accDg = 0.f, accDb = 0.f;
#pragma unroll
  for (int k = 0; k < NPAIR; ++k) accP[k] = 0.f;
  const long long total = (long long)n * v;
  const long long ntile = (total + EAM_TV - 1) / EAM_TV;
  __syncthreads();
  for (long long tile = blockIdx.x; tile < ntile; tile += gridDim.x) {
    const long long i = tile * EAM_TV + vl;
    const bool live = i < total;
    const long long b = live ? i / v : 0, vox = live ? i - b * v : 0;
    float xs[CS];
    if (live) {
#pragma unroll
      for (int k = 0; k < CS; k += VN) {
        float f[VN];
        load16(x + i * C + sub * CS + k, f);
#pragma unroll
        for (int j = 0; j < VN; ++j) xs[k + j] = f[j];
      }
    } else {
#pragma unroll
      for (int k = 0; k < CS; ++k) xs[k] = 0.f;
    }
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < CS; ++k) s += xs[k];
    s += __shfl_xor(s, 1);
    s += __shfl_xor(s, 2);
    const float mean = s / C;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < CS; ++k) {
      const float d = xs[k] - mean;
      q = fmaf(d, d, q);
    }
    q += __shfl_xor(q, 1);
    q += __shfl_xor(q, 2);
    const float rstd = rsqrtf(q / C + ln_eps());
    for (int t = sub; t < nt; t += 4) GL[t * EAM_TV + vl] = live ? gout[(b * nt + t) * v + vox] : 0.f;
    __syncthreads();
    float dxh[CS], s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < CS; ++k) {
      const int ch = sub * CS + k;
      float dl = 0.f;
      for (int t = 0; t < nt; ++t) dl = fmaf(GL[t * EAM_TV + vl], Ms[t * C + ch], dl);
      const float xh = (xs[k] - mean) * rstd;
      xs[k] = xh;
      dxh[k] = dl * G2[ch];
      s1 += dxh[k];
      s2 = fmaf(dxh[k], xh, s2);
      XH[vl * CP + ch] = xh;
      DL[vl * CP + ch] = dl;
    }
    s1 += __shfl_xor(s1, 1);
    s1 += __shfl_xor(s1, 2);
    s2 += __shfl_xor(s2, 1);
    s2 += __shfl_xor(s2, 2);
    if (live) {
      const float m1 = s1 / C, m2 = s2 / C;
#pragma unroll
      for (int k = 0; k < CS; k += VN) {
        float f[VN];
        if (accumulate) load16(dx + i * C + sub * CS + k, f);
#pragma unroll
        for (int j = 0; j < VN; ++j) {
          const float d = rstd * (dxh[k + j] - m1 - xs[k + j] * m2);
          f[j] = accumulate ? f[j] + d : d;
        }
        store16(dx + i * C + sub * CS + k, f);
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NPAIR; ++k) {
      const int e = tid + k * 256;
      if (e < nt * C) {
        const int t = e / C, ch = e - t * C;
        float a = accP[k];
        for (int u = 0; u < EAM_TV; ++u) a = fmaf(GL[t * EAM_TV + u], XH[u * CP + ch], a);
        accP[k] = a;
      }
    }
    if (tid < C) {
      float a = accDg, bb = accDb;
      for (int u = 0; u < EAM_TV; ++u) {
        a = fmaf(DL[u * CP + tid], XH[u * CP + tid], a);
        bb += DL[u * CP + tid];
      }
      accDg = a;
      accDb = bb;
    } else if (tid - C < nt && tid - C >= 0) {
      float a = accG;
      for (int u = 0; u < EAM_TV; ++u) a += GL[(tid - C) * EAM_TV + u];
      accG = a;
    }
    __syncthreads();
  }
  // part[block] = [P nt*C][Gs nt][dg2 C][db2 C]
  const int stride = nt * C + nt + 2 * C;
  float* pb = part + (long long)blockIdx.x * stride;
#pragma unroll
  for (int k = 0; k < NPAIR; ++k) {
    const int e = tid + k * 256;
    if (e < nt * C) pb[e] = accP[k];
  }
  if (tid < C) {
    pb[nt * C + nt + tid] = accDg;
    pb[nt * C + nt + C + tid] = accDb;
  } else if (tid - C < nt && tid - C >= 0) {
    pb[nt * C + tid - C] = accG;
  }
}

// fixed-order fp64 sum of the block partials -> dM [nt][c], dg2 / db2 (+= when acc_params)
__global__ void eam_attn_reduce_kernel(const float* __restrict__ part, int nblk, int nt, int c,
                                       const float* __restrict__ g2, const float* __restrict__ b2,
                                       float* __restrict__ dm, float* __restrict__ dg2, float* __restrict__ db2,
                                       int acc_params) {
  const int stride = nt * c + nt + 2 * c;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nt * c + 2 * c) return;
  if (e < nt * c) {
    const int t = e / c, ch = e - t * c;
    double p = 0, gs = 0;
    for (int b = 0; b < nblk; ++b) {
      p += part[(long long)b * stride + e];
      gs += part[(long long)b * stride + nt * c + t];
    }
    dm[e] = (float)(g2[ch] * p + b2[ch] * gs);
  } else {
    const int k = e - nt * c;  // 0..2c-1: dg2 then db2
    double s = 0;
    for (int b = 0; b < nblk; ++b) s += part[(long long)b * stride + nt * c + nt + k];
    float* dst = k < c ? dg2 + k : db2 + (k - c);
    *dst = (acc_params ? *dst : 0.f) + (float)s;
  }
}

// token-side backward, kernel 1 (one block per token): dq[t] = inv_h Wk dM[t]; dz[t] = Wq^T dq[t]
__global__ __launch_bounds__(256) void eam_param_bwd1_kernel(const float* __restrict__ dm, int c,
                                                            const float* __restrict__ wq, const float* __restrict__ wk,
                                                            float inv_h, float* __restrict__ dq,
                                                            float* __restrict__ dz) {
  __shared__ float d[256], qq[256];
  const int t = blockIdx.x, i = threadIdx.x;
  if (i < c) d[i] = dm[t * c + i];
  __syncthreads();
  if (i < c) {
    float s = 0.f;
    for (int k = 0; k < c; ++k) s = fmaf(wk[(long long)i * c + k], d[k], s);
    qq[i] = s * inv_h;
    dq[t * c + i] = s * inv_h;
  }
  __syncthreads();
  if (i < c) {
    float s = 0.f;
    for (int o = 0; o < c; ++o) s = fmaf(wq[(long long)o * c + i], qq[o], s);
    dz[t * c + i] = s;
  }
}

// kernel 2: blocks 0..c-1 = row o of dWk (into kv.weight grad rows 0..c-1; rows c..2c-1 = 0, the unused v half)
// and of dWq; block c = dg3 / db3 from dz and zhat.
__global__ __launch_bounds__(256) void eam_param_bwd2_kernel(const float* __restrict__ dm, int nt, int c,
                                                            const float* __restrict__ zhat,
                                                            const float* __restrict__ g3, const float* __restrict__ b3,
                                                            const float* __restrict__ q, const float* __restrict__ dq,
                                                            const float* __restrict__ dz, float inv_h,
                                                            float* __restrict__ dwq, float* __restrict__ dkv,
                                                            float* __restrict__ dg3, float* __restrict__ db3,
                                                            int accumulate) {
  const int o = blockIdx.x, i = threadIdx.x;
  if (i >= c) return;
  if (o < c) {
    float sk = 0.f, sq = 0.f;
    for (int t = 0; t < nt; ++t) {
      sk = fmaf(q[t * c + o], dm[t * c + i], sk);
      sq = fmaf(dq[t * c + o], fmaf(zhat[t * c + i], g3[i], b3[i]), sq);
    }
    const long long e = (long long)o * c + i;
    dkv[e] = (accumulate ? dkv[e] : 0.f) + sk * inv_h;
    if (!accumulate) dkv[(long long)c * c + e] = 0.f;
    dwq[e] = (accumulate ? dwq[e] : 0.f) + sq;
  } else {
    float sg = 0.f, sb = 0.f;
    for (int t = 0; t < nt; ++t) {
      sg = fmaf(dz[t * c + i], zhat[t * c + i], sg);
      sb += dz[t * c + i];
    }
    dg3[i] = (accumulate ? dg3[i] : 0.f) + sg;
    db3[i] = (accumulate ? db3[i] : 0.f) + sb;
  }
}

// ------------------------------------------------------------------------------------------ trilinear x s
// nn.Upsample(scale_factor=s, mode='trilinear'), align_corners=False (unet3D.py:963-965, deep_up :1138-1175):
// src = max(0, (dst + 0.5) / s - 0.5), i0 = floor(src), i1 = min(i0 + 1, n - 1), l1 = src - i0. NCDHW fp32.
struct Lin {
  int i0, i1;
  float l0, l1;
};
__device__ __forceinline__ Lin lin_src(int dst, int n_in, float inv_s) {
  float src = fmaxf(inv_s * (dst + 0.5f) - 0.5f, 0.f);
  Lin r;
  r.i0 = (int)src;
  r.i1 = r.i0 + (r.i0 < n_in - 1 ? 1 : 0);
  r.l1 = src - (float)r.i0;
  r.l0 = 1.f - r.l1;
  return r;
}

// four consecutive outputs along w per thread (one 16-B store); the d/h weights and the two source rows are shared
__global__ __launch_bounds__(256) void up_tri_fwd_kernel(const float* __restrict__ x, long long nc, int d, int h, int w,
                                                        int s, float* __restrict__ y) {
  const int od = d * s, oh = h * s, ow = w * s, ow4 = ow >> 2;
  const float inv = 1.f / (float)s;
  const long long total = nc * od * oh * ow4;
  for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const long long row = e / ow4;
    const int xw0 = (int)(e - row * ow4) * 4;
    const int xh = (int)(row % oh);
    const long long r2 = row / oh;
    const int xd = (int)(r2 % od);
    const long long ch = r2 / od;
    const float* src = x + ch * d * h * w;
    const Lin ld = lin_src(xd, d, inv), lh = lin_src(xh, h, inv);
    const float* r00 = src + ((long long)ld.i0 * h + lh.i0) * w;
    const float* r01 = src + ((long long)ld.i0 * h + lh.i1) * w;
    const float* r10 = src + ((long long)ld.i1 * h + lh.i0) * w;
    const float* r11 = src + ((long long)ld.i1 * h + lh.i1) * w;
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const Lin lw = lin_src(xw0 + j, w, inv);
      const float v0 = lh.l0 * (lw.l0 * r00[lw.i0] + lw.l1 * r00[lw.i1]) + lh.l1 * (lw.l0 * r01[lw.i0] + lw.l1 * r01[lw.i1]);
      const float v1 = lh.l0 * (lw.l0 * r10[lw.i0] + lw.l1 * r10[lw.i1]) + lh.l1 * (lw.l0 * r11[lw.i0] + lw.l1 * r11[lw.i1]);
      o[j] = ld.l0 * v0 + ld.l1 * v1;
    }
    *reinterpret_cast<f32x4*>(y + row * ow + xw0) = o;
  }
}

__global__ __launch_bounds__(256) void up_tri_fwd1_kernel(const float* __restrict__ x, long long nc, int d, int h, int w,
                                                         int s, float* __restrict__ y) {
  const int od = d * s, oh = h * s, ow = w * s;
  const float inv = 1.f / (float)s;
  const long long total = nc * od * oh * ow;
  for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    long long r = e;
    const int xw = r % ow; r /= ow;
    const int xh = r % oh; r /= oh;
    const int xd = r % od; r /= od;
    const float* src = x + r * d * h * w;
    const Lin ld = lin_src(xd, d, inv), lh = lin_src(xh, h, inv), lw = lin_src(xw, w, inv);
    auto at = [&](int a, int b, int c) { return src[((long long)a * h + b) * w + c]; };
    const float v0 = lh.l0 * (lw.l0 * at(ld.i0, lh.i0, lw.i0) + lw.l1 * at(ld.i0, lh.i0, lw.i1)) +
                     lh.l1 * (lw.l0 * at(ld.i0, lh.i1, lw.i0) + lw.l1 * at(ld.i0, lh.i1, lw.i1));
    const float v1 = lh.l0 * (lw.l0 * at(ld.i1, lh.i0, lw.i0) + lw.l1 * at(ld.i1, lh.i0, lw.i1)) +
                     lh.l1 * (lw.l0 * at(ld.i1, lh.i1, lw.i0) + lw.l1 * at(ld.i1, lh.i1, lw.i1));
    y[e] = ld.l0 * v0 + ld.l1 * v1;
  }
}

// backward along one axis (gather form, deterministic): in [outer][n*s][inner] -> out [outer][n][inner]
__global__ __launch_bounds__(256) void up_tri_axis_bwd_kernel(const float* __restrict__ dy, long long outer, int n,
                                                             long long inner, int s, float* __restrict__ dx,
                                                             int accumulate) {
  const float inv = 1.f / (float)s;
  const int no = n * s;
  const long long total = outer * n * inner;
  for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const long long in_ = e % inner;
    const long long r = e / inner;
    const int i = (int)(r % n);
    const long long ou = r / n;
    const int o_lo = max(0, (i - 1) * s), o_hi = min(no, (i + 2) * s);
    float acc = 0.f;
    for (int o = o_lo; o < o_hi; ++o) {
      const Lin l = lin_src(o, n, inv);
      float wgt = 0.f;
      if (l.i0 == i) wgt += l.l0;
      if (l.i1 == i) wgt += l.l1;
      if (wgt != 0.f) acc = fmaf(wgt, dy[(ou * no + o) * inner + in_], acc);
    }
    dx[e] = accumulate ? dx[e] + acc : acc;
  }
}

// ------------------------------------------------------------------------------------------ renew_token
// renew_token (unet3D.py:1051-1068) for one feature level, exactly as written for any batch size: per class l with
// selected voxels (nearest-resized mask == l+1), the flat sequence x[:,:][cmask] is ordered (sample, channel, voxel)
// and reshaped (C, L) with L = total selected voxels over the batch; row r's mean updates token[l][r]. At B = 1 row
// r is channel r. Chunks of 256 feature voxels; per chunk and class the selected ranks are contiguous, so each
// (chunk, class, channel) run lands in at most two rows: partials [n][chunk][cls][C][2], reduced in fixed order.
constexpr int RT_CHUNK = 256;

__device__ __forceinline__ int nearest_src(int dst, int n_out, int n_in) {
  if (n_out == n_in) return dst;
  if (n_out == 2 * n_in) return dst >> 1;
  const float scale = (float)n_in / (float)n_out;
  return min((int)floorf(dst * scale), n_in - 1);
}

__device__ __forceinline__ int voxel_class(const float* mask, int b, long long vox, int d, int h, int w, int md, int mh,
                                           int mw, int ncls) {
  const int xw = (int)(vox % w);
  const int xh = (int)((vox / w) % h);
  const int xd = (int)(vox / ((long long)w * h));
  const float lab = mask[(((long long)b * md + nearest_src(xd, d, md)) * mh + nearest_src(xh, h, mh)) * mw +
                         nearest_src(xw, w, mw)];
  const float fl = floorf(lab);
  if (lab != fl || lab < 1.f || lab > (float)ncls) return -1;
  return (int)fl - 1;
}

// counts [n][nchunk][ncls]
__global__ __launch_bounds__(RT_CHUNK) void renew_count_kernel(const float* __restrict__ mask, int d, int h, int w,
                                                              int md, int mh, int mw, int ncls, int nchunk,
                                                              int* __restrict__ cnt) {
  __shared__ int sc[32];
  const int b = blockIdx.y, ch = blockIdx.x;
  const long long v = (long long)d * h * w;
  if (threadIdx.x < 32) sc[threadIdx.x] = 0;
  __syncthreads();
  const long long vox = (long long)ch * RT_CHUNK + threadIdx.x;
  if (vox < v) {
    const int l = voxel_class(mask, b, vox, d, h, w, md, mh, mw, ncls);
    if (l >= 0) atomicAdd(&sc[l], 1);  // integer: order-independent
  }
  __syncthreads();
  if (threadIdx.x < ncls) cnt[((long long)b * nchunk + ch) * ncls + threadIdx.x] = sc[threadIdx.x];
}

// off [n][nchunk][ncls] (exclusive prefix over chunks), K [n][ncls], base [n][ncls] (= sum_{b'<b} K), L [ncls]
__global__ void renew_scan_kernel(const int* __restrict__ cnt, int n, int nchunk, int ncls, int* __restrict__ off,
                                  long long* __restrict__ K, long long* __restrict__ base, long long* __restrict__ L) {
  const int l = threadIdx.x;
  if (l >= ncls) return;
  long long tot = 0;
  for (int b = 0; b < n; ++b) {
    base[b * ncls + l] = tot;
    int run = 0;
    for (int c = 0; c < nchunk; ++c) {
      off[((long long)b * nchunk + c) * ncls + l] = run;
      run += cnt[((long long)b * nchunk + c) * ncls + l];
    }
    K[b * ncls + l] = run;
    tot += run;
  }
  L[l] = tot;
}

__device__ __forceinline__ long long row_start(long long base, int c_, long long K, long long kfirst, int C) {
  return base * C + (long long)c_ * K + kfirst;
}

template <typename T>
__global__ __launch_bounds__(RT_CHUNK) void renew_partial_kernel(const T* __restrict__ x, long long sv, long long sc_,
                                                                const float* __restrict__ mask, int d, int h, int w,
                                                                int md, int mh, int mw, int ncls, int C, int nchunk,
                                                                const int* __restrict__ cnt, const int* __restrict__ off,
                                                                const long long* __restrict__ K,
                                                                const long long* __restrict__ base,
                                                                const long long* __restrict__ L,
                                                                float* __restrict__ part) {
  __shared__ int cls[RT_CHUNK];
  const int b = blockIdx.y, chk = blockIdx.x;
  const long long v = (long long)d * h * w;
  const long long vox0 = (long long)chk * RT_CHUNK;
  {
    const long long vox = vox0 + threadIdx.x;
    cls[threadIdx.x] = vox < v ? voxel_class(mask, b, vox, d, h, w, md, mh, mw, ncls) : -1;
  }
  __syncthreads();
  const T* xb = x + (long long)b * v * C;
  // thread per (class, channel) pair; walk the chunk's voxels in order
  for (int e = threadIdx.x; e < ncls * C; e += RT_CHUNK) {
    const int l = e / C, c_ = e - l * C;
    float* dst = part + ((((long long)b * nchunk + chk) * ncls + l) * C + c_) * 2;
    const int cn = cnt[((long long)b * nchunk + chk) * ncls + l];
    if (cn == 0) {
      dst[0] = 0.f;
      dst[1] = 0.f;
      continue;
    }
    const long long Ll = L[l], Kb = K[b * ncls + l];
    const long long kf = off[((long long)b * nchunk + chk) * ncls + l];
    const long long p0 = row_start(base[b * ncls + l], c_, Kb, kf, C);
    const long long r0 = p0 / Ll;
    const long long split = (r0 + 1) * Ll - p0;  // ranks (relative) below this go to row r0
    float s0 = 0.f, s1 = 0.f;
    int k = 0;
    for (int u = 0; u < RT_CHUNK; ++u) {
      if (cls[u] != l) continue;
      const float xv = to_f(xb[(vox0 + u) * sv + (long long)c_ * sc_]);
      if (k < split) s0 += xv; else s1 += xv;
      ++k;
    }
    dst[0] = s0;
    dst[1] = s1;
  }
}

// one block per (class l, row r): token[l][r] = token[l][r] (1 - alpha) + alpha * sum / L, the sum over the runs
// that land in row r — (sample, channel) segments covering r (uniform test), their chunks strided over the
// threads, then a fixed-order block reduction (deterministic)
__global__ __launch_bounds__(256) void renew_update_kernel(const float* __restrict__ part, int n, int nchunk, int ncls,
                                                          int C, int ntok, const int* __restrict__ off,
                                                          const long long* __restrict__ K,
                                                          const long long* __restrict__ base,
                                                          const long long* __restrict__ L, float alpha,
                                                          float* __restrict__ tok) {
  const int l = blockIdx.x, r = blockIdx.y;
  const long long Ll = L[l];
  if (Ll == 0 || l >= ntok) return;  // no voxel of class l+1 at this size (:1055-1058)
  double s = 0;
  for (int b = 0; b < n; ++b) {
    const long long Kb = K[b * ncls + l];
    if (Kb == 0) continue;
    for (int c_ = 0; c_ < C; ++c_) {
      const long long seg0 = row_start(base[b * ncls + l], c_, Kb, 0, C);
      if (r < seg0 / Ll || r > (seg0 + Kb - 1) / Ll) continue;
      for (int chk = threadIdx.x; chk < nchunk; chk += blockDim.x) {
        const long long r0 = (seg0 + off[((long long)b * nchunk + chk) * ncls + l]) / Ll;
        const float* pp = part + ((((long long)b * nchunk + chk) * ncls + l) * C + c_) * 2;
        if (r0 == r) s += pp[0];
        else if (r0 + 1 == r) s += pp[1];
      }
    }
  }
  __shared__ double red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if ((int)threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float mean = (float)(red[0] / (double)Ll);
    tok[l * C + r] = tok[l * C + r] * (1.f - alpha) + mean * alpha;
  }
}

}  // namespace u3d

using namespace u3d;

extern "C" int u3d_eam_prep(const float* tok, int nt, int c, const float* g3, const float* b3, const float* wq,
                            const float* wk, float inv_heads, float* zhat, float* q, float* m, u3d_stream_t stream) {
  U3D_REQUIRE(tok && g3 && b3 && wq && wk && zhat && q && m, "eam_prep: null pointer");
  U3D_REQUIRE(nt > 0 && nt <= EAM_NT && c > 0 && c <= 256, "eam_prep: nt %d (<= %d), c %d (<= 256)", nt, EAM_NT, c);
  hipLaunchKernelGGL(eam_prep_kernel, dim3(nt), dim3(256), 0, (hipStream_t)stream, tok, c, g3, b3, wq, wk, inv_heads,
                     zhat, q, m);
  return check_launch("eam_prep_kernel");
}

extern "C" int u3d_eam_attn_fwd(int dtype, const void* x, int n, long long v, int c, const float* g2, const float* b2,
                                const float* m, int nt, float* out, u3d_stream_t stream) {
  U3D_REQUIRE(dtype == U3D_F32 || dtype == U3D_BF16, "eam_attn_fwd: bad dtype");
  U3D_REQUIRE(x && g2 && b2 && m && out && n > 0 && v > 0, "eam_attn_fwd: bad args");
  U3D_REQUIRE(nt > 0 && nt <= EAM_NT && c % 8 == 0 && c <= 256, "eam_attn_fwd: nt %d, c %d unsupported", nt, c);
  const long long total = (long long)n * v;
  const int nb = (int)std::min<long long>(2048, (total + 255) / 256);
  const size_t lds = (size_t)(nt * c + nt) * sizeof(float);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == U3D_BF16)
    hipLaunchKernelGGL(eam_attn_fwd_kernel<bf16>, dim3(nb), dim3(256), lds, s, (const bf16*)x, n, v, c, g2, b2, m, nt,
                       out);
  else
    hipLaunchKernelGGL(eam_attn_fwd_kernel<float>, dim3(nb), dim3(256), lds, s, (const float*)x, n, v, c, g2, b2, m,
                       nt, out);
  return check_launch("eam_attn_fwd_kernel");
}

extern "C" int u3d_eam_attn_bwd_blocks(int n, long long v) {
  return (int)std::max<long long>(1, std::min<long long>(256, ((long long)n * v + EAM_TV - 1) / EAM_TV));
}

extern "C" long long u3d_eam_attn_bwd_part_floats(int n, long long v, int c, int nt) {
  return (long long)u3d_eam_attn_bwd_blocks(n, v) * (nt * c + nt + 2 * c);
}

template <typename T, int C>
static void launch_eam_bwd(int nb, hipStream_t s, const void* x, int n, long long v, const float* g2, const float* m,
                           int nt, const float* gout, void* dx, int acc, float* part) {
  hipLaunchKernelGGL((eam_attn_bwd_kernel<T, C>), dim3(nb), dim3(256), 0, s, (const T*)x, n, v, g2, m, nt, gout,
                     (T*)dx, acc, part);
}

extern "C" int u3d_eam_attn_bwd(int dtype, const void* x, int n, long long v, int c, const float* g2, const float* b2,
                                const float* m, int nt, const float* gout, void* dx, int accumulate, float* part,
                                float* dm, float* dg2, float* db2, int acc_params, u3d_stream_t stream) {
  U3D_REQUIRE(dtype == U3D_F32 || dtype == U3D_BF16, "eam_attn_bwd: bad dtype");
  U3D_REQUIRE(x && g2 && b2 && m && gout && dx && part && dm && dg2 && db2 && n > 0 && v > 0, "eam_attn_bwd: bad args");
  U3D_REQUIRE(nt > 0 && nt <= EAM_NT, "eam_attn_bwd: nt %d > %d", nt, EAM_NT);
  const int nb = u3d_eam_attn_bwd_blocks(n, v);
  hipStream_t s = (hipStream_t)stream;
  const bool b16 = dtype == U3D_BF16;
  switch (c) {
    case 32: b16 ? launch_eam_bwd<bf16, 32>(nb, s, x, n, v, g2, m, nt, gout, dx, accumulate, part)
                 : launch_eam_bwd<float, 32>(nb, s, x, n, v, g2, m, nt, gout, dx, accumulate, part); break;
    case 64: b16 ? launch_eam_bwd<bf16, 64>(nb, s, x, n, v, g2, m, nt, gout, dx, accumulate, part)
                 : launch_eam_bwd<float, 64>(nb, s, x, n, v, g2, m, nt, gout, dx, accumulate, part); break;
    case 128: b16 ? launch_eam_bwd<bf16, 128>(nb, s, x, n, v, g2, m, nt, gout, dx, accumulate, part)
                  : launch_eam_bwd<float, 128>(nb, s, x, n, v, g2, m, nt, gout, dx, accumulate, part); break;
    default: return fail(U3D_EUNSUPPORTED, "eam_attn_bwd: c = %d (32, 64, 128 supported)", c);
  }
  const int ne = nt * c + 2 * c;
  hipLaunchKernelGGL(eam_attn_reduce_kernel, dim3((ne + 255) / 256), dim3(256), 0, s, part, nb, nt, c, g2, b2, dm, dg2,
                     db2, acc_params);
  return check_launch("eam_attn_bwd");
}

extern "C" int u3d_eam_param_bwd(const float* dm, int nt, int c, const float* zhat, const float* g3, const float* b3,
                                 const float* wq, const float* wk, const float* q, float inv_heads, float* dq_ws,
                                 float* dz_ws, float* dwq, float* dkv, float* dg3, float* db3, int accumulate,
                                 u3d_stream_t stream) {
  U3D_REQUIRE(dm && zhat && g3 && b3 && wq && wk && q && dq_ws && dz_ws && dwq && dkv && dg3 && db3,
              "eam_param_bwd: null pointer");
  U3D_REQUIRE(nt > 0 && nt <= EAM_NT && c > 0 && c <= 256, "eam_param_bwd: nt %d, c %d", nt, c);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(eam_param_bwd1_kernel, dim3(nt), dim3(256), 0, s, dm, c, wq, wk, inv_heads, dq_ws, dz_ws);
  hipLaunchKernelGGL(eam_param_bwd2_kernel, dim3(c + 1), dim3(256), 0, s, dm, nt, c, zhat, g3, b3, q, dq_ws, dz_ws,
                     inv_heads, dwq, dkv, dg3, db3, accumulate);
  return check_launch("eam_param_bwd");
}

extern "C" int u3d_upsample_trilinear(const float* x, long long nc, int d, int h, int w, int s, float* y,
                                      u3d_stream_t stream) {
  U3D_REQUIRE(x && y && nc > 0 && d > 0 && h > 0 && w > 0 && s >= 1, "upsample_trilinear: bad args");
  const long long total = nc * (long long)d * h * w * s * s * s;
  if ((w * s) % 4 == 0) {
    const int nb = (int)std::min<long long>(8192, (total / 4 + 255) / 256);
    hipLaunchKernelGGL(up_tri_fwd_kernel, dim3(nb), dim3(256), 0, (hipStream_t)stream, x, nc, d, h, w, s, y);
  } else {
    const int nb = (int)std::min<long long>(8192, (total + 255) / 256);
    hipLaunchKernelGGL(up_tri_fwd1_kernel, dim3(nb), dim3(256), 0, (hipStream_t)stream, x, nc, d, h, w, s, y);
  }
  return check_launch("up_tri_fwd_kernel");
}

extern "C" long long u3d_upsample_trilinear_bwd_ws_floats(long long nc, int d, int h, int w, int s) {
  return nc * (long long)d * s * h * s * w + nc * (long long)d * s * h * w;
}

extern "C" int u3d_upsample_trilinear_bwd(const float* dy, long long nc, int d, int h, int w, int s, float* dx,
                                          int accumulate, float* ws, u3d_stream_t stream) {
  U3D_REQUIRE(dy && dx && ws && nc > 0 && d > 0 && h > 0 && w > 0 && s >= 1, "upsample_trilinear_bwd: bad args");
  hipStream_t st = (hipStream_t)stream;
  float* t1 = ws;                                      // [nc][sD][sH][W]
  float* t2 = ws + nc * (long long)d * s * h * s * w;  // [nc][sD][H][W]
  auto nblk = [](long long e) { return (int)std::min<long long>(8192, (e + 255) / 256); };
  const long long e1 = nc * (long long)d * s * h * s * w, e2 = nc * (long long)d * s * h * w,
                  e3 = nc * (long long)d * h * w;
  hipLaunchKernelGGL(up_tri_axis_bwd_kernel, dim3(nblk(e1)), dim3(256), 0, st, dy, nc * d * s * h * s, w, 1LL, s, t1, 0);
  hipLaunchKernelGGL(up_tri_axis_bwd_kernel, dim3(nblk(e2)), dim3(256), 0, st, t1, nc * d * s, h, (long long)w, s, t2,
                     0);
  hipLaunchKernelGGL(up_tri_axis_bwd_kernel, dim3(nblk(e3)), dim3(256), 0, st, t2, nc, d, (long long)h * w, s, dx,
                     accumulate);
  return check_launch("up_tri_axis_bwd_kernel");
}

extern "C" long long u3d_renew_token_ws_bytes(int n, int d, int h, int w, int ncls, int c) {
  const long long v = (long long)d * h * w;
  const long long nchunk = (v + RT_CHUNK - 1) / RT_CHUNK;
  const long long ints = 2LL * n * nchunk * ncls;                     // cnt, off
  const long long lls = 2LL * n * ncls + ncls;                         // K, base, L
  const long long flt = (long long)n * nchunk * ncls * c * 2;          // partials
  return ints * 4 + 64 + lls * 8 + 64 + flt * 4;
}

extern "C" int u3d_renew_token(int dtype, const void* x, long long sv, long long sc, int n, int d, int h, int w, int c,
                               const float* mask, int md, int mh, int mw, int ncls, int ntok, float alpha, float* tok,
                               void* ws, u3d_stream_t stream) {
  U3D_REQUIRE(dtype == U3D_F32 || dtype == U3D_BF16, "renew_token: bad dtype");
  U3D_REQUIRE(x && mask && tok && ws && n > 0 && d > 0 && h > 0 && w > 0 && c > 0, "renew_token: bad args");
  U3D_REQUIRE(ncls > 0 && ncls <= 32, "renew_token: num_classes %d (<= 32)", ncls);
  const long long v = (long long)d * h * w;
  const int nchunk = (int)((v + RT_CHUNK - 1) / RT_CHUNK);
  char* p = (char*)ws;
  int* cnt = (int*)p;
  int* off = cnt + (long long)n * nchunk * ncls;
  p += ((2LL * n * nchunk * ncls * 4 + 63) / 64) * 64;
  long long* K = (long long*)p;
  long long* base = K + (long long)n * ncls;
  long long* L = base + (long long)n * ncls;
  p += ((((2LL * n * ncls + ncls) * 8) + 63) / 64) * 64;
  float* part = (float*)p;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(renew_count_kernel, dim3(nchunk, n), dim3(RT_CHUNK), 0, s, mask, d, h, w, md, mh, mw, ncls, nchunk,
                     cnt);
  hipLaunchKernelGGL(renew_scan_kernel, dim3(1), dim3(64), 0, s, cnt, n, nchunk, ncls, off, K, base, L);
  if (dtype == U3D_BF16)
    hipLaunchKernelGGL(renew_partial_kernel<bf16>, dim3(nchunk, n), dim3(RT_CHUNK), 0, s, (const bf16*)x, sv, sc, mask,
                       d, h, w, md, mh, mw, ncls, c, nchunk, cnt, off, K, base, L, part);
  else
    hipLaunchKernelGGL(renew_partial_kernel<float>, dim3(nchunk, n), dim3(RT_CHUNK), 0, s, (const float*)x, sv, sc,
                       mask, d, h, w, md, mh, mw, ncls, c, nchunk, cnt, off, K, base, L, part);
  hipLaunchKernelGGL(renew_update_kernel, dim3(ncls, c), dim3(256), 0, s, part, n, nchunk, ncls, c, ntok, off, K, base,
                     L, alpha, tok);
  return check_launch("renew_token");
}
