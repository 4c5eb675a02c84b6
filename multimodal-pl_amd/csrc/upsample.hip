// Trilinear x2 upsampling (align_corners=False) fused with the decoder skip addition, and its backward.
// Reference: self.upsamplex2 = nn.Upsample(scale_factor=2, mode='trilinear') (unet3D.py:1646) followed by
// `x = x + skip{3,2,1,0}` (unet3D.py:1764-1783); also the logit upsample of unet3D_g (:1621).
// Source index per dim (PyTorch area_pixel_compute_source_index, scale 1/2):
//   src = max(0, (o + 0.5) * 0.5 - 0.5); i0 = floor(src); i1 = i0 + (i0 < n-1); l1 = src - i0; l0 = 1 - l1.
#include <cstdlib>

#include "common.h"

namespace u3d {

struct Lerp {
  int i0, i1;
  float l0, l1;
};

__device__ __forceinline__ Lerp lerp_of(int o, int n) {
  float src = fmaxf(0.f, (o + 0.5f) * 0.5f - 0.5f);
  int i0 = (int)src;
  Lerp L;
  L.i0 = i0;
  L.i1 = i0 + (i0 < n - 1 ? 1 : 0);
  L.l1 = src - (float)i0;
  L.l0 = 1.f - L.l1;
  return L;
}

// weight of output o onto input i along one dim (0 if o does not read i)
__device__ __forceinline__ float wt_of(int o, int i, int n) {
  Lerp L = lerp_of(o, n);
  float w = 0.f;
  if (L.i0 == i) w += L.l0;
  if (L.i1 == i) w += L.l1;
  return w;
}

// grid: x = (ow, chunk) pairs of one output row, y = oh, z = n * D + od: no 64-bit index arithmetic per element
template <typename T, int VEC>
__global__ __launch_bounds__(256) void up_fwd_kernel(const T* __restrict__ x, const T* __restrict__ skip,
                                                    T* __restrict__ y, int n, int c, int d, int h, int w) {
  const int chn = c / VEC, D = 2 * d, H = 2 * h, W = 2 * w;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= W * chn) return;
  const int j = i % chn, ow = i / chn, oh = blockIdx.y, od = blockIdx.z % D, nn = blockIdx.z / D;
  const Lerp Ld = lerp_of(od, d), Lh = lerp_of(oh, h), Lw = lerp_of(ow, w);
  const T* xb = x + (long long)nn * d * h * w * c + j * VEC;
  auto at = [&](int a, int b, int e, float (&v)[VEC]) { loadv<T, VEC>(xb + ((long long)(a * h + b) * w + e) * c, v); };
  float v000[VEC], v001[VEC], v010[VEC], v011[VEC], v100[VEC], v101[VEC], v110[VEC], v111[VEC];
  at(Ld.i0, Lh.i0, Lw.i0, v000); at(Ld.i0, Lh.i0, Lw.i1, v001);
  at(Ld.i0, Lh.i1, Lw.i0, v010); at(Ld.i0, Lh.i1, Lw.i1, v011);
  at(Ld.i1, Lh.i0, Lw.i0, v100); at(Ld.i1, Lh.i0, Lw.i1, v101);
  at(Ld.i1, Lh.i1, Lw.i0, v110); at(Ld.i1, Lh.i1, Lw.i1, v111);
  const long long off = ((((long long)nn * D + od) * H + oh) * W + ow) * c + j * VEC;
  float sv[VEC];
  if (skip) loadv<T, VEC>(skip + off, sv);
  float o[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e)  // PyTorch CPU nesting order: t0*(h0*(w0*a + w1*b) + h1*(...)) + t1*(...)
    o[e] = Ld.l0 * (Lh.l0 * (Lw.l0 * v000[e] + Lw.l1 * v001[e]) + Lh.l1 * (Lw.l0 * v010[e] + Lw.l1 * v011[e])) +
           Ld.l1 * (Lh.l0 * (Lw.l0 * v100[e] + Lw.l1 * v101[e]) + Lh.l1 * (Lw.l0 * v110[e] + Lw.l1 * v111[e]));
  if (skip)
#pragma unroll
    for (int e = 0; e < VEC; ++e) o[e] += sv[e];
  storev<T, VEC>(y + off, o);
}

// bf16 form with register reuse (round 4): a thread owns the 2 x 2 outputs (oh, ow) in {2ih, 2ih+1} x {2iw, 2iw+1} of
// one output plane od and one 8-channel chunk. Along h and w those outputs read inputs i-1, i, i+1 only (2i reads
// i-1 / i, 2i+1 reads i / i+1, clamped), so 2 x 3 x 3 = 18 loads serve 4 outputs instead of 32 — the one-output
// kernel issued 8 gathered loads per output and was L2-load-bound (80 us at 2x48^3 -> 96^3 x 32). Every output is
// computed with the same Lerp weights and the same expression as up_fwd_kernel: bitwise equal.
// grid: x = (iw, chunk) pairs of one input row, y = ih, z = n * D + od
// CPG > 0 (round 5; channels per GroupNorm(16) group = c / 16, 2 / 4 / 8 / 16): the output's GroupNorm statistics from
// the epilogue. Each thread sums the stored bf16 values of its 4 outputs per group its 8-channel chunk covers (and
// their squares), the block reduces them per (group, sum | square) in a fixed order (wave shuffles, then LDS), one
// [16][2] fp32 row per block into spart ([sample][wps][16][2], wps = blocks per sample: a block never straddles
// samples), and launch_gn16_finalize combines the rows in fp64: no statistics pass over the output.
template <int CPG = 0>
__global__ __launch_bounds__(256) void up_fwd_quad_kernel(const bf16* __restrict__ x, const bf16* __restrict__ skip,
                                                         bf16* __restrict__ y, int n, int c, int d, int h, int w,
                                                         float* __restrict__ spart = nullptr) {
  constexpr bool STATS = CPG > 0;
  constexpr int NSL = STATS ? (CPG >= 8 ? 1 : 8 / CPG) : 1;  // group slots of one 8-channel chunk
  const int chn = c / 8, D = 2 * d, H = 2 * h, W = 2 * w;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  float gs[NSL], gq[NSL];
#pragma unroll
  for (int k = 0; k < NSL; ++k) gs[k] = gq[k] = 0.f;
  if (i < w * chn) {
  const int j = i % chn, iw = i / chn, ih = blockIdx.y, od = blockIdx.z % D, nn = blockIdx.z / D;
  const Lerp Ld = lerp_of(od, d);
  const bf16* xb = x + (long long)nn * d * h * w * c + j * 8;
  const int hs[3] = {max(ih - 1, 0), ih, min(ih + 1, h - 1)}, ws[3] = {max(iw - 1, 0), iw, min(iw + 1, w - 1)};
  u32x4 raw[2][3][3];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 3; ++b)
#pragma unroll
      for (int e = 0; e < 3; ++e)
        raw[a][b][e] = *reinterpret_cast<const u32x4*>(xb + ((long long)((a ? Ld.i1 : Ld.i0) * h + hs[b]) * w + ws[e]) * c);
  // tap t (0: Lerp i0, 1: i1) of output 2i + q along a dim reads slot q + t of (i-1, i, i+1) — except tap 1 of
  // output 2i at i = 0, where Lerp clamps i0 to 0 and i1 = 1 is slot 2 (selected below; all indices static)
  const bool hz = ih == 0, wz = iw == 0;
  auto pick = [&](int a, int qh, int th, int qw, int tw) -> u32x4 {
    const int hsl = qh + th, wsl = qw + tw;
    const bool halt = qh == 0 && th == 1, walt = qw == 0 && tw == 1;
    u32x4 v = raw[a][hsl][wsl];
    if (halt && walt) v = hz ? (wz ? raw[a][2][2] : raw[a][2][wsl]) : (wz ? raw[a][hsl][2] : v);
    else if (halt) v = hz ? raw[a][2][wsl] : v;
    else if (walt) v = wz ? raw[a][hsl][2] : v;
    return v;
  };
  auto un = [](const u32x4& v, int k) {
    const uint32_t u = v[k >> 1];
    return __builtin_bit_cast(float, (k & 1) ? (u & 0xFFFF0000u) : (u << 16));
  };
  // round 6: the 4 skip vectors issued with the 18 input loads (loaded inside the output loop, each was followed by a
  // wait for every load in flight: 4 more round trips per thread; 96^3 launch 73 us = 3.3 TB/s)
  u32x4 skr[2][2];
  if (skip) {
#pragma unroll
    for (int qh = 0; qh < 2; ++qh)
#pragma unroll
      for (int qw = 0; qw < 2; ++qw)
        skr[qh][qw] = *reinterpret_cast<const u32x4*>(
            skip + ((((long long)nn * D + od) * H + 2 * ih + qh) * W + 2 * iw + qw) * c + j * 8);
  }
#pragma unroll
  for (int qh = 0; qh < 2; ++qh) {
    const int oh = 2 * ih + qh;
    if (oh >= H) continue;
    const Lerp Lh = lerp_of(oh, h);
#pragma unroll
    for (int qw = 0; qw < 2; ++qw) {
      const int ow = 2 * iw + qw;
      const Lerp Lw = lerp_of(ow, w);
      const long long off = ((((long long)nn * D + od) * H + oh) * W + ow) * c + j * 8;
      u32x4 t[2][2][2];  // [a][th][tw]
#pragma unroll
      for (int a_ = 0; a_ < 2; ++a_)
#pragma unroll
        for (int th = 0; th < 2; ++th)
#pragma unroll
          for (int tw = 0; tw < 2; ++tw) t[a_][th][tw] = pick(a_, qh, th, qw, tw);
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e)  // PyTorch CPU nesting order, as up_fwd_kernel
        o[e] = Ld.l0 * (Lh.l0 * (Lw.l0 * un(t[0][0][0], e) + Lw.l1 * un(t[0][0][1], e)) +
                        Lh.l1 * (Lw.l0 * un(t[0][1][0], e) + Lw.l1 * un(t[0][1][1], e))) +
               Ld.l1 * (Lh.l0 * (Lw.l0 * un(t[1][0][0], e) + Lw.l1 * un(t[1][0][1], e)) +
                        Lh.l1 * (Lw.l0 * un(t[1][1][0], e) + Lw.l1 * un(t[1][1][1], e)));
      if (skip)
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] += un(skr[qh][qw], e);
      storev<bf16, 8>(y + off, o);
      if constexpr (STATS) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float r = to_f(from_f<bf16>(o[e]));  // the stored value
          gs[e / (CPG >= 8 ? 8 : CPG)] += r;
          gq[e / (CPG >= 8 ? 8 : CPG)] += r * r;
        }
      }
    }
  }
  }  // i < w * chn
  if constexpr (STATS) {
    // per (chunk, slot) over the block: the lanes of a wave that hold the same chunk (lane % chn) by xor shuffles,
    // then the 4 waves in order through LDS (a serial pass of 32 threads over the block's 256 rows was the tail)
    constexpr int NV = 2 * NSL;
    float v[NV];
#pragma unroll
    for (int k = 0; k < NSL; ++k) {
      v[2 * k] = gs[k];
      v[2 * k + 1] = gq[k];
    }
    for (int o = chn; o < 64; o <<= 1)
#pragma unroll
      for (int k = 0; k < NV; ++k) v[k] += __shfl_xor(v[k], o);
    __shared__ float red[4][32][NV];  // [wave][chunk][value]: chn <= 32
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane < chn)
#pragma unroll
      for (int k = 0; k < NV; ++k) red[wave][lane][k] = v[k];
    __syncthreads();
    if (threadIdx.x < 32) {
      const int g = threadIdx.x >> 1, comp = threadIdx.x & 1;
      float t = 0.f;
      for (int wv = 0; wv < (int)(blockDim.x >> 6); ++wv) {
        if constexpr (CPG >= 16) {  // chunks 2g, 2g + 1 (slot 0 each)
          t += red[wv][2 * g][comp];
          t += red[wv][2 * g + 1][comp];
        } else {
          const int jj = g / NSL, k = g - jj * NSL;
          t += red[wv][jj][2 * k + comp];
        }
      }
      const int D_ = 2 * d, od = blockIdx.z % D_, nn = blockIdx.z / D_;
      const long long wps = (long long)gridDim.x * gridDim.y * D_;
      const long long loc = ((long long)od * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
      spart[((long long)nn * wps + loc) * 32 + threadIdx.x] = t;
    }
  }
}

// outputs o (and weights) that read input i along one dim of size n (output 2n): o in {2i-1, 2i, 2i+1, 2i+2}
__device__ __forceinline__ int taps_of(int i, int n, int (&o)[4], float (&wt)[4]) {
  int k = 0;
#pragma unroll
  for (int q = -1; q <= 2; ++q) {
    const int oo = 2 * i + q;
    if (oo < 0 || oo >= 2 * n) continue;
    const float ww = wt_of(oo, i, n);
    if (ww != 0.f) {
      o[k] = oo;
      wt[k++] = ww;
    }
  }
  return k;
}

// gather form of the adjoint; grid: x = (iw, chunk) pairs of one input row, y = ih, z = n * d + id
template <typename T, int VEC>
__global__ __launch_bounds__(256) void up_bwd_kernel(const T* __restrict__ dy, T* __restrict__ dx, int n, int c, int d,
                                                    int h, int w, int accum) {
  const int chn = c / VEC, D = 2 * d, H = 2 * h, W = 2 * w;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= w * chn) return;
  const int j = i % chn, iw = i / chn, ih = blockIdx.y, id = blockIdx.z % d, nn = blockIdx.z / d;
  float acc[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) acc[e] = 0.f;
  const T* yb = dy + (long long)nn * D * H * W * c + j * VEC;
  if constexpr (VEC * sizeof(T) == 16) {
    // two output planes per round: their 4 h rows x 4 w taps (32 loads, clamped where out of range) in flight at
    // once — 2 latency rounds instead of one per (od, oh) row (up to 16). Taps in ascending order, zero-weight ones
    // skipped: the adds are taps_of's, so the result is bitwise the per-row form's (round 4).
    int ow_[4];
    float ww[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int oo = 2 * iw - 1 + q;
      const bool ok = oo >= 0 && oo < W;
      ow_[q] = ok ? oo : 2 * iw;
      ww[q] = ok ? wt_of(oo, iw, w) : 0.f;
    }
#pragma unroll
    for (int a0 = 0; a0 < 4; a0 += 2) {
      u32x4 raw[2][4][4];
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int odc = min(max(2 * id - 1 + a0 + a, 0), D - 1), ohc = min(max(2 * ih - 1 + b, 0), H - 1);
          const T* yr = yb + ((long long)odc * H + ohc) * W * c;
#pragma unroll
          for (int q = 0; q < 4; ++q) raw[a][b][q] = *reinterpret_cast<const u32x4*>(yr + ow_[q] * c);
        }
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const int od = 2 * id - 1 + a0 + a;
        const float wd = od >= 0 && od < D ? wt_of(od, id, d) : 0.f;
        if (wd == 0.f) continue;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int oh = 2 * ih - 1 + b;
          const float wh = oh >= 0 && oh < H ? wt_of(oh, ih, h) : 0.f;
          if (wh == 0.f) continue;
          float part[VEC];
#pragma unroll
          for (int e = 0; e < VEC; ++e) part[e] = 0.f;
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (ww[q] != 0.f) {
              float v[VEC];
              load16<T>(reinterpret_cast<const T*>(&raw[a][b][q]), v);
#pragma unroll
              for (int e = 0; e < VEC; ++e) part[e] = fmaf(ww[q], v[e], part[e]);
            }
          const float wdh = wd * wh;
#pragma unroll
          for (int e = 0; e < VEC; ++e) acc[e] = fmaf(wdh, part[e], acc[e]);
        }
      }
    }
    const long long off = ((((long long)nn * d + id) * h + ih) * w + iw) * c + j * VEC;
    if (accum) {
      float o[VEC];
      loadv<T, VEC>(dx + off, o);
#pragma unroll
      for (int e = 0; e < VEC; ++e) acc[e] += o[e];
    }
    storev<T, VEC>(dx + off, acc);
    return;
  }
  int od_[4], oh_[4], ow_[4];
  float wd[4], wh[4], ww[4];
  const int cd = taps_of(id, d, od_, wd), ch = taps_of(ih, h, oh_, wh), cw = taps_of(iw, w, ow_, ww);
  for (int a = 0; a < cd; ++a)
    for (int b = 0; b < ch; ++b) {
      const T* yr = yb + ((long long)od_[a] * H + oh_[b]) * W * c;
      float part[VEC];
#pragma unroll
      for (int e = 0; e < VEC; ++e) part[e] = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (q < cw) {
          float v[VEC];
          loadv<T, VEC>(yr + ow_[q] * c, v);
#pragma unroll
          for (int e = 0; e < VEC; ++e) part[e] = fmaf(ww[q], v[e], part[e]);
        }
      }
      const float wdh = wd[a] * wh[b];
#pragma unroll
      for (int e = 0; e < VEC; ++e) acc[e] = fmaf(wdh, part[e], acc[e]);
    }
  const long long off = ((((long long)nn * d + id) * h + ih) * w + iw) * c + j * VEC;
  if (accum) {
    float o[VEC];
    loadv<T, VEC>(dx + off, o);
#pragma unroll
    for (int e = 0; e < VEC; ++e) acc[e] += o[e];
  }
  storev<T, VEC>(dx + off, acc);
}

// The same gather for a 2 x 2 block of input rows (id0, id0 + 1) x (ih0, ih0 + 1) per thread: the w-partial sum of an
// output row (od, oh) is computed once and added to every input row that reads it (6 x 6 output rows for 4 input
// rows instead of 4 x 16). Each accumulator sees the same taps, weights and add order as up_bwd_kernel (od ascending,
// then oh ascending, zero-weight taps skipped), so the results are bitwise equal.
// grid: x = (iw, chunk) pairs of one input row, y = ih pair, z = n * ceil(d / 2) + id pair
template <typename T, int VEC>
__global__ __launch_bounds__(256) void up_bwd_blk_kernel(const T* __restrict__ dy, T* __restrict__ dx, int n, int c,
                                                        int d, int h, int w, int accum) {
  const int chn = c / VEC, D = 2 * d, H = 2 * h, W = 2 * w, dp = (d + 1) / 2;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= w * chn) return;
  const int j = i % chn, iw = i / chn, ih0 = 2 * blockIdx.y, id0 = 2 * (blockIdx.z % dp), nn = blockIdx.z / dp;
  // the w taps of input iw: outputs 2iw - 1 .. 2iw + 2 in order, zero weight where out of range or not read (skipped
  // below, so the fmaf chain is taps_of's); static indices keep them in registers
  int ow_[4];
  float ww[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int oo = 2 * iw - 1 + q;
    const bool ok = oo >= 0 && oo < W;
    ow_[q] = ok ? oo : 2 * iw;
    ww[q] = ok ? wt_of(oo, iw, w) : 0.f;
  }
  float acc[2][2][VEC];
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int e = 0; e < VEC; ++e) acc[p][r][e] = 0.f;
  const bool v1d = id0 + 1 < d, v1h = ih0 + 1 < h;
  const T* yb = dy + (long long)nn * D * H * W * c + j * VEC;
  for (int od = 2 * id0 - 1; od <= 2 * id0 + 4; ++od) {
    if (od < 0 || od >= D) continue;
    const float wd0 = wt_of(od, id0, d), wd1 = v1d ? wt_of(od, id0 + 1, d) : 0.f;
    if (wd0 == 0.f && wd1 == 0.f) continue;
    // the plane's 6 output rows x 4 w taps, loaded at once (clamped rows / taps are loaded but not used): one
    // latency round per od instead of one per (od, oh) row (round 4; the adds below are unchanged)
    u32x4 raw[6][4];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const int ohc = min(max(2 * ih0 - 1 + k, 0), H - 1);
      const T* yr = yb + ((long long)od * H + ohc) * W * c;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        raw[k][q] = *reinterpret_cast<const u32x4*>(yr + ow_[q] * c);
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const int oh = 2 * ih0 - 1 + k;
      const bool ohok = oh >= 0 && oh < H;
      const float wh0 = ohok ? wt_of(oh, ih0, h) : 0.f, wh1 = ohok && v1h ? wt_of(oh, ih0 + 1, h) : 0.f;
      if (wh0 == 0.f && wh1 == 0.f) continue;
      float part[VEC];
#pragma unroll
      for (int e = 0; e < VEC; ++e) part[e] = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (ww[q] != 0.f) {
          float v[VEC];
          load16<T>(reinterpret_cast<const T*>(&raw[k][q]), v);
#pragma unroll
          for (int e = 0; e < VEC; ++e) part[e] = fmaf(ww[q], v[e], part[e]);
        }
      }
      const float wdp[2] = {wd0, wd1}, whr[2] = {wh0, wh1};
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int r = 0; r < 2; ++r)
          if (wdp[p] != 0.f && whr[r] != 0.f) {
            const float wdh = wdp[p] * whr[r];
#pragma unroll
            for (int e = 0; e < VEC; ++e) acc[p][r][e] = fmaf(wdh, part[e], acc[p][r][e]);
          }
    }
  }
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      if ((p && !v1d) || (r && !v1h)) continue;
      const long long off = ((((long long)nn * d + id0 + p) * h + ih0 + r) * w + iw) * c + j * VEC;
      float o[VEC];
#pragma unroll
      for (int e = 0; e < VEC; ++e) o[e] = acc[p][r][e];
      if (accum) {
        float pv[VEC];
        loadv<T, VEC>(dx + off, pv);
#pragma unroll
        for (int e = 0; e < VEC; ++e) o[e] += pv[e];
      }
      storev<T, VEC>(dx + off, o);
    }
}

}  // namespace u3d

using namespace u3d;

// the quad kernel's block: one input row's w * c / 8 threads (192 at every trunk level) in whole waves, not 256 (a
// quarter of every block idle before round 6); longer rows: 256-thread blocks
static void up_quad_shape(int c, int w, int& gx, int& bx) {
  const int tpr = w * (c / 8);
  bx = tpr <= 256 ? (tpr + 63) / 64 * 64 : 256;
  gx = cdiv(tpr, bx);
}



extern "C" int u3d_upsample2x_add(int dtype, const void* x, int n, int c, int d, int h, int w, const void* skip, void* y,
                                  u3d_stream_t stream) {
  U3D_REQUIRE(dtype == U3D_F32 || dtype == U3D_BF16, "upsample: bad dtype");
  U3D_REQUIRE(x && y && n > 0 && c > 0 && d > 0 && h > 0 && w > 0, "upsample: bad args");
  hipStream_t s = (hipStream_t)stream;
  const int vec = dtype == U3D_BF16 ? 8 : 4;
  const bool vect = c % vec == 0;
  const int row = 2 * w * (vect ? c / vec : c);
  U3D_REQUIRE((long long)n * 2 * d < 65536 && 2 * h < 65536, "upsample: volume too large for the row grid");
  const dim3 gr(cdiv(row, 256), 2 * h, n * 2 * d), bl(256);
  if (dtype == U3D_BF16 && vect && opt(OPT_UP_QUAD) != 0) {  // UP_QUAD = 0: the one-output kernel (A/B)
    int gx, bx;
    up_quad_shape(c, w, gx, bx);
    hipLaunchKernelGGL(up_fwd_quad_kernel<0>, dim3(gx, h, n * 2 * d), dim3(bx), 0, s, (const bf16*)x,
                       (const bf16*)skip, (bf16*)y, n, c, d, h, w, nullptr);
    return check_launch("up_fwd_quad_kernel");
  }
  if (dtype == U3D_BF16) {
    if (vect) hipLaunchKernelGGL((up_fwd_kernel<bf16, 8>), gr, bl, 0, s, (const bf16*)x, (const bf16*)skip, (bf16*)y, n, c, d, h, w);
    else hipLaunchKernelGGL((up_fwd_kernel<bf16, 1>), gr, bl, 0, s, (const bf16*)x, (const bf16*)skip, (bf16*)y, n, c, d, h, w);
  } else {
    if (vect) hipLaunchKernelGGL((up_fwd_kernel<float, 4>), gr, bl, 0, s, (const float*)x, (const float*)skip, (float*)y, n, c, d, h, w);
    else hipLaunchKernelGGL((up_fwd_kernel<float, 1>), gr, bl, 0, s, (const float*)x, (const float*)skip, (float*)y, n, c, d, h, w);
  }
  return check_launch("up_fwd_kernel");
}

static bool up_stats_ok(int n, int c, int d, int h, int w) {
  const int chn = c / 8;
  return c % 16 == 0 && (c / 16 == 2 || c / 16 == 4 || c / 16 == 8 || c / 16 == 16) && 256 % chn == 0 &&
         (long long)n * 2 * d < 65536 && h < 65536;
}

extern "C" long long u3d_upsample2x_stats_ws_floats(int n, int c, int d, int h, int w) {
  if (!up_stats_ok(n, c, d, h, w)) return 0;
  int gx, bx;
  up_quad_shape(c, w, gx, bx);
  return (long long)n * gx * h * 2 * d * 32;
}

extern "C" int u3d_upsample2x_add_stats(const void* x, int n, int c, int d, int h, int w, const void* skip, void* y,
                                        float* spart, float* stats, u3d_stream_t stream) {
  U3D_REQUIRE(x && y && spart && stats && n > 0 && c > 0 && d > 0 && h > 0 && w > 0, "upsample_stats: bad args");
  U3D_REQUIRE(up_stats_ok(n, c, d, h, w), "upsample_stats: unsupported shape (c = %d)", c);
  hipStream_t s = (hipStream_t)stream;
  int gx, bx;
  up_quad_shape(c, w, gx, bx);
  const dim3 gr(gx, h, n * 2 * d), bl(bx);
  switch (c / 16) {
    case 2: hipLaunchKernelGGL(up_fwd_quad_kernel<2>, gr, bl, 0, s, (const bf16*)x, (const bf16*)skip, (bf16*)y, n, c, d, h, w, spart); break;
    case 4: hipLaunchKernelGGL(up_fwd_quad_kernel<4>, gr, bl, 0, s, (const bf16*)x, (const bf16*)skip, (bf16*)y, n, c, d, h, w, spart); break;
    case 8: hipLaunchKernelGGL(up_fwd_quad_kernel<8>, gr, bl, 0, s, (const bf16*)x, (const bf16*)skip, (bf16*)y, n, c, d, h, w, spart); break;
    default: hipLaunchKernelGGL(up_fwd_quad_kernel<16>, gr, bl, 0, s, (const bf16*)x, (const bf16*)skip, (bf16*)y, n, c, d, h, w, spart); break;
  }
  if (check_launch("up_fwd_quad_kernel<stats>")) return U3D_EHIP;
  const int wps = (int)((long long)gr.x * gr.y * 2 * d);
  return launch_gn16_finalize(spart, n, wps, (double)(c / 16) * 8.0 * d * h * w, stats, s);
}

extern "C" int u3d_upsample2x_bwd(int dtype, const void* dy, int n, int c, int d, int h, int w, void* dx, int accumulate,
                                  u3d_stream_t stream) {
  U3D_REQUIRE(dtype == U3D_F32 || dtype == U3D_BF16, "upsample_bwd: bad dtype");
  U3D_REQUIRE(dy && dx && n > 0 && c > 0 && d > 0 && h > 0 && w > 0, "upsample_bwd: bad args");
  hipStream_t s = (hipStream_t)stream;
  const int vec = dtype == U3D_BF16 ? 8 : 4;
  const bool vect = c % vec == 0;
  const int row = w * (vect ? c / vec : c);
  U3D_REQUIRE((long long)n * d < 65536 && h < 65536, "upsample_bwd: volume too large for the row grid");
  const dim3 gr(cdiv(row, 256), h, n * d), bl(256);
  // 2 x 2 input rows per thread where that still leaves >= 1024 workgroups (2x48^3 -> 96^3: 83.5 -> 61.3 us; at
  // 2x24^3 x 64 its 288 workgroups measured 30.0 -> 49.8 us, so the one-row gather stays there).
  // UP_BWD_BLK = 1 / 0 forces the choice (A/B, tests).
  const dim3 g2(cdiv(row, 256), cdiv(h, 2), n * cdiv(d, 2));
  const int eb = opt(OPT_UP_BWD_BLK);
  const bool blk = eb >= 0 ? eb != 0 : (long long)g2.x * g2.y * g2.z >= 1024;
  if (vect && blk) {
    if (dtype == U3D_BF16)
      hipLaunchKernelGGL((up_bwd_blk_kernel<bf16, 8>), g2, bl, 0, s, (const bf16*)dy, (bf16*)dx, n, c, d, h, w, accumulate);
    else
      hipLaunchKernelGGL((up_bwd_blk_kernel<float, 4>), g2, bl, 0, s, (const float*)dy, (float*)dx, n, c, d, h, w, accumulate);
    return check_launch("up_bwd_blk_kernel");
  }
  if (dtype == U3D_BF16) {
    if (vect) hipLaunchKernelGGL((up_bwd_kernel<bf16, 8>), gr, bl, 0, s, (const bf16*)dy, (bf16*)dx, n, c, d, h, w, accumulate);
    else hipLaunchKernelGGL((up_bwd_kernel<bf16, 1>), gr, bl, 0, s, (const bf16*)dy, (bf16*)dx, n, c, d, h, w, accumulate);
  } else {
    if (vect) hipLaunchKernelGGL((up_bwd_kernel<float, 4>), gr, bl, 0, s, (const float*)dy, (float*)dx, n, c, d, h, w, accumulate);
    else hipLaunchKernelGGL((up_bwd_kernel<float, 1>), gr, bl, 0, s, (const float*)dy, (float*)dx, n, c, d, h, w, accumulate);
  }
  return check_launch("up_bwd_kernel");
}
