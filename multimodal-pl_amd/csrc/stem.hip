// Stem convolutions with 1-2 input channels: conv1 1->32 (reference unet3D.py:1632, :602) and the
// stride-2 conv0 of unet3D_g (in_channel -> init_filter, :1514). K = 27*cin is far below one MFMA
// K-block, so this is a direct VALU conv: one thread per output voxel keeps all cout accumulators in
// registers; the standardised weights sit in LDS as fp32. Input is the model's fp32 NCDHW volume.
#include <cstdlib>

#include "common.h"
#include "gnpart.h"

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

// cin = 1, stride 1, cout = 32 (conv1 of every trunk, unet3D.py:1632): a thread computes FOUR consecutive w voxels
// x 32 channels, so each tap's 32 weights (8 LDS vector reads) serve four voxels and the 3 x 6 input row window is
// read once for them (the one-voxel form was LDS-bound: 216 vector reads per voxel). Same fp32 FMA chain per output
// as stem_fwd_kernel (x fp32, weights from the packed bf16/f32 image), so results are bitwise those of the generic
// kernel. One thread per (output row, group of four w voxels).
// STATS: also the GroupNorm(16, 32) statistics of the stored output (layer0's gn1 input, unet3D.py:56-73):
// per-thread fp32 sums of its 4 voxels x 2 channels per group, fp64 across the block (xor tree + waves in order)
// and the blocks (gnpart.h last-block combine).
template <typename T, bool STATS = false>
__global__ __launch_bounds__(ST) void stem1_fwd_kernel(const float* __restrict__ x, const T* __restrict__ wpk,
                                                      T* __restrict__ y, int d, int h, int w, int cin_p,
                                                      long long rows, double* __restrict__ part = nullptr,
                                                      unsigned* __restrict__ cnt = nullptr,
                                                      float* __restrict__ stats = nullptr, int n = 0) {
  __shared__ f32x4 wl[27 * 8];  // [t][co/4]
  for (int i = threadIdx.x; i < 27 * 32; i += ST) {
    const int co = i % 32, t = i / 32;
    reinterpret_cast<float*>(wl)[i] = to_f(wpk[((long long)t * 32 + co) * cin_p]);
  }
  __syncthreads();
  const int w4 = w >> 2;
  const long long item = (long long)blockIdx.x * ST + threadIdx.x;  // (output row, 4-voxel group)
  const long long row0 = item / w4;
  const bool live = row0 < rows;
  if (!STATS && !live) return;
  const long long row = live ? row0 : rows - 1;
  const int q = (int)(item - row * w4);
  const int yy = (int)(row % h);
  const long long nz = row / h;
  const int z = (int)(nz % d);
  const long long nn = nz / d;
  const int x0 = 4 * q;
  const float* xb = x + nn * d * h * w;
  float acc[4][32];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int c = 0; c < 32; ++c) acc[j][c] = 0.f;
#pragma unroll 1
  for (int kd = 0; kd < 3; ++kd) {
    const int zd = z + kd - 1;
#pragma unroll 1
    for (int kh = 0; kh < 3; ++kh) {
      const int zh = yy + kh - 1;
      const bool rowok = (unsigned)zd < (unsigned)d && (unsigned)zh < (unsigned)h;
      float in[6];
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const int zw = x0 + k - 1;
        in[k] = rowok && (unsigned)zw < (unsigned)w ? xb[((long long)zd * h + zh) * w + zw] : 0.f;
      }
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int t = (kd * 3 + kh) * 3 + kw;
#pragma unroll
        for (int c4 = 0; c4 < 8; ++c4) {
          const f32x4 wv = wl[t * 8 + c4];
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[j][4 * c4 + e] = fmaf(in[j + kw], wv[e], acc[j][4 * c4 + e]);
        }
      }
    }
  }
  T* yr = y + (row * w + x0) * 32;
  constexpr int VEC = 16 / sizeof(T);
  if (live) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int c = 0; c < 32; c += VEC) {
        float v[VEC];
#pragma unroll
        for (int e = 0; e < VEC; ++e) v[e] = acc[j][c + e];
        store16<T>(yr + j * 32 + c, v);
      }
  }
  if constexpr (STATS) {
    // a block may straddle two samples: partials per (block, which sample); a thread's rows belong to sample
    // nn = row / (d * h). fp32 within a wave (512 values), fp64 across waves and blocks.
    __shared__ double red[ST / 64][2][32];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const long long nn = row / ((long long)d * h);
    const long long nfirst = ((long long)blockIdx.x * ST / w4) / ((long long)d * h);
    const int which = (int)(nn - nfirst);  // 0 or 1: a block spans at most two samples (d * h * w / 4 >= ST)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
#pragma unroll
      for (int gq = 0; gq < 16; ++gq) {
        float s1 = 0.f, s2 = 0.f;
        if (live && which == q) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int e = 0; e < 2; ++e) {
              const float t = to_f(from_f<T>(acc[j][2 * gq + e]));  // the stored value
              s1 += t;
              s2 = fmaf(t, t, s2);
            }
        }
        for (int o = 1; o < 64; o <<= 1) {
          s1 += __shfl_xor(s1, o);
          s2 += __shfl_xor(s2, o);
        }
        if (lane == 0) {
          red[wave][q][2 * gq] = s1;
          red[wave][q][2 * gq + 1] = s2;
        }
      }
    }
    __syncthreads();
    // part[block][which][16][2] (which = 0: the first sample the block touches, 1: the next one, zeros if none)
    const int nblk = gridDim.x;
    if (threadIdx.x < 64) {
      const int q = threadIdx.x >> 5, k = threadIdx.x & 31;
      double v = 0;
      for (int wv = 0; wv < ST / 64; ++wv) v += red[wv][q][k];
      __hip_atomic_store(part + ((long long)blockIdx.x * 2 + q) * 32 + k, v, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    if (!gn_part_is_last(cnt, (unsigned)nblk)) return;
    // sample s is touched by the contiguous blocks b_lo..b_hi; block b holds it in slot s - (first sample of b)
    __shared__ double fin[ST][2];
    const long long ips = (long long)d * h * w4;  // items per sample
    const int npairs = n * 16, spl = npairs >= ST ? 1 : ST / npairs;
    for (int p0 = 0; p0 < npairs; p0 += ST) {
      const int p = p0 + threadIdx.x % min(npairs, ST), sl = threadIdx.x / min(npairs, ST);
      double s1 = 0, s2 = 0;
      if (p < npairs && sl < spl) {
        const int smp = p / 16, gq = p % 16;
        const int lo = (int)((smp * ips) / ST), hi = (int)(((smp + 1) * ips - 1) / ST);
        const int b0 = lo + (int)((long long)(hi - lo + 1) * sl / spl), b1 = lo + (int)((long long)(hi - lo + 1) * (sl + 1) / spl);
        for (int bb = b0; bb < b1; ++bb) {
          const int which = smp - (int)(((long long)bb * ST / w4) / ((long long)d * h));
          const double* q = part + ((long long)bb * 2 + which) * 32 + 2 * gq;
          s1 += __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          s2 += __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      fin[threadIdx.x][0] = s1;
      fin[threadIdx.x][1] = s2;
      __syncthreads();
      if (threadIdx.x < min(npairs, ST) && p < npairs) {
        double t1 = 0, t2 = 0;
        for (int k = 0; k < spl; ++k) {
          t1 += fin[k * min(npairs, ST) + threadIdx.x][0];
          t2 += fin[k * min(npairs, ST) + threadIdx.x][1];
        }
        const double M = (double)d * h * w * 2, mean = t1 / M;
        double var = t2 / M - mean * mean;
        if (var < 0) var = 0;
        stats[p * 2] = (float)mean;
        stats[p * 2 + 1] = (float)(1.0 / sqrt(var + 1e-5));
      }
      __syncthreads();
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


// MFMA weight gradient of the 1-channel stride-1 stem (conv1 1->32 of unet3D_baseline / unet3D at 96^3):
//   dW[co][t] = sum_v dy[v][co] * x[v + off(t)]   (M = co, N = 27 taps padded to 32, K = voxels)
// A workgroup walks 2 x 8 x 32-voxel bricks of its split; per brick the dy brick (32 KB, read transposed
// with ds_read_b64_tr_b16) and the fp32 input halo (4 x 10 x 34) sit in LDS. A k-step = 16 consecutive w
// voxels of one row, so the B fragment of tap t is 8 consecutive halo values of the shifted row. The 8
// per-wave tiles are summed in fixed order at the end; the slab rows ci > 0 are written as zeros.
constexpr int SM_BD = 2, SM_BH = 8, SM_BW = 32, SM_NV = SM_BD * SM_BH * SM_BW;
constexpr int SM_HD = SM_BD + 2, SM_HH = SM_BH + 2, SM_HW = SM_BW + 2, SM_NH = SM_HD * SM_HH * SM_HW;

typedef short sm_v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) sm_v4i16 sm_lds_v4i16;
typedef __attribute__((ext_vector_type(8))) __bf16 sm_bf16x8;

__device__ __forceinline__ sm_v4i16 sm_tr_read(const char* base, int off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (sm_lds_v4i16*)((__attribute__((address_space(3))) char*)base + off));
}

__global__ __launch_bounds__(512, 1) void stem_wgrad_mfma_kernel(const bf16* __restrict__ dy,
                                                                const float* __restrict__ x,
                                                                float* __restrict__ part, int n, int d, int h, int w,
                                                                int nbh, int nbw, int nbricks, int per_split) {
  constexpr int ROWB = 64, NT = 512, RPP = NT / 4, DYL = SM_NV / RPP, HLL = (SM_NH + NT - 1) / NT;
  __shared__ __attribute__((aligned(16))) char lds[SM_NV * ROWB + SM_NH * 4];
  char* dyt = lds;
  float* hal = reinterpret_cast<float*>(lds + SM_NV * ROWB);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ch = tid & 3, row0 = tid >> 2;
  const int b0 = blockIdx.x * per_split, b1 = min(nbricks, b0 + per_split);
  const int hq = lane >> 5, gq = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int colb = (16 * (gq & 1) + 4 * p) * 2;
  const int tap = lane & 31;  // B column
  const int ttap = min(tap, 26);
  const int toff = ((ttap / 9) * SM_HH + (ttap / 3) % 3) * SM_HW + ttap % 3;
  u32x4 pdy[DYL];
  float phl[HLL];
  f32x16 acc;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.f;
  auto origin = [&](int b, int& nn, int& d0, int& h0, int& w0) {
    int t = b;
    const int bw_ = t % nbw; t /= nbw;
    const int bh_ = t % nbh; t /= nbh;
    const int nbd = (d + SM_BD - 1) / SM_BD;
    const int bd_ = t % nbd;
    nn = t / nbd;
    d0 = bd_ * SM_BD; h0 = bh_ * SM_BH; w0 = bw_ * SM_BW;
  };
  auto prefetch = [&](int b) {
    int nn, d0, h0, w0;
    origin(b, nn, d0, h0, w0);
#pragma unroll
    for (int i = 0; i < DYL; ++i) {
      const int v = row0 + i * RPP;
      const int vw = v % SM_BW, vh = (v / SM_BW) % SM_BH, vd = v / (SM_BW * SM_BH);
      const int zd = d0 + vd, zh = h0 + vh;
      u32x4 val = {0u, 0u, 0u, 0u};
      if (zd < d && zh < h)
        val = *reinterpret_cast<const u32x4*>(dy + ((((long long)nn * d + zd) * h + zh) * w + w0 + vw) * 32 + ch * 8);
      pdy[i] = val;
    }
#pragma unroll
    for (int i = 0; i < HLL; ++i) {
      const int v = tid + i * NT;
      float val = 0.f;
      if (v < SM_NH) {
        const int hw = v % SM_HW, hh = (v / SM_HW) % SM_HH, hd = v / (SM_HW * SM_HH);
        const int zd = d0 - 1 + hd, zh = h0 - 1 + hh, zw = w0 - 1 + hw;
        if ((unsigned)zd < (unsigned)d && (unsigned)zh < (unsigned)h && (unsigned)zw < (unsigned)w)
          val = x[(((long long)nn * d + zd) * h + zh) * w + zw];
      }
      phl[i] = val;
    }
  };
  auto commit = [&]() {
#pragma unroll
    for (int i = 0; i < DYL; ++i)
      *reinterpret_cast<u32x4*>(dyt + (row0 + i * RPP) * ROWB + ch * 16) = pdy[i];
#pragma unroll
    for (int i = 0; i < HLL; ++i) {
      const int v = tid + i * NT;
      if (v < SM_NH) hal[v] = phl[i];
    }
  };
  if (b0 < b1) {
    prefetch(b0);
    commit();
  }
  __syncthreads();
  for (int b = b0; b < b1; ++b) {
    const bool more = b + 1 < b1;
    prefetch(more ? b + 1 : b);
#pragma unroll
    for (int j = 0; j < SM_NV / 16 / 8; ++j) {
      const int ks = wave + 8 * j;                 // 16 voxels: row (vd, vh), w = 16 * (ks & 1) ...
      const int k0 = (ks * 16 + 8 * hq + q) * ROWB + colb;
      const sm_bf16x8 a = __builtin_bit_cast(sm_bf16x8, __builtin_shufflevector(sm_tr_read(dyt, k0),
                                                                                 sm_tr_read(dyt, k0 + 4 * ROWB),
                                                                                 0, 1, 2, 3, 4, 5, 6, 7));
      const int v0 = ks * 16 + 8 * hq;             // first of this lane's 8 voxels
      const int vw = v0 % SM_BW, vh = (v0 / SM_BW) % SM_BH, vd = v0 / (SM_BW * SM_BH);
      const float* src = hal + (vd * SM_HH + vh) * SM_HW + vw + toff;
      typedef short v8i16 __attribute__((ext_vector_type(8)));
      v8i16 bv;
#pragma unroll
      for (int e = 0; e < 8; ++e) bv[e] = tap < 27 ? (short)from_f<bf16>(src[e]) : (short)0;
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, __builtin_bit_cast(sm_bf16x8, bv), acc, 0, 0, 0);
    }
    __syncthreads();
    if (more) commit();
    __syncthreads();
  }
  float* red = reinterpret_cast<float*>(lds);
  const int r = lane & 31;
#pragma unroll
  for (int i = 0; i < 16; ++i) red[(wave * 32 + (i & 3) + 8 * (i >> 2) + 4 * hq) * 32 + r] = acc[i];
  __syncthreads();
  // slab [27][32 co][32 ci]: ci = 0 carries dW[co][t], the rest is zero
  float* pp = part + (long long)blockIdx.x * 27 * 32 * 32;
  for (int e = tid; e < 27 * 32 * 32; e += NT) {
    const int ci = e & 31, co = (e >> 5) & 31, t = e >> 10;
    float s = 0.f;
    if (ci == 0) {
#pragma unroll
      for (int wv = 0; wv < 8; ++wv) s += red[(wv * 32 + co) * 32 + t];
    }
    pp[e] = s;
  }
}
}  // namespace u3d

using namespace u3d;

static int sdim(int d, int s) { return (d - 1) / s + 1; }  // k3 pad1: (d + 2 - 3)/s + 1

static bool stem1_on() { return opt(OPT_STEM1) != 0; }  // 0: the generic one-voxel kernel

extern "C" long long u3d_stem_fwd_stats_ws_bytes(int n, int d, int h, int w) {
  const long long items = (long long)n * d * h * (w / 4);
  return 256 + ((items + ST - 1) / ST) * 2 * 32 * 8;
}

extern "C" int u3d_stem_fwd_stats(const float* x, int n, int d, int h, int w, const void* wpk, void* y, float* stats,
                                  void* ws, u3d_stream_t stream) {
  U3D_REQUIRE(x && wpk && y && stats && ws && n >= 1 && d >= 1 && h >= 1 && w % 4 == 0 && w >= 4,
              "stem_fwd_stats: bad args (cin 1 -> 32, stride 1, w %% 4 == 0)");
  U3D_REQUIRE((long long)d * h * (w / 4) >= ST, "stem_fwd_stats: volume too small (a block must span <= 2 samples)");
  const long long rows = (long long)n * d * h, items = rows * (w / 4);
  U3D_REQUIRE(rows < 2147483647LL, "stem_fwd_stats: volume too large");
  const dim3 grid((unsigned)((items + ST - 1) / ST));
  unsigned* cnt = reinterpret_cast<unsigned*>(ws);
  double* part = reinterpret_cast<double*>(reinterpret_cast<char*>(ws) + 256);
  hipLaunchKernelGGL((stem1_fwd_kernel<bf16, true>), grid, dim3(ST), 0, (hipStream_t)stream, x, (const bf16*)wpk,
                     (bf16*)y, d, h, w, 32, rows, part, cnt, stats, n);
  return check_launch("stem1_fwd_kernel (statistics)");
}

// bf16 conv1 (cin 1 -> 32, stride 1) on the matrix cores: the 27 taps are the K dimension (padded to 32 = two k16
// steps). One wave computes 32 consecutive w voxels of one output row: the MFMA is issued transposed (A = the 32 x 32
// weight matrix [co][tap], loaded once into registers; B = the voxels' tap vectors, gathered from the fp32 input in
// L1/L2 and rounded to bf16, as torch.autocast rounds conv inputs), so a lane's accumulators are 16 channels of one
// voxel and every lane stores two 16-B chunks after one v_permlane32_swap per pair. The VALU form above spends
// 27 x 32 fp32 FMAs per voxel; this one is bound by the 64 B/voxel output stores.
__global__ __launch_bounds__(256) void stem1_mfma_fwd_kernel(const float* __restrict__ x, const bf16* __restrict__ wpk,
                                                             bf16* __restrict__ y, int d, int h, int w, int cin_p,
                                                             long long tiles, int tpr) {
  const int lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  // A fragments: weight [tap t][co r] at k = 16 s + 8 hh + e (taps >= 27 are zero)
  s16x8 wa[2];
#pragma unroll
  for (int st = 0; st < 2; ++st) {
    uint32_t pk[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int t0 = 16 * st + 8 * hh + 2 * e, t1 = t0 + 1;
      const uint32_t lo = t0 < 27 ? wpk[((long long)t0 * 32 + r) * cin_p] : 0;
      const uint32_t hi = t1 < 27 ? wpk[((long long)t1 * 32 + r) * cin_p] : 0;
      pk[e] = lo | (hi << 16);
    }
    wa[st] = __builtin_bit_cast(s16x8, (u32x4){pk[0], pk[1], pk[2], pk[3]});
  }
  __shared__ __attribute__((aligned(16))) char otile[4][32 * 64];
  char* const ot = otile[threadIdx.x >> 6];
  const long long wave0 = ((long long)blockIdx.x * 256 + threadIdx.x) >> 6, nwave = (long long)gridDim.x * 4;
  // 32-bit index math, one division chain per output row (64-bit divisions per tile cost more than the MFMAs; hoisting
  // the 16 tap offsets into registers measured slower: 78 vs 59 us)
  const int rows = (int)(tiles / tpr);
  for (int row = (int)wave0; row < rows; row += (int)nwave) {
  for (int x0 = 0; x0 < w; x0 += 32) {
    const int yy = row % h, nz = row / h, z = nz % d;
    const float* xb = x + (long long)(nz / d) * d * h * w;
    const int xv = x0 + r;
    s16x8 bfr[2];
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int tap = 16 * st + 8 * hh + e;
        const int kd = tap / 9, kh = (tap / 3) % 3, kw = tap % 3;
        const int zd = z + kd - 1, zh = yy + kh - 1, zw = xv + kw - 1;
        const bool ok = tap < 27 && (unsigned)zd < (unsigned)d && (unsigned)zh < (unsigned)h && (unsigned)zw < (unsigned)w;
        const float a = xb[ok ? ((long long)zd * h + zh) * w + zw : 0];  // clamped address: straight-line loads
        v[e] = ok ? a : 0.f;
      }
      bfr[st] = __builtin_bit_cast(s16x8, (u32x4){pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]),
                                                  pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7])});
    }
    f32x16 acc = (f32x16){};
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[0], bfr[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[1], bfr[1], acc, 0, 0, 0);
    uint32_t pk[4][2];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int e = 0; e < 2; ++e) pk[q][e] = pack_bf16x2(acc[4 * q + 2 * e], acc[4 * q + 2 * e + 1]);
#pragma unroll
    for (int q = 0; q < 4; q += 2)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const auto sw = __builtin_amdgcn_permlane32_swap(pk[q][e], pk[q + 1][e], false, false);
        pk[q][e] = sw[0];
        pk[q + 1][e] = sw[1];
      }
    // through LDS so that each store instruction writes 1 KB contiguous (the tile is 32 voxels x 64 B)
#pragma unroll
    for (int u2 = 0; u2 < 2; ++u2)
      *reinterpret_cast<u32x4*>(ot + r * 64 + 32 * u2 + 16 * hh) =
          (u32x4){pk[2 * u2][0], pk[2 * u2][1], pk[2 * u2 + 1][0], pk[2 * u2 + 1][1]};
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    const int nv = min(32, w - x0);
#pragma unroll
    for (int u2 = 0; u2 < 2; ++u2) {
      const int q = lane + 64 * u2;  // 16-B chunk of the tile
      const u32x4 v = *reinterpret_cast<const u32x4*>(ot + q * 16);
      if ((q >> 2) < nv) *reinterpret_cast<u32x4*>(y + ((long long)row * w + x0) * 32 + q * 8) = v;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  }
  }
}

// Off by default: 83 -> 59 us per launch in isolation but step-neutral (same-box A/B 6.961 vs 6.957 ms: in the step the
// stem is bound by its 113 MB of output stores), and the VALU kernel keeps the fp32 input. U3D_STEM_MFMA=1 enables it.
static bool stem1_mfma_on() {
  static const bool on = [] {
    const char* e = getenv("U3D_STEM_MFMA");
    return e && atoi(e) != 0;
  }();
  return on;
}

extern "C" int u3d_stem_fwd(int dtype, const float* x, int n, int cin, int d, int h, int w, const void* wpk, int cout,
                            int stride, void* y, u3d_stream_t stream) {
  U3D_REQUIRE(dtype == U3D_F32 || dtype == U3D_BF16, "stem_fwd: bad dtype");
  U3D_REQUIRE(x && wpk && y && cin >= 1 && cin <= 4 && cout >= 1 && (stride == 1 || stride == 2), "stem_fwd: bad args");
  hipStream_t s = (hipStream_t)stream;
  const int od = sdim(d, stride), oh = sdim(h, stride), ow = sdim(w, stride);
  const long long total = (long long)n * od * oh * ow;
  if (dtype == U3D_BF16 && cin == 1 && stride == 1 && cout == 32 && stem1_mfma_on()) {
    const int tpr = cdiv(w, 32);
    const long long tiles = (long long)n * d * h * tpr;
    U3D_REQUIRE((long long)n * d * h < (1LL << 31), "stem_fwd: too many rows");
    const unsigned grid = (unsigned)std::min<long long>(8192, ((long long)n * d * h + 3) / 4);
    hipLaunchKernelGGL(stem1_mfma_fwd_kernel, dim3(grid), dim3(256), 0, s, x, (const bf16*)wpk, (bf16*)y, d, h, w,
                       round_up(cin, 32), tiles, tpr);
    return check_launch("stem1_mfma_fwd_kernel");
  }
  if (cin == 1 && stride == 1 && cout == 32 && w % 4 == 0 && (long long)n * d * h < 2147483647LL && stem1_on()) {
    const long long rows = (long long)n * d * h, items = rows * (w / 4);
    const dim3 grid((unsigned)((items + ST - 1) / ST));
    if (dtype == U3D_BF16)
      hipLaunchKernelGGL(stem1_fwd_kernel<bf16>, grid, dim3(ST), 0, s, x, (const bf16*)wpk, (bf16*)y, d, h, w,
                         round_up(cin, 32), rows);
    else
      hipLaunchKernelGGL(stem1_fwd_kernel<float>, grid, dim3(ST), 0, s, x, (const float*)wpk, (float*)y, d, h, w,
                         round_up(cin, 32), rows);
    return check_launch("stem1_fwd_kernel");
  }
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

static bool stem_mfma_ok(int dtype, int cin, int cout, int w, int stride) {
  return dtype == U3D_BF16 && cin == 1 && cout == 32 && stride == 1 && w % SM_BW == 0;
}
static int stem_bricks(int n, int d, int h, int w) {
  return n * cdiv(d, SM_BD) * cdiv(h, SM_BH) * (w / SM_BW);
}

extern "C" int u3d_stem_wgrad_splits2(int dtype, int n, int cin, int d, int h, int w, int cout, int stride) {
  if (stem_mfma_ok(dtype, cin, cout, w, stride)) {
    const int nb = stem_bricks(n, d, h, w), per = cdiv(nb, std::min(256, nb));
    return cdiv(nb, per);  // splits that all receive bricks: no zero-filled slabs
  }
  const long long total = (long long)n * sdim(d, stride) * sdim(h, stride) * sdim(w, stride);
  return (int)std::max<long long>(1, std::min<long long>(1024, total / 2048));
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
  if (stem_mfma_ok(dtype, cin, cout, w, stride)) {
    const int nb = stem_bricks(n, d, h, w), per = cdiv(nb, nsplit), ns_eff = cdiv(nb, per);
    if (ns_eff < nsplit)
      U3D_HIP(hipMemsetAsync(partials + (long long)ns_eff * 27 * 32 * 32, 0, (size_t)(nsplit - ns_eff) * 27 * 32 * 32 * 4,
                             s));
    hipLaunchKernelGGL(stem_wgrad_mfma_kernel, dim3(ns_eff), dim3(512), 0, s, (const bf16*)dy, x, partials, n, d, h, w,
                       cdiv(h, SM_BH), w / SM_BW, nb, per);
    return check_launch("stem_wgrad_mfma_kernel");
  }
  U3D_HIP(hipMemsetAsync(partials, 0, (size_t)nsplit * 27 * cout_p * cin_p * 4, s));
  if (dtype == U3D_BF16)
    hipLaunchKernelGGL(stem_wgrad_kernel<bf16>, dim3(nsplit), dim3(ST), 0, s, (const bf16*)dy, x, partials, n, cin, d, h,
                       w, cout, cout_p, cin_p, stride, od, oh, ow, vps);
  else
    hipLaunchKernelGGL(stem_wgrad_kernel<float>, dim3(nsplit), dim3(ST), 0, s, (const float*)dy, x, partials, n, cin, d,
                       h, w, cout, cout_p, cin_p, stride, od, oh, ow, vps);
  return check_launch("stem_wgrad_kernel");
}
