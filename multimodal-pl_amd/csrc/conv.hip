// 3-D convolution as MFMA implicit GEMM on NDHWC activations (gfx950).
//
// Replaces F.conv3d in Conv3d.forward (reference unet3D.py:27), reached from NoBottleneck (:56-73),
// the trunk (:1734-1806 / :663-718 / :1568-1623) and precls_conv (:1653-1657), plus its autograd
// backward (data and weight gradients).
//
// One tap-list kernel covers every forward and data-gradient case:
//   out[n, q*so + po, co] = sum_t sum_ci  A[n, q*si + off_t, ci] * Wt[t][co][ci]
// forward:           q = output voxel, so = 1, si = stride, off_t = tap - pad
// dgrad stride 1:    q = input voxel,  si = 1, off_t = pad - tap, W packed [t][ci][co]
// dgrad stride 2:    8 parity classes p, q = class voxel, so = 2, po = p, dense sub-kernel of 1 or 2 taps/dim
// The optional prologue A = relu(x * scale[n,c] + shift[n,c]) applies GroupNorm+ReLU on load
// (unet3D.py:44-53); out-of-range taps read 0 *after* the prologue, as zero padding of the normalised
// tensor does in the reference.
#include <algorithm>
#include <cstdlib>

#include "common.h"

namespace u3d {

constexpr int BK = 32;  // channels per K-step
constexpr int NTHR = 256;

struct Geom {
  int cin, cout, cin_p, cout_p;
  int id, ih, iw;
  int od, oh, ow;
  int qd, qh, qw;
  int so, pod, poh, pow_;
  int si;
  int ntaps;
  int gn_groups;
  int nsamp, nsplit, kps;  // samples; split-K count and K-steps per split
  int mtiles, ntiles;      // igemm_bf16_kernel's 1-D grid decomposition
  float* slab;             // split-K partials [nsplit][nsamp][Mq][cout] (nsplit > 1)
  int tap_w[27];
  signed char tap_d[27], tap_h[27], tap_x[27];
};

template <typename T> struct MfmaTraits;
// bf16: v_mfma_f32_32x32x16_bf16, lane holds 8 consecutive k of its row -> one 16-B chunk per k16 step.
template <> struct MfmaTraits<bf16> {
  static constexpr int NCH = BK * 2 / 16;  // 4 chunks of 16 B per row
  __device__ static int swz(int r, int c) { return c ^ ((r >> 2) & 3); }
};
// f32: v_mfma_f32_32x32x2_f32 (exact fp32 FMA chain); lane half h uses k = 16h + 4j + e of the step,
// so each lane reads its 16 k-values as 4 contiguous 16-B chunks (4h + j).
template <> struct MfmaTraits<float> {
  static constexpr int NCH = BK * 4 / 16;  // 8 chunks
  __device__ static int swz(int r, int c) { return c ^ (r & 7); }
};

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;

template <typename T, int TM, int TN>
__device__ __forceinline__ void mfma_step(const char* As, const char* Bs, int arow0, int brow0, int lane,
                                          f32x16 (&acc)[TM][TN]) {
  using TR = MfmaTraits<T>;
  constexpr int ROWB = BK * sizeof(T);
  const int r = lane & 31, h = lane >> 5;
  if constexpr (sizeof(T) == 2) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 a[TM], b[TN];
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        int row = arow0 + tm * 32 + r;
        a[tm] = *reinterpret_cast<const bf16x8*>(As + row * ROWB + TR::swz(row, 2 * s + h) * 16);
      }
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        int row = brow0 + tn * 32 + r;
        b[tn] = *reinterpret_cast<const bf16x8*>(Bs + row * ROWB + TR::swz(row, 2 * s + h) * 16);
      }
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[tm], b[tn], acc[tm][tn], 0, 0, 0);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f32x4 a[TM], b[TN];
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        int row = arow0 + tm * 32 + r;
        a[tm] = *reinterpret_cast<const f32x4*>(As + row * ROWB + TR::swz(row, 4 * h + j) * 16);
      }
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        int row = brow0 + tn * 32 + r;
        b[tn] = *reinterpret_cast<const f32x4*>(Bs + row * ROWB + TR::swz(row, 4 * h + j) * 16);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
          for (int tn = 0; tn < TN; ++tn)
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[tm][e], b[tn][e], acc[tm][tn], 0, 0, 0);
    }
  }
}

// Build per-(n, channel) GroupNorm scale/shift in LDS: A = relu(x * sc + sh).
__device__ __forceinline__ void build_gn_table(float* sc, float* sh, int cin, int groups, const float* stats,
                                               const float* gamma, const float* beta, int n) {
  const int cpg = cin / groups;
  for (int c = threadIdx.x; c < cin; c += blockDim.x) {
    int g = c / cpg;
    float mean = stats[(n * groups + g) * 2], rstd = stats[(n * groups + g) * 2 + 1];
    float s = rstd * gamma[c];
    sc[c] = s;
    sh[c] = beta[c] - mean * s;
  }
}

// ------------------------------------------------------------------------------------------------
// forward / dgrad implicit GEMM
// grid: x = M tiles over the per-sample iteration grid, y = N tiles, z = sample
template <typename T, typename TO, int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(NTHR) void igemm_kernel(const T* __restrict__ x, const T* __restrict__ wpk,
                                                     TO* __restrict__ y, const T* __restrict__ res,
                                                     const float* __restrict__ bias, const float* __restrict__ gstat,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     Geom g) {
  using TR = MfmaTraits<T>;
  constexpr int NCH = TR::NCH;
  constexpr int VEC = 16 / sizeof(T);
  constexpr int ROWB = BK * sizeof(T);
  constexpr int A_LOADS = BM * NCH / NTHR;
  constexpr int B_CH = BN * NCH;
  constexpr int B_LOADS = (B_CH + NTHR - 1) / NTHR;
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  static_assert(A_LOADS >= 1 && WM * WN == 4, "tile");

  __shared__ __attribute__((aligned(16))) char smem[2 * (BM + BN) * ROWB];
  __shared__ float gsc[256], gsh[256];
  auto As = [&](int b) -> char* { return smem + b * (BM * ROWB); };
  auto Bs = [&](int b) -> char* { return smem + 2 * BM * ROWB + b * (BN * ROWB); };

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = blockIdx.z / g.nsplit, split = blockIdx.z % g.nsplit;
  const int bm0 = blockIdx.x * BM, bn0 = blockIdx.y * BN;
  const int Mq = g.qd * g.qh * g.qw;
  const bool has_gn = gstat != nullptr;
  if (has_gn) build_gn_table(gsc, gsh, g.cin, g.gn_groups, gstat, gamma, beta, n);

  const T* xn = x + (long long)n * g.id * g.ih * g.iw * g.cin;

  // per-thread A rows (fixed over the K loop)
  int a_row[A_LOADS], a_ch[A_LOADS], a_bd[A_LOADS], a_bh[A_LOADS], a_bw[A_LOADS];
#pragma unroll
  for (int i = 0; i < A_LOADS; ++i) {
    int id = tid + i * NTHR;
    a_row[i] = id / NCH;
    a_ch[i] = id % NCH;
    int q = bm0 + a_row[i];
    if (q < Mq) {
      int qw_ = q % g.qw, t = q / g.qw;
      int qh_ = t % g.qh, qd_ = t / g.qh;
      a_bd[i] = qd_ * g.si;
      a_bh[i] = qh_ * g.si;
      a_bw[i] = qw_ * g.si;
    } else {
      a_bd[i] = -100000;  // forces out-of-range
      a_bh[i] = 0;
      a_bw[i] = 0;
    }
  }

  const int nchunks = g.cin_p / BK;
  const int nk = g.ntaps * nchunks;

  float ra[A_LOADS][VEC];
  float rb[B_LOADS][VEC];
  bool av[A_LOADS];

  auto gload = [&](int kk) {
    const int t = kk / nchunks, c0 = (kk - t * nchunks) * BK;
    const int dd = g.tap_d[t], dh = g.tap_h[t], dw = g.tap_x[t];
#pragma unroll
    for (int i = 0; i < A_LOADS; ++i) {
      int zd = a_bd[i] + dd, zh = a_bh[i] + dh, zw = a_bw[i] + dw;
      int c = c0 + a_ch[i] * VEC;
      bool ok = (unsigned)zd < (unsigned)g.id && (unsigned)zh < (unsigned)g.ih && (unsigned)zw < (unsigned)g.iw &&
                c < g.cin;
      av[i] = ok;
      if (ok) {
        load16<T>(xn + ((long long)(zd * g.ih + zh) * g.iw + zw) * g.cin + c, ra[i]);
      } else {
#pragma unroll
        for (int e = 0; e < VEC; ++e) ra[i][e] = 0.f;
      }
    }
    const T* wt = wpk + (long long)g.tap_w[t] * g.cout_p * g.cin_p;
#pragma unroll
    for (int i = 0; i < B_LOADS; ++i) {
      int id = tid + i * NTHR;
      if (B_CH % NTHR == 0 || id < B_CH) {
        int row = id / NCH, ch = id % NCH;
        int co = bn0 + row;
        if (co < g.cout_p) {
          load16<T>(wt + (long long)co * g.cin_p + c0 + ch * VEC, rb[i]);
        } else {
#pragma unroll
          for (int e = 0; e < VEC; ++e) rb[i][e] = 0.f;
        }
      }
    }
  };
  auto swrite = [&](int kk, int buf) {
    const int t = kk / nchunks, c0 = (kk - t * nchunks) * BK;
    (void)t;
#pragma unroll
    for (int i = 0; i < A_LOADS; ++i) {
      if (has_gn && av[i]) {
        int c = c0 + a_ch[i] * VEC;
#pragma unroll
        for (int e = 0; e < VEC; ++e) ra[i][e] = fmaxf(0.f, fmaf(ra[i][e], gsc[c + e], gsh[c + e]));
      }
      store16<T>(reinterpret_cast<T*>(As(buf) + a_row[i] * ROWB + TR::swz(a_row[i], a_ch[i]) * 16), ra[i]);
    }
#pragma unroll
    for (int i = 0; i < B_LOADS; ++i) {
      int id = tid + i * NTHR;
      if (B_CH % NTHR == 0 || id < B_CH) {
        int row = id / NCH, ch = id % NCH;
        store16<T>(reinterpret_cast<T*>(Bs(buf) + row * ROWB + TR::swz(row, ch) * 16), rb[i]);
      }
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm)
#pragma unroll
    for (int tn = 0; tn < TN; ++tn)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[tm][tn][e] = 0.f;

  const int wr = wave / WN, wc = wave % WN;
  const int arow0 = wr * (BM / WM), brow0 = wc * (BN / WN);

  // split-K: this block covers K-steps [kk0, kk1)
  const int kk0 = split * g.kps, kk1 = min(nk, kk0 + g.kps);
  __syncthreads();  // gn table
  if (kk0 < kk1) {
    gload(kk0);
    swrite(kk0, 0);
  }
  __syncthreads();
  for (int kk = kk0; kk < kk1; ++kk) {
    const int cur = (kk - kk0) & 1;
    if (kk + 1 < kk1) gload(kk + 1);
    mfma_step<T, TM, TN>(As(cur), Bs(cur), arow0, brow0, lane, acc);
    if (kk + 1 < kk1) swrite(kk + 1, cur ^ 1);
    __syncthreads();
  }

  // epilogue: lane holds column co = lane&31, rows (reg&3) + 8*(reg>>2) + 4*(lane>>5)
  const int r = lane & 31, h = lane >> 5;
  const long long out_n = (long long)n * g.od * g.oh * g.ow;
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) {
    const int co = bn0 + brow0 + tn * 32 + r;
    if (co >= g.cout) continue;
    const float bv = bias ? bias[co] : 0.f;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int q = bm0 + arow0 + tm * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
        if (q >= Mq) continue;
        if (g.nsplit > 1) {  // fp32 partial slab [split][n][q][cout]; reduce kernel applies the epilogue
          g.slab[(((long long)split * g.nsamp + n) * Mq + q) * g.cout + co] = acc[tm][tn][i];
          continue;
        }
        long long ov;
        if (g.so == 1) {
          ov = q;
        } else {
          int qw_ = q % g.qw, t = q / g.qw;
          int qh_ = t % g.qh, qd_ = t / g.qh;
          ov = ((long long)(qd_ * g.so + g.pod) * g.oh + (qh_ * g.so + g.poh)) * g.ow + (qw_ * g.so + g.pow_);
        }
        const long long off = (out_n + ov) * g.cout + co;
        float v = acc[tm][tn][i] + bv;
        if (res) v += to_f(res[off]);
        y[off] = from_f<TO>(v);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// bf16 implicit GEMM with a D-deep register pipeline: the raw 16-B global loads of K-step kk+D are
// issued while step kk runs on the MFMAs, so a step costs its MFMA/LDS time instead of one global-load
// latency (the deep 12^3 / 6^3 layers have only 4 MFMAs per wave per K-step). Same tap-list geometry,
// split-K slabs and epilogue as igemm_kernel; GroupNorm+ReLU is applied when a stage is written to LDS.
template <int KC>
__device__ __forceinline__ int kswz(int r, int c) {  // conflict-free ds_read_b128 for 64-B / 128-B rows
  if constexpr (KC == 4) return c ^ ((r >> 2) & 3);
  else return c ^ ((r >> 1) & 7);
}

template <typename TO, int BM, int BN, int WM, int WN, int KC>
__global__ __launch_bounds__(NTHR) void igemm_bf16_kernel(const bf16* __restrict__ x, const bf16* __restrict__ wpk,
                                                          TO* __restrict__ y, const bf16* __restrict__ res,
                                                          const float* __restrict__ bias,
                                                          const float* __restrict__ gstat,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, Geom g) {
#ifndef U3D_IGEMM_D4
#define U3D_IGEMM_D4 3
#endif
#ifndef U3D_IGEMM_D8
#define U3D_IGEMM_D8 2
#endif
  // register pipeline depth (K-steps of global loads in flight); -DU3D_IGEMM_D4 / _D8 override (diagnostic builds)
  constexpr int NCH = KC, ROWB = KC * 16, BKC = KC * 8, D = KC == 4 ? U3D_IGEMM_D4 : U3D_IGEMM_D8;
  constexpr int A_LOADS = BM * NCH / NTHR;
  constexpr int B_CH = BN * NCH;
  constexpr int B_LOADS = (B_CH + NTHR - 1) / NTHR;
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  static_assert(A_LOADS >= 1 && WM * WN == 4, "tile");

  __shared__ __attribute__((aligned(16))) char smem[2 * (BM + BN) * ROWB + 2 * 256 * 4 + 27 * 24];
  float* gsc = reinterpret_cast<float*>(smem + 2 * (BM + BN) * ROWB);
  float* gsh = gsc + 256;
  // tap table in LDS (the kernarg copy is only reachable through dependent vector loads):
  // [t*2] voxel delta, [t*2+1] packed-weight tap; tdhw[t*4 + 0..2] = (d, h, w) offsets
  int* taps = reinterpret_cast<int*>(gsh + 256);
  int* tdhw = taps + 27 * 2;
  if (threadIdx.x < g.ntaps) {
    const int td = g.tap_d[threadIdx.x], th = g.tap_h[threadIdx.x], tx = g.tap_x[threadIdx.x];
    taps[threadIdx.x * 2] = (td * g.ih + th) * g.iw + tx;
    taps[threadIdx.x * 2 + 1] = g.tap_w[threadIdx.x];
    tdhw[threadIdx.x * 4] = td;
    tdhw[threadIdx.x * 4 + 1] = th;
    tdhw[threadIdx.x * 4 + 2] = tx;
  }
  __syncthreads();
  auto As = [&](int b) -> char* { return smem + b * (BM * ROWB); };
  auto Bs = [&](int b) -> char* { return smem + 2 * BM * ROWB + b * (BN * ROWB); };

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // 1-D grid, XCD-aware: launch id L runs on XCD L % 8; remap so each XCD owns a contiguous range of
  // work items ordered split-major -> the WGs of one XCD share one K slice (weights + activation taps
  // stay in that XCD's L2 instead of every XCD streaming the whole weight tensor).
  int wi;
  {
    const int nwg = gridDim.x, q8 = nwg >> 3, r8 = nwg & 7, xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
    wi = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
  }
  const int tiles = g.mtiles * g.ntiles * g.nsamp;
  const int split = wi / tiles, trem = wi - split * tiles;
  const int n = trem / (g.mtiles * g.ntiles), mn = trem - n * (g.mtiles * g.ntiles);
  const int bm0 = (mn % g.mtiles) * BM, bn0 = (mn / g.mtiles) * BN;
  const int Mq = g.qd * g.qh * g.qw;
  const bool has_gn = gstat != nullptr;
  if (has_gn) build_gn_table(gsc, gsh, g.cin, g.gn_groups, gstat, gamma, beta, n);
  const bf16* xn = x + (long long)n * g.id * g.ih * g.iw * g.cin;

  // per A row: voxel index of the tap-origin and a bit mask of the taps that land inside the volume, so a
  // K-step costs one LDS broadcast + a shift/test + one multiply-add per load (the step was VALU-bound)
  int a_row[A_LOADS], a_ch[A_LOADS], a_base[A_LOADS];
  unsigned a_mask[A_LOADS];
#pragma unroll
  for (int i = 0; i < A_LOADS; ++i) {
    const int id = tid + i * NTHR;
    a_row[i] = id / NCH;
    a_ch[i] = id % NCH;
    const int q = bm0 + a_row[i];
    unsigned m = 0;
    int base = 0;
    if (q < Mq) {
      const int qw_ = q % g.qw, t = q / g.qw;
      const int bd = (t / g.qh) * g.si, bh = (t % g.qh) * g.si, bw = qw_ * g.si;
      base = (bd * g.ih + bh) * g.iw + bw;
      for (int tt = 0; tt < g.ntaps; ++tt) {
        const int zd = bd + tdhw[tt * 4], zh = bh + tdhw[tt * 4 + 1], zw = bw + tdhw[tt * 4 + 2];
        if ((unsigned)zd < (unsigned)g.id && (unsigned)zh < (unsigned)g.ih && (unsigned)zw < (unsigned)g.iw)
          m |= 1u << tt;
      }
    }
    a_base[i] = base;
    a_mask[i] = m;
  }
  const int nchunks = g.cin_p / BKC;
  const int nk = g.ntaps * nchunks;

  u32x4 ra[D][A_LOADS], rb[D][B_LOADS];
  unsigned am[D];
  // every load is issued unconditionally (out-of-range lanes read a valid dummy address and are zeroed
  // afterwards): the loads in flight are then static, so the compiler's vmcnt waits stay counted.
  auto gload = [&](int kk, int slot) {
    const int t = kk / nchunks, c0 = (kk - t * nchunks) * BKC;
    const int delta = taps[t * 2];
    unsigned m = 0;
#pragma unroll
    for (int i = 0; i < A_LOADS; ++i) {
      const int c = c0 + a_ch[i] * 8;
      const bool ok = ((a_mask[i] >> t) & 1u) && c < g.cin;
      const int off = ok ? (a_base[i] + delta) * g.cin + c : 0;
      ra[slot][i] = *reinterpret_cast<const u32x4*>(xn + off);
      m |= ok ? 1u << i : 0u;
    }
    am[slot] = m;
    const bf16* wt = wpk + (long long)taps[t * 2 + 1] * g.cout_p * g.cin_p;
#pragma unroll
    for (int i = 0; i < B_LOADS; ++i) {
      const int id = min(tid + i * NTHR, B_CH - 1);
      const int row = id / NCH, ch = id % NCH, co = min(bn0 + row, g.cout_p - 1);
      rb[slot][i] = *reinterpret_cast<const u32x4*>(wt + co * g.cin_p + c0 + ch * 8);
    }
  };
  auto swrite = [&](int kk, int slot, int buf) {
    const int t = kk / nchunks, c0 = (kk - t * nchunks) * BKC;
#pragma unroll
    for (int i = 0; i < A_LOADS; ++i) {
      u32x4 v = ra[slot][i];
      const bool ok = (am[slot] >> i) & 1u;
      if (!ok) v = u32x4{0u, 0u, 0u, 0u};
      if (has_gn && ok) {
        const int c = c0 + a_ch[i] * 8;
        f32x2 sc[4], sh[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          sc[e] = f32x2{gsc[c + 2 * e], gsc[c + 2 * e + 1]};
          sh[e] = f32x2{gsh[c + 2 * e], gsh[c + 2 * e + 1]};
        }
        v = gn_relu8(v, sc, sh);
      }
      *reinterpret_cast<u32x4*>(As(buf) + a_row[i] * ROWB + kswz<KC>(a_row[i], a_ch[i]) * 16) = v;
    }
#pragma unroll
    for (int i = 0; i < B_LOADS; ++i) {
      const int id = tid + i * NTHR;
      if (B_CH % NTHR == 0 || id < B_CH) {
        const int row = id / NCH, ch = id % NCH;
        u32x4 v = rb[slot][i];
        if (bn0 + row >= g.cout_p) v = u32x4{0u, 0u, 0u, 0u};
        *reinterpret_cast<u32x4*>(Bs(buf) + row * ROWB + kswz<KC>(row, ch) * 16) = v;
      }
    }
  };

  const int wr = wave / WN, wc = wave % WN;
  const int arow0 = wr * (BM / WM), brow0 = wc * (BN / WN);
  f32x16 acc[TM][TN];
  auto stage_mfma = [&](const char* Ab, const char* Bb) {
    const int r = lane & 31, h = lane >> 5;
#pragma unroll
    for (int s = 0; s < KC / 2; ++s) {
      bf16x8 av[TM], bv[TN];
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const int row = arow0 + tm * 32 + r;
        av[tm] = *reinterpret_cast<const bf16x8*>(Ab + row * ROWB + kswz<KC>(row, 2 * s + h) * 16);
      }
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int row = brow0 + tn * 32 + r;
        bv[tn] = *reinterpret_cast<const bf16x8*>(Bb + row * ROWB + kswz<KC>(row, 2 * s + h) * 16);
      }
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[tm], bv[tn], acc[tm][tn], 0, 0, 0);
    }
  };
#pragma unroll
  for (int tm = 0; tm < TM; ++tm)
#pragma unroll
    for (int tn = 0; tn < TN; ++tn)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[tm][tn][e] = 0.f;

  const int kk0 = split * g.kps, kk1 = min(nk, kk0 + g.kps);
  __syncthreads();  // GN + tap tables
  if (kk0 < kk1) {
#pragma unroll
    for (int j = 0; j < D; ++j) gload(min(kk0 + j, kk1 - 1), j);
    swrite(kk0, 0, 0);
  }
  __syncthreads();
  // stage kk lives in register slot (kk - kk0) % D and LDS buffer (kk - kk0) & 1
  int kk = kk0;
  for (; kk + D < kk1; kk += D) {  // full groups: no conditional memory operations inside
#pragma unroll
    for (int j = 0; j < D; ++j) {
      gload(min(kk + j + D, kk1 - 1), j);  // slot j held stage kk+j, already in LDS
      const int buf = (kk + j - kk0) & 1;
      stage_mfma(As(buf), Bs(buf));
      swrite(kk + j + 1, (j + 1) % D, buf ^ 1);
      __syncthreads();
    }
  }
#pragma unroll
  for (int j = 0; j < D; ++j) {  // tail: the last 1..D stages
    if (kk + j < kk1) {
      const int buf = (kk + j - kk0) & 1;
      stage_mfma(As(buf), Bs(buf));
      if (kk + j + 1 < kk1) swrite(kk + j + 1, (j + 1) % D, buf ^ 1);
      __syncthreads();
    }
  }

  const int r = lane & 31, h = lane >> 5;
  const long long out_n = (long long)n * g.od * g.oh * g.ow;
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) {
    const int co = bn0 + brow0 + tn * 32 + r;
    if (co >= g.cout) continue;
    const float bv = bias ? bias[co] : 0.f;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int q = bm0 + arow0 + tm * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
        if (q >= Mq) continue;
        if (g.nsplit > 1) {
          g.slab[(((long long)split * g.nsamp + n) * Mq + q) * g.cout + co] = acc[tm][tn][i];
          continue;
        }
        long long ov;
        if (g.so == 1) {
          ov = q;
        } else {
          const int qw_ = q % g.qw, t = q / g.qw;
          const int qh_ = t % g.qh, qd_ = t / g.qh;
          ov = ((long long)(qd_ * g.so + g.pod) * g.oh + (qh_ * g.so + g.poh)) * g.ow + (qw_ * g.so + g.pow_);
        }
        const long long off = (out_n + ov) * g.cout + co;
        float v = acc[tm][tn][i] + bv;
        if (res) v += to_f(res[off]);
        y[off] = from_f<TO>(v);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// weight gradient: partial[s][t][co][ci] = sum_{vox in split s} dy[vox][co] * A[vox*si + off_t][ci]
// One workgroup = (co tile 32, ci tile 32, up to 4 taps) over one voxel split: the dy tile is staged
// once per K-step and shared by the 4 waves, each wave owning one tap's 32x32 accumulator.
// bf16 operands are stored transposed in LDS ([channel][voxel], k = voxel contiguous) so that the
// MFMA fragment (8 consecutive voxels of one channel) is one 16-B read; f32 keeps [voxel][channel].
template <typename T>
__global__ __launch_bounds__(NTHR) void wgrad_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                     const float* __restrict__ gstat, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, float* __restrict__ part,
                                                     Geom g, int n_samples, long long vox_per_split) {
  constexpr int KV = 32;  // voxels per K-step
  constexpr int VEC = 16 / sizeof(T);
  constexpr int CH = 32 / VEC;            // 16-B chunks per 32-channel row
  constexpr int NLD = KV * CH;             // 16-B chunks per operand tile (128 bf16, 256 f32)
  constexpr int LOADS = (NLD + NTHR - 1) / NTHR;
  constexpr int TILE_B = 32 * 32 * sizeof(T);
  static_assert(NLD <= NTHR * LOADS, "wgrad tile");
  using TR = MfmaTraits<T>;

  __shared__ __attribute__((aligned(16))) char smem[5 * TILE_B];  // dy + 4 tap tiles
  __shared__ float gsc[256], gsh[256];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ci0 = blockIdx.x * 32, co0 = blockIdx.y * 32;
  const int tgroups = (g.ntaps + 3) / 4;
  const int tg = blockIdx.z % tgroups, split = blockIdx.z / tgroups;
  const int t0 = tg * 4;
  const int ntl = min(4, g.ntaps - t0);
  const int Mq = g.qd * g.qh * g.qw;
  const long long Mtot = (long long)n_samples * Mq;
  const long long v0 = split * vox_per_split;
  const long long v1 = min(Mtot, v0 + vox_per_split);
  const bool has_gn = gstat != nullptr;

  f32x16 acc;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.f;

  int cur_gn_n = -1;
  float rdy[LOADS][VEC], rx[4][LOADS][VEC];

  for (long long vb = v0; vb < v1; vb += KV) {
    // samples can change inside a split: rebuild the GroupNorm table when the block's first voxel does
    if (has_gn) {
      int nfirst = (int)(vb / Mq);
      int nlast = (int)(min(v1, vb + KV) - 1) / Mq;
      if (nfirst != cur_gn_n || nlast != nfirst) {
        // rare: tile straddles samples -> table per voxel handled below via n check; keep first sample table
        __syncthreads();
        build_gn_table(gsc, gsh, g.cin, g.gn_groups, gstat, gamma, beta, nfirst);
        cur_gn_n = nfirst;
        __syncthreads();
      }
    }
#pragma unroll
    for (int i = 0; i < LOADS; ++i) {
      int id = tid + i * NTHR;
      if (NLD % NTHR != 0 && id >= NLD) continue;
      int vr = id / CH, ch = id % CH;
      long long v = vb + vr;
      // dy tile: [KV][32 co]
      if (v < v1 && co0 + ch * VEC < g.cout) {
        load16<T>(dy + v * g.cout + co0 + ch * VEC, rdy[i]);
      } else {
#pragma unroll
        for (int e = 0; e < VEC; ++e) rdy[i][e] = 0.f;
      }
      int nn = 0, qd_ = 0, qh_ = 0, qw_ = 0;
      if (v < v1) {
        nn = (int)(v / Mq);
        int q = (int)(v - (long long)nn * Mq);
        qw_ = q % g.qw;
        int t = q / g.qw;
        qh_ = t % g.qh;
        qd_ = t / g.qh;
      }
      const int c = ci0 + ch * VEC;
#pragma unroll
      for (int tl = 0; tl < 4; ++tl) {
        bool ok = false;
        if (tl < ntl && v < v1 && c < g.cin) {
          int t = t0 + tl;
          int zd = qd_ * g.si + g.tap_d[t], zh = qh_ * g.si + g.tap_h[t], zw = qw_ * g.si + g.tap_x[t];
          ok = (unsigned)zd < (unsigned)g.id && (unsigned)zh < (unsigned)g.ih && (unsigned)zw < (unsigned)g.iw;
          if (ok) {
            load16<T>(x + (((long long)nn * g.id + zd) * g.ih * g.iw + (long long)zh * g.iw + zw) * g.cin + c,
                      rx[tl][i]);
            if (has_gn) {
              if (nn == cur_gn_n) {
#pragma unroll
                for (int e = 0; e < VEC; ++e) rx[tl][i][e] = fmaxf(0.f, fmaf(rx[tl][i][e], gsc[c + e], gsh[c + e]));
              } else {  // straddling tile: compute the affine from global stats directly
                const int cpg = g.cin / g.gn_groups;
#pragma unroll
                for (int e = 0; e < VEC; ++e) {
                  int gg = (c + e) / cpg;
                  float mean = gstat[(nn * g.gn_groups + gg) * 2], rstd = gstat[(nn * g.gn_groups + gg) * 2 + 1];
                  float s = rstd * gamma[c + e];
                  rx[tl][i][e] = fmaxf(0.f, fmaf(rx[tl][i][e], s, beta[c + e] - mean * s));
                }
              }
            }
          }
        }
        if (!ok) {
#pragma unroll
          for (int e = 0; e < VEC; ++e) rx[tl][i][e] = 0.f;
        }
      }
    }
    __syncthreads();  // previous step's reads done
    // stage to LDS
#pragma unroll
    for (int i = 0; i < LOADS; ++i) {
      int id = tid + i * NTHR;
      if (NLD % NTHR != 0 && id >= NLD) continue;
      int vr = id / CH, ch = id % CH;
      if constexpr (sizeof(T) == 2) {
        // transposed [c][v]: element (c = ch*8+e, v = vr) -> row c, chunk vr/8, elem vr%8
        bf16* d0 = reinterpret_cast<bf16*>(smem);
#pragma unroll
        for (int e = 0; e < VEC; ++e) {
          int row = ch * VEC + e;
          d0[row * 32 + TR::swz(row, vr >> 3) * 8 + (vr & 7)] = from_f<bf16>(rdy[i][e]);
        }
#pragma unroll
        for (int tl = 0; tl < 4; ++tl) {
          bf16* dt = reinterpret_cast<bf16*>(smem + (1 + tl) * TILE_B);
#pragma unroll
          for (int e = 0; e < VEC; ++e) {
            int row = ch * VEC + e;
            dt[row * 32 + TR::swz(row, vr >> 3) * 8 + (vr & 7)] = from_f<bf16>(rx[tl][i][e]);
          }
        }
      } else {
        // natural [v][c], fp32
        float* d0 = reinterpret_cast<float*>(smem);
        *reinterpret_cast<f32x4*>(d0 + vr * 32 + ch * 4) = f32x4{rdy[i][0], rdy[i][1], rdy[i][2], rdy[i][3]};
#pragma unroll
        for (int tl = 0; tl < 4; ++tl) {
          float* dt = reinterpret_cast<float*>(smem + (1 + tl) * TILE_B);
          *reinterpret_cast<f32x4*>(dt + vr * 32 + ch * 4) =
              f32x4{rx[tl][i][0], rx[tl][i][1], rx[tl][i][2], rx[tl][i][3]};
        }
      }
    }
    __syncthreads();
    if (wave < ntl) {
      const int r = lane & 31, h = lane >> 5;
      const char* At = smem;                       // dy^T : A[co][vox]
      const char* Bt = smem + (1 + wave) * TILE_B; // act  : B[vox][ci] (stored [ci][vox] for bf16)
      if constexpr (sizeof(T) == 2) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          bf16x8 a = *reinterpret_cast<const bf16x8*>(At + r * 64 + TR::swz(r, 2 * s + h) * 16);
          bf16x8 b = *reinterpret_cast<const bf16x8*>(Bt + r * 64 + TR::swz(r, 2 * s + h) * 16);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
        }
      } else {
        const float* Af = reinterpret_cast<const float*>(At);
        const float* Bf = reinterpret_cast<const float*>(Bt);
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          int vv = 16 * h + e;
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(Af[vv * 32 + r], Bf[vv * 32 + r], acc, 0, 0, 0);
        }
      }
    }
  }
  // store partial: D[row = co][col = ci]: lane col = ci0 + (lane&31), rows co = (i&3)+8(i>>2)+4h
  if (wave < ntl) {
    const int r = lane & 31, h = lane >> 5;
    const int t = g.tap_w[t0 + wave];
    float* p = part + ((long long)split * g.ntaps + t) * g.cout_p * g.cin_p;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      int co = co0 + (i & 3) + 8 * (i >> 2) + 4 * h;
      p[(long long)co * g.cin_p + ci0 + r] = acc[i];
    }
  }
}

// ------------------------------------------------------------------------------------------------
static void fill_taps(Geom& g, int ksize, bool transpose) {
  int p = ksize / 2, t = 0;
  for (int a = 0; a < ksize; ++a)
    for (int b = 0; b < ksize; ++b)
      for (int c = 0; c < ksize; ++c) {
        g.tap_w[t] = (a * ksize + b) * ksize + c;
        g.tap_d[t] = transpose ? p - a : a - p;
        g.tap_h[t] = transpose ? p - b : b - p;
        g.tap_x[t] = transpose ? p - c : c - p;
        ++t;
      }
  g.ntaps = t;
}

// split-K epilogue: y[map(n, q)][co] = sum_s slab[s][n][q][co] (+ bias) (+ residual)
template <typename T, typename TO>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(Geom g, const T* __restrict__ res,
                                                           const float* __restrict__ bias, TO* __restrict__ y) {
  const int Mq = g.qd * g.qh * g.qw;
  const long long per = (long long)g.nsamp * Mq * g.cout;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < per; i += (long long)gridDim.x * 256) {
    const int co = (int)(i % g.cout);
    const long long nq = i / g.cout;
    const int q = (int)(nq % Mq), n = (int)(nq / Mq);
    float v = bias ? bias[co] : 0.f;
    for (int s = 0; s < g.nsplit; ++s) v += g.slab[s * per + i];
    long long ov;
    if (g.so == 1) {
      ov = q;
    } else {
      int qw_ = q % g.qw, t = q / g.qw;
      int qh_ = t % g.qh, qd_ = t / g.qh;
      ov = ((long long)(qd_ * g.so + g.pod) * g.oh + (qh_ * g.so + g.poh)) * g.ow + (qw_ * g.so + g.pow_);
    }
    const long long off = ((long long)n * g.od * g.oh * g.ow + ov) * g.cout + co;
    if (res) v += to_f(res[off]);
    y[off] = from_f<TO>(v);
  }
}

template <typename T, typename TO>
static int launch_igemm(Geom g, int n, const T* x, const T* wpk, TO* y, const T* res, const float* bias,
                        const float* st, const float* ga, const float* be, float* ws, long long ws_bytes,
                        hipStream_t s) {
  const int Mq = g.qd * g.qh * g.qw;
  if (Mq <= 0) return U3D_OK;
  const int env_bn = opt(OPT_IGEMM_BN), env_ns = opt(OPT_IGEMM_NS), env_target = opt(OPT_IGEMM_TARGET);
  int BN = g.cout_p <= 32 ? 32 : (sizeof(T) == 2 && g.cout_p >= 128) ? 128 : 64;
  const bool auto_bn = opt(OPT_IGEMM_AUTO) != 0;
  if (sizeof(T) == 2 && auto_bn) {
    // too few output tiles to fill the CUs: narrower N tiles before splitting K (measured, tools/igemm_sweep.sh:
    // 48^3 64->128 s2 91 -> 66 us at BN 64, 12^3 256->256 s2 50 -> 37 us at BN 32)
    auto ntile = [&](int bn) { return (long long)cdiv(Mq, 128) * cdiv(g.cout, bn) * n; };
    if (BN > 32 && ntile(BN) < 256) BN /= 2;
    if (BN > 32 && ntile(BN) < 64) BN /= 2;
  }
  if (env_bn && sizeof(T) == 2 && env_bn <= g.cout_p) BN = env_bn;  // experiments
  const long long tiles = (long long)cdiv(Mq, 128) * cdiv(g.cout, BN) * n;
  const int nk = g.ntaps * (g.cin_p / BK);
  // split K when the output tiles cannot fill the 256 CUs (deep, small-volume layers)
  int ns = 1;
  if (ws && tiles < 256 && nk >= 8) {
    ns = (int)std::min<long long>(nk / 4, (env_target + tiles - 1) / tiles);
    if (env_ns > 0) ns = std::min(env_ns, nk);
    if (sizeof(T) == 2 && ns > 8) ns = ns / 8 * 8;  // split-major XCD mapping: one K slice per XCD
    const long long slab1 = (long long)n * Mq * g.cout * 4;
    while (ns > 1 && ns * slab1 > ws_bytes) --ns;
  }
  g.nsamp = n;
  g.nsplit = ns;
  g.kps = (nk + ns - 1) / ns;
  g.slab = ns > 1 ? ws : nullptr;
  if constexpr (sizeof(T) == 2) {
    // 256-row M tiles (8 MFMAs per wave per K step instead of 4: half the barriers and LDS stage writes per flop) for
    // large unsplit BN = 64 launches (the stride-2 layer-1/2 forwards), IGEMM_BM = 128 / 256 forces (A/B)
    const int env_bm = opt(OPT_IGEMM_BM);
    const bool bm256 = BN == 64 && ns == 1 && (env_bm == 256 || (env_bm == 0 && (long long)cdiv(Mq, 256) *
                                                                                 cdiv(g.cout, 64) * n >= 256));
    g.mtiles = cdiv(Mq, bm256 ? 256 : 128);
    g.ntiles = cdiv(g.cout, BN);
    if (g.cin_p % 64 == 0) {  // 64-channel stages: twice the MFMAs per barrier
      g.kps = (g.ntaps * (g.cin_p / 64) + ns - 1) / ns;
      g.nsplit = ns = std::min(ns, g.ntaps * (g.cin_p / 64));
    }
    dim3 grid(g.mtiles * g.ntiles * n * ns);
    const bool k64 = g.cin_p % 64 == 0;
    if (BN == 32) {
      if (k64)
        hipLaunchKernelGGL((igemm_bf16_kernel<TO, 128, 32, 4, 1, 8>), grid, dim3(NTHR), 0, s, x, wpk, y, res, bias, st,
                           ga, be, g);
      else
        hipLaunchKernelGGL((igemm_bf16_kernel<TO, 128, 32, 4, 1, 4>), grid, dim3(NTHR), 0, s, x, wpk, y, res, bias, st,
                           ga, be, g);
    } else if (BN == 64 && bm256) {
      if (k64)
        hipLaunchKernelGGL((igemm_bf16_kernel<TO, 256, 64, 2, 2, 8>), grid, dim3(NTHR), 0, s, x, wpk, y, res, bias, st,
                           ga, be, g);
      else
        hipLaunchKernelGGL((igemm_bf16_kernel<TO, 256, 64, 2, 2, 4>), grid, dim3(NTHR), 0, s, x, wpk, y, res, bias, st,
                           ga, be, g);
    } else if (BN == 64) {
      if (k64)
        hipLaunchKernelGGL((igemm_bf16_kernel<TO, 128, 64, 2, 2, 8>), grid, dim3(NTHR), 0, s, x, wpk, y, res, bias, st,
                           ga, be, g);
      else
        hipLaunchKernelGGL((igemm_bf16_kernel<TO, 128, 64, 2, 2, 4>), grid, dim3(NTHR), 0, s, x, wpk, y, res, bias, st,
                           ga, be, g);
    } else {
      if (k64)
        hipLaunchKernelGGL((igemm_bf16_kernel<TO, 128, 128, 2, 2, 8>), grid, dim3(NTHR), 0, s, x, wpk, y, res, bias,
                           st, ga, be, g);
      else
        hipLaunchKernelGGL((igemm_bf16_kernel<TO, 128, 128, 2, 2, 4>), grid, dim3(NTHR), 0, s, x, wpk, y, res, bias,
                           st, ga, be, g);
    }
  } else if (BN == 32) {
    dim3 grid(cdiv(Mq, 128), cdiv(g.cout, 32), n * ns);
    hipLaunchKernelGGL((igemm_kernel<T, TO, 128, 32, 4, 1>), grid, dim3(NTHR), 0, s, x, wpk, y, res, bias, st, ga,
                       be, g);
  } else {
    dim3 grid(cdiv(Mq, 128), cdiv(g.cout, 64), n * ns);
    hipLaunchKernelGGL((igemm_kernel<T, TO, 128, 64, 2, 2>), grid, dim3(NTHR), 0, s, x, wpk, y, res, bias, st, ga,
                       be, g);
  }
  int rc = check_launch("igemm_kernel");
  if (rc || ns == 1) return rc;
  const long long per = (long long)n * Mq * g.cout;
  const int nb = (int)std::min<long long>(4096, (per + 255) / 256);
  hipLaunchKernelGGL((splitk_reduce_kernel<T, TO>), dim3(nb), dim3(256), 0, s, g, res, bias, y);
  return check_launch("splitk_reduce_kernel");
}

static int out_dim(int d, int k, int s) { return (d + 2 * (k / 2) - k) / s + 1; }

}  // namespace u3d

using namespace u3d;

extern "C" int u3d_conv_fwd(int dtype, const void* x, int n, int cin, int d, int h, int w, const void* wpk, int cout,
                            int ksize, int stride, const float* gn_stats, const float* gn_gamma, const float* gn_beta,
                            int gn_groups, const void* residual, const float* bias, void* y, int y_f32,
                            float* ws, long long ws_bytes, u3d_stream_t stream) {
  U3D_REQUIRE(dtype == U3D_F32 || dtype == U3D_BF16, "conv_fwd: bad dtype %d", dtype);
  U3D_REQUIRE(ksize == 1 || ksize == 3, "conv_fwd: ksize %d unsupported", ksize);
  U3D_REQUIRE(stride == 1 || stride == 2, "conv_fwd: stride %d unsupported", stride);
  U3D_REQUIRE(cin % 8 == 0 && cin <= 4096, "conv_fwd: cin %d must be a multiple of 8 (stem: u3d_stem_fwd)", cin);
  U3D_REQUIRE(cout >= 1 && n >= 1 && d >= 1 && h >= 1 && w >= 1, "conv_fwd: bad shape");
  U3D_REQUIRE(x && wpk && y, "conv_fwd: null pointer");
  U3D_REQUIRE(!gn_stats || (gn_gamma && gn_beta && gn_groups > 0 && cin % gn_groups == 0 && cin <= 256),
              "conv_fwd: bad GroupNorm prologue (groups %d, cin %d)", gn_groups, cin);
  U3D_REQUIRE(!(y_f32 && residual), "conv_fwd: residual with fp32 output unsupported");
  Geom g{};
  g.cin = cin;
  g.cout = cout;
  g.cin_p = round_up(cin, 32);
  g.cout_p = round_up(cout, 32);
  g.id = d; g.ih = h; g.iw = w;
  g.od = out_dim(d, ksize, stride); g.oh = out_dim(h, ksize, stride); g.ow = out_dim(w, ksize, stride);
  g.qd = g.od; g.qh = g.oh; g.qw = g.ow;
  g.so = 1; g.pod = g.poh = g.pow_ = 0;
  g.si = stride;
  g.gn_groups = gn_groups;
  fill_taps(g, ksize, false);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == U3D_BF16) {
    if (y_f32)
      return launch_igemm<bf16, float>(g, n, (const bf16*)x, (const bf16*)wpk, (float*)y, nullptr, bias, gn_stats,
                                       gn_gamma, gn_beta, ws, ws_bytes, s);
    return launch_igemm<bf16, bf16>(g, n, (const bf16*)x, (const bf16*)wpk, (bf16*)y, (const bf16*)residual, bias,
                                    gn_stats, gn_gamma, gn_beta, ws, ws_bytes, s);
  }
  return launch_igemm<float, float>(g, n, (const float*)x, (const float*)wpk, (float*)y, (const float*)residual, bias,
                                    gn_stats, gn_gamma, gn_beta, ws, ws_bytes, s);
}

extern "C" int u3d_conv_dgrad(int dtype, const void* dy, int n, int cout, const void* wpk_dgrad, int cin, int d,
                              int h, int w, int ksize, int stride, void* dx, float* ws, long long ws_bytes,
                              u3d_stream_t stream) {
  U3D_REQUIRE(dtype == U3D_F32 || dtype == U3D_BF16, "conv_dgrad: bad dtype %d", dtype);
  U3D_REQUIRE(ksize == 1 || ksize == 3, "conv_dgrad: ksize %d unsupported", ksize);
  U3D_REQUIRE(stride == 1 || stride == 2, "conv_dgrad: stride %d unsupported", stride);
  U3D_REQUIRE(cout % 8 == 0, "conv_dgrad: cout %d must be a multiple of 8", cout);
  U3D_REQUIRE(dy && wpk_dgrad && dx, "conv_dgrad: null pointer");
  U3D_REQUIRE(stride == 1 || (d % 2 == 0 && h % 2 == 0 && w % 2 == 0), "conv_dgrad: stride 2 needs even dims");
  hipStream_t s = (hipStream_t)stream;
  Geom g{};
  g.cin = cout;  // contraction over the forward's output channels
  g.cout = cin;
  g.cin_p = round_up(cout, 32);
  g.cout_p = round_up(cin, 32);
  g.od = d; g.oh = h; g.ow = w;
  const int od = out_dim(d, ksize, stride), oh = out_dim(h, ksize, stride), ow = out_dim(w, ksize, stride);
  g.id = od; g.ih = oh; g.iw = ow;
  g.gn_groups = 0;
  auto run = [&](const Geom& gg) -> int {
    if (dtype == U3D_BF16)
      return launch_igemm<bf16, bf16>(gg, n, (const bf16*)dy, (const bf16*)wpk_dgrad, (bf16*)dx, nullptr, nullptr,
                                      nullptr, nullptr, nullptr, ws, ws_bytes, s);
    return launch_igemm<float, float>(gg, n, (const float*)dy, (const float*)wpk_dgrad, (float*)dx, nullptr, nullptr,
                                      nullptr, nullptr, nullptr, ws, ws_bytes, s);
  };
  if (stride == 1) {
    g.qd = d; g.qh = h; g.qw = w;
    g.so = 1; g.si = 1;
    fill_taps(g, ksize, true);
    return run(g);
  }
  // stride 2: x = 2q + p. ksize 3 (pad 1): p=0 -> tap 1 at y=q; p=1 -> tap 0 at y=q+1, tap 2 at y=q.
  // ksize 1 (pad 0): p=0 -> tap 0 at y=q; p=1 -> no contribution (zero).
  // ksize 1 (pad 0): only the even-parity class gets a contribution; the rest is zero (a streaming memset is as
  // fast as any fused zero-fill: writing the zeros from the GEMM epilogue measured 2.3x slower)
  if (ksize == 1) U3D_HIP(hipMemsetAsync(dx, 0, (size_t)n * d * h * w * cin * (dtype == U3D_BF16 ? 2 : 4), s));
  g.so = 2; g.si = 1;
  g.qd = d / 2; g.qh = h / 2; g.qw = w / 2;
  for (int pd = 0; pd < 2; ++pd)
    for (int ph = 0; ph < 2; ++ph)
      for (int pw = 0; pw < 2; ++pw) {
        int taps1[3][2][2];  // per dim: list of (tap index, offset)
        int cnt[3];
        int par[3] = {pd, ph, pw};
        bool empty = false;
        for (int a = 0; a < 3; ++a) {
          if (ksize == 3) {
            if (par[a] == 0) { taps1[a][0][0] = 1; taps1[a][0][1] = 0; cnt[a] = 1; }
            else { taps1[a][0][0] = 0; taps1[a][0][1] = 1; taps1[a][1][0] = 2; taps1[a][1][1] = 0; cnt[a] = 2; }
          } else {
            if (par[a] == 0) { taps1[a][0][0] = 0; taps1[a][0][1] = 0; cnt[a] = 1; }
            else { cnt[a] = 0; empty = true; }
          }
        }
        if (empty) continue;
        Geom gc = g;
        gc.pod = pd; gc.poh = ph; gc.pow_ = pw;
        int t = 0;
        for (int i = 0; i < cnt[0]; ++i)
          for (int j = 0; j < cnt[1]; ++j)
            for (int k = 0; k < cnt[2]; ++k) {
              gc.tap_w[t] = (taps1[0][i][0] * ksize + taps1[1][j][0]) * ksize + taps1[2][k][0];
              gc.tap_d[t] = taps1[0][i][1];
              gc.tap_h[t] = taps1[1][j][1];
              gc.tap_x[t] = taps1[2][k][1];
              ++t;
            }
        gc.ntaps = t;
        int rc = run(gc);
        if (rc) return rc;
      }
  return U3D_OK;
}

extern "C" int u3d_conv_wgrad_splits(int n, int cin, int d, int h, int w, int cout, int ksize, int stride) {
  const long long M = (long long)n * out_dim(d, ksize, stride) * out_dim(h, ksize, stride) * out_dim(w, ksize, stride);
  const int ntaps = ksize * ksize * ksize;
  const long long tiles = (long long)cdiv(cin, 32) * cdiv(cout, 32) * ((ntaps + 3) / 4);
  long long want = cdiv(2048, tiles);
  long long maxs = std::max(1LL, M / 1024);  // keep >= 1024 voxels per split
  return (int)std::max(1LL, std::min(want, maxs));
}

extern "C" int u3d_conv_wgrad(int dtype, const void* dy, const void* x, int n, int cin, int d, int h, int w, int cout,
                              int ksize, int stride, const float* gn_stats, const float* gn_gamma,
                              const float* gn_beta, int gn_groups, float* partials, int nsplit,
                              u3d_stream_t stream) {
  U3D_REQUIRE(dtype == U3D_F32 || dtype == U3D_BF16, "conv_wgrad: bad dtype %d", dtype);
  U3D_REQUIRE(ksize == 1 || ksize == 3, "conv_wgrad: ksize %d unsupported", ksize);
  U3D_REQUIRE(stride == 1 || stride == 2, "conv_wgrad: stride %d unsupported", stride);
  U3D_REQUIRE(cin % 8 == 0 && cout % 8 == 0, "conv_wgrad: channels must be multiples of 8");
  U3D_REQUIRE(nsplit >= 1, "conv_wgrad: nsplit");
  U3D_REQUIRE(!gn_stats || (gn_gamma && gn_beta && gn_groups > 0 && cin % gn_groups == 0 && cin <= 256),
              "conv_wgrad: bad GroupNorm prologue");
  Geom g{};
  g.cin = cin;
  g.cout = cout;
  g.cin_p = round_up(cin, 32);
  g.cout_p = round_up(cout, 32);
  g.id = d; g.ih = h; g.iw = w;
  g.od = g.qd = out_dim(d, ksize, stride);
  g.oh = g.qh = out_dim(h, ksize, stride);
  g.ow = g.qw = out_dim(w, ksize, stride);
  g.so = 1; g.si = stride;
  g.gn_groups = gn_groups;
  fill_taps(g, ksize, false);
  const long long M = (long long)n * g.qd * g.qh * g.qw;
  long long vps = (M + nsplit - 1) / nsplit;
  vps = (vps + 31) / 32 * 32;
  hipStream_t s = (hipStream_t)stream;
  // every (split, tap, co_p, ci_p) entry is written by exactly one workgroup (zeros in the padding)
  dim3 grid(g.cin_p / 32, g.cout_p / 32, ((g.ntaps + 3) / 4) * nsplit);
  if (dtype == U3D_BF16)
    hipLaunchKernelGGL(wgrad_kernel<bf16>, grid, dim3(NTHR), 0, s, (const bf16*)dy, (const bf16*)x, gn_stats,
                       gn_gamma, gn_beta, partials, g, n, vps);
  else
    hipLaunchKernelGGL(wgrad_kernel<float>, grid, dim3(NTHR), 0, s, (const float*)dy, (const float*)x, gn_stats,
                       gn_gamma, gn_beta, partials, g, n, vps);
  return check_launch("wgrad_kernel");
}
