// Classifier head of the trunk: precls_conv = GroupNorm + ReLU + 1^3 conv (cin -> cout <= 32, + bias) at full
// resolution (reference unet3D.py:1653-1657 / :647-650), forward and data gradient, bf16 activations.
//
// At 96^3 x 2 the head is pure streaming (32 -> 16 channels: 64 B in, 64 B fp32 out per voxel, 1 kFLOP per
// voxel): one wave handles 32 voxels per step with the operands loaded straight from global memory in MFMA
// fragment layout (no LDS), GN+ReLU applied in registers, the weights (B fragments) held in registers for
// the whole grid-stride loop.
//   forward : logits[v][co] = sum_ci relu(gn(x))[v][ci] W[co][ci] + b[co]   (fp32 out, as the reference returns)
//   backward: dA[v][ci] = sum_co dy[v][co] W[co][ci] (bf16), plus dy in bf16 for the weight gradient and the
//             per-block column sums of dy (bias gradient partials) — the fp32 dy is read once.
#include "common.h"
#include "loss_grad.h"

namespace u3d {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;

constexpr int HD_T = 256;  // 4 waves
#ifndef HD_ND
#define HD_ND 2  // head_loss_bwd_kernel: tiles in flight per wave (3, 4: measured equal)
#endif
#ifndef HD_ND_GN
#define HD_ND_GN 2
#endif
constexpr int HD_GMAX = 2048;  // TR forward with GN: n * cin <= HD_GMAX (per-block LDS coefficient table)

__device__ __forceinline__ bf16x8 as_frag(u32x4 v) { return __builtin_bit_cast(bf16x8, v); }

// KS = cin / 16 k-steps (cin in {16, 32, 48, 64})
// TR (cout % 8 == 0): the MFMA is issued transposed (A = weights, B = voxel rows), so after one permlane32 swap a
// lane holds 8 consecutive channels x 2 of ONE voxel and writes them as 16-B stores (the untransposed form writes
// 16 scalar 4-B stores per lane, half the lanes idle at cout = 16); the next tile's rows are loaded before the
// current tile's MFMA and stores.
template <int KS, bool TR>
__global__ __launch_bounds__(HD_T) void head_fwd_kernel(const bf16* __restrict__ x, long long v, int cin,
                                                       const bf16* __restrict__ wpk, int cout, int cin_p,
                                                       const float* __restrict__ bias, const float* __restrict__ st,
                                                       const float* __restrict__ ga, const float* __restrict__ be,
                                                       int groups, int n, float* __restrict__ y) {
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  // B fragments: lane (col co = r, half h) holds W[co][16 s + 8 h .. +7]
  bf16x8 bw[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s)
    bw[s] = as_frag(*reinterpret_cast<const u32x4*>(wpk + (long long)r * cin_p + 16 * s + 8 * h));
  const long long tiles = (n * v + 31) / 32;
  const long long wid = (long long)blockIdx.x * (HD_T / 64) + (threadIdx.x >> 6);
  const long long nw = (long long)gridDim.x * (HD_T / 64);
  int gn_n = -1;
  f32x2 sc[KS][4], sh[KS][4];
  if constexpr (TR) {
    // GroupNorm scale / shift of every (sample, channel) in LDS, filled once per block (the per-sample coefficient
    // loads inline in the loop held ~80 registers live and cut the occupancy of this streaming kernel to 2 waves)
    __shared__ f32x2 gtab[HD_GMAX];
    if (st) {
      for (int i = threadIdx.x; i < n * cin; i += HD_T) {
        const int nn = i / cin, c = i - nn * cin, gg = c / (cin / groups);
        const float mean = st[(nn * groups + gg) * 2], rstd = st[(nn * groups + gg) * 2 + 1];
        const float sc_ = rstd * ga[c];
        gtab[i] = f32x2{sc_, be[c] - mean * sc_};
      }
      __syncthreads();
    }
    // bias of this lane's two 8-channel runs (8h .. 8h+7 and 16+8h .. 16+8h+7) after the swap
    float b0[8], b1[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      b0[e] = bias && 8 * h + e < cout ? bias[8 * h + e] : 0.f;
      b1[e] = bias && 16 + 8 * h + e < cout ? bias[16 + 8 * h + e] : 0.f;
    }
    auto load = [&](long long tile, u32x4 (&a)[KS]) {
      const long long row = tile * 32 + r;
      const bool ok = tile < tiles && row < n * v;
#pragma unroll
      for (int s = 0; s < KS; ++s) {  // clamped row, no branch around the load (its wait would land right after it)
        const u32x4 t = *reinterpret_cast<const u32x4*>(x + (ok ? row : 0) * cin + 16 * s + 8 * h);
        a[s] = ok ? t : u32x4{0u, 0u, 0u, 0u};
      }
    };
    u32x4 a[KS], an[KS];
    load(wid, a);
    for (long long tile = wid; tile < tiles; tile += nw) {
      load(tile + nw, an);  // next tile's rows in flight under this tile's MFMAs and stores
      const long long row = tile * 32 + r;
      const bool ok = row < n * v;
      const int nn = ok ? (int)((unsigned)row / (unsigned)v) : 0;  // n * v < 2^31 (host check): 32-bit division
      if (st && ok) {
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          f32x2 sc_[4], sh_[4];
          const f32x2* t = gtab + nn * cin + 16 * s + 8 * h;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const f32x2 p0 = t[2 * e], p1 = t[2 * e + 1];
            sc_[e] = f32x2{p0[0], p1[0]};
            sh_[e] = f32x2{p0[1], p1[1]};
          }
          a[s] = gn_relu8(a[s], sc_, sh_);
        }
      }
      f32x16 acc;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
      for (int s = 0; s < KS; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bw[s], as_frag(a[s]), acc, 0, 0, 0);
      // acc[4q + e] = channel 8q + 4h + e of voxel row; swap so lane h holds 8h..8h+7 and 16+8h..16+8h+7
#pragma unroll
      for (int q = 0; q < 4; q += 2)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[4 * q + e]),
                                                           __float_as_uint(acc[4 * q + 4 + e]), false, false);
          acc[4 * q + e] = __uint_as_float(sw[0]);
          acc[4 * q + 4 + e] = __uint_as_float(sw[1]);
        }
      if (ok) {
        float* yr = y + row * cout;
        if (8 * h < cout) {
          *reinterpret_cast<f32x4*>(yr + 8 * h) = f32x4{acc[0] + b0[0], acc[1] + b0[1], acc[2] + b0[2], acc[3] + b0[3]};
          *reinterpret_cast<f32x4*>(yr + 8 * h + 4) =
              f32x4{acc[4] + b0[4], acc[5] + b0[5], acc[6] + b0[6], acc[7] + b0[7]};
        }
        if (16 + 8 * h < cout) {
          *reinterpret_cast<f32x4*>(yr + 16 + 8 * h) =
              f32x4{acc[8] + b1[0], acc[9] + b1[1], acc[10] + b1[2], acc[11] + b1[3]};
          *reinterpret_cast<f32x4*>(yr + 20 + 8 * h) =
              f32x4{acc[12] + b1[4], acc[13] + b1[5], acc[14] + b1[6], acc[15] + b1[7]};
        }
      }
#pragma unroll
      for (int s = 0; s < KS; ++s) a[s] = an[s];
    }
    return;
  }
  const float bv = r < cout && bias ? bias[r] : 0.f;
  for (long long tile = wid; tile < tiles; tile += nw) {
    const long long row = tile * 32 + r;  // this lane's A row (voxel over all samples)
    const bool ok = row < n * v;
    const int nn = ok ? (int)(row / v) : 0;
    if (st && nn != gn_n) {
      gn_n = nn;
#pragma unroll
      for (int s = 0; s < KS; ++s) gn_coef8(st, ga, be, groups, cin, nn, 16 * s + 8 * h, sc[s], sh[s]);
    }
    u32x4 a[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      a[s] = ok ? *reinterpret_cast<const u32x4*>(x + row * cin + 16 * s + 8 * h) : u32x4{0u, 0u, 0u, 0u};
      if (st && ok) a[s] = gn_relu8(a[s], sc[s], sh[s]);
    }
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_frag(a[s]), bw[s], acc, 0, 0, 0);
    // acc[i]: row (i&3) + 8(i>>2) + 4h, column co = r
    if (r < cout) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const long long orow = tile * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
        if (orow < n * v) y[orow * cout + r] = acc[i] + bv;
      }
    }
  }
}

// dA = dy W: A operand = dy tile (32 voxels x cout, fp32 -> bf16 in registers), B = W^T from the data-grad
// pack [ci_p][co_p]; 2 k-steps cover cout <= 32. Also writes dy as bf16 [v][cout_p8] and per-block dy column sums.
__global__ __launch_bounds__(HD_T) void head_bwd_kernel(const float* __restrict__ dy, long long rows, int cout,
                                                       const bf16* __restrict__ wpd, int cout_p, int cin,
                                                       bf16* __restrict__ dA, bf16* __restrict__ dyb, int cout8,
                                                       float* __restrict__ dbp, int tr) {
  __shared__ float red[HD_T / 64][32];
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5, wave = threadIdx.x >> 6;
  bf16x8 bw[2][2];  // [k-step][n-tile of 32 ci]
  const int ntn = (cin + 31) / 32;
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int tn = 0; tn < 2; ++tn) {
      const int ci = tn * 32 + r, co = 16 * s + 8 * h;
      bw[s][tn] = (tn < ntn && co < cout_p)
                      ? as_frag(*reinterpret_cast<const u32x4*>(wpd + (long long)ci * cout_p + co))
                      : as_frag(u32x4{0u, 0u, 0u, 0u});
    }
  float colsum[2][8];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int e = 0; e < 8; ++e) colsum[s][e] = 0.f;
  const long long tiles = (rows + 31) / 32;
  const long long wid = (long long)blockIdx.x * (HD_T / 64) + wave;
  const long long nw = (long long)gridDim.x * (HD_T / 64);
  for (long long tile = wid; tile < tiles; tile += nw) {
    const long long row = tile * 32 + r;
    const bool ok = row < rows;
    u32x4 a[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float f[8];
      const int cb = 16 * s + 8 * h;
      if (ok && cb + 8 <= cout && (cout & 3) == 0) {  // two 16-B loads
        const f32x4 u0 = *reinterpret_cast<const f32x4*>(dy + row * cout + cb);
        const f32x4 u1 = *reinterpret_cast<const f32x4*>(dy + row * cout + cb + 4);
        f[0] = u0[0]; f[1] = u0[1]; f[2] = u0[2]; f[3] = u0[3];
        f[4] = u1[0]; f[5] = u1[1]; f[6] = u1[2]; f[7] = u1[3];
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = ok && cb + e < cout ? dy[row * cout + cb + e] : 0.f;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) colsum[s][e] += f[e];
      store16<bf16>(reinterpret_cast<bf16*>(&a[s]), f);
      if (ok && 16 * s + 8 * h < cout8) *reinterpret_cast<u32x4*>(dyb + row * cout8 + 16 * s + 8 * h) = a[s];
    }
#pragma unroll
    for (int tn = 0; tn < 2; ++tn) {
      if (tn >= ntn) break;
      f32x16 acc;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = 0.f;
      if (tr) {  // transposed: D[ci][voxel], a lane ends with 8 consecutive ci x 2 of its voxel -> 16-B stores
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bw[0][tn], as_frag(a[0]), acc, 0, 0, 0);
        if (cout_p > 16) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bw[1][tn], as_frag(a[1]), acc, 0, 0, 0);
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
        if (ok) {
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            const int ci = tn * 32 + 16 * u + 8 * h;
            if (ci < cin)
              *reinterpret_cast<u32x4*>(dA + row * cin + ci) =
                  u32x4{pk[2 * u][0], pk[2 * u][1], pk[2 * u + 1][0], pk[2 * u + 1][1]};
          }
        }
        continue;
      }
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_frag(a[0]), bw[0][tn], acc, 0, 0, 0);
      if (cout_p > 16) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_frag(a[1]), bw[1][tn], acc, 0, 0, 0);
      const int ci = tn * 32 + r;
      if (ci < cin) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const long long orow = tile * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
          if (orow < rows) dA[orow * cin + ci] = from_f<bf16>(acc[i]);
        }
      }
    }
  }
  // bias-gradient partials: lanes (r, h) hold columns 16 s + 8 h + e summed over their rows; reduce the 32
  // rows of the wave (lanes with equal h), then the waves in fixed order
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float t = colsum[s][e];
      for (int o = 16; o > 0; o >>= 1) t += __shfl_xor(t, o, 32);
      colsum[s][e] = t;
    }
  if (r == 0) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int e = 0; e < 8; ++e) red[wave][16 * s + 8 * h + e] = colsum[s][e];
  }
  __syncthreads();
  if (threadIdx.x < 32) {
    float t = 0.f;
    for (int w = 0; w < HD_T / 64; ++w) t += red[w][threadIdx.x];
    if (threadIdx.x < cout) dbp[(long long)blockIdx.x * cout + threadIdx.x] = t;
  }
}

// The head's data gradient with the partial-label loss gradient formed in registers (the bench's loss: softmax over
// 16 classes + per-class BCE): dlogits never reaches HBM (-2 x 113 MB per step at 2 x 96^3). Lanes r and r + 32 hold
// one voxel's classes 0-7 / 8-15 (the 8 channels each feeds the MFMA) and form their gradients as loss_bwd_kernel
// does (dice_bce_softmax_grad8, bitwise dice_bce_softmax_grad16); the rest is head_bwd_kernel's transposed path with
// the same grid, so dA, the bf16 dy and the bias partials equal the two-kernel form's bit for bit. The next tile's
// logits and label are loaded before this tile's math.
// GN (round 6): the head's input x = relu(gn(x0)) prologue's GroupNorm backward starts here, as the data-gradient
// ring's epilogue does it (u3d_conv32_ring_dgrad_gn): per (sample, block, channel) (sum g, sum g * xhat) of
// g = relu-mask * dA, from the stored bf16 dA and the bf16 x0 at the same voxel (gn_bwd_partial's per-element terms) —
// the separate partial pass over dA and x0 goes (2 x 113 MB at 2 x 96^3 -> 1 x 113 MB here). Blocks never straddle
// samples (grid = n x bps, tiles of 32 voxels inside one sample: v % 32 == 0); parts[n][bps][cin][2].
template <bool GN>
__global__ __launch_bounds__(HD_T) void head_loss_bwd_kernel(const float* __restrict__ lg, const float* __restrict__ lab,
                                                            long long rows, const float* __restrict__ wt,
                                                            const double* __restrict__ sums,
                                                            const float* __restrict__ gout, const bf16* __restrict__ wpd,
                                                            int cin, bf16* __restrict__ dA, bf16* __restrict__ dyb,
                                                            float* __restrict__ dbp, const bf16* __restrict__ x0 = nullptr,
                                                            const float* __restrict__ gst = nullptr,
                                                            const float* __restrict__ gga = nullptr,
                                                            const float* __restrict__ gbe = nullptr, int ggroups = 0,
                                                            long long v = 0, int bps = 1,
                                                            float* __restrict__ gparts = nullptr,
                                                            float* __restrict__ dbias = nullptr,
                                                            unsigned* __restrict__ cnt = nullptr) {
  constexpr int cout = 16, cout_p = 32;
  __shared__ float red[HD_T / 64][32];
  __shared__ f32x4 gtb[GN ? 64 : 1];  // per channel (scale, shift, rstd, mean) of the block's sample
  __shared__ float kd_a[16], kd_b[16], kb[16];
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5, wave = threadIdx.x >> 6;
  if (threadIdx.x < 16) {
    float a, b, e;
    dice_bce_coefs(threadIdx.x, 16, sums, wt, gout, 1, (double)rows, a, b, e);
    kd_a[threadIdx.x] = a;
    kd_b[threadIdx.x] = b;
    kb[threadIdx.x] = e;
  }
  bf16x8 bw[2][2];  // [k-step][n-tile of 32 ci]
  const int ntn = (cin + 31) / 32;
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int tn = 0; tn < 2; ++tn) {
      const int ci = tn * 32 + r, co = 16 * s + 8 * h;
      bw[s][tn] = (tn < ntn && co < cout_p)
                      ? as_frag(*reinterpret_cast<const u32x4*>(wpd + (long long)ci * cout_p + co))
                      : as_frag(u32x4{0u, 0u, 0u, 0u});
    }
  float colsum[2][8];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int e = 0; e < 8; ++e) colsum[s][e] = 0.f;
  __syncthreads();
  // GN: block b runs tiles of sample b / bps only (row offset row0); otherwise the whole grid strides over all rows
  const int smp = GN ? (int)(blockIdx.x / bps) : 0;
  const long long row0 = GN ? (long long)smp * v : 0, rows_b = GN ? row0 + v : rows;
  const long long tiles = GN ? v / 32 : (rows + 31) / 32;
  const long long wid = (long long)(GN ? blockIdx.x % bps : blockIdx.x) * (HD_T / 64) + wave;
  const long long nw = (long long)(GN ? bps : gridDim.x) * (HD_T / 64);
  float g1[16], g2[16];  // GN: (sum g, sum g * xhat) of this lane's 16 channels 16 u + 8 h + e
#pragma unroll
  for (int e = 0; e < 16; ++e) g1[e] = g2[e] = 0.f;
  if constexpr (GN) {
    if (threadIdx.x < cin) {
      const int c = threadIdx.x, gr = c / (cin / ggroups);
      const float mu = gst[(smp * ggroups + gr) * 2], rs = gst[(smp * ggroups + gr) * 2 + 1];
      const float scv = rs * gga[c];
      gtb[c] = f32x4{scv, gbe[c] - mu * scv, rs, mu};
    }
    __syncthreads();
  }
  // GN: x0 at this lane's two 8-channel runs of its voxel (where the swap below leaves its dA), prefetched with the
  // logits
  auto load = [&](long long tile, f32x4 (&q)[2], float& t, u32x4 (&xq)[2]) {  // clamped row, no branch around loads
    long long row = row0 + tile * 32 + r;
    row = row < rows_b ? row : rows_b - 1;
#pragma unroll
    for (int k = 0; k < 2; ++k) q[k] = *reinterpret_cast<const f32x4*>(lg + row * 16 + 8 * h + 4 * k);
    t = lab[row];
    if constexpr (GN) {
#pragma unroll
      for (int u = 0; u < 2; ++u) xq[u] = *reinterpret_cast<const u32x4*>(x0 + row * cin + 16 * u + 8 * h);
    }
  };
  // ND tiles' loads in flight per wave (register buffers rotated by moves each tile): the kernel is load-latency-bound with one tile of look-ahead (round 6: 64 us at 2 x 96^3 = 4.5 TB/s).
  // Tiles are still visited in the order tile, tile + nw, ... (the bias partials' summation order is unchanged).
  constexpr int ND = GN ? HD_ND_GN : HD_ND;
  f32x4 qb[ND][2];
  float tb[ND];
  u32x4 xb[ND][2];
#pragma unroll
  for (int k = 0; k < ND; ++k) load(wid + k * nw, qb[k], tb[k], xb[k]);
  auto body = [&](long long tile, const f32x4 (&cur)[2], float tcur, const u32x4 (&xq)[2]) {
    const long long row = row0 + tile * 32 + r;
    const bool ok = row < rows_b;
    float gr[8];
    dice_bce_softmax_grad8(cur, tcur, h, kd_a, kd_b, kb, gr);
    u32x4 a[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float f[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = ok && s == 0 ? gr[e] : 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) colsum[s][e] += f[e];
      store16<bf16>(reinterpret_cast<bf16*>(&a[s]), f);
      if (ok && s == 0) *reinterpret_cast<u32x4*>(dyb + row * cout + 8 * h) = a[s];
    }
#pragma unroll
    for (int tn = 0; tn < 2; ++tn) {
      if (tn >= ntn) break;
      f32x16 acc;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = 0.f;
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bw[0][tn], as_frag(a[0]), acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bw[1][tn], as_frag(a[1]), acc, 0, 0, 0);
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
      if (ok) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int ci = tn * 32 + 16 * u + 8 * h;
          if (ci < cin)
            *reinterpret_cast<u32x4*>(dA + row * cin + ci) =
                u32x4{pk[2 * u][0], pk[2 * u][1], pk[2 * u + 1][0], pk[2 * u + 1][1]};
        }
      }
      if constexpr (GN) {
        if (tn == 0) {  // (cin == 32: one n-tile; the stored bf16 dA and x0, as gn_bwd_partial reads them)
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            const u32x4 av = u32x4{pk[2 * u][0], pk[2 * u][1], pk[2 * u + 1][0], pk[2 * u + 1][1]};
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const uint32_t aw = av[e >> 1], xw = xq[u][e >> 1];
              const float a = __uint_as_float((e & 1) ? (aw & 0xffff0000u) : (aw << 16));
              const float xv = __uint_as_float((e & 1) ? (xw & 0xffff0000u) : (xw << 16));
              const f32x4 t = gtb[16 * u + 8 * h + e];
              const float gd = ok && fmaf(xv, t[0], t[1]) > 0.f ? a : 0.f;  // the forward prologue's relu test
              g1[8 * u + e] += gd;
              g2[8 * u + e] = fmaf(gd, (xv - t[3]) * t[2], g2[8 * u + e]);
            }
          }
        }
      }
    }
  };
  for (long long tile = wid; tile < tiles; tile += nw) {
    const f32x4 c[2] = {qb[0][0], qb[0][1]};
    const float tc = tb[0];
    const u32x4 xc[2] = {xb[0][0], xb[0][1]};
#pragma unroll
    for (int k = 0; k + 1 < ND; ++k) {  // rotate (register moves)
      qb[k][0] = qb[k + 1][0];
      qb[k][1] = qb[k + 1][1];
      tb[k] = tb[k + 1];
      xb[k][0] = xb[k + 1][0];
      xb[k][1] = xb[k + 1][1];
    }
    load(tile + ND * nw, qb[ND - 1], tb[ND - 1], xb[ND - 1]);
    body(tile, c, tc, xc);
  }
  if constexpr (GN) {
    // per channel over the block: the 32 lanes of a half hold the same channels (xor over r), then the 4 waves in
    // order; one [cin][2] row per block into parts[sample][block of the sample]
    __shared__ float gred[HD_T / 64][64][2];
#pragma unroll
    for (int e = 0; e < 16; ++e)
#pragma unroll
      for (int o = 1; o < 32; o <<= 1) {
        g1[e] += __shfl_xor(g1[e], o, 32);
        g2[e] += __shfl_xor(g2[e], o, 32);
      }
    if (r == 0) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int c = 16 * (e >> 3) + 8 * h + (e & 7);
        gred[wave][c][0] = g1[e];
        gred[wave][c][1] = g2[e];
      }
    }
    __syncthreads();
    if (threadIdx.x < 2 * cin) {
      const int c = threadIdx.x >> 1, k = threadIdx.x & 1;
      float t = 0.f;
#pragma unroll
      for (int w_ = 0; w_ < HD_T / 64; ++w_) t += gred[w_][c][k];
      gparts[(((long long)smp * bps + blockIdx.x % bps) * cin + c) * 2 + k] = t;
    }
  }
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float t = colsum[s][e];
      for (int o = 16; o > 0; o >>= 1) t += __shfl_xor(t, o, 32);
      colsum[s][e] = t;
    }
  if (r == 0) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int e = 0; e < 8; ++e) red[wave][16 * s + 8 * h + e] = colsum[s][e];
  }
  __syncthreads();
  if (threadIdx.x < 32) {
    float t = 0.f;
    for (int w = 0; w < HD_T / 64; ++w) t += red[w][threadIdx.x];
    if (threadIdx.x < cout) {
      if (GN && dbias)  // agent-scope (sc1) store: read by the last-arriving block below
        __hip_atomic_store(dbp + (long long)blockIdx.x * cout + threadIdx.x, t, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      else
        dbp[(long long)blockIdx.x * cout + threadIdx.x] = t;
    }
  }
  if constexpr (GN) {
    // round 6: the bias gradient summed by the launch's last-arriving block (fixed row order, fp64) instead of two
    // channel-sum launches after it; the counter is left zeroed
    if (dbias == nullptr) return;
    __shared__ unsigned s_last;
    __shared__ double cs[16];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = old == gridDim.x - 1;
      if (s_last) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!s_last) return;
    lastarriver_rowsum<HD_T>(dbp, 1, (int)gridDim.x, cout, cs);
    __syncthreads();
    if (threadIdx.x < cout) dbias[threadIdx.x] = (float)cs[threadIdx.x];
  }
}

// grid cap: 768 = three 4-wave blocks per CU, resident at once at the backward's 148 VGPRs (2048 ran it in 2.7
// rounds). 2 x 96^3 x 32 -> 16 (tools/kbench.py headf96 / headb96, gpurun_out/r04_hd): forward 37.3 -> 36.0 us,
// backward 62.2 -> 57.3 us; 1024 / 1280 blocks: backward 66-70 us
static int head_blocks(long long rows) {
  return (int)std::min<long long>(opt(OPT_HEAD_NB), std::max<long long>(1, (rows + 127) / 128));
}

}  // namespace u3d

using namespace u3d;

extern "C" int u3d_head_fwd(const void* x, int n, long long v, int cin, const void* wpk, int cout, const float* bias,
                            const float* gn_stats, const float* gn_gamma, const float* gn_beta, int gn_groups,
                            float* y, u3d_stream_t stream) {
  U3D_REQUIRE(x && wpk && y && n >= 1 && v >= 1, "head_fwd: bad args");
  U3D_REQUIRE(cin % 16 == 0 && cin >= 16 && cin <= 64 && cout >= 1 && cout <= 32, "head_fwd: cin %d / cout %d", cin,
              cout);
  U3D_REQUIRE(!gn_stats || (gn_gamma && gn_beta && gn_groups > 0 && cin % gn_groups == 0), "head_fwd: bad GN");
  U3D_REQUIRE((long long)n * v < (1LL << 31), "head_fwd: n * v must be < 2^31");
  const int cin_p = round_up(cin, 32);
  const int nb = head_blocks(n * v);
  hipStream_t s = (hipStream_t)stream;
#define HF(KS, TR)                                                                                                   \
  hipLaunchKernelGGL((head_fwd_kernel<KS, TR>), dim3(nb), dim3(HD_T), 0, s, (const bf16*)x, v, cin, (const bf16*)wpk, \
                     cout, cin_p, bias, gn_stats, gn_gamma, gn_beta, gn_groups, n, y)
  if (cout % 8 == 0 && opt(OPT_HEAD_TR) != 0 && (!gn_stats || (long long)n * cin <= HD_GMAX)) {
    switch (cin / 16) {
      case 1: HF(1, true); break;
      case 2: HF(2, true); break;
      case 3: HF(3, true); break;
      default: HF(4, true); break;
    }
  } else {
    switch (cin / 16) {
      case 1: HF(1, false); break;
      case 2: HF(2, false); break;
      case 3: HF(3, false); break;
      default: HF(4, false); break;
    }
  }
#undef HF
  return check_launch("head_fwd_kernel");
}

extern "C" int u3d_head_bwd_blocks(long long rows) { return head_blocks(rows); }

extern "C" int u3d_head_bwd(const float* dy, long long rows, int cout, const void* wpk_dgrad, int cin, void* dA,
                            void* dy_bf16, float* dbias_partials, u3d_stream_t stream) {
  U3D_REQUIRE(dy && wpk_dgrad && dA && dy_bf16 && dbias_partials && rows >= 1, "head_bwd: bad args");
  U3D_REQUIRE(cout >= 1 && cout <= 32 && cin % 8 == 0 && cin <= 64, "head_bwd: cout %d / cin %d", cout, cin);
  const int cout_p = round_up(cout, 32), cout8 = round_up(cout, 8);
  const int tr = opt(OPT_HEAD_TR) != 0 ? 1 : 0;  // 0: untransposed scalar dA stores
  hipLaunchKernelGGL(head_bwd_kernel, dim3(head_blocks(rows)), dim3(HD_T), 0, (hipStream_t)stream, dy, rows, cout,
                     (const bf16*)wpk_dgrad, cout_p, cin, (bf16*)dA, (bf16*)dy_bf16, cout8, dbias_partials, tr);
  return check_launch("head_bwd_kernel");
}

// Fused form of u3d_partial_loss_bwd (softmax, uce 1, C = 16, fp32 dlogits) followed by u3d_head_bwd on the result
// (cout = C): the same dA, bf16 dy and bias partials without the dlogits tensor. rows = S * V voxels (the loss's
// count), logits / labels as u3d_partial_loss_bwd takes them (NDHWC fp32 logits, fp32 labels).
extern "C" int u3d_head_loss_bwd(const float* logits, const float* labels, long long rows, int C, const float* weights,
                                 const double* sums, const float* grad_out, const void* wpk_dgrad, int cin, void* dA,
                                 void* dy_bf16, float* dbias_partials, u3d_stream_t stream) {
  U3D_REQUIRE(logits && labels && weights && sums && grad_out && wpk_dgrad && dA && dy_bf16 && dbias_partials &&
                  rows >= 1,
              "head_loss_bwd: bad args");
  U3D_REQUIRE(C == 16 && cin % 8 == 0 && cin >= 8 && cin <= 64, "head_loss_bwd: C %d (16 only) / cin %d", C, cin);
  hipLaunchKernelGGL(head_loss_bwd_kernel<false>, dim3(head_blocks(rows)), dim3(HD_T), 0, (hipStream_t)stream, logits,
                     labels, rows, weights, sums, grad_out, (const bf16*)wpk_dgrad, cin, (bf16*)dA, (bf16*)dy_bf16,
                     dbias_partials);
  return check_launch("head_loss_bwd_kernel");
}

// Round 6: blocks per sample of u3d_head_loss_bwd_gn (its parts[n][bps][cin][2] and dbias_partials[n * bps][C]); 0 where
// the GN form does not apply (v % 32 != 0, cin != 32).
extern "C" int u3d_head_loss_bwd_gn_bps(int n, long long v, int cin) {
  if (n < 1 || v < 32 || v % 32 != 0 || cin != 32 || (long long)n * v >= (1LL << 31)) return 0;
  // 2 blocks per CU (the GN form's ~200 VGPRs leave 2 waves per SIMD; the plain form's 768 = 3 per CU would run as
  // 1.5 rounds of blocks)
  return std::max(1, (int)std::min<long long>(opt(OPT_HEAD_GN_NB), ((long long)n * v + 127) / 128) / n);
}

// u3d_head_loss_bwd plus the GroupNorm-backward partials of the head's GN + ReLU prologue (x0 = its input, gn_* = its
// GroupNorm) into parts[n][bps][cin][2] = (sum g, sum g * xhat) per block of one sample, bps =
// u3d_head_loss_bwd_gn_bps(n, v, cin); u3d_gn_bwd_parts then finalizes and applies them. dbias_partials holds n * bps
// rows; with dbias (+ cnt: one zeroed unsigned, left zeroed) the launch's last block also sums them into dbias[C].
// dA, dy and the bias gradient are those of u3d_head_loss_bwd up to the bias partials' summation order.
extern "C" int u3d_head_loss_bwd_gn(const float* logits, const float* labels, int n, long long v, int C,
                                    const float* weights, const double* sums, const float* grad_out,
                                    const void* wpk_dgrad, int cin, void* dA, void* dy_bf16, float* dbias_partials,
                                    const void* x0, const float* gn_stats, const float* gn_gamma, const float* gn_beta,
                                    int gn_groups, float* parts, float* dbias, unsigned* cnt, u3d_stream_t stream) {
  const int bps = u3d_head_loss_bwd_gn_bps(n, v, cin);
  U3D_REQUIRE(bps > 0 && C == 16, "head_loss_bwd_gn: needs C = 16, cin = 32, v %% 32 == 0");
  U3D_REQUIRE(logits && labels && weights && sums && grad_out && wpk_dgrad && dA && dy_bf16 && dbias_partials && x0 &&
                  gn_stats && gn_gamma && gn_beta && gn_groups > 0 && cin % gn_groups == 0 && parts && (!dbias || cnt),
              "head_loss_bwd_gn: bad args");
  hipLaunchKernelGGL(head_loss_bwd_kernel<true>, dim3(n * bps), dim3(HD_T), 0, (hipStream_t)stream, logits, labels,
                     (long long)n * v, weights, sums, grad_out, (const bf16*)wpk_dgrad, cin, (bf16*)dA, (bf16*)dy_bf16,
                     dbias_partials, (const bf16*)x0, gn_stats, gn_gamma, gn_beta, gn_groups, v, bps, parts, dbias, cnt);
  return check_launch("head_loss_bwd_kernel<GN>");
}
