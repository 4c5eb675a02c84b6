// 32 -> 32 channel 3^3 stride-1 convolution (forward and data gradient), bf16, halo-brick form (gfx950).
//
// These convolutions (layer0, x1_resb at the full 96^3 resolution) carry ~51% of the U-Net's FLOPs
// (SURVEY §2.1). As a GEMM they are M = voxels (1.77M) x N = 32 x K = 27*32, so each A fragment is used by
// exactly one 32-wide MFMA column block; the design keeps the MFMA pipe fed from LDS:
//   * a persistent workgroup of 8 waves (two per SIMD) walks output bricks of 2 x 8 x 32 voxels;
//   * per brick the input halo (4 x 10 x 34 voxels x 32 ch) is staged once into LDS with the GroupNorm +
//     ReLU prologue applied once per element (not once per tap) and zero padding after it; the next brick's
//     halo is prefetched into registers while the MFMAs run;
//   * the weights of all 27 taps (55 KB) stay in LDS for the workgroup's lifetime;
//   * LDS images are "chunk-planar": plane c holds 16 B (8 channels) of every row, so the 32 consecutive
//     rows of an MFMA A fragment are 512 contiguous bytes (conflict-free ds_read_b128) and every tap's
//     window is the same per-lane address plus a compile-time offset;
//   * each wave computes two 32-voxel w-rows x 32 co; the B fragment is shared by both.
// Data gradient = the same kernel with the flipped tap offsets and the [t][ci][co] weight pack.
// Reference: F.conv3d in Conv3d.forward (unet3D.py:27) via NoBottleneck (:56-73) and its autograd.
#include "common.h"

namespace u3d {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;

constexpr int CB_BD = 2, CB_BH = 8, CB_BW = 32;
constexpr int CB_HD = CB_BD + 2, CB_HH = CB_BH + 2, CB_HW = CB_BW + 2;
constexpr int CB_NH = CB_HD * CB_HH * CB_HW;            // 1360 halo rows
constexpr int CB_NWR = 27 * 32;                          // weight rows (t, co)
constexpr int CB_NT = 512;
constexpr int CB_LD = (CB_NH + CB_NT / 4 - 1) / (CB_NT / 4);  // 11 prefetch loads per thread
constexpr int CB_PS = CB_NH * 16 + 64;                   // LDS plane stride (+64 B: conflict-free staging writes)
constexpr int CB_MAXN = 16;

struct CBGeom {
  int n, d, h, w;
  int nbd, nbh, nbw;
  int nbricks;
  int gn_groups;
};

template <bool FLIP>
__global__ __launch_bounds__(CB_NT, 1) void conv32_brick_kernel(const bf16* __restrict__ x, const bf16* __restrict__ wpk,
                                                               bf16* __restrict__ y, const bf16* __restrict__ res,
                                                               const float* __restrict__ gstat,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ beta, CBGeom g) {
  // one LDS object: halo image | weights | per-wave epilogue tile (32 voxels x 64 B)
  __shared__ __attribute__((aligned(16))) char smem[4 * CB_PS + 4 * CB_NWR * 16 + 8 * 2048];
  char* const hal = smem;
  char* const wts = smem + 4 * CB_PS;
  char* const ept = smem + 4 * CB_PS + 4 * CB_NWR * 16 + (threadIdx.x >> 6) * 2048;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int ch = tid & 3, row0 = tid >> 2;  // staging: fixed 8-channel chunk per thread, rows row0 + 128 i
  const bool has_gn = gstat != nullptr;
  // weights: plane ch, row t*32 + co
  for (int i = tid; i < CB_NWR * 4; i += CB_NT) {
    const int c = i / CB_NWR, row = i % CB_NWR;
    *reinterpret_cast<u32x4*>(wts + (c * CB_NWR + row) * 16) =
        *reinterpret_cast<const u32x4*>(wpk + row * 32 + c * 8);
  }

  u32x4 pre[CB_LD];
  f32x2 sc[4], sh[4];
  int gn_n = -1;
  auto brick_origin = [&](int b, int& nn, int& d0, int& h0, int& w0) {
    int t = b;
    const int bw_ = t % g.nbw; t /= g.nbw;
    const int bh_ = t % g.nbh; t /= g.nbh;
    const int bd_ = t % g.nbd;
    nn = t / g.nbd;
    d0 = bd_ * CB_BD; h0 = bh_ * CB_BH; w0 = bw_ * CB_BW;
  };
  // 4 consecutive threads read the 64 B (32 channels) of one voxel: fully coalesced loads. vmask bit i =
  // halo row i of this thread lies inside the volume (GN applies there; padding stays zero).
  unsigned vmask = 0;
  auto prefetch = [&](int b) {
    int nn, d0, h0, w0;
    brick_origin(b, nn, d0, h0, w0);
    int rb = row0;
    asm volatile("" : "+v"(rb));  // keep the row decomposition in the loop (no hoisted, spilled invariants)
    unsigned m = 0;
#pragma unroll
    for (int i = 0; i < CB_LD; ++i) {
      const int row = rb + i * (CB_NT / 4);
      u32x4 v = {0u, 0u, 0u, 0u};
      if (row < CB_NH) {
        const int hw = row % CB_HW, hh = (row / CB_HW) % CB_HH, hd = row / (CB_HW * CB_HH);
        const int zd = d0 - 1 + hd, zh = h0 - 1 + hh, zw = w0 - 1 + hw;
        if ((unsigned)zd < (unsigned)g.d && (unsigned)zh < (unsigned)g.h && (unsigned)zw < (unsigned)g.w) {
          v = *reinterpret_cast<const u32x4*>(x + ((((long long)nn * g.d + zd) * g.h + zh) * g.w + zw) * 32 + ch * 8);
          m |= 1u << i;
        }
      }
      pre[i] = v;
    }
    vmask = m;
  };
  auto commit = [&](int b) {
    if (has_gn) {
      int t = b / (g.nbw * g.nbh * g.nbd);
      if (t != gn_n) {
        gn_n = t;
        gn_coef8(gstat, gamma, beta, g.gn_groups, 32, t, ch * 8, sc, sh);
      }
    }
#pragma unroll
    for (int i = 0; i < CB_LD; ++i) {
      const int row = row0 + i * (CB_NT / 4);
      if (row < CB_NH) {
        u32x4 v = pre[i];
        if (has_gn && ((vmask >> i) & 1u)) v = gn_relu8(v, sc, sh);
        *reinterpret_cast<u32x4*>(hal + ch * CB_PS + row * 16) = v;
      }
    }
  };

  // XCD-aware brick order: with a full 256-WG grid, XCD x (= blockIdx % 8) walks one contiguous eighth of
  // the bricks, so the 32 bricks it runs at a time are spatial neighbours and their shared halo rows hit
  // its L2 instead of being fetched once per XCD.
  int b, bend, bstep;
  if (gridDim.x == 256) {
    const int per = (g.nbricks + 7) >> 3, xcd = blockIdx.x & 7;
    b = xcd * per + (blockIdx.x >> 3);
    bend = min(g.nbricks, (xcd + 1) * per);
    bstep = 32;
  } else {
    b = blockIdx.x;
    bend = g.nbricks;
    bstep = gridDim.x;
  }
  if (b >= bend) return;
  prefetch(b);
  commit(b);
  __syncthreads();
  // per-lane fragment bases: A row of tap (0,0,0) for w-row tm: ((tm)*HH + wave)*HW + r ; plane (2s + h)
  const char* abase = hal + h * CB_PS + (wave * CB_HW + r) * 16;
  const char* bbase = wts + (h * CB_NWR + r) * 16;
  for (; b < bend; b += bstep) {
    const int bn = b + bstep;
    const bool more = bn < bend;
    prefetch(more ? bn : b);  // unconditional: keeps the prefetch registers phi-free (no copies, no early wait)
    int nn, d0, h0, w0;
    brick_origin(b, nn, d0, h0, w0);
    // residual of this brick's two w-rows (16-B chunks q = lane + 64 u of each row): loaded before the MFMAs
    // so their latency hides under them
    u32x4 rv[2][2];
    const long long orow[2] = {(((long long)nn * g.d + d0) * g.h + h0 + wave) * g.w + w0,
                               (((long long)nn * g.d + d0 + 1) * g.h + h0 + wave) * g.w + w0};
    const bool ok[2] = {d0 < g.d && h0 + wave < g.h, d0 + 1 < g.d && h0 + wave < g.h};
    if (res) {
#pragma unroll
      for (int tm = 0; tm < 2; ++tm)
#pragma unroll
        for (int u = 0; u < 2; ++u)
          rv[tm][u] = ok[tm] ? *reinterpret_cast<const u32x4*>(res + orow[tm] * 32 + (lane + 64 * u) * 8)
                             : u32x4{0u, 0u, 0u, 0u};
    }
    f32x16 acc0, acc1;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc0[e] = acc1[e] = 0.f;
    // 54 steps (tap t, k16 half s); fragments of step i+1 are read while step i's MFMAs run
    auto aoff = [](int st) {
      const int t = st >> 1, s = st & 1;
      const int td = t / 9, th = (t / 3) % 3, tw = t % 3;
      const int od = FLIP ? 2 - td : td, oh = FLIP ? 2 - th : th, ow = FLIP ? 2 - tw : tw;
      return ((od * CB_HH + oh) * CB_HW + ow) * 16 + 2 * s * CB_PS;
    };
    auto boff = [](int st) { return (2 * (st & 1) * CB_NWR + (st >> 1) * 32) * 16; };
    bf16x8 ca0 = *reinterpret_cast<const bf16x8*>(abase + aoff(0));
    bf16x8 ca1 = *reinterpret_cast<const bf16x8*>(abase + aoff(0) + CB_HH * CB_HW * 16);
    bf16x8 cb = *reinterpret_cast<const bf16x8*>(bbase + boff(0));
#pragma unroll
    for (int st = 0; st < 54; ++st) {
      bf16x8 na0 = ca0, na1 = ca1, nb = cb;
      if (st + 1 < 54) {
        na0 = *reinterpret_cast<const bf16x8*>(abase + aoff(st + 1));
        na1 = *reinterpret_cast<const bf16x8*>(abase + aoff(st + 1) + CB_HH * CB_HW * 16);
        nb = *reinterpret_cast<const bf16x8*>(bbase + boff(st + 1));
      }
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ca0, cb, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ca1, cb, acc1, 0, 0, 0);
      ca0 = na0;
      ca1 = na1;
      cb = nb;
    }
    __syncthreads();  // all waves done reading the halo before it is overwritten
    if (more) commit(bn);
    // epilogue through the wave's LDS tile: lane column co = r, rows w = (i&3) + 8(i>>2) + 4h of w-row
    // (d0+tm, h0+wave) -> [w][co] bf16, read back as 16-B chunks (one fully coalesced 1 KB store per row half)
#pragma unroll
    for (int tm = 0; tm < 2; ++tm) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int w = (i & 3) + 8 * (i >> 2) + 4 * h;
        *reinterpret_cast<bf16*>(ept + w * 64 + r * 2) = from_f<bf16>(tm ? acc1[i] : acc0[i]);
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int q = lane + 64 * u;
        u32x4 v = *reinterpret_cast<const u32x4*>(ept + q * 16);
        if (res) {
          float a[8], c[8];
          load16<bf16>(reinterpret_cast<const bf16*>(&v), a);
          load16<bf16>(reinterpret_cast<const bf16*>(&rv[tm][u]), c);
#pragma unroll
          for (int e = 0; e < 8; ++e) a[e] += c[e];
          store16<bf16>(reinterpret_cast<bf16*>(&v), a);
        }
        if (ok[tm]) *reinterpret_cast<u32x4*>(y + orow[tm] * 32 + q * 8) = v;
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
    }
    __syncthreads();
  }
}

}  // namespace u3d

using namespace u3d;

extern "C" int u3d_conv32_brick(int flip, const void* x, int n, int d, int h, int w, const void* wpk,
                                const float* gn_stats, const float* gn_gamma, const float* gn_beta, int gn_groups,
                                const void* residual, void* y, u3d_stream_t stream) {
  U3D_REQUIRE(x && wpk && y && n >= 1 && n <= CB_MAXN, "conv32_brick: bad args (n <= %d)", CB_MAXN);
  U3D_REQUIRE(!gn_stats || (gn_gamma && gn_beta && gn_groups > 0 && 32 % gn_groups == 0), "conv32_brick: bad GN");
  CBGeom g{};
  g.n = n; g.d = d; g.h = h; g.w = w;
  g.nbd = cdiv(d, CB_BD); g.nbh = cdiv(h, CB_BH); g.nbw = cdiv(w, CB_BW);
  g.nbricks = n * g.nbd * g.nbh * g.nbw;
  g.gn_groups = gn_groups;
  const int grid = std::min(g.nbricks, 256);
  hipStream_t s = (hipStream_t)stream;
  if (flip)
    hipLaunchKernelGGL(conv32_brick_kernel<true>, dim3(grid), dim3(CB_NT), 0, s, (const bf16*)x, (const bf16*)wpk,
                       (bf16*)y, (const bf16*)residual, gn_stats, gn_gamma, gn_beta, g);
  else
    hipLaunchKernelGGL(conv32_brick_kernel<false>, dim3(grid), dim3(CB_NT), 0, s, (const bf16*)x, (const bf16*)wpk,
                       (bf16*)y, (const bf16*)residual, gn_stats, gn_gamma, gn_beta, g);
  return check_launch("conv32_brick_kernel");
}
