// Stride-2 3^3 data gradient (the transposed convolution of a stride-2 forward conv), bf16, one launch.
//
// Reference: autograd of F.conv3d(stride=2, padding=1) in Conv3d.forward (unet3D.py:27) for the first conv of
// every down-sampling NoBottleneck (layer1..4 .0.conv1, _make_layer unet3D.py:1666-1686).
//
// dx[2q + p] = sum over the taps of parity class p of dy[q + delta] . W[tap]: per dim, p = 0 takes tap 1 at
// delta 0, p = 1 takes tap 0 at delta 1 and tap 2 at delta 0 — the 27 taps split into 8 parity classes, and
// the dy window a tap reads is one of 8 shifts delta in {0,1}^3 of a q-brick.
//   * one workgroup (4 waves; 8 in the U3D_S2_NT = 512 build) = one q-brick of up to 128 (256) dy voxels x one
//     32-channel dx tile; each wave owns 32 q rows and ALL 8 parity accumulators (8 x 32x32 fp32), so one
//     workgroup writes the whole 2x-sized dx region of its brick: every dx voxel is produced once, with no
//     zero-fill and no per-class launches;
//   * K loop = 32-channel dy chunks: the dy halo ((bd+1)(bh+1)(bw+1) voxels) and the 27 taps' weights of
//     the chunk are staged once in LDS (chunk-planar, padded planes: conflict-free staging writes); each of
//     the 8 shifted A fragments is read once per k16 step and feeds the 1..8 taps that use that shift;
//   * two workgroups per CU: one's chunk loads and dx stores run under the other's MFMAs (the 512-thread build
//     prefetches the next chunk into registers instead);
//   * the MFMA is issued transposed (A = weights, B = dy rows), so a lane's accumulators are dx channels of one voxel:
//     the epilogue stores them as 16-B chunks straight from registers (one v_permlane32_swap per pair).
#include "common.h"

namespace u3d {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;

// U3D_S2_NT = 256 (default since round 4): 4-wave workgroups of up to 128 q voxels, two per CU (76 KB of LDS and 248
// VGPRs each), no register prefetch — the other workgroup's MFMAs cover a workgroup's loads and dx stores; 512: one
// 8-wave workgroup per CU (236 VGPRs), the next chunk prefetched into registers under its own MFMAs. Kernel A/B
// (2 x 96^3 / 48^3 / 24^3 / 12^3 levels, gpurun_out/r04_h): 64 / 38.8 / 30.2 / 29.1 -> 62.6 / 28.2 / 26.9 / 24.3 us
#ifndef U3D_S2_NT
#define U3D_S2_NT 256
#endif
constexpr int S2_NT = U3D_S2_NT;
constexpr bool S2_PF = S2_NT == 512;             // register prefetch of the next chunk
constexpr int S2_MAXQ = S2_NT / 2;               // q voxels per brick (32 per wave)
constexpr int S2_HMAX = S2_NT == 512 ? 512 : 320;  // halo rows (max)
constexpr int S2_PS = S2_HMAX * 16 + 64;         // halo plane stride
constexpr int S2_NWR = 27 * 32;                  // weight rows (tap, co)
constexpr int S2_WPS = S2_NWR * 16 + 64;         // weight plane stride
constexpr int S2_HLD = S2_HMAX * 4 / S2_NT;      // 4 halo loads per thread
constexpr int S2_WLD = (S2_NWR * 4 + S2_NT - 1) / S2_NT;  // 7 weight loads per thread
constexpr int S2_LDS = 4 * S2_PS + 4 * S2_WPS;

struct S2Geom {
  int n, qd, qh, qw;       // dy spatial dims (the forward's output)
  int D, H, W;             // dx spatial dims (the forward's input)
  int cy, cy_p, cx, cx_p;  // dy channels (contraction), dx channels (output)
  int bd, bh, bw;          // q-brick
  int hh, hw, nh;          // halo pitch (bh+1, bw+1) and rows
  int nbd, nbh, nbw, nct;  // bricks per dim, 32-wide dx channel tiles
  int nvq;                 // q voxels per brick (<= S2_MAXQ)
};

__global__ __launch_bounds__(S2_NT, 512 / S2_NT) void dgrad_s2_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ wpk,
                                                           bf16* __restrict__ dx, S2Geom g) {
  __shared__ __attribute__((aligned(16))) char smem[S2_LDS];
  char* const hal = smem;
  char* const wts = smem + 4 * S2_PS;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;

  int bid;  // XCD-aware: each XCD owns a contiguous range of (brick, co tile) -> shared halo rows in its L2
  {
    const int nwg = gridDim.x, q = nwg >> 3, rr = nwg & 7, xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
    bid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + loc;
  }
  int b = bid / g.nct;
  const int co0 = (bid - b * g.nct) * 32;
  const int bw_ = b % g.nbw; b /= g.nbw;
  const int bh_ = b % g.nbh; b /= g.nbh;
  const int bd_ = b % g.nbd;
  const int nn = b / g.nbd;
  const int q0d = bd_ * g.bd, q0h = bh_ * g.bh, q0w = bw_ * g.bw;

  static_assert(S2_NT == 512 || S2_NT == 256, "workgroup size");
  // this lane's q row (clamped into the brick for the idle rows of the last tile)
  const int v = min(wave * 32 + r, g.nvq - 1);
  const int vw = v % g.bw, vh = (v / g.bw) % g.bh, vd = v / (g.bw * g.bh);
  const int arow = (vd * g.hh + vh) * g.hw + vw;
  const bool active = wave * 32 < g.nvq;

  const int sch = tid & 3, srow0 = tid >> 2;
  u32x4 hpre[S2_HLD], wpre[S2_WLD];
  // buffer loads with 32-bit offsets (host: operands below 2 GiB); a masked piece gets the out-of-range sentinel and
  // reads zeros with no branch around the load, so the prefetch's wait is not pulled up to a branch merge ahead of
  // the MFMAs it should overlap
  const auto yrs = __builtin_amdgcn_make_buffer_rsrc((void*)dy, 0, g.n * g.qd * g.qh * g.qw * g.cy * 2, 0x00020000);
  const auto wrs = __builtin_amdgcn_make_buffer_rsrc((void*)wpk, 0, 27 * g.cx_p * g.cy_p * 2, 0x00020000);
  auto halo_load = [&](int c) {
#pragma unroll
    for (int i = 0; i < S2_HLD; ++i) {
      const int row = srow0 + i * (S2_NT / 4);
      const int xw = row % g.hw, xh = (row / g.hw) % g.hh, xd = row / (g.hw * g.hh);
      const int zd = q0d + xd, zh = q0h + xh, zw = q0w + xw, cc = c * 32 + sch * 8;
      const bool ok = row < g.nh && zd < g.qd && zh < g.qh && zw < g.qw && cc < g.cy;
      const unsigned off = ok ? (unsigned)(((((nn * g.qd + zd) * g.qh + zh) * g.qw + zw) * g.cy + cc) * 2) : 0xFFFFFFF0u;
      hpre[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(yrs, off, 0, 0));
    }
  };
  auto w_load = [&](int c) {  // rows (tap t, co): 4 consecutive threads read one row's 64 B
#pragma unroll
    for (int i = 0; i < S2_WLD; ++i) {
      const int id = tid + i * S2_NT;
      const int row = id >> 2, t = row >> 5, co = co0 + (row & 31);
      const bool ok = id < S2_NWR * 4 && co < g.cx_p;
      const unsigned off = ok ? (unsigned)(((t * g.cx_p + co) * g.cy_p + c * 32 + (id & 3) * 8) * 2) : 0xFFFFFFF0u;
      wpre[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wrs, off, 0, 0));
    }
  };
  auto commit = [&]() {
#pragma unroll
    for (int i = 0; i < S2_HLD; ++i) {
      const int row = srow0 + i * (S2_NT / 4);
      if (row < g.nh) *reinterpret_cast<u32x4*>(hal + sch * S2_PS + row * 16) = hpre[i];
    }
#pragma unroll
    for (int i = 0; i < S2_WLD; ++i) {
      const int id = tid + i * S2_NT;
      if (id < S2_NWR * 4) *reinterpret_cast<u32x4*>(wts + (id & 3) * S2_WPS + (id >> 2) * 16) = wpre[i];
    }
  };

  f32x16 acc[8];
#pragma unroll
  for (int p = 0; p < 8; ++p)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[p][e] = 0.f;

  const int nchunk = g.cy_p / 32;
  halo_load(0);
  w_load(0);
  commit();
  __syncthreads();
  for (int c = 0; c < nchunk; ++c) {
    const bool more = c + 1 < nchunk;
    if (S2_PF && more) {
      halo_load(c + 1);
      w_load(c + 1);
    }
    if (active) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int plane = 2 * s + hh;
        const char* ab = hal + plane * S2_PS + arow * 16;
        const char* bb = wts + plane * S2_WPS + r * 16;
        // shift (dd, dh, dw) in {0,1}^3; per dim: shift 1 -> (tap 0, p 1); shift 0 -> (tap 1, p 0), (tap 2, p 1)
#pragma unroll
        for (int sh = 0; sh < 8; ++sh) {
          const int dd = sh >> 2, dh = (sh >> 1) & 1, dw = sh & 1;
          const bf16x8 a = *reinterpret_cast<const bf16x8*>(ab + ((dd * g.hh + dh) * g.hw + dw) * 16);
#pragma unroll
          for (int kd = 0; kd < (dd ? 1 : 2); ++kd)
#pragma unroll
            for (int kh = 0; kh < (dh ? 1 : 2); ++kh)
#pragma unroll
              for (int kw = 0; kw < (dw ? 1 : 2); ++kw) {
                const int td = dd ? 0 : 1 + kd, th = dh ? 0 : 1 + kh, tw = dw ? 0 : 1 + kw;
                const int p = ((td != 1) << 2) | ((th != 1) << 1) | (tw != 1);
                const int t = (td * 3 + th) * 3 + tw;
                const bf16x8 bv = *reinterpret_cast<const bf16x8*>(bb + t * 32 * 16);
                acc[p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bv, a, acc[p], 0, 0, 0);  // D[dx ch][voxel]
              }
        }
      }
    }
    __syncthreads();
    if (more) {
      if (!S2_PF) {
        halo_load(c + 1);
        w_load(c + 1);
      }
      commit();
      __syncthreads();
    }
  }

  // epilogue straight from the accumulators (the MFMA is issued transposed: A = weights, B = dy rows): lane (r, hh)
  // holds dx channels 8q + 4hh + e (q, e < 4) of q voxel r in every parity class; one v_permlane32_swap per pair
  // leaves it channels 8hh..8hh+7 and 16+8hh..16+8hh+7, stored as two 16-B chunks per class (no LDS pass)
  const int vv = wave * 32 + r;
  const int uw = vv % g.bw, uh = (vv / g.bw) % g.bh, ud = vv / (g.bw * g.bh);
  const bool qok = active && vv < g.nvq && q0d + ud < g.qd && q0h + uh < g.qh && q0w + uw < g.qw;
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    uint32_t pk[4][2];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int e = 0; e < 2; ++e) pk[q][e] = pack_bf16x2(acc[p][4 * q + 2 * e], acc[p][4 * q + 2 * e + 1]);
#pragma unroll
    for (int q = 0; q < 4; q += 2)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const auto sw = __builtin_amdgcn_permlane32_swap(pk[q][e], pk[q + 1][e], false, false);
        pk[q][e] = sw[0];
        pk[q + 1][e] = sw[1];
      }
    const int xd = 2 * (q0d + ud) + (p >> 2), xh = 2 * (q0h + uh) + ((p >> 1) & 1), xw = 2 * (q0w + uw) + (p & 1);
    if (qok && xd < g.D && xh < g.H && xw < g.W) {
      bf16* const row = dx + ((((long long)nn * g.D + xd) * g.H + xh) * g.W + xw) * g.cx;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int co = co0 + 16 * u + 8 * hh;
        if (co < g.cx)
          *reinterpret_cast<u32x4*>(row + co) = (u32x4){pk[2 * u][0], pk[2 * u][1], pk[2 * u + 1][0], pk[2 * u + 1][1]};
      }
    }
  }
}

}  // namespace u3d

using namespace u3d;

// dy [n, od, oh, ow, cout] (od = (d-1)/2+1 ...) -> dx [n, d, h, w, cin]; W packed [27][cin_p][cout_p] (dgrad pack)
extern "C" int u3d_conv_dgrad_s2(const void* dy, int n, int cout, const void* wpk_dgrad, int cin, int d, int h, int w,
                                 void* dx, u3d_stream_t stream) {
  U3D_REQUIRE(dy && wpk_dgrad && dx && n >= 1 && d >= 1 && h >= 1 && w >= 1, "conv_dgrad_s2: bad args");
  U3D_REQUIRE(cout % 8 == 0 && cin % 8 == 0, "conv_dgrad_s2: channels must be multiples of 8");
  S2Geom g{};
  g.n = n;
  g.D = d; g.H = h; g.W = w;
  g.qd = (d - 1) / 2 + 1; g.qh = (h - 1) / 2 + 1; g.qw = (w - 1) / 2 + 1;
  g.cy = cout; g.cy_p = round_up(cout, 32); g.cx = cin; g.cx_p = round_up(cin, 32);
  // q-brick: up to S2_MAXQ voxels, w extent first (contiguous dy rows), extents that tile the volume evenly,
  // halo <= S2_HMAX rows
  auto even = [](int q, int mx) { return cdiv(q, cdiv(q, std::max(1, mx))); };
  g.bw = even(g.qw, 16);
  g.bh = even(g.qh, S2_MAXQ / (g.bw * 2));
  g.bd = even(g.qd, std::min(g.qd, S2_MAXQ / (g.bw * g.bh)));
  while ((g.bd + 1) * (g.bh + 1) * (g.bw + 1) > S2_HMAX && g.bd > 1) --g.bd;
  while ((g.bd + 1) * (g.bh + 1) * (g.bw + 1) > S2_HMAX && g.bh > 1) --g.bh;
  U3D_REQUIRE((g.bd + 1) * (g.bh + 1) * (g.bw + 1) <= S2_HMAX, "conv_dgrad_s2: halo too large");
  g.nvq = g.bd * g.bh * g.bw;
  g.hh = g.bh + 1; g.hw = g.bw + 1;
  g.nh = (g.bd + 1) * g.hh * g.hw;
  g.nbd = cdiv(g.qd, g.bd); g.nbh = cdiv(g.qh, g.bh); g.nbw = cdiv(g.qw, g.bw);
  g.nct = g.cx_p / 32;
  const long long nwg = (long long)n * g.nbd * g.nbh * g.nbw * g.nct;
  U3D_REQUIRE(nwg < (1LL << 31), "conv_dgrad_s2: grid too large");
  U3D_REQUIRE((long long)n * g.qd * g.qh * g.qw * g.cy * 2 < (1LL << 31) - 64 &&
              27LL * g.cx_p * g.cy_p * 2 < (1LL << 31) - 64,
              "conv_dgrad_s2: dy / weights beyond the 2 GiB buffer-offset range");
  hipLaunchKernelGGL(dgrad_s2_kernel, dim3((unsigned)nwg), dim3(S2_NT), 0, (hipStream_t)stream, (const bf16*)dy,
                     (const bf16*)wpk_dgrad, (bf16*)dx, g);
  return check_launch("dgrad_s2_kernel");
}
