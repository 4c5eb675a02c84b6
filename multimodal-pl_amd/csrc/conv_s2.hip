// Stride-2 3^3 convolution forward (pad 1), bf16, halo-brick form with the GroupNorm+ReLU prologue at staging.
//
// Reference: F.conv3d(stride=2, padding=1) in Conv3d.forward (unet3D.py:27) — conv1 of the first NoBottleneck of
// layer1..4 (_make_layer unet3D.py:1666-1686), the encoder's down-sampling convs.
//
// The implicit GEMM ran these at ~11% of the MFMA peak: every K step gathered a 128-voxel A tile from L2 at one tap's
// shifted, stride-2 positions (27 gathers of the same input per output tile). Here one workgroup owns an output brick
// of 2 x 4 x 16 voxels x one 32-channel co tile and stages its input halo (5 x 9 x 33 voxels, the receptive field of
// the brick) ONCE per 32-channel chunk, with GN + ReLU applied once per element; all 27 taps read it from LDS.
//   * LDS: halo chunk-planar (plane = 8 channels, 16 B per halo row) with the w axis parity-split (even w first, then
//     odd): tap c = 0 / 1 / 2 of an output row of 16 voxels reads 16 CONSECUTIVE rows (even, odd, even+1), so the
//     16-lane groups of ds_read_b128 are conflict-free; the 27 taps' weights of the chunk [plane][tap][co] (55 KB);
//   * MFMA transposed (A = weights, B = halo rows): a lane's accumulators are 16 channels of one voxel, stored as
//     two 16-B chunks after one v_permlane32_swap per pair (no LDS epilogue tile);
//   * 8 waves: wave w owns row tile w & 3 (32 voxels = 2 h-rows x 16 w) and k16 half w >> 2 of every tap (27
//     MFMAs per chunk); the two halves are added through LDS in the epilogue;
//   * persistent workgroups (LDS admits one per CU) walk (brick, co tile) units with the next unit's / chunk's halo
//     and weights loaded into registers while the current one's MFMAs run.
#include "common.h"

namespace u3d {

constexpr int F2_BD = 2, F2_BH = 4, F2_BW = 16;                         // output brick
constexpr int F2_HD = 2 * F2_BD + 1, F2_HH = 2 * F2_BH + 1, F2_HW = 2 * F2_BW + 1;  // input halo 5 x 9 x 33
constexpr int F2_NH = F2_HD * F2_HH * F2_HW;                             // 1485 rows
constexpr int F2_NT = 512;
constexpr int F2_PS = F2_NH * 16 + 64;                                   // halo plane stride (+64 B: staging writes)
constexpr int F2_HLD = (F2_NH * 4 + F2_NT - 1) / F2_NT;                  // 12 halo loads per thread
constexpr int F2_WR = 27 * 32;                                           // weight rows per plane (tap, co)
constexpr int F2_WPS = F2_WR * 16 + 64;
constexpr int F2_WLD = (F2_WR * 4 + F2_NT - 1) / F2_NT;                  // 7 weight loads per thread

struct F2Geom {
  int n, d, h, w;        // input
  int od, oh, ow;        // output
  int cin, cin_p, cout, cout_p;
  int nbd, nbh, nbw, nct;
  int units;             // n * bricks * co tiles
  int groups;
  int nbrick;            // n * bricks
};

__device__ __forceinline__ int f2_seg(int r) {  // as gb_seg / gb_pos of conv_brick_gen.hip: 16-lane groups read
  return (r < 4 || (r >= 12 && r < 16) || (r >= 20 && r < 28)) ? 0 : 1;  // 16 consecutive w of one h-row
}
__device__ __forceinline__ int f2_pos(int r) {
  if (r < 4) return r;
  if (r < 12) return r - 4;
  if (r < 20) return r - 8;
  if (r < 28) return r - 12;
  return r - 16;
}

template <bool GN>
__global__ __launch_bounds__(F2_NT, 1) void convs2_fwd_kernel(const bf16* __restrict__ x, const bf16* __restrict__ wpk,
                                                             bf16* __restrict__ y, const float* __restrict__ gstat,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ beta, F2Geom g) {
  __shared__ __attribute__((aligned(16))) char hal[4 * F2_PS];
  __shared__ __attribute__((aligned(16))) char wl[4 * F2_WPS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, hh = lane >> 5;
  const int rt = wave & 3, kk = wave >> 2;
  const int nchunk = g.cin_p / 32;

  // this lane's B row (tap (0,0,0)) for its voxel (vd, vh, vw) of row tile rt
  const int vd = rt >> 1, vh = 2 * (rt & 1) + f2_seg(r), vw = f2_pos(r);
  const int brow = ((2 * vd) * F2_HH + 2 * vh) * F2_HW + vw;

  auto unit_geom = [&](int u, int& nn, int& d0, int& h0, int& w0, int& co0) __attribute__((always_inline)) {
    const int ct = u % g.nct;
    int b = u / g.nct;
    const int bw = b % g.nbw;
    b /= g.nbw;
    const int bh = b % g.nbh;
    b /= g.nbh;
    const int bd = b % g.nbd;
    nn = b / g.nbd;
    d0 = bd * F2_BD;
    h0 = bh * F2_BH;
    w0 = bw * F2_BW;
    co0 = ct * 32;
  };

  // staging: thread -> (halo row q >> 2, plane q & 3): 4 lanes read one voxel's 64 B of the chunk
  u32x4 hpre[F2_HLD], wpre[F2_WLD];
  unsigned hok = 0;  // bit i: halo load i is inside the volume (GN is applied to those only; the rest stay 0)
  int cur_nn = 0;
  auto stage_load = [&](int u, int c, bool wts = true) __attribute__((always_inline)) {
    int nn, d0, h0, w0, co0;
    unit_geom(u, nn, d0, h0, w0, co0);
    hok = 0;
#pragma unroll
    for (int i = 0; i < F2_HLD; ++i) {
      const int q = tid + i * F2_NT, row = q >> 2, pl = q & 3;
      const int hw = row % F2_HW, hr = (row / F2_HW) % F2_HH, hd = row / (F2_HW * F2_HH);
      const int zd = 2 * d0 - 1 + hd, zh = 2 * h0 - 1 + hr, zw = 2 * w0 - 1 + hw;
      const bool ok = row < F2_NH && (unsigned)zd < (unsigned)g.d && (unsigned)zh < (unsigned)g.h &&
                      (unsigned)zw < (unsigned)g.w && c * 32 + pl * 8 < g.cin;
      const long long off = ok ? ((((long long)nn * g.d + zd) * g.h + zh) * g.w + zw) * g.cin + c * 32 + pl * 8 : 0;
      const u32x4 v = *reinterpret_cast<const u32x4*>(x + off);  // clamped address: straight-line loads
      hpre[i] = ok ? v : (u32x4){0u, 0u, 0u, 0u};
      hok |= (ok ? 1u : 0u) << i;
    }
#pragma unroll
    for (int i = 0; i < F2_WLD; ++i) {  // q -> (tap, co, plane), plane fastest: 64 contiguous bytes per 4 lanes
      if (!wts) break;
      const int q = tid + i * F2_NT, pl = q & 3, tc = q >> 2, t = tc >> 5, co = co0 + (tc & 31);
      const bool ok = q < F2_WR * 4 && co < g.cout_p;
      const u32x4 v = *reinterpret_cast<const u32x4*>(
          wpk + (ok ? ((long long)t * g.cout_p + co) * g.cin_p + c * 32 + pl * 8 : 0));
      wpre[i] = ok ? v : (u32x4){0u, 0u, 0u, 0u};
    }
    cur_nn = nn;
  };
  auto stage_commit = [&](int c, bool wts = true) __attribute__((always_inline)) {
    f32x2 sc[4], sh[4];
    if constexpr (GN) gn_coef8(gstat, gamma, beta, g.groups, g.cin, cur_nn, c * 32 + (tid & 3) * 8, sc, sh);
#pragma unroll
    for (int i = 0; i < F2_HLD; ++i) {
      const int q = tid + i * F2_NT, row = q >> 2, pl = q & 3;
      if (row < F2_NH) {
        const int hw = row % F2_HW, line = row / F2_HW;
        const int lrow = line * F2_HW + ((hw & 1) ? (F2_HW + 1) / 2 + (hw >> 1) : (hw >> 1));
        u32x4 v = hpre[i];
        if constexpr (GN) {
          const u32x4 a = gn_relu8(v, sc, sh);
          v = ((hok >> i) & 1u) ? a : v;
        }
        *reinterpret_cast<u32x4*>(hal + pl * F2_PS + lrow * 16) = v;
      }
    }
#pragma unroll
    for (int i = 0; i < F2_WLD; ++i) {
      if (!wts) break;
      const int q = tid + i * F2_NT, pl = q & 3, tc = q >> 2;
      if (q < F2_WR * 4) *reinterpret_cast<u32x4*>(wl + pl * F2_WPS + tc * 16) = wpre[i];
    }
  };

  // Walk: workgroup i runs on XCD i % 8 (round-robin dispatch). The bricks are split into 8 contiguous ranges, one
  // per XCD; on an XCD, slot s = i / 8 works co tile s % nct of brick stream s / nct, so the nct workgroups of a stream
  // read the same halos at about the same time through that XCD's L2, and a workgroup keeps one co tile (with one
  // 32-channel chunk its weights are staged once).
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, nslot = gridDim.x >> 3;
  const int ct = slot % g.nct, stream = slot / g.nct, nstream = nslot / g.nct;
  const int b_lo = (int)((long long)g.nbrick * xcd / 8), b_hi = (int)((long long)g.nbrick * (xcd + 1) / 8);
  int bk = b_lo + stream, c = 0;
  if (stream >= nstream || bk >= b_hi) return;
  int u = bk * g.nct + ct;
  stage_load(u, 0);
  stage_commit(0);
  __syncthreads();
  f32x16 acc = (f32x16){};
  for (;;) {
    // the next step's loads fly under this step's MFMAs
    int nbk = bk, nc = c + 1;
    if (nc == nchunk) {
      nc = 0;
      nbk = bk + nstream;
    }
    const bool more = nbk < b_hi;
    const int nu = nbk * g.nct + ct;
    const bool wsame = nchunk == 1;  // same co tile, same chunk: the weights in LDS stay valid
    if (more) stage_load(nu, nc, !wsame);
    {
      const int pl = 2 * kk + hh;
      const char* hb = hal + pl * F2_PS + brow * 16;
      const char* wb = wl + pl * F2_WPS + r * 16;
#pragma unroll
      for (int t = 0; t < 27; ++t) {
        const int ta = t / 9, tb = (t / 3) % 3, tcw = t % 3;
        const int toff = (ta * F2_HH + tb) * F2_HW + (tcw == 1 ? (F2_HW + 1) / 2 : tcw == 2 ? 1 : 0);
        const s16x8 a = *reinterpret_cast<const s16x8*>(wb + t * 32 * 16);
        const s16x8 b = *reinterpret_cast<const s16x8*>(hb + toff * 16);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
      }
    }
    __syncthreads();  // every wave done with this step's LDS data
    if (c == nchunk - 1) {
      // epilogue of unit u: k16 halves added through LDS (the halo region is free until the next commit)
      float* red = reinterpret_cast<float*>(hal) + rt * 16 * 64;
      if (kk == 1)
#pragma unroll
        for (int i = 0; i < 16; ++i) red[i * 64 + lane] = acc[i];
      __syncthreads();
      if (kk == 0) {
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] += red[i * 64 + lane];
        int nn, d0, h0, w0, co0;
        unit_geom(u, nn, d0, h0, w0, co0);
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
        const int zd = d0 + vd, zh = h0 + vh, zw = w0 + vw;
        if (zd < g.od && zh < g.oh && zw < g.ow) {
          bf16* yp = y + ((((long long)nn * g.od + zd) * g.oh + zh) * g.ow + zw) * g.cout + co0 + 8 * hh;
#pragma unroll
          for (int v2 = 0; v2 < 2; ++v2)
            if (co0 + 16 * v2 + 8 * hh < g.cout)
              *reinterpret_cast<u32x4*>(yp + 16 * v2) =
                  (u32x4){pk[2 * v2][0], pk[2 * v2][1], pk[2 * v2 + 1][0], pk[2 * v2 + 1][1]};
        }
      }
      acc = (f32x16){};
      __syncthreads();  // the reduction scratch is read before the commit overwrites it
    }
    if (!more) break;
    u = nu;
    bk = nbk;
    c = nc;
    stage_commit(c, !wsame);
    __syncthreads();
  }
}

}  // namespace u3d

using namespace u3d;

extern "C" int u3d_conv_fwd_s2(const void* x, int n, int cin, int d, int h, int w, const void* wpk, int cout,
                               const float* gn_stats, const float* gn_gamma, const float* gn_beta, int gn_groups,
                               void* y, u3d_stream_t stream) {
  U3D_REQUIRE(x && wpk && y && n >= 1 && d >= 1 && h >= 1 && w >= 1, "conv_fwd_s2: bad args");
  U3D_REQUIRE(cin % 8 == 0 && cout % 8 == 0, "conv_fwd_s2: channels must be multiples of 8");
  U3D_REQUIRE(!gn_stats || (gn_gamma && gn_beta && gn_groups > 0 && cin % gn_groups == 0), "conv_fwd_s2: bad GN");
  F2Geom g{};
  g.n = n; g.d = d; g.h = h; g.w = w;
  g.od = (d - 1) / 2 + 1; g.oh = (h - 1) / 2 + 1; g.ow = (w - 1) / 2 + 1;
  g.cin = cin; g.cin_p = round_up(cin, 32); g.cout = cout; g.cout_p = round_up(cout, 32);
  g.nbd = cdiv(g.od, F2_BD); g.nbh = cdiv(g.oh, F2_BH); g.nbw = cdiv(g.ow, F2_BW);
  g.nct = g.cout_p / 32;
  const long long units = (long long)n * g.nbd * g.nbh * g.nbw * g.nct;
  U3D_REQUIRE(units < (1LL << 30), "conv_fwd_s2: too many units");
  g.units = (int)units;
  g.nbrick = (int)(units / g.nct);
  g.groups = gn_stats ? gn_groups : 0;
  static const int cus = [] {
    int dev = 0, m = 256;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess) m = prop.multiProcessorCount;
    return m;
  }();
  // 8 XCDs x (slots per XCD, a multiple of the co tiles); one workgroup per CU (LDS)
  const int per_xcd = std::max(g.nct, cus / 8 / g.nct * g.nct);
  U3D_REQUIRE(g.nct <= 32, "conv_fwd_s2: cout %d > 1024", cout);
  const int grid = 8 * per_xcd;
  hipStream_t s = (hipStream_t)stream;
  if (gn_stats)
    hipLaunchKernelGGL(convs2_fwd_kernel<true>, dim3(grid), dim3(F2_NT), 0, s, (const bf16*)x, (const bf16*)wpk,
                       (bf16*)y, gn_stats, gn_gamma, gn_beta, g);
  else
    hipLaunchKernelGGL(convs2_fwd_kernel<false>, dim3(grid), dim3(F2_NT), 0, s, (const bf16*)x, (const bf16*)wpk,
                       (bf16*)y, nullptr, nullptr, nullptr, g);
  return check_launch("convs2_fwd_kernel");
}
