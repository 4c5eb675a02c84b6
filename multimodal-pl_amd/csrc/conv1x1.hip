// 1^3 convolution, stride 1 or 2, bf16, as a streaming GEMM with the GroupNorm+ReLU prologue applied to the
// operand in registers: y[n, vo, :] = W . relu(gn(x))[n, vi(vo), :].
//
// Reference: the 1^3 convs of the U-Net (F.conv3d in Conv3d.forward, unet3D.py:27): the downsample branch of each
// stage's first NoBottleneck (GN -> ReLU -> conv 1^3 stride 2, _make_layer unet3D.py:1666-1686) and of the decoder
// blocks whose channel count changes (stride 1), and the stride-1 1^3 data gradients of the latter.
//
// These layers have 2 x cin x cout flops per voxel against (cin + cout) x 2 bytes: memory-bound. The generic implicit
// GEMM ran them latency-bound (one short-lived workgroup per 128-voxel tile: one load round, a few MFMAs, one store)
// and needed the GN materialised first for cin >= 64. Here:
//   * one workgroup = 4 waves on one (sample, group of up to 4 32-channel co tiles); the group's weights
//     [co][k] (<= 128 x 256 bf16) and the sample's GN scale/shift per input channel are staged once in LDS;
//   * each wave walks 32-voxel tiles of the sample (grid-stride); a lane loads its voxel's 16-B channel chunks
//     (stride 2: the voxel at (2d, 2h, 2w)) straight into the MFMA B fragment, applies GN + ReLU in registers, and
//     the NEXT tile's loads are issued before this tile's MFMAs, so HBM latency hides under the math;
//   * the MFMA is issued transposed (A = weights, B = voxels): a lane's accumulators are 16 channels of one voxel,
//     one v_permlane32_swap per pair turns them into two 16-B row stores.
#include "common.h"

namespace u3d {

constexpr int C1_NT = 256;

struct C1Geom {
  int n, d, h, w;     // input dims
  int od, oh, ow;     // output dims
  int stride;
  int cx, cy;         // input / output channels (multiples of 8)
  int wpitch;         // packed weight row pitch (elements)
  int groups;         // GN groups (0: no prologue)
  int vo;             // output voxels per sample
  int ntile;          // 32-voxel tiles per sample
};

template <int KS, int NCT, bool GN>
__global__ __launch_bounds__(C1_NT) void conv1x1_kernel(const bf16* __restrict__ x, const bf16* __restrict__ wpk,
                                                       bf16* __restrict__ y, const float* __restrict__ st,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, C1Geom g) {
  constexpr int K = KS * 16;
  constexpr int LDW = K + 8;  // +16 B per row: the 32 rows of an A fragment start in different banks
  __shared__ __attribute__((aligned(16))) bf16 wl[NCT * 32 * LDW];
  __shared__ __attribute__((aligned(16))) float cf[GN ? 2 * K : 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, hh = lane >> 5;
  const int n = blockIdx.y, co_base = blockIdx.z * NCT * 32;

  // weights of this co group: rows co_base .. +NCT*32 of the packed [cy_p][wpitch] image (zero padded). All of a
  // thread's loads are issued before its LDS writes (a load-store loop would pay one HBM latency per 16 B).
  {
    constexpr int NCH = NCT * 32 * (K / 8), PER = (NCH + C1_NT - 1) / C1_NT;
    const int rows = (g.cy + 31) & ~31;  // the image has round_up(cy, 32) rows
    u32x4 v[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = tid + j * C1_NT, row = i / (K / 8), ch = i - row * (K / 8);
      const bool ok = i < NCH && ch * 8 < g.wpitch && co_base + row < rows;
      const u32x4 t = *reinterpret_cast<const u32x4*>(wpk + (ok ? (long long)(co_base + row) * g.wpitch + ch * 8 : 0));
      v[j] = ok ? t : (u32x4){0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = tid + j * C1_NT, row = i / (K / 8), ch = i - row * (K / 8);
      if (i < NCH) *reinterpret_cast<u32x4*>(wl + row * LDW + ch * 8) = v[j];
    }
  }
  if constexpr (GN) {
    const int cpg = g.cx / g.groups;
    for (int c = tid; c < K; c += C1_NT) {
      float s = 0.f, b = 0.f;
      if (c < g.cx) {
        const int gr = c / cpg;
        const float mean = st[(n * g.groups + gr) * 2], rstd = st[(n * g.groups + gr) * 2 + 1];
        s = rstd * gamma[c];
        b = beta[c] - mean * s;
      }
      cf[c] = s;
      cf[K + c] = b;
    }
  }
  __syncthreads();

  const long long in_base = (long long)n * g.d * g.h * g.w;
  const long long out_base = (long long)n * g.vo;
  const int ohw = g.oh * g.ow;
  auto load_tile = [&](int t, u32x4 (&raw)[KS]) __attribute__((always_inline)) {
    int vo = t * 32 + r;
    vo = vo < g.vo ? vo : g.vo - 1;  // clamped: straight-line loads; the stores are guarded
    long long vi = vo;
    if (g.stride == 2) {
      const int a = vo / ohw, rem = vo - a * ohw, b = rem / g.ow, c = rem - b * g.ow;
      vi = ((long long)(2 * a) * g.h + 2 * b) * g.w + 2 * c;
    }
    const bf16* p = x + (in_base + vi) * g.cx;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {  // chunks past cx (cx % 16 == 8): clamped address, then zeroed by a select
      const int c = ks * 16 + 8 * hh;
      const u32x4 v = *reinterpret_cast<const u32x4*>(p + (c < g.cx ? c : g.cx - 8));
      raw[ks] = c < g.cx ? v : (u32x4){0u, 0u, 0u, 0u};
    }
  };

  const int stride_t = gridDim.x * 4;
  int t = blockIdx.x * 4 + wave;
  u32x4 raw[KS];
  if (t < g.ntile) load_tile(t, raw);
  for (; t < g.ntile; t += stride_t) {
    s16x8 bfr[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      u32x4 v = raw[ks];
      if constexpr (GN) {
        int c0 = ks * 16 + 8 * hh;
        asm volatile("" : "+v"(c0));  // opaque: keeps the LDS coefficient reads in the loop (hoisted, they took
                                      // 16 registers per k step and spilled at cx = 256)
        f32x2 sc[4], sh[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          sc[e] = (f32x2){cf[c0 + 2 * e], cf[c0 + 2 * e + 1]};
          sh[e] = (f32x2){cf[K + c0 + 2 * e], cf[K + c0 + 2 * e + 1]};
        }
        v = gn_relu8(v, sc, sh);  // channels past cx: scale = shift = 0 -> 0
      }
      bfr[ks] = __builtin_bit_cast(s16x8, v);
    }
    const int vo = t * 32 + r;
    if (t + stride_t < g.ntile) load_tile(t + stride_t, raw);  // next tile in flight under the MFMAs
    f32x16 acc[NCT];
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) acc[ct] = (f32x16){};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        const s16x8 a = *reinterpret_cast<const s16x8*>(wl + (ct * 32 + r) * LDW + ks * 16 + 8 * hh);
        acc[ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bfr[ks], acc[ct], 0, 0, 0);
      }
    // lane (r, hh): acc[ct][4q + e] = channel ct*32 + 8q + 4hh + e of voxel r -> after the swap, lane (r, hh) holds
    // channels 8hh..8hh+7 and 16+8hh..16+8hh+7 of the tile
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      uint32_t pk[4][2];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 2; ++e) pk[q][e] = pack_bf16x2(acc[ct][4 * q + 2 * e], acc[ct][4 * q + 2 * e + 1]);
#pragma unroll
      for (int q = 0; q < 4; q += 2)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const auto sw = __builtin_amdgcn_permlane32_swap(pk[q][e], pk[q + 1][e], false, false);
          pk[q][e] = sw[0];
          pk[q + 1][e] = sw[1];
        }
      if (vo < g.vo) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int co = co_base + ct * 32 + 16 * u + 8 * hh;
          if (co < g.cy)
            *reinterpret_cast<u32x4*>(y + (out_base + vo) * g.cy + co) =
                (u32x4){pk[2 * u][0], pk[2 * u][1], pk[2 * u + 1][0], pk[2 * u + 1][1]};
        }
      }
    }
  }
}

template <int KS, int NCT>
static void launch_c1(bool gn, dim3 grid, hipStream_t s, const bf16* x, const bf16* w, bf16* y, const float* st,
                      const float* ga, const float* be, const C1Geom& g) {
  if (gn)
    hipLaunchKernelGGL((conv1x1_kernel<KS, NCT, true>), grid, dim3(C1_NT), 0, s, x, w, y, st, ga, be, g);
  else
    hipLaunchKernelGGL((conv1x1_kernel<KS, NCT, false>), grid, dim3(C1_NT), 0, s, x, w, y, st, ga, be, g);
}

template <int KS>
static void launch_c1_k(int nct, bool gn, dim3 grid, hipStream_t s, const bf16* x, const bf16* w, bf16* y,
                        const float* st, const float* ga, const float* be, const C1Geom& g) {
  if (nct == 1) launch_c1<KS, 1>(gn, grid, s, x, w, y, st, ga, be, g);
  else if (nct == 2) launch_c1<KS, 2>(gn, grid, s, x, w, y, st, ga, be, g);
  else launch_c1<KS, 4>(gn, grid, s, x, w, y, st, ga, be, g);
}

}  // namespace u3d

using namespace u3d;

extern "C" int u3d_conv1x1(const void* x, int n, int cx, int d, int h, int w, const void* wpk, int wpitch, int cy,
                           int stride, const float* gn_stats, const float* gn_gamma, const float* gn_beta,
                           int gn_groups, void* y, u3d_stream_t stream) {
  U3D_REQUIRE(x && wpk && y && n >= 1 && n <= 65535 && d >= 1 && h >= 1 && w >= 1, "conv1x1: bad args");
  U3D_REQUIRE(cx % 8 == 0 && cy % 8 == 0 && cx <= 256 && cy <= 256 && wpitch >= cx, "conv1x1: channels (%d, %d)", cx,
              cy);
  U3D_REQUIRE(stride == 1 || stride == 2, "conv1x1: stride %d", stride);
  U3D_REQUIRE(!gn_stats || (gn_gamma && gn_beta && gn_groups > 0 && cx % gn_groups == 0), "conv1x1: bad GN");
  C1Geom g{};
  g.n = n; g.d = d; g.h = h; g.w = w;
  g.stride = stride;
  g.od = (d - 1) / stride + 1; g.oh = (h - 1) / stride + 1; g.ow = (w - 1) / stride + 1;
  const long long vo = (long long)g.od * g.oh * g.ow;
  U3D_REQUIRE(vo < (1LL << 31) - 64 && (long long)d * h * w < (1LL << 31), "conv1x1: volume too large");
  g.vo = (int)vo;
  g.ntile = (int)((vo + 31) / 32);
  g.cx = cx; g.cy = cy; g.wpitch = wpitch;
  g.groups = gn_stats ? gn_groups : 0;
  const int ks = cx <= 32 ? 2 : cx <= 64 ? 4 : cx <= 128 ? 8 : 16;
  const int nct_all = (cy + 31) / 32;
  const int nct = nct_all >= 4 ? 4 : nct_all >= 2 ? 2 : 1;  // co tiles per workgroup (1, 2, 4); the rest over grid.z
  const int gz = (nct_all + nct - 1) / nct;
  // enough workgroups for ~8 waves per CU over the whole launch, at least one tile per wave
  const long long want = std::max<long long>(1, 2048 / ((long long)n * gz));
  const int gx = (int)std::max<long long>(1, std::min<long long>(want, (g.ntile + 3) / 4));
  dim3 grid(gx, n, gz);
  hipStream_t s = (hipStream_t)stream;
  const bf16* xp = (const bf16*)x;
  const bf16* wp = (const bf16*)wpk;
  bf16* yp = (bf16*)y;
  const bool gn = gn_stats != nullptr;
  switch (ks) {
    case 2: launch_c1_k<2>(nct, gn, grid, s, xp, wp, yp, gn_stats, gn_gamma, gn_beta, g); break;
    case 4: launch_c1_k<4>(nct, gn, grid, s, xp, wp, yp, gn_stats, gn_gamma, gn_beta, g); break;
    case 8: launch_c1_k<8>(nct, gn, grid, s, xp, wp, yp, gn_stats, gn_gamma, gn_beta, g); break;
    default: launch_c1_k<16>(nct, gn, grid, s, xp, wp, yp, gn_stats, gn_gamma, gn_beta, g); break;
  }
  return check_launch("conv1x1_kernel");
}
