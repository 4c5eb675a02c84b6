// 3^3 stride-1 convolution (forward / data gradient) for the small deep-level volumes (24^3, 12^3, 6^3 of the
// 96^3 U-Net: 128 / 256 channels), bf16, halo-brick form sized for PARALLELISM rather than reuse.
//
// Reference: F.conv3d in Conv3d.forward (unet3D.py:27) through NoBottleneck (:56-73) at layer2..4, fusion and
// x8/x4 decoder blocks, and its autograd data gradient.
//
// At 12^3 x 2 samples a layer is 3456 output voxels x 256 channels = 864 output tiles of 32x32 with a
// 6912-deep contraction: the implicit GEMM's 128x128 tiles leave most CUs idle or need split-K slabs, and
// re-read every tap's operands through L2. Here:
//   * one workgroup (8 waves) = one brick of up to 256 output voxels x one 32-channel output tile; each wave
//     owns one 32-voxel row tile and the full contraction (27 taps x cin) -> no split-K, no slab traffic;
//   * the brick's extents divide the volume evenly (3x6x12 at 12^3, 6^3 whole at 6^3) so few rows idle;
//   * K loop = 32-channel input chunks: the input halo ((bd+2)(bh+2)(bw+2) voxels) is staged once per chunk
//     into LDS with GroupNorm + ReLU applied once per element, the 27 taps' weights of the chunk beside it;
//     the 27 taps are 27 shifted windows of the halo (per-lane row + tap offset); the next chunk is prefetched
//     into registers while the MFMAs run;
//   * epilogue through LDS: coalesced 64-B voxel rows, residual added on the way out.
// FLIP = data gradient: flipped tap offsets with the [t][ci][co] pack, no prologue.
#include "common.h"
#include "diag.h"

namespace u3d {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;

// U3D_SC_NT = 512: one 8-wave workgroup of up to 256 output voxels per CU (105 KB of LDS); 256: 4-wave workgroups
// of up to 128 voxels, two per CU (<= 80 KB each: smaller halo, GN table for cin <= 640)
#ifndef U3D_SC_NT
#define U3D_SC_NT 512
#endif
constexpr int SC_NT = U3D_SC_NT;
constexpr int SC_MAXV = SC_NT / 2;               // output voxels per brick (32 per wave)
constexpr int SC_HMAX = SC_NT == 512 ? 640 : 320;  // halo rows (max)
constexpr int SC_PS = SC_HMAX * 16 + 64;         // halo plane stride (+64 B: conflict-free staging writes)
constexpr int SC_NWR = 27 * 32;                  // weight rows (tap, co)
constexpr int SC_WPS = SC_NWR * 16 + 64;         // weight plane stride
constexpr int SC_HLD = SC_HMAX * 4 / SC_NT;      // 5 halo loads per thread
constexpr int SC_WLD = (SC_NWR * 4 + SC_NT - 1) / SC_NT;  // 7 weight loads per thread
constexpr int SC_LDS = 4 * SC_PS + 4 * SC_WPS;
constexpr int SC_MAXC = SC_NT == 512 ? 1024 : 640;  // GN prologue: cin_p <= SC_MAXC (per-channel table after SC_LDS)
static_assert(SC_NT == 512 || SC_LDS + SC_MAXC * 8 <= 81920, "two workgroups per CU");

struct SCGeom {
  int n, d, h, w;
  int cin, cin_p, cout, cout_p;
  int bd, bh, bw;          // output brick
  int hh, hw, nh;          // halo pitch (bh+2, bw+2) and rows
  int nbd, nbh, nbw, nct;  // bricks per dim, 32-wide output channel tiles
  int nv;                  // voxels per brick (<= 256)
  int gn_groups;
  int nks, cpk;            // K split: workgroups per output tile, 32-channel chunks per split
  float* slab;             // fp32 partials [nks][n][d][h][w][cout] when nks > 1
  // round 5: in-kernel split-K combine (cnt != nullptr, nks > 1) and optional output GroupNorm(16) statistics
  unsigned* cnt;           // [tiles + 1] zeroed arrival counters (per output tile, then one for the statistics)
  float* spart;            // [n][nbd*nbh*nbw][16][2] fp32 partials of the output statistics (stats != nullptr)
  float* stats;            // [n][16][2] (mean, rstd) of the output, or nullptr
  int cpg;                 // output channels per GroupNorm group (cout / 16; 4, 8 or 16)
  // round 5, data gradient (flip) through the combine: the backward of the GroupNorm + ReLU on x (the forward's input,
  // channels = this launch's cout) — per (sample, brick, channel) (sum g, sum g*xhat) of g = relu-mask * dA, then the
  // apply coefficients coef[n][5][cout] and dgamma / dbeta by the workgroup completing the last tile
  const bf16* gbx;
  const float *gbstat, *gbgamma, *gbbeta;
  int gbgroups;
  float* gbparts;          // [n][bricks][cout][2]
  float *coef, *dgamma, *dbeta;
};

// -DU3D_STAMPS phases (diag.h): 0 a chunk's MFMAs, 1 the next chunk's commit (GN + LDS writes) and its barrier, 2 the
// barrier after the MFMAs; "other" = the first chunk's loads and commit (the epilogue is after the last stamp)
U3D_STAMP_BUFFER(sc_stamps, 1024, u3d_diag_small_stamps)
U3D_STAMP_BUFFER(sc_tail, 256, u3d_diag_small_tail)  // TailStamps: 16 per workgroup

template <bool FLIP>
__global__ __launch_bounds__(SC_NT, 512 / SC_NT) void conv_small_kernel(const bf16* __restrict__ x, const bf16* __restrict__ wpk,
                                                             bf16* __restrict__ y, const bf16* __restrict__ res,
                                                             const float* __restrict__ gstat,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ beta, SCGeom g) {
  __shared__ __attribute__((aligned(16))) char smem[SC_LDS + SC_MAXC * 8];
  char* const hal = smem;
  char* const wts = smem + 4 * SC_PS;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  PhaseStamps ps;
  ps.begin();
  const int r = lane & 31, hh = lane >> 5;

  int bid;  // XCD-aware: each XCD owns a contiguous range of (brick, co tile)
  {
    const int nwg = gridDim.x, q = nwg >> 3, rr = nwg & 7, xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
    bid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + loc;
  }
  const int ks = bid % g.nks;
  int b = bid / g.nks;
  const int co0 = (b % g.nct) * 32;
  b /= g.nct;
  const int bw_ = b % g.nbw; b /= g.nbw;
  const int bh_ = b % g.nbh; b /= g.nbh;
  const int bd_ = b % g.nbd;
  const int nn = b / g.nbd;
  const int o0d = bd_ * g.bd, o0h = bh_ * g.bh, o0w = bw_ * g.bw;

  const int v = min(wave * 32 + r, g.nv - 1);
  const int vw = v % g.bw, vh = (v / g.bw) % g.bh, vd = v / (g.bw * g.bh);
  const int arow = (vd * g.hh + vh) * g.hw + vw;  // halo row of tap (0,0,0)
  const bool active = wave * 32 < g.nv;
  const bool has_gn = gstat != nullptr;

  const int sch = tid & 3, srow0 = tid >> 2;
  u32x4 hpre[SC_HLD], wpre[SC_WLD];
  unsigned hmask = 0;
  // buffer loads with 32-bit offsets (host: operands below 2 GiB); a masked piece gets the out-of-range sentinel and
  // reads zeros with no branch around the load (a branch merge pulls the prefetch's wait up ahead of the MFMAs)
  const auto xrs = __builtin_amdgcn_make_buffer_rsrc((void*)x, 0, g.n * g.d * g.h * g.w * g.cin * 2, 0x00020000);
  const auto wrs = __builtin_amdgcn_make_buffer_rsrc((void*)wpk, 0, 27 * g.cout_p * g.cin_p * 2, 0x00020000);
  auto halo_load = [&](int c) {
    unsigned m = 0;
#pragma unroll
    for (int i = 0; i < SC_HLD; ++i) {
      const int row = srow0 + i * (SC_NT / 4);
      const int xw = row % g.hw, xh = (row / g.hw) % g.hh, xd = row / (g.hw * g.hh);
      const int zd = o0d - 1 + xd, zh = o0h - 1 + xh, zw = o0w - 1 + xw, cc = c * 32 + sch * 8;
      const bool ok = row < g.nh && (unsigned)zd < (unsigned)g.d && (unsigned)zh < (unsigned)g.h &&
                      (unsigned)zw < (unsigned)g.w && cc < g.cin;
      const unsigned off = ok ? (unsigned)(((((nn * g.d + zd) * g.h + zh) * g.w + zw) * g.cin + cc) * 2) : 0xFFFFFFF0u;
      hpre[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0));
      m |= (ok ? 1u : 0u) << i;
    }
    hmask = m;
  };
  auto w_load = [&](int c) {
#pragma unroll
    for (int i = 0; i < SC_WLD; ++i) {
      const int id = tid + i * SC_NT;
      const int row = id >> 2, t = row >> 5, co = co0 + (row & 31);
      const bool ok = id < SC_NWR * 4 && co < g.cout_p;
      const unsigned off = ok ? (unsigned)(((t * g.cout_p + co) * g.cin_p + c * 32 + (id & 3) * 8) * 2) : 0xFFFFFFF0u;
      wpre[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wrs, off, 0, 0));
    }
  };
  // GN scale/shift of this workgroup's sample per input channel, in LDS (filled once): the staging reads its 8
  // channels there at commit time. (Computing them from global loads next to the chunk prefetch made the wait for
  // those loads drain the halo/weight prefetch before the MFMAs.)
  f32x2* const gtab = reinterpret_cast<f32x2*>(smem + SC_LDS);
  int stg_c = 0;  // chunk of the staged prefetch
  auto commit = [&]() {
    f32x2 sc[4], sh[4];
    if (has_gn) {
      const f32x2* t = gtab + stg_c * 32 + sch * 8;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const f32x2 a0 = t[2 * e], a1 = t[2 * e + 1];
        sc[e] = f32x2{a0[0], a1[0]};
        sh[e] = f32x2{a0[1], a1[1]};
      }
    }
#pragma unroll
    for (int i = 0; i < SC_HLD; ++i) {
      const int row = srow0 + i * (SC_NT / 4);
      if (row < g.nh) {
        u32x4 val = hpre[i];
        if (has_gn && ((hmask >> i) & 1u)) val = gn_relu8(val, sc, sh);
        *reinterpret_cast<u32x4*>(hal + sch * SC_PS + row * 16) = val;
      }
    }
#pragma unroll
    for (int i = 0; i < SC_WLD; ++i) {
      const int id = tid + i * SC_NT;
      if (id < SC_NWR * 4) *reinterpret_cast<u32x4*>(wts + (id & 3) * SC_WPS + (id >> 2) * 16) = wpre[i];
    }
  };

  f32x16 acc;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.f;

  const int c0 = ks * g.cpk, c1 = min(g.cin_p / 32, c0 + g.cpk);
  halo_load(c0);
  w_load(c0);
  stg_c = c0;
  if (has_gn) {
    for (int i = tid; i < min(g.cin_p, SC_MAXC); i += SC_NT) {
      const int c = min(i, g.cin - 1), gg = c / (g.cin / g.gn_groups);
      const float mean = gstat[(nn * g.gn_groups + gg) * 2], rstd = gstat[(nn * g.gn_groups + gg) * 2 + 1];
      const float sc_ = rstd * gamma[c];
      gtab[i] = f32x2{sc_, beta[c] - mean * sc_};
    }
    __syncthreads();
  }
  commit();
  __syncthreads();
  for (int c = c0; c < c1; ++c) {
    const bool more = c + 1 < c1;
    if (more) {
      halo_load(c + 1);
      w_load(c + 1);
      stg_c = c + 1;
    }
    ps.mark_now();
    ps.step(true);
    if (active) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int plane = 2 * s + hh;
        const char* ab = hal + plane * SC_PS + arow * 16;
        const char* bb = wts + plane * SC_WPS + r * 16;
#pragma unroll
        for (int t = 0; t < 27; ++t) {
          const int td = t / 9, th = (t / 3) % 3, tw = t % 3;
          const int od = FLIP ? 2 - td : td, oh = FLIP ? 2 - th : th, ow = FLIP ? 2 - tw : tw;
          const bf16x8 a = *reinterpret_cast<const bf16x8*>(ab + ((od * g.hh + oh) * g.hw + ow) * 16);
          const bf16x8 bv = *reinterpret_cast<const bf16x8*>(bb + t * 32 * 16);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bv, acc, 0, 0, 0);
        }
      }
    }
    ps.lap(0);
    __syncthreads();
    ps.lap(2);
    if (more) {
      commit();
      __syncthreads();
      ps.lap(1);
    }
  }
  ps.end(sc_stamps, blockIdx.x & 1023, wave, lane);
  TailStamps ts(sc_tail, blockIdx.x & 1023, tid == 0);
  if (g.nks > 1) {  // fp32 partial through the wave's LDS tile: 128-B rows, coalesced
    float* const ept = reinterpret_cast<float*>(smem + wave * 4096);
    if (active) {
#pragma unroll
      for (int i = 0; i < 16; ++i) ept[((i & 3) + 8 * (i >> 2) + 4 * hh) * 32 + r] = acc[i];
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    const long long per = (long long)g.n * g.d * g.h * g.w * g.cout;  // floats per slab
    // (write-through sc1 16-B stores where the combine runs in this launch: the last-arriving workgroup of the tile
    // reads them with sc1 loads, MI355X_MICROARCH.md visibility table, counter row)
    const auto srs = __builtin_amdgcn_make_buffer_rsrc((void*)g.slab, 0, (int)(g.nks * per * 4), 0x00020000);
    if (active) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int qi = lane + 64 * u, part = qi & 7, row = qi >> 3;
        const int vv = wave * 32 + row;
        const int uw = vv % g.bw, uh = (vv / g.bw) % g.bh, ud = vv / (g.bw * g.bh);
        const int zd = o0d + ud, zh = o0h + uh, zw = o0w + uw, co = co0 + part * 4;
        if (vv < g.nv && zd < g.d && zh < g.h && zw < g.w && co < g.cout) {
          const long long e = ks * per + ((((long long)nn * g.d + zd) * g.h + zh) * g.w + zw) * g.cout + co;
          const f32x4 val = *reinterpret_cast<const f32x4*>(ept + qi * 4);
          if (g.cnt)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, val), srs, (int)(e * 4), 0, 16);
          else
            *reinterpret_cast<f32x4*>(g.slab + e) = val;
        }
      }
    }
    ts.mark<1>();
    if (!g.cnt) return;  // the separate small_reduce_kernel sums the slabs
    // ---- in-kernel split-K combine (round 5): the workgroup that completes its output tile last sums the tile's
    // nks slabs in slab order (bitwise the small_reduce_kernel sums), adds the residual and stores y
    __shared__ unsigned s_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
    __syncthreads();
    ts.mark<2>();
    const int tile = bid / g.nks;
    if (tid == 0) {
      const unsigned old = __hip_atomic_fetch_add(g.cnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = old == (unsigned)(g.nks - 1);
      if (s_last) __hip_atomic_store(g.cnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    ts.mark<3>();
    if (!s_last) return;
    float ls[8], lq[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) ls[k] = lq[k] = 0.f;
    const int cpg = g.stats ? g.cpg : 32;
    // GroupNorm-backward partials (flip with gbx): this thread's 4 channels are fixed (part = tid & 7)
    float bsc[4], bsh[4], bmu[4], brs[4], b1[4], b2[4];
    if (g.gbx) {
      const int gcpg = g.cout / g.gbgroups;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = min(co0 + (tid & 7) * 4 + e, g.cout - 1), gr = c / gcpg;
        bmu[e] = g.gbstat[(nn * g.gbgroups + gr) * 2];
        brs[e] = g.gbstat[(nn * g.gbgroups + gr) * 2 + 1];
        bsc[e] = brs[e] * g.gbgamma[c];
        bsh[e] = g.gbbeta[c] - bmu[e] * bsc[e];
        b1[e] = b2[e] = 0.f;
      }
    }
    // every load of the thread's 4 output pieces (nks slabs, residual, x) in flight before the first add: one memory
    // round trip; then the adds in slab order
    const int ypb = g.n * g.d * g.h * g.w * g.cout * 2;  // bytes of y / residual / x (host: < 2 GiB)
    const auto rrs = __builtin_amdgcn_make_buffer_rsrc((void*)res, 0, res ? ypb : 0, 0x00020000);
    const auto xrs2 = __builtin_amdgcn_make_buffer_rsrc((void*)g.gbx, 0, g.gbx ? ypb : 0, 0x00020000);
    // with a second hand-off (statistics / GroupNorm-backward partials) the y stores wait until this workgroup's
    // partials are published: its vmcnt(0) drain then covers only the partial store, not the tile's y stores
    const bool defer_y = g.stats || g.gbx;
    uint2 yv[4];
    long long yoff[4];
    bool yok[4];
    auto store_y = [&]() {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (yok[k]) *reinterpret_cast<uint2*>(y + yoff[k]) = yv[k];
    };
    auto combine = [&](auto nsc) {
      constexpr int NS = decltype(nsc)::value;
      static_assert(4 * SC_NT / 8 == SC_MAXV, "4 pieces of 4 channels per thread cover the brick's 32-channel tile");
      f32x4 t[4][NS];
      u32x2 rq[4], xq[4];
      long long vo[4];
      bool ok[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int q = tid + SC_NT * k, vv = q >> 3, part = q & 7;
        const int uw = vv % g.bw, uh = (vv / g.bw) % g.bh, ud = vv / (g.bw * g.bh);
        const int zd = o0d + ud, zh = o0h + uh, zw = o0w + uw, co = co0 + part * 4;
        ok[k] = vv < g.nv && zd < g.d && zh < g.h && zw < g.w && co < g.cout;
        vo[k] = ok[k] ? ((((long long)nn * g.d + zd) * g.h + zh) * g.w + zw) * g.cout + co : 0;
#pragma unroll
        for (int s_ = 0; s_ < NS; ++s_) {
          const bool in = ok[k] && s_ < g.nks;
          t[k][s_] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                   srs, in ? (int)((s_ * per + vo[k]) * 4) : (int)0xFFFFFFF0u, 0, 16));
        }
        const int yo = ok[k] ? (int)(vo[k] * 2) : (int)0xFFFFFFF0u;
        if (res) rq[k] = __builtin_amdgcn_raw_buffer_load_b64(rrs, yo, 0, 0);
        if (g.gbx) xq[k] = __builtin_amdgcn_raw_buffer_load_b64(xrs2, yo, 0, 0);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        yok[k] = false;
        if (!ok[k]) continue;
        const int part = (tid + SC_NT * k) & 7;
        f32x4 v = t[k][0];
#pragma unroll
        for (int s_ = 1; s_ < NS; ++s_)
          if (s_ < g.nks) v += t[k][s_];
        if (res) {
          v[0] += __uint_as_float(rq[k][0] << 16);
          v[1] += __uint_as_float(rq[k][0] & 0xffff0000u);
          v[2] += __uint_as_float(rq[k][1] << 16);
          v[3] += __uint_as_float(rq[k][1] & 0xffff0000u);
        }
        uint2 o;
        o.x = (uint32_t)from_f<bf16>(v[0]) | ((uint32_t)from_f<bf16>(v[1]) << 16);
        o.y = (uint32_t)from_f<bf16>(v[2]) | ((uint32_t)from_f<bf16>(v[3]) << 16);
        if (defer_y) {
          yv[k] = o;
          yoff[k] = vo[k];
          yok[k] = true;
        } else {
          *reinterpret_cast<uint2*>(y + vo[k]) = o;
        }
        if (g.gbx) {  // exactly gn_bwd_partial's per-element terms on the stored bf16 dA and x
          const float xv[4] = {__uint_as_float(xq[k][0] << 16), __uint_as_float(xq[k][0] & 0xffff0000u),
                               __uint_as_float(xq[k][1] << 16), __uint_as_float(xq[k][1] & 0xffff0000u)};
          const float dv[4] = {__uint_as_float(o.x << 16), __uint_as_float(o.x & 0xffff0000u),
                               __uint_as_float(o.y << 16), __uint_as_float(o.y & 0xffff0000u)};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float xh = (xv[e] - bmu[e]) * brs[e];
            const float gd = fmaf(xv[e], bsc[e], bsh[e]) > 0.f ? dv[e] : 0.f;
            b1[e] += gd;
            b2[e] = fmaf(gd, xh, b2[e]);
          }
        }
        if (g.stats) {  // the stored values' group sums (4 channels of one group: cpg >= 4)
          const float a0 = __uint_as_float(o.x << 16), a1 = __uint_as_float(o.x & 0xffff0000u);
          const float a2 = __uint_as_float(o.y << 16), a3 = __uint_as_float(o.y & 0xffff0000u);
          const float ss = (a0 + a1) + (a2 + a3), qq = (a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3);
          const int gi = (part * 4) / cpg;
#pragma unroll
          for (int k2 = 0; k2 < 8; ++k2) {
            ls[k2] += gi == k2 ? ss : 0.f;
            lq[k2] += gi == k2 ? qq : 0.f;
          }
        }
      }
    };
    if (g.nks <= 2)
      combine(std::integral_constant<int, 2>{});
    else if (g.nks <= 4)
      combine(std::integral_constant<int, 4>{});
    else
      combine(std::integral_constant<int, 8>{});
    ts.mark<4>();
    if (g.gbx) {
      // per channel of the tile over the workgroup: lanes with the same tid & 7 (xor 8, 16, 32), then the waves in order
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int o2 = 8; o2 < 64; o2 <<= 1) {
          b1[e] += __shfl_xor(b1[e], o2);
          b2[e] += __shfl_xor(b2[e], o2);
        }
      float* const red = reinterpret_cast<float*>(smem);  // [wave][32 channels][2]
      __syncthreads();
      if (lane < 8)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          red[(wave * 32 + lane * 4 + e) * 2] = b1[e];
          red[(wave * 32 + lane * 4 + e) * 2 + 1] = b2[e];
        }
      __syncthreads();
      const int nbr = g.nbd * g.nbh * g.nbw, brick = (bd_ * g.nbh + bh_) * g.nbw + bw_;
      if (tid < 64 && co0 + (tid >> 1) < g.cout) {
        float t2 = 0.f;
#pragma unroll
        for (int wv = 0; wv < SC_NT / 64; ++wv) t2 += red[wv * 64 + tid];
        __hip_atomic_store(g.gbparts + (((long long)nn * nbr + brick) * g.cout + co0) * 2 + tid, t2, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);  // sc1
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      ts.mark<5>();
      const int ntiles = (int)(gridDim.x / g.nks);
      if (tid == 0) {
        const unsigned old = __hip_atomic_fetch_add(g.cnt + ntiles, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = old == (unsigned)(ntiles - 1);
        if (s_last) __hip_atomic_store(g.cnt + ntiles, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
      ts.mark<6>();
      store_y();
      if (!s_last) return;
      // gn_bwd_parts_finalize + gn_bwd_coefs: per (n, c) fp64 sums over the bricks in order, then the coefficients
      double* const cs = reinterpret_cast<double*>(smem);  // [n * cout][2] (<= 8192 doubles: host-checked)
      lastarriver_rowsum<SC_NT>(g.gbparts, g.n, nbr, 2 * g.cout, cs);
      __syncthreads();
      const int gcpg = g.cout / g.gbgroups;
      const double M = (double)g.d * g.h * g.w * gcpg;
      for (int p = tid; p < g.n * g.cout; p += SC_NT) {
        const int n2 = p / g.cout, c = p - n2 * g.cout, gr = c / gcpg;
        double a = 0, bb = 0;
        for (int k2 = 0; k2 < gcpg; ++k2) {
          const int cc = gr * gcpg + k2;
          a += (double)g.gbgamma[cc] * cs[2 * (n2 * g.cout + cc)];
          bb += (double)g.gbgamma[cc] * cs[2 * (n2 * g.cout + cc) + 1];
        }
        const float ca = (float)(a / M), cb = (float)(bb / M);
        const float mu = g.gbstat[(n2 * g.gbgroups + gr) * 2], rs = g.gbstat[(n2 * g.gbgroups + gr) * 2 + 1];
        const float scv = rs * g.gbgamma[c];
        float* oc = g.coef + (long long)n2 * 5 * g.cout;
        oc[c] = scv;
        oc[g.cout + c] = g.gbbeta[c] - mu * scv;
        oc[2 * g.cout + c] = rs * g.gbgamma[c];
        oc[3 * g.cout + c] = -rs * rs * cb;
        oc[4 * g.cout + c] = -rs * ca + rs * rs * cb * mu;
      }
      for (int c = tid; c < g.cout; c += SC_NT) {
        double tg = 0, tb = 0;
        for (int n2 = 0; n2 < g.n; ++n2) {
          tb += cs[2 * (n2 * g.cout + c)];
          tg += cs[2 * (n2 * g.cout + c) + 1];
        }
        if (g.dgamma) g.dgamma[c] = (float)tg;
        if (g.dbeta) g.dbeta[c] = (float)tb;
      }
      ts.mark<7>();
      return;
    }
    if (!g.stats) return;
    // ---- output GroupNorm(16) statistics: this tile's groups reduced over the workgroup (fixed order), one partial
    // row per (sample, brick); the workgroup completing the last tile combines them in fp64 (one launch, no pass)
    float sv[16];
#pragma unroll
    for (int k2 = 0; k2 < 8; ++k2) {
      sv[2 * k2] = ls[k2];
      sv[2 * k2 + 1] = lq[k2];
    }
    const float tot = wave_sum_transposed<16>(sv, lane);  // lane l: value l >> 2 = (group slot, sum | square)
    float* const red = reinterpret_cast<float*>(smem);     // (LDS free: the MFMA loop is done)
    __syncthreads();
    if ((lane & 3) == 0) red[wave * 16 + (lane >> 2)] = tot;
    __syncthreads();
    const int gpt = 32 / cpg, nbr = g.nbd * g.nbh * g.nbw, brick = (bd_ * g.nbh + bh_) * g.nbw + bw_;
    if (tid < 2 * gpt) {
      float t2 = 0.f;
#pragma unroll
      for (int wv = 0; wv < SC_NT / 64; ++wv) t2 += red[wv * 16 + tid];
      const int gr = co0 / cpg + (tid >> 1);
      __hip_atomic_store(g.spart + ((long long)nn * nbr + brick) * 32 + gr * 2 + (tid & 1), t2, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);  // sc1
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    ts.mark<5>();
    const int ntiles = (int)(gridDim.x / g.nks);
    if (tid == 0) {
      const unsigned old = __hip_atomic_fetch_add(g.cnt + ntiles, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = old == (unsigned)(ntiles - 1);
      if (s_last) __hip_atomic_store(g.cnt + ntiles, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    ts.mark<6>();
    store_y();
    if (!s_last) return;
    double* const cs = reinterpret_cast<double*>(smem) + 64;  // [n * 16][2] (past the wave rows in `red`)
    lastarriver_rowsum<SC_NT>(g.spart, g.n, nbr, 32, cs);
    __syncthreads();
    for (int p = tid; p < g.n * 16; p += SC_NT) {
      const double m = (double)g.cpg * g.d * g.h * g.w;
      const double mean = cs[2 * p] / m;
      double var = cs[2 * p + 1] / m - mean * mean;
      if (var < 0) var = 0;
      g.stats[p * 2] = (float)mean;
      g.stats[p * 2 + 1] = (float)(1.0 / sqrt(var + 1e-5));
    }
    ts.mark<7>();
    return;
  }

  // epilogue: wave tile [32 rows][32 co] bf16 (2 KB) -> 16-B chunks, 4 lanes per output voxel
  char* const ept = smem + wave * 2048;
  if (active) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = (i & 3) + 8 * (i >> 2) + 4 * hh;
      *reinterpret_cast<bf16*>(ept + (row * 32 + r) * 2) = from_f<bf16>(acc[i]);
    }
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  if (active) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int qi = lane + 64 * u, part = qi & 3, row = qi >> 2;
      const int vv = wave * 32 + row;
      const int uw = vv % g.bw, uh = (vv / g.bw) % g.bh, ud = vv / (g.bw * g.bh);
      const int zd = o0d + ud, zh = o0h + uh, zw = o0w + uw, co = co0 + part * 8;
      if (vv < g.nv && zd < g.d && zh < g.h && zw < g.w && co < g.cout) {
        const long long off = ((((long long)nn * g.d + zd) * g.h + zh) * g.w + zw) * g.cout + co;
        u32x4 val = *reinterpret_cast<const u32x4*>(ept + qi * 16);
        if (res) {
          float a[8], q[8];
          load16<bf16>(reinterpret_cast<const bf16*>(&val), a);
          load16<bf16>(res + off, q);
#pragma unroll
          for (int e = 0; e < 8; ++e) a[e] += q[e];
          store16<bf16>(reinterpret_cast<bf16*>(&val), a);
        }
        *reinterpret_cast<u32x4*>(y + off) = val;
      }
    }
  }
}

// y = bf16(sum_s slab[s] (+ residual)), 4 channels per thread, splits summed in fixed order
__global__ __launch_bounds__(256) void small_reduce_kernel(const float* __restrict__ slab, int nks, long long per4,
                                                           const bf16* __restrict__ res, bf16* __restrict__ y) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < per4; i += (long long)gridDim.x * 256) {
    f32x4 v = reinterpret_cast<const f32x4*>(slab)[i];
    for (int s = 1; s < nks; ++s) v += reinterpret_cast<const f32x4*>(slab)[s * per4 + i];
    if (res) {
      const uint2 q = reinterpret_cast<const uint2*>(res)[i];
      v[0] += __uint_as_float(q.x << 16);
      v[1] += __uint_as_float(q.x & 0xffff0000u);
      v[2] += __uint_as_float(q.y << 16);
      v[3] += __uint_as_float(q.y & 0xffff0000u);
    }
    uint2 o;
    o.x = (uint32_t)from_f<bf16>(v[0]) | ((uint32_t)from_f<bf16>(v[1]) << 16);
    o.y = (uint32_t)from_f<bf16>(v[2]) | ((uint32_t)from_f<bf16>(v[3]) << 16);
    reinterpret_cast<uint2*>(y)[i] = o;
  }
}

}  // namespace u3d

using namespace u3d;

struct SCGb {  // the GroupNorm-backward partials of the data gradient (u3d_conv_small_dgrad_gn)
  const void* x;
  const float *stats, *gamma, *beta;
  int groups;
  float *parts, *coef, *dgamma, *dbeta;
};
static int conv_small_impl(int flip, const void* x, int n, int cin, int d, int h, int w, const void* wpk, int cout,
                           const float* gn_stats, const float* gn_gamma, const float* gn_beta, int gn_groups,
                           const void* residual, void* y, float* ws, long long ws_bytes, unsigned* cnt,
                           float* spart, float* stats_out, int* nks_out, u3d_stream_t stream,
                           const SCGb* gb = nullptr, bool plan_only = false);

extern "C" int u3d_conv_small(int flip, const void* x, int n, int cin, int d, int h, int w, const void* wpk, int cout,
                              const float* gn_stats, const float* gn_gamma, const float* gn_beta, int gn_groups,
                              const void* residual, void* y, float* ws, long long ws_bytes, u3d_stream_t stream) {
  return conv_small_impl(flip, x, n, cin, d, h, w, wpk, cout, gn_stats, gn_gamma, gn_beta, gn_groups, residual, y, ws,
                         ws_bytes, nullptr, nullptr, nullptr, nullptr, stream);
}

// Round 5 form: the split-K slabs are combined inside the conv launch by the last-arriving workgroup of each output
// tile (no small_reduce_kernel), and with stats_out the output's GroupNorm(16) statistics come from that combine (no
// statistics pass). cnt: u3d_conv_small_cnt_bytes() of ZEROED memory (left zeroed); spart: u3d_conv_small_spart_floats.
// Statistics need the contraction split (nks > 1) and cout in {64, 128, 256} (4..16 channels per group); where a
// launch cannot produce them it returns 0 with *stats_made = 0 and the caller takes the statistics pass.
extern "C" long long u3d_conv_small_cnt_bytes(int n, int d, int h, int w, int cout) {
  return 4LL * (n * cdiv(d, 1) * cdiv(h, 1) * cdiv(w, 1) * cdiv(cout, 32) + 1);  // >= tiles + 1 (bricks >= 1 voxel)
}
extern "C" long long u3d_conv_small_spart_floats(int n, int d, int h, int w) {
  return 32LL * n * d * h * w;  // >= n * bricks * 32
}
extern "C" int u3d_conv_small2(int flip, const void* x, int n, int cin, int d, int h, int w, const void* wpk, int cout,
                               const float* gn_stats, const float* gn_gamma, const float* gn_beta, int gn_groups,
                               const void* residual, void* y, float* ws, long long ws_bytes, unsigned* cnt,
                               float* spart, float* stats_out, int* stats_made, u3d_stream_t stream) {
  U3D_REQUIRE(cnt && stats_made, "conv_small2: needs the counter workspace and stats_made");
  int nks = 0;
  // the statistics form's own limits (one thread per (sample, group) in the finalize, 31-bit slab offsets): past
  // them the launch declines with *stats_made = 0 and the caller runs the statistics pass
  const bool want = stats_out && spart && !flip && cout % 16 == 0 &&
                    (cout / 16 == 4 || cout / 16 == 8 || cout / 16 == 16) && n * 16 <= SC_NT &&
                    8LL * n * d * h * w * cout * 4 < (1LL << 31);
  const int rc = conv_small_impl(flip, x, n, cin, d, h, w, wpk, cout, gn_stats, gn_gamma, gn_beta, gn_groups, residual,
                                 y, ws, ws_bytes, cnt, want ? spart : nullptr, want ? stats_out : nullptr, &nks, stream);
  *stats_made = rc == 0 && want && nks > 1 && nks <= 8;
  return rc;
}

static int conv_small_impl(int flip, const void* x, int n, int cin, int d, int h, int w, const void* wpk, int cout,
                           const float* gn_stats, const float* gn_gamma, const float* gn_beta, int gn_groups,
                           const void* residual, void* y, float* ws, long long ws_bytes, unsigned* cnt,
                           float* spart, float* stats_out, int* nks_out, u3d_stream_t stream,
                           const SCGb* gb, bool plan_only) {
  U3D_REQUIRE(x && wpk && y && n >= 1 && d >= 1 && h >= 1 && w >= 1, "conv_small: bad args");
  U3D_REQUIRE(cin % 8 == 0 && cout % 8 == 0, "conv_small: channels must be multiples of 8");
  U3D_REQUIRE(!gn_stats || (!flip && gn_gamma && gn_beta && gn_groups > 0 && cin % gn_groups == 0),
              "conv_small: bad GN prologue");
  U3D_REQUIRE(!gn_stats || round_up(cin, 32) <= SC_MAXC, "conv_small: GN prologue supports cin <= %d", SC_MAXC);
  SCGeom g{};
  g.n = n; g.d = d; g.h = h; g.w = w;
  g.cin = cin; g.cin_p = round_up(cin, 32); g.cout = cout; g.cout_p = round_up(cout, 32);
  g.gn_groups = gn_groups;
  auto even = [](int q, int mx) { return cdiv(q, cdiv(q, std::max(1, mx))); };
  g.bw = even(w, 16);
  g.bh = even(h, SC_MAXV / (g.bw * 2));
  g.bd = even(d, std::min(d, SC_MAXV / (g.bw * g.bh)));
  while ((g.bd + 2) * (g.bh + 2) * (g.bw + 2) > SC_HMAX && g.bd > 1) --g.bd;
  while ((g.bd + 2) * (g.bh + 2) * (g.bw + 2) > SC_HMAX && g.bh > 1) --g.bh;
  while ((g.bd + 2) * (g.bh + 2) * (g.bw + 2) > SC_HMAX && g.bw > 1) --g.bw;
  g.nv = g.bd * g.bh * g.bw;
  g.hh = g.bh + 2; g.hw = g.bw + 2;
  g.nh = (g.bd + 2) * g.hh * g.hw;
  g.nbd = cdiv(d, g.bd); g.nbh = cdiv(h, g.bh); g.nbw = cdiv(w, g.bw);
  g.nct = g.cout_p / 32;
  const long long tiles = (long long)n * g.nbd * g.nbh * g.nbw * g.nct;
  // split the contraction over workgroups until ~2 workgroups per CU: the per-CU operand stream (55 KB of
  // weights + the halo per 32-channel chunk), not the MFMAs, bounds these small layers
  const int nchunk = g.cin_p / 32;
  const long long target = std::max(1, opt(OPT_SMALL_WGS));  // workgroups aimed at
  int nks = (int)std::min<long long>(nchunk, std::max<long long>(1, (target + tiles - 1) / tiles));
  const long long slab1 = (long long)n * d * h * w * cout * 4;
  if (cout % 4) nks = 1;
  while (nks > 1 && (!ws || nks * slab1 > ws_bytes)) --nks;
  g.cpk = cdiv(nchunk, nks);
  g.nks = cdiv(nchunk, g.cpk);
  g.slab = g.nks > 1 ? ws : nullptr;
  if (nks_out) *nks_out = g.nks;
  g.cnt = g.nks > 1 && g.nks <= 8 ? cnt : nullptr;  // in-kernel combine where there are (<= 8) slabs to combine
  g.stats = g.cnt ? stats_out : nullptr;
  g.spart = g.stats ? spart : nullptr;
  g.cpg = cout / 16;
  if (plan_only) return 0;
  if (gb && g.cnt) {
    U3D_REQUIRE(flip && !residual && gb->groups > 0 && cout % gb->groups == 0 && (long long)n * cout * 2 <= 8192,
                "conv_small_dgrad_gn: bad GroupNorm-backward args");
    g.gbx = (const bf16*)gb->x;
    g.gbstat = gb->stats; g.gbgamma = gb->gamma; g.gbbeta = gb->beta; g.gbgroups = gb->groups;
    g.gbparts = gb->parts; g.coef = gb->coef; g.dgamma = gb->dgamma; g.dbeta = gb->dbeta;
    g.stats = nullptr;
  }
  U3D_REQUIRE(!g.stats || (n * 16 <= SC_NT && g.nks * (long long)n * d * h * w * cout * 4 < (1LL << 31)),
              "conv_small2: statistics form limits");
  const long long nwg = tiles * g.nks;
  U3D_REQUIRE(nwg < (1LL << 31), "conv_small: grid too large");
  U3D_REQUIRE((long long)n * d * h * w * std::max(cin, cout) * 2 < (1LL << 31) - 64 && 27LL * g.cout_p * g.cin_p * 2 < (1LL << 31) - 64,
              "conv_small: operands beyond the 2 GiB buffer-offset range");
  hipStream_t s = (hipStream_t)stream;
  if (flip)
    hipLaunchKernelGGL(conv_small_kernel<true>, dim3((unsigned)nwg), dim3(SC_NT), 0, s, (const bf16*)x,
                       (const bf16*)wpk, (bf16*)y, (const bf16*)residual, gn_stats, gn_gamma, gn_beta, g);
  else
    hipLaunchKernelGGL(conv_small_kernel<false>, dim3((unsigned)nwg), dim3(SC_NT), 0, s, (const bf16*)x,
                       (const bf16*)wpk, (bf16*)y, (const bf16*)residual, gn_stats, gn_gamma, gn_beta, g);
  int rc = check_launch("conv_small_kernel");
  if (rc || g.nks == 1 || g.cnt) return rc;
  const long long per4 = slab1 / 16;
  hipLaunchKernelGGL(small_reduce_kernel, dim3((unsigned)std::min<long long>(4096, (per4 + 255) / 256)), dim3(256), 0,
                     s, ws, g.nks, per4, (const bf16*)residual, (bf16*)y);
  return check_launch("small_reduce_kernel");
}

// Round 5: data gradient of conv(relu(gn(x))) for the small deep-level volumes with the GroupNorm backward's partial
// pass AND its coefficient finalize inside the launch (the split-K combine computes the bf16 dA, reads x at the same
// addresses, sums g = relu-mask * dA and g * xhat per (sample, brick, channel); the workgroup completing the last tile
// forms the apply coefficients coef[n][5][cin] and dgamma / dbeta as gn_bwd_parts_finalize does). Then only
// u3d_gn_bwd_apply_coef runs. cin / cout are the FORWARD conv's: dy has cout, dx / x have cin; wpk = the dgrad pack.
// parts: u3d_conv_small_gb_parts_floats floats; cnt: u3d_conv_small_cnt_bytes(n, d, h, w, cin) zeroed bytes.
// *made = 0 (nothing launched; the caller takes the separate passes) where the launch would not split its
// contraction over 2..8 workgroups.
extern "C" long long u3d_conv_small_gb_parts_floats(int n, int d, int h, int w, int cin) {
  return 2LL * n * d * h * w * cin;  // >= n * bricks * cin * 2
}
extern "C" int u3d_conv_small_dgrad_gn(const void* dy, int n, int cout, int d, int h, int w, const void* wpk_dgrad,
                                       int cin, const void* x, const float* gn_stats, const float* gn_gamma,
                                       const float* gn_beta, int gn_groups, void* dx, float* ws, long long ws_bytes,
                                       unsigned* cnt, float* parts, float* coef, float* dgamma, float* dbeta,
                                       int* made, u3d_stream_t stream) {
  U3D_REQUIRE(dy && x && dx && cnt && parts && coef && made && gn_stats && gn_gamma && gn_beta,
              "conv_small_dgrad_gn: bad args");
  *made = 0;
  int nks = 0;
  int rc = conv_small_impl(1, dy, n, cout, d, h, w, wpk_dgrad, cin, nullptr, nullptr, nullptr, 0, nullptr, dx, ws,
                           ws_bytes, cnt, nullptr, nullptr, &nks, stream, nullptr, true);
  if (rc) return rc;
  if (nks < 2 || nks > 8 || (long long)n * cin * 2 > 8192) return 0;
  const SCGb gb{x, gn_stats, gn_gamma, gn_beta, gn_groups, parts, coef, dgamma, dbeta};
  rc = conv_small_impl(1, dy, n, cout, d, h, w, wpk_dgrad, cin, nullptr, nullptr, nullptr, 0, nullptr, dx, ws,
                       ws_bytes, cnt, nullptr, nullptr, &nks, stream, &gb);
  if (rc == 0) *made = 1;
  return rc;
}
