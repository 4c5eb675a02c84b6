// Weight gradient of the 3^3 stride-1 convolutions, depth-streaming ring form (gfx950).
//
//   dW[t][co][ci] = sum_{n, q} dy[n, q, co] * A[n, q + t - 1, ci],   A = relu(gn(x)) (prologue)
//
// Same contract as u3d_conv_wgrad_brick (fp32 partial slabs [split][27][cout_p][cin_p]), different schedule:
//   * workgroup = one (32 co) x (32 ci) tile x a contiguous range of OUTPUT PLANES in (column, d) order, a
//     column being (n, 16-row h tile, 16-voxel w tile); it walks down d, so each input plane (18 x 18 halo
//     rows) is staged once for three output planes, and each dy plane once;
//   * LDS: a ring of 4 input planes + 2 dy planes, rows channel-contiguous (64 B); the plane written at a step
//     start (GroupNorm + ReLU applied once per element) is the one loaded a full step earlier, the next
//     plane's loads then fly under the MFMAs; one barrier per output plane;
//   * k = the 256 voxels of an output plane, 16 per MFMA (one 16-voxel w row): both operands are read
//     transposed (ds_read_b64_tr_b16), every lane addressing its own (shifted) row, so the 27 tap windows
//     come from the same staged planes with no data movement; wave w owns taps w, w+8, w+16 (, w+24) and
//     shares its dy fragment between them.
// Reference: autograd of F.conv3d in Conv3d.forward (unet3D.py:27).
#include <type_traits>

#include "common.h"
#include "diag.h"

namespace u3d {
namespace {

typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;

__device__ __forceinline__ v4i16 trd(const char* lds_base, int byte_off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_v4i16*)((__attribute__((address_space(3))) char*)lds_base + byte_off));
}
__device__ __forceinline__ bf16x8 frag2(v4i16 lo, v4i16 hi) {
  typedef short v8i16 __attribute__((ext_vector_type(8)));
  v8i16 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}
template <int I, int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor<I + 1, N>(f);
  }
}

#ifndef U3D_WRING_M16
#define U3D_WRING_M16 1
#endif
constexpr int WR_ROWB = 64;
constexpr int WR_NT = 512;
// plane tile PH x PW (16 x 16; 12 x 24 for 24-wide planes and 12 x 12 for 12-wide ones, so that no k step is
// spent on voxels past the volume): the k index of an output plane runs over its PH*PW voxels flattened (h, w), 16
// per MFMA; each lane addresses its own voxel's (shifted) halo row, so any tile shape works.
template <int PH, int PW, bool MM>
struct WRT {
  static constexpr int HH = PH + 2, HW = PW + 2;
  static constexpr int NR = HH * HW;                 // halo rows per input plane (324 at 16 x 16)
  static constexpr int NV = PH * PW;                 // voxels per output plane (256 = 16 k16 steps)
  static constexpr int KS = NV / 16;
  // M16 (default where the plane tile holds whole 32-voxel k steps: 16 x 16, 12 x 24): v_mfma_f32_16x16x32_bf16, the
  // same cycles per flop as 32x32x16 at a higher held clock (MI355X_MICROARCH.md, DVFS item 7). Its fragments are 16
  // channels x 8 voxels, so the rows are stored half-planar: plane = 16 channels (32 B per row); the 8 consecutive
  // rows a half-wave reads per ds_read_b64_tr_b16 are then 256 contiguous bytes (conflict-free), and the plane
  // stride = 128 mod 256 B keeps the staging writes (two rows x two planes per 8-lane group) conflict-free too.
  static constexpr bool M16 = MM;
  static constexpr int RP = M16 ? 32 : WR_ROWB;                               // row pitch within a plane
  static constexpr int HP = M16 ? (NR * 32 + 255) / 256 * 256 + 128 : 0;      // input half-plane stride
  static constexpr int DHP = M16 ? (NV * 32 + 255) / 256 * 256 + 128 : 0;     // dy half-plane stride
  static constexpr int SLOT = M16 ? 2 * HP : NR * WR_ROWB;
  static constexpr int DSLOT = M16 ? 2 * DHP : NV * WR_ROWB;
  static constexpr int LX = (NR * 4 + WR_NT - 1) / WR_NT;  // input pieces per thread and plane
  static constexpr int LY = (NV * 4 + WR_NT - 1) / WR_NT;  // dy pieces
  static_assert(NV % 16 == 0, "k steps of 16 voxels");
};

struct WRGeom {
  int n, d, h, w, cin, cout, cin_p, cout_p;
  int ph, pw;  // plane tile
  int nbh, nbw;
  long long planes;  // output planes per channel tile = n * nbh * nbw * d
  int per;           // output planes per split
  int gn_groups;
  long long xbytes, ybytes;
};

struct WRPlane {
  int n, h0, w0, zin;
  bool valid, out;
};

struct WRWalk {
  long long o_next, o_end;
  int col, zin, zfirst, zlast;
  bool done;
  __device__ void start_run(const WRGeom& g) {
    if (o_next >= o_end) { done = true; return; }
    col = (int)(o_next / g.d);
    zfirst = (int)(o_next - (long long)col * g.d);
    zlast = (int)min<long long>(g.d, zfirst + (o_end - o_next));
    o_next += zlast - zfirst;
    zin = zfirst - 1;
  }
  __device__ WRPlane next(const WRGeom& g) {
    WRPlane p{};
    if (!done && zin > zlast) start_run(g);
    if (done) return p;
    int c = col;
    const int bw_ = c % g.nbw; c /= g.nbw;
    const int bh_ = c % g.nbh;
    p.n = c / g.nbh;
    p.h0 = bh_ * g.ph;
    p.w0 = bw_ * g.pw;
    p.zin = zin;
    p.valid = true;
    p.out = zin >= zfirst + 1;
    ++zin;
    return p;
  }
};

// -DU3D_STAMPS phases (diag.h): 0 the staged plane's write (incl. its loads' wait), 1 compute, 2 the barrier
U3D_STAMP_BUFFER(wr_stamps, 4096, u3d_diag_wgrad_stamps)
}  // namespace

template <bool GN, int PH = 16, int PW = 16>
__global__ __launch_bounds__(WR_NT, 1) void wgrad_ring_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                             const float* __restrict__ gstat,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ beta, float* __restrict__ part,
                                                             WRGeom g) {
  // (the 12 x 24 tile without the GroupNorm prologue keeps 32x32x16: its 16x16x32 form spills)
  using T = WRT<PH, PW, U3D_WRING_M16 != 0 && (PH * PW) % 32 == 0 && (GN || PW == 16)>;
  constexpr int WR_HW = T::HW, WR_NR = T::NR, WR_NV = T::NV, WR_SLOT = T::SLOT, WR_DSLOT = T::DSLOT, WR_LX = T::LX,
                WR_LY = T::LY, WR_PW = PW;
  __shared__ __attribute__((aligned(16))) char lds[4 * WR_SLOT + 2 * WR_DSLOT + 1024];
  char* const ring = lds;
  char* const dyr = lds + 4 * WR_SLOT;
  char* const junk = dyr + 2 * WR_DSLOT;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ch = tid & 3;
  diag_prio_second_half(wave);
  const TileSplit ts = xcd_tile_split();  // XCD-aware: the channel tiles of neighbouring plane ranges share an L2
  const int ci0 = ts.tx * 32, co0 = ts.ty * 32, split = ts.split;
  WRWalk walk{};
  walk.o_next = (long long)split * g.per;
  walk.o_end = min(g.planes, walk.o_next + g.per);
  walk.done = false;
  walk.zin = 1;
  walk.zlast = 0;

  const auto xrs = __builtin_amdgcn_make_buffer_rsrc((void*)x, 0, (int)g.xbytes, 0x00020000);
  const auto yrs = __builtin_amdgcn_make_buffer_rsrc((void*)dy, 0, (int)g.ybytes, 0x00020000);
  f32x2 sc[4], sh[4];
  int gn_n = -1;
  const bool cok = ci0 + ch * 8 < g.cin, dok = co0 + ch * 8 < g.cout;

  // per-lane staging offsets hoisted out of the walk (round 4): a lane's halo row / dy voxel of piece i is the same
  // in every plane, so its byte offset is a per-lane constant plus a wave-uniform plane base, and its in-volume test
  // changes only with the column (n, h0, w0) — per plane and piece one add and one select instead of ~30 VALU + SALU
  int xlo[WR_LX], ylo[WR_LY];
#pragma unroll
  for (int i = 0; i < WR_LX; ++i) {  // (dead for the 12 x 24 / 12 x 12 tiles: see HOIST)
    const int row = (tid >> 2) + i * (WR_NT / 4);
    xlo[i] = (((row / WR_HW) * g.w + row % WR_HW) * g.cin + ci0 + ch * 8) * 2;
  }
#pragma unroll
  for (int i = 0; i < WR_LY; ++i) {
    const int v = (tid >> 2) + i * (WR_NT / 4);
    ylo[i] = (((v / WR_PW) * g.w + v % WR_PW) * g.cout + co0 + ch * 8) * 2;
  }
  unsigned xin = 0, yin = 0;
  int col_h0 = -1, col_w0 = -1;
  auto column = [&](const WRPlane& p) {
    if (p.valid && (p.h0 != col_h0 || p.w0 != col_w0)) {  // uniform: once per run of the walk
      col_h0 = p.h0;
      col_w0 = p.w0;
      xin = yin = 0;
#pragma unroll
      for (int i = 0; i < WR_LX; ++i) {
        const int row = (tid >> 2) + i * (WR_NT / 4);
        const bool ok = cok && row < WR_NR && (unsigned)(p.h0 - 1 + row / WR_HW) < (unsigned)g.h &&
                        (unsigned)(p.w0 - 1 + row % WR_HW) < (unsigned)g.w;
        xin |= (ok ? 1u : 0u) << i;
      }
#pragma unroll
      for (int i = 0; i < WR_LY; ++i) {
        const int v = (tid >> 2) + i * (WR_NT / 4);
        const bool ok = dok && v < WR_NV && p.h0 + v / WR_PW < g.h && p.w0 + v % WR_PW < g.w;
        yin |= (ok ? 1u : 0u) << i;
      }
    }
  };
  // (hoisted only for the 16 x 16 tiles: the 12 x 24 tile's register budget has no room for the six offsets)
  constexpr bool HOIST = PW == 16;
  // Staging, one 16-B piece at a time (round 5): piece i of plane p into vx[i] / vy[i]; bit i of m = the x row is
  // inside the volume. The step writes the staged plane's pieces between its MFMA sub-steps and reloads each piece's
  // register with the next plane right after (one register set: as a separate phase before the MFMAs the staging took
  // 40% of the step, r04 stamps of the 16 x 16 form).
  auto load_x = [&](const WRPlane& p, int i, u32x4 (&vx)[WR_LX], unsigned& m) {
    bool ok;
    unsigned off;
    if constexpr (!HOIST) {
      const int row = (tid >> 2) + i * (WR_NT / 4);
      const int hw = row % WR_HW, hh = row / WR_HW;
      const int zh = p.h0 - 1 + hh, zw = p.w0 - 1 + hw;
      ok = p.valid && cok && row < WR_NR && (unsigned)p.zin < (unsigned)g.d && (unsigned)zh < (unsigned)g.h &&
           (unsigned)zw < (unsigned)g.w;
      off = ok ? (unsigned)(((((p.n * g.d + p.zin) * g.h + zh) * g.w + zw) * g.cin + ci0 + ch * 8) * 2) : 0xFFFFFFF0u;
    } else {
      const bool pv = p.valid && (unsigned)p.zin < (unsigned)g.d;
      const int xb = (((p.n * g.d + p.zin) * g.h + p.h0 - 1) * g.w + p.w0 - 1) * g.cin * 2;
      ok = pv && ((xin >> i) & 1u);
      off = ok ? (unsigned)(xb + xlo[i]) : 0xFFFFFFF0u;
    }
    vx[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0));
    m = (m & ~(1u << i)) | ((ok ? 1u : 0u) << i);
  };
  auto load_y = [&](const WRPlane& p, int i, u32x4 (&vy)[WR_LY]) {
    unsigned off;
    if constexpr (!HOIST) {
      const int v = (tid >> 2) + i * (WR_NT / 4);
      const int zh = p.h0 + v / WR_PW, zw = p.w0 + v % WR_PW, zo = p.zin - 1;
      const bool ok = p.valid && p.out && dok && v < WR_NV && zh < g.h && zw < g.w;
      off = ok ? (unsigned)(((((p.n * g.d + zo) * g.h + zh) * g.w + zw) * g.cout + co0 + ch * 8) * 2) : 0xFFFFFFF0u;
    } else {
      const bool po = p.valid && p.out;
      const int yb = (((p.n * g.d + p.zin - 1) * g.h + p.h0) * g.w + p.w0) * g.cout * 2;
      off = po && ((yin >> i) & 1u) ? (unsigned)(yb + ylo[i]) : 0xFFFFFFF0u;
    }
    vy[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(yrs, off, 0, 0));
  };
  auto load_plane = [&](const WRPlane& p, u32x4 (&vx)[WR_LX], u32x4 (&vy)[WR_LY], unsigned& m) {
    if constexpr (HOIST) column(p);
#pragma unroll
    for (int i = 0; i < WR_LX; ++i) load_x(p, i, vx, m);
#pragma unroll
    for (int i = 0; i < WR_LY; ++i) load_y(p, i, vy);
  };
  auto gn_refresh = [&](const WRPlane& p) {
    if (GN && p.valid && p.n != gn_n) {
      gn_n = p.n;
      gn_coef8(gstat, gamma, beta, g.gn_groups, g.cin, p.n, ci0 + ch * 8, sc, sh);
    }
  };
  auto write_x = [&](int i, const u32x4 (&vx)[WR_LX], unsigned m, int slot) {
    const int row = (tid >> 2) + i * (WR_NT / 4);
    u32x4 val = vx[i];
    if constexpr (GN) {
      val = gn_relu8(val, sc, sh);
      if (!((m >> i) & 1u)) val = u32x4{0u, 0u, 0u, 0u};  // padding stays zero after the prologue
    }
    const int lo = T::M16 ? (ch >> 1) * T::HP + row * 32 + (ch & 1) * 16 : row * WR_ROWB + ch * 16;
    char* dst = row < WR_NR ? ring + slot * WR_SLOT + lo : junk + (tid & 63) * 16;
    *reinterpret_cast<u32x4*>(dst) = val;
  };
  auto write_y = [&](int i, const u32x4 (&vy)[WR_LY], int dslot) {
    const int v = (tid >> 2) + i * (WR_NT / 4);
    if (WR_NV % (WR_NT / 4) == 0 || v < WR_NV)
      *reinterpret_cast<u32x4*>(dyr + dslot * WR_DSLOT +
                                (T::M16 ? (ch >> 1) * T::DHP + v * 32 + (ch & 1) * 16 : v * WR_ROWB + ch * 16)) = vy[i];
  };

  constexpr int MAXT = 4;  // taps per wave: t = wave + 8j
  f32x16 acc[MAXT];    // 32x32x16: D[co 32][ci 32] per tap
  f32x4 acc4[MAXT][4];  // M16: [tap][co block cb * 2 + ci block cib] (16 x 16 each)
#pragma unroll
  for (int j = 0; j < MAXT; ++j) {
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) acc4[j][e] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  int tap_row[MAXT], tap_d[MAXT];
#pragma unroll
  for (int j = 0; j < MAXT; ++j) {
    const int t = min(wave + 8 * j, 26);
    tap_d[j] = t / 9;
    tap_row[j] = (((t / 3) % 3) * WR_HW + t % 3) * T::RP;
  }
  const int ntap = (27 - wave + 7) / 8;  // 4 for waves 0-2, 3 for 3-7
  // fragment lane geometry: group gq = lane>>4, in-group lane i = lane&15 -> (q = i>>2, p = i&3)
  const int hh = lane >> 5, gq = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int colb = (16 * (gq & 1) + 4 * pp) * 2;
  int lrow[2];
#pragma unroll
  for (int m = 0; m < 2; ++m) lrow[m] = 8 * hh + 4 * m + q;  // this lane's voxel k within a 16-voxel k step
  // k step ks, half m: byte offsets of the lane's voxel f = 16 ks + lrow[m] in the dy plane (flattened) and of its
  // halo row (f + 2 (f / PW): the halo rows are PW + 2 wide) in an input slot
  auto dyoff = [&](int ks, int m) { return (16 * ks + lrow[m]) * WR_ROWB + colb; };
  // (16 ks = a PW + b at compile time, so f / PW = a + [lrow >= PW - b]: one compare per fragment, no division)
  auto xoff = [&](int ks, int m) {
    const int a = 16 * ks / WR_PW, b = 16 * ks % WR_PW;
    return (a * WR_HW + b + lrow[m] + (lrow[m] >= WR_PW - b ? 2 : 0)) * WR_ROWB + colb;
  };

  auto compute = [&](int dslot, int s0, int s1, int s2, auto ntc, auto&& side) {
    constexpr int NTP = decltype(ntc)::value;
    (void)s1;
    (void)s2;
    int tb[NTP];  // slot of tap depth td = (s0 + td) & 3 (the three slots are consecutive): no indexed array
#pragma unroll
    for (int j = 0; j < NTP; ++j) tb[j] = ((s0 + tap_d[j]) & 3) * WR_SLOT + tap_row[j];
    const char* dbase = dyr + dslot * WR_DSLOT;
    if constexpr (T::M16) {
      // 32-voxel k steps; sub-step u = (k step u >> 1, ci block u & 1): per sub-step NTP x 2 MFMAs (taps x co blocks).
      // A = dy^T (co rows), B = the tap's input rows (ci columns). Lane (group g4 = lane >> 4, q, pp) addresses voxel
      // rows 4 g4 + q (m = 0) and 16 + 4 g4 + q (m = 1) of the k step — the K order of a weight gradient is free, and
      // each half-wave's tr read then covers 8 consecutive voxels (never across a tile row for PW = 16, 24).
      constexpr int KS2 = T::NV / 32;
      const int g4 = lane >> 4;
      const int v16[2] = {4 * g4 + q, 16 + 4 * g4 + q};
      auto dyo = [&](int ks, int m, int cb) { return cb * T::DHP + (32 * ks + v16[m]) * 32 + 8 * pp; };
      auto xo = [&](int ks, int m) {  // halo row of voxel 32 ks + v: 32 ks = a PW + b, one wrap at most (PW >= 16)
        const int a = 32 * ks / WR_PW, b = 32 * ks % WR_PW, v = v16[m];
        return (a * WR_HW + b + v + (v >= WR_PW - b ? 2 : 0)) * 32 + 8 * pp;
      };
      bf16x8 fa2[2][2], fb2[2][NTP];
      auto rdA = [&](int ks) {
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
          fa2[ks & 1][cb] = frag2(trd(dbase, dyo(ks, 0, cb)), trd(dbase, dyo(ks, 1, cb)));
      };
      auto rdB = [&](int u) {
        const int x0 = xo(u >> 1, 0) + (u & 1) * T::HP, x1 = xo(u >> 1, 1) + (u & 1) * T::HP;
#pragma unroll
        for (int j = 0; j < NTP; ++j) fb2[u & 1][j] = frag2(trd(ring, tb[j] + x0), trd(ring, tb[j] + x1));
      };
      rdA(0);
      rdB(0);
      __builtin_amdgcn_sched_barrier(0);
      sfor<0, 2 * KS2>([&](auto uc) {
        constexpr int u = decltype(uc)::value, ks = u >> 1, cib = u & 1;
        if constexpr (u + 1 < 2 * KS2) {
          if constexpr (((u + 1) & 1) == 0) rdA((u + 1) >> 1);
          rdB(u + 1);
        }
        side(uc);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < NTP; ++j)
#pragma unroll
          for (int cb = 0; cb < 2; ++cb)
            acc4[j][cb * 2 + cib] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa2[ks & 1][cb], fb2[u & 1][j], acc4[j][cb * 2 + cib], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      });
      return;
    }
    constexpr int LA = GN ? (PW == 16 ? 1 : 0) : 2;  // fragment lookahead (k16 steps): what the registers allow
    bf16x8 fa[LA + 1], fb[LA + 1][NTP];
    auto rd = [&](int ks, int k) {
      fa[k] = frag2(trd(dbase, dyoff(ks, 0)), trd(dbase, dyoff(ks, 1)));
      const int x0 = xoff(ks, 0), x1 = xoff(ks, 1);
#pragma unroll
      for (int j = 0; j < NTP; ++j) fb[k][j] = frag2(trd(ring, tb[j] + x0), trd(ring, tb[j] + x1));
    };
#pragma unroll
    for (int k = 0; k < LA; ++k) rd(k, k);
    __builtin_amdgcn_sched_barrier(0);
    sfor<0, T::KS>([&](auto kc) {
      constexpr int ks = decltype(kc)::value;
      if constexpr (ks + LA < T::KS) rd(ks + LA, (ks + LA) % (LA + 1));
      side(kc);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < NTP; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[ks % (LA + 1)], fb[ks % (LA + 1)][j], acc[j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    });
  };

  u32x4 vx[WR_LX], vy[WR_LY];
  unsigned vm = 0;
  constexpr int NSUB = T::M16 ? 2 * (T::NV / 32) : T::KS;  // MFMA sub-steps per computed plane
  static_assert(WR_LX + WR_LY <= NSUB, "one staging piece per sub-step at most");
  PhaseStamps ps;
  ps.begin();
  WRPlane pw = walk.next(g);
  load_plane(pw, vx, vy, vm);
  WRPlane pc{};
  int s = 0;
  while (pw.valid || (pc.valid && pc.out)) {
    ps.mark_now();
    gn_refresh(pw);
    const WRPlane pl = walk.next(g);
    if constexpr (HOIST) column(pl);
    const int xs = s & 3, ds = s & 1;
    const bool wv = pw.valid, wo = pw.valid && pw.out;
    // sub-step u: piece u (x pieces first, then dy) of plane s written, its register reloaded with plane s+1's
    auto side = [&](auto uc) __attribute__((always_inline)) {
      constexpr int u = decltype(uc)::value;
      if constexpr (u < WR_LX) {
        if (wv) write_x(u, vx, vm, xs);
        load_x(pl, u, vx, vm);
      } else if constexpr (u < WR_LX + WR_LY) {
        if (wo) write_y(u - WR_LX, vy, ds);
        load_y(pl, u - WR_LX, vy);
      }
    };
    ps.lap(0);
    ps.step(pc.valid && pc.out);
    if (pc.valid && pc.out) {
      if (ntap == 4)
        compute((s - 1) & 1, (s - 3) & 3, (s - 2) & 3, (s - 1) & 3, std::integral_constant<int, 4>{}, side);
      else
        compute((s - 1) & 1, (s - 3) & 3, (s - 2) & 3, (s - 1) & 3, std::integral_constant<int, 3>{}, side);
    } else {
      sfor<0, WR_LX + WR_LY>([&](auto uc) { side(uc); });
    }
    ps.lap(1);
    __syncthreads();
    ps.lap(2);
    pc = pw;
    pw = pl;
    ++s;
  }
  ps.end(wr_stamps, (blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)) & 4095, wave, lane);
  // D[row = co][col = ci]: lane col ci0 + (lane&31), rows co0 + (i&3) + 8(i>>2) + 4h. Buffer stores with 32-bit
  // offsets computed here (the host keeps the slabs below 2 GiB): no 64-bit addresses held across the walk.
  int t0 = tid;
  asm volatile("" : "+v"(t0));
  const int r = t0 & 31, w8 = t0 >> 6;
  const auto prs = __builtin_amdgcn_make_buffer_rsrc((void*)part, 0, 0x7FFFFFFF, 0x00020000);
  if constexpr (T::M16) {  // lane: D[co 16 cb + 4 (lane >> 4) + k][ci 16 cib + (lane & 15)] of each (cb, cib) block
    const int l16 = t0 & 15, g4 = (t0 >> 4) & 3;
#pragma unroll
    for (int j = 0; j < MAXT; ++j) {
      if (j < ntap) {
        const int tt = w8 + 8 * j;
#pragma unroll
        for (int blk = 0; blk < 4; ++blk) {
          const int cb = blk >> 1, cib = blk & 1;
          const int base = ((split * 27 + tt) * g.cout_p + co0 + 16 * cb + 4 * g4) * g.cin_p + ci0 + 16 * cib + l16;
          const u32x4 ua = __builtin_bit_cast(u32x4, acc4[j][blk]);  // (whole-vector bit_cast: see below)
#pragma unroll
          for (int k = 0; k < 4; ++k)
            __builtin_amdgcn_raw_buffer_store_b32(ua[k], prs, (unsigned)((base + k * g.cin_p) * 4), 0, 0);
        }
      }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < MAXT; ++j) {
    if (j < ntap) {
      const int tt = w8 + 8 * j;
      const int base = ((split * 27 + tt) * g.cout_p + co0 + 4 * hh) * g.cin_p + ci0 + r;
      // (the whole accumulator is bit-cast first: a bit_cast of a single element of the fp32 vector fed to
      // raw_buffer_store_b32 is miscompiled by ROCm 7.2 clang into stores of element 0)
      typedef __attribute__((ext_vector_type(16))) uint32_t u32x16;
      const u32x16 ua = __builtin_bit_cast(u32x16, acc[j]);
#pragma unroll
      for (int i = 0; i < 16; ++i)
        __builtin_amdgcn_raw_buffer_store_b32(ua[i], prs, (unsigned)((base + ((i & 3) + 8 * (i >> 2)) * g.cin_p) * 4),
                                              0, 0);
    }
  }
}


// ---------------------------------------------------------------------------------------------------------------------
// Round 4: the 16 x 16-tile weight-gradient ring (96^3 and 48^3 levels) with LDS-DMA staging.
// In-kernel stamps of the register-staged kernel above (r04, -DU3D_STAMPS): the younger wave of each SIMD pair spent
// 18% of its time writing the staged plane (waiting for its loads, GroupNorm, ds_write) and 22% issuing the next plane's
// loads, both between two barriers with no MFMA beside them, at a held clock of 2.31 GHz. Here every staging byte goes
// global -> LDS by `buffer_load_dwordx4 ... lds` (no VGPRs, no write phase), issued between the MFMA sub-steps:
//   * x: into a 5-slot ring in the final half-planar layout (row pitch 32 B, 16 channels per half-plane); the GroupNorm +
//     ReLU prologue runs IN PLACE one step later (each lane transforms the 16 B its own DMA wrote, after a counted
//     vmcnt: no barrier needed between the DMA and the transform);
//   * dy: into a 3-slot ring, no transform;
//   * 5 / 3 slots because a DMA lands while the step's MFMAs read their three (one) slots and one slot is being
//     transformed; the plane barrier is a bare s_barrier behind an lgkmcnt(0) wait (a __syncthreads would drain the
//     DMAs in flight: vmcnt(0)).
// One DMA instruction = 32 rows x 32 B of one half-plane (1 KB, lane-contiguous: lane L -> row 32 i + L / 2, chunk L & 1).
// x half-plane: 324 halo rows -> 11 instructions (the last one spills 28 rows into padding: 352 rows per half-plane);
// waves 0-3 fill half 0, waves 4-7 half 1 (instructions wv, wv + 4, wv + 8; wave 3's third one is a dummy into junk);
// dy half-plane: 256 voxels -> 8 instructions, two per wave. LDS: 5 x 22.5 KB + 3 x 16 KB + 1 KB = 159 KB.
constexpr int WD_HROWS = 352;
constexpr int WD_HP = WD_HROWS * 32;  // x half-plane
constexpr int WD_SLOT = 2 * WD_HP;
constexpr int WD_DHP = 256 * 32;      // dy half-plane
constexpr int WD_DSLOT = 2 * WD_DHP;
constexpr int WD_NXS = 5, WD_NDS = 3;
#ifndef U3D_WD_LA
#define U3D_WD_LA 1
#endif
constexpr int WD_LA = U3D_WD_LA;  // MFMA sub-steps of fragment reads in flight
constexpr int WD_LDS = WD_NXS * WD_SLOT + WD_NDS * WD_DSLOT + 1024;
static_assert(WD_LDS <= 160 * 1024, "LDS");

// buffer_load_dwordx4 ... lds as inline asm: the compiler's wait-count pass treats the builtin's LDS write as aliasing
// every later ds_read and puts an s_waitcnt vmcnt(0) in front of the next MFMA fragment read (measured in the ISA),
// which would serialise each DMA with the MFMA chain. The kernel orders the DMAs itself: a counted vmcnt before the
// in-place transform and an lgkmcnt-only barrier (the hardware counts the asm loads in vmcnt like any other, so every
// wait the compiler inserts for its own loads stays conservative). rsrc = the 4-dword buffer descriptor (SGPRs),
// m0 = the wave-uniform LDS destination, off = this lane's byte offset.
typedef __attribute__((ext_vector_type(4))) unsigned u32x4s;
__device__ __forceinline__ u32x4s buf_desc(const void* base, int bytes) {
  const unsigned long long a = (unsigned long long)base;
  return u32x4s{(unsigned)a, (unsigned)(a >> 32) & 0xffffu, (unsigned)bytes, 0x00020000u};
}
// (m0 is a reserved register: clang warns that the clobber may not be honoured. The kernel's own code never uses m0 —
// checked in the ISA, tools/disasm.py — so the clobber only documents the asm's side effect.)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void dma16(const u32x4s& rsrc, const char* lds_dst, unsigned off) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)lds_dst);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %2, 0 offen lds" : : "v"(off), "s"(m0),
               "s"(rsrc) : "memory", "m0");
}
#pragma clang diagnostic pop

template <bool GN>
__global__ __launch_bounds__(WR_NT, 1) void wgrad_ring_dma_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                                 const float* __restrict__ gstat,
                                                                 const float* __restrict__ gamma,
                                                                 const float* __restrict__ beta,
                                                                 float* __restrict__ part, WRGeom g) {
  constexpr int HW = 18, NR = 324, PW = 16, KS2 = 8;  // 16 x 16 plane tile: 18 x 18 halo rows, 8 k steps of 32 voxels
  __shared__ __attribute__((aligned(16))) char lds[WD_LDS];
  char* const ring = lds;
  char* const dyr = lds + WD_NXS * WD_SLOT;
  char* const junk = dyr + WD_NDS * WD_DSLOT;
  // (wave through readfirstlane: the compiler then knows every per-wave choice — tap count, DMA half — is uniform and
  // emits scalar branches; an exec-masked branch makes its wait-count pass drain all loads at the join)
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hf = wave >> 2, wv = wave & 3;  // DMA half-plane / wave within it
  const int cofs = 16 * hf + 8 * (lane & 1);  // this lane's 8 channels (DMA + transform) within the 32-channel tile
  const TileSplit ts = xcd_tile_split();
  const int ci0 = ts.tx * 32, co0 = ts.ty * 32, split = ts.split;
  WRWalk walk{};
  walk.o_next = (long long)split * g.per;
  walk.o_end = min(g.planes, walk.o_next + g.per);
  walk.done = false;
  walk.zin = 1;
  walk.zlast = 0;
  const u32x4s xrs = buf_desc(x, (int)g.xbytes), yrs = buf_desc(dy, (int)g.ybytes);
  f32x2 sc[4], sh[4];
  int gn_n = -1;
  const bool cok = ci0 + cofs < g.cin, dok = co0 + cofs < g.cout;

  // Per-lane DMA addressing, hoisted out of the walk: a lane's row of x piece j (instruction i = wv + 4 j) is the halo
  // row (hh, hw) = divmod(32 i + lane / 2, 18) of every plane, its dy voxel (v / 16, v % 16), v = 32 i + lane / 2; so
  // its byte offset is a per-lane constant plus a wave-uniform plane base, and its in-volume test changes only with
  // the column (n, h0, w0). Per plane and piece that leaves one add and one select (the per-plane integer address math
  // of the first version cost ~30 VALU + SALU per piece, issue slots the MFMA chain needs: r04 stamps / ISA).
  int xlo[3], ylo[2], xhh[3], xhw[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int row = 32 * (wv + 4 * j) + (lane >> 1);
    xhh[j] = row / HW;
    xhw[j] = row % HW;
    xlo[j] = ((xhh[j] * g.w + xhw[j]) * g.cin + ci0 + cofs) * 2;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int v = 32 * (wv + 4 * j) + (lane >> 1);
    ylo[j] = (((v >> 4) * g.w + (v & 15)) * g.cout + co0 + cofs) * 2;
  }
  unsigned xin = 0, yin = 0;  // per column: bit j = x piece j's row / dy piece j's voxel inside the volume
  int col_h0 = -1, col_w0 = -1;
  auto column = [&](const WRPlane& p) {
    if (p.valid && (p.h0 != col_h0 || p.w0 != col_w0)) {  // uniform: once per run of the walk
      col_h0 = p.h0;
      col_w0 = p.w0;
      xin = yin = 0;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int i = wv + 4 * j, row = 32 * i + (lane >> 1);
        const bool ok = cok && i < 11 && row < NR && (unsigned)(p.h0 - 1 + xhh[j]) < (unsigned)g.h &&
                        (unsigned)(p.w0 - 1 + xhw[j]) < (unsigned)g.w;
        xin |= (ok ? 1u : 0u) << j;
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int v = 32 * (wv + 4 * j) + (lane >> 1);
        const bool ok = dok && p.h0 + (v >> 4) < g.h && p.w0 + (v & 15) < g.w;
        yin |= (ok ? 1u : 0u) << j;
      }
    }
  };
  // DMA of x piece j of plane p into slot xs; bit j of m = the lane's row is in the volume
  auto dma_x = [&](const WRPlane& p, int j, int xs, unsigned& m) {
    const int i = wv + 4 * j;
    const bool pv = p.valid && (unsigned)p.zin < (unsigned)g.d;  // uniform
    const int base = (((p.n * g.d + p.zin) * g.h + p.h0 - 1) * g.w + p.w0 - 1) * g.cin * 2;
    const bool ok = pv && ((xin >> j) & 1u);
    const unsigned off = ok ? (unsigned)(base + xlo[j]) : 0xFFFFFFF0u;
    dma16(xrs, i < 11 ? ring + xs * WD_SLOT + hf * WD_HP + i * 1024 : junk, off);
    m = (j == 0 ? 0u : m) | ((ok ? 1u : 0u) << j);
  };
  auto dma_y = [&](const WRPlane& p, int j, int ds) {
    const int i = wv + 4 * j;
    const bool pv = p.valid && p.out;
    const int base = (((p.n * g.d + p.zin - 1) * g.h + p.h0) * g.w + p.w0) * g.cout * 2;
    const unsigned off = pv && ((yin >> j) & 1u) ? (unsigned)(base + ylo[j]) : 0xFFFFFFF0u;
    dma16(yrs, dyr + ds * WD_DSLOT + hf * WD_DHP + i * 1024, off);
  };
  // in-place GroupNorm + ReLU of x piece j in slot xs (the 16 B this lane's own DMA wrote; padding rows stay zero)
  auto xform_x = [&](int j, int xs, unsigned m) {
    const int i = wv + 4 * j;
    char* a = (i < 11 ? ring + xs * WD_SLOT + hf * WD_HP + i * 1024 : junk) + lane * 16;
    u32x4 v = *reinterpret_cast<u32x4*>(a);
    v = gn_relu8(v, sc, sh);
    if (!((m >> j) & 1u)) v = u32x4{0u, 0u, 0u, 0u};
    *reinterpret_cast<u32x4*>(a) = v;
  };
  auto gn_refresh = [&](const WRPlane& p) {
    if (GN && p.valid && p.n != gn_n) {
      gn_n = p.n;
      gn_coef8(gstat, gamma, beta, g.gn_groups, g.cin, p.n, ci0 + cofs, sc, sh);
    }
  };
  auto bar = [&]() {  // plane barrier: the transforms' LDS writes done, the DMAs in flight stay in flight
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };

  constexpr int MAXT = 4;
  f32x4 acc4[MAXT][4];
#pragma unroll
  for (int j = 0; j < MAXT; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) acc4[j][e] = f32x4{0.f, 0.f, 0.f, 0.f};
  int tap_row[MAXT], tap_d[MAXT];
#pragma unroll
  for (int j = 0; j < MAXT; ++j) {
    const int t = min(wave + 8 * j, 26);
    tap_d[j] = t / 9;
    tap_row[j] = (((t / 3) % 3) * HW + t % 3) * 32;
  }
  const int ntap = (27 - wave + 7) / 8;
  const int q = (lane & 15) >> 2, pp = lane & 3, g4 = lane >> 4;
  const int v16[2] = {4 * g4 + q, 16 + 4 * g4 + q};

  // output plane from x slots s0, s0+1, s0+2 (mod 5) and dy slot ds; side(u) = the staging ops of sub-step u
  auto compute = [&](int ds, int s0, auto ntc, auto&& side) __attribute__((always_inline)) {
    constexpr int NTP = decltype(ntc)::value;
    int tb[NTP];
#pragma unroll
    for (int j = 0; j < NTP; ++j) {
      const int sl = s0 + tap_d[j];
      tb[j] = (sl >= WD_NXS ? sl - WD_NXS : sl) * WD_SLOT + tap_row[j];
    }
    const char* dbase = dyr + ds * WD_DSLOT;
    auto dyo = [&](int ks, int m, int cb) { return cb * WD_DHP + (32 * ks + v16[m]) * 32 + 8 * pp; };
    auto xo = [&](int ks, int m) {
      const int a = 32 * ks / PW, b = 32 * ks % PW, v = v16[m];
      return (a * HW + b + v + (v >= PW - b ? 2 : 0)) * 32 + 8 * pp;
    };
    // fragment lookahead: the reads of sub-step u + WD_LA are issued before the MFMAs of sub-step u
    constexpr int NB = WD_LA + 1, NA = (WD_LA + 1) / 2 + 1;
    bf16x8 fa2[NA][2], fb2[NB][NTP];
    auto rdA = [&](int ks) {
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) fa2[ks % NA][cb] = frag2(trd(dbase, dyo(ks, 0, cb)), trd(dbase, dyo(ks, 1, cb)));
    };
    auto rdB = [&](int u) {
      const int x0 = xo(u >> 1, 0) + (u & 1) * WD_HP, x1 = xo(u >> 1, 1) + (u & 1) * WD_HP;
#pragma unroll
      for (int j = 0; j < NTP; ++j) fb2[u % NB][j] = frag2(trd(ring, tb[j] + x0), trd(ring, tb[j] + x1));
    };
    sfor<0, WD_LA>([&](auto uc) {
      constexpr int u = decltype(uc)::value;
      if constexpr ((u & 1) == 0) rdA(u >> 1);
      rdB(u);
    });
    __builtin_amdgcn_sched_barrier(0);
    sfor<0, 2 * KS2>([&](auto uc) {
      constexpr int u = decltype(uc)::value, ks = u >> 1, cib = u & 1;
      if constexpr (u + WD_LA < 2 * KS2) {
        if constexpr (((u + WD_LA) & 1) == 0) rdA((u + WD_LA) >> 1);
        rdB(u + WD_LA);
      }
      side(uc);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < NTP; ++j)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
          acc4[j][cb * 2 + cib] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa2[ks % NA][cb], fb2[u % NB][j],
                                                                          acc4[j][cb * 2 + cib], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    });
  };

  PhaseStamps ps;
  ps.begin();
  // plane counter s: plane s sits in x slot s % 5 / dy slot s % 3 (DMA'd during step s-1, transformed at step s)
  unsigned ma = 0, mb = 0;  // row masks of the planes in flight (rotating)
  WRPlane pw = walk.next(g);  // plane 0
  gn_refresh(pw);
  column(pw);
#pragma unroll
  for (int j = 0; j < 3; ++j) dma_x(pw, j, 0, ma);
#pragma unroll
  for (int j = 0; j < 2; ++j) dma_y(pw, j, 0);
  WRPlane pc{};
  int x5 = 0, d3 = 0;  // s % 5, s % 3
  auto step = [&](unsigned& mcur, unsigned& mnxt) __attribute__((always_inline)) {
    const WRPlane pl = walk.next(g);  // plane s + 1
    const int xn = x5 == WD_NXS - 1 ? 0 : x5 + 1, dn = d3 == WD_NDS - 1 ? 0 : d3 + 1;
    gn_refresh(pw);
    column(pl);
    // sub-steps 0-4: DMA plane s+1; 6-8: transform plane s (its DMAs were issued a step ago: vmcnt(5) leaves only the
    // five just issued in flight)
    auto side = [&](auto uc) __attribute__((always_inline)) {
      constexpr int u = decltype(uc)::value;
      if constexpr (u < 3) dma_x(pl, u, xn, mnxt);
      else if constexpr (u < 5) dma_y(pl, u - 3, dn);
      else if constexpr (u >= 6 && u < 9) {
        if constexpr (u == 6) {
          __builtin_amdgcn_sched_barrier(0);
          asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
          __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (GN) xform_x(u - 6, x5, mcur);
      }
    };
    ps.mark_now();
    ps.step(pc.valid && pc.out);
    if (pc.valid && pc.out) {
      const int s0 = x5 >= 3 ? x5 - 3 : x5 + 2, dsc = d3 == 0 ? 2 : d3 - 1;  // planes s-3.. / dy of plane s-1
      if (ntap == 4)
        compute(dsc, s0, std::integral_constant<int, 4>{}, side);
      else
        compute(dsc, s0, std::integral_constant<int, 3>{}, side);
    } else {
      sfor<0, 2 * KS2>([&](auto uc) { side(uc); });
    }
    ps.lap(1);
    bar();
    ps.lap(2);
    pc = pw;
    pw = pl;
    x5 = xn;
    d3 = dn;
  };
  while (pw.valid || (pc.valid && pc.out)) {
    step(ma, mb);
    if (!(pw.valid || (pc.valid && pc.out))) break;
    step(mb, ma);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may land after the workgroup's LDS is released
  ps.end(wr_stamps, (blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)) & 4095, wave, lane);
  int t0 = tid;
  asm volatile("" : "+v"(t0));
  const int w8 = t0 >> 6;
  const auto prs = __builtin_amdgcn_make_buffer_rsrc((void*)part, 0, 0x7FFFFFFF, 0x00020000);
  const int l16 = t0 & 15, gq = (t0 >> 4) & 3;
#pragma unroll
  for (int j = 0; j < MAXT; ++j) {
    if (j < ntap) {
      const int tt = w8 + 8 * j;
#pragma unroll
      for (int blk = 0; blk < 4; ++blk) {
        const int cb = blk >> 1, cib = blk & 1;
        const int base = ((split * 27 + tt) * g.cout_p + co0 + 16 * cb + 4 * gq) * g.cin_p + ci0 + 16 * cib + l16;
        const u32x4 ua = __builtin_bit_cast(u32x4, acc4[j][blk]);
#pragma unroll
        for (int k = 0; k < 4; ++k)
          __builtin_amdgcn_raw_buffer_store_b32(ua[k], prs, (unsigned)((base + k * g.cin_p) * 4), 0, 0);
      }
    }
  }
}

}  // namespace u3d

using namespace u3d;

static void wr_geom(int n, int cin, int d, int h, int w, int cout, WRGeom& g) {
  g = WRGeom{};
  g.n = n; g.d = d; g.h = h; g.w = w; g.cin = cin; g.cout = cout;
  g.cin_p = round_up(cin, 32); g.cout_p = round_up(cout, 32);
  // plane tile: 16 x 16 unless the plane is 12- or 24-wide (and not a multiple of 16), where 16-wide tiles would spend
  // 1/3 (24) or 1/4 (12) of every k step on voxels past the volume
  g.ph = g.pw = 16;
  if (opt(OPT_WR_TILE16) == 0 && w % 16 != 0 && w % 12 == 0 && h % 12 == 0) {
    g.ph = 12;
    g.pw = w % 24 == 0 ? 24 : 12;
  }
  g.nbh = cdiv(h, g.ph); g.nbw = cdiv(w, g.pw);
  g.planes = (long long)n * g.nbh * g.nbw * d;
  g.xbytes = (long long)n * d * h * w * cin * 2;
  g.ybytes = (long long)n * d * h * w * cout * 2;
}


extern "C" int u3d_conv_wgrad_ring_splits_target(int n, int cin, int d, int h, int w, int cout, int wgs) {
  WRGeom g;
  wr_geom(n, cin, d, h, w, cout, g);
  const long long tiles = (long long)(g.cin_p / 32) * (g.cout_p / 32);
  const long long target = std::max(1, wgs);  // workgroups aimed at
  const long long want = std::max(1LL, std::min(g.planes, target / tiles));
  const long long per = (g.planes + want - 1) / want;
  return (int)((g.planes + per - 1) / per);  // every split receives planes: no zero-filled slabs
}

// one workgroup per CU (OPT_WR_WGS, default 256): each split's plane range is walked by one resident workgroup
extern "C" int u3d_conv_wgrad_ring_splits(int n, int cin, int d, int h, int w, int cout) {
  return u3d_conv_wgrad_ring_splits_target(n, cin, d, h, w, cout, opt(OPT_WR_WGS));
}

extern "C" int u3d_conv_wgrad_ring(const void* dy, const void* x, int n, int cin, int d, int h, int w, int cout,
                                   const float* gn_stats, const float* gn_gamma, const float* gn_beta, int gn_groups,
                                   float* partials, int nsplit, u3d_stream_t stream) {
  U3D_REQUIRE(dy && x && partials && nsplit >= 1 && n >= 1, "wgrad_ring: bad args");
  U3D_REQUIRE(cin % 8 == 0 && cout % 8 == 0, "wgrad_ring: channels must be multiples of 8");
  U3D_REQUIRE(!gn_stats || (gn_gamma && gn_beta && gn_groups > 0 && cin % gn_groups == 0), "wgrad_ring: bad GN");
  WRGeom g;
  wr_geom(n, cin, d, h, w, cout, g);
  U3D_REQUIRE(g.xbytes < (1LL << 31) && g.ybytes < (1LL << 31), "wgrad_ring: tensors beyond the 2 GiB offset range");
  U3D_REQUIRE((long long)nsplit * 27 * g.cout_p * g.cin_p * 4 < (1LL << 31), "wgrad_ring: partial slabs beyond 2 GiB");
  g.per = (int)((g.planes + nsplit - 1) / nsplit);
  g.gn_groups = gn_groups;
  const int ns_eff = (int)((g.planes + g.per - 1) / g.per);
  hipStream_t s = (hipStream_t)stream;
  if (ns_eff < nsplit)  // trailing slabs would stay unwritten
    U3D_HIP(hipMemsetAsync(partials + (long long)ns_eff * 27 * g.cout_p * g.cin_p, 0,
                           (size_t)(nsplit - ns_eff) * 27 * g.cout_p * g.cin_p * 4, s));
  dim3 grid(g.cin_p / 32, g.cout_p / 32, ns_eff);
#define U3D_WR(GN_, PH_, PW_)                                                                                       \
  hipLaunchKernelGGL((wgrad_ring_kernel<GN_, PH_, PW_>), grid, dim3(WR_NT), 0, s, (const bf16*)dy, (const bf16*)x, \
                     gn_stats, gn_gamma, gn_beta, partials, g)
  const bool gn = gn_stats != nullptr;
  if (g.pw == 24) {
    if (gn) U3D_WR(true, 12, 24); else U3D_WR(false, 12, 24);
  } else if (g.pw == 12) {
    if (gn) U3D_WR(true, 12, 12); else U3D_WR(false, 12, 12);
  } else {  // 16 x 16 tiles: LDS-DMA staging (round 4; the register-staged 16 x 16 form was dropped in round 5)
    if (gn)
      hipLaunchKernelGGL((wgrad_ring_dma_kernel<true>), grid, dim3(WR_NT), 0, s, (const bf16*)dy, (const bf16*)x,
                         gn_stats, gn_gamma, gn_beta, partials, g);
    else
      hipLaunchKernelGGL((wgrad_ring_dma_kernel<false>), grid, dim3(WR_NT), 0, s, (const bf16*)dy, (const bf16*)x,
                         gn_stats, gn_gamma, gn_beta, partials, g);
  }
#undef U3D_WR
  return check_launch("wgrad_ring_kernel");
}
