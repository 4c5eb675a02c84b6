// Weight gradient of the 3^3 convolutions on bf16 NDHWC tensors, halo-brick form (gfx950).
//
//   dW[t][co][ci] = sum_{n, q}  dy[n, q, co] * A[n, q*s + t - 1, ci],   A = relu(gn(x)) (prologue)
//
// One workgroup (8 waves) owns a (32 co) x (32 ci) tile for ALL 27 taps and a range of output bricks
// (BD x BH x BW voxels). Per brick the dy brick and the input halo brick ((BD-1)s+3 x (BH-1)s+3 x (BW-1)s+3
// voxels, GroupNorm+ReLU applied once per element) sit in LDS in their natural channel-contiguous layout;
// the next brick's dy + halo are prefetched into registers while the MFMAs run. Both MFMA operands need
// the voxel index as the k dimension, i.e. a transposed read of channel-contiguous rows:
// ds_read_b64_tr_b16 gives it, and because every lane supplies its own row address the 27 shifted tap
// windows of the halo are read with no data movement (row address = brick voxel row + tap offset). The dy
// fragment is shared by all taps of a wave. Reference: autograd of F.conv3d in Conv3d.forward (unet3D.py:27).
#include <cstdlib>
#include <type_traits>

#include "common.h"

namespace u3d {

typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
struct WBGeom {
  int n;
  int cin, cout, cin_p, cout_p;
  int id, ih, iw;
  int od, oh, ow;
  int nbd, nbh, nbw;  // bricks per dim
  long long nbricks;  // n * nbd * nbh * nbw
  long long per_split;
  int gn_groups;
};

__device__ __forceinline__ v4i16 tr_read(const char* lds_base, int byte_off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_v4i16*)((__attribute__((address_space(3))) char*)lds_base + byte_off));
}

__device__ __forceinline__ bf16x8 frag_from(v4i16 lo, v4i16 hi) {
  typedef short v8i16 __attribute__((ext_vector_type(8)));
  v8i16 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// BUF: operands below 2 GiB -> branch-free buffer loads with 32-bit offsets (a masked piece reads zeros at the
// sentinel offset; a divergent branch around each prefetch load pulls its wait ahead of the MFMAs it should overlap)
template <int BD, int BH, int BW, int S, int NCO = 1, bool BUF = false>
__global__ __launch_bounds__(512, 1) void wgrad_brick_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                            const float* __restrict__ gstat,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta, float* __restrict__ part,
                                                            WBGeom g) {
  constexpr int NV = BD * BH * BW, NKS = NV / 16;
  constexpr int HD = (BD - 1) * S + 3, HH = (BH - 1) * S + 3, HW = (BW - 1) * S + 3, NH = HD * HH * HW;
  constexpr int ROWB = 64;           // 32 bf16 channels per LDS halo row
  constexpr int DROWB = 64 * NCO;    // dy rows: the NCO output-channel tiles of the workgroup side by side
  constexpr int NT = 512;
  constexpr int RPP = NT / 4;                       // halo rows per pass (thread t: chunk t&3 of row t>>2)
  constexpr int DCH = 4 * NCO, DRPP = NT / DCH;     // dy: 8-channel chunks per row, rows per pass
  constexpr int DYL = (NV + DRPP - 1) / DRPP;       // dy loads per thread
  constexpr int HLL = (NH + RPP - 1) / RPP;         // halo loads per thread
  static_assert(NV % 32 == 0, "brick voxels (an even number of 16-voxel k-steps)");
  __shared__ __attribute__((aligned(16))) char lds[NV * DROWB + NH * ROWB];
  char* dyt = lds;
  char* hal = lds + NV * DROWB;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ch = tid & 3, row0 = tid >> 2;  // fixed halo channel chunk per thread
  const int dch = tid % DCH, drow0 = tid / DCH;
  const TileSplit ts = xcd_tile_split();  // XCD-aware: the channel tiles of neighbouring brick ranges share an L2
  const int ci0 = ts.tx * 32, co0 = ts.ty * 32 * NCO;
  const long long b0 = (long long)ts.split * g.per_split;
  const long long b1 = min(g.nbricks, b0 + g.per_split);
  const bool has_gn = gstat != nullptr;

  constexpr int MAXT = 4;  // taps per wave: t = wave + 8j
  f32x16 acc[MAXT][NCO];
#pragma unroll
  for (int j = 0; j < MAXT; ++j)
#pragma unroll
    for (int c = 0; c < NCO; ++c)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[j][c][e] = 0.f;
  // stride 2: every halo w line is stored parity-split (even w first, then odd), so the lanes of a fragment read,
  // for any tap, CONSECUTIVE rows (w = 2 vw + tw -> vw, HWE + vw, vw + 1 for tw = 0, 1, 2) instead of every other row
  // (2-way bank conflicts)
  constexpr int HWE = S == 2 ? (HW + 1) / 2 : 0;
  auto wpos = [&](int hw) { return S == 2 ? ((hw & 1) ? HWE + (hw >> 1) : (hw >> 1)) : hw; };
  // tap j's halo row offset, formed where it is used (an array of 4 held across the loop cost 4 VGPRs)
  auto tap_off_of = [&](int j) {
    const int t = min(wave + 8 * j, 26);
    const int td = t / 9, th = (t / 3) % 3, tw = t % 3;
    return ((td * HH + th) * HW + (S == 2 ? (tw == 1 ? HWE : tw >> 1) : tw)) * ROWB;
  };
  const int ntap = (27 - wave + 7) / 8;  // 4 for waves 0-2, 3 for 3-7

  // fragment lane geometry: group gq = lane>>4, in-group lane i = lane&15 -> (q = i>>2, p = i&3)
  const int h = lane >> 5, gq = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int colb = (16 * (gq & 1) + 4 * p) * 2;  // byte offset of this lane's 4 columns

  u32x4 pdy[DYL], phl[HLL];
  // the GroupNorm coefficients of the current sample in LDS (per 8-channel chunk), read only inside commit: held in
  // registers across the MFMA loop they pushed the 3-plane stride-2 form past 256 VGPRs
  __shared__ f32x2 gsc[4][4], gsh[4][4];
  int gn_n = -1;

  auto decode = [&](long long b, int& n, int& od0, int& oh0, int& ow0) {
    long long t = b;
    const int bw_ = (int)(t % g.nbw); t /= g.nbw;
    const int bh_ = (int)(t % g.nbh); t /= g.nbh;
    const int bd_ = (int)(t % g.nbd);
    n = (int)(t / g.nbd);
    od0 = bd_ * BD; oh0 = bh_ * BH; ow0 = bw_ * BW;
  };
  const auto yrs = __builtin_amdgcn_make_buffer_rsrc((void*)dy, 0, BUF ? g.n * g.od * g.oh * g.ow * g.cout * 2 : 0,
                                                     0x00020000);
  const auto xrs = __builtin_amdgcn_make_buffer_rsrc((void*)x, 0, BUF ? g.n * g.id * g.ih * g.iw * g.cin * 2 : 0,
                                                     0x00020000);
  auto prefetch = [&](long long b) {
    int n, od0, oh0, ow0;
    decode(b, n, od0, oh0, ow0);
#pragma unroll
    for (int i = 0; i < DYL; ++i) {
      const int v = drow0 + i * DRPP;
      const int vw = v % BW, vh = (v / BW) % BH, vd = v / (BW * BH);
      const int zd = od0 + vd, zh = oh0 + vh, zw = ow0 + vw, co = co0 + dch * 8;
      const bool ok = v < NV && zd < g.od && zh < g.oh && zw < g.ow && co < g.cout;
      if constexpr (BUF) {
        const unsigned off = ok ? (unsigned)(((((n * g.od + zd) * g.oh + zh) * g.ow + zw) * g.cout + co) * 2) : 0xFFFFFFF0u;
        pdy[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(yrs, off, 0, 0));
      } else {
        u32x4 val = {0u, 0u, 0u, 0u};
        if (ok)
          val = *reinterpret_cast<const u32x4*>(dy + ((((long long)n * g.od + zd) * g.oh + zh) * g.ow + zw) * g.cout + co);
        pdy[i] = val;
      }
    }
    const int id0 = od0 * S - 1, ih0 = oh0 * S - 1, iw0 = ow0 * S - 1, c = ci0 + ch * 8;
#pragma unroll
    for (int i = 0; i < HLL; ++i) {
      const int v = row0 + i * RPP;
      const int hw = v % HW, hh = (v / HW) % HH, hd = v / (HW * HH);
      const int zd = id0 + hd, zh = ih0 + hh, zw = iw0 + hw;
      const bool ok = v < NH && (unsigned)zd < (unsigned)g.id && (unsigned)zh < (unsigned)g.ih &&
                      (unsigned)zw < (unsigned)g.iw && c < g.cin;
      if constexpr (BUF) {
        const unsigned off = ok ? (unsigned)(((((n * g.id + zd) * g.ih + zh) * g.iw + zw) * g.cin + c) * 2) : 0xFFFFFFF0u;
        phl[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0));
      } else {
        u32x4 val = {0u, 0u, 0u, 0u};
        if (ok)
          val = *reinterpret_cast<const u32x4*>(x + ((((long long)n * g.id + zd) * g.ih + zh) * g.iw + zw) * g.cin + c);
        phl[i] = val;
      }
    }
  };
  auto commit = [&](long long b) {
    int n, od0, oh0, ow0;
    decode(b, n, od0, oh0, ow0);
    if (has_gn && n != gn_n) {  // n is uniform over the workgroup: the barrier is reached by all or none
      gn_n = n;
      if (tid < 4) {
        f32x2 sc[4], sh[4];
        gn_coef8(gstat, gamma, beta, g.gn_groups, g.cin, n, ci0 + tid * 8, sc, sh);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          gsc[tid][k] = sc[k];
          gsh[tid][k] = sh[k];
        }
      }
      __syncthreads();
    }
    f32x2 sc[4], sh[4];
    if (has_gn) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        sc[k] = gsc[ch][k];
        sh[k] = gsh[ch][k];
      }
    }
#pragma unroll
    for (int i = 0; i < DYL; ++i) {
      const int v = drow0 + i * DRPP;
      if (v < NV) *reinterpret_cast<u32x4*>(dyt + v * DROWB + dch * 16) = pdy[i];
    }
    const int id0 = od0 * S - 1, ih0 = oh0 * S - 1, iw0 = ow0 * S - 1;
#pragma unroll
    for (int i = 0; i < HLL; ++i) {
      const int v = row0 + i * RPP;
      if (v < NH) {
        u32x4 val = phl[i];
        const int hw = v % HW, hl = v - hw;  // hl = (hd * HH + hh) * HW
        if (has_gn) {
          const int hh = (v / HW) % HH, hd = v / (HW * HH);
          const int zd = id0 + hd, zh = ih0 + hh, zw = iw0 + hw;
          if ((unsigned)zd < (unsigned)g.id && (unsigned)zh < (unsigned)g.ih && (unsigned)zw < (unsigned)g.iw)
            val = gn_relu8(val, sc, sh);
        }
        *reinterpret_cast<u32x4*>(hal + (hl + wpos(hw)) * ROWB + ch * 16) = val;
      }
    }
  };

  if (b0 < b1) {
    prefetch(b0);
    commit(b0);
  }
  __syncthreads();
  for (long long b = b0; b < b1; ++b) {
    const bool more = b + 1 < b1;
    prefetch(more ? b + 1 : b);
    // K loop over the brick's voxels, 16 per MFMA; software-pipelined: the fragments of step ks+1 are read
    // while step ks's MFMAs run, and the tap count is a compile-time constant per wave (4 or 3) so the loop
    // has no divergent branches between the LDS reads and the MFMAs
    auto kloop = [&](auto ntc) {
      constexpr int NT = decltype(ntc)::value;
      auto rows = [&](int ks, int (&ar)[2], int (&hr)[2]) {
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          const int k = ks * 16 + 8 * h + 4 * m + q;
          const int vw = k % BW, vh = (k / BW) % BH, vd = k / (BW * BH);
          ar[m] = k * DROWB + colb;
          hr[m] = ((vd * S * HH + vh * S) * HW + (S == 2 ? vw : vw * S)) * ROWB + colb;
        }
      };
      auto frags = [&](int ks, bf16x8 (&a)[NCO], bf16x8 (&bb)[NT]) {
        int ar[2], hr[2];
        rows(ks, ar, hr);
#pragma unroll
        for (int c = 0; c < NCO; ++c) a[c] = frag_from(tr_read(dyt, ar[0] + 64 * c), tr_read(dyt, ar[1] + 64 * c));
#pragma unroll
        for (int j = 0; j < NT; ++j)
          bb[j] = frag_from(tr_read(hal, hr[0] + tap_off_of(j)), tr_read(hal, hr[1] + tap_off_of(j)));
      };
      auto mfmas = [&](const bf16x8 (&a)[NCO], const bf16x8 (&bb)[NT]) {
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
          for (int c = 0; c < NCO; ++c)
            acc[j][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[c], bb[j], acc[j][c], 0, 0, 0);
      };
      if constexpr (NCO == 1) {
        bf16x8 a0[NCO], a1[NCO], b0[NT], b1[NT];
        frags(0, a0, b0);
#pragma unroll 1
        for (int ks = 0; ks < NKS; ks += 2) {
          frags(ks + 1, a1, b1);  // NKS is even
          mfmas(a0, b0);
          if (ks + 2 < NKS) frags(ks + 2, a0, b0);
          mfmas(a1, b1);
        }
      } else {  // twice the accumulators: no fragment lookahead (the other wave of the SIMD covers the LDS reads)
#pragma unroll 1
        for (int ks = 0; ks < NKS; ++ks) {
          int ar[2], hr[2];
          rows(ks, ar, hr);
          bf16x8 a0[NCO];
#pragma unroll
          for (int c = 0; c < NCO; ++c) a0[c] = frag_from(tr_read(dyt, ar[0] + 64 * c), tr_read(dyt, ar[1] + 64 * c));
          // one tap's halo fragment at a time (4 VGPRs live instead of 16: the 3-plane stride-2 form fits 256)
#pragma unroll
          for (int j = 0; j < NT; ++j) {
            const bf16x8 bj = frag_from(tr_read(hal, hr[0] + tap_off_of(j)), tr_read(hal, hr[1] + tap_off_of(j)));
#pragma unroll
            for (int c = 0; c < NCO; ++c)
              acc[j][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0[c], bj, acc[j][c], 0, 0, 0);
          }
        }
      }
    };
    if (ntap == 4)
      kloop(std::integral_constant<int, 4>{});
    else
      kloop(std::integral_constant<int, 3>{});
    __syncthreads();  // everyone done with this brick's LDS
    if (more) commit(b + 1);
    __syncthreads();
  }
  // D[row = co][col = ci]: lane col ci0 + (lane&31), rows co0 + (i&3) + 8(i>>2) + 4h. Buffer stores with 32-bit
  // offsets computed here (the host keeps the slabs below 2 GiB): no 64-bit addresses held across the brick loop.
  int t0 = tid;
  asm volatile("" : "+v"(t0));
  const int r = t0 & 31, w8 = t0 >> 6, h8 = (t0 >> 5) & 1;
  const auto prs = __builtin_amdgcn_make_buffer_rsrc((void*)part, 0, 0x7FFFFFFF, 0x00020000);
#pragma unroll
  for (int j = 0; j < MAXT; ++j) {
    if (j < ntap) {
      const int tt = w8 + 8 * j;
#pragma unroll
      for (int c = 0; c < NCO; ++c) {
        const int base = ((ts.split * 27 + tt) * g.cout_p + co0 + 32 * c + 4 * h8) * g.cin_p + ci0 + r;
        // (the whole accumulator is bit-cast first: a bit_cast of a single element of the fp32 vector fed to
        // raw_buffer_store_b32 is miscompiled by ROCm 7.2 clang into stores of element 0)
        typedef __attribute__((ext_vector_type(16))) uint32_t u32x16;
        const u32x16 ua = __builtin_bit_cast(u32x16, acc[j][c]);
#pragma unroll
        for (int i = 0; i < 16; ++i)
          __builtin_amdgcn_raw_buffer_store_b32(ua[i], prs, (unsigned)((base + ((i & 3) + 8 * (i >> 2)) * g.cin_p) * 4),
                                                0, 0);
      }
    }
  }
}


// ------------------------------------------------------------------------------------------------------
// 1^3 weight gradient (downsample convs, fusion / classifier heads): dW[co][ci] = sum_q dy[q][co] A[q*s][ci].
// No halo: a workgroup streams chunks of 512 output voxels (linear order) of its split; the dy chunk and
// the (strided) A chunk are staged channel-contiguous in LDS, read transposed (ds_read_b64_tr_b16), and the
// 32 k16 steps of a chunk are spread over the 8 waves; the 8 per-wave partial tiles are summed in LDS in
// fixed order at the end (deterministic). Memory-bound by design (16-32 flop/B): the next chunk is
// prefetched into registers while the current one is consumed.
#ifndef U3D_W1_NV
#define U3D_W1_NV 512
#endif
constexpr int W1_NV = U3D_W1_NV;  // output voxels per chunk

struct W1Geom {
  int cin, cout, cin_p, cout_p;
  int id, ih, iw;
  int od, oh, ow;
  long long nvox;  // n * od * oh * ow
  long long per_split;
  int gn_groups;
};

template <int S, bool BUF = false>
__global__ __launch_bounds__(512, 1) void wgrad1_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                       const float* __restrict__ gstat,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, float* __restrict__ part,
                                                       W1Geom g) {
  constexpr int ROWB = 64, NT = 512, RPP = NT / 4, LD = W1_NV / RPP;  // 4 loads per operand per thread
  __shared__ __attribute__((aligned(16))) char lds[2 * W1_NV * ROWB];
  char* dyt = lds;
  char* at = lds + W1_NV * ROWB;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ch = tid & 3, row0 = tid >> 2;
  const TileSplit ts = xcd_tile_split();
  const int ci0 = ts.tx * 32, co0 = ts.ty * 32;
  const long long v0 = (long long)ts.split * g.per_split;
  const long long v1 = min(g.nvox, v0 + g.per_split);
  const bool has_gn = gstat != nullptr;
  const int h = lane >> 5, gq = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int colb = (16 * (gq & 1) + 4 * p) * 2;

  u32x4 pdy[LD], pa[LD];
  int pn[LD];
  f32x2 sc[4], sh[4];
  int gn_n = -1;
  f32x16 acc;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.f;

  // BUF (operands below 2 GiB): branch-free buffer loads with 32-bit offsets and indices (a divergent branch around
  // each prefetch load pulls its wait ahead of the MFMAs it should overlap)
  const auto yrs = __builtin_amdgcn_make_buffer_rsrc((void*)dy, 0, BUF ? (int)(g.nvox * g.cout * 2) : 0, 0x00020000);
  const auto xrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)x, 0, BUF ? (int)((long long)g.nvox / ((long long)g.od * g.oh * g.ow) * g.id * g.ih * g.iw * g.cin * 2) : 0,
      0x00020000);
  auto prefetch = [&](long long c0) {
#pragma unroll
    for (int i = 0; i < LD; ++i) {
      const long long v = c0 + row0 + i * RPP;
      if constexpr (BUF) {
        const int vi = (int)v, co = co0 + ch * 8, ci = ci0 + ch * 8;
        const bool ok = v < v1;
        int n, src;
        if (S == 1) {
          n = vi / (g.od * g.oh * g.ow);
          src = vi;
        } else {
          int t = vi;
          const int qw = t % g.ow; t /= g.ow;
          const int qh = t % g.oh; t /= g.oh;
          const int qd = t % g.od;
          n = t / g.od;
          src = ((n * g.id + 2 * qd) * g.ih + 2 * qh) * g.iw + 2 * qw;
        }
        const unsigned ob = ok && co < g.cout ? (unsigned)((vi * g.cout + co) * 2) : 0xFFFFFFF0u;
        const unsigned oa = ok && ci < g.cin ? (unsigned)((src * g.cin + ci) * 2) : 0xFFFFFFF0u;
        pdy[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(yrs, ob, 0, 0));
        pa[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(xrs, oa, 0, 0));
        pn[i] = ok ? n : -1;
        continue;
      }
      u32x4 a = {0u, 0u, 0u, 0u}, b = {0u, 0u, 0u, 0u};
      int n = -1;
      if (v < v1) {
        const int co = co0 + ch * 8, ci = ci0 + ch * 8;
        if (co < g.cout) b = *reinterpret_cast<const u32x4*>(dy + v * g.cout + co);
        long long src;
        if (S == 1) {
          src = v;
          n = (int)(v / ((long long)g.od * g.oh * g.ow));
        } else {
          long long t = v;
          const int qw = (int)(t % g.ow); t /= g.ow;
          const int qh = (int)(t % g.oh); t /= g.oh;
          const int qd = (int)(t % g.od);
          n = (int)(t / g.od);
          src = (((long long)n * g.id + 2 * qd) * g.ih + 2 * qh) * g.iw + 2 * qw;
        }
        if (ci < g.cin) a = *reinterpret_cast<const u32x4*>(x + src * g.cin + ci);
      }
      pdy[i] = b;
      pa[i] = a;
      pn[i] = n;
    }
  };
  auto commit = [&]() {
#pragma unroll
    for (int i = 0; i < LD; ++i) {
      const int v = row0 + i * RPP;
      u32x4 a = pa[i];
      if (has_gn && pn[i] >= 0) {
        if (pn[i] != gn_n) {
          gn_n = pn[i];
          gn_coef8(gstat, gamma, beta, g.gn_groups, g.cin, gn_n, ci0 + ch * 8, sc, sh);
        }
        a = gn_relu8(a, sc, sh);
      }
      *reinterpret_cast<u32x4*>(dyt + v * ROWB + ch * 16) = pdy[i];
      *reinterpret_cast<u32x4*>(at + v * ROWB + ch * 16) = a;
    }
  };

  if (v0 < v1) {
    prefetch(v0);
    commit();
  }
  __syncthreads();
  for (long long c0 = v0; c0 < v1; c0 += W1_NV) {
    const bool more = c0 + W1_NV < v1;
    prefetch(more ? c0 + W1_NV : c0);
#pragma unroll
    for (int j = 0; j < W1_NV / 16 / 8; ++j) {
      const int ks = wave + 8 * j;
      const int k0 = (ks * 16 + 8 * h + q) * ROWB + colb, k1 = k0 + 4 * ROWB;
      const bf16x8 a = frag_from(tr_read(dyt, k0), tr_read(dyt, k1));
      const bf16x8 b = frag_from(tr_read(at, k0), tr_read(at, k1));
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
    }
    __syncthreads();
    if (more) commit();
    __syncthreads();
  }
  // fixed-order sum of the 8 per-wave tiles: D[row = co][col = ci], lane col = lane&31, rows (i&3)+8(i>>2)+4h
  float* red = reinterpret_cast<float*>(lds);
  const int r = lane & 31;
#pragma unroll
  for (int i = 0; i < 16; ++i) red[(wave * 32 + (i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = acc[i];
  __syncthreads();
  float* pp = part + (long long)ts.split * g.cout_p * g.cin_p;
  for (int e = tid; e < 1024; e += NT) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) s += red[w * 1024 + e];
    const int co = e >> 5, ci = e & 31;
    pp[(long long)(co0 + co) * g.cin_p + ci0 + ci] = s;
  }
}

}  // namespace u3d

using namespace u3d;

static int wgrad_bd() { return opt(OPT_WGRAD_BD) == 2 ? 2 : 3; }  // brick depth of the stride-1 kernel

// stride 2: a workgroup covers two 32-wide output-channel tiles, so the 8x-larger input halo of a stride-2 brick is
// staged (and GroupNorm'd) once for 64 output channels
static int wb_nco(int stride, int cout) { return stride == 2 && opt(OPT_WB_S2CO64) != 0 && round_up(cout, 32) % 64 == 0 ? 2 : 1; }

static void brick_dims(int stride, int* bd, int* bh, int* bw) {
  if (stride == 1) { *bd = wgrad_bd(); *bh = 8; *bw = 16; }
  else { *bd = opt(OPT_WB_S2BD) == 2 ? 2 : 3; *bh = 4; *bw = 8; }
}

extern "C" int u3d_conv_wgrad_brick_splits(int n, int cin, int d, int h, int w, int cout, int stride) {
  int bd, bh, bw;
  brick_dims(stride, &bd, &bh, &bw);
  const int od = (d - 1) / stride + 1, oh = (h - 1) / stride + 1, ow = (w - 1) / stride + 1;
  const long long nb = (long long)n * cdiv(od, bd) * cdiv(oh, bh) * cdiv(ow, bw);
  const long long tiles = (long long)cdiv(cin, 32) * (cdiv(cout, 32) / wb_nco(stride, cout));
  const long long target = std::max(1, opt(OPT_WB_WGS));  // workgroups aimed at
  long long want = std::max(1LL, target / tiles);
  const long long ns = std::max(1LL, std::min(want, nb));
  const long long per = (nb + ns - 1) / ns;
  return (int)((nb + per - 1) / per);  // splits that all receive bricks: no zero-filled slabs
}

extern "C" int u3d_conv_wgrad_brick(const void* dy, const void* x, int n, int cin, int d, int h, int w, int cout,
                                    int stride, const float* gn_stats, const float* gn_gamma, const float* gn_beta,
                                    int gn_groups, float* partials, int nsplit, u3d_stream_t stream) {
  U3D_REQUIRE(dy && x && partials && nsplit >= 1, "wgrad_brick: null pointer");
  U3D_REQUIRE(stride == 1 || stride == 2, "wgrad_brick: stride %d", stride);
  U3D_REQUIRE(cin % 8 == 0 && cout % 8 == 0, "wgrad_brick: channels must be multiples of 8");
  U3D_REQUIRE((long long)nsplit * 27 * round_up(cin, 32) * round_up(cout, 32) * 4 < (1LL << 31),
              "wgrad_brick: partial slabs beyond the 2 GiB offset range");
  U3D_REQUIRE(!gn_stats || (gn_gamma && gn_beta && gn_groups > 0 && cin % gn_groups == 0),
              "wgrad_brick: bad GroupNorm prologue");
  WBGeom g{};
  g.n = n;
  g.cin = cin; g.cout = cout; g.cin_p = round_up(cin, 32); g.cout_p = round_up(cout, 32);
  g.id = d; g.ih = h; g.iw = w;
  g.od = (d - 1) / stride + 1; g.oh = (h - 1) / stride + 1; g.ow = (w - 1) / stride + 1;
  int bd, bh, bw;
  brick_dims(stride, &bd, &bh, &bw);
  g.nbd = cdiv(g.od, bd); g.nbh = cdiv(g.oh, bh); g.nbw = cdiv(g.ow, bw);
  g.nbricks = (long long)n * g.nbd * g.nbh * g.nbw;
  g.per_split = (g.nbricks + nsplit - 1) / nsplit;
  g.gn_groups = gn_groups;
  const int ns_eff = (int)((g.nbricks + g.per_split - 1) / g.per_split);
  hipStream_t s = (hipStream_t)stream;
  if (ns_eff < nsplit)  // trailing slabs would stay unwritten
    U3D_HIP(hipMemsetAsync(partials + (long long)ns_eff * 27 * g.cout_p * g.cin_p, 0,
                           (size_t)(nsplit - ns_eff) * 27 * g.cout_p * g.cin_p * 4, s));
  const int nco = wb_nco(stride, cout);
  dim3 grid(g.cin_p / 32, g.cout_p / 32 / nco, ns_eff);
  // buffer loads where both operands fit the 32-bit offset range (the > 2 GiB whole-volume case keeps 64-bit loads)
  const bool buf = (long long)n * g.od * g.oh * g.ow * cout * 2 < (1LL << 31) - 64 &&
                   (long long)n * d * h * w * cin * 2 < (1LL << 31) - 64;
#define U3D_WB(BD_, BH_, BW_, S_, NCO_)                                                                            \
  do {                                                                                                             \
    if (buf)                                                                                                       \
      hipLaunchKernelGGL((wgrad_brick_kernel<BD_, BH_, BW_, S_, NCO_, true>), grid, dim3(512), 0, s,               \
                         (const bf16*)dy, (const bf16*)x, gn_stats, gn_gamma, gn_beta, partials, g);               \
    else                                                                                                           \
      hipLaunchKernelGGL((wgrad_brick_kernel<BD_, BH_, BW_, S_, NCO_, false>), grid, dim3(512), 0, s,              \
                         (const bf16*)dy, (const bf16*)x, gn_stats, gn_gamma, gn_beta, partials, g);               \
  } while (0)
  if (stride == 2 && bd == 3 && nco == 2) U3D_WB(3, 4, 8, 2, 2);
  else if (stride == 2 && bd == 3) U3D_WB(3, 4, 8, 2, 1);
  else if (stride == 2 && nco == 2) U3D_WB(2, 4, 8, 2, 2);
  else if (stride == 1 && bd == 2) U3D_WB(2, 8, 16, 1, 1);
  else if (stride == 1) U3D_WB(3, 8, 16, 1, 1);
  else U3D_WB(2, 4, 8, 2, 1);
#undef U3D_WB
  return check_launch("wgrad_brick_kernel");
}

extern "C" int u3d_conv_wgrad1_splits(int n, int cin, int d, int h, int w, int cout, int stride) {
  const int od = (d - 1) / stride + 1, oh = (h - 1) / stride + 1, ow = (w - 1) / stride + 1;
  const long long chunks = ((long long)n * od * oh * ow + W1_NV - 1) / W1_NV;
  const long long tiles = (long long)cdiv(cin, 32) * cdiv(cout, 32);
  long long want = std::max(1LL, 256 / tiles);
  const long long ns = std::max(1LL, std::min(want, chunks));
  const long long per = (chunks + ns - 1) / ns;
  return (int)((chunks + per - 1) / per);  // splits that all receive voxels: no zero-filled slabs
}

extern "C" int u3d_conv_wgrad1(const void* dy, const void* x, int n, int cin, int d, int h, int w, int cout, int stride,
                               const float* gn_stats, const float* gn_gamma, const float* gn_beta, int gn_groups,
                               float* partials, int nsplit, u3d_stream_t stream) {
  U3D_REQUIRE(dy && x && partials && nsplit >= 1, "wgrad1: null pointer");
  U3D_REQUIRE(stride == 1 || stride == 2, "wgrad1: stride %d", stride);
  U3D_REQUIRE(cin % 8 == 0 && cout % 8 == 0, "wgrad1: channels must be multiples of 8");
  U3D_REQUIRE(!gn_stats || (gn_gamma && gn_beta && gn_groups > 0 && cin % gn_groups == 0), "wgrad1: bad GN");
  W1Geom g{};
  g.cin = cin; g.cout = cout; g.cin_p = round_up(cin, 32); g.cout_p = round_up(cout, 32);
  g.id = d; g.ih = h; g.iw = w;
  g.od = (d - 1) / stride + 1; g.oh = (h - 1) / stride + 1; g.ow = (w - 1) / stride + 1;
  g.nvox = (long long)n * g.od * g.oh * g.ow;
  const long long chunks = (g.nvox + W1_NV - 1) / W1_NV;
  g.per_split = (chunks + nsplit - 1) / nsplit * W1_NV;
  g.gn_groups = gn_groups;
  const int ns_eff = (int)((g.nvox + g.per_split - 1) / g.per_split);
  hipStream_t s = (hipStream_t)stream;
  if (ns_eff < nsplit)
    U3D_HIP(hipMemsetAsync(partials + (long long)ns_eff * g.cout_p * g.cin_p, 0,
                           (size_t)(nsplit - ns_eff) * g.cout_p * g.cin_p * 4, s));
  dim3 grid(g.cin_p / 32, g.cout_p / 32, ns_eff);
  // buffer loads and 32-bit indices where both operands fit the 32-bit offset range
  const bool buf = g.nvox * cout * 2 < (1LL << 31) - 64 && (long long)n * d * h * w * cin * 2 < (1LL << 31) - 64;
#define U3D_W1(S_)                                                                                                \
  do {                                                                                                            \
    if (buf)                                                                                                      \
      hipLaunchKernelGGL((wgrad1_kernel<S_, true>), grid, dim3(512), 0, s, (const bf16*)dy, (const bf16*)x,        \
                         gn_stats, gn_gamma, gn_beta, partials, g);                                               \
    else                                                                                                          \
      hipLaunchKernelGGL((wgrad1_kernel<S_, false>), grid, dim3(512), 0, s, (const bf16*)dy, (const bf16*)x,       \
                         gn_stats, gn_gamma, gn_beta, partials, g);                                               \
  } while (0)
  if (stride == 1) U3D_W1(1);
  else U3D_W1(2);
#undef U3D_W1
  return check_launch("wgrad1_kernel");
}
