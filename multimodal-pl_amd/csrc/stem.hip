// Stem convolutions with 1-2 input channels: conv1 1->32 (reference unet3D.py:1632, :602) and the
// stride-2 conv0 of unet3D_g (in_channel -> init_filter, :1514). K = 27*cin is far below one MFMA
// K-block, so this is a direct VALU conv: one thread per output voxel keeps all cout accumulators in
// registers; the standardised weights sit in LDS as fp32. Input is the model's fp32 NCDHW volume.
#include "common.h"

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
// x 32 channels from the 3 x 6 input window of each (kd, kh) row. The weights are wave-uniform: a one-block kernel
// first writes them as a contiguous fp32 [27][32] table (the packed image holds them at a 32-element stride), which
// the main kernel reads with wide scalar loads (scalar cache) and feeds to v_pk_fma_f32 as SGPR pairs with the input
// value broadcast to both halves: the kernel is bound by packed FMAs (864 per voxel, two per lane-instruction) and
// the 64 B/voxel output stores; no LDS. Same fp32 FMA chain per output (taps in order, fma(x, w, acc)) as
// stem_fwd_kernel, so results are bitwise those of the generic kernel. One thread per (output row, 4-voxel group).
template <typename T>
__global__ __launch_bounds__(1024) void stem1_wtab_kernel(const T* __restrict__ wpk, int cin_p, float* __restrict__ wt) {
  const int i = threadIdx.x;  // (t, co)
  if (i < 27 * 32) wt[i] = to_f(wpk[(long long)i * cin_p]);
}

// conv1 (cin 1 -> 32, stride 1), one voxel per lane, packed FMAs (v_pk_fma_f32) with the weights from a contiguous fp32
// table read by scalar loads: the 64-B output rows of consecutive lanes are consecutive, so each 16-B store
// instruction of a wave covers 4 KB (round 3: a four-voxels-per-lane form, lanes 256 B apart, measured 91 vs 69 us at
// 2x96^3); the three w-neighbours of a tap row are three coalesced loads. Same fp32 FMA chain per output as the
// generic kernel (OPT_STEM1 = 0): bitwise equal.
// STATS (bf16 only, round 5): the output's GroupNorm(16) partial sums from the epilogue — per voxel the two channels
// of each group (the stored bf16 values) summed and squared, reduced over the wave transposed (wave_sum_transposed:
// lane l ends with value l >> 1 = (group, sum | square)) and over the block's 4 waves in order, one [16][2] row per
// block into spart ([sample][wps][16][2]; blocks never straddle samples: the host requires d*h*w % ST == 0), then
// launch_gn16_finalize: no separate statistics pass over the 2 x 96^3 x 32 output.
template <typename T, bool STATS = false>
__global__ __launch_bounds__(ST) void stem1_fwd_kernel(const float* __restrict__ x, const float* __restrict__ wt,
                                                       T* __restrict__ y, int d, int h, int w, long long nvox,
                                                       float* __restrict__ spart = nullptr) {
  __shared__ __attribute__((aligned(16))) char tr[sizeof(T) == 2 ? ST / 64 : 1][64 * 64];  // bf16: 4 KB per wave
  __shared__ float red[STATS ? ST / 64 : 1][32];
  const long long v0 = (long long)blockIdx.x * ST + (threadIdx.x & ~63);  // the wave's first voxel
  const long long vr = (long long)blockIdx.x * ST + threadIdx.x;
  if constexpr (sizeof(T) != 2) {
    if (vr >= nvox) return;
  }
  const long long v = vr < nvox ? vr : nvox - 1;  // (bf16: every lane takes part in the wave's LDS transpose)
  const int xx = (int)(v % w);
  const long long r = v / w;
  const int yy = (int)(r % h);
  const long long nz = r / h;
  const int z = (int)(nz % d);
  const long long nn = nz / d;
  const float* xb = x + nn * d * h * w;
  f32x2 acc[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) acc[c] = (f32x2){0.f, 0.f};
#pragma unroll 1
  for (int kd = 0; kd < 3; ++kd) {
    const int zd = z + kd - 1;
#pragma unroll 1
    for (int kh = 0; kh < 3; ++kh) {
      const int zh = yy + kh - 1;
      const bool rowok = (unsigned)zd < (unsigned)d && (unsigned)zh < (unsigned)h;
      float in[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int zw = xx + k - 1;
        in[k] = rowok && (unsigned)zw < (unsigned)w ? xb[((long long)zd * h + zh) * w + zw] : 0.f;
      }
      const int t0 = (kd * 3 + kh) * 3;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const float* wr = wt + (t0 + kw) * 32;
        const f32x2 xv = {in[kw], in[kw]};
#pragma unroll
        for (int c = 0; c < 16; ++c) acc[c] = __builtin_elementwise_fma(xv, (f32x2){wr[2 * c], wr[2 * c + 1]}, acc[c]);
      }
    }
  }
  constexpr int VEC = 16 / sizeof(T);
  if constexpr (sizeof(T) == 2) {
    // through the wave's LDS block: lane l's 4 chunks go to row l (chunk slot XOR (l >> 2) & 3: conflict-free), then
    // lane l reads linear chunks l + 64k, so each store instruction writes 1 KB of consecutive voxels
    char* wb = tr[threadIdx.x >> 6];
    const int l = threadIdx.x & 63;
#pragma unroll
    for (int c4 = 0; c4 < 4; ++c4) {
      float o[VEC];
#pragma unroll
      for (int e = 0; e < VEC; ++e) o[e] = acc[(8 * c4 + e) >> 1][(8 * c4 + e) & 1];
      u32x4 pk;
      store16<T>(reinterpret_cast<T*>(&pk), o);
      *reinterpret_cast<u32x4*>(wb + l * 64 + 16 * (c4 ^ ((l >> 2) & 3))) = pk;
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int p = l + 64 * k, vx = p >> 2, c4 = p & 3;
      const u32x4 pk = *reinterpret_cast<const u32x4*>(wb + vx * 64 + 16 * (c4 ^ ((vx >> 2) & 3)));
      if (v0 + vx < nvox) *reinterpret_cast<u32x4*>(y + (v0 + vx) * 32 + 8 * c4) = pk;
    }
    if constexpr (STATS) {
      float sv[32];
      const bool ok = vr < nvox;
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const float a = ok ? to_f(from_f<bf16>(acc[g][0])) : 0.f, b = ok ? to_f(from_f<bf16>(acc[g][1])) : 0.f;
        sv[2 * g] = a + b;
        sv[2 * g + 1] = a * a + b * b;
      }
      const float t = wave_sum_transposed<32>(sv, l);
      if ((l & 1) == 0) red[threadIdx.x >> 6][l >> 1] = t;
      __syncthreads();
      if (threadIdx.x < 32) {
        float r = 0.f;
#pragma unroll
        for (int wv = 0; wv < ST / 64; ++wv) r += red[wv][threadIdx.x];
        spart[(long long)blockIdx.x * 32 + threadIdx.x] = r;
      }
    }
  } else {
    T* yr = y + v * 32;
#pragma unroll
    for (int c = 0; c < 32; c += VEC) {
      float o[VEC];
#pragma unroll
      for (int e = 0; e < VEC; ++e) o[e] = acc[(c + e) >> 1][(c + e) & 1];
      store16<T>(yr + c, o);
    }
  }
}

// Round 6: conv1 (cin 1 -> 32, stride 1, bf16 output) on the matrix cores. K = the 27 taps (padded to 32): one
// v_mfma_f32_16x16x32_bf16 per (16 voxels, 16 output channels), A = the standardised weights [co][tap], B = the taps of
// 16 voxels. The operands are bf16 — what the reference's autocast conv1 multiplies (the input volume and the
// weight cast to bf16; unet3D.py:1632 under torch.autocast) — so the products are exact and only the fp32 summation
// order differs from an fp64 conv on the same operands. The VALU form (stem1_fwd_kernel) spends 432 packed fp32 FMAs
// per voxel on fp32 operands (57 us at 2 x 96^3, VALU-bound); here a lane loads its voxel's 27 taps, writes them as one
// 64-B bf16 row of the wave's LDS block, and the wave runs 8 MFMAs per 64 voxels. The accumulators (lane: 4
// channels of one voxel) go back through the same LDS block so every store instruction writes 1 KB of consecutive
// voxels; STATS: the GroupNorm(16) partial sums of the stored bf16 values as stem1_fwd_kernel<.., true> (same spart
// layout, another fp32 order).
template <bool STATS>
__global__ __launch_bounds__(ST) void stem1_mfma_kernel(const float* __restrict__ x, const float* __restrict__ wt,
                                                        bf16* __restrict__ y, int d, int h, int w, long long nvox,
                                                        float* __restrict__ spart = nullptr) {
  typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
  __shared__ __attribute__((aligned(16))) char tr[ST / 64][64 * 64];  // per wave: 64 rows x 64 B
  __shared__ float red[STATS ? ST / 64 : 1][32];
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6, r16 = l & 15, q = l >> 4;
  const long long v0 = (long long)blockIdx.x * ST + wv * 64;  // the wave's first voxel
  const long long vr = v0 + l;
  const long long v = vr < nvox ? vr : nvox - 1;
  const int xx = (int)(v % w);
  const long long rr = v / w;
  const int yy = (int)(rr % h);
  const long long nz = rr / h;
  const int z = (int)(nz % d);
  const long long nn = nz / d;
  const float* xb = x + nn * d * h * w;
  char* const wb = tr[wv];
  auto swz = [](int row, int c) { return 16 * (c ^ ((row >> 2) & 3)); };
  {  // this lane's 27 taps (t = (kd * 3 + kh) * 3 + kw) as bf16, taps 27..31 zero, into row l
    float tv[32];
#pragma unroll
    for (int kd = 0; kd < 3; ++kd)
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const int zd = z + kd - 1, zh = yy + kh - 1, zw = xx + kw - 1;
          const bool ok = (unsigned)zd < (unsigned)d && (unsigned)zh < (unsigned)h && (unsigned)zw < (unsigned)w;
          tv[(kd * 3 + kh) * 3 + kw] = ok ? xb[((long long)zd * h + zh) * w + zw] : 0.f;
        }
#pragma unroll
    for (int t = 27; t < 32; ++t) tv[t] = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      u32x4 pk;
#pragma unroll
      for (int k = 0; k < 4; ++k) pk[k] = pack_bf16x2(tv[8 * c + 2 * k], tv[8 * c + 2 * k + 1]);
      *reinterpret_cast<u32x4*>(wb + l * 64 + swz(l, c)) = pk;
    }
  }
  // A fragments: lane (r16, q) holds W[co = 16 cb + r16][taps 8q .. 8q + 7] (bf16-valued fp32 table: exact)
  bf16x8_t af[2];
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
    u32x4 pk;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int t0 = 8 * q + 2 * k, t1 = t0 + 1;
      pk[k] = pack_bf16x2(t0 < 27 ? wt[t0 * 32 + 16 * cb + r16] : 0.f, t1 < 27 ? wt[t1 * 32 + 16 * cb + r16] : 0.f);
    }
    af[cb] = __builtin_bit_cast(bf16x8_t, pk);
  }
  __builtin_amdgcn_wave_barrier();
  f32x4 acc[4][2];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int row = 16 * g + r16;
    const bf16x8_t bf = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u32x4*>(wb + row * 64 + swz(row, q)));
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
      acc[g][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[cb], bf, (f32x4){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
  }
  __builtin_amdgcn_wave_barrier();
  // D[co = 16 cb + 4q + i][voxel 16 g + r16] -> row (16 g + r16), channels 16 cb + 4 q .. + 3 (8 B)
  float gs[2][2], gq[2][2];  // STATS: [cb][group 8 cb + 2 q + j] (sum, squares) of the stored values
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int j = 0; j < 2; ++j) gs[cb][j] = gq[cb][j] = 0.f;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int row = 16 * g + r16;
    const bool ok = v0 + row < nvox;
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      const uint32_t lo = pack_bf16x2(acc[g][cb][0], acc[g][cb][1]), hi = pack_bf16x2(acc[g][cb][2], acc[g][cb][3]);
      const int cbyte = 32 * cb + 8 * q;  // byte offset of channel 16 cb + 4 q in the 64-B row
      *reinterpret_cast<uint2*>(wb + row * 64 + swz(row, cbyte >> 4) + (cbyte & 15)) = uint2{lo, hi};
      if constexpr (STATS) {
        const float a0 = __uint_as_float(lo << 16), a1 = __uint_as_float(lo & 0xffff0000u);
        const float a2 = __uint_as_float(hi << 16), a3 = __uint_as_float(hi & 0xffff0000u);
        gs[cb][0] += ok ? a0 + a1 : 0.f;
        gq[cb][0] += ok ? a0 * a0 + a1 * a1 : 0.f;
        gs[cb][1] += ok ? a2 + a3 : 0.f;
        gq[cb][1] += ok ? a2 * a2 + a3 * a3 : 0.f;
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int k = 0; k < 4; ++k) {  // lane-linear 16-B chunks: each store instruction writes 1 KB of consecutive voxels
    const int p = l + 64 * k, vx = p >> 2, c4 = p & 3;
    const u32x4 pk = *reinterpret_cast<const u32x4*>(wb + vx * 64 + swz(vx, c4));
    if (v0 + vx < nvox) *reinterpret_cast<u32x4*>(y + (v0 + vx) * 32 + 8 * c4) = pk;
  }
  if constexpr (STATS) {
    // over the 16 lanes of each q (xor over r16), then the block's waves in order; red[wave][2 * group + k]
#pragma unroll
    for (int o = 1; o < 16; o <<= 1)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          gs[cb][j] += __shfl_xor(gs[cb][j], o);
          gq[cb][j] += __shfl_xor(gq[cb][j], o);
        }
    if (r16 == 0) {
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int grp = 8 * cb + 2 * q + j;
          red[wv][2 * grp] = gs[cb][j];
          red[wv][2 * grp + 1] = gq[cb][j];
        }
    }
    __syncthreads();
    if (threadIdx.x < 32) {
      float t = 0.f;
#pragma unroll
      for (int w_ = 0; w_ < ST / 64; ++w_) t += red[w_][threadIdx.x];
      spart[(long long)blockIdx.x * 32 + threadIdx.x] = t;
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
// A workgroup walks SM_BD x 8 x 32-voxel bricks of its split; per brick the dy brick (SM_BD x 16 KB, read transposed
// with ds_read_b64_tr_b16) and the fp32 input halo (4 x 10 x 34) sit in LDS. A k-step = 16 consecutive w
// voxels of one row, so the B fragment of tap t is 8 consecutive halo values of the shifted row. The 8
// per-wave tiles are summed in fixed order at the end; the slab rows ci > 0 are written as zeros.
#ifndef U3D_SM_BD
#define U3D_SM_BD 4  // round 6: 4-plane bricks (64 KB of dy per brick in flight; 2 planes: 46.6 us at 2 x 96^3)
#endif
constexpr int SM_BD = U3D_SM_BD, SM_BH = 8, SM_BW = 32, SM_NV = SM_BD * SM_BH * SM_BW;
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
#ifndef U3D_ABL_STEMW
#define U3D_ABL_STEMW 0  // timing-only ablations: 1 = one MFMA step per brick, 2 = only the ci = 0 slab column stored
#endif
#pragma unroll
    for (int j = 0; j < ((U3D_ABL_STEMW & 1) ? 1 : SM_NV / 16 / 8); ++j) {
      const int ks = wave + 8 * j;                 // 16 voxels: row (vd, vh), w = 16 * (ks & 1) ...
      const int k0 = (ks * 16 + 8 * hq + q) * ROWB + colb;
      const sm_bf16x8 a = __builtin_bit_cast(sm_bf16x8, __builtin_shufflevector(sm_tr_read(dyt, k0),
                                                                                 sm_tr_read(dyt, k0 + 4 * ROWB),
                                                                                 0, 1, 2, 3, 4, 5, 6, 7));
      const int v0 = ks * 16 + 8 * hq;             // first of this lane's 8 voxels
      const int vw = v0 % SM_BW, vh = (v0 / SM_BW) % SM_BH, vd = v0 / (SM_BW * SM_BH);
      const float* src = hal + (vd * SM_HH + vh) * SM_HW + vw + toff;  // in range for every lane (ttap clamped)
      // round 6: the 8 halo reads issued unconditionally and converted in pairs (v_cvt_pk_bf16_f32, the rounding of
      // from_f<bf16>); the padded taps 27-31 zeroed by a select. A per-element branch had made each read wait alone.
      typedef float f32x8 __attribute__((ext_vector_type(8)));
      typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
      f32x8 fv;
#pragma unroll
      for (int e = 0; e < 8; ++e) fv[e] = src[e];
      u32x4v bw = __builtin_bit_cast(u32x4v, __builtin_convertvector(fv, sm_bf16x8));
      const unsigned keep = tap < 27 ? 0xFFFFFFFFu : 0u;
#pragma unroll
      for (int e = 0; e < 4; ++e) bw[e] &= keep;
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, __builtin_bit_cast(sm_bf16x8, bw), acc, 0, 0, 0);
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
    if (!(U3D_ABL_STEMW & 2) || ci == 0) pp[e] = s;
  }
}
}  // namespace u3d

using namespace u3d;

static int sdim(int d, int s) { return (d - 1) / s + 1; }  // k3 pad1: (d + 2 - 3)/s + 1

static bool stem1_on() { return opt(OPT_STEM1) != 0; }  // 0: the generic one-voxel kernel

extern "C" long long u3d_stem_fwd_ws_bytes(void) { return 27 * 32 * 4; }

extern "C" long long u3d_stem1_stats_ws_floats(int n, int d, int h, int w) {
  const long long v = (long long)d * h * w;
  return v % ST == 0 ? (long long)n * (v / ST) * 32 : 0;  // 0: not supported (blocks would straddle samples)
}

extern "C" int u3d_stem1_fwd_stats(const float* x, int n, int d, int h, int w, const void* wpk, void* y, void* ws,
                                   float* spart, float* stats, u3d_stream_t stream) {
  U3D_REQUIRE(x && wpk && y && ws && spart && stats && n >= 1 && d >= 1 && h >= 1 && w >= 1, "stem1_fwd_stats: bad args");
  const long long v = (long long)d * h * w;
  U3D_REQUIRE(v % ST == 0, "stem1_fwd_stats: d*h*w = %lld not a multiple of %d", v, ST);
  hipStream_t s = (hipStream_t)stream;
  float* wt = static_cast<float*>(ws);
  const long long nvox = (long long)n * v;
  hipLaunchKernelGGL(stem1_wtab_kernel<bf16>, dim3(1), dim3(1024), 0, s, (const bf16*)wpk, 32, wt);
  if (opt(OPT_STEM_MFMA) != 0)
    hipLaunchKernelGGL(stem1_mfma_kernel<true>, dim3((unsigned)(nvox / ST)), dim3(ST), 0, s, x, wt, (bf16*)y, d, h, w,
                       nvox, spart);
  else
    hipLaunchKernelGGL((stem1_fwd_kernel<bf16, true>), dim3((unsigned)(nvox / ST)), dim3(ST), 0, s, x, wt, (bf16*)y, d,
                       h, w, nvox, spart);
  if (check_launch("stem1_fwd_kernel<stats>")) return U3D_EHIP;
  return launch_gn16_finalize(spart, n, (int)(v / ST), 2.0 * (double)v, stats, s);
}

extern "C" int u3d_stem_fwd(int dtype, const float* x, int n, int cin, int d, int h, int w, const void* wpk, int cout,
                            int stride, void* y, void* ws, u3d_stream_t stream) {
  U3D_REQUIRE(dtype == U3D_F32 || dtype == U3D_BF16, "stem_fwd: bad dtype");
  U3D_REQUIRE(x && wpk && y && cin >= 1 && cin <= 4 && cout >= 1 && (stride == 1 || stride == 2), "stem_fwd: bad args");
  hipStream_t s = (hipStream_t)stream;
  const int od = sdim(d, stride), oh = sdim(h, stride), ow = sdim(w, stride);
  const long long total = (long long)n * od * oh * ow;
  if (cin == 1 && stride == 1 && cout == 32 && stem1_on()) {
    U3D_REQUIRE(ws, "stem_fwd: the conv1 kernel needs a workspace of u3d_stem_fwd_ws_bytes()");
    const long long rows = (long long)n * d * h;
    float* wt = static_cast<float*>(ws);
    const long long nvox = rows * w;
    const dim3 g1((unsigned)((nvox + ST - 1) / ST));
    if (dtype == U3D_BF16) {
      hipLaunchKernelGGL(stem1_wtab_kernel<bf16>, dim3(1), dim3(1024), 0, s, (const bf16*)wpk, round_up(cin, 32), wt);
      if (opt(OPT_STEM_MFMA) != 0)
        hipLaunchKernelGGL(stem1_mfma_kernel<false>, g1, dim3(ST), 0, s, x, wt, (bf16*)y, d, h, w, nvox, nullptr);
      else
        hipLaunchKernelGGL(stem1_fwd_kernel<bf16>, g1, dim3(ST), 0, s, x, wt, (bf16*)y, d, h, w, nvox);
    } else {
      hipLaunchKernelGGL(stem1_wtab_kernel<float>, dim3(1), dim3(1024), 0, s, (const float*)wpk, round_up(cin, 32), wt);
      hipLaunchKernelGGL(stem1_fwd_kernel<float>, g1, dim3(ST), 0, s, x, wt, (float*)y, d, h, w, nvox);
    }
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
