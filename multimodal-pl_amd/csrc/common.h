// Shared device helpers for libu3d (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <algorithm>
#include <string>
#include <type_traits>

#include "../../include/u3d.h"

namespace u3d {

// ------------------------------------------------------------------------------------------ errors
void set_error(const std::string& msg);
int fail(int code, const char* fmt, ...);
int check_launch(const char* what);

// Host-side tuning options. The defaults ARE the product path (each choice measured); the values are
// read once from the environment (U3D_<NAME>, for A/B scripts) at the first query and may be changed in-process with
// u3d_set_option (tests comparing two routings). Nothing here changes results except through the routing it selects.
enum Opt : int {
  OPT_IGEMM_BN,       // implicit-GEMM N tile override (0 = auto)
  OPT_IGEMM_NS,       // implicit-GEMM split-K override (0 = auto)
  OPT_IGEMM_TARGET,   // implicit-GEMM workgroups aimed at
  OPT_IGEMM_AUTO,     // narrow N tiles before split-K where tiles cannot fill the CUs
  OPT_CONVG_CO32,     // -1 auto, 0 / 1 force 64- / 32-channel co tiles of the generic brick conv
  OPT_CONVG_PERSIST,  // persistent generic brick conv (0: one-shot kernel)
  OPT_CONVG_BW8,      // -1 auto, 0 / 1 force 16- / 8-wide persistent bricks
  OPT_RING_KR,        // -1 default, 0: no weight steps in registers in the ring conv
  OPT_RING_WGS,       // ring conv persistent grid target
  OPT_RING_SC,        // work-stealing ring: output planes per sub-chunk (0 = default)
  OPT_SMALL_WGS,      // small-volume conv workgroups aimed at
  OPT_GN_MAXBLK,      // GroupNorm reduction blocks over all samples
  OPT_HEAD_TR,        // transposed classifier head (0: untransposed store path)
  OPT_STEM1,          // conv1 (1 -> 32) one-voxel-per-lane kernel, packed FMAs, scalar weight table (0: generic kernel)
  OPT_UP_BWD_BLK,     // -1 auto, 0 / 1 force the one-row / 2x2-row trilinear backward
  OPT_WGRAD_BD,       // stride-1 brick weight-gradient brick depth (2 or 3)
  OPT_WB_WGS,         // brick weight-gradient workgroups aimed at
  OPT_WR_TILE16,      // 1: 16 x 16 weight-gradient ring tiles everywhere
  OPT_WR_WGS,         // weight-gradient ring workgroups aimed at
  OPT_WB_S2CO64,      // stride-2 brick weight gradient: two co tiles per workgroup (0: one)
  OPT_IGEMM_BM,       // bf16 implicit GEMM M tile: 0 auto (256 for large unsplit BN 64 launches), 128 / 256 force
  OPT_WSTD_ROW,       // weight-standardisation backward: one row per block from registers (0: chunked LDS kernel)
  OPT_UP_QUAD,        // bf16 trilinear x2 upsample: 2 x 2 outputs per thread from 18 loads (0: one output, 8 loads)
  OPT_LOSS_PAIR,      // loss forward, 16 classes softmax + BCE: each voxel's classes over a lane pair (0: one lane)
  OPT_HEAD_NB,        // classifier head / head backward blocks (at most)
  OPT_HEAD_GN_NB,     // head backward with the prologue GN's partials: blocks over all samples (at most)
  OPT_STEM_MFMA,      // bf16 conv1 (1 -> 32) on the matrix cores, bf16 operands (0: the fp32 packed-FMA kernel)
  OPT_WB_S2BD,        // stride-2 brick weight-gradient brick depth in output planes (2 or 3)
  OPT_COUNT
};
int opt(Opt o);

#define U3D_REQUIRE(cond, ...)                                  \
  do {                                                          \
    if (!(cond)) return ::u3d::fail(U3D_EINVAL, __VA_ARGS__);   \
  } while (0)
#define U3D_HIP(expr)                                                               \
  do {                                                                              \
    hipError_t e_ = (expr);                                                         \
    if (e_ != hipSuccess)                                                           \
      return ::u3d::fail(U3D_EHIP, "%s: %s", #expr, hipGetErrorString(e_));         \
  } while (0)

// compile-time loop: f(std::integral_constant<int, I>) for I in [I0, N)
template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// ------------------------------------------------------------------------------------- bf16 / f32
typedef uint16_t bf16;  // bf16 stored as its bit pattern

__device__ __forceinline__ float to_f(float v) { return v; }
__device__ __forceinline__ float to_f(bf16 v) { return __uint_as_float(((uint32_t)v) << 16); }

template <typename T> __device__ __forceinline__ T from_f(float v);
template <> __device__ __forceinline__ float from_f<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16 from_f<bf16>(float v) {
  __hip_bfloat16 h = __float2bfloat16(v);  // RNE, v_cvt_pk_bf16_f32 on gfx950
  return *reinterpret_cast<bf16*>(&h);
}

typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;

typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
typedef __attribute__((ext_vector_type(2))) short s16x2;

// two floats -> packed bf16 pair (lo = a), one v_cvt_pk_bf16_f32 (round to nearest even)
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, bf16x2_t));
}
// max(x, 0) of both bf16 halves (v_pk_max_i16)
__device__ __forceinline__ uint32_t relu_bf16x2(uint32_t u) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s16x2, u), (s16x2){0, 0}));
}

// Sum of 8 per-lane values over the 32 lanes of each wave half, transposed: afterwards lane r (r = lane & 31) holds
// the total of value (r >> 2) & 7 (fixed order, so deterministic; every lane of a group of 4 holds the same bits).
// Butterfly where each step keeps the half of the values whose index bit equals the lane bit: lane bit 4 by
// v_permlane16_swap (no selects), bit 3 by DPP row_ror:8 (= xor 8 within a row), bit 2 by ds_swizzle xor 4, then
// the remaining lanes bits 1, 0 add by DPP quad_perm (xor 2, xor 1). 20 instructions for 8 values (the generic
// __shfl_xor butterfly compiled to ~3x that: bpermute index math and exec-mask selects).
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float half_sum8_transposed(float (&v)[8], int r) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // lane bit 4: rows 0 / 1 (and 2 / 3) exchange values i / i + 4
    const auto sw = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(uint32_t, v[i]),
                                                     __builtin_bit_cast(uint32_t, v[i + 4]), false, false);
    // (hipcc of ROCm 7.2 folds sw[0] + sw[1] into sw[0] + sw[0] — seen in the ISA of a two-line kernel; the empty
    // asm hides the second result from that combine)
    uint32_t hi = sw[1];
    asm volatile("" : "+v"(hi));
    v[i] = __builtin_bit_cast(float, sw[0]) + __builtin_bit_cast(float, hi);
  }
  const bool b3 = (r & 8) != 0, b2 = (r & 4) != 0;
#pragma unroll
  for (int i = 0; i < 2; ++i) {  // lane bit 3
    const float keep = b3 ? v[i + 2] : v[i], send = b3 ? v[i] : v[i + 2];
    v[i] = keep + dpp_mov<0x128>(send);  // row_ror:8
  }
  {  // lane bit 2
    const float keep = b2 ? v[1] : v[0], send = b2 ? v[0] : v[1];
    v[0] = keep + __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, send), 0x101F));
  }
  v[0] += dpp_mov<0x4E>(v[0]);  // quad_perm [2,3,0,1]: xor 2 (a + b and b + a: the same bits)
  v[0] += dpp_mov<0xB1>(v[0]);  // quad_perm [1,0,3,2]: xor 1
  return v[0];
}

// Sum of N (a power of two, <= 32) per-lane values over the 64 lanes of a wave, transposed: afterwards lane l holds
// the wave total of value index (l >> (6 - log2 N)) & (N - 1) (for N = 32: l >> 1); the lanes of a group of 64 / N
// hold the same bits. Each xor step keeps the half of the values whose index bit equals the lane bit, so the work
// halves every step (N - 1 + 6 - log2 N shuffles instead of 6 N). Fixed order: deterministic.
template <int N, int O = 32>
__device__ __forceinline__ void wave_sum_transposed_step(float (&v)[N], int lane) {
  if constexpr (O >= 1) {
    constexpr int M = N >> (5 - (O == 32 ? 5 : O == 16 ? 4 : O == 8 ? 3 : O == 4 ? 2 : O == 2 ? 1 : 0));  // values left
    if constexpr (M > 1) {
      constexpr int H = M / 2;
      const bool b = (lane & O) != 0;
#pragma unroll
      for (int i = 0; i < H; ++i) {
        const float keep = b ? v[i + H] : v[i], send = b ? v[i] : v[i + H];
        v[i] = keep + __shfl_xor(send, O);
      }
    } else {
      v[0] += __shfl_xor(v[0], O);
    }
    wave_sum_transposed_step<N, O / 2>(v, lane);
  }
}
template <int N>
__device__ __forceinline__ float wave_sum_transposed(float (&v)[N], int lane) {
  static_assert(N >= 1 && N <= 32 && (N & (N - 1)) == 0, "N: power of two <= 32");
  wave_sum_transposed_step<N, 32>(v, lane);
  return v[0];
}

// The combine of a launch's last-arriving workgroup over the partial rows the launch's workgroups wrote (sc1 stores):
// out[r * K + k] (fp64, LDS) = sum over w < nw of rows[(r * nw + w) * K + k], for r < nr, k < K (K % 4 == 0).
// L lanes per (row r, column quad), L the largest power of two <= 64 with all items in one pass of NT threads; lane l
// sums w = l, l + L, ... in order with 8 sc1 16-B loads in flight (r05: the first form, one dependent load pair per
// iteration, cost its conv launch 8-11 us), then an xor tree over the L lanes. Fixed order: deterministic.
// Every thread of the workgroup must call it (shuffles); `out` is read after the caller's barrier.
template <int NT>
__device__ __forceinline__ void lastarriver_rowsum(const float* rows, int nr, int nw, int K, double* out) {
  const int nq = K >> 2, items = nr * nq;
  int L = 64;
  while (L > 1 && items * L > NT) L >>= 1;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)rows, 0, 0x7FFFFFFF, 0x00020000);
  const int tid = threadIdx.x, l = tid & (L - 1);
  for (int i0 = 0; i0 < items; i0 += NT / L) {
    const int it = i0 + tid / L;
    double a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    if (it < items) {
      const int r = it / nq, q = it - r * nq;
      const int base = (r * nw * K + 4 * q) * 4;
      for (int w0 = l; w0 < nw; w0 += 8 * L) {
        f32x4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int w = w0 + u * L;
          v[u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                               rs, w < nw ? base + w * K * 4 : (int)0xFFFFFFF0u, 0, 16));
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (w0 + u * L < nw) {
            a0 += v[u][0];
            a1 += v[u][1];
            a2 += v[u][2];
            a3 += v[u][3];
          }
      }
    }
    for (int o = L >> 1; o > 0; o >>= 1) {
      a0 += __shfl_xor(a0, o);
      a1 += __shfl_xor(a1, o);
      a2 += __shfl_xor(a2, o);
      a3 += __shfl_xor(a3, o);
    }
    if (it < items && l == 0) {
      const int r = it / nq, q = it - r * nq;
      double* o4 = out + r * K + 4 * q;
      o4[0] = a0;
      o4[1] = a1;
      o4[2] = a2;
      o4[3] = a3;
    }
  }
}

// GroupNorm(16) statistics from per-workgroup partials [sample][wps][16][2] (fp32 sums of values and squares): one
// wave per (sample, group), fixed-order fp64 combine (conv_ring.hip). m = values per group and sample.
int launch_gn16_finalize(const float* spart, int n, int wps, double m, float* stats, hipStream_t s);

// 16-byte vector of T: 8 bf16 or 4 f32.
template <typename T> struct Vec16 { static constexpr int N = 16 / sizeof(T); };

template <typename T>
__device__ __forceinline__ void load16(const T* p, float (&v)[Vec16<T>::N]) {
  u32x4 r = *reinterpret_cast<const u32x4*>(p);
  if constexpr (sizeof(T) == 4) {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = __uint_as_float(r[i]);
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(r[i] << 16);
      v[2 * i + 1] = __uint_as_float(r[i] & 0xffff0000u);
    }
  }
}

template <typename T>
__device__ __forceinline__ void store16(T* p, const float (&v)[Vec16<T>::N]) {
  u32x4 r;
  if constexpr (sizeof(T) == 4) {
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = __float_as_uint(v[i]);
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = pack_bf16x2(v[2 * i], v[2 * i + 1]);
  }
  *reinterpret_cast<u32x4*>(p) = r;
}

// N-wide load/store: 16-B vector when N fills 16 bytes, scalar otherwise (odd channel counts).
template <typename T, int N>
__device__ __forceinline__ void loadv(const T* p, float (&v)[N]) {
  if constexpr (N * sizeof(T) == 16) {
    load16<T>(p, v);
  } else {
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = to_f(p[i]);
  }
}
template <typename T, int N>
__device__ __forceinline__ void storev(T* p, const float (&v)[N]) {
  if constexpr (N * sizeof(T) == 16) {
    store16<T>(p, v);
  } else {
#pragma unroll
    for (int i = 0; i < N; ++i) p[i] = from_f<T>(v[i]);
  }
}

// GroupNorm apply + ReLU on 8 packed bf16 channels: relu(x * sc + sh), scalar fp32 fma per channel, one
// v_cvt_pk_bf16_f32 (RNE) per pair and the ReLU on the packed bf16 pair as a signed 16-bit max (v_pk_max_i16:
// a negative bf16 has its sign bit set; rounding preserves the sign, so relu(round(x)) == round(relu(x))).
// Scalar, not v_pk_fma_f32: these run between MFMAs, where a packed fp32 op costs ~22 cycles more than the two
// scalar fmas it replaces (MI355X_MICROARCH.md, filler prices); the results are bitwise the same (one fma each).
__device__ __forceinline__ u32x4 gn_relu8(u32x4 v, const f32x2 (&sc)[4], const f32x2 (&sh)[4]) {
  u32x4 o;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float f0 = fmaf(__uint_as_float(v[e] << 16), sc[e][0], sh[e][0]);
    const float f1 = fmaf(__uint_as_float(v[e] & 0xffff0000u), sc[e][1], sh[e][1]);
    o[e] = relu_bf16x2(pack_bf16x2(f0, f1));
  }
  return o;
}

// per-thread scale/shift of channels c0 .. c0+7 (clamped) of sample n for gn_relu8
// (buffer loads: 32-bit offsets from scalar bases, so a caller that refreshes the table inside a loop holds no
// per-lane 64-bit addresses across it)
__device__ __forceinline__ void gn_coef8(const float* __restrict__ st, const float* __restrict__ gamma,
                                         const float* __restrict__ beta, int groups, int cin, int n, int c0,
                                         f32x2 (&sc)[4], f32x2 (&sh)[4]) {
  const int cpg = cin / groups;
  const auto srs = __builtin_amdgcn_make_buffer_rsrc((void*)st, 0, 0x7FFFFFFF, 0x00020000);
  const auto grs = __builtin_amdgcn_make_buffer_rsrc((void*)gamma, 0, 0x7FFFFFFF, 0x00020000);
  const auto brs = __builtin_amdgcn_make_buffer_rsrc((void*)beta, 0, 0x7FFFFFFF, 0x00020000);
  asm volatile("" : "+v"(c0));  // the channel offsets are formed here, not hoisted into the caller's loop
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = min(c0 + e, cin - 1), gg = c / cpg;
    const int so = (n * groups + gg) * 8;
    const float mean = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(srs, so, 0, 0));
    const float rstd = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(srs, so + 4, 0, 0));
    const float s = rstd * __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(grs, c * 4, 0, 0));
    sc[e >> 1][e & 1] = s;
    sh[e >> 1][e & 1] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(brs, c * 4, 0, 0)) - mean * s;
  }
}

// -------------------------------------------------------------------------------- wave reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// (channel tile x, channel tile y, work split) of a 3-D grid whose x / y enumerate channel tiles and z the splits of
// the work. Workgroups are dispatched round-robin over the 8 XCDs in linear order (x fastest); this remaps so that
// XCD k runs a contiguous range of (split, tile) indices, tile fastest: all channel tiles of a few consecutive splits
// run on one XCD at the same time and read their shared operand rows (the same input rows for every output-channel
// tile, the same dy rows for every input-channel tile) through that XCD's L2 instead of once per XCD from HBM.
struct TileSplit {
  int tx, ty, split;
};
__device__ __forceinline__ TileSplit xcd_tile_split() {
  const int nt = gridDim.x * gridDim.y, total = nt * gridDim.z;
  const int L = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  const int q = total >> 3, rr = total & 7, xcd = L & 7, loc = L >> 3;
  const int N = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + loc;
  const int tile = N % nt;
  return TileSplit{tile % (int)gridDim.x, tile / (int)gridDim.x, N / nt};
}

__host__ __device__ inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }
__host__ __device__ inline int round_up(int a, int b) { return (a + b - 1) / b * b; }

}  // namespace u3d
