// Batched weight preparation: the weight standardisation of EVERY conv of the trunk (reference
// Conv3d.forward, unet3D.py:21-26) and its backward in five launches per step instead of three per conv.
// Per-conv descriptors travel in the kernel arguments (no host->device copy, graph-capturable).
//   forward : (1) row statistics, one block per output channel (coalesced row reads, fp64 sums);
//             (2) packing, one block per (conv, 16 co x 32 ci tile): the tile's [co][ci][t] rows are staged
//                 through LDS once (coalesced), then written as the forward pack [t][co][ci] and the
//                 data-grad pack [t][ci][co] (zero padding included).
//   backward: (3) split slabs summed in fixed order (fp64, up to 32 slab groups per block) into slab 0;
//             (4) per-row sums of g and g*W_hat (one block per output channel);
//             (5) dW = (g - mean(g) - W_hat * sum(g W_hat)/(K-1)) / std per tile, g and W staged through LDS
//                 so that dW is written in parameter order [co][ci][t] with full-row stores.
#include "common.h"

namespace u3d {

constexpr int WB_T = 256;   // threads of the row / sum kernels
constexpr int WB_TT = 512;  // threads of the tile kernels
constexpr int WB_CO = 16;   // co rows per pack/apply tile
constexpr int WB_CI = 32;   // ci columns per pack/apply tile

struct WRow {  // kernels (1) and (4): one block per output channel
  const float* w;
  const float* g;
  float* st;
  float* rowbuf;
  int cout, cin, k3, b0;
};
struct WPack {  // kernels (2) and (5): one block per 16 x 32 tile
  const float* w;
  const float* st;  // nullptr: no standardisation
  void* pf;         // (2) forward pack
  void* pd;         // (2) data-grad pack (nullable)
  const float* g;   // (5) summed slab
  const float* rowbuf;
  float* dw;
  int cout, cin, k3, acc, b0;
};
struct WSum {
  float* p;
  int ns, per4, sg, b0;  // sg = slab groups per block (power of 2), 256/sg float4 columns per block
};
template <typename D>
struct WBatch {
  int count;
  D d[U3D_WSTD_BATCH_MAX];
};

// the descriptor whose block range holds blk (b0 ascending): binary search over the kernel-argument batch (the linear
// walk was up to 48 dependent scalar loads at the start of every block)
template <typename B>
__device__ __forceinline__ int find_desc(const B& bt, int blk) {
  int lo = 0, hi = bt.count - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (bt.d[mid].b0 <= blk) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

template <typename T>
__device__ __forceinline__ T block_sum(T v, T* red) {  // WB_T threads, fixed order
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  T t = 0;
#pragma unroll
  for (int i = 0; i < WB_T / 64; ++i) t += red[i];
  __syncthreads();
  return t;
}

// (1) mean / unbiased std of one row, as Conv3d.forward computes them. Rows up to WS_RV * 4 * WB_T floats (every trunk
// conv: cin * 27 <= 6912) are read once, as 16-B vectors held in registers for both sums (K = cin * k3 is a multiple
// of 8 and rows start 16-B aligned); longer or unaligned rows (a weight view at an odd offset) take the two-pass scalar
// walk.
constexpr int WS_RV = 7;
__global__ __launch_bounds__(WB_T) void wstd_stats_kernel(WBatch<WRow> bt) {
  __shared__ double red[WB_T / 64];
  const WRow& D = bt.d[find_desc(bt, blockIdx.x)];
  const int co = blockIdx.x - D.b0;
  const int K = D.cin * D.k3;
  const float* wr = D.w + (long long)co * K;
  if (K <= WS_RV * 4 * WB_T && K % 4 == 0 && (((uintptr_t)D.w) & 15) == 0) {
    f32x4 r[WS_RV];
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < WS_RV; ++j) {
      const int i = (threadIdx.x + j * WB_T) * 4;
      r[j] = i < K ? *reinterpret_cast<const f32x4*>(wr + i) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int j = 0; j < WS_RV; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) s += r[j][e];
    const float mean = (float)(block_sum(s, red) / K);
    double v = 0.0;
#pragma unroll
    for (int j = 0; j < WS_RV; ++j)
      if ((threadIdx.x + j * WB_T) * 4 < K)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float c = r[j][e] - mean;
          v += (double)c * c;
        }
    const float var = (float)(block_sum(v, red) / (K > 1 ? K - 1 : 1));  // torch.var: unbiased
    if (threadIdx.x == 0) {
      D.st[co * 2] = mean;
      D.st[co * 2 + 1] = sqrtf(var + 1e-12f);
    }
    return;
  }
  double s = 0.0;
  for (int i = threadIdx.x; i < K; i += WB_T) s += wr[i];
  const float mean = (float)(block_sum(s, red) / K);
  double v = 0.0;
  for (int i = threadIdx.x; i < K; i += WB_T) {
    const float c = wr[i] - mean;
    v += (double)c * c;
  }
  const float var = (float)(block_sum(v, red) / (K > 1 ? K - 1 : 1));  // torch.var: unbiased
  if (threadIdx.x == 0) {
    D.st[co * 2] = mean;
    D.st[co * 2 + 1] = sqrtf(var + 1e-12f);
  }
}

// stage rows co0..co0+15, columns [ci0*K3, (ci0+32)*K3) of a [cout][cin*K3] fp32 matrix into LDS (zero padded)
// (16-B loads, all issued before the LDS stores, when the rows are 16-B aligned: K3 = 27 with cin % 4 == 0, or
// K3 = 1 with cin % 4 == 0 — every trunk conv; scalar otherwise, e.g. the 1-channel stem)
template <int K3>
__device__ __forceinline__ void stage_rows(float* s, const float* __restrict__ src, int cout, int cin, int co0,
                                           int ci0) {
  constexpr int SEG = WB_CI * K3, RS = SEG + 1, NQ = WB_CO * SEG / 4, QL = (NQ + WB_TT - 1) / WB_TT;
  const int K = cin * K3, valid = min(WB_CI, cin - ci0) * K3;
  if (cin % 4 == 0 && (((uintptr_t)src) & 15) == 0) {
    f32x4 v[QL];
#pragma unroll
    for (int i = 0; i < QL; ++i) {
      const int q = threadIdx.x + i * WB_TT, r = q / (SEG / 4), c = (q - r * (SEG / 4)) * 4, co = co0 + r;
      v[i] = (q < NQ && co < cout && c < valid) ? *reinterpret_cast<const f32x4*>(src + (long long)co * K + ci0 * K3 + c)
                                                 : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < QL; ++i) {
      const int q = threadIdx.x + i * WB_TT, r = q / (SEG / 4), c = (q - r * (SEG / 4)) * 4;
      if (q < NQ)
#pragma unroll
        for (int e = 0; e < 4; ++e) s[r * RS + c + e] = v[i][e];
    }
    return;
  }
  for (int e = threadIdx.x; e < WB_CO * SEG; e += WB_TT) {
    const int r = e / SEG, c = e - r * SEG, co = co0 + r;
    s[r * RS + c] = (co < cout && c < valid) ? src[(long long)co * K + ci0 * K3 + c] : 0.f;
  }
}

template <typename T, int K3>
__device__ __forceinline__ void pack_tile(const WPack& D, float* ws, const float* mu, const float* sg, int co0,
                                          int ci0) {
  constexpr int RS = WB_CI * K3 + 1;
  const int cout_p = round_up(D.cout, 32), cin_p = round_up(D.cin, 32);
  stage_rows<K3>(ws, D.w, D.cout, D.cin, co0, ci0);
  __syncthreads();
  T* pf = reinterpret_cast<T*>(D.pf);
  T* pd = reinterpret_cast<T*>(D.pd);
  // padding (co >= cout or ci >= cin) stays exactly zero: standardise real entries only
  auto val = [&](int r, int c, int t) {
    const float v = ws[r * RS + c * K3 + t];
    return (co0 + r < D.cout && ci0 + c < D.cin) ? (v - mu[r]) / sg[r] : 0.f;
  };
  if constexpr (sizeof(T) == 2) {
    // bf16: 8 consecutive outputs per thread, one 16-B store (v_cvt_pk_bf16_f32 = the RNE of from_f<bf16>)
    for (int e = threadIdx.x; e < K3 * WB_CO * (WB_CI / 8); e += WB_TT) {  // (t, r, c8), c8 fastest
      const int c8 = e % (WB_CI / 8), r = (e / (WB_CI / 8)) % WB_CO, t = e / (WB_CI / 8 * WB_CO);
      u32x4 o;
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = pack_bf16x2(val(r, c8 * 8 + 2 * q, t), val(r, c8 * 8 + 2 * q + 1, t));
      *reinterpret_cast<u32x4*>(pf + ((long long)t * cout_p + co0 + r) * cin_p + ci0 + c8 * 8) = o;
    }
    if (pd) {
      for (int e = threadIdx.x; e < K3 * WB_CI * (WB_CO / 8); e += WB_TT) {  // (t, c, r8), r8 fastest
        const int r8 = e % (WB_CO / 8), c = (e / (WB_CO / 8)) % WB_CI, t = e / (WB_CO / 8 * WB_CI);
        u32x4 o;
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = pack_bf16x2(val(r8 * 8 + 2 * q, c, t), val(r8 * 8 + 2 * q + 1, c, t));
        *reinterpret_cast<u32x4*>(pd + ((long long)t * cin_p + ci0 + c) * cout_p + co0 + r8 * 8) = o;
      }
    }
  } else {
    for (int e = threadIdx.x; e < K3 * WB_CO * WB_CI; e += WB_TT) {  // (t, r, c), c fastest
      const int c = e % WB_CI, r = (e / WB_CI) % WB_CO, t = e / (WB_CI * WB_CO);
      pf[((long long)t * cout_p + co0 + r) * cin_p + ci0 + c] = from_f<T>(val(r, c, t));
    }
    if (pd) {
      for (int e = threadIdx.x; e < K3 * WB_CO * WB_CI; e += WB_TT) {  // (t, c, r), r fastest
        const int r = e % WB_CO, c = (e / WB_CO) % WB_CI, t = e / (WB_CI * WB_CO);
        pd[((long long)t * cin_p + ci0 + c) * cout_p + co0 + r] = from_f<T>(val(r, c, t));
      }
    }
  }
}

// (2) forward pack [t][co][ci] + data-grad pack [t][ci][co] of one 16 x 32 tile
template <typename T>
__global__ __launch_bounds__(WB_TT) void wstd_pack_kernel(WBatch<WPack> bt) {
  __shared__ float ws[WB_CO * (WB_CI * 27 + 1)];
  __shared__ float mu[WB_CO], sg[WB_CO];
  const WPack& D = bt.d[find_desc(bt, blockIdx.x)];
  const int nci = round_up(D.cin, 32) / WB_CI;
  const int tile = blockIdx.x - D.b0, co0 = (tile / nci) * WB_CO, ci0 = (tile % nci) * WB_CI;
  if (threadIdx.x < WB_CO) {
    const int co = co0 + threadIdx.x;
    const bool s = D.st && co < D.cout;
    mu[threadIdx.x] = s ? D.st[co * 2] : 0.f;
    sg[threadIdx.x] = s ? D.st[co * 2 + 1] : 1.f;
  }
  if (D.k3 == 27)
    pack_tile<T, 27>(D, ws, mu, sg, co0, ci0);
  else
    pack_tile<T, 1>(D, ws, mu, sg, co0, ci0);
}

// (3) slab 0 <- sum_s slab s. Thread (group q < sg, column) sums slabs q, q+sg, ... in fp64; the groups are
// then combined in order q = 0..sg-1 (fixed order: deterministic).
__global__ __launch_bounds__(WB_T) void wstd_sum_slabs_kernel(WBatch<WSum> bt) {
  __shared__ double red[WB_T][4];
  const WSum& D = bt.d[find_desc(bt, blockIdx.x)];
  const int nc = WB_T / D.sg;
  const int q = threadIdx.x / nc, col = threadIdx.x - q * nc;
  const long long i = (long long)(blockIdx.x - D.b0) * nc + col;
  const bool in = i < D.per4;
  const f32x4* p = reinterpret_cast<const f32x4*>(D.p);
  double a[4] = {0, 0, 0, 0};
  if (in && q < D.ns) {
    const int step = D.sg, last = q + (D.ns - 1 - q) / step * step;  // this group's last slab
    // rounds of 8 loads in flight, the partial last round with clamped addresses (straight-line loads; a slab
    // count below 8 per group, e.g. the 4-16 slabs of the 12^3 / 6^3 weights, is not a chain of dependent loads);
    // the adds run in slab order, so the sum is that of the serial walk
    for (int s = q; s < D.ns; s += 8 * step) {
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = p[(long long)min(s + u * step, last) * D.per4 + i];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (s + u * step < D.ns)
#pragma unroll
          for (int e = 0; e < 4; ++e) a[e] += v[u][e];
    }
  }
  if (D.sg == 1) {
    if (in) reinterpret_cast<f32x4*>(D.p)[i] = f32x4{(float)a[0], (float)a[1], (float)a[2], (float)a[3]};
    return;
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) red[threadIdx.x][e] = a[e];
  __syncthreads();
  if (q == 0 && in) {
    double t[4] = {0, 0, 0, 0};
    for (int gq = 0; gq < D.sg; ++gq)
#pragma unroll
      for (int e = 0; e < 4; ++e) t[e] += red[gq * nc + col][e];
    reinterpret_cast<f32x4*>(D.p)[i] = f32x4{(float)t[0], (float)t[1], (float)t[2], (float)t[3]};
  }
}

// (4+5) dW of 8 output channels: pass 1 accumulates the row sums of g and g*W_hat over 32-channel chunks
// staged through LDS (w rows [co][ci][t] contiguous, g [t][co][ci] rows contiguous), pass 2 re-stages the
// chunks and writes dW = (g - mean(g) - W_hat * sum(g W_hat)/(K-1)) / std in parameter order (contiguous rows).
// WG_T / WG_R threads per row, fixed-order reductions (deterministic). 4 rows per block: twice the blocks of 8 and
// half the LDS, so more blocks stream per CU (the kernel is latency-bound on its chunk stage / barrier chain).
constexpr int WG_R = 4, WG_T = 256, WG_TPR = WG_T / WG_R;

template <int K3>
__device__ __forceinline__ void wgrad_stage(const WPack& D, float* ws, float* gs, int co0, int ci0) {
  // 16-B loads, all issued before the LDS stores (the stage is latency-bound otherwise)
  constexpr int SEG = WB_CI * K3, WQ = WG_R * SEG / 4, GQ = K3 * WG_R * WB_CI / 4;
  constexpr int WL = (WQ + WG_T - 1) / WG_T, GL = (GQ + WG_T - 1) / WG_T;
  const int cout_p = round_up(D.cout, 32), cin_p = round_up(D.cin, 32);
  const int K = D.cin * K3, valid = min(WB_CI, D.cin - ci0) * K3;
  f32x4 wv[WL], gv[GL];
#pragma unroll
  for (int i = 0; i < WL; ++i) {  // w rows [co][ci0*K3 ..): valid is a multiple of 4 (cin % 8 == 0 or K3 == 27 ... )
    const int q = threadIdx.x + i * WG_T, r = q / (SEG / 4), c = (q - r * (SEG / 4)) * 4, co = co0 + r;
    wv[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (q < WQ && D.st && co < D.cout) {
      const float* src = D.w + (long long)co * K + ci0 * K3 + c;
      if (c + 4 <= valid && (((uintptr_t)src) & 15) == 0) {
        wv[i] = *reinterpret_cast<const f32x4*>(src);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) wv[i][e] = c + e < valid ? src[e] : 0.f;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < GL; ++i) {  // g rows [t][co][ci0 .. ci0+32): 8 x 16 B each
    const int q = threadIdx.x + i * WG_T, c = (q % (WB_CI / 4)) * 4, r = (q / (WB_CI / 4)) % WG_R,
              t = q / (WB_CI / 4 * WG_R);
    gv[i] = (q < GQ && co0 + r < D.cout)
                ? *reinterpret_cast<const f32x4*>(D.g + ((long long)t * cout_p + co0 + r) * cin_p + ci0 + c)
                : f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int i = 0; i < WL; ++i) {
    const int q = threadIdx.x + i * WG_T, r = q / (SEG / 4), c = (q - r * (SEG / 4)) * 4;
    if (q < WQ)
#pragma unroll
      for (int e = 0; e < 4; ++e) ws[r * (SEG + 1) + c + e] = wv[i][e];
  }
#pragma unroll
  for (int i = 0; i < GL; ++i) {
    const int q = threadIdx.x + i * WG_T, c = (q % (WB_CI / 4)) * 4, r = (q / (WB_CI / 4)) % WG_R,
              t = q / (WB_CI / 4 * WG_R);
    if (q < GQ)
#pragma unroll
      for (int e = 0; e < 4; ++e) gs[(t * WG_R + r) * (WB_CI + 1) + c + e] = gv[i][e];
  }
}

template <int K3>
__device__ __forceinline__ void wgrad_rows(const WPack& D, int co0) {
  constexpr int SEG = WB_CI * K3;
  __shared__ float ws[WG_R * (SEG + 1)];
  __shared__ float gs[K3 * WG_R * (WB_CI + 1)];
  __shared__ float f1s[WG_R], f2s[WG_R];
  const int tid = threadIdx.x, r = tid / WG_TPR, l = tid % WG_TPR, co = co0 + r;
  const bool std_ = D.st != nullptr, rok = co < D.cout;
  const float mu = std_ && rok ? D.st[co * 2] : 0.f;
  const float rsg = std_ && rok ? 1.f / D.st[co * 2 + 1] : 1.f;
  const int K = D.cin * K3;
  if (std_) {
    float m1 = 0.f, m2 = 0.f;
    for (int ci0 = 0; ci0 < D.cin; ci0 += WB_CI) {
      __syncthreads();
      wgrad_stage<K3>(D, ws, gs, co0, ci0);
      __syncthreads();
      const int valid = min(WB_CI, D.cin - ci0) * K3;
      for (int e = l; e < valid; e += WG_TPR) {
        const int c = e / K3, t = e - c * K3;
        const float gv = gs[(t * WG_R + r) * (WB_CI + 1) + c];
        m1 += gv;
        m2 = fmaf(gv, (ws[r * (SEG + 1) + e] - mu) * rsg, m2);
      }
    }
    double d1 = m1, d2 = m2;
    for (int o = WG_TPR / 2; o > 0; o >>= 1) {
      d1 += __shfl_xor(d1, o, WG_TPR);
      d2 += __shfl_xor(d2, o, WG_TPR);
    }
    if (l == 0) {
      f1s[r] = (float)(d1 / K);
      f2s[r] = (float)(d2 / (K > 1 ? K - 1 : 1));
    }
  }
  __syncthreads();
  const float f1 = std_ ? f1s[r] : 0.f, f2 = std_ ? f2s[r] : 0.f;
  const bool staged = std_ && D.cin <= WB_CI;  // one chunk: pass 1 left it in LDS
  for (int ci0 = 0; ci0 < D.cin; ci0 += WB_CI) {
    if (!staged) {
      __syncthreads();
      wgrad_stage<K3>(D, ws, gs, co0, ci0);
      __syncthreads();
    }
    if (!rok) continue;
    const int valid = min(WB_CI, D.cin - ci0) * K3;
    float* o = D.dw + (long long)co * K + ci0 * K3;
    for (int e = l; e < valid; e += WG_TPR) {
      const int c = e / K3, t = e - c * K3;
      const float gv = gs[(t * WG_R + r) * (WB_CI + 1) + c];
      const float v = std_ ? (gv - f1 - (ws[r * (SEG + 1) + e] - mu) * rsg * f2) * rsg : gv;
      o[e] = (D.acc ? o[e] : 0.f) + v;
    }
  }
}

__global__ __launch_bounds__(WG_T) void wstd_grad_kernel(WBatch<WPack> bt) {
  const WPack& D = bt.d[find_desc(bt, blockIdx.x)];
  const int co0 = (blockIdx.x - D.b0) * WG_R;
  if (D.k3 == 27)
    wgrad_rows<27>(D, co0);
  else
    wgrad_rows<1>(D, co0);
}

// (4+5), one row per block (round 4): the row's K = cin * k^3 (w, g) pairs are loaded at once — NPT per thread,
// straight into registers, w and dW in parameter order (coalesced), g gathered from its [t][co][ci] layout — then the
// row sums (fp32 per thread in a fixed order, fp64 across the block in a fixed order) and dW from the same registers.
// One load round-trip per row instead of the chunk stage / barrier chain of wstd_grad_kernel, whose 64-block launch
// of a 256x256 layer took 44 us (latency-bound, r04 trace); wstd_grad_kernel stays for rows longer than 56 x 256.
// (round 5) the row of g is read coalesced in its [t][ci] order into LDS and re-read per thread in parameter order
// [ci][t] (the per-element gather read one float per 4 KB+ stride: the kernel ran at ~2.5 TB/s of useful bytes)
template <int NPT>
__global__ __launch_bounds__(WB_T) void wstd_grad_row_kernel(WBatch<WPack> bt) {
  __shared__ double red[WB_T / 64][2];
  __shared__ float fs[2];
  __shared__ float gl[NPT * WB_T];
  // round 6: the descriptor by value (one scalar fetch, not a kernel-argument reload ahead of every load), g's (t, ci)
  // from a fixed ci and a t stride where cin divides the block (every trunk conv: no per-element integer division —
  // ~40 instructions between consecutive loads before), and w's loads issued with g's, ahead of the LDS stores
  const WPack D = bt.d[find_desc(bt, blockIdx.x)];
  const int co = blockIdx.x - D.b0, tid = threadIdx.x;
  const int K3 = D.k3, K = D.cin * K3, cout_p = round_up(D.cout, 32), cin_p = round_up(D.cin, 32);
  const bool std_ = D.st != nullptr;
  const float mu = std_ ? D.st[co * 2] : 0.f;
  const float rsg = std_ ? 1.f / D.st[co * 2 + 1] : 1.f;
  const float* wr = D.w + (long long)co * K;
  float wv[NPT], gv[NPT];
  // buffer loads: an element past the row gets the out-of-range sentinel offset and reads 0 with no branch around the
  // load (plain predicated loads came out as one branch + wait per element)
  const auto wrs = __builtin_amdgcn_make_buffer_rsrc((void*)wr, 0, 0x7FFFFFF0, 0x00020000);
  auto load_w = [&]() {
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      const int e = tid + i * WB_T;
      const unsigned off = e < K && std_ ? (unsigned)e * 4u : 0xFFFFFFF0u;
      wv[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(wrs, off, 0, 0));
    }
  };
  if (WB_T % D.cin == 0) {  // uniform: element j = tid + i * WB_T has ci = tid % cin, t = tid / cin + i * WB_T / cin
    const int ci = tid % D.cin, t0 = tid / D.cin, ts = WB_T / D.cin;
    const auto grs = __builtin_amdgcn_make_buffer_rsrc((void*)D.g, 0, 0x7FFFFFF0, 0x00020000);
    const unsigned g0 = (unsigned)(((t0 * cout_p + co) * cin_p + ci) * 4), gs = (unsigned)(ts * cout_p * cin_p * 4);
    float gt[NPT];
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      const unsigned off = tid + i * WB_T < K ? g0 + (unsigned)i * gs : 0xFFFFFFF0u;
      gt[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(grs, off, 0, 0));
    }
    load_w();
#pragma unroll
    for (int i = 0; i < NPT; ++i)
      if (tid + i * WB_T < K) gl[ci * K3 + t0 + i * ts] = gt[i];
  } else {  // g[t][co][ci], element j = t * cin + ci -> LDS slot ci * K3 + t (parameter order)
    float gt[NPT];
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      const int j = tid + i * WB_T;
      const int t = j / D.cin, ci = j - t * D.cin;
      gt[i] = j < K ? D.g[((long long)t * cout_p + co) * cin_p + ci] : 0.f;
    }
    load_w();
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      const int j = tid + i * WB_T;
      const int t = j / D.cin, ci = j - t * D.cin;
      if (j < K) gl[ci * K3 + t] = gt[i];
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    const int e = tid + i * WB_T;
    gv[i] = e < K ? gl[e] : 0.f;
  }
  float f1 = 0.f, f2 = 0.f;
  if (std_) {
    float m1 = 0.f, m2 = 0.f;
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      m1 += gv[i];
      m2 = fmaf(gv[i], (wv[i] - mu) * rsg, m2);
    }
    double d1 = m1, d2 = m2;
    for (int o = 32; o > 0; o >>= 1) {
      d1 += __shfl_xor(d1, o);
      d2 += __shfl_xor(d2, o);
    }
    if ((tid & 63) == 0) {
      red[tid >> 6][0] = d1;
      red[tid >> 6][1] = d2;
    }
    __syncthreads();
    if (tid == 0) {
      double t1 = 0, t2 = 0;
      for (int w = 0; w < WB_T / 64; ++w) {
        t1 += red[w][0];
        t2 += red[w][1];
      }
      fs[0] = (float)(t1 / K);
      fs[1] = (float)(t2 / (K > 1 ? K - 1 : 1));
    }
    __syncthreads();
    f1 = fs[0];
    f2 = fs[1];
  }
  float* o = D.dw + (long long)co * K;
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    const int e = tid + i * WB_T;
    if (e < K) {
      const float v = std_ ? (gv[i] - f1 - (wv[i] - mu) * rsg * f2) * rsg : gv[i];
      o[e] = (D.acc ? o[e] : 0.f) + v;
    }
  }
}

}  // namespace u3d

using namespace u3d;

extern "C" int u3d_wstd_fwd_batch(int dtype, const u3d_wstd_desc* descs, int count, u3d_stream_t stream) {
  U3D_REQUIRE(dtype == U3D_F32 || dtype == U3D_BF16, "wstd_fwd_batch: bad dtype %d", dtype);
  U3D_REQUIRE(descs && count >= 0 && count <= U3D_WSTD_BATCH_MAX, "wstd_fwd_batch: count must be <= %d",
              U3D_WSTD_BATCH_MAX);
  if (count == 0) return U3D_OK;
  WBatch<WRow> sb{};
  WBatch<WPack> pb{};
  int sblocks = 0, pblocks = 0;
  for (int i = 0; i < count; ++i) {
    const u3d_wstd_desc& s = descs[i];
    U3D_REQUIRE(s.w && s.wpk_fwd && s.cout > 0 && s.cin > 0 && (s.ksize == 1 || s.ksize == 3),
                "wstd_fwd_batch: bad descriptor %d", i);
    U3D_REQUIRE(!s.standardize || s.wstats, "wstd_fwd_batch: descriptor %d needs wstats", i);
    const int k3 = s.ksize * s.ksize * s.ksize;
    if (s.standardize) {
      sb.d[sb.count++] = WRow{s.w, nullptr, s.wstats, nullptr, s.cout, s.cin, k3, sblocks};
      sblocks += s.cout;
    }
    pb.d[pb.count++] = WPack{s.w, s.standardize ? s.wstats : nullptr, s.wpk_fwd, s.wpk_dgrad, nullptr, nullptr,
                             nullptr, s.cout, s.cin, k3, 0, pblocks};
    pblocks += (round_up(s.cout, 32) / WB_CO) * (round_up(s.cin, 32) / WB_CI);
  }
  hipStream_t st = (hipStream_t)stream;
  if (sb.count) {
    hipLaunchKernelGGL(wstd_stats_kernel, dim3(sblocks), dim3(WB_T), 0, st, sb);
    int rc = check_launch("wstd_stats_kernel");
    if (rc) return rc;
  }
  if (dtype == U3D_BF16)
    hipLaunchKernelGGL(wstd_pack_kernel<bf16>, dim3(pblocks), dim3(WB_TT), 0, st, pb);
  else
    hipLaunchKernelGGL(wstd_pack_kernel<float>, dim3(pblocks), dim3(WB_TT), 0, st, pb);
  return check_launch("wstd_pack_kernel");
}

extern "C" long long u3d_wstd_bwd_scratch_bytes(const u3d_wstd_desc* descs, int count) {
  (void)descs;
  (void)count;
  return 256;  // no scratch needed any more (row sums stay in LDS); kept for the ABI
}

extern "C" int u3d_wstd_bwd_batch(const u3d_wstd_desc* descs, int count, float* scratch, u3d_stream_t stream) {
  (void)scratch;
  U3D_REQUIRE(descs && count >= 0 && count <= U3D_WSTD_BATCH_MAX, "wstd_bwd_batch: count must be <= %d",
              U3D_WSTD_BATCH_MAX);
  if (count == 0) return U3D_OK;
  hipStream_t st = (hipStream_t)stream;
  WBatch<WSum> sb{};
  WBatch<WPack> ab{};
  int sblocks = 0, ablocks = 0, maxk = 0;
  for (int i = 0; i < count; ++i) {
    const u3d_wstd_desc& s = descs[i];
    U3D_REQUIRE(s.part && s.w && s.dw && s.nsplit >= 1 && s.cout > 0 && s.cin > 0 && (s.ksize == 1 || s.ksize == 3),
                "wstd_bwd_batch: bad descriptor %d", i);
    U3D_REQUIRE(!s.standardize || s.wstats, "wstd_bwd_batch: descriptor %d needs wstats", i);
    const int k3 = s.ksize * s.ksize * s.ksize;
    if (s.nsplit > 1) {
      const long long per4 = (long long)k3 * round_up(s.cout, 32) * round_up(s.cin, 32) / 4;
      int sg = 1;
      while (sg < 32 && s.nsplit > 16 * sg) sg *= 2;  // <= ~16 slabs per thread
      sb.d[sb.count++] = WSum{s.part, s.nsplit, (int)per4, sg, sblocks};
      sblocks += cdiv(per4, WB_T / sg);
    }
    ab.d[ab.count++] = WPack{s.w, s.standardize ? s.wstats : nullptr, nullptr, nullptr, s.part, nullptr, s.dw,
                             s.cout, s.cin, k3, s.accumulate, ablocks};
    ablocks += cdiv(s.cout, WG_R);
    maxk = std::max(maxk, s.cin * k3);
  }
  // one row per block where every row fits the register form (U3D_WSTD_ROW=0: the chunked kernel, A/B)
  const int npt = cdiv(maxk, WB_T);
  if (opt(OPT_WSTD_ROW) != 0 && npt <= 56) {
    int rb = 0;
    for (int i = 0; i < ab.count; ++i) {
      ab.d[i].b0 = rb;
      rb += ab.d[i].cout;
    }
    if (sb.count) {
      hipLaunchKernelGGL(wstd_sum_slabs_kernel, dim3(sblocks), dim3(WB_T), 0, st, sb);
      int rc = check_launch("wstd_sum_slabs_kernel");
      if (rc) return rc;
    }
#define U3D_WROW(N) hipLaunchKernelGGL(wstd_grad_row_kernel<N>, dim3(rb), dim3(WB_T), 0, st, ab)
    if (npt <= 4) U3D_WROW(4);
    else if (npt <= 8) U3D_WROW(8);
    else if (npt <= 16) U3D_WROW(16);
    else if (npt <= 28) U3D_WROW(28);
    else U3D_WROW(56);
#undef U3D_WROW
    return check_launch("wstd_grad_row_kernel");
  }
  if (sb.count) {
    hipLaunchKernelGGL(wstd_sum_slabs_kernel, dim3(sblocks), dim3(WB_T), 0, st, sb);
    int rc = check_launch("wstd_sum_slabs_kernel");
    if (rc) return rc;
  }
  hipLaunchKernelGGL(wstd_grad_kernel, dim3(ablocks), dim3(WG_T), 0, st, ab);
  return check_launch("wstd_grad_kernel");
}

// Round 5: the slab sum of ONE weight gradient right after the launch that wrote its slabs (they then sit in L2 / the
// Infinity Cache instead of being re-read from HBM by the batched sum at the end of the backward). Same kernel, same
// slab groups, same order: slab 0 ends bitwise equal to the batched form's.
extern "C" int u3d_wgrad_sum_slabs(float* part, int nsplit, int k3, int cout, int cin, u3d_stream_t stream) {
  U3D_REQUIRE(part && nsplit >= 1 && (k3 == 1 || k3 == 27) && cout > 0 && cin > 0, "wgrad_sum_slabs: bad args");
  if (nsplit == 1) return U3D_OK;
  const long long per4 = (long long)k3 * round_up(cout, 32) * round_up(cin, 32) / 4;
  int sg = 1;
  while (sg < 32 && nsplit > 16 * sg) sg *= 2;  // as u3d_wstd_bwd_batch
  WBatch<WSum> sb{};
  sb.d[sb.count++] = WSum{part, nsplit, (int)per4, sg, 0};
  hipLaunchKernelGGL(wstd_sum_slabs_kernel, dim3(cdiv(per4, WB_T / sg)), dim3(WB_T), 0, (hipStream_t)stream, sb);
  return check_launch("wstd_sum_slabs_kernel");
}
