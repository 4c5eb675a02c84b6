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

template <typename B>
__device__ __forceinline__ int find_desc(const B& bt, int blk) {
  int i = 0;
  while (i + 1 < bt.count && bt.d[i + 1].b0 <= blk) ++i;
  return i;
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

// (1) mean / unbiased std of one row, as Conv3d.forward computes them
__global__ __launch_bounds__(WB_T) void wstd_stats_kernel(WBatch<WRow> bt) {
  __shared__ double red[WB_T / 64];
  const WRow& D = bt.d[find_desc(bt, blockIdx.x)];
  const int co = blockIdx.x - D.b0;
  const int K = D.cin * D.k3;
  const float* wr = D.w + (long long)co * K;
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
template <int K3>
__device__ __forceinline__ void stage_rows(float* s, const float* __restrict__ src, int cout, int cin, int co0,
                                           int ci0) {
  constexpr int SEG = WB_CI * K3, RS = SEG + 1;
  const int K = cin * K3, valid = min(WB_CI, cin - ci0) * K3;
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
  if (in) {
    const int step = D.sg;
    int s = q;
    for (; s + 7 * step < D.ns; s += 8 * step) {
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = p[(long long)(s + u * step) * D.per4 + i];
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int e = 0; e < 4; ++e) a[e] += v[u][e];
    }
    for (; s < D.ns; s += step) {
      const f32x4 v = p[(long long)s * D.per4 + i];
#pragma unroll
      for (int e = 0; e < 4; ++e) a[e] += v[e];
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

// (4) per-row mean(g) and sum(g * W_hat)/(K-1), one block per row; g read along ci (contiguous)
__global__ __launch_bounds__(WB_T) void wstd_rowgrad_kernel(WBatch<WRow> bt) {
  __shared__ double red[WB_T / 64];
  const WRow& D = bt.d[find_desc(bt, blockIdx.x)];
  const int co = blockIdx.x - D.b0;
  const int K = D.cin * D.k3, cout_p = round_up(D.cout, 32), cin_p = round_up(D.cin, 32);
  const float mean = D.st[co * 2], rsd = 1.f / D.st[co * 2 + 1];
  const float* wr = D.w + (long long)co * K;
  double m1 = 0.0, m2 = 0.0;
  const int n = D.k3 * D.cin;
  for (int j = threadIdx.x; j < n; j += WB_T) {  // j = t * cin + ci
    const int t = j / D.cin, ci = j - t * D.cin;
    const float gv = D.g[((long long)t * cout_p + co) * cin_p + ci];
    const float wh = (wr[ci * D.k3 + t] - mean) * rsd;
    m1 += gv;
    m2 += (double)gv * wh;
  }
  const double s1 = block_sum(m1, red), s2 = block_sum(m2, red);
  if (threadIdx.x == 0) {
    D.rowbuf[co * 2] = (float)(s1 / K);
    D.rowbuf[co * 2 + 1] = (float)(s2 / (K > 1 ? K - 1 : 1));
  }
}

template <int K3>
__device__ __forceinline__ void apply_tile(const WPack& D, float* ws, float* gs, const float* mu, const float* rsg,
                                           const float* f1, const float* f2, int co0, int ci0) {
  constexpr int SEG = WB_CI * K3, RS = SEG + 1, GSZ = WB_CO * WB_CI + 1;
  const int cout_p = round_up(D.cout, 32), cin_p = round_up(D.cin, 32);
  const bool std_ = D.st != nullptr;
  if (std_) stage_rows<K3>(ws, D.w, D.cout, D.cin, co0, ci0);
  for (int e = threadIdx.x; e < K3 * WB_CO * WB_CI; e += WB_TT) {  // g[t][co][ci] rows: coalesced along ci
    const int c = e % WB_CI, r = (e / WB_CI) % WB_CO, t = e / (WB_CI * WB_CO);
    gs[t * GSZ + r * WB_CI + c] = D.g[((long long)t * cout_p + co0 + r) * cin_p + ci0 + c];
  }
  __syncthreads();
  const int K = D.cin * K3, valid = min(WB_CI, D.cin - ci0) * K3;
  for (int e = threadIdx.x; e < WB_CO * SEG; e += WB_TT) {  // (r, c, t), t fastest = parameter order
    const int r = e / SEG, ct = e - r * SEG, c = ct / K3, t = ct - c * K3, co = co0 + r;
    if (co >= D.cout || ct >= valid) continue;
    const float gv = gs[t * GSZ + r * WB_CI + c];
    float v = gv;
    if (std_) {
      const float wh = (ws[r * RS + ct] - mu[r]) * rsg[r];
      v = (gv - f1[r] - wh * f2[r]) * rsg[r];
    }
    float* o = D.dw + (long long)co * K + ci0 * K3 + ct;
    *o = (D.acc ? *o : 0.f) + v;
  }
}

// (5) dW of one 16 x 32 tile in parameter order
__global__ __launch_bounds__(WB_TT) void wstd_apply_kernel(WBatch<WPack> bt) {
  __shared__ float ws[WB_CO * (WB_CI * 27 + 1)];
  __shared__ float gs[27 * (WB_CO * WB_CI + 1)];
  __shared__ float mu[WB_CO], rsg[WB_CO], f1[WB_CO], f2[WB_CO];
  const WPack& D = bt.d[find_desc(bt, blockIdx.x)];
  const int nci = round_up(D.cin, 32) / WB_CI;
  const int tile = blockIdx.x - D.b0, co0 = (tile / nci) * WB_CO, ci0 = (tile % nci) * WB_CI;
  if (threadIdx.x < WB_CO) {
    const int co = co0 + threadIdx.x;
    const bool s = D.st && co < D.cout;
    mu[threadIdx.x] = s ? D.st[co * 2] : 0.f;
    rsg[threadIdx.x] = s ? 1.f / D.st[co * 2 + 1] : 1.f;
    f1[threadIdx.x] = s ? D.rowbuf[co * 2] : 0.f;
    f2[threadIdx.x] = s ? D.rowbuf[co * 2 + 1] : 0.f;
  }
  if (D.k3 == 27)
    apply_tile<27>(D, ws, gs, mu, rsg, f1, f2, co0, ci0);
  else
    apply_tile<1>(D, ws, gs, mu, rsg, f1, f2, co0, ci0);
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
  long long rows = 0;
  for (int i = 0; i < count; ++i) rows += descs[i].cout;
  return rows * 2 * (long long)sizeof(float);
}

extern "C" int u3d_wstd_bwd_batch(const u3d_wstd_desc* descs, int count, float* scratch, u3d_stream_t stream) {
  U3D_REQUIRE(descs && count >= 0 && count <= U3D_WSTD_BATCH_MAX, "wstd_bwd_batch: count must be <= %d",
              U3D_WSTD_BATCH_MAX);
  if (count == 0) return U3D_OK;
  U3D_REQUIRE(scratch, "wstd_bwd_batch: scratch required (u3d_wstd_bwd_scratch_bytes)");
  hipStream_t st = (hipStream_t)stream;
  WBatch<WSum> sb{};
  WBatch<WRow> rb{};
  WBatch<WPack> ab{};
  int sblocks = 0, rblocks = 0, ablocks = 0;
  long long roff = 0;
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
    float* rowbuf = scratch + roff;
    roff += 2LL * s.cout;
    if (s.standardize) {
      rb.d[rb.count++] = WRow{s.w, s.part, s.wstats, rowbuf, s.cout, s.cin, k3, rblocks};
      rblocks += s.cout;
    }
    ab.d[ab.count++] = WPack{s.w, s.standardize ? s.wstats : nullptr, nullptr, nullptr, s.part, rowbuf, s.dw,
                             s.cout, s.cin, k3, s.accumulate, ablocks};
    ablocks += (round_up(s.cout, 32) / WB_CO) * (round_up(s.cin, 32) / WB_CI);
  }
  if (sb.count) {
    hipLaunchKernelGGL(wstd_sum_slabs_kernel, dim3(sblocks), dim3(WB_T), 0, st, sb);
    int rc = check_launch("wstd_sum_slabs_kernel");
    if (rc) return rc;
  }
  if (rb.count) {
    hipLaunchKernelGGL(wstd_rowgrad_kernel, dim3(rblocks), dim3(WB_T), 0, st, rb);
    int rc = check_launch("wstd_rowgrad_kernel");
    if (rc) return rc;
  }
  hipLaunchKernelGGL(wstd_apply_kernel, dim3(ablocks), dim3(WB_TT), 0, st, ab);
  return check_launch("wstd_apply_kernel");
}
