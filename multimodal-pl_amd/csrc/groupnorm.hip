// GroupNorm statistics and the backward of relu(group_norm(x)) on NDHWC tensors.
// Reference: nn.GroupNorm(G, C) + nn.ReLU in NoBottleneck (unet3D.py:44-53), fusionConv (:1640-1642),
// precls_conv (:1653-1655), GAP (:1659-1661). The forward apply is fused into the consumer conv's
// prologue (conv.hip), so only statistics are produced here.
//
// Determinism: each block reduces a fixed voxel range into per-channel fp32 partials (of values shifted
// by a per-group constant, so the sum of squares does not cancel); the LAST block to finish (completion
// counter, agent-scope release/acquire) combines blocks and channels in fp64 in a fixed order — one launch for
// the statistics, two for the backward (partial+final, apply). No float atomics.
//
// Workspace (u3d_gn_workspace_bytes): [256 B completion counters][partials n x nblk x 2 x c f32][coef n x 5 x c
// f32]. It must be zero-filled when first allocated; every launch leaves its counter at zero again.
#include <cstdlib>

#include "common.h"

namespace u3d {

constexpr int GT = 512;
constexpr int GN_CNT_BYTES = 256;
constexpr int GN_PAIRS_MAX = 2048;  // n * c of the backward's last-block combine (LDS)

struct RedGeom {
  int n, c, groups, cpg, nblk, vpb, chn, vlanes;  // chn = 16-B chunks per voxel, vlanes = voxels per pass
  long long v;
  int fh, fw, ch, cw;  // u3d_gn_bwd2_s2: fine h, w (x) and compact h, w (da2 = a stride-2 1^3 data gradient)
  long long cv;        // compact voxels per sample
  float rhw, rfw;      // 1 / (fh * fw), 1 / fw (s2_index; voxels per sample < 2^24)
};

// quotient of 0 <= x < 2^24 by d from x * (1/d) in fp32 (off by at most one, corrected): ~6 instructions instead of
// the ~30 of a 32-bit integer division per voxel
__device__ __forceinline__ int div_small(int x, int d, float rd) {
  int q = (int)((float)x * rd);
  q -= q * d > x;
  q += (q + 1) * d <= x;
  return q;
}

// da2 of u3d_gn_bwd2_s2 is the stride-2 1^3 conv's data gradient at the conv's OUTPUT resolution: nonzero only at
// fine voxels with all coordinates even. Returns its compact index, or -1 (odd voxel: dA2 = 0).
__device__ __forceinline__ long long s2_index(long long vv, const RedGeom& g) {
  const int vi = (int)vv, hw = g.fh * g.fw;
  const int a = div_small(vi, hw, g.rhw), rem = vi - a * hw, b = div_small(rem, g.fw, g.rfw), c = rem - b * g.fw;
  return ((a | b | c) & 1) ? -1 : ((long long)(a >> 1) * g.ch + (b >> 1)) * g.cw + (c >> 1);
}

// U3D_GN2_COND (default 1): the compact operand is read with a buffer load whose offset is the out-of-range sentinel
// for odd voxels — zeros with no memory request and no branch (a branch around a plain load made the compiler wait
// for it inside the branch: one round trip per voxel); 0: a clamped straight-line load for every voxel (round 3).
#ifndef U3D_GN2_COND
#define U3D_GN2_COND 1
#endif
template <typename T, bool S2>
__device__ __forceinline__ void load_da2(const T* __restrict__ da2, const RedGeom& g, int n, long long vv, int j,
                                         long long off, float (&d2)[16 / sizeof(T)]) {
  constexpr int VEC = 16 / sizeof(T);
  if constexpr (S2) {
    const long long ci = s2_index(vv, g);
    if (U3D_GN2_COND) {  // host: n * cv * c * sizeof(T) < 2 GiB
      const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)da2, 0, (int)(g.n * g.cv * g.c * (int)sizeof(T)),
                                                        0x00020000);
      const unsigned bo = ci >= 0 ? (unsigned)((((long long)n * g.cv + ci) * g.c + j * VEC) * sizeof(T)) : 0xFFFFFFF0u;
      const u32x4 r = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, bo, 0, 0));
      if constexpr (sizeof(T) == 4) {
#pragma unroll
        for (int i = 0; i < 4; ++i) d2[i] = __uint_as_float(r[i]);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          d2[2 * i] = __uint_as_float(r[i] << 16);
          d2[2 * i + 1] = __uint_as_float(r[i] & 0xffff0000u);
        }
      }
      return;
    }
    load16<T>(da2 + ((long long)n * g.cv + (ci < 0 ? 0 : ci)) * g.c + j * VEC, d2);  // clamped: straight-line load
    if (ci < 0)
#pragma unroll
      for (int e = 0; e < VEC; ++e) d2[e] = 0.f;
  } else {
    load16<T>(da2 + off, d2);
  }
}

// Round 6: fine-voxel coordinates advanced incrementally along a loop's fixed voxel stride (no per-voxel divisions:
// s2_index's two quotients were most of the S2 kernels' extra instructions), and da2 read by compact index
struct Crd {
  int z, y, x;
};
__device__ __forceinline__ Crd crd_of(long long v, const RedGeom& g) {
  const int vi = (int)v, hw = g.fh * g.fw;
  const int a = vi / hw, rem = vi - a * hw, b = rem / g.fw;
  return Crd{a, b, rem - b * g.fw};
}
__device__ __forceinline__ Crd crd_add(Crd c, const Crd& s, const RedGeom& g) {  // s: a stride's (z, y, x), y < fh, x < fw
  c.x += s.x;
  const int cx = c.x >= g.fw;
  c.x -= cx ? g.fw : 0;
  c.y += s.y + cx;
  const int cy = c.y >= g.fh;
  c.y -= cy ? g.fh : 0;
  c.z += s.z + cy;
  return c;
}
// da2 (compact) at fine voxel c of sample n, zeros at odd voxels or past the volume (ok = false)
template <typename T>
__device__ __forceinline__ void load_da2_crd(const T* __restrict__ da2, const RedGeom& g, int n, const Crd& c, bool ok,
                                             int j, float (&d2)[16 / sizeof(T)]) {
  constexpr int VEC = 16 / sizeof(T);
  const bool ev = ok && ((c.z | c.y | c.x) & 1) == 0;
  const long long ci = ((long long)(c.z >> 1) * g.ch + (c.y >> 1)) * g.cw + (c.x >> 1);
  const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)da2, 0, (int)(g.n * g.cv * g.c * (int)sizeof(T)), 0x00020000);
  const unsigned bo = ev ? (unsigned)((((long long)n * g.cv + ci) * g.c + j * VEC) * sizeof(T)) : 0xFFFFFFF0u;
  const u32x4 r = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, bo, 0, 0));
  if constexpr (sizeof(T) == 4) {
#pragma unroll
    for (int i = 0; i < 4; ++i) d2[i] = __uint_as_float(r[i]);
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      d2[2 * i] = __uint_as_float(r[i] << 16);
      d2[2 * i + 1] = __uint_as_float(r[i] & 0xffff0000u);
    }
  }
}

// reduction blocks over all samples
static long long gn_max_blocks() { return std::max(1, opt(OPT_GN_MAXBLK)); }

static RedGeom make_geom(int n, int c, long long v, int groups, int vec) {
  RedGeom g{};
  g.n = n;
  g.c = c;
  g.v = v;
  g.groups = groups;
  g.cpg = groups > 0 ? c / groups : 0;
  g.chn = c / vec;
  g.vlanes = std::max(1, GT / g.chn);
  // blocks in all ~ bytes / 64 KB, 16..256 (512 threads, 32 KB of loads in flight each): every CU streams on
  // the big tensors, and the partials stay few enough for a one-round last-block combine
  const long long bytes = v * n * c * (vec == 8 ? 2 : 4);
  const long long nb = std::min<long long>(gn_max_blocks(), std::max<long long>(16, bytes >> 16));
  long long want = std::max<long long>((long long)g.vlanes * 4, (v * n + nb - 1) / nb);
  g.vpb = (int)((want + g.vlanes - 1) / g.vlanes * g.vlanes);
  g.nblk = (int)((v + g.vpb - 1) / g.vpb);
  return g;
}

// Block-level per-channel reduction of VEC-wide per-thread partials into out[c] for c < C. Thread t holds chunk
// j = t % chn of voxel lane t / chn. When chn divides the wave (64 % chn == 0) the lanes of one chunk are chn apart
// inside a wave: an xor-shuffle tree over offsets chn..32 reduces them, then the 8 waves' rows are summed through
// LDS in wave order (log2(64/chn) shuffles + 8 LDS reads instead of a serial walk over the voxel lanes).
// Deterministic either way (fixed tree / order).
template <int VEC, int NV>
__device__ __forceinline__ void block_channel_reduce(float (&acc)[NV][VEC], float* lds, const RedGeom& g,
                                                     float* out /*[NV][C]*/) {
  const int tid = threadIdx.x;
  constexpr int NW = GT / 64;
  if (g.chn <= 64 && (64 % g.chn) == 0 && NW * NV * g.c <= GT * VEC) {
    const int lane = tid & 63, wave = tid >> 6;
    for (int o = g.chn; o < 64; o <<= 1)
#pragma unroll
      for (int k = 0; k < NV; ++k)
#pragma unroll
        for (int e = 0; e < VEC; ++e) acc[k][e] += __shfl_xor(acc[k][e], o);
    __syncthreads();  // lds may still be read by a previous reduction
    if (lane < g.chn)
#pragma unroll
      for (int k = 0; k < NV; ++k)
#pragma unroll
        for (int e = 0; e < VEC; ++e) lds[(wave * NV + k) * g.c + lane * VEC + e] = acc[k][e];
    __syncthreads();
    for (int i = tid; i < NV * g.c; i += GT) {
      const int k = i / g.c, c = i - k * g.c;
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) s += lds[(w * NV + k) * g.c + c];
      __hip_atomic_store(out + k * g.c + c, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sc1: write-through
    }
    return;
  }
  const int active = g.vlanes * g.chn;
  for (int k = 0; k < NV; ++k) {
    __syncthreads();
    if (tid < active)
      for (int e = 0; e < VEC; ++e) lds[tid * VEC + e] = acc[k][e];
    __syncthreads();
    for (int c = tid; c < g.c; c += GT) {
      const int j = c / VEC, e = c % VEC;
      float s = 0.f;
      for (int l = 0; l < g.vlanes; ++l) s += lds[(l * g.chn + j) * VEC + e];
      __hip_atomic_store(out + k * g.c + c, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sc1: write-through
    }
  }
}

// True (in every thread) for the block that finished last. Hand-off without fences (MI355X guide, inter-
// workgroup visibility): partials are written with sc1 (write-through) stores, every wave drains them
// (vmcnt(0)) before the barrier, one lane per block adds to the counter (agent scope), and the last block
// reads the partials with sc1 loads (L2-served, not a stale L1).
__device__ __forceinline__ bool block_is_last(unsigned* cnt, unsigned total) {
  __shared__ unsigned s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) s_last = atomicAdd(cnt, 1u) == total - 1;
  __syncthreads();
  if (s_last && threadIdx.x == 0) atomicExch(cnt, 0u);  // ready for the next launch
  return s_last;
}

__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Last-block combine, phase 1: cs[p] = (sum_b P[n][b][0][c], sum_b P[n][b][1][c]) in fp64 for p = n*C + c.
// Threads run along channels (coalesced partial rows) and over block slices; slices combine in fixed order.
__device__ __forceinline__ void combine_channels(const float* __restrict__ ws, const RedGeom& g, double (*cs)[2],
                                                 int nv = 2, int k0 = 0) {
  __shared__ double part[GT][2];
  const int tid = threadIdx.x, npairs = g.n * g.c;
  const int spl = npairs >= GT ? 1 : GT / npairs;
  for (int p0 = 0; p0 < npairs; p0 += GT) {
    const int p = p0 + tid % min(npairs, GT), sl = tid / min(npairs, GT);
    double s1 = 0, s2 = 0;
    if (p < npairs && sl < spl) {
      const int nn = p / g.c, c = p % g.c;
      // partials of other blocks (rows of nv x C per block; this pass reads rows k0, k0 + 1): sc1 loads only
      const float* q = ws + (long long)nn * g.nblk * nv * g.c + k0 * g.c + c;
      // 16 predicated loads in flight per round, then the adds in block order (the same order as a serial walk):
      // the combine costs ceil(nblk / (8 spl)) latency rounds instead of one per block
      for (int b0 = sl; b0 < g.nblk; b0 += 8 * spl) {
        float a[8], bb[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int b = min(b0 + u * spl, g.nblk - 1);  // clamped address: straight-line loads, no branches
          a[u] = ld_sc1(q + (long long)b * nv * g.c);
          bb[u] = ld_sc1(q + (long long)b * nv * g.c + g.c);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const bool ok = b0 + u * spl < g.nblk;
          s1 += ok ? a[u] : 0.f;
          s2 += ok ? bb[u] : 0.f;
        }
      }
    }
    part[tid][0] = s1;
    part[tid][1] = s2;
    __syncthreads();
    if (tid < min(npairs - p0, GT)) {
      double t1 = 0, t2 = 0;
      for (int k = 0; k < spl; ++k) {
        t1 += part[k * min(npairs, GT) + tid][0];
        t2 += part[k * min(npairs, GT) + tid][1];
      }
      cs[p0 + tid][0] = t1;
      cs[p0 + tid][1] = t2;
    }
    __syncthreads();
  }
}

template <typename T>
__global__ __launch_bounds__(GT) void gn_stats_kernel(const T* __restrict__ x, RedGeom g, float* __restrict__ ws,
                                                     unsigned* __restrict__ cnt, float* __restrict__ stats) {
  constexpr int VEC = 16 / sizeof(T);
  __shared__ float lds[GT * VEC];
  const int n = blockIdx.y, blk = blockIdx.x, tid = threadIdx.x;
  const T* xn = x + (long long)n * g.v * g.c;
  const int j = tid % g.chn, vl = tid / g.chn;
  float acc[2][VEC];
  for (int e = 0; e < VEC; ++e) acc[0][e] = acc[1][e] = 0.f;
  if (vl < g.vlanes) {
    float shift[VEC];
    for (int e = 0; e < VEC; ++e) shift[e] = to_f(xn[((j * VEC + e) / g.cpg) * g.cpg]);  // x[n, voxel 0, first ch of group]
    const long long v0 = (long long)blk * g.vpb, v1 = std::min<long long>(g.v, v0 + g.vpb);
    // rounds of 8 predicated loads (64 KB per CU in flight): a small tensor costs one latency round, not one per
    // voxel; voxels past the range read as the shift (d = 0), so the sums are those of the serial walk
    for (long long v = v0 + vl; v < v1; v += 8 * g.vlanes) {
      float xv[8][VEC];
#pragma unroll
      for (int u = 0; u < 8; ++u) load16<T>(xn + std::min(v + u * g.vlanes, v1 - 1) * g.c + j * VEC, xv[u]);
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int e = 0; e < VEC; ++e) {
          const float d = v + u * g.vlanes < v1 ? xv[u][e] - shift[e] : 0.f;
          acc[0][e] += d;
          acc[1][e] = fmaf(d, d, acc[1][e]);
        }
    }
  }
  block_channel_reduce<VEC, 2>(acc, lds, g, ws + ((long long)n * g.nblk + blk) * 2 * g.c);
  if (!block_is_last(cnt, (unsigned)(g.n * g.nblk))) return;
  // combine: per (n, c) sums over the blocks, then per (n, group) over its channels, fixed order, fp64
  __shared__ double cs[GN_PAIRS_MAX][2];
  // the first group's shift is loaded before the combine (its latency overlaps the partial loads)
  const float sh0 = tid < g.n * g.groups ? to_f(x[(long long)(tid / g.groups) * g.v * g.c + (tid % g.groups) * g.cpg]) : 0.f;
  combine_channels(ws, g, cs);
  for (int p = tid; p < g.n * g.groups; p += GT) {
    const int nn = p / g.groups, gr = p % g.groups;
    double s1 = 0, s2 = 0;
    for (int k = 0; k < g.cpg; ++k) {
      s1 += cs[nn * g.c + gr * g.cpg + k][0];
      s2 += cs[nn * g.c + gr * g.cpg + k][1];
    }
    const double M = (double)g.v * g.cpg;
    const double shift = p == tid ? sh0 : to_f(x[(long long)nn * g.v * g.c + gr * g.cpg]);
    const double dm = s1 / M;
    double var = s2 / M - dm * dm;
    if (var < 0) var = 0;
    stats[(nn * g.groups + gr) * 2] = (float)(shift + dm);
    stats[(nn * g.groups + gr) * 2 + 1] = (float)(1.0 / sqrt(var + 1e-5));
  }
}

// (2) apply coefficients per (n, c) from the per-(n, c) sums cs; (3) dgamma / dbeta per c (gn_bwd_partial's last
// block and gn_bwd_parts_finalize)
__device__ __forceinline__ void gn_bwd_coefs(const double (*cs)[2], const RedGeom& g, const float* __restrict__ stats,
                                             const float* __restrict__ gamma, const float* __restrict__ beta,
                                             float* __restrict__ coef, float* __restrict__ dgamma,
                                             float* __restrict__ dbeta, int accp) {
  const int tid = threadIdx.x, npairs = g.n * g.c;
  const double M = (double)g.v * g.cpg;
  for (int p = tid; p < npairs; p += GT) {
    const int nn = p / g.c, c = p % g.c, gr = c / g.cpg;
    double a = 0, bb = 0;
    for (int k = 0; k < g.cpg; ++k) {
      const int cc = gr * g.cpg + k;
      a += (double)gamma[cc] * cs[nn * g.c + cc][0];
      bb += (double)gamma[cc] * cs[nn * g.c + cc][1];
    }
    const float ca = (float)(a / M), cb = (float)(bb / M);
    const float mu = stats[(nn * g.groups + gr) * 2], rs = stats[(nn * g.groups + gr) * 2 + 1];
    const float scv = rs * gamma[c];
    float* o = coef + (long long)nn * 5 * g.c;
    o[c] = scv;
    o[g.c + c] = beta[c] - mu * scv;
    o[2 * g.c + c] = rs * gamma[c];
    o[3 * g.c + c] = -rs * rs * cb;
    o[4 * g.c + c] = -rs * ca + rs * rs * cb * mu;
  }
  for (int c = tid; c < g.c; c += GT) {
    double tg = 0, tb = 0;
    for (int nn = 0; nn < g.n; ++nn) {
      tb += cs[nn * g.c + c][0];
      tg += cs[nn * g.c + c][1];
    }
    if (dgamma) dgamma[c] = (accp ? dgamma[c] : 0.f) + (float)tg;
    if (dbeta) dbeta[c] = (accp ? dbeta[c] : 0.f) + (float)tb;
  }
}

// backward: per channel s1 = sum g, s2 = sum g*xhat (g = m*dA, m = the forward prologue's relu test
// x*sc + sh > 0), then in the last block the apply coefficients of every (n, c), SoA coef[n][5][C]:
//   sc, sh, alpha = rs*gamma_c, bx = -rs^2 * b_g, d = -rs*a_g + rs^2*b_g*mu
// with a_g = sum_{c in g} gamma_c s1_c / M, b_g = sum gamma_c s2_c / M, so that
//   dx = alpha * m * dA + bx * x + d  ==  rs * (gamma*m*dA - a_g - xhat * b_g)   (autograd of GN, unet3D.py:44-53)
// and dgamma_c = sum_n s2, dbeta_c = sum_n s1.
template <typename T>
__global__ __launch_bounds__(GT) void gn_bwd_partial(const T* __restrict__ da, const T* __restrict__ x, RedGeom g,
                                                    const float* __restrict__ stats, const float* __restrict__ gamma,
                                                    const float* __restrict__ beta, float* __restrict__ ws,
                                                    unsigned* __restrict__ cnt, float* __restrict__ coef,
                                                    float* __restrict__ dgamma, float* __restrict__ dbeta, int accp) {
  constexpr int VEC = 16 / sizeof(T);
  __shared__ float lds[GT * VEC];
  __shared__ double cs[GN_PAIRS_MAX][2];
  const int n = blockIdx.y, blk = blockIdx.x, tid = threadIdx.x;
  const long long base = (long long)n * g.v * g.c;
  const int j = tid % g.chn, vl = tid / g.chn;
  float acc[2][VEC];
  for (int e = 0; e < VEC; ++e) acc[0][e] = acc[1][e] = 0.f;
  if (vl < g.vlanes) {
    float mu[VEC], rs[VEC], sc[VEC], sh[VEC];
    for (int e = 0; e < VEC; ++e) {
      const int c = j * VEC + e, gr = c / g.cpg;
      mu[e] = stats[(n * g.groups + gr) * 2];
      rs[e] = stats[(n * g.groups + gr) * 2 + 1];
      sc[e] = rs[e] * gamma[c];
      sh[e] = beta[c] - mu[e] * sc[e];
    }
    const long long v0 = (long long)blk * g.vpb, v1 = std::min<long long>(g.v, v0 + g.vpb);
    auto step = [&](const float (&xv)[VEC], const float (&dv)[VEC]) {
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        const float xh = (xv[e] - mu[e]) * rs[e];
        const float gd = fmaf(xv[e], sc[e], sh[e]) > 0.f ? dv[e] : 0.f;
        acc[0][e] += gd;
        acc[1][e] = fmaf(gd, xh, acc[1][e]);
      }
    };
    // rounds of 4 predicated voxel pairs (8 loads in flight); past the range dA = 0 contributes nothing
    for (long long v = v0 + vl; v < v1; v += 4 * g.vlanes) {
      float xv[4][VEC], dv[4][VEC];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long long vv = std::min(v + u * g.vlanes, v1 - 1);
        load16<T>(x + base + vv * g.c + j * VEC, xv[u]);
        load16<T>(da + base + vv * g.c + j * VEC, dv[u]);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (v + u * g.vlanes >= v1)
#pragma unroll
          for (int e = 0; e < VEC; ++e) dv[u][e] = 0.f;
        step(xv[u], dv[u]);
      }
    }
  }
  block_channel_reduce<VEC, 2>(acc, lds, g, ws + ((long long)n * g.nblk + blk) * 2 * g.c);
  if (!block_is_last(cnt, (unsigned)(g.n * g.nblk))) return;
  // (1) per (n, c): fp64 sums over the blocks, fixed order
  combine_channels(ws, g, cs);
  gn_bwd_coefs(cs, g, stats, gamma, beta, coef, dgamma, dbeta, accp);
}

// The same backward when its per-channel partials come from the data-gradient ring's epilogue
// (u3d_conv32_ring_dgrad_gn): parts [n][nparts][c][2] = (sum g, sum g*xhat) of one workgroup; one block sums them
// per (n, c) in fp64 in a fixed order (deterministic) and writes the apply coefficients.
// Round 6: 1024 threads with 8 independent loads in flight each (was 512 x 4): at 96^3 (n = 2, 32 channels, 128 parts
// per sample) every thread sums its 8 rows in one load round instead of 4 dependent rounds (the finalize was
// latency-bound: 6.7 us per launch, 9 launches per step). Same slices, same fixed order within and across them as
// any other thread count gives for its slicing: deterministic.
constexpr int GPF = 1024;
__global__ __launch_bounds__(GPF) void gn_bwd_parts_finalize(const float* __restrict__ parts, int nparts, RedGeom g,
                                                             const float* __restrict__ stats,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ beta, float* __restrict__ coef,
                                                             float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                             int accp) {
  __shared__ double cs[GN_PAIRS_MAX][2];
  __shared__ double red[GPF][2];
  // GPF / npairs threads per (n, c) pair (fixed slices of the parts, independent loads in flight), then the slices
  // in fixed order: deterministic, latency of ~nparts / slices loads instead of nparts dependent ones
  const int tid = threadIdx.x, npairs = g.n * g.c;
  const int spl = npairs >= GPF ? 1 : GPF / npairs;
  for (int p0 = 0; p0 < npairs; p0 += GPF) {
    const int p = p0 + tid % min(npairs, GPF), sl = tid / min(npairs, GPF);
    double s1 = 0, s2 = 0;
    if (p < npairs && sl < spl) {
      const int nn = p / g.c, c = p % g.c;
      const float* q = parts + (long long)nn * nparts * 2 * g.c + 2 * c;
      int b = sl;
      for (; b + 7 * spl < nparts; b += 8 * spl) {
        float2 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float2*>(q + (long long)(b + u * spl) * 2 * g.c);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          s1 += v[u].x;
          s2 += v[u].y;
        }
      }
      for (; b < nparts; b += spl) {
        const float2 v = *reinterpret_cast<const float2*>(q + (long long)b * 2 * g.c);
        s1 += v.x;
        s2 += v.y;
      }
    }
    red[tid][0] = s1;
    red[tid][1] = s2;
    __syncthreads();
    if (tid < min(npairs - p0, GPF)) {
      double t1 = 0, t2 = 0;
      for (int k = 0; k < spl; ++k) {
        t1 += red[k * min(npairs, GPF) + tid][0];
        t2 += red[k * min(npairs, GPF) + tid][1];
      }
      cs[p0 + tid][0] = t1;
      cs[p0 + tid][1] = t2;
    }
    __syncthreads();
  }
  if (tid < GT) gn_bwd_coefs(cs, g, stats, gamma, beta, coef, dgamma, dbeta, accp);  // (GT-strided loops)
}

// dx (+)= alpha*m*dA + bx*x + d per element; grid (blocks, n): a thread's 16-B channel chunk is fixed (the
// grid stride is a multiple of the chunks per voxel), so its 5 x VEC coefficients load once into registers.
// Round 6: ACC a template parameter and GA_U voxels per round with every load issued before the math: with the
// runtime `accum` branch around the dx load the compiler waited for all loads right after it, one voxel (2-3 loads)
// in flight per thread per round trip (5 launches of 60 us per step at 96^3). Same arithmetic per element.
#ifndef U3D_GA_U
#define U3D_GA_U 1  // (2, 4: measured slower, gpurun_out/r06hh)
#endif
template <typename T, bool ACC>
__global__ __launch_bounds__(GT) void gn_bwd_apply(const T* __restrict__ da, const T* __restrict__ x, RedGeom g,
                                                  const float* __restrict__ coef, T* __restrict__ dx) {
  constexpr int VEC = 16 / sizeof(T), U = U3D_GA_U;
  const int n = blockIdx.y;
  const int first = blockIdx.x * blockDim.x + threadIdx.x, stride = gridDim.x * blockDim.x;  // chn | blockDim
  const int j = first % g.chn;
  float cf[5][VEC];
  const float* cb = coef + (long long)n * 5 * g.c + j * VEC;
#pragma unroll
  for (int k = 0; k < 5; ++k)
#pragma unroll
    for (int e = 0; e < VEC; ++e) cf[k][e] = cb[k * g.c + e];
  const T* xn = x + (long long)n * g.v * g.c + j * VEC;
  const T* dan = da + (long long)n * g.v * g.c + j * VEC;
  T* dxn = dx + (long long)n * g.v * g.c + j * VEC;
  const long long vstep = stride / g.chn;
  for (long long vox = first / g.chn; vox < g.v; vox += U * vstep) {
    float xv[U][VEC], dv[U][VEC], o[U][VEC];
#pragma unroll
    for (int u = 0; u < U; ++u) {  // clamped straight-line loads
      const long long off = std::min(vox + u * vstep, g.v - 1) * g.c;
      load16<T>(xn + off, xv[u]);
      load16<T>(dan + off, dv[u]);
      if constexpr (ACC) load16<T>(dxn + off, o[u]);
    }
    __builtin_amdgcn_sched_barrier(0);  // all of the round's loads ahead of its math and stores
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        const float gd = fmaf(xv[u][e], cf[0][e], cf[1][e]) > 0.f ? dv[u][e] : 0.f;
        const float r = fmaf(cf[2][e], gd, fmaf(cf[3][e], xv[u][e], cf[4][e]));
        o[u][e] = ACC ? o[u][e] + r : r;
      }
      if (vox + u * vstep < g.v) store16<T>(dxn + (vox + u * vstep) * g.c, o[u]);
    }
  }
}
template <typename T>
static void launch_gn_bwd_apply(dim3 grid, int thr, hipStream_t s, const T* da, const T* x, const RedGeom& g,
                                const float* coef, T* dx, int accum) {
  if (accum)
    hipLaunchKernelGGL((gn_bwd_apply<T, true>), grid, dim3(thr), 0, s, da, x, g, coef, dx);
  else
    hipLaunchKernelGGL((gn_bwd_apply<T, false>), grid, dim3(thr), 0, s, da, x, g, coef, dx);
}


#ifndef U3D_GN2_PR
#define U3D_GN2_PR 4
#endif
// Two GroupNorm consumers of the SAME activation x with the same statistics (NoBottleneck gn1 and the downsample
// GN of the first block of a stage, unet3D.py:44-53 + _make_layer :1666-1686): one partial pass over x, dA1, dA2
// (per set k: s1_k = sum m_k dA_k, s2_k = sum m_k dA_k xhat) and one apply writing
//   dx (+)= alpha1 m1 dA1 + alpha2 m2 dA2 + (bx1 + bx2) x + (d1 + d2)
// instead of two full backward passes (x read 4 times, dx written twice). coef2 [2][n][5][C].
template <typename T, bool S2>
__global__ __launch_bounds__(GT) void gn_bwd2_partial(const T* __restrict__ da1, const T* __restrict__ da2,
                                                     const T* __restrict__ x, RedGeom g, const float* __restrict__ stats,
                                                     const float* __restrict__ gamma1, const float* __restrict__ beta1,
                                                     const float* __restrict__ gamma2, const float* __restrict__ beta2,
                                                     float* __restrict__ ws, unsigned* __restrict__ cnt,
                                                     float* __restrict__ coef, float* __restrict__ dgamma1,
                                                     float* __restrict__ dbeta1, float* __restrict__ dgamma2,
                                                     float* __restrict__ dbeta2, int accp) {
  constexpr int VEC = 16 / sizeof(T);
  __shared__ float lds[GT * VEC];
  __shared__ double cs[GN_PAIRS_MAX][2];
  const int n = blockIdx.y, blk = blockIdx.x, tid = threadIdx.x;
  const long long base = (long long)n * g.v * g.c;
  const int j = tid % g.chn, vl = tid / g.chn;
  float acc[4][VEC];
  for (int e = 0; e < VEC; ++e) acc[0][e] = acc[1][e] = acc[2][e] = acc[3][e] = 0.f;
  if (vl < g.vlanes) {
    float mu[VEC], rs[VEC], sc1[VEC], sh1[VEC], sc2[VEC], sh2[VEC];
    for (int e = 0; e < VEC; ++e) {
      const int c = j * VEC + e, gr = c / g.cpg;
      mu[e] = stats[(n * g.groups + gr) * 2];
      rs[e] = stats[(n * g.groups + gr) * 2 + 1];
      sc1[e] = rs[e] * gamma1[c];
      sh1[e] = beta1[c] - mu[e] * sc1[e];
      sc2[e] = rs[e] * gamma2[c];
      sh2[e] = beta2[c] - mu[e] * sc2[e];
    }
    const long long v0 = (long long)blk * g.vpb, v1 = std::min<long long>(g.v, v0 + g.vpb);
    auto step = [&](const float (&xv)[VEC], const float (&d1)[VEC], const float (&d2)[VEC]) {
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        const float xh = (xv[e] - mu[e]) * rs[e];
        const float g1 = fmaf(xv[e], sc1[e], sh1[e]) > 0.f ? d1[e] : 0.f;
        const float g2 = fmaf(xv[e], sc2[e], sh2[e]) > 0.f ? d2[e] : 0.f;
        acc[0][e] += g1;
        acc[1][e] = fmaf(g1, xh, acc[1][e]);
        acc[2][e] += g2;
        acc[3][e] = fmaf(g2, xh, acc[3][e]);
      }
    };
    constexpr int PR = U3D_GN2_PR;  // voxels per round (3 predicated loads each)
    Crd cr{}, s1{}, sr{};  // S2: coordinates of v, the strides vlanes and PR * vlanes
    if constexpr (S2) {
      cr = crd_of(v0 + vl, g);
      s1 = crd_of(g.vlanes, g);
      sr = crd_of((long long)PR * g.vlanes, g);
    }
    for (long long v = v0 + vl; v < v1; v += PR * g.vlanes) {
      float xv[PR][VEC], d1[PR][VEC], d2[PR][VEC];
      Crd cu = cr;
#pragma unroll
      for (int u = 0; u < PR; ++u) {
        const long long vv = std::min(v + u * g.vlanes, v1 - 1);
        const long long off = base + vv * g.c + j * VEC;
        load16<T>(x + off, xv[u]);
        load16<T>(da1 + off, d1[u]);
        if constexpr (S2) {
          load_da2_crd<T>(da2, g, n, cu, v + u * g.vlanes < v1, j, d2[u]);
          cu = crd_add(cu, s1, g);
        } else {
          load_da2<T, S2>(da2, g, n, vv, j, off, d2[u]);
        }
      }
      if constexpr (S2) cr = crd_add(cr, sr, g);
#pragma unroll
      for (int u = 0; u < PR; ++u) {
        if (v + u * g.vlanes >= v1)
#pragma unroll
          for (int e = 0; e < VEC; ++e) d1[u][e] = d2[u][e] = 0.f;
        step(xv[u], d1[u], d2[u]);
      }
    }
  }
  block_channel_reduce<VEC, 4>(acc, lds, g, ws + ((long long)n * g.nblk + blk) * 4 * g.c);
  if (!block_is_last(cnt, (unsigned)(g.n * g.nblk))) return;
  const int npairs = g.n * g.c;
  const double M = (double)g.v * g.cpg;
  for (int k = 0; k < 2; ++k) {
    const float* gamma = k ? gamma2 : gamma1;
    const float* beta = k ? beta2 : beta1;
    combine_channels(ws, g, cs, 4, 2 * k);
    for (int p = tid; p < npairs; p += GT) {
      const int nn = p / g.c, c = p % g.c, gr = c / g.cpg;
      double a = 0, bb = 0;
      for (int q = 0; q < g.cpg; ++q) {
        const int cc = gr * g.cpg + q;
        a += (double)gamma[cc] * cs[nn * g.c + cc][0];
        bb += (double)gamma[cc] * cs[nn * g.c + cc][1];
      }
      const float ca = (float)(a / M), cb = (float)(bb / M);
      const float mu = stats[(nn * g.groups + gr) * 2], rs = stats[(nn * g.groups + gr) * 2 + 1];
      const float scv = rs * gamma[c];
      float* o = coef + ((long long)k * g.n + nn) * 5 * g.c;
      o[c] = scv;
      o[g.c + c] = beta[c] - mu * scv;
      o[2 * g.c + c] = rs * gamma[c];
      o[3 * g.c + c] = -rs * rs * cb;
      o[4 * g.c + c] = -rs * ca + rs * rs * cb * mu;
    }
    float* dg = k ? dgamma2 : dgamma1;
    float* db = k ? dbeta2 : dbeta1;
    for (int c = tid; c < g.c; c += GT) {
      double tg = 0, tb = 0;
      for (int nn = 0; nn < g.n; ++nn) {
        tb += cs[nn * g.c + c][0];
        tg += cs[nn * g.c + c][1];
      }
      if (dg) dg[c] = (accp ? dg[c] : 0.f) + (float)tg;
      if (db) db[c] = (accp ? db[c] : 0.f) + (float)tb;
    }
    __syncthreads();  // cs is rebuilt for the second set
  }
}

template <typename T, bool S2, bool ACC>
__global__ __launch_bounds__(GT) void gn_bwd2_apply(const T* __restrict__ da1, const T* __restrict__ da2,
                                                   const T* __restrict__ x, RedGeom g, const float* __restrict__ coef,
                                                   T* __restrict__ dx) {
  constexpr int VEC = 16 / sizeof(T);
  const int n = blockIdx.y;
  const int first = blockIdx.x * blockDim.x + threadIdx.x, stride = gridDim.x * blockDim.x;  // chn | blockDim
  const int j = first % g.chn;
  float sc1[VEC], sh1[VEC], al1[VEC], sc2[VEC], sh2[VEC], al2[VEC], bx[VEC], dd[VEC];
  const float* c1 = coef + (long long)n * 5 * g.c + j * VEC;
  const float* c2 = coef + ((long long)g.n + n) * 5 * g.c + j * VEC;
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    sc1[e] = c1[e];
    sh1[e] = c1[g.c + e];
    al1[e] = c1[2 * g.c + e];
    sc2[e] = c2[e];
    sh2[e] = c2[g.c + e];
    al2[e] = c2[2 * g.c + e];
    bx[e] = c1[3 * g.c + e] + c2[3 * g.c + e];
    dd[e] = c1[4 * g.c + e] + c2[4 * g.c + e];
  }
  const long long nb = (long long)n * g.v * g.c + j * VEC;
  const int vstep = stride / g.chn;
  Crd cr{}, s1{}, s2{};  // S2: coordinates of vox, the strides vstep and 2 vstep
  if constexpr (S2) {
    cr = crd_of(first / g.chn, g);
    s1 = crd_of(vstep, g);
    s2 = crd_of(2LL * vstep, g);
  }
  for (long long vox = first / g.chn; vox < g.v; vox += 2LL * vstep) {  // rounds of 2 voxels (up to 8 loads)
    float xv[2][VEC], d1[2][VEC], d2[2][VEC], o[2][VEC];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const long long vv = std::min(vox + (long long)u * vstep, g.v - 1);
      const long long off = nb + vv * g.c;
      load16<T>(x + off, xv[u]);
      load16<T>(da1 + off, d1[u]);
      if constexpr (S2)
        load_da2_crd<T>(da2, g, n, u ? crd_add(cr, s1, g) : cr, vox + (long long)u * vstep < g.v, j, d2[u]);
      else
        load_da2<T, S2>(da2, g, n, vv, j, off, d2[u]);
      if constexpr (ACC) load16<T>(dx + off, o[u]);  // (a template flag: no branch, no wait behind it)
    }
    if constexpr (S2) cr = crd_add(cr, s2, g);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        const float g1 = fmaf(xv[u][e], sc1[e], sh1[e]) > 0.f ? d1[u][e] : 0.f;
        const float g2 = fmaf(xv[u][e], sc2[e], sh2[e]) > 0.f ? d2[u][e] : 0.f;
        const float r = fmaf(al1[e], g1, fmaf(al2[e], g2, fmaf(bx[e], xv[u][e], dd[e])));
        o[u][e] = ACC ? o[u][e] + r : r;
      }
      if (vox + (long long)u * vstep < g.v) store16<T>(dx + nb + (vox + (long long)u * vstep) * g.c, o[u]);
    }
  }
}

// y = relu(x * scale[n,c] + shift[n,c]) materialised (8 channels per thread): used ahead of the implicit
// GEMM on the small deep-layer activations so its K loop carries no GroupNorm arithmetic.
// grid (blocks, n): one sample per grid row; the grid stride (blocks x 256 vectors) is a
// multiple of c / 8 (c <= 256 divides 2048), so a thread's 8-channel chunk and its GroupNorm coefficients are fixed
// for the whole loop (no per-element 64-bit index division or coefficient reloads)
template <typename T>
__global__ __launch_bounds__(256) void gn_apply_kernel(const T* __restrict__ x, T* __restrict__ y, int n, int c,
                                                       long long v, int groups, const float* __restrict__ st,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta) {
  constexpr int VEC = 8;
  const int c8 = c / VEC, nn = blockIdx.y;
  const long long per = v * c8;
  const long long i0 = blockIdx.x * 256LL + threadIdx.x, stride = (long long)gridDim.x * 256;
  f32x2 sc[4], sh[4];
  gn_coef8(st, gamma, beta, groups, c, nn, (int)(i0 % c8) * VEC, sc, sh);
  const T* xs = x + (long long)nn * per * VEC;
  T* ys = y + (long long)nn * per * VEC;
  for (long long i = i0; i < per; i += 4 * stride) {  // rounds of 4 vectors, clamped loads, guarded stores
    float a[4][VEC];
#pragma unroll
    for (int u = 0; u < 4; ++u) loadv<T, VEC>(xs + std::min(i + u * stride, i + (per - 1 - i) / stride * stride) * VEC, a[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
      for (int e = 0; e < VEC; ++e) a[u][e] = fmaxf(0.f, fmaf(a[u][e], sc[e >> 1][e & 1], sh[e >> 1][e & 1]));
      if (i + u * stride < per) storev<T, VEC>(ys + (i + u * stride) * VEC, a[u]);
    }
  }
}
}  // namespace u3d

using namespace u3d;

extern "C" long long u3d_gn_workspace_bytes(int n, int c, long long v) {
  long long nb = 0;
  for (int vec : {4, 8}) nb = std::max<long long>(nb, make_geom(n, c, v, 1, vec).nblk);
  return GN_CNT_BYTES + (long long)n * nb * 4 * c * 4 + 256 + 2LL * n * c * 5 * 4;  // room for u3d_gn_bwd2
}

static float* gn_coef_ptr(float* ws, const RedGeom& g) {
  return reinterpret_cast<float*>(reinterpret_cast<char*>(ws) + GN_CNT_BYTES +
                                  (((long long)g.n * g.nblk * 4 * g.c * 4 + 255) / 256) * 256);
}
static float* gn_part_ptr(float* ws) { return reinterpret_cast<float*>(reinterpret_cast<char*>(ws) + GN_CNT_BYTES); }

extern "C" int u3d_gn_stats(int dtype, const void* x, int n, int c, long long v, int groups, float* stats, float* ws,
                            u3d_stream_t stream) {
  U3D_REQUIRE(dtype == U3D_F32 || dtype == U3D_BF16, "gn_stats: bad dtype");
  U3D_REQUIRE(x && stats && ws && n > 0 && v > 0 && groups > 0 && c % groups == 0, "gn_stats: bad args");
  const int vec = dtype == U3D_BF16 ? 8 : 4;
  U3D_REQUIRE(c % vec == 0 && c / vec <= GT, "gn_stats: channels %d unsupported", c);
  U3D_REQUIRE(n * c <= GN_PAIRS_MAX, "gn_stats: n * c must be <= %d", GN_PAIRS_MAX);
  RedGeom g = make_geom(n, c, v, groups, vec);
  hipStream_t s = (hipStream_t)stream;
  unsigned* cnt = reinterpret_cast<unsigned*>(ws);
  if (dtype == U3D_BF16)
    hipLaunchKernelGGL(gn_stats_kernel<bf16>, dim3(g.nblk, n), dim3(GT), 0, s, (const bf16*)x, g, gn_part_ptr(ws), cnt,
                       stats);
  else
    hipLaunchKernelGGL(gn_stats_kernel<float>, dim3(g.nblk, n), dim3(GT), 0, s, (const float*)x, g, gn_part_ptr(ws),
                       cnt, stats);
  return check_launch("gn_stats");
}

extern "C" int u3d_gn_bwd(int dtype, const void* da, const void* x, int n, int c, long long v, int groups,
                          const float* stats, const float* gamma, const float* beta, void* dx, int accumulate,
                          float* dgamma, float* dbeta, int accumulate_params, float* ws, u3d_stream_t stream) {
  U3D_REQUIRE(dtype == U3D_F32 || dtype == U3D_BF16, "gn_bwd: bad dtype");
  U3D_REQUIRE(da && x && stats && gamma && beta && dx && ws && groups > 0 && c % groups == 0, "gn_bwd: bad args");
  const int vec = dtype == U3D_BF16 ? 8 : 4;
  U3D_REQUIRE(c % vec == 0 && c <= 256, "gn_bwd: channels %d unsupported", c);
  U3D_REQUIRE(n * c <= GN_PAIRS_MAX, "gn_bwd: n * c must be <= %d", GN_PAIRS_MAX);
  RedGeom g = make_geom(n, c, v, groups, vec);
  hipStream_t s = (hipStream_t)stream;
  unsigned* cnt = reinterpret_cast<unsigned*>(ws) + 1;
  float* coef = gn_coef_ptr(ws, g);
  const long long nvec = v * g.chn;  // per sample
  const int athr = GT / g.chn * g.chn;  // a multiple of the chunks per voxel: each thread keeps one chunk
  const int ablk = (int)std::min<long long>(std::max(1, 4096 / n), (nvec + athr - 1) / athr);
  if (dtype == U3D_BF16) {
    hipLaunchKernelGGL(gn_bwd_partial<bf16>, dim3(g.nblk, n), dim3(GT), 0, s, (const bf16*)da, (const bf16*)x, g, stats,
                       gamma, beta, gn_part_ptr(ws), cnt, coef, dgamma, dbeta, accumulate_params);
    launch_gn_bwd_apply<bf16>(dim3(ablk, n), athr, s, (const bf16*)da, (const bf16*)x, g, coef, (bf16*)dx, accumulate);
  } else {
    hipLaunchKernelGGL(gn_bwd_partial<float>, dim3(g.nblk, n), dim3(GT), 0, s, (const float*)da, (const float*)x, g,
                       stats, gamma, beta, gn_part_ptr(ws), cnt, coef, dgamma, dbeta, accumulate_params);
    launch_gn_bwd_apply<float>(dim3(ablk, n), athr, s, (const float*)da, (const float*)x, g, coef, (float*)dx,
                               accumulate);
  }
  return check_launch("gn_bwd");
}

extern "C" int u3d_gn_bwd_parts(const void* da, const void* x, int n, int c, long long v, int groups, const float* stats,
                                const float* gamma, const float* beta, const float* parts, int nparts, void* dx,
                                int accumulate, float* dgamma, float* dbeta, int accumulate_params, float* ws,
                                u3d_stream_t stream) {
  U3D_REQUIRE(da && x && stats && gamma && beta && parts && nparts >= 1 && dx && ws && groups > 0 && c % groups == 0,
              "gn_bwd_parts: bad args");
  U3D_REQUIRE(c % 8 == 0 && c <= 256 && n * c <= GN_PAIRS_MAX, "gn_bwd_parts: channels %d unsupported", c);
  RedGeom g = make_geom(n, c, v, groups, 8);
  hipStream_t s = (hipStream_t)stream;
  float* coef = gn_coef_ptr(ws, g);
  const long long nvec = v * g.chn;
  const int athr = GT / g.chn * g.chn;
  const int ablk = (int)std::min<long long>(std::max(1, 4096 / n), (nvec + athr - 1) / athr);
  hipLaunchKernelGGL(gn_bwd_parts_finalize, dim3(1), dim3(GPF), 0, s, parts, nparts, g, stats, gamma, beta, coef, dgamma,
                     dbeta, accumulate_params);
  launch_gn_bwd_apply<bf16>(dim3(ablk, n), athr, s, (const bf16*)da, (const bf16*)x, g, coef, (bf16*)dx, accumulate);
  return check_launch("gn_bwd_parts");
}

// Round 5: the apply pass of the GroupNorm backward alone, from apply coefficients coef[n][5][c] a producer already
// formed (u3d_conv_small_dgrad_gn: partials and finalize inside the data-gradient launch). bf16.
extern "C" int u3d_gn_bwd_apply_coef(const void* da, const void* x, int n, int c, long long v, int groups,
                                     const float* coef, void* dx, int accumulate, u3d_stream_t stream) {
  U3D_REQUIRE(da && x && coef && dx && n >= 1 && groups > 0 && c % groups == 0, "gn_bwd_apply_coef: bad args");
  U3D_REQUIRE(c % 8 == 0 && c <= 256, "gn_bwd_apply_coef: channels %d unsupported", c);
  RedGeom g = make_geom(n, c, v, groups, 8);
  const long long nvec = v * g.chn;
  const int athr = GT / g.chn * g.chn;
  const int ablk = (int)std::min<long long>(std::max(1, 4096 / n), (nvec + athr - 1) / athr);
  launch_gn_bwd_apply<bf16>(dim3(ablk, n), athr, (hipStream_t)stream, (const bf16*)da, (const bf16*)x, g, coef,
                            (bf16*)dx, accumulate);
  return check_launch("gn_bwd_apply_coef");
}

extern "C" int u3d_gn_apply(int dtype, const void* x, int n, int c, long long v, int groups, const float* stats,
                            const float* gamma, const float* beta, void* y, u3d_stream_t stream) {
  U3D_REQUIRE(dtype == U3D_F32 || dtype == U3D_BF16, "gn_apply: bad dtype");
  U3D_REQUIRE(x && y && stats && gamma && beta && n >= 1 && c % 8 == 0 && groups > 0 && c % groups == 0,
              "gn_apply: bad args (c %% 8 == 0)");
  U3D_REQUIRE(c <= 256, "gn_apply: channels %d > 256", c);
  const long long per = v * (c / 8);
  const dim3 grid((unsigned)std::max<long long>(1, std::min<long long>(std::max(1, 2048 / n), (per + 1023) / 1024)),
                  (unsigned)n);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == U3D_BF16)
    hipLaunchKernelGGL(gn_apply_kernel<bf16>, grid, dim3(256), 0, s, (const bf16*)x, (bf16*)y, n, c, v, groups,
                       stats, gamma, beta);
  else
    hipLaunchKernelGGL(gn_apply_kernel<float>, grid, dim3(256), 0, s, (const float*)x, (float*)y, n, c, v,
                       groups, stats, gamma, beta);
  return check_launch("gn_apply_kernel");
}

#ifndef U3D_GN2_APV
#define U3D_GN2_APV 16
#endif
template <bool S2>
static int gn_bwd2_launch(int dtype, const void* da1, const void* da2, const void* x, int n, int c, long long v,
                          int fh, int fw, int groups, const float* stats, const float* gamma1, const float* beta1,
                          const float* gamma2, const float* beta2, void* dx, int accumulate, float* dgamma1,
                          float* dbeta1, float* dgamma2, float* dbeta2, int accumulate_params, float* ws,
                          u3d_stream_t stream) {
  U3D_REQUIRE(dtype == U3D_F32 || dtype == U3D_BF16, "gn_bwd2: bad dtype");
  U3D_REQUIRE(da1 && da2 && x && stats && gamma1 && beta1 && gamma2 && beta2 && dx && ws && groups > 0 &&
              c % groups == 0, "gn_bwd2: bad args");
  const int vec = dtype == U3D_BF16 ? 8 : 4;
  U3D_REQUIRE(c % vec == 0 && c <= 256, "gn_bwd2: channels %d unsupported", c);
  U3D_REQUIRE(n * c <= GN_PAIRS_MAX, "gn_bwd2: n * c must be <= %d", GN_PAIRS_MAX);
  RedGeom g = make_geom(n, c, v, groups, vec);
  if (S2) {
    U3D_REQUIRE(v < (1LL << 24) && fh > 0 && fw > 0 && v % ((long long)fh * fw) == 0, "gn_bwd2_s2: bad dims");
    const int fd = (int)(v / ((long long)fh * fw));
    g.fh = fh; g.fw = fw;
    g.ch = (fh - 1) / 2 + 1; g.cw = (fw - 1) / 2 + 1;
    g.cv = (long long)((fd - 1) / 2 + 1) * g.ch * g.cw;
    U3D_REQUIRE(n * g.cv * c * (dtype == U3D_BF16 ? 2 : 4) < (1LL << 31) - 64,
                "gn_bwd2_s2: compact gradient beyond the 2 GiB buffer-offset range");
    g.rhw = 1.f / (float)((long long)fh * fw);
    g.rfw = 1.f / (float)fw;
  }
  hipStream_t s = (hipStream_t)stream;
  unsigned* cnt = reinterpret_cast<unsigned*>(ws) + 2;
  float* coef = gn_coef_ptr(ws, g);
  const long long nvec = v * g.chn;
  const int athr = GT / g.chn * g.chn;
  // U3D_GN2_APV vectors per apply thread where that still leaves >= 200 blocks (its 2 x 5 x VEC coefficient loads
  // amortised over more voxels: 2 x 96^3 x 32 160 -> 155 us, 48^3 48.2 -> 46.3), else 4 (24^3: 27 -> 37 us with 16)
  const long long apv = n * ((nvec + U3D_GN2_APV * athr - 1) / (U3D_GN2_APV * athr)) >= 200 ? U3D_GN2_APV : 4;
  const int ablk = (int)std::min<long long>(std::max(1, 4096 / n), (nvec + apv * athr - 1) / (apv * athr));
  if (dtype == U3D_BF16) {
    hipLaunchKernelGGL((gn_bwd2_partial<bf16, S2>), dim3(g.nblk, n), dim3(GT), 0, s, (const bf16*)da1,
                       (const bf16*)da2, (const bf16*)x, g, stats, gamma1, beta1, gamma2, beta2, gn_part_ptr(ws), cnt,
                       coef, dgamma1, dbeta1, dgamma2, dbeta2, accumulate_params);
    if (accumulate)
      hipLaunchKernelGGL((gn_bwd2_apply<bf16, S2, true>), dim3(ablk, n), dim3(athr), 0, s, (const bf16*)da1,
                         (const bf16*)da2, (const bf16*)x, g, coef, (bf16*)dx);
    else
      hipLaunchKernelGGL((gn_bwd2_apply<bf16, S2, false>), dim3(ablk, n), dim3(athr), 0, s, (const bf16*)da1,
                         (const bf16*)da2, (const bf16*)x, g, coef, (bf16*)dx);
  } else {
    hipLaunchKernelGGL((gn_bwd2_partial<float, S2>), dim3(g.nblk, n), dim3(GT), 0, s, (const float*)da1,
                       (const float*)da2, (const float*)x, g, stats, gamma1, beta1, gamma2, beta2, gn_part_ptr(ws),
                       cnt, coef, dgamma1, dbeta1, dgamma2, dbeta2, accumulate_params);
    if (accumulate)
      hipLaunchKernelGGL((gn_bwd2_apply<float, S2, true>), dim3(ablk, n), dim3(athr), 0, s, (const float*)da1,
                         (const float*)da2, (const float*)x, g, coef, (float*)dx);
    else
      hipLaunchKernelGGL((gn_bwd2_apply<float, S2, false>), dim3(ablk, n), dim3(athr), 0, s, (const float*)da1,
                         (const float*)da2, (const float*)x, g, coef, (float*)dx);
  }
  return check_launch("gn_bwd2");
}

extern "C" int u3d_gn_bwd2(int dtype, const void* da1, const void* da2, const void* x, int n, int c, long long v,
                           int groups, const float* stats, const float* gamma1, const float* beta1,
                           const float* gamma2, const float* beta2, void* dx, int accumulate, float* dgamma1,
                           float* dbeta1, float* dgamma2, float* dbeta2, int accumulate_params, float* ws,
                           u3d_stream_t stream) {
  return gn_bwd2_launch<false>(dtype, da1, da2, x, n, c, v, 0, 0, groups, stats, gamma1, beta1, gamma2, beta2, dx,
                               accumulate, dgamma1, dbeta1, dgamma2, dbeta2, accumulate_params, ws, stream);
}

extern "C" int u3d_gn_bwd2_s2(int dtype, const void* da1, const void* da2c, const void* x, int n, int c, int d, int h,
                              int w, int groups, const float* stats, const float* gamma1, const float* beta1,
                              const float* gamma2, const float* beta2, void* dx, int accumulate, float* dgamma1,
                              float* dbeta1, float* dgamma2, float* dbeta2, int accumulate_params, float* ws,
                              u3d_stream_t stream) {
  return gn_bwd2_launch<true>(dtype, da1, da2c, x, n, c, (long long)d * h * w, h, w, groups, stats, gamma1, beta1,
                              gamma2, beta2, dx, accumulate, dgamma1, dbeta1, dgamma2, dbeta2, accumulate_params, ws,
                              stream);
}
