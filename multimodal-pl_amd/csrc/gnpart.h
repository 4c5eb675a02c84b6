// GroupNorm(G) statistics accumulated by the kernel that PRODUCES the activation (an epilogue), so the next
// GroupNorm (NoBottleneck gn1 / gn2, downsample GN, fusion / head GN: unet3D.py:44-53) needs no statistics pass.
//
// Contract for a producer: each thread owns one fixed 8-channel chunk j = tid % chn (chn = C / 8 divides the block
// size) and accumulates, in fp64 over the elements it writes, the (sum, sum of squares) of the GS = max(1, 8 / cpg)
// groups that chunk covers (slot s = channels [s * cpg, (s + 1) * cpg) of the chunk). gn_part_block() reduces them
// over the block in a fixed order (xor shuffles inside a wave, waves in index order through LDS) and writes the
// block's G pairs with write-through stores; gn_part_last() lets the last block of the launch combine every block
// of every sample in a fixed order (fp64) into stats [n][G] = (mean, rstd), eps 1e-5 (biased variance, as
// nn.GroupNorm). Deterministic whatever the block timing. Sums are unshifted but fp64: the cancellation in
// E[x^2] - mean^2 costs ~1e-16 (1 + mean^2 / var) relative.
#pragma once
#include "common.h"

namespace u3d {

template <int GS>
__device__ __forceinline__ void gn_part_add8(double (&acc)[GS][2], const float (&v)[8], int cpg) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int s = GS == 1 ? 0 : e / cpg;
    const double t = v[e];
    acc[s][0] += t;
    acc[s][1] = fma(t, t, acc[s][1]);
  }
}

// Block partials -> part[blk][G][2] (fp64, write-through). NT threads, chn = C / 8 chunks (power of two <= 64).
template <int GS, int NT>
__device__ __forceinline__ void gn_part_block(double (&acc)[GS][2], int chn, int cpg, int G, double* __restrict__ part) {
  __shared__ double red[NT / 64][64][GS][2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int s = 0; s < GS; ++s)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      double v = acc[s][q];
      for (int o = chn; o < 64; o <<= 1) v += __shfl_xor(v, o);
      if (lane < chn) red[wave][lane][s][q] = v;
    }
  __syncthreads();
  if (tid < G) {
    const int g = tid;
    // group g: chunks j0 .. j0 + max(1, cpg / 8) - 1, slot s (cpg < 8) or 0
    const int j0 = g * cpg / 8, nj = cpg >= 8 ? cpg / 8 : 1, s = cpg >= 8 ? 0 : (g * cpg % 8) / cpg;
    double s1 = 0, s2 = 0;
    for (int w = 0; w < NT / 64; ++w)
      for (int j = j0; j < j0 + nj; ++j) {
        s1 += red[w][j][GS == 1 ? 0 : s][0];
        s2 += red[w][j][GS == 1 ? 0 : s][1];
      }
    __hip_atomic_store(part + g * 2, s1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(part + g * 2 + 1, s2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// After every block wrote its partials: true in the last block to arrive (the counter is reset for the next
// launch). Partials were written through (sc1); each wave drains its stores before the barrier.
__device__ __forceinline__ bool gn_part_is_last(unsigned* cnt, unsigned total) {
  __shared__ unsigned s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) s_last = atomicAdd(cnt, 1u) == total - 1;
  __syncthreads();
  if (s_last && threadIdx.x == 0) atomicExch(cnt, 0u);
  return s_last;
}

// Last block: stats[n][G] from part[n][nblk][G][2]; M = elements per group. NT threads: pair p = (n, g) per
// thread slice, slices of the block range combined in index order.
template <int NT>
__device__ __forceinline__ void gn_part_finalize(const double* __restrict__ part, int n, int nblk, int G, double M,
                                                 float* __restrict__ stats) {
  __shared__ double fin[NT][2];
  const int tid = threadIdx.x, npairs = n * G;
  const int spl = npairs >= NT ? 1 : NT / npairs;
  for (int p0 = 0; p0 < npairs; p0 += NT) {
    const int p = p0 + tid % min(npairs, NT), sl = tid / min(npairs, NT);
    double s1 = 0, s2 = 0;
    if (p < npairs && sl < spl) {
      const int nn = p / G, g = p % G;
      const int b0 = (int)((long long)nblk * sl / spl), b1 = (int)((long long)nblk * (sl + 1) / spl);
      const double* q0 = part + ((long long)nn * nblk * G + g) * 2;
      int b = b0;
      for (; b + 8 <= b1; b += 8) {  // 16 independent loads in flight, then the adds in block order
        double v[8][2];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          v[u][0] = __hip_atomic_load(q0 + (long long)(b + u) * G * 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          v[u][1] = __hip_atomic_load(q0 + (long long)(b + u) * G * 2 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          s1 += v[u][0];
          s2 += v[u][1];
        }
      }
      for (; b < b1; ++b) {
        s1 += __hip_atomic_load(q0 + (long long)b * G * 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s2 += __hip_atomic_load(q0 + (long long)b * G * 2 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    fin[tid][0] = s1;
    fin[tid][1] = s2;
    __syncthreads();
    if (tid < min(npairs, NT) && p < npairs) {
      double t1 = 0, t2 = 0;
      for (int k = 0; k < spl; ++k) {
        t1 += fin[k * min(npairs, NT) + tid][0];
        t2 += fin[k * min(npairs, NT) + tid][1];
      }
      const double mean = t1 / M;
      double var = t2 / M - mean * mean;
      if (var < 0) var = 0;
      stats[p * 2] = (float)mean;
      stats[p * 2 + 1] = (float)(1.0 / sqrt(var + 1e-5));
    }
    __syncthreads();
  }
}

}  // namespace u3d
