// Diagnostic hooks of the persistent ring kernels, in one place (never active in the product build).
//
// A -DU3D_STAMPS build (tools/build_variant.sh) lets a ring kernel record s_memtime / s_memrealtime stamps and
// per-phase cycle sums into a buffer of its own (a __device__ array of its translation unit, read back with
// u3d_diag_*_stamps): the clock the chip holds inside the kernel (MI355X_MICROARCH.md, DVFS item 6) and where a
// persistent walk spends its cycles. Nothing else reads the buffer and no output depends on it. A -DU3D_PRIO build
// raises the static wave priority of the second-dispatched half of a workgroup (MI355X_MICROARCH.md, two waves per
// SIMD, item 4). Without either flag every hook below is an empty inline function and the kernels compile to the same
// code as with no hook at all.
#pragma once
#include "common.h"

namespace u3d {

#ifdef U3D_STAMPS
__device__ __forceinline__ unsigned long long stamp_clk() {
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long t = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
__device__ __forceinline__ unsigned long long stamp_real() { return __builtin_amdgcn_s_memrealtime(); }

// Per wave: [t0, t1 (s_memtime), r0, r1 (s_memrealtime), phase 0, phase 1, phase 2 cycles, steps | compute steps << 32]
struct PhaseStamps {
  unsigned long long t0, r0, p0, p1, p2, n, mark;
  __device__ __forceinline__ void begin() {
    t0 = stamp_clk();
    r0 = stamp_real();
    p0 = p1 = p2 = n = 0;
    mark = t0;
  }
  __device__ __forceinline__ void mark_now() { mark = stamp_clk(); }
  // cycles since the last mark / lap into phase `ph` (0, 1 or 2)
  __device__ __forceinline__ void lap(int ph) {
    const unsigned long long t = stamp_clk(), dt = t - mark;
    if (ph == 0) p0 += dt; else if (ph == 1) p1 += dt; else p2 += dt;
    mark = t;
  }
  __device__ __forceinline__ void step(bool compute) { n += 1ull + (compute ? (1ull << 32) : 0ull); }
  // lets a phase include the wait for the loads it staged (stamps builds only)
  __device__ __forceinline__ void settle(bool pending) {
    if (pending) __builtin_amdgcn_s_waitcnt(0);
  }
  __device__ __forceinline__ void end(unsigned long long* buf, int wg, int wave, int lane) {
    const unsigned long long t1 = stamp_clk(), r1 = stamp_real();
    if (lane == 0) {
      unsigned long long* o = buf + ((long long)wg * 8 + wave) * 8;
      o[0] = t0; o[1] = t1; o[2] = r0; o[3] = r1; o[4] = p0; o[5] = p1; o[6] = p2; o[7] = n;
    }
  }
};
// Up to 8 s_memtime marks of one workgroup's tail (after its main loop), written by thread 0 when the object leaves
// scope (any return path), with the s_memrealtime at that point: buf[wg * 16 + 0..7] marks (0 = not reached),
// buf[wg * 16 + 8] the real time at exit.
struct TailStamps {
  unsigned long long t[8];
  unsigned long long* buf;
  int wg;
  bool writer;
  __device__ __forceinline__ TailStamps(unsigned long long* b, int w, bool wr) : buf(b), wg(w), writer(wr) {
#pragma unroll
    for (int i = 1; i < 8; ++i) t[i] = 0;
    t[0] = stamp_clk();
  }
  template <int K>
  __device__ __forceinline__ void mark() { t[K] = stamp_clk(); }
  __device__ __forceinline__ ~TailStamps() {
    const unsigned long long re = stamp_real();
    if (writer) {
#pragma unroll
      for (int i = 0; i < 8; ++i) buf[(long long)wg * 16 + i] = t[i];
      buf[(long long)wg * 16 + 8] = re;
    }
  }
};
// the buffer of WGS workgroups x 8 waves and its host reader
#define U3D_STAMP_BUFFER(NAME, WGS, READER)                                                                   \
  __device__ unsigned long long NAME[(WGS) * 8 * 8];                                                          \
  extern "C" int READER(void* out, long long nbytes) {                                                        \
    U3D_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(NAME), std::min<long long>(nbytes, sizeof(NAME))));           \
    return 0;                                                                                                 \
  }
#else
struct PhaseStamps {
  __device__ __forceinline__ void begin() {}
  __device__ __forceinline__ void mark_now() {}
  __device__ __forceinline__ void lap(int) {}
  __device__ __forceinline__ void step(bool) {}
  __device__ __forceinline__ void settle(bool) {}
  __device__ __forceinline__ void end(unsigned long long*, int, int, int) {}
};
struct TailStamps {
  __device__ __forceinline__ TailStamps(unsigned long long*, int, bool) {}
  template <int K>
  __device__ __forceinline__ void mark() {}
};
#define U3D_STAMP_BUFFER(NAME, WGS, READER) static constexpr unsigned long long* NAME = nullptr;
#endif

// static priority 1 for waves 4..7 of an 8-wave workgroup (-DU3D_PRIO builds)
__device__ __forceinline__ void diag_prio_second_half(int wave) {
#ifdef U3D_PRIO
  if (__builtin_amdgcn_readfirstlane(wave) >= 4) __builtin_amdgcn_s_setprio(1);
#else
  (void)wave;
#endif
}

}  // namespace u3d
