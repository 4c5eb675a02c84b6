// 3^3 stride-2 convolution, forward, bf16: cin = 32 -> cout = 64 with the GroupNorm + ReLU prologue (layer1.0.conv1 of
// the 96^3 U-Net: NoBottleneck's first conv of a downsampling stage, unet3D.py:45 / :56-73), as a persistent walk over
// INPUT planes (round 5). The implicit GEMM it replaces applied the GroupNorm to every gathered
// element (27 / 8 times per input element) and was issue-bound at ~11% of the MFMA peak.
//
//   * a workgroup owns a contiguous range of output planes in (column, z) order, a column being (n, 8-row oh tile,
//     16-voxel ow tile); output plane z reads input planes 2z-1, 2z, 2z+1, so walking down z the workgroup stages every
//     input plane of the column's halo (17 x 33 rows x 32 channels) ONCE, with GroupNorm + ReLU applied once per element,
//     and each step computes everything that one staged plane contributes: an even plane 2z the taps kd = 1 of output z,
//     an odd plane 2z+1 the taps kd = 2 of output z (which then completes) and kd = 0 of output z+1 — two LDS slots
//     (the plane computed, the plane written), one barrier per input plane;
//   * the staged rows of an input h-row are split by column parity (17 even, 16 odd), so the 16 output voxels of a
//     voxel block read 16 consecutive rows for every tap (conflict-free ds_read_b128), and an odd plane's B fragment
//     serves two taps (kd = 0 and kd = 2);
//   * the weight fragments of the wave's 16-channel output block: the 18 taps kd = 0, 2 (odd planes) in registers, the 9
//     taps kd = 1 (even planes) in LDS beside the two plane slots (all 27 in registers spilled);
//     v_mfma_f32_16x16x32_bf16 with A = weights (rows = output channels), B = staged input rows (columns = voxels): a lane's 4 accumulators per voxel block are 4 consecutive output channels = one GroupNorm(16) group of
//     the 64-channel output, whose (sum, sum of squares) the epilogue accumulates for the next GroupNorm's statistics,
//     finalized by the workgroup that arrives last (no statistics pass).
#include "common.h"
#include "diag.h"

namespace u3d {
namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;

constexpr int S2_OH = 8, S2_OW = 16;                      // output tile (h, w) of a column
constexpr int S2_IH = 2 * S2_OH + 1;                      // 17 input h-rows
constexpr int S2_NE = S2_OW + 1, S2_RPH = 2 * S2_OW + 1;  // 17 even + 16 odd input columns = 33 rows per h-row
constexpr int S2_NR = S2_IH * S2_RPH;                     // 561 staged rows per plane
constexpr int S2_PS = (S2_NR * 16 + 255) / 256 * 256;     // chunk-plane stride (8 channels of every row)
constexpr int S2_SS = 4 * S2_PS;                          // LDS slot (one input plane, 32 channels)
constexpr int S2_NT = 512;
constexpr int S2_LD = (S2_NR * 4 + S2_NT - 1) / S2_NT;    // 5 staged 16-B pieces per thread and plane

struct S2Geom {
  int n, d, h, w;        // input volume
  int od, oh, ow;        // output volume
  int nbh, nbw;          // output tiles per plane
  long long pps;         // output tile-planes per sample = nbh * nbw * od
  int per, wps;          // output tile-planes per workgroup, workgroups per sample (never straddling samples)
  int xbytes;            // bytes of x (< 2^31: buffer offsets)
  int gn_groups;
  float* spart;          // [n][wps][16][2] statistics partials (nullptr: no statistics)
  float* stats;          // [n][16][2] (mean, rstd)
  unsigned* cnt;         // zeroed arrival counter
};

struct S2Plane {
  int n, oh0, ow0, p, zf, zl;
  bool valid;
};

// the workgroup's output range [o, o_end) as runs (column, zf..zl-1); each run stages input planes 2 zf - 1 .. 2 zl - 1
struct S2Walk {
  long long o_next, o_end;
  int p, plast, zf, zl, cn, ch0, cw0;
  bool done;
  __device__ void start_run(const S2Geom& g) {
    if (o_next >= o_end) {
      done = true;
      return;
    }
    const int col = (int)(o_next / g.od);
    zf = (int)(o_next - (long long)col * g.od);
    zl = (int)min<long long>(g.od, zf + (o_end - o_next));
    o_next += zl - zf;
    p = 2 * zf - 1;
    plast = 2 * zl - 1;
    int c = col;
    const int bw_ = c % g.nbw;
    c /= g.nbw;
    const int bh_ = c % g.nbh;
    cn = c / g.nbh;
    ch0 = bh_ * S2_OH;
    cw0 = bw_ * S2_OW;
  }
  __device__ S2Plane next(const S2Geom& g) {
    S2Plane q{};
    if (!done && p > plast) start_run(g);
    if (done) return q;
    q.n = cn;
    q.oh0 = ch0;
    q.ow0 = cw0;
    q.p = p;
    q.zf = zf;
    q.zl = zl;
    q.valid = true;
    ++p;
    return q;
  }
};

}  // namespace

// -DU3D_STAMPS phases (diag.h): 0 the staged plane's GN + LDS write (incl. its loads' wait), 1 compute, 2 the barrier
U3D_STAMP_BUFFER(s2_stamps, 1024, u3d_diag_s2_stamps)

__global__ __launch_bounds__(S2_NT, 1) void conv_s2_ring_kernel(const bf16* __restrict__ x, const bf16* __restrict__ wpk,
                                                               bf16* __restrict__ y, const float* __restrict__ gstat,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ beta, S2Geom g) {
  // LDS: two input-plane slots, the kd = 1 taps' weights (chunk-planar: plane c = 8 input channels of every (tap, co)
  // row, 16 B per row, so a fragment's 16 lanes read 256 contiguous bytes), junk for the staging lanes past the plane
  constexpr int WPL = 9 * 64 * 16;  // weight chunk-plane stride (a multiple of 256 B)
  __shared__ __attribute__((aligned(16))) char smem[2 * S2_SS + 4 * WPL + 1024];
  char* const ring = smem;
  char* const wts = smem + 2 * S2_SS;
  char* const junk = wts + 4 * WPL;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  PhaseStamps ps;  // (from kernel entry: "other" = the weight prologue, the load issue and the walk)
  ps.begin();
  const int l16 = lane & 15, q4 = lane >> 4;
  const int rg = wave >> 2, cb = wave & 3;  // output rows 4 rg .. 4 rg + 3 of the tile, channels 16 cb .. 16 cb + 15
  const int ch = (tid >> 3) & 3, srow = (tid & 7) + 8 * (tid >> 5);  // staging: 8 consecutive rows of one chunk plane

  // XCD-aware range order (as the stride-1 ring): XCD x runs a contiguous eighth of the ranges
  int bid = blockIdx.x;
  {
    const int nwg = gridDim.x, q = nwg >> 3, rr = nwg & 7, xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
    bid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + loc;
  }
  const int smp = bid / g.wps, jw = bid - smp * g.wps;
  S2Walk walk{};
  walk.o_next = (long long)smp * g.pps + (long long)jw * g.per;
  walk.o_end = min((long long)(smp + 1) * g.pps, walk.o_next + g.per);
  walk.done = false;
  walk.p = 1;
  walk.plast = 0;  // forces start_run on the first next()

  // the wave's weight fragments W[t][co = 16 cb + l16][ci = 8 q4 .. 8 q4 + 7] (pack [27][64][32]): the 18 taps of kd = 0
  // and kd = 2 (the odd planes' MFMAs) in registers, the 9 of kd = 1 (even planes) in LDS — all 27 in registers spilled
  bf16x8 wreg[18];
#pragma unroll
  for (int j = 0; j < 18; ++j) {
    const int t = j < 9 ? j : j + 9;
    wreg[j] = *reinterpret_cast<const bf16x8*>(wpk + ((t * 64 + 16 * cb + l16) * 32 + 8 * q4));
  }
  {  // kd = 1 taps: row (t - 9) * 64 + co, chunk plane c; all of a thread's loads issued before its stores
    constexpr int NWL = (9 * 64 * 4 + S2_NT - 1) / S2_NT;
    u32x4 wl[NWL];
#pragma unroll
    for (int k = 0; k < NWL; ++k) {
      const int i = tid + k * S2_NT;
      if (i < 9 * 64 * 4) wl[k] = *reinterpret_cast<const u32x4*>(wpk + ((9 * 64 + (i >> 2)) * 32 + (i & 3) * 8));
    }
#pragma unroll
    for (int k = 0; k < NWL; ++k) {
      const int i = tid + k * S2_NT;
      if (i < 9 * 64 * 4) *reinterpret_cast<u32x4*>(wts + (i & 3) * WPL + (i >> 2) * 16) = wl[k];
    }
  }
  const char* const wb1 = wts + q4 * WPL + (16 * cb + l16) * 16;  // + (t - 9) * 64 * 16

  // staging: piece i = halo row srow + 128 i (row -> h-row hr = row / 33, column slot cs = row % 33: even input column
  // 2 cs for cs < 17, odd 2 (cs - 17) + 1 after); per-lane byte offsets relative to the column's plane base, hoisted
  const auto xrs = __builtin_amdgcn_make_buffer_rsrc((void*)x, 0, g.xbytes, 0x00020000);
  int plo[S2_LD], phr[S2_LD], pwc[S2_LD];
#pragma unroll
  for (int i = 0; i < S2_LD; ++i) {
    const int row = srow + i * (S2_NT / 4);
    const int hr = row / S2_RPH, cs = row - hr * S2_RPH;
    phr[i] = hr;
    pwc[i] = cs < S2_NE ? 2 * cs : 2 * (cs - S2_NE) + 1;
    plo[i] = ((hr * g.w + pwc[i]) * 32 + ch * 8) * 2;
  }
  unsigned pin = 0;
  int col_h0 = -1, col_w0 = -1;
  u32x4 v[S2_LD];
  unsigned vm = 0;
  auto load_plane = [&](const S2Plane& p) {
    if (p.valid && (p.oh0 != col_h0 || p.ow0 != col_w0)) {  // uniform: once per run
      col_h0 = p.oh0;
      col_w0 = p.ow0;
      pin = 0;
#pragma unroll
      for (int i = 0; i < S2_LD; ++i) {
        const int row = srow + i * (S2_NT / 4);
        const bool ok = row < S2_NR && (unsigned)(2 * p.oh0 - 1 + phr[i]) < (unsigned)g.h &&
                        (unsigned)(2 * p.ow0 - 1 + pwc[i]) < (unsigned)g.w;
        pin |= (ok ? 1u : 0u) << i;
      }
    }
    const bool pv = p.valid && (unsigned)p.p < (unsigned)g.d;  // (p = -1 / d: zero padding)
    const int base = (((p.n * g.d + p.p) * g.h + 2 * p.oh0 - 1) * g.w + 2 * p.ow0 - 1) * 64;
    vm = 0;
#pragma unroll
    for (int i = 0; i < S2_LD; ++i) {
      const bool ok = pv && ((pin >> i) & 1u);
      const unsigned off = ok ? (unsigned)(base + plo[i]) : 0xFFFFFFF0u;
      v[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0));
      vm |= (ok ? 1u : 0u) << i;
    }
  };
  f32x2 sc[4], sh[4];
  int gn_n = -1;
  auto write_plane = [&](const S2Plane& p, int slot) {
    if (p.n != gn_n) {  // uniform
      gn_n = p.n;
      gn_coef8(gstat, gamma, beta, g.gn_groups, 32, p.n, ch * 8, sc, sh);
    }
#pragma unroll
    for (int i = 0; i < S2_LD; ++i) {
      const int row = srow + i * (S2_NT / 4);
      u32x4 val = gn_relu8(v[i], sc, sh);
      if (!((vm >> i) & 1u)) val = u32x4{0u, 0u, 0u, 0u};  // padding stays zero after the prologue
      char* dst = row < S2_NR ? ring + slot * S2_SS + ch * S2_PS + row * 16 : junk + lane * 16;
      *reinterpret_cast<u32x4*>(dst) = val;
    }
  };

  f32x4 accA[4], accB[4];  // output finishing next (accA) / the one after it (accB), per voxel block
#pragma unroll
  for (int i = 0; i < 4; ++i) accA[i] = accB[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float gs = 0.f, gq = 0.f;  // statistics of group 4 cb + q4 (this lane's 4 channels)

  auto epilogue = [&](const S2Plane& p, int z) {
    const int c = 16 * cb + 4 * q4;
#pragma unroll
    for (int vb = 0; vb < 4; ++vb) {
      const int oh = p.oh0 + 4 * rg + vb, ow = p.ow0 + l16;
      const bool ok = oh < g.oh && ow < g.ow;
      const uint32_t lo = pack_bf16x2(accA[vb][0], accA[vb][1]), hi = pack_bf16x2(accA[vb][2], accA[vb][3]);
      if (g.spart) {
        const float a0 = __uint_as_float(lo << 16), a1 = __uint_as_float(lo & 0xffff0000u);
        const float a2 = __uint_as_float(hi << 16), a3 = __uint_as_float(hi & 0xffff0000u);
        gs += ok ? (a0 + a1) + (a2 + a3) : 0.f;
        gq += ok ? (a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3) : 0.f;
      }
      if (ok) {
        const long long o = ((((long long)p.n * g.od + z) * g.oh + oh) * g.ow + ow) * 64 + c;
        *reinterpret_cast<uint2*>(y + o) = uint2{lo, hi};
      }
    }
  };

  // everything staged input plane p (LDS slot `slot`) contributes; B fragment of tap (kh, kw) and voxel block vb:
  // row (2 (4 rg + vb) + kh) * 33 + (kw = 0: 0, 1: 17, 2: 1) + l16 of chunk plane q4
  auto compute = [&](const S2Plane& p, int slot) {
    const bool odd = (p.p & 1) != 0;
    const int zlo = odd ? (p.p - 1) >> 1 : p.p >> 1;  // odd: finishing output (kd = 2); even: output p / 2 (kd = 1)
    const bool has2 = odd && zlo >= p.zf, has0 = odd && zlo + 1 < p.zl;
    const char* bb = ring + slot * S2_SS + q4 * S2_PS + ((8 * rg) * S2_RPH + l16) * 16;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int cofs = kw == 0 ? 0 : (kw == 1 ? S2_NE : 1);
        bf16x8 bf[4];
#pragma unroll
        for (int vb = 0; vb < 4; ++vb)
          bf[vb] = *reinterpret_cast<const bf16x8*>(bb + ((2 * vb + kh) * S2_RPH + cofs) * 16);
        const int t = kh * 3 + kw;
        if (odd) {
          if (has2)
#pragma unroll
            for (int vb = 0; vb < 4; ++vb) accA[vb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wreg[9 + t], bf[vb], accA[vb], 0, 0, 0);
          if (has0)
#pragma unroll
            for (int vb = 0; vb < 4; ++vb) accB[vb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wreg[t], bf[vb], accB[vb], 0, 0, 0);
        } else {
          const bf16x8 wa = *reinterpret_cast<const bf16x8*>(wb1 + t * 64 * 16);
#pragma unroll
          for (int vb = 0; vb < 4; ++vb) accA[vb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa, bf[vb], accA[vb], 0, 0, 0);
        }
      }
    if (odd) {
      if (has2) epilogue(p, zlo);
#pragma unroll
      for (int vb = 0; vb < 4; ++vb) {
        accA[vb] = accB[vb];
        accB[vb] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };

  // step s: write plane s (loaded during step s-1) into slot s & 1, load plane s+1, compute plane s-1 (slot (s-1) & 1)
  S2Plane pw = walk.next(g);
  load_plane(pw);
  S2Plane pc{};
  int s = 0;
  while (pw.valid || pc.valid) {
    ps.mark_now();
    if (pw.valid) write_plane(pw, s & 1);
    ps.lap(0);
    const S2Plane pl = walk.next(g);
    load_plane(pl);
    ps.mark_now();
    ps.step(pc.valid);
    if (pc.valid) compute(pc, (s - 1) & 1);
    ps.lap(1);
    __syncthreads();
    ps.lap(2);
    pc = pw;
    pw = pl;
    ++s;
  }
  ps.end(s2_stamps, blockIdx.x & 1023, wave, lane);

  if (g.spart == nullptr) return;
  // ---- GroupNorm(16) statistics of the output: lanes with the same q4 hold the same group (xor over l16), the two
  // waves of a channel block in order (LDS), one [16][2] row per workgroup; the last-arriving workgroup combines the
  // rows of every sample in fp64 (fixed order: deterministic)
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) {
    gs += __shfl_xor(gs, o);
    gq += __shfl_xor(gq, o);
  }
  float* const red = reinterpret_cast<float*>(smem);  // [wave][4 q4][2] (the ring is idle after the last barrier)
  if (l16 == 0) {
    red[(wave * 4 + q4) * 2] = gs;
    red[(wave * 4 + q4) * 2 + 1] = gq;
  }
  __syncthreads();
  if (tid < 32) {
    const int gr = tid >> 1, k = tid & 1, cb_ = gr >> 2, q_ = gr & 3;  // group 4 cb + q4
    const float t2 = red[((0 * 4 + cb_) * 4 + q_) * 2 + k] + red[((1 * 4 + cb_) * 4 + q_) * 2 + k];
    __hip_atomic_store(g.spart + (long long)bid * 32 + tid, t2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sc1
  }
  __shared__ unsigned s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const unsigned old = __hip_atomic_fetch_add(g.cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = old == gridDim.x - 1;
    if (s_last) __hip_atomic_store(g.cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!s_last) return;
  double* const cs = reinterpret_cast<double*>(smem) + 64;  // [n * 16][2] (past the wave rows in `red`)
  lastarriver_rowsum<S2_NT>(g.spart, g.n, g.wps, 32, cs);
  __syncthreads();
  const double m = 4.0 * g.od * g.oh * g.ow;  // values per group and sample: 4 channels
  for (int pr = tid; pr < g.n * 16; pr += S2_NT) {
    const double mean = cs[2 * pr] / m;
    double var = cs[2 * pr + 1] / m - mean * mean;
    if (var < 0) var = 0;
    g.stats[pr * 2] = (float)mean;
    g.stats[pr * 2 + 1] = (float)(1.0 / sqrt(var + 1e-5));
  }
}

}  // namespace u3d

using namespace u3d;

static int s2_wgs() { return std::max(1, opt(OPT_RING_WGS)); }  // the persistent grid target of the rings

static bool s2_geom(int n, int cin, int d, int h, int w, int cout, S2Geom& g) {
  if (cin != 32 || cout != 64 || n < 1 || n * 16 > S2_NT || d < 1 || h < 1 || w < 1) return false;
  const long long xb = (long long)n * d * h * w * 64;
  if (xb >= (1LL << 31)) return false;
  g = S2Geom{};
  g.n = n; g.d = d; g.h = h; g.w = w;
  g.od = (d - 1) / 2 + 1; g.oh = (h - 1) / 2 + 1; g.ow = (w - 1) / 2 + 1;
  g.nbh = cdiv(g.oh, S2_OH); g.nbw = cdiv(g.ow, S2_OW);
  g.pps = (long long)g.nbh * g.nbw * g.od;
  const long long wps0 = std::max<long long>(1, std::min<long long>(g.pps, s2_wgs() / n));
  g.per = (int)((g.pps + wps0 - 1) / wps0);
  g.wps = (int)((g.pps + g.per - 1) / g.per);
  g.xbytes = (int)xb;
  return true;
}

// Which stride-2 3^3 forward shapes the input-plane walk serves (1) — cin 32 -> cout 64 bf16, x < 2 GiB, n <= 32.
extern "C" int u3d_conv_s2_ring_ok(int n, int cin, int d, int h, int w, int cout) {
  S2Geom g;
  return s2_geom(n, cin, d, h, w, cout, g) ? 1 : 0;
}

// floats of the statistics partials (spart) of u3d_conv_s2_ring
extern "C" long long u3d_conv_s2_ring_ws_floats(int n, int d, int h, int w) {
  S2Geom g;
  if (!s2_geom(n, 32, d, h, w, 64, g)) return 0;
  return (long long)n * g.wps * 32;
}

// y = conv3d(relu(gn(x)), W, stride 2, padding 1): x [n][d][h][w][32] bf16, wpk the forward pack [27][64][32], y
// [n][od][oh][ow][64] bf16; gn_* the GroupNorm on x (required). With stats_out: the output's GroupNorm(16) statistics
// [n][16][2] = (mean, rstd) from the epilogue (spart: u3d_conv_s2_ring_ws_floats floats; cnt: one ZEROED unsigned,
// left zeroed).
extern "C" int u3d_conv_s2_ring(const void* x, int n, int d, int h, int w, const void* wpk, const float* gn_stats,
                                const float* gn_gamma, const float* gn_beta, int gn_groups, void* y, float* spart,
                                float* stats_out, unsigned* cnt, u3d_stream_t stream) {
  U3D_REQUIRE(x && wpk && y && gn_stats && gn_gamma && gn_beta && gn_groups > 0 && 32 % gn_groups == 0,
              "conv_s2_ring: bad args");
  U3D_REQUIRE(!stats_out || (spart && cnt), "conv_s2_ring: statistics need spart and cnt");
  S2Geom g;
  U3D_REQUIRE(s2_geom(n, 32, d, h, w, 64, g), "conv_s2_ring: unsupported shape");
  g.gn_groups = gn_groups;
  if (stats_out) {
    g.spart = spart;
    g.stats = stats_out;
    g.cnt = cnt;
  }
  hipLaunchKernelGGL(conv_s2_ring_kernel, dim3((unsigned)(n * g.wps)), dim3(S2_NT), 0, (hipStream_t)stream,
                     (const bf16*)x, (const bf16*)wpk, (bf16*)y, gn_stats, gn_gamma, gn_beta, g);
  return check_launch("conv_s2_ring_kernel");
}
