// 32 -> 32 channel 3^3 stride-1 convolution (forward and data gradient), bf16, depth-streaming ring form
// (gfx950). Same contract as conv32_brick (u3d_conv32_brick), different schedule:
//
//   * a persistent workgroup (8 waves) owns a contiguous range of OUTPUT PLANES in (column, d) order, a column
//     being (n, 8-row h tile, 32-voxel w tile); it walks down d, so each input plane (10 x 34 halo rows x 32
//     ch) is staged once and used by three output planes (the brick form staged 4 input planes per 2 outputs);
//   * LDS keeps a ring of 4 staged planes: output plane z is computed from the three slots holding z-1, z,
//     z+1 while the fourth slot receives the next plane, so staging (global loads one step ahead in
//     registers, GroupNorm + ReLU applied once per element, LDS writes issued between the MFMAs) overlaps the
//     MFMAs and each output plane costs ONE barrier;
//   * the weights of all 27 taps stay in LDS (55 KB), the first KR (tap, co block) fragments also in registers;
//   * v_mfma_f32_16x16x32_bf16 issued transposed (A = weights, B = input rows): a lane's accumulators are 4
//     consecutive output channels of one voxel per (voxel block, co block), so after one permlane16 swap per pair
//     every lane stores 16-B chunks straight from registers (no LDS epilogue tile), and the residual is added in
//     the same layout. (Rounds 1-2 ran 32x32x16; the 16x16x32 form holds a higher clock, round 3.)
// Data gradient = the same kernel with the flipped tap offsets and the [t][ci][co] weight pack.
// Reference: F.conv3d in Conv3d.forward (unet3D.py:27) via NoBottleneck (:56-73) and its autograd.
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "diag.h"

namespace u3d {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;

constexpr int RG_BH = 8, RG_BW = 32, RG_HH = RG_BH + 2, RG_HW = RG_BW + 2;
constexpr int RG_NR = RG_HH * RG_HW;                 // 340 halo rows per plane
// chunk-plane stride (plane = 8 channels of every halo row): a multiple of 64 dwords, because one 16-lane ds_read_b128
// group of a v_mfma_f32_16x16x32_bf16 fragment spans two chunk planes; the staging writes 8 consecutive rows of one
// plane per 8-lane group, conflict-free as well
constexpr int RG_PS = (RG_NR * 16 + 255) / 256 * 256;
constexpr int RG_SS = 4 * RG_PS;                     // ring slot stride
constexpr int RG_NT = 512;
constexpr int RG_LD = (RG_NR * 4 + RG_NT - 1) / RG_NT;  // 3 staged 16-B pieces per thread and plane
constexpr int RG_NWR = 27 * 32;                      // weight rows (t, co)
#ifndef U3D_ABL_RING
#define U3D_ABL_RING 0
#endif
#ifndef RG_HOIST
#define RG_HOIST 1
#endif
// -DU3D_STAMPS phases (diag.h): 0 the steps' MFMAs + the staging side work between them, 1 the steps' heads (claims,
// GN table, walk), 2 the barriers
U3D_STAMP_BUFFER(rg_stamps, 2048, u3d_diag_ring_stamps)

struct RGGeom {
  int n, d, h, w;
  int nbh, nbw;
  long long planes;  // output planes = n * nbh * nbw * d
  long long xbytes;  // bytes of x (and of the residual / y): < 2^31, the buffer-offset range
  int per;           // output planes per workgroup
  int gn_groups;
  long long pps;     // output planes per sample; workgroups never straddle samples (per-sample GN statistics)
  int wps;           // workgroups per sample
  int sc, rmax;      // work-stealing mode: output planes per sub-chunk, sub-chunks per (full) range
  float* fstats;     // round 5: output GroupNorm(16) statistics finalized in-kernel (with fcnt; static forward only)
  unsigned* fcnt;    // zeroed arrival counter (left zeroed)
  float *coef, *dgamma, *dbeta;  // round 5, data gradient + GN partials: the finalize in-kernel (with fcnt)
};

// One staged input plane: column (n, h0, w0), input depth zin (-1 / d = zero padding), and whether it is the
// third plane of a triple (output zin - 1 follows it).
struct RGPlane {
  int n, h0, w0, zin;
  bool valid, out;
  int chunk;  // work-stealing mode: the sub-chunk the plane's output belongs to (statistics slot)
};

// Walks the workgroup's output range [o, o_end) as a sequence of input planes: each maximal run of outputs
// z0..z1-1 inside one column stages zin = z0-1 .. z1.
// The column coordinates (n, h0, w0) are decoded once per run (the divisions are off the per-plane path).
struct RGWalk {
  long long o_next, o_end;
  int zin, zfirst, zlast;
  int cn, ch0, cw0;
  bool done;
  __device__ void start_run(const RGGeom& g) {
    if (o_next >= o_end) { done = true; return; }
    const int col = (int)(o_next / g.d);
    zfirst = (int)(o_next - (long long)col * g.d);
    zlast = (int)min<long long>(g.d, zfirst + (o_end - o_next));
    o_next += zlast - zfirst;
    zin = zfirst - 1;
    int c = col;
    const int bw_ = c % g.nbw; c /= g.nbw;
    const int bh_ = c % g.nbh;
    cn = c / g.nbh;
    ch0 = bh_ * RG_BH;
    cw0 = bw_ * RG_BW;
  }
  __device__ RGPlane next(const RGGeom& g) {
    RGPlane p{};
    if (!done && zin > zlast) start_run(g);
    if (done) return p;
    p.n = cn;
    p.h0 = ch0;
    p.w0 = cw0;
    p.zin = zin;
    p.valid = true;
    p.out = zin >= zfirst + 1;
    ++zin;
    return p;
  }
};

// Q (work-stealing mode): each workgroup still owns the static range of output planes, split into sub-chunks of g.sc
// planes, and claims them front to back (one 64-bit compare-and-swap per sub-chunk on its range's word (front,
// stolen), lane 0, vector atomics) while walking the range as before; a workgroup whose range is exhausted steals
// sub-chunks from the BACK of other ranges. A workgroup that starts late (CUs held by a concurrent kernel, e.g.
// RCCL's all-reduce during the data-parallel backward) finds the back of its range already done by others, so the
// tail is one sub-chunk instead of a whole range; uncontended, the walk is the static one. GroupNorm statistics go
// to per-(sub-chunk, wave) slots (fixed-order finalize: deterministic whatever the assignment). The last workgroup
// to exit resets the words and the exit counter to zero for the next launch.
// The MFMA is v_mfma_f32_16x16x32_bf16 (round 3: the same cycles per flop as 32x32x16, but the chip holds a higher
// clock under it, MI355X_MICROARCH.md DVFS item 7): per tap (K = its 32 input channels) 4 MFMAs per wave = 2 voxel
// blocks x 2 output-channel blocks. KR = weight fragments (tap, co block) held in registers.
// XN (round 6, forward with the GroupNorm prologue only): the staged, normalised input relu(gn(x)) of the tile's own
// rows (not the halo) is also stored to xno (bf16 NDHWC, x's shape), so the conv's weight gradient reads it as is
// (wgrad_ring_dma_kernel<false>: no second GroupNorm transform of every staged x piece in the backward).
template <bool FLIP, bool GN, bool RES, int KR, bool Q = false, bool XN = false>
__global__ __launch_bounds__(RG_NT, 1) void conv32_ring_kernel(const bf16* __restrict__ x, const bf16* __restrict__ wpk,
                                                              bf16* __restrict__ y, const bf16* __restrict__ res,
                                                              const float* __restrict__ gstat,
                                                              const float* __restrict__ gamma,
                                                              const float* __restrict__ beta, float* __restrict__ spart,
                                                              RGGeom g, int* __restrict__ queue = nullptr,
                                                              bf16* __restrict__ xno = nullptr) {
  // GN on the forward (!FLIP): GroupNorm + ReLU prologue on the staged input. GN on the data gradient (FLIP): the
  // backward of that prologue's GroupNorm starts in the epilogue — res = x (the forward's pre-GroupNorm input), and
  // per channel (sum g, sum g*xhat) of g = relu-mask * dA go to spart[workgroup][32][2] (u3d_gn_bwd_parts finishes)
  constexpr bool PRO = GN && !FLIP, GB = GN && FLIP, LDR = RES || GB;
  static_assert(!(GB && (Q || RES)), "the fused GroupNorm backward runs on the static data-gradient ring only");
  static_assert(!XN || (PRO && !Q && RG_HOIST), "the normalised side output belongs to the static GN forward");
  __shared__ __attribute__((aligned(16))) char smem[4 * RG_SS + 4 * RG_NWR * 16 + 1024 + 512 + (GB ? 576 : 0)];
  char* const ring = smem;
  char* const wts = smem + 4 * RG_SS;
  char* const junk = wts + 4 * RG_NWR * 16;  // target of the staging lanes past the plane's last row
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  PhaseStamps ps;  // (from kernel entry: "other" = the weight prologue and the last plane's epilogue)
  ps.begin();
  diag_prio_second_half(wave);
  // staging: fixed 8-channel chunk (plane) per thread, 8 threads = 8 consecutive rows of one plane (a wave covers 16
  // whole rows = 1 KB of contiguous voxels per load)
  const int ch = (tid >> 3) & 3;
  const int srow = (tid & 7) + 8 * (tid >> 5);
  const int l16 = lane & 15, q4 = lane >> 4;  // fragment lane geometry: row / column, k group

  // XCD-aware range order: XCD x (= blockIdx % 8) runs a contiguous eighth of the output planes, so the
  // columns it works on at a time are neighbours whose halo rows meet in its L2.
  int bid = blockIdx.x;
  {
    const int nwg = gridDim.x, q = nwg >> 3, rr = nwg & 7, xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
    bid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + loc;
  }
  RGWalk walk{};
  int* const qslot = reinterpret_cast<int*>(smem + 4 * RG_SS + 4 * RG_NWR * 16 + 1024 + 256);  // claim broadcast
  unsigned long long* const words = reinterpret_cast<unsigned long long*>(queue);
  // range b = (sample, jw) of the static schedule: [o0, o0 + len), sub-chunks of g.sc planes
  auto range_len = [&](int b) {
    const int jw_ = b % g.wps;
    return (int)min<long long>(g.per, g.pps - (long long)jw_ * g.per);
  };
  auto range_o0 = [&](int b) { return (long long)(b / g.wps) * g.pps + (long long)(b % g.wps) * g.per; };
  auto nsub = [&](int b) { return (range_len(b) + g.sc - 1) / g.sc; };
  // Claims are single 64-bit atomic adds on the range's word (front | stolen << 32); the returned old value decides:
  // the owner's add of 1 wins sub-chunk `front` iff front + stolen < R, a thief's add of 2^32 wins sub-chunk
  // R - 1 - stolen under the same test. Adds serialise, so no sub-chunk is won twice; a losing add only overshoots
  // a counter of a range that is exhausted anyway. The owner's add is fire-and-forget (lane 0 keeps the old value
  // and publishes the verdict a step later), so claiming never stalls the walk.
  auto claim_ok = [&](unsigned long long old, int b) {
    return (unsigned)old + (unsigned)(old >> 32) < (unsigned)nsub(b);
  };
  // wave 0 only (all 64 lanes): steal the last unclaimed sub-chunk of another range, scanning 64 ranges per load
  // round; returns the global sub-chunk id (lane-uniform) or -1
  auto steal = [&]() -> int {
    const int nwg = (int)gridDim.x;
    for (int base = 1; base < nwg; base += 64) {
      for (;;) {
        const int v = (bid + base + lane) % nwg;
        bool cand = false;
        if (base + lane < nwg) {
          const unsigned long long w = __hip_atomic_load(&words[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          cand = claim_ok(w, v);
        }
        const unsigned long long m = __ballot(cand);
        if (!m) break;  // nothing left in these 64 ranges
        const int l = __builtin_ctzll(m), vv = (bid + base + l) % nwg;
        int got = -1;
        if (lane == 0) {
          const unsigned long long old = atomicAdd(&words[vv], 1ull << 32);
          if (claim_ok(old, vv)) got = vv * g.rmax + (int)((unsigned)nsub(vv) - 1 - (unsigned)(old >> 32));
        }
        got = __shfl(got, 0);
        if (got >= 0) return got;  // else lost a race on vv: rescan
      }
    }
    return -1;
  };
  bool own = true;        // walking the own range (claims pending at sub-chunk boundaries)
  int claimed = -1;       // own sub-chunks claimed so far: 0..claimed
  int issued = -1;        // own claim in flight (lane 0 holds the old word in claim_old)
  int check = -1;         // own claim whose verdict is in qslot[1] after this step's barrier
  unsigned long long claim_old = 0;
  int nxt = -1;           // steal mode: stolen sub-chunk waiting to be walked (-1: none)
  if constexpr (Q) {
    if (tid == 0) qslot[0] = claim_ok(atomicAdd(&words[bid], 1ull), bid);
  } else {
    const int smp = bid / g.wps, jw = bid - smp * g.wps;
    walk.o_next = (long long)smp * g.pps + (long long)jw * g.per;
    walk.o_end = min((long long)(smp + 1) * g.pps, walk.o_next + g.per);
    walk.done = false;
    walk.zin = 1;
    walk.zlast = 0;  // forces start_run on the first next()
  }

  {  // weights: plane c, row t*32 + co. Every load of a thread is issued before its first LDS store (r05 stamps: the
     // rolled loop waited on each of its 7 loads in turn, ~10 us of every launch's prologue)
    constexpr int NWL = (RG_NWR * 4 + RG_NT - 1) / RG_NT;
    u32x4 wl[NWL];
#pragma unroll
    for (int k = 0; k < NWL; ++k) {
      const int i = tid + k * RG_NT, c = i / RG_NWR, row = i % RG_NWR;
      if (i < RG_NWR * 4) wl[k] = *reinterpret_cast<const u32x4*>(wpk + row * 32 + c * 8);
    }
#pragma unroll
    for (int k = 0; k < NWL; ++k) {
      const int i = tid + k * RG_NT;
      if (i < RG_NWR * 4) *reinterpret_cast<u32x4*>(wts + i * 16) = wl[k];  // (c * RG_NWR + row = i)
    }
  }
  // k16 step st = (tap t = st >> 1, half s = st & 1): this lane's weight fragment is W[t][co = r][16s + 8h ..]
  // weight fragment st = (tap st >> 1, co block st & 1): W[t][co = 16 (st & 1) + l16][8 q4 ..] (whole taps only)
  constexpr int KRX = KR & ~1;
  bf16x8 wreg[KRX > 0 ? KRX : 1];
#pragma unroll
  for (int st = 0; st < KRX; ++st)
    wreg[st] = *reinterpret_cast<const bf16x8*>(wpk + ((st >> 1) * 32 + 16 * (st & 1) + l16) * 32 + 8 * q4);

  // buffer loads: out-of-range offsets return zeros with no branch around the load (no exec-masked paths whose
  // merge would make the wait-count insertion pessimistic)
  const auto xrs = __builtin_amdgcn_make_buffer_rsrc((void*)x, 0, (int)g.xbytes, 0x00020000);
  const auto rrs = __builtin_amdgcn_make_buffer_rsrc((void*)res, 0, LDR ? (int)g.xbytes : 0, 0x00020000);
  f32x2 sc[4], sh[4];
  int gn_n = -1;
  // branch-free staging: out-of-volume rows load a valid dummy address and are zeroed when written
  // staged piece i of plane p (16 B of one halo row) into v[i]; bit i of m = the row is inside the volume
  // (round 4, RG_HOIST) a lane's halo row of piece i is the same in every plane: its byte offset is a per-lane constant
  // plus a wave-uniform plane base, and its in-volume test changes only with the column — per piece and plane one add
  // and one select instead of the integer address math (r04 stamps / ISA: issue slots the MFMA chain needs)
#if RG_HOIST
  int plo[RG_LD];
#pragma unroll
  for (int i = 0; i < RG_LD; ++i) {
    const int row = srow + i * (RG_NT / 4);
    plo[i] = (((row / RG_HW) * g.w + row % RG_HW) * 64 + ch * 16);
  }
  unsigned pin = 0;
  int col_h0 = -1, col_w0 = -1;
  unsigned pint = 0;  // XN: bit i = piece i's halo row is one of the tile's own rows (stored to xno)
  if constexpr (XN) {
#pragma unroll
    for (int i = 0; i < RG_LD; ++i) {
      const int row = srow + i * (RG_NT / 4), hh = row / RG_HW, hw = row % RG_HW;
      pint |= (row < RG_NR && hh >= 1 && hh <= RG_BH && hw >= 1 && hw <= RG_BW ? 1u : 0u) << i;
    }
  }
#endif
  const auto nrs = __builtin_amdgcn_make_buffer_rsrc((void*)xno, 0, XN ? (int)g.xbytes : 0, 0x00020000);
  auto load_piece = [&](const RGPlane& p, int i, u32x4 (&v)[RG_LD], unsigned& m) {
#if RG_HOIST
    if (i == 0 && p.valid && (p.h0 != col_h0 || p.w0 != col_w0)) {  // uniform: once per run of the walk
      col_h0 = p.h0;
      col_w0 = p.w0;
      pin = 0;
#pragma unroll
      for (int j = 0; j < RG_LD; ++j) {
        const int row = srow + j * (RG_NT / 4);
        const bool ok = row < RG_NR && (unsigned)(p.h0 - 1 + row / RG_HW) < (unsigned)g.h &&
                        (unsigned)(p.w0 - 1 + row % RG_HW) < (unsigned)g.w;
        pin |= (ok ? 1u : 0u) << j;
      }
    }
    const int base = (((p.n * g.d + p.zin) * g.h + p.h0 - 1) * g.w + p.w0 - 1) * 64;
    const bool ok = p.valid && (unsigned)p.zin < (unsigned)g.d && ((pin >> i) & 1u);
    const unsigned off = ok ? (unsigned)(base + plo[i]) : 0xFFFFFFF0u;
#else
    const int row = srow + i * (RG_NT / 4);
    const int hw = row % RG_HW, hh = row / RG_HW;
    const int zh = p.h0 - 1 + hh, zw = p.w0 - 1 + hw;
    const bool ok = p.valid && row < RG_NR && (unsigned)p.zin < (unsigned)g.d && (unsigned)zh < (unsigned)g.h &&
                    (unsigned)zw < (unsigned)g.w;
    const unsigned off = ok ? (unsigned)((((p.n * g.d + p.zin) * g.h + zh) * g.w + zw) * 64 + ch * 16) : 0xFFFFFFF0u;
#endif
    v[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0));
    m = (i == 0 ? 0u : m) | ((ok ? 1u : 0u) << i);
  };
  auto load_plane = [&](const RGPlane& p, u32x4 (&v)[RG_LD], unsigned& m) {
#pragma unroll
    for (int i = 0; i < RG_LD; ++i) load_piece(p, i, v, m);
  };
  auto gn_table = [&](const RGPlane& p) {
    if (PRO && p.valid && p.n != gn_n) {
      gn_n = p.n;
      gn_coef8(gstat, gamma, beta, g.gn_groups, 32, p.n, ch * 8, sc, sh);
    }
  };
  auto write_piece = [&](int i, const u32x4& v, unsigned m, int slot, int xbase) {
    const int row = srow + i * (RG_NT / 4);
    u32x4 val = v;
#if !(U3D_ABL_RING & 1)  // (timing-only ablation builds, tools/build_variant.sh: bit 0 = GroupNorm prologue compiled out)
    if constexpr (PRO) val = gn_relu8(v, sc, sh);
    if constexpr (PRO) if (!((m >> i) & 1u)) val = u32x4{0u, 0u, 0u, 0u};  // padding stays zero after the prologue
#endif
    char* dst = row < RG_NR ? ring + slot * RG_SS + ch * RG_PS + row * 16 : junk + (tid & 63) * 16;
    *reinterpret_cast<u32x4*>(dst) = val;
#if RG_HOIST
    if constexpr (XN) {  // the tile's own in-volume rows: an out-of-range offset drops the store (no branch)
      const unsigned off = ((m & pint) >> i) & 1u ? (unsigned)(xbase + plo[i]) : 0xFFFFFFF0u;
      __builtin_amdgcn_raw_buffer_store_b128(val, nrs, off, 0, 0);
    }
#endif
  };

  // A computed output plane waiting for its epilogue: the epilogue (bf16 pack, permlane swap, residual add,
  // stores) of plane k runs between the MFMAs of plane k+1, so it is off the per-plane critical path.
  struct Pending {
    f32x4 a4[4];   // [voxel block vb * 2 + co block cb]
    u32x4 rv[2];   // residual of voxel blocks 0, 1
    long long vox;
    bool ok, ok1;  // voxel blocks 0 and 1 inside the volume
    int chunk;
  };
  Pending pend;
  pend.ok = pend.ok1 = false;
  pend.vox = 0;
  pend.chunk = -1;
  pend.rv[0] = pend.rv[1] = u32x4{0u, 0u, 0u, 0u};  // (GB reads them before the first computed plane)
  // GroupNorm(16, 32) statistics of the output (GN variants = the forward convs whose outputs feed the next
  // GroupNorm), from the fp32 values just before the final bf16 rounding (no unpack; the voxel's in-volume flag
  // selects): 4 (sum, sum of squares) pairs per lane, fp32 over the lane's voxels, reduced per workgroup at the end.
  // Without residual acc a4[vb*2 + cb][k] is channel 16 cb + 4 q4 + k -> slot 2 cb + k/2 = group 8 cb + 2 q4 + k/2;
  // with residual the post-swap values are channels 16 (q4 & 1) + 8 (q4 >> 1) + e -> slot e/2 = group
  // 8 (q4 & 1) + 4 (q4 >> 1) + e/2. Lanes with the same q4 hold the same groups.
  constexpr int NSL = 4;  // statistics slots per lane
  constexpr int XR = 16;  // lanes sharing a slot's group (xor-reduced)
  auto slot_group = [&](int j) { return RES ? 8 * (q4 & 1) + 4 * (q4 >> 1) + j : 8 * (j >> 1) + 2 * q4 + (j & 1); };
  const bool slot_writer = (lane & (XR - 1)) == 0;
  float gs[NSL], gq[NSL];
#pragma unroll
  for (int j = 0; j < NSL; ++j) gs[j] = gq[j] = 0.f;
  int acc_chunk = -1;
  // GB: this lane's 8 channels after the swap (cbase..cbase+7) of the workgroup's one sample: mask coefficients
  // (the forward prologue's x*sc + sh > 0 test), xhat = (x - mu)*rs, and (sum g, sum g*xhat) accumulators
  // (table in LDS [channel][sc, sh, rs, -mu*rs]: registers are what the weight steps need; entry c at c + c / 8, so
  // the 4 channel chunks a ds_read_b128 lane group reads sit in different banks: unpadded, chunks 0 and 16 collided,
  // SQ_LDS_BANK_CONFLICT = 10% of the ring's LDS cycles, r04)
  float bs1[GB ? 8 : 1], bs2[GB ? 8 : 1];
  f32x4* const gtab = reinterpret_cast<f32x4*>(smem + 4 * RG_SS + 4 * RG_NWR * 16 + 1536);
  if constexpr (GB) {
    if (tid < 32) {
      const int smp = bid / g.wps, gr = tid / (32 / g.gn_groups);
      const float mu = gstat[(smp * g.gn_groups + gr) * 2], rs = gstat[(smp * g.gn_groups + gr) * 2 + 1];
      const float scv = rs * gamma[tid];
      gtab[tid + (tid >> 3)] = f32x4{scv, beta[tid] - mu * scv, rs, mu};
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) bs1[e] = bs2[e] = 0.f;
  }
  // work-queue mode: the statistics of one chunk, per wave: reduce over the wave's voxels (xor within the 32-lane
  // halves) and write slot (chunk, wave); no barrier, so it can run inside the MFMA chain
  auto flush = [&](int c) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < NSL; ++j)
#pragma unroll
      for (int o = 1; o < XR; o <<= 1) {
        gs[j] += __shfl_xor(gs[j], o);
        gq[j] += __shfl_xor(gq[j], o);
      }
    if (slot_writer) {
#pragma unroll
      for (int j = 0; j < NSL; ++j) {
        const int grp = slot_group(j);
        spart[((long long)c * (RG_NT / 64) + wave) * 32 + grp * 2] = gs[j];
        spart[((long long)c * (RG_NT / 64) + wave) * 32 + grp * 2 + 1] = gq[j];
      }
    }
#pragma unroll
    for (int j = 0; j < NSL; ++j) gs[j] = gq[j] = 0.f;
  };
  auto epilogue = [&](const Pending& p) __attribute__((always_inline)) {
    if constexpr (Q && PRO) {
      if (spart != nullptr && p.chunk != acc_chunk) {
        if (acc_chunk >= 0) flush(acc_chunk);
        acc_chunk = p.chunk;
      }
    }
    // lane (l16, q4): a4[vb*2 + cb][k] = channel 16 cb + 4 q4 + k of voxel 16 vb + l16. Pack to bf16 pairs, then
    // one permlane16 swap per pair (odd 16-lane rows of the co-block-0 value <-> even rows of the co-block-1
    // value): an even-row lane then holds channels 8m..8m+7 (m = q4 >> 1), an odd-row lane 16+8m..16+8m+7, of its
    // voxel -> one 16-B store per voxel block.
    const int cbase = 16 * (q4 & 1) + 8 * (q4 >> 1);
#pragma unroll
    for (int vb = 0; vb < 2; ++vb) {
      const bool okv = vb ? p.ok1 : p.ok;
      if constexpr (PRO && !RES && !(U3D_ABL_RING & 2)) {  // (ablation bit 1: output statistics compiled out)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float t = okv ? p.a4[vb * 2 + cb][k] : 0.f;  // select: rows past the volume may be non-finite
            gs[2 * cb + (k >> 1)] += t;
            gq[2 * cb + (k >> 1)] = fmaf(t, t, gq[2 * cb + (k >> 1)]);
          }
      }
      uint32_t pk[2][2];
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int e = 0; e < 2; ++e) pk[cb][e] = pack_bf16x2(p.a4[vb * 2 + cb][2 * e], p.a4[vb * 2 + cb][2 * e + 1]);
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const auto sw = __builtin_amdgcn_permlane16_swap(pk[0][e], pk[1][e], false, false);
        pk[0][e] = sw[0];
        pk[1][e] = sw[1];
      }
      u32x4 v = {pk[0][0], pk[0][1], pk[1][0], pk[1][1]};
      if constexpr (RES) {
        float a[8], c[8];
        load16<bf16>(reinterpret_cast<const bf16*>(&v), a);
        load16<bf16>(reinterpret_cast<const bf16*>(&p.rv[vb]), c);
#pragma unroll
        for (int e = 0; e < 8; ++e) a[e] += c[e];
        if constexpr (GN && !(U3D_ABL_RING & 2)) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float t = okv ? a[e] : 0.f;
            gs[e >> 1] += t;
            gq[e >> 1] = fmaf(t, t, gq[e >> 1]);
          }
        }
        store16<bf16>(reinterpret_cast<bf16*>(&v), a);
      }
      if constexpr (GB) {  // from the stored bf16 dA, as u3d_gn_bwd's partial pass reads it
        float a[8], xv[8];
        load16<bf16>(reinterpret_cast<const bf16*>(&v), a);
        load16<bf16>(reinterpret_cast<const bf16*>(&p.rv[vb]), xv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const f32x4 t = gtab[cbase + (cbase >> 3) + e];
          const bool m = okv && fmaf(xv[e], t[0], t[1]) > 0.f;  // selects: rows past the volume may be non-finite
          bs1[e] += m ? a[e] : 0.f;
          bs2[e] = fmaf(m ? a[e] : 0.f, m ? (xv[e] - t[3]) * t[2] : 0.f, bs2[e]);
        }
      }
      if (okv) *reinterpret_cast<u32x4*>(y + (p.vox + 16 * vb) * 32 + cbase) = v;
    }
  };

  // output plane from the three slots s0 (z-1), s1 (z), s2 (z+1); the staging writes of the staged plane, the
  // loads of the next one (side(st), at compile-time MFMA steps) and the previous plane's epilogue are issued between
  // the MFMAs. H = 1 places them at later steps (15.., epilogue 44): staggering the two waves of a SIMD pair that way
  // (waves >= 4 on H = 1, MI355X_MICROARCH.md two waves per SIMD, item 9) measured equal or 2-3% slower at 96^3
  // (profiles/r03_ring_ablations.log), so every wave runs H = 0.
  auto compute = [&](const RGPlane& pc, int s0, int s1, int s2, auto hc, auto&& side) __attribute__((always_inline)) {
    // 16x16x32: per tap (K = 32 input channels) 4 MFMAs = (voxel block vb: row voxels 16 vb..) x (co block cb);
    // A = weights (rows = output channels), B = input rows (columns = voxels): a lane's accumulators are 4
    // consecutive channels of one voxel per (vb, cb). Fragments: lane (l16, q4) reads 16 B of chunk plane q4
    // (channels 8 q4 ..) of row l16 of the block: the 4 chunk planes of one row are one tap's K.
    const int zo = pc.zin - 1;
    const int zh = pc.h0 + wave, zw = pc.w0 + l16;
    Pending nw;
    nw.chunk = pc.chunk;
    nw.ok = zh < g.h && zw < g.w;
    nw.ok1 = zh < g.h && zw + 16 < g.w;
    nw.vox = (((long long)pc.n * g.d + zo) * g.h + zh) * g.w + zw;
    nw.rv[0] = nw.rv[1] = u32x4{0u, 0u, 0u, 0u};
    if constexpr (LDR) {  // the 16 B this lane stores after the swap, per voxel block (residual, or GB's x)
      const int cb2 = 2 * (16 * (q4 & 1) + 8 * (q4 >> 1));
      const unsigned r0 = nw.ok ? (unsigned)(nw.vox * 64 + cb2) : 0xFFFFFFC0u;
      const unsigned r1 = nw.ok1 ? (unsigned)((nw.vox + 16) * 64 + cb2) : 0xFFFFFFC0u;
      nw.rv[0] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rrs, r0, 0, 0));
      nw.rv[1] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rrs, r1, 0, 0));
    }
    const int sl[3] = {FLIP ? s2 : s0, s1, FLIP ? s0 : s2};
    const char* ibase = ring + q4 * RG_PS + (wave * RG_HW + l16) * 16;
    const char* wbase = wts + (q4 * RG_NWR + l16) * 16;
    auto ioff = [&](int t) {
      const int td = t / 9, th = (t / 3) % 3, tw = t % 3;
      const int oh = FLIP ? 2 - th : th, ow = FLIP ? 2 - tw : tw;
      return sl[td] * RG_SS + (oh * RG_HW + ow) * 16;
    };
#pragma unroll
    for (int i = 0; i < 4; ++i) nw.a4[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    constexpr int LA = 2;  // taps of fragments in flight
    bf16x8 fi[LA + 1][2], fw[LA + 1][2];
    auto rd = [&](int t, int k) {
      const int o = ioff(t);
      fi[k][0] = *reinterpret_cast<const bf16x8*>(ibase + o);
      fi[k][1] = *reinterpret_cast<const bf16x8*>(ibase + o + 16 * 16);
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const int st = 2 * t + cb;
        if (st < KRX)
          fw[k][cb] = wreg[st < KRX ? st : 0];
        else
          fw[k][cb] = *reinterpret_cast<const bf16x8*>(wbase + (t * 32 + 16 * cb) * 16);
      }
    };
#pragma unroll
    for (int k = 0; k < LA; ++k) rd(k, k);
    auto tstep = [&](auto tc) {
      constexpr int t = decltype(tc)::value;
      if constexpr (t + LA < 27) rd(t + LA, (t + LA) % (LA + 1));
      side(std::integral_constant<int, t - 1>{});
      if constexpr (t == 15) epilogue(pend);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int vb = 0; vb < 2; ++vb)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
          nw.a4[vb * 2 + cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[t % (LA + 1)][cb], fi[t % (LA + 1)][vb],
                                                                       nw.a4[vb * 2 + cb], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    };
    __builtin_amdgcn_sched_barrier(0);
    static_for<0, 27>(tstep);
    pend = nw;
  };

  // step s: load plane s+1 into registers, write plane s (loaded during step s-1) into slot s&3, compute the
  // output whose triple ends at plane s-1, barrier. Unrolled by two so the register sets swap statically.
  u32x4 va[RG_LD], vb[RG_LD];
  unsigned ma = 0, mb = 0;
  auto set_range = [&](long long o0, long long o1) {
    walk.o_next = o0;
    walk.o_end = o1;
    walk.done = false;
    walk.zin = 1;
    walk.zlast = 0;
  };
  // statistics slot of the next output plane, tracked incrementally (no divisions in the walk): own mode counts the
  // range's outputs (sub-chunk k = count / sc), a stolen range is one sub-chunk
  int own_cnt = 0, own_k = 0, stolen_id = -1;
  auto start_stolen = [&](int id) {  // walk sub-chunk id (= range * rmax + k)
    stolen_id = id;
    const int b = id / g.rmax, k = id - b * g.rmax;
    const long long o0 = range_o0(b) + (long long)k * g.sc;
    set_range(o0, min(range_o0(b) + range_len(b), o0 + g.sc));
  };
  if constexpr (Q) {
    __syncthreads();  // the claim of sub-chunk 0
    if (qslot[0]) {
      claimed = 0;
      set_range(range_o0(bid), range_o0(bid) + range_len(bid));
    } else {  // the whole range was stolen before this workgroup started
      own = false;
      walk.done = true;
      if (wave == 0) {
        const int st_ = steal();
        if (lane == 0) qslot[2] = st_;
      }
      __syncthreads();
      nxt = qslot[2];
    }
  }
  // next input plane of the walk. Own mode: staging the first plane whose output starts own sub-chunk k issues the
  // claim of k (result read at the next step, two steps before that output is computed). Steal mode: a finished
  // range hands over to the stolen sub-chunk fetched one ahead, and lane 0 steals the one after it.
  auto next_plane = [&]() __attribute__((always_inline)) {
    RGPlane p = walk.next(g);
    if constexpr (Q) {
      if (own && !p.valid) {  // own range done: from now on steal (uniform branch; one extra barrier per workgroup)
        own = false;
        if (wave == 0) {
          const int st_ = steal();
          if (lane == 0) qslot[3] = st_;
        }
        __syncthreads();
        nxt = qslot[3];
      }
      if (!own && !p.valid && nxt >= 0) {  // next stolen range; steal the one after it now (wave 0)
        start_stolen(nxt);
        nxt = -2;
        if (wave == 0) {
          const int st_ = steal();
          if (lane == 0) qslot[2] = st_;
        }
        p = walk.next(g);
      }
      if (p.valid && p.out) {
        if (own) {
          const int k = own_k;
          p.chunk = bid * g.rmax + k;
          if (++own_cnt == g.sc) {
            own_cnt = 0;
            ++own_k;
          }
          if (k > claimed && issued < 0 && check < 0) {
            issued = k;
            if (tid == 0) claim_old = atomicAdd(&words[bid], 1ull);
          }
        } else {
          p.chunk = stolen_id;
        }
      }
    }
    return p;
  };
  RGPlane pw = next_plane();  // plane 0
  load_plane(pw, va, ma);
  __syncthreads();            // weights visible
  RGPlane pc{};               // plane s-1 (compute)
  int s = 0;
  // The staged plane is written at the start of the step, BEFORE the next plane's loads are issued: its loads
  // (a full step old) are then the oldest in flight, so no wait inside the MFMA chain can fall on a young load.
  auto step = [&](u32x4 (&vcur)[RG_LD], unsigned& mcur, u32x4 (&vnxt)[RG_LD], unsigned& mnxt) {
    if constexpr (Q) {
      if (nxt == -2) nxt = qslot[2];
      if (check >= 0) {  // verdict of the claim issued two steps ago; its first plane is pc now
        if (qslot[1]) {
          claimed = check;
        } else {  // sub-chunks check.. were stolen: the own range ends before pc's output
          pc.out = false;
          pw.out = false;
          walk.done = true;
          own = false;
          if (wave == 0) {
            const int st_ = steal();
            if (lane == 0) qslot[2] = st_;
          }
          __syncthreads();
          nxt = qslot[2];
        }
        check = -1;
      }
      if (issued >= 0) {  // publish last step's claim (its atomic has long returned); read after this barrier
        if (tid == 0) qslot[1] = claim_ok(claim_old, bid);
        check = issued;
        issued = -1;
      }
    }
    gn_table(pw);
    const int slot = s & 3;
    const int xbase = XN ? (((pw.n * g.d + pw.zin) * g.h + pw.h0 - 1) * g.w + pw.w0 - 1) * 64 : 0;
    const RGPlane pl = next_plane();  // plane s+1
    // side work of the step, k = 0 .. 2 RG_LD - 1: even k writes staged piece k/2 of plane s into slot s & 3 (its
    // loads were issued a full step ago), odd k issues the load of piece k/2 of plane s + 1
    auto side = [&](auto kc) __attribute__((always_inline)) {
      constexpr int k = decltype(kc)::value;
      if constexpr (k >= 0 && k < 2 * RG_LD) {
        if constexpr ((k & 1) == 0) {
          if (pw.valid) write_piece(k >> 1, vcur[k >> 1], mcur, slot, xbase);
        } else {
          load_piece(pl, k >> 1, vnxt, mnxt);
        }
      }
    };
    ps.lap(1);  // phase 1: the step's head (claims, GN table, walk) since the previous barrier
    if (pc.valid && pc.out) {
      compute(pc, (s - 3) & 3, (s - 2) & 3, (s - 1) & 3, std::integral_constant<int, 0>{}, side);
    } else {
      static_for<0, 2 * RG_LD>(side);
    }
    ps.lap(0);  // phase 0: the step's MFMAs and staging (compute-less steps included)
    ps.step(pc.valid && pc.out);
    __syncthreads();
    ps.lap(2);
    pc = pw;
    pw = pl;
    ++s;
  };
  while (pw.valid || (pc.valid && pc.out)) {
    step(va, ma, vb, mb);
    if (!(pw.valid || (pc.valid && pc.out))) break;
    step(vb, mb, va, ma);
  }
  epilogue(pend);  // the last computed plane (ok = false if none)
  if (!Q) ps.end(rg_stamps, blockIdx.x & 2047, wave, lane);
  if constexpr (Q) {
    if constexpr (PRO) {
      if (spart != nullptr && acc_chunk >= 0) flush(acc_chunk);
    }
    int* const exits = reinterpret_cast<int*>(words + gridDim.x);
    // a claim issued in the last step(s) may still be in flight: consume its result (waits for the atomic) so that
    // every claim of this workgroup has landed before its exit is counted (device-scope atomics of one lane, in
    // order; no fence: an agent-scope release would write back the XCD's whole L2)
    if (tid == 0 && issued >= 0) qslot[1] = claim_ok(claim_old, bid);
    if (tid == 0 && atomicAdd(exits, 1) == (int)gridDim.x - 1) {  // every workgroup is past its last claim
      for (unsigned b = 0; b < gridDim.x; ++b) atomicExch(&words[b], 0ull);
      atomicExch(exits, 0);
    }
    return;
  }
  if constexpr (GB) {
    // lanes with the same q4 hold the same 8 channels: reduce over l16, then over the waves in fixed order (LDS)
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int o = 1; o < XR; o <<= 1) {
        bs1[e] += __shfl_xor(bs1[e], o);
        bs2[e] += __shfl_xor(bs2[e], o);
      }
    float* red = reinterpret_cast<float*>(ring);  // [wave][channel 32][2]
    if (slot_writer) {
      const int cb0 = 16 * (q4 & 1) + 8 * (q4 >> 1);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[(wave * 32 + cb0 + e) * 2] = bs1[e];
        red[(wave * 32 + cb0 + e) * 2 + 1] = bs2[e];
      }
    }
    __syncthreads();
    if (tid < 64) {
      float t = 0.f;
#pragma unroll
      for (int wv = 0; wv < RG_NT / 64; ++wv) t += red[wv * 64 + tid];
      if (g.fcnt)  // write-through: the finalizing workgroup reads it in this launch
        __hip_atomic_store(spart + (long long)bid * 64 + tid, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else
        spart[(long long)bid * 64 + tid] = t;  // [sample][wps][channel][2]: bid = sample * wps + jw
    }
    if (g.fcnt) {
      // Round 5: gn_bwd_parts_finalize by the workgroup that arrives last (one launch less): every wave drains, one lane
      // per workgroup adds to the arrival counter, the last arriver sums the partial rows per (sample, channel) in fp64
      // (8 lanes per pair strided over the sample's workgroups, then an xor tree in fixed order: deterministic) and
      // forms the apply coefficients coef[n][5][32] and dgamma / dbeta exactly as gn_bwd_coefs does.
      __shared__ unsigned s_last;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        const unsigned old = __hip_atomic_fetch_add(g.fcnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = old == gridDim.x - 1;
        if (s_last) __hip_atomic_store(g.fcnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
      if (!s_last) return;
      double* const cs = reinterpret_cast<double*>(ring);  // [n * 32][2]
      lastarriver_rowsum<RG_NT>(spart, g.n, g.wps, 64, cs);
      __syncthreads();
      const int gcpg = 32 / g.gn_groups;
      const double M = (double)g.d * g.h * g.w * gcpg;
      for (int pr = tid; pr < g.n * 32; pr += RG_NT) {
        const int nn = pr >> 5, c = pr & 31, gr = c / gcpg;
        double a = 0, bb = 0;
        for (int k2 = 0; k2 < gcpg; ++k2) {
          const int cc = gr * gcpg + k2;
          a += (double)gamma[cc] * cs[2 * (nn * 32 + cc)];
          bb += (double)gamma[cc] * cs[2 * (nn * 32 + cc) + 1];
        }
        const float ca = (float)(a / M), cb = (float)(bb / M);
        const float mu = gstat[(nn * g.gn_groups + gr) * 2], rs = gstat[(nn * g.gn_groups + gr) * 2 + 1];
        const float scv = rs * gamma[c];
        float* oc = g.coef + (long long)nn * 5 * 32;
        oc[c] = scv;
        oc[32 + c] = beta[c] - mu * scv;
        oc[64 + c] = rs * gamma[c];
        oc[96 + c] = -rs * rs * cb;
        oc[128 + c] = -rs * ca + rs * rs * cb * mu;
      }
      if (tid < 32) {
        double tg = 0, tb = 0;
        for (int nn = 0; nn < g.n; ++nn) {
          tb += cs[2 * (nn * 32 + tid)];
          tg += cs[2 * (nn * 32 + tid) + 1];
        }
        if (g.dgamma) g.dgamma[tid] = (float)tg;
        if (g.dbeta) g.dbeta[tid] = (float)tb;
      }
    }
  } else if constexpr (GN) {
    if (spart == nullptr) return;
    // lanes with the same q4 hold the same groups: reduce over l16 (xor within 16-lane rows), then over the waves in
    // fixed order through LDS (the ring is idle: every step ended with a barrier)
#pragma unroll
    for (int j = 0; j < NSL; ++j)
#pragma unroll
      for (int o = 1; o < XR; o <<= 1) {
        gs[j] += __shfl_xor(gs[j], o);
        gq[j] += __shfl_xor(gq[j], o);
      }
    float* red = reinterpret_cast<float*>(ring);  // [wave][group 16][2]
    if (slot_writer) {
#pragma unroll
      for (int j = 0; j < NSL; ++j) {
        const int grp = slot_group(j);
        red[(wave * 16 + grp) * 2] = gs[j];
        red[(wave * 16 + grp) * 2 + 1] = gq[j];
      }
    }
    __syncthreads();
    if (tid < 32) {
      float t = 0.f;
#pragma unroll
      for (int wv = 0; wv < RG_NT / 64; ++wv) t += red[wv * 32 + tid];
      if (g.fcnt)  // write-through: the finalizing workgroup reads it in this launch
        __hip_atomic_store(spart + (long long)bid * 32 + tid, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else
        spart[(long long)bid * 32 + tid] = t;  // [sample][wps][group][2]: bid = sample * wps + jw
    }
    if (g.fcnt) {
      // Round 5: ring_gn_finalize_kernel's combine by the workgroup that arrives last (one launch less): every wave
      // drains, one lane per workgroup adds to the arrival counter (agent scope), the last arriver reads the partial
      // rows with sc1 loads; 16 lanes per (sample, group) strided over the sample's workgroups, xor tree in fixed order.
      __shared__ unsigned s_last;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        const unsigned old = __hip_atomic_fetch_add(g.fcnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = old == gridDim.x - 1;
        if (s_last) __hip_atomic_store(g.fcnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
      if (s_last) {
        double* const cs = reinterpret_cast<double*>(ring) + 2048;  // [n * 16][2] (past the stats rows in `red`)
        lastarriver_rowsum<RG_NT>(spart, g.n, g.wps, 32, cs);
        __syncthreads();
        const double m = 2.0 * g.d * g.h * g.w;
        for (int p = tid; p < g.n * 16; p += RG_NT) {
          const double mean = cs[2 * p] / m;
          double var = cs[2 * p + 1] / m - mean * mean;
          if (var < 0) var = 0;
          g.fstats[p * 2] = (float)mean;
          g.fstats[p * 2 + 1] = (float)(1.0 / sqrt(var + 1e-5));
        }
      }
    }
  }
}

// stats[n][16] = (mean, rstd) of GroupNorm(16, 32) from per-workgroup partial rows [n][wps][16][2] (ring, stem,
// upsample): one 256-thread block per (n, group), threads strided over the rows with 8 loads in flight (r05: one wave
// with a dependent load per row took 12.5 us at the stem's 3456 rows per sample), then the wave butterflies and the
// 4 waves in order (fixed order: deterministic)
__global__ __launch_bounds__(256) void ring_gn_finalize_kernel(const float* __restrict__ spart, int n, int wps, double m,
                                                              float* __restrict__ stats) {
  __shared__ double red[4][2];
  const int p = blockIdx.x, nn = p / 16, gr = p % 16, tid = threadIdx.x;
  const float2* rows = reinterpret_cast<const float2*>(spart + (long long)nn * wps * 32 + gr * 2);
  double s1 = 0, s2 = 0;
  for (int w0 = tid; w0 < wps; w0 += 8 * 256) {
    float2 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int w = w0 + u * 256;
      v[u] = w < wps ? rows[(long long)w * 16] : make_float2(0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      s1 += v[u].x;
      s2 += v[u].y;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    s1 += __shfl_xor(s1, o);
    s2 += __shfl_xor(s2, o);
  }
  if ((tid & 63) == 0) {
    red[tid >> 6][0] = s1;
    red[tid >> 6][1] = s2;
  }
  __syncthreads();
  if (tid == 0) {
    const double t1 = ((red[0][0] + red[1][0]) + red[2][0]) + red[3][0];
    const double t2 = ((red[0][1] + red[1][1]) + red[2][1]) + red[3][1];
    const double mean = t1 / m;
    double var = t2 / m - mean * mean;
    if (var < 0) var = 0;
    stats[p * 2] = (float)mean;
    stats[p * 2 + 1] = (float)(1.0 / sqrt(var + 1e-5));
  }
}

int launch_gn16_finalize(const float* spart, int n, int wps, double m, float* stats, hipStream_t s) {
  hipLaunchKernelGGL(ring_gn_finalize_kernel, dim3(n * 16), dim3(256), 0, s, spart, n, wps, m, stats);
  return check_launch("ring_gn_finalize_kernel");
}

}  // namespace u3d

using namespace u3d;

#ifndef U3D_RING_GB_KR
#define U3D_RING_GB_KR 8  // weight steps in registers beside the fused GroupNorm-backward state
#endif

#ifndef U3D_RING_XN_KR
#define U3D_RING_XN_KR 14
#endif
#ifndef U3D_RING_XN_KR_RES
#define U3D_RING_XN_KR_RES 10
#endif

static int ring_kr(int dflt) {  // RING_KR = 0: no weight steps in registers (experiments)
  const int kr = opt(OPT_RING_KR);
  return kr < 0 ? dflt : kr;
}

static int ring_wgs() { return std::max(1, opt(OPT_RING_WGS)); }  // persistent grid target: one workgroup per CU
static int conv32_ring_impl(int flip, const void* x, int n, int d, int h, int w, const void* wpk,
                            const float* gn_stats, const float* gn_gamma, const float* gn_beta, int gn_groups,
                            const void* residual, void* y, float* stats_out, float* stats_ws, u3d_stream_t stream,
                            float* fstats = nullptr, unsigned* fcnt = nullptr, void* xn = nullptr) {
  U3D_REQUIRE(x && wpk && y && n >= 1 && d >= 1 && h >= 1 && w >= 1, "conv32_ring: bad args");
  U3D_REQUIRE(!gn_stats || (gn_gamma && gn_beta && gn_groups > 0 && 32 % gn_groups == 0), "conv32_ring: bad GN");
  U3D_REQUIRE(!stats_out || (gn_stats && stats_ws), "conv32_ring: output statistics need the GN prologue + ws");
  U3D_REQUIRE(!xn || (gn_stats && !flip && xn != x), "conv32_ring: the normalised side output needs the GN prologue");
  RGGeom g{};
  g.n = n; g.d = d; g.h = h; g.w = w;
  g.nbh = cdiv(h, RG_BH); g.nbw = cdiv(w, RG_BW);
  g.pps = (long long)g.nbh * g.nbw * d;
  g.planes = (long long)n * g.pps;
  g.xbytes = (long long)n * d * h * w * 64;
  U3D_REQUIRE(g.xbytes < (1LL << 31), "conv32_ring: tensor of %lld bytes beyond the 2 GiB buffer-offset range",
              g.xbytes);
  // ~256 persistent workgroups, split evenly per sample (no workgroup straddles two samples)
  const long long wps0 = std::max<long long>(1, std::min<long long>(g.pps, ring_wgs() / n));
  g.per = (int)((g.pps + wps0 - 1) / wps0);
  g.wps = (int)((g.pps + g.per - 1) / g.per);
  const long long grid = (long long)n * g.wps;
  g.gn_groups = gn_groups;
  if (stats_out && fcnt && fstats) {
    g.fstats = fstats;
    g.fcnt = fcnt;
  }
  hipStream_t s = (hipStream_t)stream;
  float* sp = stats_out ? stats_ws : nullptr;
#define RG_LAUNCH(F, G, R, K)                                                                                  \
  hipLaunchKernelGGL((conv32_ring_kernel<F, G, R, K>), dim3((unsigned)grid), dim3(RG_NT), 0, s, (const bf16*)x, \
                     (const bf16*)wpk, (bf16*)y, (const bf16*)residual, gn_stats, gn_gamma, gn_beta, sp, g)
#define RG_KR(F, G, R, K)                  \
  do {                                     \
    if (kr) RG_LAUNCH(F, G, R, K);         \
    else RG_LAUNCH(F, G, R, 0);            \
  } while (0)
  U3D_REQUIRE(!(flip && (gn_stats || residual)), "conv32_ring: the data gradient takes no prologue / residual");
  // register budget (2 waves per SIMD): GN + residual holds 12 weight steps, GN 16, the others 27
  const bool kr = ring_kr(1) != 0;
  if (xn) {  // (two weight steps fewer: the side store's offsets)
#define RG_XN(R, K)                                                                                                 \
  hipLaunchKernelGGL((conv32_ring_kernel<false, true, R, K, false, true>), dim3((unsigned)grid), dim3(RG_NT), 0, s, \
                     (const bf16*)x, (const bf16*)wpk, (bf16*)y, (const bf16*)residual, gn_stats, gn_gamma, gn_beta, \
                     sp, g, nullptr, (bf16*)xn)
    if (residual) RG_XN(true, U3D_RING_XN_KR_RES);
    else RG_XN(false, U3D_RING_XN_KR);
#undef RG_XN
    return check_launch("conv32_ring_kernel (normalised side output)");
  }
  if (flip) RG_KR(true, false, false, 27);
  else if (gn_stats && residual) RG_KR(false, true, true, 12);  // + the statistics accumulators: 12 steps
  else if (gn_stats) RG_KR(false, true, false, 16);  // (12 measured equal: 124.6 vs 124.8 us)
  else if (residual) RG_KR(false, false, true, 20);
  else RG_KR(false, false, false, 27);
#undef RG_KR
#undef RG_LAUNCH
  return check_launch("conv32_ring_kernel");
}

// ------------------------------------------------------------------------------------------- work-stealing mode
static int ring_sc_env() { return opt(OPT_RING_SC); }  // output planes per sub-chunk (0 = default)

// the static split of conv32_ring_impl (~256 workgroups, ranges of `per` planes never straddling samples), each
// range cut into sub-chunks of about a ninth of it (>= 3 planes); a third when the launch accumulates GroupNorm
// statistics (each sub-chunk boundary costs a per-wave reduction inside the MFMA chain)
static void ring_q_geom(int n, int d, int h, int w, RGGeom& g, bool stats = false) {
  g = RGGeom{};
  g.n = n; g.d = d; g.h = h; g.w = w;
  g.nbh = cdiv(h, RG_BH); g.nbw = cdiv(w, RG_BW);
  g.pps = (long long)g.nbh * g.nbw * d;
  g.planes = (long long)n * g.pps;
  g.xbytes = (long long)n * d * h * w * 64;
  const long long wps0 = std::max<long long>(1, std::min<long long>(g.pps, ring_wgs() / n));
  g.per = (int)((g.pps + wps0 - 1) / wps0);
  g.wps = (int)((g.pps + g.per - 1) / g.per);
  const int env = ring_sc_env();
  // >= 3 planes: a claim's verdict (two steps after its first plane is staged) lands before the next boundary
  const int parts = stats ? 3 : 9;
  g.sc = std::min(g.per, std::max(3, env > 0 ? env : (g.per + parts - 1) / parts));
  g.rmax = (g.per + g.sc - 1) / g.sc;
}


extern "C" int u3d_conv32_ring_q_stats_ws_floats(int n, int d, int h, int w) {
  RGGeom g;
  ring_q_geom(n, d, h, w, g, true);
  return n * g.wps * g.rmax * (RG_NT / 64) * 32;
}

extern "C" int u3d_conv32_ring_q_queue_bytes(int n, int d, int h, int w) {
  RGGeom g;
  ring_q_geom(n, d, h, w, g);
  return 8 * (n * g.wps + 1);
}

extern "C" int u3d_conv32_ring_q(int flip, const void* x, int n, int d, int h, int w, const void* wpk,
                                 const float* gn_stats, const float* gn_gamma, const float* gn_beta, int gn_groups,
                                 const void* residual, void* y, float* stats_ws, int* queue, u3d_stream_t stream) {
  U3D_REQUIRE(x && wpk && y && queue && n >= 1 && d >= 1 && h >= 1 && w >= 1, "conv32_ring_q: bad args");
  U3D_REQUIRE(!gn_stats || (gn_gamma && gn_beta && gn_groups > 0 && 32 % gn_groups == 0), "conv32_ring_q: bad GN");
  U3D_REQUIRE(!stats_ws || gn_stats, "conv32_ring_q: output statistics need the GN prologue");
  U3D_REQUIRE(!(flip && (gn_stats || residual)), "conv32_ring_q: the data gradient takes no prologue / residual");
  RGGeom g;
  ring_q_geom(n, d, h, w, g, stats_ws != nullptr);
  U3D_REQUIRE(g.xbytes < (1LL << 31), "conv32_ring_q: tensor of %lld bytes beyond the 2 GiB buffer-offset range",
              g.xbytes);
  g.gn_groups = gn_groups;
  const unsigned grid = (unsigned)(n * g.wps);
  hipStream_t s = (hipStream_t)stream;
#define RQ_LAUNCH(F, G, R, K)                                                                                     \
  hipLaunchKernelGGL((conv32_ring_kernel<F, G, R, K, true>), dim3(grid), dim3(RG_NT), 0, s, (const bf16*)x, \
                     (const bf16*)wpk, (bf16*)y, (const bf16*)residual, gn_stats, gn_gamma, gn_beta, stats_ws, g, queue)
  // register budget: the claim state costs the weight steps of the static variants a few registers
  if (flip) RQ_LAUNCH(true, false, false, 16);
  else if (gn_stats && residual) RQ_LAUNCH(false, true, true, 4);
  else if (gn_stats) RQ_LAUNCH(false, true, false, 8);
  else if (residual) RQ_LAUNCH(false, false, true, 14);
  else RQ_LAUNCH(false, false, false, 16);
#undef RQ_LAUNCH
  return check_launch("conv32_ring_kernel (work stealing)");
}

// stats[n][16] from the per-(sub-chunk, wave) partials of the work-stealing ring: one 256-thread block per sample,
// each thread sums whole slot rows (16 groups x 2) of its slots in index order (slots of sub-chunks a short last
// range does not have are skipped), then the threads' fp64 rows are combined in a fixed-order LDS tree
__global__ __launch_bounds__(256) void ring_gn_finalize_q_kernel(const float* __restrict__ spart, RGGeom g, double m,
                                                                float* __restrict__ stats) {
  __shared__ double red[256][33];
  const int nn = blockIdx.x, t = threadIdx.x;
  constexpr int NW = RG_NT / 64;
  double acc[32];
#pragma unroll
  for (int e = 0; e < 32; ++e) acc[e] = 0;
  const int per_range = g.rmax * NW, nslot = g.wps * per_range;
  const float* row0 = spart + (long long)nn * nslot * 32;
  for (int i = t; i < nslot; i += 256) {  // independent loads: the slots of all ranges at once
    const int jw = i / per_range, k = (i - jw * per_range) / NW;
    const int len = (int)std::min<long long>(g.per, g.pps - (long long)jw * g.per);
    if (k * g.sc >= len) continue;
    const f32x4* r = reinterpret_cast<const f32x4*>(row0 + (long long)i * 32);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const f32x4 v = r[q];
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[4 * q + e] += v[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 32; ++e) red[t][e] = acc[e];
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (t < st)
#pragma unroll
      for (int e = 0; e < 32; ++e) red[t][e] += red[t + st][e];
    __syncthreads();
  }
  if (t < 16) {
    const double mean = red[0][2 * t] / m;
    double var = red[0][2 * t + 1] / m - mean * mean;
    if (var < 0) var = 0;
    stats[(nn * 16 + t) * 2] = (float)mean;
    stats[(nn * 16 + t) * 2 + 1] = (float)(1.0 / sqrt(var + 1e-5));
  }
}

extern "C" int u3d_conv32_ring_q_stats_finalize(const float* stats_ws, int n, int d, int h, int w, float* stats_out,
                                                u3d_stream_t stream) {
  U3D_REQUIRE(stats_ws && stats_out && n >= 1 && d >= 1 && h >= 1 && w >= 1, "conv32_ring_q_stats_finalize: bad args");
  RGGeom g;
  ring_q_geom(n, d, h, w, g, true);
  hipLaunchKernelGGL(ring_gn_finalize_q_kernel, dim3(n), dim3(256), 0, (hipStream_t)stream, stats_ws, g,
                     2.0 * d * h * w, stats_out);
  return check_launch("ring_gn_finalize_q_kernel");
}

extern "C" int u3d_conv32_ring(int flip, const void* x, int n, int d, int h, int w, const void* wpk,
                               const float* gn_stats, const float* gn_gamma, const float* gn_beta, int gn_groups,
                               const void* residual, void* y, u3d_stream_t stream) {
  return conv32_ring_impl(flip, x, n, d, h, w, wpk, gn_stats, gn_gamma, gn_beta, gn_groups, residual, y, nullptr,
                          nullptr, stream);
}

// Data gradient of conv(relu(gn(x))) with the GroupNorm backward's partial pass in its epilogue: dA = conv^T(dy) is
// stored as by u3d_conv32_ring(flip = 1), and parts[n][wps][32][2] (wps = u3d_conv32_ring_wps(n, d, h, w)) receives
// each workgroup's per-channel (sum g, sum g*xhat), g = dA where the forward prologue's relu passed (u3d_gn_bwd's
// partial pass, groupnorm.hip). u3d_gn_bwd_parts then writes dx. Static schedule only (deterministic partials).
extern "C" int u3d_conv32_ring_wps(int n, int d, int h, int w) {
  if (n < 1 || d < 1 || h < 1 || w < 1) return -1;
  const long long pps = (long long)cdiv(h, RG_BH) * cdiv(w, RG_BW) * d;
  const long long wps0 = std::max<long long>(1, std::min<long long>(pps, ring_wgs() / n));
  const long long per = (pps + wps0 - 1) / wps0;
  return (int)((pps + per - 1) / per);
}

static int ring_dgrad_gn_impl(const void* dy, int n, int d, int h, int w, const void* wpk_dgrad, const void* x,
                              const float* gn_stats, const float* gn_gamma, const float* gn_beta, int gn_groups,
                              void* da, float* parts, float* coef, float* dgamma, float* dbeta, unsigned* cnt,
                              u3d_stream_t stream);

extern "C" int u3d_conv32_ring_dgrad_gn(const void* dy, int n, int d, int h, int w, const void* wpk_dgrad,
                                        const void* x, const float* gn_stats, const float* gn_gamma,
                                        const float* gn_beta, int gn_groups, void* da, float* parts,
                                        u3d_stream_t stream) {
  return ring_dgrad_gn_impl(dy, n, d, h, w, wpk_dgrad, x, gn_stats, gn_gamma, gn_beta, gn_groups, da, parts, nullptr,
                            nullptr, nullptr, nullptr, stream);
}

// Round 5: u3d_conv32_ring_dgrad_gn with the GroupNorm-backward finalize inside the launch (its last-arriving workgroup
// writes coef[n][5][32] and dgamma / dbeta[32] as u3d_gn_bwd_parts' finalize would); follow with u3d_gn_bwd_apply_coef.
// cnt: one ZEROED unsigned, left zeroed.
extern "C" int u3d_conv32_ring_dgrad_gn_fused(const void* dy, int n, int d, int h, int w, const void* wpk_dgrad,
                                              const void* x, const float* gn_stats, const float* gn_gamma,
                                              const float* gn_beta, int gn_groups, void* da, float* parts, float* coef,
                                              float* dgamma, float* dbeta, unsigned* cnt, u3d_stream_t stream) {
  U3D_REQUIRE(coef && cnt && n * 32 * 2 * 8 <= 4 * RG_SS, "conv32_ring_dgrad_gn_fused: bad args");
  return ring_dgrad_gn_impl(dy, n, d, h, w, wpk_dgrad, x, gn_stats, gn_gamma, gn_beta, gn_groups, da, parts, coef,
                            dgamma, dbeta, cnt, stream);
}

static int ring_dgrad_gn_impl(const void* dy, int n, int d, int h, int w, const void* wpk_dgrad, const void* x,
                              const float* gn_stats, const float* gn_gamma, const float* gn_beta, int gn_groups,
                              void* da, float* parts, float* coef, float* dgamma, float* dbeta, unsigned* cnt,
                              u3d_stream_t stream) {
  U3D_REQUIRE(dy && wpk_dgrad && x && da && parts && n >= 1 && d >= 1 && h >= 1 && w >= 1,
              "conv32_ring_dgrad_gn: bad args");
  U3D_REQUIRE(gn_stats && gn_gamma && gn_beta && gn_groups > 0 && 32 % gn_groups == 0, "conv32_ring_dgrad_gn: bad GN");
  RGGeom g{};
  g.n = n; g.d = d; g.h = h; g.w = w;
  g.nbh = cdiv(h, RG_BH); g.nbw = cdiv(w, RG_BW);
  g.pps = (long long)g.nbh * g.nbw * d;
  g.planes = (long long)n * g.pps;
  g.xbytes = (long long)n * d * h * w * 64;
  U3D_REQUIRE(g.xbytes < (1LL << 31), "conv32_ring_dgrad_gn: tensor of %lld bytes beyond the 2 GiB buffer-offset range",
              g.xbytes);
  const long long wps0 = std::max<long long>(1, std::min<long long>(g.pps, ring_wgs() / n));
  g.per = (int)((g.pps + wps0 - 1) / wps0);
  g.wps = (int)((g.pps + g.per - 1) / g.per);
  g.gn_groups = gn_groups;
  if (cnt) {
    g.fcnt = cnt;
    g.coef = coef;
    g.dgamma = dgamma;
    g.dbeta = dbeta;
  }
  const long long grid = (long long)n * g.wps;
  const bool kr = ring_kr(1) != 0;
#define RG_GB(K)                                                                                               \
  hipLaunchKernelGGL((conv32_ring_kernel<true, true, false, K>), dim3((unsigned)grid), dim3(RG_NT), 0,         \
                     (hipStream_t)stream, (const bf16*)dy, (const bf16*)wpk_dgrad, (bf16*)da, (const bf16*)x,  \
                     gn_stats, gn_gamma, gn_beta, parts, g)
  if (kr) RG_GB(U3D_RING_GB_KR);
  else RG_GB(0);
#undef RG_GB
  return check_launch("conv32_ring_dgrad_gn");
}

extern "C" int u3d_conv32_ring_stats_ws_floats(int n) { return 64 * std::max(256, n); }

extern "C" int u3d_conv32_ring_stats(const void* x, int n, int d, int h, int w, const void* wpk, const float* gn_stats,
                                     const float* gn_gamma, const float* gn_beta, int gn_groups, const void* residual,
                                     void* y, float* stats_ws, u3d_stream_t stream) {
  U3D_REQUIRE(stats_ws, "conv32_ring_stats: null statistics workspace");
  return conv32_ring_impl(0, x, n, d, h, w, wpk, gn_stats, gn_gamma, gn_beta, gn_groups, residual, y, stats_ws,
                          stats_ws, stream);
}

// Round 6: u3d_conv32_ring_stats that also stores the normalised input relu(gn(x)) (bf16 NDHWC, x's shape) to xn,
// for the conv's weight gradient (u3d_conv_wgrad_ring without gn_stats on xn: bitwise the GN form's partials).
extern "C" int u3d_conv32_ring_stats_xn(const void* x, int n, int d, int h, int w, const void* wpk,
                                        const float* gn_stats, const float* gn_gamma, const float* gn_beta,
                                        int gn_groups, const void* residual, void* y, void* xn, float* stats_ws,
                                        u3d_stream_t stream) {
  U3D_REQUIRE(stats_ws && xn && gn_stats, "conv32_ring_stats_xn: null statistics workspace / side output / GN");
  return conv32_ring_impl(0, x, n, d, h, w, wpk, gn_stats, gn_gamma, gn_beta, gn_groups, residual, y, stats_ws,
                          stats_ws, stream, nullptr, nullptr, xn);
}

extern "C" int u3d_conv32_ring_stats_finalize(const float* stats_ws, int n, int d, int h, int w, float* stats_out,
                                              u3d_stream_t stream) {
  U3D_REQUIRE(stats_ws && stats_out && n >= 1 && d >= 1 && h >= 1 && w >= 1, "conv32_ring_stats_finalize: bad args");
  const long long pps = (long long)cdiv(h, RG_BH) * cdiv(w, RG_BW) * d;  // same split as conv32_ring_impl
  const long long wps0 = std::max<long long>(1, std::min<long long>(pps, ring_wgs() / n));
  const long long per = (pps + wps0 - 1) / wps0;
  const int wps = (int)((pps + per - 1) / per);
  hipLaunchKernelGGL(ring_gn_finalize_kernel, dim3(n * 16), dim3(256), 0, (hipStream_t)stream, stats_ws, n, wps,
                     2.0 * d * h * w, stats_out);
  return check_launch("ring_gn_finalize_kernel");
}

// Round 5: u3d_conv32_ring_stats with the statistics finalized by the launch's last-arriving workgroup into stats_out
// (no u3d_conv32_ring_stats_finalize launch). cnt: one ZEROED unsigned, left zeroed.
extern "C" int u3d_conv32_ring_stats_fused(const void* x, int n, int d, int h, int w, const void* wpk,
                                           const float* gn_stats, const float* gn_gamma, const float* gn_beta,
                                           int gn_groups, const void* residual, void* y, float* stats_ws,
                                           float* stats_out, unsigned* cnt, u3d_stream_t stream) {
  U3D_REQUIRE(stats_ws && stats_out && cnt, "conv32_ring_stats_fused: null statistics buffers");
  U3D_REQUIRE(n * 16 <= 4096, "conv32_ring_stats_fused: n too large");
  return conv32_ring_impl(0, x, n, d, h, w, wpk, gn_stats, gn_gamma, gn_beta, gn_groups, residual, y, stats_ws,
                          stats_ws, stream, stats_out, cnt);
}
