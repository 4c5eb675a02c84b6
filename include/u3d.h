/*
 * libu3d — C ABI of the MI355X-native (gfx950 / CDNA4) 3D U-Net segmentation path.
 *
 * Drop-in boundary (SURVEY.md §8b row B'). The reference (TThuraya/multimodal-PL) is pure Python +
 * PyTorch; every entry point below replaces one ATen op (or fused group of ops) that the reference's
 * Python reaches, cited as reference file:line. Callers are the autograd Functions in
 * multimodal-pl_amd/u3d/ (loaded with ctypes); nothing here knows about torch.
 *
 * Conventions
 *  - Activations are NDHWC ("channels-last-3d"), element type `dtype` (U3D_F32 or U3D_BF16), fp32 math.
 *    Logits / loss inputs are fp32 NDHWC. Model input volumes are fp32 NCDHW (as the reference gets them).
 *  - Packed conv weights are [k^3][cout_p][cin_p] (forward) / [k^3][cin_p][cout_p] (data-grad) with
 *    cout_p = round_up(cout, 32), cin_p = round_up(cin, 32), zero padded.
 *  - GroupNorm statistics are float [n][groups][2] = (mean, rstd).
 *  - Every call is asynchronous on `stream` (a hipStream_t; pass torch's current stream). Buffers are
 *    caller-owned; the library never allocates device memory. Workspace sizes come from *_workspace().
 *  - Return 0 on success, else U3D_EINVAL / U3D_EUNSUPPORTED / U3D_EHIP with a thread-local message in
 *    u3d_last_error().
 */
#ifndef U3D_H_
#define U3D_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define U3D_OK 0
#define U3D_EINVAL 1
#define U3D_EUNSUPPORTED 2
#define U3D_EHIP 3

#define U3D_F32 0
#define U3D_BF16 1

typedef void* u3d_stream_t; /* hipStream_t */

const char* u3d_last_error(void);
int u3d_abi_version(void);
/* Host-side tuning options (csrc/common.h enum Opt; names without the U3D_ prefix, e.g. "CONVG_PERSIST"). The defaults
 * are the measured product routing; the environment (U3D_<NAME>) is read once at the first query, for A/B scripts;
 * these two calls change / read a value in-process (tests comparing two routings). No reference counterpart. */
int u3d_set_option(const char* name, int value);
int u3d_get_option(const char* name, int* value);

/* ---------------------------------------------------------------- weight standardisation (A1)
 * Replaces Conv3d.forward's weight.mean(...)/torch.var/div, unet3D.py:21-26, and packs the weight for
 * the implicit-GEMM kernels. standardize=0 packs only (nn.Conv3d of precls_conv, unet3D.py:633). */
int u3d_wstd_fwd(int dtype, const float* w, int cout, int cin, int ksize, int standardize, void* wpk_fwd,
                 void* wpk_dgrad, float* wstats, u3d_stream_t stream);
/* Backward of the above: sums `nsplit` wgrad partial slabs [nsplit][k^3][cout_p][cin_p] (IN PLACE into
 * slab 0) and maps dW_hat -> dW [cout][cin][k^3] through the standardisation (unet3D.py:22-26 autograd). */
int u3d_wstd_bwd(float* dwpk_partials, int nsplit, const float* w, const float* wstats, int cout, int cin,
                 int ksize, int standardize, float* dw, int accumulate, u3d_stream_t stream);

/* Batched forms: every conv of the trunk in one launch (Conv3d.forward of each module, unet3D.py:21-27).
 * Forward uses w, wpk_fwd, wpk_dgrad (nullable), wstats (required when standardize), cout, cin, ksize,
 * standardize. Backward uses part/nsplit (summed in place into slab 0), w, wstats, dw, accumulate. */
typedef struct u3d_wstd_desc {
  const float* w;
  void* wpk_fwd;
  void* wpk_dgrad;
  float* wstats;
  float* part;
  float* dw;
  int cout, cin, ksize, standardize, nsplit, accumulate;
} u3d_wstd_desc;
/* Fused SGD step over up to U3D_SGD_BATCH_MAX fp32 tensors (torch.optim.SGD semantics: d = g (+ wd*p),
 * buf = momentum*buf + (1-dampening)*d (buf = d when init), d = nesterov ? d + momentum*buf : buf, p -= lr*d;
 * maximize negates g). lr is read from device memory (graph-capturable LR changes). Reference: the SGD of
 * train_amos_atlas_final.py:132-135,378. */
typedef struct {
  float* p;
  const float* g;
  float* buf; /* momentum buffer (nullptr when momentum == 0) */
  long long n;
} u3d_sgd_desc;
#define U3D_SGD_BATCH_MAX 48
int u3d_sgd_step(const u3d_sgd_desc* descs, int count, const float* lr, float momentum, float dampening,
                 float weight_decay, int nesterov, int maximize, int init, u3d_stream_t stream);

#define U3D_WSTD_BATCH_MAX 48
int u3d_wstd_fwd_batch(int dtype, const u3d_wstd_desc* descs, int count, u3d_stream_t stream);
/* scratch: device fp32 buffer of u3d_wstd_bwd_scratch_bytes(descs, count) bytes (per-row sums) */
long long u3d_wstd_bwd_scratch_bytes(const u3d_wstd_desc* descs, int count);
int u3d_wstd_bwd_batch(const u3d_wstd_desc* descs, int count, float* scratch, u3d_stream_t stream);
/* Round 5: slab 0 <- the sum of slabs 0..nsplit-1 of ONE weight gradient's partials [nsplit][k3][cout_p][cin_p]
 * (the sum u3d_wstd_bwd_batch runs, same order, bitwise equal), launched right after the weight-gradient kernel so the
 * slabs are re-read from cache; pass nsplit = 1 to the standardisation backward afterwards. */
int u3d_wgrad_sum_slabs(float* part, int nsplit, int k3, int cout, int cin, u3d_stream_t stream);

/* ---------------------------------------------------------------- 3-D convolution (A1-A3, A7)
 * F.conv3d(relu(group_norm(x)), W_hat, bias, stride, pad=k//2) (unet3D.py:27, 44-53, 1640-1657) as one
 * MFMA implicit GEMM: M = output voxels, N = cout, K = k^3 * cin. If gn_stats != NULL the GroupNorm
 * apply + ReLU runs in the operand prologue (zero padding stays zero). residual (same layout as y) is
 * added in the epilogue (NoBottleneck `out + residual`, unet3D.py:71); bias (fp32 [cout]) too.
 * y_f32 != 0 writes fp32 output (logit head) whatever dtype is. ksize in {1,3}; stride in {1,2};
 * cin % 8 == 0 (use u3d_stem_fwd for cin <= 4). ws (nullable, ws_bytes) holds fp32 split-K slabs for
 * deep small-volume layers whose output tiles cannot fill the chip; results are identical either way up
 * to fp32 summation order. */
int u3d_conv_fwd(int dtype, const void* x, int n, int cin, int d, int h, int w, const void* wpk, int cout,
                 int ksize, int stride, const float* gn_stats, const float* gn_gamma, const float* gn_beta,
                 int gn_groups, const void* residual, const float* bias, void* y, int y_f32, float* ws,
                 long long ws_bytes, u3d_stream_t stream);
/* Data gradient: dA = conv_transpose(dy, W_hat) into dA [n][d][h][w][cin] (overwritten), where (d,h,w)
 * is the forward INPUT grid. Stride-2 layers run as 8 parity-class dense sub-convolutions. */
int u3d_conv_dgrad(int dtype, const void* dy, int n, int cout, const void* wpk_dgrad, int cin, int d, int h,
                   int w, int ksize, int stride, void* dx, float* ws, long long ws_bytes, u3d_stream_t stream);
/* Weight gradient partial slabs: partials[s][t][co][ci] = sum over voxel split s of dy * A, with
 * A = relu(gn(x)) recomputed in the prologue (same gn_* as the forward call). */
int u3d_conv_wgrad_splits(int n, int cin, int d, int h, int w, int cout, int ksize, int stride);
int u3d_conv_wgrad(int dtype, const void* dy, const void* x, int n, int cin, int d, int h, int w, int cout,
                   int ksize, int stride, const float* gn_stats, const float* gn_gamma, const float* gn_beta,
                   int gn_groups, float* partials, int nsplit, u3d_stream_t stream);

/* bf16 stride-2 3^3 data gradient in ONE launch (replaces the 8 parity-class launches of u3d_conv_dgrad):
 * dy [n][od][oh][ow][cout] (od = (d-1)/2+1) -> dx [n][d][h][w][cin] (overwritten), wpk = data-grad pack
 * [27][cin_p][cout_p]. Autograd of F.conv3d(stride=2, padding=1) in Conv3d.forward (reference unet3D.py:27). */
int u3d_conv_dgrad_s2(const void* dy, int n, int cout, const void* wpk_dgrad, int cin, int d, int h, int w, void* dx,
                      u3d_stream_t stream);

/* bf16 1^3 convolution, stride 1 or 2 (pad 0): y [n][od][oh][ow][cy] = W . relu(gn(x)) at the input voxel
 * (s*od, s*oh, s*ow); x [n][d][h][w][cx], W = packed [round_up(cy, 32)][wpitch] bf16 (the forward pack of a 1^3
 * weight, wpitch = round_up(cx, 32); or the data-gradient pack [cin_p][cout_p] of a stride-1 1^3 conv, which makes
 * this its data gradient). gn_stats = NULL: no prologue. cx, cy multiples of 8, <= 256. Replaces F.conv3d for the
 * 1^3 downsample / channel-change convs (reference unet3D.py:27 via NoBottleneck :56-73, _make_layer :1666-1686). */
int u3d_conv1x1(const void* x, int n, int cx, int d, int h, int w, const void* wpk, int wpitch, int cy, int stride,
                const float* gn_stats, const float* gn_gamma, const float* gn_beta, int gn_groups, void* y,
                u3d_stream_t stream);

/* bf16 3^3 stride-1 conv for the small deep-level volumes (24^3 and below): one workgroup = a brick of <= 256
 * output voxels x 32 output channels with the whole contraction (no split-K slabs), GN+ReLU prologue applied
 * once per staged element, residual epilogue. flip/wpk/cin/cout as u3d_convg_brick. When there are too few
 * (brick, co tile) pairs to occupy the GPU the contraction is split over workgroups into fp32 partials in ws
 * (ws_bytes; nullptr/0 = no split) summed in fixed order by a second kernel. */
int u3d_conv_small(int flip, const void* x, int n, int cin, int d, int h, int w, const void* wpk, int cout,
                   const float* gn_stats, const float* gn_gamma, const float* gn_beta, int gn_groups,
                   const void* residual, void* y, float* ws, long long ws_bytes, u3d_stream_t stream);

/* Round 5 form of u3d_conv_small: the split-K partials are combined INSIDE the launch by each output tile's
 * last-arriving workgroup (fixed slab order: bitwise the two-kernel result; write-through slab stores, agent-scope
 * arrival counters), and with stats_out (forward, cout in {64, 128, 256}) the output's GroupNorm(16) statistics
 * [n][16][2] = (mean, rstd) from that combine: per-(sample, brick) fp32 partials in spart, fp64 fixed-order finalize
 * by the workgroup completing the last tile. cnt: u3d_conv_small_cnt_bytes bytes, ZERO-FILLED before first use (every
 * launch leaves it zeroed); spart: u3d_conv_small_spart_floats floats. *stats_made = 1 when stats_out was written
 * (it needs the contraction split over 2..8 workgroups); 0: the caller takes u3d_gn_stats. */
long long u3d_conv_small_cnt_bytes(int n, int d, int h, int w, int cout);
long long u3d_conv_small_spart_floats(int n, int d, int h, int w);
int u3d_conv_small2(int flip, const void* x, int n, int cin, int d, int h, int w, const void* wpk, int cout,
                    const float* gn_stats, const float* gn_gamma, const float* gn_beta, int gn_groups,
                    const void* residual, void* y, float* ws, long long ws_bytes, unsigned* cnt, float* spart,
                    float* stats_out, int* stats_made, u3d_stream_t stream);
/* Round 5: data gradient of conv(relu(gn(x))) on the small-volume kernel with the GroupNorm backward's partial sums and
 * its coefficient finalize inside the launch (the split-K combine reads x at dA's addresses; the workgroup completing
 * the last tile writes coef[n][5][cin] and dgamma / dbeta[cin] as gn_bwd_parts_finalize would). cin / cout are the
 * FORWARD conv's channels (dy: cout; x, dx: cin), wpk_dgrad the data-gradient pack. cnt: u3d_conv_small_cnt_bytes(n,
 * d, h, w, cin) ZEROED bytes; parts: u3d_conv_small_gb_parts_floats floats. *made = 0: nothing launched (the launch
 * would not split its contraction); the caller then takes u3d_conv_small + u3d_gn_bwd. Follow with
 * u3d_gn_bwd_apply_coef. Reference: autograd of NoBottleneck's relu(gn(x)) -> conv3x3x3 (unet3D.py:44-73). */
long long u3d_conv_small_gb_parts_floats(int n, int d, int h, int w, int cin);
int u3d_conv_small_dgrad_gn(const void* dy, int n, int cout, int d, int h, int w, const void* wpk_dgrad, int cin,
                            const void* x, const float* gn_stats, const float* gn_gamma, const float* gn_beta,
                            int gn_groups, void* dx, float* ws, long long ws_bytes, unsigned* cnt, float* parts,
                            float* coef, float* dgamma, float* dbeta, int* made, u3d_stream_t stream);
/* the apply pass of the GroupNorm backward from precomputed coefficients coef[n][5][c] (bf16 dA, x, dx) */
int u3d_gn_bwd_apply_coef(const void* da, const void* x, int n, int c, long long v, int groups, const float* coef,
                          void* dx, int accumulate, u3d_stream_t stream);

/* Round 5: 3^3 stride-2 forward conv of relu(gn(x)), bf16, cin 32 -> cout 64 (layer1.0.conv1 at 96^3; reference
 * unet3D.py:45, :56-73) as a persistent walk over input planes: each input plane of a column's halo staged once with the
 * GroupNorm + ReLU applied once per element, both contributions of an odd plane (kd = 2 of output z, kd = 0 of z + 1)
 * from one fragment. wpk = forward pack [27][64][32]. With stats_out the output's GroupNorm(16) statistics [n][16][2]
 * from the epilogue, finalized by the last-arriving workgroup (spart: u3d_conv_s2_ring_ws_floats floats; cnt: one
 * ZEROED unsigned, left zeroed). u3d_conv_s2_ring_ok: 1 where the shape is served (x < 2 GiB, n <= 32). */
int u3d_conv_s2_ring_ok(int n, int cin, int d, int h, int w, int cout);
long long u3d_conv_s2_ring_ws_floats(int n, int d, int h, int w);
int u3d_conv_s2_ring(const void* x, int n, int d, int h, int w, const void* wpk, const float* gn_stats,
                     const float* gn_gamma, const float* gn_beta, int gn_groups, void* y, float* spart, float* stats_out,
                     unsigned* cnt, u3d_stream_t stream);

/* Classifier head precls_conv (unet3D.py:1653-1657): GN+ReLU + 1^3 conv cin (16..64, %16) -> cout (<= 32) + bias,
 * bf16 NDHWC input, fp32 NDHWC logits [n*v][cout]; wpk = forward pack [1][cout_p][cin_p]. Streaming MFMA kernel
 * (operands straight from global memory in fragment layout). */
int u3d_head_fwd(const void* x, int n, long long v, int cin, const void* wpk, int cout, const float* bias,
                 const float* gn_stats, const float* gn_gamma, const float* gn_beta, int gn_groups, float* y,
                 u3d_stream_t stream);
/* Head data gradient in one pass over the fp32 dlogits dy [rows][cout]: dA = dy W (bf16 [rows][cin], wpk_dgrad =
 * [1][cin_p][cout_p] pack), dy_bf16 [rows][round8(cout)] (the weight-gradient operand) and per-block bias-gradient
 * partials dbias_partials [u3d_head_bwd_blocks(rows)][cout] (sum them with u3d_channel_sum). */
int u3d_head_bwd_blocks(long long rows);
int u3d_head_bwd(const float* dy, long long rows, int cout, const void* wpk_dgrad, int cin, void* dA, void* dy_bf16,
                 float* dbias_partials, u3d_stream_t stream);
/* u3d_partial_loss_bwd (softmax, uce 1, C = 16 classes, fp32) fused into u3d_head_bwd on its result (round 5): the
 * loss gradient is formed per voxel in registers and never stored; dA, dy_bf16 and dbias_partials equal the two calls'
 * bit for bit. rows = S * V (the loss's voxel count); logits / labels / weights / sums / grad_out as for
 * u3d_partial_loss_bwd, wpk_dgrad / cin / outputs as for u3d_head_bwd with cout = C.
 * Replaces the pair EDiceLoss_partial.backward (loss_partial.py:59-99 through autograd) -> precls_conv backward
 * (unet3D.py:1653-1657) for the bench's loss. */
int u3d_head_loss_bwd(const float* logits, const float* labels, long long rows, int C, const float* weights,
                      const double* sums, const float* grad_out, const void* wpk_dgrad, int cin, void* dA,
                      void* dy_bf16, float* dbias_partials, u3d_stream_t stream);
/* u3d_head_loss_bwd for n samples of v voxels that also takes the partial sums of the backward of the head's own
 * GroupNorm + ReLU prologue (round 6; x0 bf16 [n][v][cin] = the prologue's input, gn_* its GroupNorm): parts
 * [n][bps][cin][2] = (sum g, sum g * xhat), g = dA where gn(x0) > 0, per block of one sample, for u3d_gn_bwd_parts
 * (nparts = bps = u3d_head_loss_bwd_gn_bps(n, v, cin); 0 = the form does not apply: needs cin = 32, v % 32 == 0).
 * dbias_partials holds n * bps rows; with dbias (nullable; cnt = one zeroed unsigned, left zeroed) the launch's last
 * workgroup sums them into dbias[C] (fixed order). Replaces the pair precls_conv backward -> the GroupNorm backward of its input
 * (unet3D.py:1653-1657 behind the decoder's last GN + ReLU, :1644-1650) as one pass over dA instead of two. */
int u3d_head_loss_bwd_gn_bps(int n, long long v, int cin);
int u3d_head_loss_bwd_gn(const float* logits, const float* labels, int n, long long v, int C, const float* weights,
                         const double* sums, const float* grad_out, const void* wpk_dgrad, int cin, void* dA,
                         void* dy_bf16, float* dbias_partials, const void* x0, const float* gn_stats,
                         const float* gn_gamma, const float* gn_beta, int gn_groups, float* parts, float* dbias,
                         unsigned* cnt, u3d_stream_t stream);

/* bf16 32->32 3^3 stride-1 conv (cin = cout = 32; the full-resolution layers) in halo-brick form with the
 * weights held in registers: flip=0 forward (wpk = forward pack, optional GN+ReLU prologue and residual),
 * flip=1 data gradient (wpk = data-grad pack, no prologue). Same results as u3d_conv_fwd/_dgrad; n <= 16. */
int u3d_conv32_brick(int flip, const void* x, int n, int d, int h, int w, const void* wpk, const float* gn_stats,
                     const float* gn_gamma, const float* gn_beta, int gn_groups, const void* residual, void* y,
                     u3d_stream_t stream);

/* Same operation and arguments as u3d_conv32_brick, depth-streaming schedule (conv_ring.hip): a workgroup walks
 * a range of output planes down d through a 4-plane LDS ring (each input plane staged once, staging overlapped
 * with the MFMAs, one barrier per plane). Any n, d, h, w. */
int u3d_conv32_ring(int flip, const void* x, int n, int d, int h, int w, const void* wpk, const float* gn_stats,
                    const float* gn_gamma, const float* gn_beta, int gn_groups, const void* residual, void* y,
                    u3d_stream_t stream);
/* u3d_conv32_ring forward with the GroupNorm prologue that also accumulates the GroupNorm(16, 32) statistics of
 * its (stored, bf16) output in the epilogue (per-workgroup partials in stats_ws, u3d_conv32_ring_stats_ws_floats(n)
 * floats); u3d_conv32_ring_stats_finalize turns them into (mean, rstd) [n][16][2], eps 1e-5 — so the next GroupNorm
 * (NoBottleneck gn2 / the next block's gn1, unet3D.py:44-53) needs no statistics pass over the output. */
int u3d_conv32_ring_stats_ws_floats(int n);
int u3d_conv32_ring_stats(const void* x, int n, int d, int h, int w, const void* wpk, const float* gn_stats,
                          const float* gn_gamma, const float* gn_beta, int gn_groups, const void* residual, void* y,
                          float* stats_ws, u3d_stream_t stream);
int u3d_conv32_ring_stats_finalize(const float* stats_ws, int n, int d, int h, int w, float* stats_out,
                                   u3d_stream_t stream);
/* Round 6: u3d_conv32_ring_stats that also stores the input after its GroupNorm + ReLU prologue, relu(gn(x)) (bf16
 * NDHWC, x's shape, caller-owned, not aliasing x), to xn — the operand of the conv's weight gradient
 * (unet3D.py:27 F.conv3d's backward w.r.t. the weight, fed by NoBottleneck's relu(gn) :56-73): u3d_conv_wgrad_ring
 * without gn_stats on xn gives bitwise the partials of the GroupNorm form on x, without re-normalising every staged
 * piece. */
int u3d_conv32_ring_stats_xn(const void* x, int n, int d, int h, int w, const void* wpk, const float* gn_stats,
                             const float* gn_gamma, const float* gn_beta, int gn_groups, const void* residual, void* y,
                             void* xn, float* stats_ws, u3d_stream_t stream);
/* Round 5: u3d_conv32_ring_stats with the statistics finalized by the launch's last-arriving workgroup straight into
 * stats_out[n][16][2] (no u3d_conv32_ring_stats_finalize launch; fixed-order fp64 combine, agent-scope arrival counter
 * cnt: one ZEROED unsigned, left zeroed by every launch). */
int u3d_conv32_ring_stats_fused(const void* x, int n, int d, int h, int w, const void* wpk, const float* gn_stats,
                                const float* gn_gamma, const float* gn_beta, int gn_groups, const void* residual,
                                void* y, float* stats_ws, float* stats_out, unsigned* cnt, u3d_stream_t stream);
/* Work-stealing form of u3d_conv32_ring / u3d_conv32_ring_stats (same operation, same outputs bitwise): each
 * workgroup claims the sub-chunks of its static range of output planes front to back and, once done, steals
 * sub-chunks from the back of other ranges (64-bit compare-and-swap per claim), so workgroups that start late (CUs
 * held by a concurrent kernel, e.g. an RCCL all-reduce overlapping the backward) leave no full-range tail.
 * queue = u3d_conv32_ring_q_queue_bytes(n, d, h, w) bytes of caller-owned device memory, zero on entry; the kernel
 * leaves it zero (one queue per concurrently running launch). stats_ws (nullable; needs the GN prologue) receives
 * per-(sub-chunk, wave) GroupNorm(16) partials of the output, u3d_conv32_ring_q_stats_ws_floats(n, d, h, w)
 * floats, turned into (mean, rstd) [n][16][2] by u3d_conv32_ring_q_stats_finalize (fixed order, fp64:
 * deterministic whatever the assignment). */
int u3d_conv32_ring_q_queue_bytes(int n, int d, int h, int w);
int u3d_conv32_ring_q_stats_ws_floats(int n, int d, int h, int w);
int u3d_conv32_ring_q(int flip, const void* x, int n, int d, int h, int w, const void* wpk, const float* gn_stats,
                      const float* gn_gamma, const float* gn_beta, int gn_groups, const void* residual, void* y,
                      float* stats_ws, int* queue, u3d_stream_t stream);
int u3d_conv32_ring_q_stats_finalize(const float* stats_ws, int n, int d, int h, int w, float* stats_out,
                                     u3d_stream_t stream);
/* Data gradient of conv(relu(gn(x))) (flip = 1 ring, wpk = the data-gradient pack) with the GroupNorm backward's
 * partial pass fused into the epilogue: da = conv^T(dy) exactly as u3d_conv32_ring(1, ...), and parts receives
 * [n][u3d_conv32_ring_wps(n, d, h, w)][32][2] floats = per workgroup and channel (sum g, sum g * xhat), g = da where
 * the forward prologue's relu passed (x = that prologue's input, gn_* = its GroupNorm). u3d_gn_bwd_parts finishes
 * the backward. Replaces u3d_gn_bwd's partial pass over (da, x) (NoBottleneck gn1/gn2 backward, unet3D.py:44-53). */
int u3d_conv32_ring_wps(int n, int d, int h, int w);
int u3d_conv32_ring_dgrad_gn(const void* dy, int n, int d, int h, int w, const void* wpk_dgrad, const void* x,
                             const float* gn_stats, const float* gn_gamma, const float* gn_beta, int gn_groups,
                             void* da, float* parts, u3d_stream_t stream);
/* Round 5: u3d_conv32_ring_dgrad_gn with the GroupNorm-backward finalize inside the launch: its last-arriving workgroup
 * writes the apply coefficients coef[n][5][32] and dgamma / dbeta[32] (as u3d_gn_bwd_parts' finalize would; fixed
 * fp64 order); follow with u3d_gn_bwd_apply_coef. cnt: one ZEROED unsigned, left zeroed. */
int u3d_conv32_ring_dgrad_gn_fused(const void* dy, int n, int d, int h, int w, const void* wpk_dgrad, const void* x,
                                   const float* gn_stats, const float* gn_gamma, const float* gn_beta, int gn_groups,
                                   void* da, float* parts, float* coef, float* dgamma, float* dbeta, unsigned* cnt,
                                   u3d_stream_t stream);
/* Stride-1 3^3 weight gradient, depth-streaming ring schedule (wgrad_ring.hip): same partial-slab contract as
 * u3d_conv_wgrad_brick ([nsplit][27][cout_p][cin_p] fp32, summed by the caller in fixed order); a split is a
 * contiguous range of 16x16-voxel output planes walked down d. */
int u3d_conv_wgrad_ring_splits(int n, int cin, int d, int h, int w, int cout);
/* Split count aimed at `wgs` workgroups instead of one per CU. With wgs = 3 x the CU count the launch is a grid of
 * short plane ranges that the hardware dispatcher hands to whichever CU is free, so a concurrent kernel holding CUs
 * (the data-parallel all-reduce of train_amos_atlas_final.py:375) delays a third of a range, not a whole one; every
 * split still owns a fixed contiguous range and its own slab (deterministic sums), at 3x the slab bytes. */
int u3d_conv_wgrad_ring_splits_target(int n, int cin, int d, int h, int w, int cout, int wgs);
int u3d_conv_wgrad_ring(const void* dy, const void* x, int n, int cin, int d, int h, int w, int cout,
                        const float* gn_stats, const float* gn_gamma, const float* gn_beta, int gn_groups,
                        float* partials, int nsplit, u3d_stream_t stream);

/* bf16 3^3 stride-1 conv for any cin/cout (multiples of 8) in halo-brick form: 4x8x16-voxel bricks x 64-channel
 * co tiles, 32-channel input chunks staged once per brick (GN+ReLU prologue), weights streamed per tap plane.
 * flip/wpk as u3d_conv32_brick (for flip=1, cin/cout are the data-gradient's input/output channels). */
int u3d_convg_brick(int flip, const void* x, int n, int cin, int d, int h, int w, const void* wpk, int cout,
                    const float* gn_stats, const float* gn_gamma, const float* gn_beta, int gn_groups,
                    const void* residual, void* y, u3d_stream_t stream);

/* u3d_convg_brick forward (flip = 0) that also returns the GroupNorm(16) statistics [n][16][2] (mean, rstd) of its
 * output (after the residual add, of the stored bf16 values) — the input of the next GroupNorm in NoBottleneck
 * (unet3D.py:44-53) — from per-unit channel-pair partials accumulated in the persistent kernel's epilogue
 * (stats_ws, >= u3d_convg_brick_stats_ws_floats floats) and a fixed-order fp64 finalize. Replaces the separate
 * statistics pass over y. Requires cout % 32 == 0 and cin <= 256 with a GN prologue. */
long long u3d_convg_brick_stats_ws_floats(int n, int d, int h, int w, int cout);
int u3d_convg_brick_stats(const void* x, int n, int cin, int d, int h, int w, const void* wpk, int cout,
                          const float* gn_stats, const float* gn_gamma, const float* gn_beta, int gn_groups,
                          const void* residual, void* y, float* stats_ws, long long ws_floats, float* stats_out,
                          u3d_stream_t stream);
/* Round 5: u3d_convg_brick_stats with the statistics finalized by the launch's last-arriving workgroup (no separate
 * finalize launch); cnt: one ZEROED unsigned, left zeroed. */
int u3d_convg_brick_stats_fused(const void* x, int n, int cin, int d, int h, int w, const void* wpk, int cout,
                                const float* gn_stats, const float* gn_gamma, const float* gn_beta, int gn_groups,
                                const void* residual, void* y, float* stats_ws, long long ws_floats, float* stats_out,
                                unsigned* cnt, u3d_stream_t stream);

/* Data gradient of conv(relu(gn(x))) for the persistent brick (48^3 / 24^3 levels) with the GroupNorm backward's
 * partial pass (per channel sum g and sum g*xhat, g = relu-mask * dA) taken in its epilogue: dx = dA as
 * u3d_convg_brick(flip = 1), parts[n][nparts][cin][2] per brick for u3d_gn_bwd_parts. cin / cout are the FORWARD
 * conv's (dy has cout channels, x and dx cin); gn_* = the GroupNorm on x (unet3D.py:44-53). nparts =
 * u3d_convg_brick_gn_nparts(...) (0: the persistent kernel does not run this shape; take u3d_convg_brick + u3d_gn_bwd).
 * Replaces the gn_bwd_partial pass of u3d_gn_bwd at these levels (reference: the autograd of F.group_norm after
 * Conv3d, unet3D.py:27, :44-73). */
int u3d_convg_brick_gn_nparts(int n, int cin, int d, int h, int w, int cout);
int u3d_convg_brick_dgrad_gn(const void* dy, int n, int cout, int d, int h, int w, const void* wpk_dgrad, int cin,
                             const void* x, const float* gn_stats, const float* gn_gamma, const float* gn_beta,
                             int gn_groups, void* dx, float* parts, int nparts, u3d_stream_t stream);

/* bf16 3^3 weight gradient in halo-brick form (ds_read_b64_tr_b16 operands, all 27 taps per workgroup);
 * same partial-slab output as u3d_conv_wgrad (nsplit from u3d_conv_wgrad_brick_splits). */
int u3d_conv_wgrad_brick_splits(int n, int cin, int d, int h, int w, int cout, int stride);
int u3d_conv_wgrad_brick(const void* dy, const void* x, int n, int cin, int d, int h, int w, int cout, int stride,
                         const float* gn_stats, const float* gn_gamma, const float* gn_beta, int gn_groups,
                         float* partials, int nsplit, u3d_stream_t stream);

/* bf16 1^3 weight gradient (downsample convs, fusion / classifier heads; stride 1 or 2), same slab layout
 * [nsplit][1][cout_p][cin_p]; streams 512-voxel chunks, memory-bound (nsplit from u3d_conv_wgrad1_splits). */
int u3d_conv_wgrad1_splits(int n, int cin, int d, int h, int w, int cout, int stride);
int u3d_conv_wgrad1(const void* dy, const void* x, int n, int cin, int d, int h, int w, int cout, int stride,
                    const float* gn_stats, const float* gn_gamma, const float* gn_beta, int gn_groups,
                    float* partials, int nsplit, u3d_stream_t stream);

/* Stem conv with cin <= 4 (conv1 1->32, unet3D.py:1632; conv0 2->f stride 2, :1514): fp32 NCDHW input, NDHWC
 * output, direct VALU conv with fp32 input (conv1 1 -> 32 stride 1: packed FMAs with scalar-loaded weights from a
 * contiguous fp32 table written into ws, u3d_stem_fwd_ws_bytes() bytes; ws may be NULL for the other shapes). */
long long u3d_stem_fwd_ws_bytes(void);
int u3d_stem_fwd(int dtype, const float* x, int n, int cin, int d, int h, int w, const void* wpk, int cout,
                 int stride, void* y, void* ws, u3d_stream_t stream);
/* conv1 (bf16, cin 1 -> 32, stride 1) with the output's GroupNorm(16) statistics from its epilogue (round 5): per-block
 * fp32 partials into spart (u3d_stem1_stats_ws_floats floats; 0 = shape not supported: d*h*w must be a multiple of
 * 256), fp64 fixed-order finalize into stats[n][16][2] = (mean, rstd), as u3d_gn_stats computes them. Replaces
 * u3d_stem_fwd + u3d_gn_stats for the trunk's stem (unet3D.py:1632 feeding layer0's GroupNorms, :44-53). */
long long u3d_stem1_stats_ws_floats(int n, int d, int h, int w);
int u3d_stem1_fwd_stats(const float* x, int n, int d, int h, int w, const void* wpk, void* y, void* ws, float* spart,
                        float* stats, u3d_stream_t stream);
/* split count for u3d_stem_wgrad given its dtype/channels (the bf16 1->32 stride-1 stem runs on MFMA) */
int u3d_stem_wgrad_splits2(int dtype, int n, int cin, int d, int h, int w, int cout, int stride);
int u3d_stem_wgrad_splits(int n, int d, int h, int w, int stride);
int u3d_stem_wgrad(int dtype, const void* dy, const float* x, int n, int cin, int d, int h, int w, int cout,
                   int stride, float* partials, int nsplit, u3d_stream_t stream);

/* ---------------------------------------------------------------- GroupNorm (A4) statistics / backward
 * nn.GroupNorm(G, C) statistics (biased variance, eps 1e-5): stats[n][g] = (mean, 1/sqrt(var+eps)).
 * Deterministic: per-block shifted partial sums in fp32, combined in fp64 in fixed order by the last block to
 * finish (one launch). ws (u3d_gn_workspace_bytes) must be ZERO-FILLED when first allocated: its first 256 B
 * hold completion counters that every launch leaves at zero (calls sharing one ws must be stream-ordered). */
long long u3d_gn_workspace_bytes(int n, int c, long long v);
int u3d_gn_stats(int dtype, const void* x, int n, int c, long long v, int groups, float* stats, float* ws,
                 u3d_stream_t stream);
/* y = relu(x * scale + shift) with the GroupNorm affine of `stats`/gamma/beta (unet3D.py:44-53), NDHWC,
 * c % 8 == 0: materialised ahead of the implicit GEMM for small deep-layer activations. */
int u3d_gn_apply(int dtype, const void* x, int n, int c, long long v, int groups, const float* stats,
                 const float* gamma, const float* beta, void* y, u3d_stream_t stream);
/* Backward of relu(group_norm(x)) given dA (grad wrt the ReLU output): dx (+)= ..., dgamma/dbeta (+)= ...
 * Two launches (partial sums + last-block combine into per-(n,c) coefficients; elementwise apply); same ws
 * rules as u3d_gn_stats; n * c <= 2048, <= 64 channels per group. */
int u3d_gn_bwd(int dtype, const void* da, const void* x, int n, int c, long long v, int groups,
               const float* stats, const float* gamma, const float* beta, void* dx, int accumulate,
               float* dgamma, float* dbeta, int accumulate_params, float* ws, u3d_stream_t stream);
/* u3d_gn_bwd (bf16) from per-channel partials already summed by the producer (u3d_conv32_ring_dgrad_gn): parts
 * [n][nparts][c][2] = (sum g, sum g * xhat); a one-block fixed-order fp64 finalize writes the coefficients and
 * dgamma/dbeta, then the same elementwise apply as u3d_gn_bwd. Same ws rules. */
int u3d_gn_bwd_parts(const void* da, const void* x, int n, int c, long long v, int groups, const float* stats,
                     const float* gamma, const float* beta, const float* parts, int nparts, void* dx, int accumulate,
                     float* dgamma, float* dbeta, int accumulate_params, float* ws, u3d_stream_t stream);
/* Backward of two GroupNorm+ReLU consumers of the same x with the same statistics (NoBottleneck gn1 and the
 * downsample GN of a stage's first block, unet3D.py:44-53, :1666-1686): dx (+)= GN-bwd(dA1; gamma1, beta1) +
 * GN-bwd(dA2; gamma2, beta2) in one partial pass and one apply pass; dgamma/dbeta of both (+= when acc). */
int u3d_gn_bwd2(int dtype, const void* da1, const void* da2, const void* x, int n, int c, long long v, int groups,
                const float* stats, const float* gamma1, const float* beta1, const float* gamma2, const float* beta2,
                void* dx, int accumulate, float* dgamma1, float* dbeta1, float* dgamma2, float* dbeta2,
                int accumulate_params, float* ws, u3d_stream_t stream);

/* u3d_gn_bwd2 where da2 is the data gradient of a stride-2 1^3 conv (the stage's downsample branch) given at that
 * conv's OUTPUT resolution, da2c [n][(d-1)/2+1][(h-1)/2+1][(w-1)/2+1][c]: it is nonzero only at the x voxels with all
 * coordinates even, so it is neither scattered to the full grid nor zero-filled. x [n][d][h][w][c]. Same semantics
 * as u3d_gn_bwd2 otherwise (backward of gn1 + downsample GN of NoBottleneck, reference unet3D.py:44-73). */
int u3d_gn_bwd2_s2(int dtype, const void* da1, const void* da2c, const void* x, int n, int c, int d, int h, int w,
                   int groups, const float* stats, const float* gamma1, const float* beta1, const float* gamma2,
                   const float* beta2, void* dx, int accumulate, float* dgamma1, float* dbeta1, float* dgamma2,
                   float* dbeta2, int accumulate_params, float* ws, u3d_stream_t stream);

/* ---------------------------------------------------------------- trilinear x2 upsample + skip (A6)
 * nn.Upsample(scale_factor=2, mode='trilinear') (align_corners=False) then `+ skip`
 * (unet3D.py:1646, 1764-1783). x [n][d][h][w][c] -> y [n][2d][2h][2w][c]; skip nullable. */
int u3d_upsample2x_add(int dtype, const void* x, int n, int c, int d, int h, int w, const void* skip, void* y,
                       u3d_stream_t stream);
/* bf16 u3d_upsample2x_add with the output's GroupNorm(16) statistics from its epilogue (round 5): per-block fp32
 * partials into spart (u3d_upsample2x_stats_ws_floats floats; 0 = shape not supported: c/16 in {2,4,8,16}), fp64
 * fixed-order finalize into stats[n][16][2] = (mean, rstd). Replaces upsample + u3d_gn_stats for the decoder input
 * of each x{8,4,2,1}_resb block (unet3D.py:1764-1783 feeding NoBottleneck's GroupNorms :44-53). */
long long u3d_upsample2x_stats_ws_floats(int n, int c, int d, int h, int w);
int u3d_upsample2x_add_stats(const void* x, int n, int c, int d, int h, int w, const void* skip, void* y, float* spart,
                             float* stats, u3d_stream_t stream);
int u3d_upsample2x_bwd(int dtype, const void* dy, int n, int c, int d, int h, int w, void* dx, int accumulate,
                       u3d_stream_t stream);

/* ---------------------------------------------------------------- small elementwise / reductions */
int u3d_add_inplace(int dtype, void* y, const void* x, long long numel, u3d_stream_t stream);
/* Diagnostics (tools/kbench.py, concurrency tests): nwg single-CU workgroups spinning iters dependent FMAs — the
 * one-GPU stand-in for an RCCL all-reduce holding CUs while the backward's persistent kernels run. */
int u3d_diag_occupy(int nwg, long long iters, float* out, u3d_stream_t stream);
/* y[r][c] = c < cin ? x[r][c] : 0, c < cout, converted between U3D_F32 / U3D_BF16 (fp32 logit gradients ->
 * the head's GEMM operand, channel-padded to a multiple of 8) */
int u3d_cast(int dtype_in, const void* x, int dtype_out, void* y, long long rows, int cin, int cout,
             u3d_stream_t stream);
/* out[c] (+)= sum over rows of x[row][c] (conv bias gradient), fp64 combine */
int u3d_channel_sum(int dtype, const void* x, long long rows, int c, float* out, int accumulate, float* ws,
                    u3d_stream_t stream);
long long u3d_channel_sum_workspace_bytes(long long rows, int c);

/* ---------------------------------------------------------------- partial-label Dice + BCE (A10, A11, A13)
 * EDiceLoss_partial(C)(logits, target, mask=[w], soft_max, uce), loss_partial.py:71-99 / DiceLoss :10-57.
 * logits fp32 [S][V][C] (NDHWC), labels fp32 [S][V] (integer-valued), weights fp32 [C] (= mask[0][:C]).
 * sums (fp64 [C][4]) = per class (sum p*t, sum p^2, sum t, sum BCE) over the whole batch; loss fp32[1].
 * uce: 0 = Dice only, 1 = + sum_c w_c BCE_c (EDiceLoss_partial), 2 = + cross entropy of the logits (softmax only;
 * nn.CrossEntropyLoss mean, unweighted: EDiceLoss_full, loss_partial.py:102-135). */
long long u3d_loss_workspace_bytes(int S, long long V, int C);
int u3d_partial_loss_fwd(const float* logits, const float* labels, int S, long long V, int C, int softmax,
                         const float* weights, int uce, double* sums, float* loss, float* ws, u3d_stream_t stream);
/* dlogits (dtype_out, [S][V][C]) = d loss / d logits * grad_out[0] (device scalar) */
int u3d_partial_loss_bwd(int dtype_out, const float* logits, const float* labels, int S, long long V, int C,
                         int softmax, const float* weights, int uce, const double* sums, const float* grad_out,
                         void* dlogits, u3d_stream_t stream);

/* Partial-label target (A12, train_amos_atlas_final.py:252-255): out = labels with every label l in [lmin, lmax]
 * whose mask[s][l] == 0 set to 0; mask int64 [S][mask_stride] (mask_stride 0 = one vector for the batch), length M. */
int u3d_partial_target(const float* labels, int S, long long V, const long long* mask, int mask_stride, int M,
                       int lmin, int lmax, float* out, u3d_stream_t stream);

/* ---------------------------------------------------------------- hard Dice metric (A14)
 * get_dice(preds, labels, t_id, atlas=None, num_class), evaluate_amos.py:128-154 with dice_score :92-102:
 * argmax(softmax(logits)) per voxel; counts[s][l-1] = (sum P*T, sum P, sum T) for l = 1..num_class, and
 * metrics[l-1] = (dice, sensitivity, precision) averaged over samples in fp32 like the reference. */
/* Sliding-window inference (evaluate_amos.py:198-279): full[n][c][D][H][W] += scale * pred * g and (when
 * add_count) count[n][D][H][W] += g for one tile at (d1, y1, x1); pred = the tile's NDHWC fp32 logits [n][td][th][tw][C];
 * g = gd[a] gh[b] gw[e] (each profile max 1), zeros -> gmin; flips bit0/1/2 = the prediction of a d/h/w-flipped
 * input (read mirrored). u3d_window_normalize divides full by count. */
int u3d_window_accumulate(const float* pred, int n, int C, int td, int th, int tw, const float* gd, const float* gh,
                          const float* gw, float gmin, float scale, float* full, float* count, int D, int H, int W,
                          int d1, int y1, int x1, int flips, int add_count, u3d_stream_t stream);
int u3d_window_normalize(float* full, const float* count, int n, int C, long long dhw, u3d_stream_t stream);

int u3d_dice_metric(const float* logits, const float* labels, int S, long long V, int C, int num_class,
                    long long* counts, float* metrics, long long* argmax /* nullable, [S][V] */,
                    u3d_stream_t stream);
/* get_dice2 (evaluate_amos.py:156-182, atlas=None): refine [nt organs][2 classes][V] by element strides (organ
 * rsn, class rsc, voxel rsv), labels [V] (one volume); per organ l the binary prediction argmax(softmax) == 1 vs
 * labels == l+1: counts [nt][3] int64 (TP, P, T), metrics [nt][3] fp32 (dice, sensitivity, precision as
 * dice_score / senc_score / spec_score compute them), argmax [nt][V] int64 (nullable). nt <= 64. */
int u3d_dice_metric_binary(const float* refine, int nt, long long V, long long rsn, long long rsc, long long rsv,
                           const float* labels, long long* counts, float* metrics, long long* argmax,
                           u3d_stream_t stream);

/* ---------------------------------------------------------------- DynConv 8,8,2 head of UNet3D (A8, A9)
 * GAP (unet3D.py:1659-1663): out[n][c] = mean_v relu(group_norm(x))[n][v][c] */
int u3d_gn_relu_mean(int dtype, const void* x, int n, int c, long long v, int groups, const float* stats,
                     const float* gamma, const float* beta, float* out, u3d_stream_t stream);
/* controller (unet3D.py:1664, 1753-1759): params[n] = W cat(feat[n], onehot(task[n], kt)) + b, W [m][kf+kt] */
int u3d_dyn_controller(const float* feat, int n, int kf, const long long* task, int kt, const float* w,
                       const float* b, int m, float* params, u3d_stream_t stream);
/* heads_forward (unet3D.py:1720-1732, 1788-1804): h fp32 [n][v][8] -> out fp32 [n][v][2] */
int u3d_dynhead_fwd(const float* h, const float* params, int n, long long v, float* out, u3d_stream_t stream);
/* DynConv head backward (autograd of heads_forward, unet3D.py:1720-1732): from dlogits [n][v][2] and the head
 * input h [n][v][8] (recomputed MLP): dh [n][v][8] and dparams [n][162] (layout of params; per-block partials
 * part [n][u3d_dynhead_bwd_blocks(v)][162] summed in fixed order). */
int u3d_dynhead_bwd_blocks(long long v);
int u3d_dynhead_bwd(const float* h, const float* params, const float* dlogits, int n, long long v, float* dh,
                    float* part, float* dparams, u3d_stream_t stream);
/* Controller (1^3 conv kf+kt -> m, bias) backward: dw [m][kf+kt], db [m] (+= when accumulate), and the GAP's
 * AdaptiveAvgPool3d backward: dA [n][v][kf] (dtype) = (W^T dparams)[n][k] / v (the GN+ReLU input gradient of the
 * GAP, unet3D.py:1659-1663), ready for u3d_gn_bwd. */
int u3d_dyn_controller_bwd(int dtype, const float* feat, int n, int kf, const long long* task, int kt, const float* w,
                           const float* dparams, int m, float* dw, float* db, int accumulate, long long v, void* dA,
                           u3d_stream_t stream);

/* ---------------------------------------------------------------- unet3D_with_feam3 attention branch (f2)
 * EAM (unet3D.py:142-212) as used by unet3D_with_feam3.forward (:1131-1175): only `attn` = q k^T is kept, averaged
 * over the heads (cattn.mean(1)), which equals sum_c M[t][c] LN2(x_n)[c] with M = (1/h) q Wk.
 * u3d_eam_prep: per token t: zhat = LN3 normalised token (eps 1e-5), q = Wq (zhat g3 + b3), M = inv_heads q Wk
 * (Wk = kv.weight rows 0..c-1). tok/zhat/q/m [nt][c] fp32; wq, wk [c][c]. nt <= 16, c <= 256. */
int u3d_eam_prep(const float* tok, int nt, int c, const float* g3, const float* b3, const float* wq, const float* wk,
                 float inv_heads, float* zhat, float* q, float* m, u3d_stream_t stream);
/* att[n][t][v] (fp32, NCDHW) = sum_c M[t][c] LayerNorm(x[n][v][:]; g2, b2)[c]; x NDHWC dtype, c % 8 == 0 */
int u3d_eam_attn_fwd(int dtype, const void* x, int n, long long v, int c, const float* g2, const float* b2,
                     const float* m, int nt, float* out, u3d_stream_t stream);
/* Backward of u3d_eam_attn_fwd from gout [n][nt][v]: dx (dtype NDHWC, += when accumulate), dM [nt][c], dg2/db2
 * ([c], += when acc_params). part: u3d_eam_attn_bwd_part_floats(...) floats (fixed-order block partials). c in
 * {32, 64, 128}. */
int u3d_eam_attn_bwd_blocks(int n, long long v);
long long u3d_eam_attn_bwd_part_floats(int n, long long v, int c, int nt);
int u3d_eam_attn_bwd(int dtype, const void* x, int n, long long v, int c, const float* g2, const float* b2,
                     const float* m, int nt, const float* gout, void* dx, int accumulate, float* part, float* dm,
                     float* dg2, float* db2, int acc_params, u3d_stream_t stream);
/* Token-side backward: from dM -> dWq [c][c], d(kv.weight) [2c][c] (v half = 0), dg3, db3 (norm3). dq_ws, dz_ws
 * [nt][c] scratch. The token itself is detached (:1134). */
int u3d_eam_param_bwd(const float* dm, int nt, int c, const float* zhat, const float* g3, const float* b3,
                      const float* wq, const float* wk, const float* q, float inv_heads, float* dq_ws, float* dz_ws,
                      float* dwq, float* dkv, float* dg3, float* db3, int accumulate, u3d_stream_t stream);
/* nn.Upsample(scale_factor=s, mode='trilinear'), align_corners=False (unet3D.py:963-965, deep_up maps): NCDHW fp32
 * x [nc][d][h][w] -> y [nc][sd][sh][sw]; backward by three separable gather passes (ws: *_bwd_ws_floats). */
int u3d_upsample_trilinear(const float* x, long long nc, int d, int h, int w, int s, float* y, u3d_stream_t stream);
long long u3d_upsample_trilinear_bwd_ws_floats(long long nc, int d, int h, int w, int s);
int u3d_upsample_trilinear_bwd(const float* dy, long long nc, int d, int h, int w, int s, float* dx, int accumulate,
                               float* ws, u3d_stream_t stream);
/* renew_token (unet3D.py:1051-1068) for one feature level x ([n][v][c] with element strides sv (voxel), sc
 * (channel); batch stride v*c: NDHWC sv=c,sc=1; NCDHW sv=1,sc=v) and the full-size label mask [n][md][mh][mw]
 * (nearest-resized): token[l] (ntok rows of c) <- (1-alpha) token[l] + alpha * mean of row r of x[:,:][mask==l+1]
 * reshaped (c, -1) (B > 1 row quirk kept), for every class l < ncls with selected voxels. ws:
 * u3d_renew_token_ws_bytes. */
long long u3d_renew_token_ws_bytes(int n, int d, int h, int w, int ncls, int c);
int u3d_renew_token(int dtype, const void* x, long long sv, long long sc, int n, int d, int h, int w, int c,
                    const float* mask, int md, int mh, int mw, int ncls, int ntok, float alpha, float* tok, void* ws,
                    u3d_stream_t stream);

/* ---------------------------------------------------------------- consistency branch of get_loss (f2/f3)
 * losses.py:131-178: for every organ g with label_t[g] == 0 and every map k (natt attention maps through a sigmoid,
 * then softmax(logits)[g+1]) the soft Dice vs t = softmax(refine[g])[1] over the refiner-confident voxels
 * (t > 1-confi or t < confi), weighted [0.125,0.25,0.5,1][k] * weight_feature / (nt - supcount). Layouts by element
 * strides: att maps (organ att_sc, voxel att_sv), logits (voxel lsv, class lsc), refine (organ rsn, class rsc,
 * voxel rsv). Outputs: aux[1] (the weighted sum), dice [nt][4], coef [nt][4][2] (for the backward). Batch 1. */
long long u3d_consistency_ws_bytes(int nt);
int u3d_consistency_fwd(const float* att0, const float* att1, const float* att2, int natt, long long att_sc,
                        long long att_sv, const float* logits, long long lsv, long long lsc, int C, const float* refine,
                        long long rsn, long long rsc, long long rsv, const float* label_t, int nt, long long V,
                        float confi, float weight_feature, float* aux, float* dice, float* coef, void* ws,
                        u3d_stream_t stream);
/* gradients (scaled by grad_out[0]): datt_k [nt][V] contiguous, dlogits [V][C] contiguous (NDHWC) */
int u3d_consistency_bwd(const float* att0, const float* att1, const float* att2, int natt, long long att_sc,
                        long long att_sv, const float* logits, long long lsv, long long lsc, int C, const float* refine,
                        long long rsn, long long rsc, long long rsv, const float* label_t, int nt, long long V,
                        float confi, const float* coef, const float* grad_out, float* datt0, float* datt1,
                        float* datt2, float* dlogits, u3d_stream_t stream);
/* EDiceLoss_full2 (loss_partial.py:137-170) on contiguous x, t, m (nullable) of V elements: masked soft dice of
 * sigmoid(x) (or x) vs t, + mean BCEWithLogits(x, t) when uce. ws: 128*4 doubles. coef[3] feeds the backward. */
int u3d_edice_full2_fwd(const float* x, const float* t, const float* m, long long V, int sigmoid, int uce,
                        float* loss, float* coef, void* ws, u3d_stream_t stream);
int u3d_edice_full2_bwd(const float* x, const float* t, const float* m, long long V, int sigmoid, const float* coef,
                        const float* grad_out, float* dx, u3d_stream_t stream);

/* ---------------------------------------------------------------- training data path (f4, MOTSDataset.py)
 * u3d_volume_stats: [mean, population std, min, max] of x[0..V) followed by count - V zeros (the padding of
 * pad_image, which truncate's np.mean / np.std see), fp64, fixed order; ws u3d_volume_stats_ws_bytes.
 * u3d_crop_transpose: out[c][dd][hh][ww] = f(src[c][b0+hh][c0+ww][a0+dd]) (zero outside src = pad_image), f = copy /
 * CT truncate (clip +-325, /325) / MRI (x - stats[0]) / stats[1] (truncate :171-186, crop :364-371, transpose
 * :376-378). u3d_aug_*: the batchgenerators intensity transforms of my_collate (:33-52) with host-drawn
 * parameters: additive Gaussian noise (counter-based RNG), one separable pass of scipy's gaussian_filter ('reflect',
 * fp64 accumulation) along the middle axis of [outer][L][inner], x*mul + add, contrast around the mean with the
 * range preserved (stats from u3d_volume_stats). */
long long u3d_volume_stats_ws_bytes(void);
int u3d_volume_stats(const float* x, long long V, long long count, float* out4, void* ws, u3d_stream_t stream);
int u3d_crop_transpose(const float* src, int C, int sh, int sw, int sd, int b0, int c0, int a0, int ch, int cw, int cd,
                       int mode, const float* stats, float* out, u3d_stream_t stream);
int u3d_aug_noise(float* x, long long V, float sigma, unsigned long long seed, u3d_stream_t stream);
int u3d_aug_blur_axis(const float* x, float* y, long long outer, int L, long long inner, const float* w, int radius,
                      u3d_stream_t stream);
int u3d_aug_affine(float* x, long long V, float mul, float add, u3d_stream_t stream);
int u3d_aug_contrast(float* x, long long V, float factor, const float* stats, int preserve_range,
                     u3d_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* U3D_H_ */
