"""Native executor for the reference U-Net trunks (unet3D.py): forward records a tape of backward closures,
backward replays it in reverse. Every value is produced by a libu3d kernel; torch provides memory and the
stream. Activations live NDHWC in the compute dtype (fp32 parity mode or bf16 fast mode) with fp32 master
weights; weight standardisation is re-applied from the fp32 master each step (unet3D.py:21-26).

Graph (reference unet3D.forward :1734-1806 / unet3D_baseline.forward :663-718 / unet3D_g.forward :1568-1623):
  stem conv1 (or conv0 s2 -> conv1) -> layer0..4 (NoBottleneck :40-73) -> fusionConv (GN,ReLU,1^3)
  -> 4 x [trilinear x2 + skip -> x{8,4,2,1}_resb] -> precls_conv (GN,ReLU,1^3+bias) [-> x2 upsample (unet3D_g)]
"""
from dataclasses import dataclass

import torch

from . import ops
from .loss import DeferredLossGrad


@dataclass(frozen=True)
class TrunkCfg:
    layers: tuple = (1, 2, 2, 2, 2)
    groups: int = 16          # GroupNorm groups inside NoBottleneck / downsample
    fusion_groups: int = 16
    head_groups: int = 16
    conv0: bool = False       # unet3D_g: stride-2 stem conv0 then a plain conv1
    final_up: bool = False    # unet3D_g: x2 trilinear upsample of the logits
    weight_std: bool = True


class Act:
    """An NDHWC activation, its cached GroupNorm statistics and its accumulated gradient."""
    __slots__ = ("t", "stats", "grad", "gn_pend")

    def __init__(self, t):
        self.t = t
        self.stats = {}
        self.grad = None
        self.gn_pend = None  # the parked (dA, gn, key, compact) of a block's downsample GN until gn1's backward fuses both


class Tape:
    def __init__(self, params, dtype, record):
        self.P = params
        self.dtype = dtype
        self.record = record
        self.packs = {}
        self.pgrad = {}
        self.ops = []
        self.sink = None
        self.std = True
        self.pending = []   # weight grads waiting for the batched standardisation backward

    def prepack(self, plan):
        """Standardise + pack every conv weight of ``plan`` [(key, standardize, need_dgrad)] in one launch."""
        todo = [(k, s, d and self.record) for k, s, d in plan if k not in self.packs and k + ".weight" in self.P]
        res = ops.wstd_fwd_batch([(self.P[k + ".weight"], s, d) for k, s, d in todo], self.dtype)
        for (k, _, _), r in zip(todo, res):
            self.packs[k] = r

    def conv_plan(self, cfg):
        """The convs trunk()/head() run: (key, standardize, need_dgrad). Absent keys are skipped."""
        std = cfg.weight_std
        plan = [("conv0", std, False), ("conv1", std, True)] if cfg.conv0 else [("conv1", std, False)]
        blocks = [f"layer{i}.{b}." for i in range(5) for b in range(cfg.layers[i])]
        blocks += [n + ".0." for n in ("x8_resb", "x4_resb", "x2_resb", "x1_resb")]
        for pre in blocks:
            plan += [(pre + c, std, True) for c in ("conv1", "downsample.2", "conv2")]
        plan += [("fusionConv.2", std, True), ("precls_conv.2", False, True)]
        plan += [(f"deepout{k}.2", False, True) for k in (1, 2, 3)]  # unet3D_with_feam3 deep supervision
        return plan

    def pend_wgrad(self, part, ns, W, st, std, name):
        self.pending.append((part, ns, W, st, std, self.grad_out(name, W), False, name))
        if self.sink is not None:
            self.sink.note_pending(name)  # sets sink.flush_due when the parked gradients complete a DDP bucket

    def flush_wgrads(self):
        """Slab sum + standardisation backward of the pending weight gradients, in one batched launch pair.
        Batched at the end of the backward (or at a DDP bucket boundary): flushing after every conv measured
        7.33 vs 6.61 ms/step (r03, gpurun_out/r03i/flush), the per-conv launches cost more than the Infinity Cache
        residency of the slabs saves; a side-stream flush measured 7.93 vs 7.83 (round 2)."""
        if not self.pending:
            return
        ops.wstd_bwd_batch([p[:7] for p in self.pending])
        names = [p[7] for p in self.pending]
        self.pending = []
        for n in names:
            self.grad_done(n)

    # ------------------------------------------------------------------ helpers
    def packed(self, key, standardize, need_dgrad=True):
        if key not in self.packs:
            self.packs[key] = ops.wstd_fwd(self.P[key + ".weight"], self.dtype, standardize,
                                           need_dgrad and self.record)
        return self.packs[key]

    def stats(self, act, G):
        if G not in act.stats:
            act.stats[G] = ops.gn_stats(act.t, G)
        return act.stats[G]

    def acc_grad(self, act, g):
        if act.grad is None:
            act.grad = g
        else:
            ops.add_(act.grad, g)

    def grad_out(self, name, like):
        """Destination of a parameter gradient: a DDP bucket view when data-parallel, else a fresh tensor."""
        t = self.sink.out(name) if self.sink is not None else None
        if t is None:
            t = torch.empty_like(like)
        self.pgrad[name] = t
        return t

    def grad_done(self, name):
        if self.sink is not None:
            self.sink.done(name)

    # ------------------------------------------------------------------ ops
    def stem(self, x, key, stride):
        """conv with cin <= 4 from the fp32 NCDHW input volume (unet3D.py:1632 / :1514)."""
        W = self.P[key + ".weight"]
        pf, _, st = self.packed(key, self.std, need_dgrad=False)
        y, st16 = ops.stem_fwd_stats(x, pf, W.shape[0], stride, self.dtype)
        out = Act(y)
        if st16 is not None:
            out.stats[16] = st16  # GroupNorm(16) statistics from the conv1 epilogue (layer0's gn1 / gn2 read them)
        if self.record:
            def bwd():
                if out.grad is None:
                    return
                part, ns = ops.stem_wgrad(out.grad, x, stride)
                self.pend_wgrad(part, ns, W, st, self.std, key + ".weight")
            self.ops.append(bwd)
        return out

    def gn_conv(self, x, key, k, stride, gn_key=None, G=0, residual=None, bias=False, out_f32=False,
                standardize=None, pair=None):
        """conv(relu(gn(x))) [+ residual] [+ bias] — Conv3d/conv3x3x3 :16-35 behind GN+ReLU :44-53."""
        std = self.std if standardize is None else standardize
        W = self.P[key + ".weight"]
        cout, cin = W.shape[0], W.shape[1]
        pf, pd, st = self.packed(key, std)
        gn = None
        if gn_key is not None:
            gn = (self.stats(x, G), self.P[gn_key + ".weight"], self.P[gn_key + ".bias"], G)
        b = self.P[key + ".bias"] if bias else None
        head = out_f32 and residual is None and ops.use_head(x.t.dtype, cin, cout, k, stride)
        st16 = None
        xn = None  # relu(gn(x)) stored by the forward ring: the weight gradient's operand (no GN prologue there)
        if head:  # precls_conv: streaming MFMA head (head.hip)
            y = ops.head_fwd(x.t, pf, cout, b, gn)
        elif self.record and b is None and not out_f32 and ops.ring_xn_ok(x.t, cout, k, stride, gn):
            y, st16, xn = ops.conv_fwd_stats_xn(x.t, pf, cout, k, stride, gn,
                                                residual.t if residual is not None else None)
        elif b is None and not out_f32 and residual is None and ops.s2_normalise_once(x.t, cin, cout, k, stride, gn):
            # stride-2 3^3 conv on the implicit GEMM: relu(gn(x)) materialised once (the GEMM's prologue normalised
            # every gathered element, 27/8 times per input element) and reused by the weight gradient
            xn = ops.gn_apply(x.t, *gn)
            y, st16 = ops.conv_fwd_stats(xn, pf, cout, k, stride, None)
        elif gn is not None and b is None and not out_f32 and (cout == 32 or (ops.BRICK_STATS and cout % 32 == 0)):
            y, st16 = ops.conv_fwd_stats(x.t, pf, cout, k, stride, gn, residual.t if residual is not None else None)
        else:
            y = ops.conv_fwd(x.t, pf, cout, k, stride, gn, residual.t if residual is not None else None, b, out_f32)
        out = Act(y)
        if head and cout == 16:
            self.head_out = out  # the partial loss may hand its gradient to this head unformed (_TrunkFn)
        if st16 is not None:
            out.stats[16] = st16  # GroupNorm(16) statistics from the conv epilogue (consumed by the next GN)
        if self.record:
            def bwd():
                dy = out.grad
                if dy is None:
                    if pair == "finish" and x.gn_pend:  # the parked partner still owes its GN backward
                        dA2, gn2, key2, s2c = x.gn_pend.pop()
                        self.gn_bwd_one(x, ops.expand_s2(dA2, x.t.shape[:4]) if s2c else dA2, gn2, key2, G)
                    return
                parts = None  # GroupNorm-backward partials a data-gradient pass took (head or ring epilogue)
                if head:  # dA, bf16 dy and the bias gradient in one pass over the fp32 dlogits
                    db = self.grad_out(key + ".bias", b) if bias else None
                    if isinstance(dy, DeferredLossGrad):  # the loss gradient formed inside the head's pass
                        lg_, lab_, wt_, sums_, go_ = dy.payload
                        assert lg_.data_ptr() == y.data_ptr() and lg_.shape == y.shape, "deferred loss gradient: not this head's logits"
                        if gn is not None and pair is None and ops.head_gn_parts_ok(lg_, x.t, cin, gn):
                            # the prologue GroupNorm's backward partials in the same pass (no partial pass over dA)
                            dA, dyT, parts = ops.head_loss_bwd(lg_, lab_, wt_, sums_, go_, pd, cin, dbias=db,
                                                               x0=x.t, gn=gn)
                        else:
                            dA, dyT = ops.head_loss_bwd(lg_, lab_, wt_, sums_, go_, pd, cin, dbias=db)
                    else:
                        dA, dyT = ops.head_bwd(dy, pd, cin, dbias=db)
                    if bias:
                        self.grad_done(key + ".bias")
                else:
                    if bias:
                        ops.channel_sum(dy, out=self.grad_out(key + ".bias", b))
                        self.grad_done(key + ".bias")
                    if residual is not None:
                        self.acc_grad(residual, dy)
                    dyT = ops.cast(dy, self.dtype, pad_to=8)  # GEMM operand: channels padded to 8 (2-class head)
                if xn is not None:
                    part, ns = ops.conv_wgrad(dyT, xn, k, stride, None)
                else:
                    part, ns = ops.conv_wgrad(dyT, x.t, k, stride, gn)
                if ops.EAGER_SLAB_SUM and ns >= ops.EAGER_SLAB_MIN:
                    part, ns = ops.sum_slabs(part, ns, cout, cin)
                self.pend_wgrad(part, ns, W, st, std, key + ".weight")
                s2c = (gn is not None and pair == "park" and k == 1 and stride == 2 and ops.S2_COMPACT
                       and ops._use_conv1x1(dyT.dtype, dyT.shape[-1], cin, 1, dyT.shape[0])
                       and ops.s2_compact_ok(x.t.shape, cin, dyT.element_size()))
                if gn is not None and not head and pair != "park" and not (pair == "finish" and x.gn_pend):
                    fused = ops.conv_dgrad_gn(dyT, pd, cin, x.t, k, stride, gn,  # GN-bwd partials in the epilogue
                                              dgb=lambda: (self.grad_out(gn_key + ".weight", gn[1]),
                                                           self.grad_out(gn_key + ".bias", gn[2])))
                    if fused is not None:
                        dA, parts = fused
                if parts is not None:
                    pass
                elif s2c:  # kept at the conv's output resolution: the paired GN backward reads it in place
                    dA = ops.conv_dgrad_1x1s2_compact(dyT, pd, cin)
                elif not head:
                    dA = ops.conv_dgrad(dyT, pd, cin, x.t.shape[:4], k, stride)
                if gn is not None and pair == "park":
                    x.gn_pend = [(dA, gn, gn_key, s2c)]  # the block's gn1 backward (runs next) finishes the pair
                elif gn is not None and pair == "finish" and x.gn_pend:
                    dA2, gn2, key2, s2c2 = x.gn_pend.pop()
                    dps = []
                    for key_, g_ in ((gn_key, gn), (key2, gn2)):
                        dps.append((self.grad_out(key_ + ".weight", g_[1]), self.grad_out(key_ + ".bias", g_[2])))
                    x.grad = ops.gn_bwd2(dA, dA2, x.t, gn[0], (gn[1], gn[2]), (gn2[1], gn2[2]), G, dx=x.grad,
                                         accumulate=x.grad is not None, dparams1=dps[0], dparams2=dps[1],
                                         da2_s2=s2c2)
                    for key_ in (gn_key, key2):
                        self.grad_done(key_ + ".weight")
                        self.grad_done(key_ + ".bias")
                elif gn is not None:
                    self.gn_bwd_one(x, dA, gn, gn_key, G, parts)
                else:
                    self.acc_grad(x, dA)
            self.ops.append(bwd)
        return out

    def gn_bwd_one(self, x, dA, gn, gn_key, G, parts=None):
        if isinstance(parts, tuple) and parts[0] == "coef":  # partials, finalize and dgamma / dbeta done in the dgrad
            x.grad = ops.gn_bwd_apply_coef(dA, x.t, parts[1], G, dx=x.grad, accumulate=x.grad is not None)
            self.grad_done(gn_key + ".weight")
            self.grad_done(gn_key + ".bias")
            return
        dg = self.grad_out(gn_key + ".weight", gn[1])
        db = self.grad_out(gn_key + ".bias", gn[2])
        if parts is not None:  # partial sums already taken by the data-gradient ring (ops.conv_dgrad_gn)
            x.grad = ops.gn_bwd_parts(dA, x.t, parts, gn[0], gn[1], gn[2], G, dx=x.grad,
                                      accumulate=x.grad is not None, dgamma=dg, dbeta=db)
        else:
            x.grad = ops.gn_bwd(dA, x.t, gn[0], gn[1], gn[2], G, dx=x.grad,
                                accumulate=x.grad is not None, dgamma=dg, dbeta=db)
        self.grad_done(gn_key + ".weight")
        self.grad_done(gn_key + ".bias")

    def up_add(self, x, skip, stats=False):
        """upsamplex2 (trilinear, align_corners=False) + skip, unet3D.py:1646 / :1764-1783. ``stats``: the output feeds
        GroupNorm(16)s (a decoder block): take its statistics from the upsample's epilogue."""
        if stats:
            y, st16 = ops.upsample2x_add_stats(x.t, skip.t if skip is not None else None)
            out = Act(y)
            if st16 is not None:
                out.stats[16] = st16
        else:
            out = Act(ops.upsample2x_add(x.t, skip.t if skip is not None else None))
        if self.record:
            def bwd():
                dy = out.grad
                if dy is None:
                    return
                if skip is not None:
                    self.acc_grad(skip, dy)
                x.grad = ops.upsample2x_bwd(dy, tuple(x.t.shape), dx=x.grad, accumulate=x.grad is not None)
            self.ops.append(bwd)
        return out

    def block(self, x, pre, stride, G):
        """NoBottleneck.forward, unet3D.py:56-73."""
        # gn1 and the downsample GN read x with the same statistics: their backward runs as one fused pass (the
        # downsample's backward runs first in the reversed tape and parks its dA, gn1's finishes the pair)
        pair = pre + "downsample.2.weight" in self.P and ops.GN_BWD_PAIRS
        h = self.gn_conv(x, pre + "conv1", 3, stride, gn_key=pre + "gn1", G=G, pair="finish" if pair else None)
        if pre + "downsample.2.weight" in self.P:
            r = self.gn_conv(x, pre + "downsample.2", 1, stride, gn_key=pre + "downsample.0", G=G,
                             pair="park" if pair else None)
        else:
            r = x
        return self.gn_conv(h, pre + "conv2", 3, 1, gn_key=pre + "gn2", G=G, residual=r)

    # ------------------------------------------------------------------ graph
    def trunk(self, x, cfg):
        self.std = cfg.weight_std
        self.prepack(self.conv_plan(cfg))
        if cfg.conv0:
            t = self.stem(x, "conv0", 2)
            t = self.gn_conv(t, "conv1", 3, 1)
        else:
            t = self.stem(x, "conv1", 1)
        skips = []
        for i in range(5):
            for b in range(cfg.layers[i]):
                stride = 2 if (i > 0 and b == 0) else 1
                t = self.block(t, f"layer{i}.{b}.", stride, cfg.groups)
            skips.append(t)
        f = self.gn_conv(t, "fusionConv.2", 1, 1, gn_key="fusionConv.0", G=cfg.fusion_groups)
        bott = f
        self.dec = []  # decoder features after x8/x4/x2/x1_resb (unet3D_with_feam3 heads read the first three)
        for name, s in zip(["x8_resb", "x4_resb", "x2_resb", "x1_resb"], [skips[3], skips[2], skips[1], skips[0]]):
            u = self.up_add(f, s, stats=cfg.groups == 16)
            f = self.block(u, name + ".0.", 1, cfg.groups)
            self.dec.append(f)
        return f, bott

    def head(self, f, cfg):
        lg = self.gn_conv(f, "precls_conv.2", 1, 1, gn_key="precls_conv.0", G=cfg.head_groups, bias=True,
                          out_f32=True, standardize=False)
        if cfg.final_up:
            lg = self.up_add(lg, None)
        return lg

    def backward(self, out_act, grad):
        out_act.grad = grad
        for fn in reversed(self.ops):
            fn()
            if self.sink is not None and self.sink.flush_due:
                self.sink.flush_due = False
                self.flush_wgrads()
        self.flush_wgrads()
        self.ops = []


def compute_dtype(explicit=None):
    """bf16 under torch.autocast('cuda') (the reference's --FP16 amp path), fp32 otherwise."""
    if explicit is not None:
        return explicit
    if torch.is_autocast_enabled("cuda"):
        return torch.bfloat16
    return torch.float32


class _TrunkFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cfg, dtype, names, x, *tensors):
        from .ddp import current_sink
        P = dict(zip(names, tensors))
        tape = Tape(P, dtype, record=True)
        tape.sink = current_sink()
        if tape.sink is not None:
            tape.sink.begin()
        f, _ = tape.trunk(x, cfg)
        lg = tape.head(f, cfg)
        ctx.tape, ctx.out, ctx.names = tape, lg, names
        out = lg.t.permute(0, 4, 1, 2, 3)
        ctx.link = None
        if getattr(tape, "head_out", None) is lg:  # logits straight from the streaming head (no final upsample)
            ctx.link = object()
            out._u3d_head_link = ctx.link  # the partial loss hands its gradient back unformed (loss.DeferredLossGrad)
        return out

    @staticmethod
    def backward(ctx, g):
        tape = ctx.tape
        if isinstance(g, DeferredLossGrad) and ctx.link is not None and g.link is ctx.link and g.unformed():
            tape.backward(ctx.out, g)  # to the head's backward as is (ops.head_loss_bwd)
        else:
            if isinstance(g, DeferredLossGrad):
                g = g.materialize()
            g = g.permute(0, 2, 3, 4, 1)
            if not g.is_contiguous():
                g = g.contiguous()
            tape.backward(ctx.out, g.float())
        if tape.sink is not None:
            tape.sink.finish()
        grads = [tape.pgrad.get(n) for n in ctx.names]
        if tape.sink is not None:
            grads = tape.sink.returned(ctx.names, grads)
        ctx.tape = ctx.out = None
        return (None, None, None, None, *grads)


def run_trunk(cfg, x, named_params, dtype=None):
    """Forward the trunk + classification head. Returns NCDHW-shaped fp32 logits (NDHWC storage)."""
    dtype = compute_dtype(dtype)
    ops.require_device(x)
    if x.dtype != torch.float32 or not x.is_contiguous():
        x = x.float().contiguous()
    names = [n for n, _ in named_params]
    tensors = [p for _, p in named_params]
    if torch.is_grad_enabled() and any(p.requires_grad for p in tensors):
        return _TrunkFn.apply(cfg, dtype, names, x, *tensors)
    with torch.no_grad():
        tape = Tape(dict(zip(names, tensors)), dtype, record=False)
        f, _ = tape.trunk(x, cfg)
        lg = tape.head(f, cfg)
        return lg.t.permute(0, 4, 1, 2, 3)
