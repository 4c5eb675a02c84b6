"""Autograd Function for the fused partial-label Dice + BCE loss (reference loss_partial.py:59-99)."""
import torch
from torch.utils import _pytree as pytree

from . import ops

MODE_SIGMOID, MODE_SOFTMAX, MODE_IDENTITY = 0, 1, 2


def ndhwc_view(x):
    """[S, C, D, H, W] -> NDHWC-contiguous [S, D, H, W, C] (free when x came from the native head)."""
    y = x.permute(0, 2, 3, 4, 1)
    return y if y.is_contiguous() else y.contiguous()


def class_weights(mask, C, device):
    """mask[0] of the reference (only the first sample's supervision vector is used, loss_partial.py:87)."""
    if mask is None:
        return torch.ones(C, dtype=torch.float32, device=device)
    w = mask[0]
    if not torch.is_tensor(w):
        w = torch.tensor(w)
    if w.numel() < C:
        raise IndexError(f"index {w.numel()} is out of bounds for dimension 0 with size {w.numel()} "
                         f"(mask[0] shorter than the {C} classes, as the reference's weight[i] would fail)")
    return w.reshape(-1)[:C].to(device=device, dtype=torch.float32)


class DeferredLossGrad(torch.Tensor):
    """The partial loss's gradient w.r.t. the trunk's logits, handed back unformed when the logits came straight from
    the streaming head (trunk._TrunkFn tags them): the trunk's backward passes it to the head, whose backward forms the
    loss gradient in registers (ops.head_loss_bwd) — the fp32 dlogits tensor (113 MB at 2 x 96^3 x 16) is never
    written or read. Anything else that touches it (a hook, torch.autograd.grad on the logits, a sum with another
    gradient) goes through __torch_dispatch__, which forms the real gradient first (ops.partial_loss_bwd): every
    reader sees the same values as without the hand-off."""

    @staticmethod
    def __new__(cls, like, make, payload, link):
        shape, stride, dtype, device = like
        r = torch.Tensor._make_wrapper_subclass(cls, shape, strides=stride, dtype=dtype, device=device)
        r._make, r.payload, r.link, r._real = make, payload, link, None
        return r

    def unformed(self):
        return self._real is None

    def materialize(self):
        if self._real is None:
            self._real = self._make()
            self.payload = None
        return self._real

    __torch_function__ = torch._C._disabled_torch_function_impl

    @classmethod
    def __torch_dispatch__(cls, func, types, args=(), kwargs=None):
        def real(t):
            return t.materialize() if isinstance(t, DeferredLossGrad) else t
        return func(*pytree.tree_map(real, args), **pytree.tree_map(real, kwargs or {}))

    def __repr__(self):
        return f"DeferredLossGrad(shape={tuple(self.shape)}, formed={self._real is not None})"


class _PartialLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, weights, mode, uce):
        lg = ndhwc_view(logits.float())
        lab = target.float().contiguous()
        loss, sums = ops.partial_loss_fwd(lg, lab, weights, mode, uce)
        ctx.save_for_backward(lg, lab, weights, sums)
        ctx.mode, ctx.uce = mode, uce
        link = getattr(logits, "_u3d_head_link", None)
        ctx.link = (link if ops.HEAD_LOSS_FUSED and link is not None and mode == MODE_SOFTMAX and int(uce) == 1
                    and lg.shape[-1] == 16 and lg.dtype == torch.float32 else None)
        ctx.like = (tuple(logits.shape), tuple(logits.stride()), logits.dtype, logits.device)
        return loss.reshape(())

    @staticmethod
    def backward(ctx, g):
        lg, lab, weights, sums = ctx.saved_tensors
        go = g.reshape(1).float().contiguous()
        mode, uce = ctx.mode, ctx.uce

        def form():
            return ops.partial_loss_bwd(lg, lab, weights, sums, go, mode, uce).permute(0, 4, 1, 2, 3)
        if ctx.link is not None:
            return DeferredLossGrad(ctx.like, form, (lg, lab, weights, sums, go), ctx.link), None, None, None, None
        return form(), None, None, None, None


def partial_loss(logits, target, weights, mode=MODE_SOFTMAX, uce=True):
    ops.require_device(logits, target)
    if target.shape[0] != logits.shape[0] or target.numel() * logits.shape[1] != logits.numel():
        raise AssertionError(f"predict {tuple(logits.shape)} & target {tuple(target.shape)} shape do not match")
    return _PartialLossFn.apply(logits, target, weights, mode, uce)


# ------------------------------------------------------------------ consistency branch (losses.py:131-178)
def _voxel_strides(t, lead):
    """Element strides (lead dims..., voxel) of a [*lead, D, H, W] view whose spatial dims are voxel-linear
    (NCDHW or an NCDHW view of NDHWC storage); otherwise a contiguous copy is made."""
    st, sh = t.stride(), t.shape
    d = len(st) - 3
    if st[d + 1] == sh[d + 2] * st[d + 2] and st[d] == sh[d + 1] * st[d + 1]:
        return t, [st[i] for i in range(lead)] + [st[d + 2]]
    t = t.contiguous()
    return t, [t.stride(i) for i in range(lead)] + [1]


def _consist_args(logits, atts, refine, label_t):
    lg, (_, lsc, lsv) = _voxel_strides(logits.float(), 2)
    ref, (rsn, rsc, rsv) = _voxel_strides(refine.detach().float(), 2)
    aa = []
    asc = asv = 0
    for a in atts:
        a2, (_, asc, asv) = _voxel_strides(a.float(), 2)
        aa.append(a2)
    lt = label_t.to(device=logits.device, dtype=torch.float32).contiguous()
    return lg, lsv, lsc, ref, rsn, rsc, rsv, aa, asc, asv, lt


class _ConsistFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, refine, label_t, weight_feature, confi, *atts):
        lg, lsv, lsc, ref, rsn, rsc, rsv, aa, asc, asv, lt = _consist_args(logits, atts, refine, label_t)
        C, nt = lg.shape[1], lt.numel()
        V = lg.numel() // C
        dev = logits.device
        ptr = [a.data_ptr() for a in aa] + [None] * (3 - len(aa))
        aux = torch.empty(1, dtype=torch.float32, device=dev)
        dice = torch.empty((nt, 4), dtype=torch.float32, device=dev)
        coef = torch.empty((nt, 4, 2), dtype=torch.float32, device=dev)
        ws = ops.WS.get(_lib_query("u3d_consistency_ws_bytes", nt), dev, slot=7)
        ops.call("u3d_consistency_fwd", ptr[0], ptr[1], ptr[2], len(aa), asc, asv, lg.data_ptr(), lsv, lsc, C,
                 ref.data_ptr(), rsn, rsc, rsv, lt.data_ptr(), nt, V, float(confi), float(weight_feature),
                 aux.data_ptr(), dice.data_ptr(), coef.data_ptr(), ws.data_ptr(), ops._stream())
        ctx.save_for_backward(lg, ref, lt, coef, *aa)
        ctx.geo = (lsv, lsc, C, rsn, rsc, rsv, nt, V, asc, asv, float(confi), tuple(logits.shape))
        ctx.dice = dice
        return aux.reshape(())

    @staticmethod
    def backward(ctx, g):
        lg, ref, lt, coef, *aa = ctx.saved_tensors
        lsv, lsc, C, rsn, rsc, rsv, nt, V, asc, asv, confi, shape = ctx.geo
        dev = lg.device
        go = g.reshape(1).float().contiguous()
        datt = [torch.empty(a.shape, dtype=torch.float32, device=dev) for a in aa]
        dp = [d.data_ptr() for d in datt] + [None] * (3 - len(aa))
        ap = [a.data_ptr() for a in aa] + [None] * (3 - len(aa))
        n, _, D, H, W = shape
        dl = torch.empty((n, D, H, W, C), dtype=torch.float32, device=dev)
        ops.call("u3d_consistency_bwd", ap[0], ap[1], ap[2], len(aa), asc, asv, lg.data_ptr(), lsv, lsc, C,
                 ref.data_ptr(), rsn, rsc, rsv, lt.data_ptr(), nt, V, confi, coef.data_ptr(), go.data_ptr(),
                 dp[0], dp[1], dp[2], dl.data_ptr(), ops._stream())
        return (dl.permute(0, 4, 1, 2, 3), None, None, None, None, *datt)


def _lib_query(name, *a):
    from ._lib import query
    return query(name, *a)


def consistency_aux(logits, attns, refine, label_t, weight_feature, confi=0.10):
    """aux term of get_loss's refiner branch (losses.py:158-174): one fused pass over the voxels per organ."""
    ops.require_device(logits, refine, *attns)
    if logits.shape[0] != 1:
        raise IndexError("get_loss consistency: the reference indexes the maps with a [1, 1, ...] mask "
                         "(losses.py:167-169), batch must be 1")
    if len(attns) > 3:
        raise ValueError("at most 3 attention maps (unet3D_with_feam3)")
    sp = tuple(logits.shape[2:])
    for a in attns:
        if tuple(a.shape[2:]) != sp:
            raise IndexError(f"The shape of the mask {sp} does not match the shape of the indexed tensor "
                             f"{tuple(a.shape[2:])} (the reference needs deep_up=True maps, losses.py:167-169)")
    return _ConsistFn.apply(logits, refine, label_t, weight_feature, confi, *attns)


class _Full2Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, t, m, sigmoid, uce):
        xc, tc = x.float().contiguous(), t.float().contiguous()
        mc = m.float().contiguous() if m is not None else None
        V = xc.numel()
        loss = torch.empty(1, dtype=torch.float32, device=x.device)
        coef = torch.empty(3, dtype=torch.float32, device=x.device)
        ws = ops.WS.get(128 * 4 * 8, x.device, slot=8)
        ops.call("u3d_edice_full2_fwd", xc.data_ptr(), tc.data_ptr(), mc.data_ptr() if mc is not None else None, V,
                 int(sigmoid), int(uce), loss.data_ptr(), coef.data_ptr(), ws.data_ptr(), ops._stream())
        ctx.save_for_backward(xc, tc, coef, *( [mc] if mc is not None else []))
        ctx.sigmoid, ctx.has_m, ctx.shape = sigmoid, mc is not None, x.shape
        return loss.reshape(())

    @staticmethod
    def backward(ctx, g):
        xc, tc, coef, *mm = ctx.saved_tensors
        dx = torch.empty_like(xc)
        ops.call("u3d_edice_full2_bwd", xc.data_ptr(), tc.data_ptr(), mm[0].data_ptr() if mm else None, xc.numel(),
                 int(ctx.sigmoid), coef.data_ptr(), g.reshape(1).float().contiguous().data_ptr(), dx.data_ptr(),
                 ops._stream())
        return dx.reshape(ctx.shape), None, None, None, None


def edice_full2(inputs, target, uce=True, mask=None, sigmoid=True):
    ops.require_device(inputs, target)
    if inputs.numel() != target.numel() or (mask is not None and mask.numel() != target.numel()):
        raise IndexError(f"EDiceLoss_full2: inputs {tuple(inputs.shape)}, target {tuple(target.shape)}, mask "
                         f"{None if mask is None else tuple(mask.shape)} must cover the same voxels")
    return _Full2Fn.apply(inputs, target, mask, bool(sigmoid), bool(uce))
