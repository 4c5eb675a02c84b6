"""UNet3D (DynConv 8,8,2) on the native executor, forward and backward: trunk + GAP + controller + per-sample
dynamic heads (reference unet3D.py:1659-1664, 1688-1732, 1734-1806).

Forward: trunk -> precls_conv (8 channels, fp32) ; GAP = mean_v relu(GN(16,256)(bottleneck)) ; params =
controller(cat(GAP, onehot(task, 7))) ; logits = 8->8->8->2 MLP per voxel with each sample's own params.
Backward (one autograd Function around the whole model): dynamic-head backward (dh + 162 parameter grads per
sample), controller backward (dW, db, and the GAP's dA broadcast = AdaptiveAvgPool3d backward), GAP GroupNorm
backward into the bottleneck gradient, then the trunk tape with the head gradient. Every value is a libu3d kernel.
"""
import torch

from . import ops, trunk
from ._lib import call, query
from .ddp import current_sink


def _dyn_forward(tape, cfg, x, task_id, P):
    f, bott = tape.trunk(x, cfg)
    head = tape.head(f, cfg)                       # Act: [n, d, h, w, 8] fp32 (precls_conv)
    n, d, h, w, _ = head.t.shape
    b = bott.t
    st = tape.stats(bott, 16)
    feat = torch.empty((n, 256), dtype=torch.float32, device=x.device)
    call("u3d_gn_relu_mean", ops.dt_code(b.dtype), b.data_ptr(), n, 256, b.numel() // (n * 256), 16, st.data_ptr(),
         P["GAP.0.weight"].data_ptr(), P["GAP.0.bias"].data_ptr(), feat.data_ptr(), ops._stream())
    task = task_id.to(device=x.device, dtype=torch.int64).contiguous()
    params = torch.empty((n, 162), dtype=torch.float32, device=x.device)
    wc = P["controller.weight"].reshape(162, 263).contiguous()
    call("u3d_dyn_controller", feat.data_ptr(), n, 256, task.data_ptr(), 7, wc.data_ptr(),
         P["controller.bias"].data_ptr(), 162, params.data_ptr(), ops._stream())
    out = torch.empty((n, d, h, w, 2), dtype=torch.float32, device=x.device)
    call("u3d_dynhead_fwd", head.t.data_ptr(), params.data_ptr(), n, d * h * w, out.data_ptr(), ops._stream())
    return head, bott, st, feat, task, params, wc, out


class _DynFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cfg, dtype, names, x, task_id, *tensors):
        P = dict(zip(names, tensors))
        tape = trunk.Tape(P, dtype, record=True)
        tape.sink = current_sink()
        if tape.sink is not None:
            tape.sink.begin()
        head, bott, st, feat, task, params, wc, out = _dyn_forward(tape, cfg, x, task_id, P)
        ctx.state = (tape, head, bott, st, feat, task, params, wc)
        ctx.names = names
        return out.permute(0, 4, 1, 2, 3)

    @staticmethod
    def backward(ctx, g):
        tape, head, bott, st, feat, task, params, wc = ctx.state
        P = tape.P
        g = g.permute(0, 2, 3, 4, 1).float().contiguous()          # [n, d, h, w, 2]
        n = g.shape[0]
        v = g.numel() // (n * 2)
        # (1) dynamic heads: dh [n, v, 8] and the per-sample parameter gradients [n, 162]
        dh = torch.empty(head.t.shape, dtype=torch.float32, device=g.device)
        nb = query("u3d_dynhead_bwd_blocks", v)
        part = torch.empty((n, nb, 162), dtype=torch.float32, device=g.device)
        dparams = torch.empty((n, 162), dtype=torch.float32, device=g.device)
        call("u3d_dynhead_bwd", head.t.data_ptr(), params.data_ptr(), g.data_ptr(), n, v, dh.data_ptr(),
             part.data_ptr(), dparams.data_ptr(), ops._stream())
        # (2) controller: dW, db; dfeat -> GAP dA broadcast over the bottleneck voxels
        dwc = tape.grad_out("controller.weight", P["controller.weight"])
        dbc = tape.grad_out("controller.bias", P["controller.bias"])
        b = bott.t
        vb = b.numel() // (n * 256)
        dA = torch.empty_like(b)
        call("u3d_dyn_controller_bwd", ops.dt_code(b.dtype), feat.data_ptr(), n, 256, task.data_ptr(), 7,
             wc.data_ptr(), dparams.data_ptr(), 162, dwc.data_ptr(), dbc.data_ptr(), 0, vb, dA.data_ptr(),
             ops._stream())
        tape.grad_done("controller.weight")
        tape.grad_done("controller.bias")
        # (3) GAP GroupNorm + ReLU backward into the bottleneck (fusionConv output) gradient
        dg = tape.grad_out("GAP.0.weight", P["GAP.0.weight"])
        dbb = tape.grad_out("GAP.0.bias", P["GAP.0.bias"])
        bott.grad = ops.gn_bwd(dA, b, st, P["GAP.0.weight"], P["GAP.0.bias"], 16, dgamma=dg, dbeta=dbb)
        tape.grad_done("GAP.0.weight")
        tape.grad_done("GAP.0.bias")
        # (4) trunk + precls head
        tape.backward(head, dh)
        if tape.sink is not None:
            tape.sink.finish()
        grads = [tape.pgrad.get(nm) for nm in ctx.names]
        if tape.sink is not None:
            grads = tape.sink.returned(ctx.names, grads)
        ctx.state = None
        return (None, None, None, None, None, *grads)


def run_unet3d(model, x, task_id):
    ops.require_device(x)
    cfg = model._u3d_cfg
    dtype = trunk.compute_dtype(getattr(model, "compute_dtype", None))
    x = x.float().contiguous()
    named = list(model.named_parameters())
    if torch.is_grad_enabled() and any(p.requires_grad for _, p in named):
        names = [nm for nm, _ in named]
        return _DynFn.apply(cfg, dtype, names, x, task_id, *[p for _, p in named])
    with torch.no_grad():
        tape = trunk.Tape(dict(named), dtype, record=False)
        out = _dyn_forward(tape, cfg, x, task_id, dict(named))[-1]
    return out.permute(0, 4, 1, 2, 3)
