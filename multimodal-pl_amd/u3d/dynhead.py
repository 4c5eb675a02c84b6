"""UNet3D (DynConv 8,8,2) forward on the native executor: trunk + GAP + controller + per-sample dynamic
heads (reference unet3D.py:1734-1806). Backward of the dynamic head is a next-round item; training this
model raises instead of silently falling back."""
import torch

from . import ops, trunk
from ._lib import call


class _NoGradDyn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, out, *params):
        return out

    @staticmethod
    def backward(ctx, g):
        raise NotImplementedError("UNet3D DynConv head backward is not built yet (trunk models train natively: "
                                  "unet3D_baseline, unet3D_g)")


def run_unet3d(model, x, task_id):
    ops.require_device(x)
    cfg = model._u3d_cfg
    dtype = trunk.compute_dtype(getattr(model, "compute_dtype", None))
    x = x.float().contiguous()
    P = dict(model.named_parameters())
    with torch.no_grad():
        tape = trunk.Tape(P, dtype, record=False)
        f, bott = tape.trunk(x, cfg)
        head = tape.head(f, cfg)                       # [n, d, h, w, 8] fp32 (precls_conv)
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
    out = out.permute(0, 4, 1, 2, 3)
    if torch.is_grad_enabled() and any(p.requires_grad for p in P.values()):
        out = _NoGradDyn.apply(out, *[p for p in P.values() if p.requires_grad][:1])
    return out
