"""Drop-in fused SGD for the native path: torch.optim.SGD's constructor, param_groups, state_dict and update
rule (reference train_amos_atlas_final.py:132-135 builds SGD(lr, momentum=0.9, weight_decay=1e-4); the poly
LR of utils.py:53-60 writes param_groups[0]['lr'] once per epoch), with the whole step in one libu3d launch
per 48 tensors (u3d_sgd_step) instead of torch's 3-5 foreach passes.

The learning rate lives in a one-element device tensor per group, refreshed from param_groups on every step()
call and by sync_lr() — a hipGraph that captured step() reads the current value on replay
(GraphedStep calls sync_lr() before each replay). The tensor is rewritten only when param_groups' lr differs from the
value last written (an unchanged lr cost a fill launch in front of every replay).
"""
import ctypes

import torch

from . import _lib
from .ops import _stream, require_device


class SGD(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, momentum=0, dampening=0, weight_decay=0, nesterov=False, *,
                 maximize=False):
        if lr < 0.0:
            raise ValueError(f"Invalid learning rate: {lr}")
        if momentum < 0.0:
            raise ValueError(f"Invalid momentum value: {momentum}")
        if weight_decay < 0.0:
            raise ValueError(f"Invalid weight_decay value: {weight_decay}")
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                        nesterov=nesterov, maximize=maximize)
        super().__init__(params, defaults)
        self._lr_dev = {}
        self._lr_val = {}  # group -> the lr value last written into its device tensor

    def _write_lr(self, gi, group):
        lr = float(group["lr"])
        if self._lr_val.get(gi) != lr:
            self._lr_dev[gi].fill_(lr)
            self._lr_val[gi] = lr

    def _lr_tensor(self, gi, group, device):
        t = self._lr_dev.get(gi)
        if t is None or t.device != device:
            t = torch.empty((1,), dtype=torch.float32, device=device)
            self._lr_dev[gi] = t
            self._lr_val.pop(gi, None)
            self._write_lr(gi, group)
        return t

    def sync_lr(self):
        """Write every group's current lr into its device tensor where it changed (outside any graph capture)."""
        for gi, group in enumerate(self.param_groups):
            if self._lr_dev.get(gi) is not None:
                self._write_lr(gi, group)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        capturing = torch.cuda.is_current_stream_capturing()
        from . import ops as _ops
        _ops.WEIGHT_GEN[0] += 1          # the native update does not bump autograd versions: invalidate packs
        if capturing:                    # replays update the weights without running this code: no pack cache
            _ops.PACK_CACHE_OK[0] = False
            _ops._PACK_CACHE.clear()
        for gi, group in enumerate(self.param_groups):
            params = [p for p in group["params"] if p.grad is not None]
            if not params:
                continue
            require_device(*params)
            for p in params:
                if p.dtype != torch.float32 or p.grad.dtype != torch.float32 or p.grad.is_sparse or \
                        not p.is_contiguous():
                    raise _lib.U3DError("u3d SGD: fp32 dense parameters and gradients only")
            lr_t = self._lr_tensor(gi, group, params[0].device)
            if not capturing:
                self._write_lr(gi, group)
            mom = float(group["momentum"])
            fresh, old = [], []
            for p in params:  # state only with momentum, as torch.optim.SGD keeps it
                if mom != 0 and self.state[p].get("momentum_buffer") is None:
                    self.state[p]["momentum_buffer"] = torch.empty_like(p)
                    fresh.append(p)
                else:
                    old.append(p)
            for plist, init in ((fresh, 1), (old, 0)):
                for i in range(0, len(plist), _lib.SGD_BATCH_MAX):
                    chunk = plist[i:i + _lib.SGD_BATCH_MAX]
                    descs, keep = [], []  # keep: contiguous copies alive until the launch is queued
                    for p in chunk:
                        g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                        keep.append(g)
                        buf = self.state[p].get("momentum_buffer") if mom != 0 else None
                        descs.append(_lib.SgdDesc(p.data_ptr(), g.data_ptr(),
                                                  buf.data_ptr() if buf is not None else None, p.numel()))
                    arr = (_lib.SgdDesc * len(descs))(*descs)
                    _lib.call("u3d_sgd_step", ctypes.addressof(arr), len(descs), lr_t.data_ptr(), mom,
                              float(group["dampening"]), float(group["weight_decay"]), int(group["nesterov"]),
                              int(group["maximize"]), init, _stream())
        return loss
