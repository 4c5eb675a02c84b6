"""Drop-in for the train-step helpers of the reference utils.py (lr_poly :53-54, adjust_learning_rate :56-60,
extant_file :62-70, all_reduce_tensor :72-74, seedfix :116-149, get_logger :43-51)."""
import argparse
import os

import numpy as np
import torch
import torch.distributed as dist


def get_logger(snapshot_path):
    try:
        from tensorboardX import SummaryWriter
    except ImportError:  # tensorboardX is optional; keep the call sites working
        class SummaryWriter:  # noqa: D401
            def __init__(self, *a, **k):
                pass

            def add_scalar(self, *a, **k):
                pass

            def close(self):
                pass
    return SummaryWriter(snapshot_path)


def lr_poly(base_lr, iter, max_iter, power):
    return base_lr * ((1 - float(iter) / max_iter) ** (power))


def adjust_learning_rate(optimizer, i_iter, lr, num_stemps, power):
    """Poly LR on param_groups[0] (set once per epoch in the reference driver, :198)."""
    lr = lr_poly(lr, i_iter, num_stemps, power)
    optimizer.param_groups[0]["lr"] = lr
    return lr


def extant_file(x):
    if not os.path.exists(x):
        raise argparse.ArgumentTypeError("{0} does not exist".format(x))
    return x


def all_reduce_tensor(tensor, world_size=1, norm=True):
    """Mean (norm=True) / sum over ranks when torch.distributed is initialised; the reference's single-process
    stub returns torch.mean(tensor)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        t = tensor.clone()
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        if norm:
            t.div_(dist.get_world_size())
        return t
    return torch.mean(tensor)


def mask_aug(mask, aug_times=2):
    """Reference utils.py:76-114: [B, 1, D, H, W] -> [B * aug_times, 1, D, H, W], each sample repeated aug_times
    times in a row (sample-major). Host-side numpy as in the reference: the output is np.zeros(..., dtype=mask.dtype),
    so a torch tensor argument raises TypeError there exactly as it does in the reference."""
    if aug_times <= 1:
        return mask
    out = np.zeros((mask.shape[0] * aug_times,) + tuple(mask.shape[1:]), dtype=mask.dtype)
    for i in range(mask.shape[0]):
        for j in range(aug_times):
            out[i * aug_times + j] = mask[i]
    return out


def seedfix(seed):
    import random

    import numpy as np

    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False
