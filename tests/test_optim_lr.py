"""u3d.optim.SGD keeps its learning rate in a device tensor per group (read by a captured step on replay): sync_lr()
rewrites it exactly when param_groups' lr changed (CPU tensors stand in for the device one)."""
import os
import sys

import torch

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "multimodal-pl_amd")]
from u3d.optim import SGD  # noqa: E402


def test_sync_lr_writes_only_changes():
    p = torch.nn.Parameter(torch.zeros(4))
    opt = SGD([p], lr=0.1, momentum=0.9)
    t = opt._lr_tensor(0, opt.param_groups[0], torch.device("cpu"))
    assert t.item() == torch.tensor(0.1).item()
    t.fill_(-1.0)                      # a value sync_lr would overwrite if it wrote
    opt.sync_lr()
    assert t.item() == -1.0            # unchanged lr: no write
    opt.param_groups[0]["lr"] = 0.05
    opt.sync_lr()
    assert t.item() == torch.tensor(0.05).item()
    opt.param_groups[0]["lr"] = 0.05
    t.fill_(-2.0)
    opt.sync_lr()
    assert t.item() == -2.0
