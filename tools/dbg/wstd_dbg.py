import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "..", "multimodal-pl_amd")]
import torch
from u3d import ops
torch.manual_seed(5)
gpu = torch.device("cuda:0")
shapes = [(32, 1, 3, True), (32, 32, 3, True), (64, 32, 3, True), (64, 32, 1, True), (320, 256, 3, True),
          (8, 32, 1, False), (24, 40, 3, True)]
ws = [torch.randn(co, ci, k, k, k, device=gpu) * 0.1 + 0.01 for co, ci, k, _ in shapes]
for dt in (torch.float32, torch.bfloat16):
    outs = ops.wstd_fwd_batch([(w, std, ci > 4) for w, (co, ci, k, std) in zip(ws, shapes)], dt)
    for w, (co, ci, k, std), (pf, pd, st) in zip(ws, shapes, outs):
        pf1, pd1, st1 = ops.wstd_fwd(w, dt, std, need_dgrad=ci > 4)
        d = (pf.float() - pf1.float()).abs()
        idx = (d == d.max()).nonzero()[0].tolist()
        print(dt, (co, ci, k, std), "maxdiff", d.max().item(), "at", idx, pf[tuple(idx)].item(), pf1[tuple(idx)].item(),
              "st", None if st is None else (st - st1).abs().max().item())
