"""The end-of-backward weight-gradient batch (u3d_wstd_bwd_batch: slab sum + standardisation backward) of the bench
step, timed alone with its slabs cold (a 1 GiB fill between replays evicts L2 / the Infinity Cache): the slab sets the
step really produces (recorded from one eager step of the bench model). Usage: python tools/r05_slab.py"""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "multimodal-pl_amd"),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")]
import torch  # noqa: E402
from u3d import ops  # noqa: E402

dev = torch.device("cuda:0")
import unet3D  # noqa: E402
from loss_functions.loss_partial import EDiceLoss_partial  # noqa: E402

torch.manual_seed(0)
model = unet3D.unet3D_baseline([1, 2, 2, 2, 2], num_classes=16, weight_std=True).to(dev).train()
crit = EDiceLoss_partial(16)
from bench import synthetic  # noqa: E402
x, lb, mb = synthetic(2, 96, dev, 1000, "ct")
tgt, mask = lb.squeeze(1), mb.to(dev)
rec = []
orig = ops.wstd_bwd_batch


def spy(items):
    rec.append([tuple(it) for it in items])
    return orig(items)


ops.wstd_bwd_batch = spy
with torch.autocast("cuda", dtype=torch.bfloat16):
    logits, _, _ = model(x)
loss = crit(logits, tgt, mask=[mask])
loss.backward()
torch.cuda.synchronize()
ops.wstd_bwd_batch = orig
items = [it for call in rec for it in call]
slab_mb = sum(it[0].numel() * 4 for it in items if it[1] > 1) / 1e6
print(f"{len(rec)} batch call(s), {len(items)} weights, {sum(1 for it in items if it[1] > 1)} with slabs, "
      f"{slab_mb:.1f} MB of slabs; splits: {sorted(set(it[1] for it in items))}")
flush = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
one = [(it[0][:1].clone(), 1) + tuple(it[2:]) for it in items]


def timed(fn, reps=10):
    g = torch.cuda.CUDAGraph()
    fn()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        for _ in range(reps):
            flush.fill_(1)
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


t_f = timed(lambda: None)
t_all = timed(lambda: orig(items))
t_row = timed(lambda: orig(one))
print(f"fill alone {t_f:.1f} us; batch (sum + rows) {t_all - t_f:.1f} us; rows alone (1 slab) {t_row - t_f:.1f} us; "
      f"sum ~{t_all - t_row:.1f} us = {slab_mb / 1e6 / max(t_all - t_row, 1e-3) * 1e6:.2f} TB/s")
