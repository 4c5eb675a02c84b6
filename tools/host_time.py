"""Host enqueue time of the eager bench step vs its GPU time: is the kernel-by-kernel launch path host-bound?
Usage: python tools/host_time.py [steps]"""
import os
import sys
import time

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "multimodal-pl_amd")]
import torch  # noqa: E402
import unet3D  # noqa: E402
from loss_functions.loss_partial import EDiceLoss_partial  # noqa: E402
from u3d.optim import SGD  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
model = unet3D.unet3D_baseline([1, 2, 2, 2, 2], num_classes=16, weight_std=True).to(dev).train()
opt = SGD(model.parameters(), lr=5e-4, momentum=0.9, weight_decay=1e-4)
crit = EDiceLoss_partial(16)
import bench  # noqa: E402  (the bench's own synthetic batch)
x, lb, mb = bench.synthetic(2, 96, dev, 1000, "ct")
target, mask = lb.squeeze(1), mb.to(dev)


def step():
    opt.zero_grad(set_to_none=True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        logits, _, _ = model(x)
    loss = crit(logits, target, mask=[mask])
    loss.backward()
    opt.step()
    return loss


n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
for _ in range(3):
    step()
torch.cuda.synchronize()
t0 = time.perf_counter()
enq = []
for _ in range(n):
    a = time.perf_counter()
    step()
    enq.append(time.perf_counter() - a)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"host enqueue per step {1e3 * sum(enq) / n:.3f} ms (min {1e3 * min(enq):.3f}); wall per step "
      f"{1e3 * (t2 - t0) / n:.3f} ms; drain after enqueue {1e3 * (t2 - t1):.3f} ms")
