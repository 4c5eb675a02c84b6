"""Per-op timing of one training step at 2x96^3 bf16: wraps every u3d.ops entry point with HIP events on
torch's current stream (the stream libu3d launches on) and prints a table by (op, shape)."""
import collections
import functools
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "multimodal-pl_amd")]
import torch  # noqa: E402
from u3d import ops  # noqa: E402

dev = torch.device("cuda:0")
REC = []


def sig(name, args):
    parts = []
    for a in args[:3]:
        if torch.is_tensor(a):
            parts.append("x".join(map(str, a.shape)))
        elif isinstance(a, (int, float)):
            parts.append(str(a))
    return name + "(" + ",".join(parts) + ")"


def wrap(name):
    f = getattr(ops, name)

    @functools.wraps(f)
    def g(*a, **k):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r = f(*a, **k)
        e1.record()
        extra = ""
        if name == "conv_fwd":
            extra = f" k{a[3]} s{a[4]} co{a[2]}"
        if name in ("conv_dgrad",):
            extra = f" k{a[4]} s{a[5]} ci{a[2]}"
        if name in ("conv_wgrad",):
            extra = f" k{a[2]} s{a[3]}"
        REC.append((sig(name, a) + extra, e0, e1))
        return r
    setattr(ops, name, g)


for n in ["conv_fwd", "conv_dgrad", "conv_wgrad", "gn_stats", "gn_bwd", "gn_apply", "upsample2x_add",
          "upsample2x_bwd", "add_", "cast", "channel_sum", "partial_loss_fwd", "partial_loss_bwd", "stem_fwd",
          "stem_wgrad", "wstd_fwd_batch", "wstd_bwd_batch"]:
    wrap(n)

import unet3D  # noqa: E402
from loss_functions.loss_partial import EDiceLoss_partial  # noqa: E402

s = int(sys.argv[1]) if len(sys.argv) > 1 else 96
torch.manual_seed(0)
m = unet3D.unet3D_baseline([1, 2, 2, 2, 2], num_classes=16, weight_std=True).to(dev).train()
opt = torch.optim.SGD(m.parameters(), lr=5e-4, momentum=0.9, weight_decay=1e-4)
crit = EDiceLoss_partial(16)
x = (torch.rand((2, 1, s, s, s), device=dev) * 2 - 1)
t = torch.randint(0, 16, (2, s, s, s), device=dev).float()
mk = torch.ones(16, dtype=torch.long, device=dev)


def step():
    opt.zero_grad(set_to_none=True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        lg, _, _ = m(x)
    loss = crit(lg, t, mask=[mk])
    loss.backward()
    opt.step()


for _ in range(3):
    step()
torch.cuda.synchronize()
NS = 5
REC.clear()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(NS):
    step()
e1.record()
torch.cuda.synchronize()
tot = e0.elapsed_time(e1) / NS
agg = collections.defaultdict(lambda: [0, 0.0])
cat = collections.defaultdict(float)
for k, a, b in REC:
    dt = a.elapsed_time(b) / NS
    agg[k][0] += 1
    agg[k][1] += dt
    cat[k.split("(")[0]] += dt
print(f"step {tot:.3f} ms; ops sum {sum(cat.values()):.3f} ms")
for k, v in sorted(cat.items(), key=lambda kv: -kv[1]):
    print(f"  {v:7.3f} ms  {k}")
print("--- by op/shape")
for k, (n, v) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"  {v * 1e3:8.1f} us  x{n // NS:2d}  {k}")
