"""Debug: per-replay losses of the graphed step vs eager at a given patch size."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "multimodal-pl_amd")]
import torch
import unet3D
from loss_functions.loss_partial import EDiceLoss_partial
from u3d.graph import GraphedStep

dev = torch.device("cuda:0")
s = int(sys.argv[1]) if len(sys.argv) > 1 else 96
amp = True
g = torch.Generator().manual_seed(5)
bs = []
for _ in range(2):
    x = (torch.rand((2, 1, s, s, s), generator=g) * 2 - 1).to(dev)
    lab = torch.randint(0, 16, (2, s, s, s), generator=g).float().to(dev)
    mask = (torch.rand(16, generator=g) < 0.7).long().to(dev)
    bs.append((x, lab, mask))


def run(graph):
    torch.manual_seed(0)
    m = unet3D.unet3D_baseline([1, 2, 2, 2, 2], num_classes=16, weight_std=True).to(dev).train()
    opt = torch.optim.SGD(m.parameters(), lr=5e-4, momentum=0.9, weight_decay=1e-4)
    crit = EDiceLoss_partial(16)
    x, t, k = (u.clone() for u in bs[0])

    def step():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            lg, _, _ = m(x)
        loss = crit(lg, t, mask=[k])
        loss.backward()
        opt.step()
        return loss
    out = []
    if graph:
        gs = GraphedStep(step, (x, t, k), warmup=3, optimizer=opt)
        for i in range(6):
            out.append(gs(*bs[i % 2]).item())
    else:
        for _ in range(3):
            step()
        for i in range(6):
            for d, src in zip((x, t, k), bs[i % 2]):
                d.copy_(src)
            out.append(step().item())
    nan = [n for n, p in m.named_parameters() if not torch.isfinite(p).all()]
    return out, nan[:5]


print("eager", run(False), flush=True)
print("graph", run(True), flush=True)

if len(sys.argv) > 2:
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    import bench
    torch.manual_seed(0)
    m = unet3D.unet3D_baseline([1, 2, 2, 2, 2], num_classes=16, weight_std=True).to(dev).train()
    opt = torch.optim.SGD(m.parameters(), lr=5e-4, momentum=0.9, weight_decay=1e-4)
    crit = EDiceLoss_partial(16)
    x, t, k = (u.clone() for u in bs[0])

    def step():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            lg, _, _ = m(x)
        loss = crit(lg, t, mask=[k])
        loss.backward()
        opt.step()
        return loss
    gs = GraphedStep(step, (x, t, k), warmup=3, optimizer=opt)
    out = gs(*bs[1])
    torch.cuda.synchronize()
    print("before", out.item(), out.data_ptr(), flush=True)
    snap = {n: p.detach().clone() for n, p in m.named_parameters()}
    gsnap = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
    r = bench.dominant_kernel_roofline(dev, 2, s)
    torch.cuda.synchronize()
    print("after", out.item(), flush=True)
    print("param changed", [n for n, p in m.named_parameters() if not torch.equal(p, snap[n])][:5])
    print("grad changed", [n for n, p in m.named_parameters() if not torch.equal(p.grad, gsnap[n])][:5])
    from u3d import ops
    print({k: (v.data_ptr(), v.numel()) for k, v in ops.WS.buf.items()})
