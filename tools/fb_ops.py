"""Diagnostic: which Python call sites issue the device copies / fills of the forced-bucket step (torch.profiler with
stacks over 2 steps after warm-up). Usage: python tools/fb_ops.py [--plain]"""
import collections
import os
import socket
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "multimodal-pl_amd")]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    import bench
    from loss_functions.loss_partial import EDiceLoss_partial
    from u3d.ddp import U3DDataParallel
    from u3d.optim import SGD
    import unet3D
    dev = torch.device("cuda:0")
    plain = "--plain" in sys.argv
    if not plain:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    model = bench.build_model(dev) if hasattr(bench, "build_model") else None
    if model is None:
        model = unet3D.unet3D_baseline([1, 2, 2, 2, 2], num_classes=16, weight_std=True).to(dev).train()
    net = model if plain else U3DDataParallel(model, force_buckets=True)
    opt = SGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    x, lab, mask = bench.synthetic(2, 96, dev, 1000, "ct")
    lab = lab.squeeze(1)
    crit = EDiceLoss_partial(16)

    def step():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            lg, _, _ = net(x)
        loss = crit(lg, lab, mask=[mask.to(dev)])
        loss.backward()
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
        for _ in range(2):
            step()
        torch.cuda.synchronize()
    sites = collections.Counter()
    for ev in prof.events():
        if ev.name in ("aten::copy_", "aten::fill_", "aten::zero_", "aten::zeros", "aten::clone", "aten::contiguous",
                       "aten::to", "aten::_to_copy"):
            st = [f for f in (ev.stack or []) if "torch/" not in f and "<built-in" not in f][:3]
            sites[(ev.name, " < ".join(st))] += 1
    for (name, st), n in sites.most_common(40):
        print(f"{n / 2:6.1f}/step {name:16s} {st}")
    if not plain:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
