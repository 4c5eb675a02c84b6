"""Host-side cost of the eager data-parallel step (RCCL at world 1, forced buckets): wall per step with the GPU
synchronised only at the end, then a cProfile of 5 steps (top cumulative entries). Usage: python tools/ddp_host.py"""
import cProfile
import os
import pstats
import socket
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "multimodal-pl_amd"), REPO]
os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    import unet3D
    from loss_functions.loss_partial import EDiceLoss_partial
    from u3d.ddp import U3DDataParallel
    from u3d.optim import SGD
    torch.manual_seed(0)
    model = unet3D.unet3D_baseline([1, 2, 2, 2, 2], num_classes=16, weight_std=True).to(dev).train()
    net = U3DDataParallel(model, force_buckets=True)
    opt = SGD(model.parameters(), lr=5e-4, momentum=0.9, weight_decay=1e-4)
    crit = EDiceLoss_partial(16)
    x, lab, mask = bench.synthetic(2, 96, dev, 1000)
    lab, mask = lab.squeeze(1), mask.to(dev)

    def step():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            lg, _, _ = net(x)
        loss = crit(lg, lab, mask=[mask])
        loss.backward()
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host {1e3 * (t1 - t0) / 10:.3f} ms/step issued, wall {1e3 * (t2 - t0) / 10:.3f} ms/step; "
          f"flag reads {len(net.bucketer._used)} sets cached")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
