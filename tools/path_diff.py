"""Diagnostic: the sequence of native calls (ops.call names) of the plain bf16 step vs the U3DDataParallel step
(RCCL world 1, forced buckets; PD_HOLD=1: the DDP_TOLERANT latch), and the gradient differences."""
import os
import socket
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "multimodal-pl_amd"), os.path.join(R, "tests")]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
from test_gpu_ddp import MASK, _build  # noqa: E402


def main():
    from loss_functions.loss_partial import EDiceLoss_partial
    from oracle.weights_recipe import input_volume, label_volume
    from u3d import _lib, ops
    from u3d.ddp import U3DDataParallel
    dev = torch.device("cuda:0")
    x = torch.from_numpy(input_volume((2, 1, 64, 64, 64), seed=61, kind="ct")).to(dev)
    lab = torch.from_numpy(label_volume((2, 64, 64, 64), 16, seed=62)).to(dev)
    mask = [torch.tensor(MASK)]
    calls = []
    real = _lib.call
    ops.call = lambda name, *a: (calls.append(name), real(name, *a))[1]

    def step(m, net):
        m.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            lg, _, _ = net(x)
        loss = EDiceLoss_partial(16)(lg.float() * m.extra_scale, lab, mask=mask)
        loss.backward()
        torch.cuda.synchronize()
        return {k: p.grad.detach().double().clone() for k, p in m.named_parameters()}

    m = _build(dev)
    g0 = step(m, m)
    c0 = list(calls)
    calls.clear()
    if os.environ.get("PD_HOLD", "1") == "1":
        ops.DDP_TOLERANT[0] = True
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    m2 = _build(dev)
    net = U3DDataParallel(m2, bucket_mb=1.0, force_buckets=True)
    g1 = step(m2, net)
    dist.destroy_process_group()
    c1 = list(calls)
    import difflib
    diff = [d for d in difflib.unified_diff(c0, c1, lineterm="", n=2)]
    print(f"plain: {len(c0)} calls, ddp: {len(c1)} calls; diff lines: {len(diff)}")
    print("\n".join(diff[:200]))
    rel = {k: ((g1[k] - g0[k]).norm() / g0[k].norm().clamp_min(1e-30)).item() for k in g0}
    worst = sorted(rel.items(), key=lambda kv: -kv[1])[:8]
    print("worst:", ", ".join(f"{k} {v:.2e}" for k, v in worst))


if __name__ == "__main__":
    main()
