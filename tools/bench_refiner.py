"""Refiner training step: unet3D_g([1]*5, num_classes=2, init_filter=24, in_channel=2)
(train_amos_atlas_final.py:120) on B x 2 x 64 x 192 x 192 bf16 (B = organs in tlist), get_loss_refine
(losses.py:46-62) against a synthetic label volume, backward, SGD. Prints one JSON line (voxels/s, ms/step)."""
import argparse
import json
import os
import sys
import time

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(REPO, "multimodal-pl_amd"), REPO]
import torch  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=3)
    p.add_argument("--shape", type=int, nargs=3, default=[64, 192, 192])
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    a = p.parse_args()
    import unet3D
    from loss_functions.losses import get_loss_refine
    from u3d.optim import SGD
    dev = torch.device("cuda:0")
    torch.manual_seed(0)  # random-init weights (the module's own init; nothing from oracle/)
    m = unet3D.unet3D_g([1, 1, 1, 1, 1], num_classes=2, weight_std=True, init_filter=24, in_channel=2)
    m = m.to(dev).train()
    m.compute_dtype = torch.bfloat16
    opt = SGD(m.parameters(), lr=5e-4, momentum=0.9, weight_decay=1e-4)
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.rand((a.batch, 2) + tuple(a.shape), generator=g).to(dev)
    lab = torch.randint(0, 14, (1, 1) + tuple(a.shape), generator=g).float().to(dev)
    dlist = list(range(2, 2 + a.batch))

    def step():
        opt.zero_grad(set_to_none=True)
        out = m(x)
        loss = get_loss_refine(out, lab, dlist, 1)
        loss.backward()
        opt.step()
        return loss

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    vox = a.batch * a.shape[0] * a.shape[1] * a.shape[2]
    print(json.dumps({"metric": "refiner train voxels/sec (unet3D_g f=24 in=2 + get_loss_refine)", "value": vox / dt,
                      "unit": "voxels/s", "ms_per_step": dt * 1e3, "batch": a.batch, "shape": a.shape,
                      "dtype": "bf16", "loss": float(loss.detach()), "data": "synthetic"}))


if __name__ == "__main__":
    main()
