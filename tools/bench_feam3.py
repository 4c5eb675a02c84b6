"""Main-model training step of the reference driver: unet3D_with_feam3([1,2,2,2,2],
num_classes=14, weight_std=True, deep_up=True) (train_amos_atlas_final.py:118, run_amos_atlas_final.sh:16) on one
1 x 1 x 64 x 192 x 192 patch per GPU (batch 3 over 3 GPUs in the run), bf16. One step = forward (logits, 3
attention maps upsampled to full size, 3 deep maps, stored features) + get_loss (pre-train: EDiceLoss_partial;
--consistency: + the refiner-consistency branch, losses.py:131-178, against a fixed synthetic refiner output) +
backward + SGD + renew_token (:391). Inputs, the partial-label target and the renew mask are resident before
timing (the driver builds them with host-side torch ops). Prints one JSON line."""
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
    p.add_argument("--shape", type=int, nargs=3, default=[64, 192, 192])
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--consistency", action="store_true")
    a = p.parse_args()
    import unet3D
    from loss_functions.losses import get_loss
    from u3d.optim import SGD
    dev = torch.device("cuda:0")
    nc = 14
    torch.manual_seed(0)  # random-init weights (the module's own init; nothing from oracle/)
    m = unet3D.unet3D_with_feam3([1, 2, 2, 2, 2], num_classes=nc, weight_std=True, deep_up=True)
    m = m.to(dev).train()
    m.compute_dtype = torch.bfloat16
    opt = SGD(m.parameters(), lr=5e-4, momentum=0.9, weight_decay=1e-4)
    g = torch.Generator(device="cpu").manual_seed(0)
    sp = tuple(a.shape)
    x = ((torch.rand((1, 1) + sp, generator=g) * 2000 - 1000).clamp(-325, 325) / 325).to(dev)
    lab = torch.randint(0, nc, (1, 1) + sp, generator=g).float().to(dev)
    mvec = torch.tensor([1, 1, 1, 1, 1, 0, 1, 1, 0, 1, 1, 1, 1, 1, 0], dtype=torch.int64, device=dev)
    label_d = mvec[1:nc].float()
    refine = (torch.randn((nc - 1, 2) + sp, generator=g) * 3).to(dev) if a.consistency else None
    fmask = lab.clone()

    def step():
        opt.zero_grad(set_to_none=True)
        preds, attns, deep, feats = m(x)
        loss, _ = get_loss(preds, 0, [], lab, [mvec], None, attns, refine, label_d if a.consistency else None,
                           weight_feature=0.1)
        loss.backward()
        opt.step()
        m.renew_token(feats, fmask)
        return loss

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    vox = sp[0] * sp[1] * sp[2]
    print(json.dumps({"metric": "feam3 train voxels/sec (unet3D_with_feam3 deep_up + get_loss"
                      + (" + consistency" if a.consistency else " pre-train") + " + bwd + SGD + renew_token)",
                      "value": vox / dt, "unit": "voxels/s", "ms_per_step": dt * 1e3, "shape": list(sp),
                      "dtype": "bf16", "loss": float(loss.detach()), "data": "synthetic"}))


if __name__ == "__main__":
    main()
