"""Run-to-run determinism of the native bf16 training step (diagnostic): the same model / batch stepped N times
from the same weights; prints the largest gradient difference between runs per parameter (0 = bitwise)."""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "multimodal-pl_amd"), os.path.join(R, "tests")]
import torch  # noqa: E402
from test_gpu_ddp import MASK, _build  # noqa: E402


def main():
    from loss_functions.loss_partial import EDiceLoss_partial
    from oracle.weights_recipe import input_volume, label_volume
    dev = torch.device("cuda:0")
    x = torch.from_numpy(input_volume((2, 1, 64, 64, 64), seed=61, kind="ct")).to(dev)
    lab = torch.from_numpy(label_volume((2, 64, 64, 64), 16, seed=62)).to(dev)
    mask = [torch.tensor(MASK)]
    m = _build(dev)
    runs = []
    for _ in range(int(os.environ.get("DET_RUNS", "3"))):
        m.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            lg, _, _ = m(x)
        loss = EDiceLoss_partial(16)(lg.float() * m.extra_scale, lab, mask=mask)
        loss.backward()
        torch.cuda.synchronize()
        runs.append({k: p.grad.detach().double().clone() for k, p in m.named_parameters()})
    if os.environ.get("DET_TOGGLE"):  # the same step with one ops flag flipped (ops.<DET_TOGGLE> = not ...)
        from u3d import ops
        setattr(ops, os.environ["DET_TOGGLE"], not getattr(ops, os.environ["DET_TOGGLE"]))
        m.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            lg, _, _ = m(x)
        loss = EDiceLoss_partial(16)(lg.float() * m.extra_scale, lab, mask=mask)
        loss.backward()
        torch.cuda.synchronize()
        runs.append({k: p.grad.detach().double().clone() for k, p in m.named_parameters()})
        print("last run: ops." + os.environ["DET_TOGGLE"], "flipped")
    for i in range(1, len(runs)):
        diffs = {k: ((runs[i][k] - runs[0][k]).norm() / runs[0][k].norm().clamp_min(1e-30)).item() for k in runs[0]}
        worst = sorted(diffs.items(), key=lambda kv: -kv[1])[:6]
        nz = sum(1 for v in diffs.values() if v > 0)
        print(f"run {i} vs 0: {nz} of {len(diffs)} parameters differ; worst:",
              ", ".join(f"{k} {v:.2e}" for k, v in worst), flush=True)


if __name__ == "__main__":
    main()
