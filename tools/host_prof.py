"""Host (Python) cost of the eager bench step: cProfile over 10 steps with the autograd engine on the calling thread
(torch.autograd.set_multithreading_enabled(False), so the native tapes' backward closures are profiled too), plus the
host time per step (launch-only, no sync) against the GPU time per step."""
import cProfile
import os
import pstats
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "multimodal-pl_amd")]
import torch  # noqa: E402


def main():
    import bench
    import unet3D
    from loss_functions.loss_partial import EDiceLoss_partial
    from u3d.optim import SGD
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = unet3D.unet3D_baseline([1, 2, 2, 2, 2], num_classes=16, weight_std=True).to(dev).train()
    opt = SGD(model.parameters(), lr=5e-4, momentum=0.9, weight_decay=1e-4)
    x, lab, mask = bench.synthetic(2, 96, dev, 1000, "ct")
    lab = lab.squeeze(1)
    mask = mask.to(dev)
    crit = EDiceLoss_partial(16)

    def step():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            lg, _, _ = model(x)
        loss = crit(lg, lab, mask=[mask])
        loss.backward()
        opt.step()

    torch.autograd.set_multithreading_enabled(False)
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    # host launch time per step (the GPU runs behind; 3 steps keep the queue from filling)
    hs = []
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step()
        hs.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        step()
    e1.record()
    torch.cuda.synchronize()
    print(f"host launch time per step {min(hs) * 1e3:.2f} ms (min of 3); eager wall per step {e0.elapsed_time(e1) / 10:.2f} ms")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(10):
        step()
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(35)
    st.sort_stats("cumulative").print_stats(45)


if __name__ == "__main__":
    main()
