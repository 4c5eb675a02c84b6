"""hipGraph replay of the whole training step (u3d.graph.GraphedStep) does exactly what the eager step does:
same losses, same updated weights, step after step (every kernel re-runs on replay)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(dev, seed=0):
    import unet3D
    from loss_functions.loss_partial import EDiceLoss_partial

    torch.manual_seed(seed)
    m = unet3D.unet3D_baseline([1, 2, 2, 2, 2], num_classes=16, weight_std=True).to(dev).train()
    opt = torch.optim.SGD(m.parameters(), lr=1e-2, momentum=0.9, weight_decay=1e-4)
    return m, opt, EDiceLoss_partial(16)


def _batches(dev, n=4, s=32):
    g = torch.Generator().manual_seed(5)
    out = []
    for _ in range(n):
        x = (torch.rand((2, 1, s, s, s), generator=g) * 2 - 1).to(dev)
        lab = torch.randint(0, 16, (2, s, s, s), generator=g).float().to(dev)
        mask = (torch.rand(16, generator=g) < 0.7).long().to(dev)
        out.append((x, lab, mask))
    return out


@pytest.mark.parametrize("amp", [False, True])
def test_graphed_step_matches_eager(gpu, amp):
    from u3d.graph import GraphedStep

    bs = _batches(gpu)

    def make_step(m, opt, crit, x, t, mk):
        def step():
            opt.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
                lg, _, _ = m(x)
            loss = crit(lg, t, mask=[mk])
            loss.backward()
            opt.step()
            return loss
        return step

    # eager: 3 steps on batch 0 (= the graph's warm-up), then batches 1..3
    mA, oA, cA = _setup(gpu)
    xA, tA, kA = (t.clone() for t in bs[0])
    stepA = make_step(mA, oA, cA, xA, tA, kA)
    for _ in range(3):
        stepA()
    lossA = []
    for b in bs[1:]:
        for dst, src in zip((xA, tA, kA), b):
            dst.copy_(src)
        lossA.append(stepA().item())

    mB, oB, cB = _setup(gpu)
    xB, tB, kB = (t.clone() for t in bs[0])
    g = GraphedStep(make_step(mB, oB, cB, xB, tB, kB), (xB, tB, kB), warmup=3, optimizer=oB)
    lossB = [g(*b).item() for b in bs[1:]]
    torch.cuda.synchronize()
    assert lossA == pytest.approx(lossB, rel=1e-6, abs=1e-7)
    for (n, pa), (_, pb) in zip(mA.named_parameters(), mB.named_parameters()):
        torch.testing.assert_close(pa, pb, rtol=1e-6, atol=1e-7, msg=n)



def test_graphed_step_follows_lr_changes(gpu):
    """A poly-LR style schedule written into param_groups between replays reaches the captured u3d SGD update."""
    from u3d.graph import GraphedStep
    from u3d.optim import SGD

    bs = _batches(gpu)
    sched = [1e-2, 5e-3, 5e-3, 2e-3]

    def setup():
        m, _, crit = _setup(gpu)
        return m, SGD(m.parameters(), lr=1e-2, momentum=0.9, weight_decay=1e-4), crit

    def make_step(m, opt, crit, x, t, mk):
        def step():
            opt.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                lg, _, _ = m(x)
            loss = crit(lg, t, mask=[mk])
            loss.backward()
            opt.step()
            return loss
        return step

    mA, oA, cA = setup()
    xA, tA, kA = (t.clone() for t in bs[0])
    stepA = make_step(mA, oA, cA, xA, tA, kA)
    for _ in range(3):
        stepA()
    for i, b in enumerate(bs[1:] + bs[:1]):
        for dst, src in zip((xA, tA, kA), b):
            dst.copy_(src)
        oA.param_groups[0]["lr"] = sched[i]
        stepA()

    mB, oB, cB = setup()
    xB, tB, kB = (t.clone() for t in bs[0])
    g = GraphedStep(make_step(mB, oB, cB, xB, tB, kB), (xB, tB, kB), warmup=3, optimizer=oB)
    for i, b in enumerate(bs[1:] + bs[:1]):
        oB.param_groups[0]["lr"] = sched[i]
        g(*b)
    torch.cuda.synchronize()
    for (n, pa), (_, pb) in zip(mA.named_parameters(), mB.named_parameters()):
        torch.testing.assert_close(pa, pb, rtol=1e-6, atol=1e-7, msg=n)
