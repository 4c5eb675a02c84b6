"""u3d.optim.SGD (one fused launch per 48 tensors) against torch.optim.SGD: same update rule, momentum buffer
initialisation, weight decay, nesterov/dampening/maximize variants, LR changes between steps, state_dict keys."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kw", [dict(momentum=0.9, weight_decay=1e-4), dict(momentum=0.0),
                                dict(momentum=0.8, dampening=0.1, weight_decay=1e-3),
                                dict(momentum=0.9, nesterov=True), dict(momentum=0.5, maximize=True)])
def test_sgd_matches_torch(gpu, kw):
    from u3d.optim import SGD
    torch.manual_seed(0)
    shapes = [(32, 1, 3, 3, 3), (32,), (7,), (256, 256, 3, 3, 3), (5, 3)] + [(3,)] * 60   # > 48 tensors
    pa = [torch.randn(s, device=gpu) for s in shapes]
    pb = [p.clone() for p in pa]
    pa = [torch.nn.Parameter(p) for p in pa]
    pb = [torch.nn.Parameter(p) for p in pb]
    oa = torch.optim.SGD(pa, lr=0.05, **kw)
    ob = SGD(pb, lr=0.05, **kw)
    for it in range(4):
        for a, b in zip(pa, pb):
            g = torch.randn_like(a)
            a.grad, b.grad = g.clone(), g.clone()
        if it == 2:
            oa.param_groups[0]["lr"] = ob.param_groups[0]["lr"] = 0.01
        oa.step()
        ob.step()
    for a, b in zip(pa, pb):
        torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-6)
    sa, sb = oa.state_dict()["state"], ob.state_dict()["state"]
    assert set(sa) == set(sb) and all(set(sa[k]) == set(sb[k]) for k in sa)
