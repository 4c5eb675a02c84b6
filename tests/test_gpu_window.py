"""Sliding-window inference: evaluate_amos.predict_sliding (device accumulation through
u3d_window_accumulate / u3d_window_normalize) against the float64 restatement oracle.ref_cpu.predict_sliding of
reference evaluate_amos.py:198-279, on the same per-tile network outputs."""
import numpy as np
import pytest
import torch

from oracle import ref_cpu as O

pytestmark = pytest.mark.gpu

WIN_TOL = 2e-5   # fp32 device accumulation vs the reference's float64 host accumulation (relative to max |logit|)


class _RampNet(torch.nn.Module):
    """Position-dependent (so flip bugs show) deterministic stand-in: out[:, c] = x * ramp_c + 0.1 c."""

    def __init__(self, classes, k=1.0):
        super().__init__()
        self.k = torch.nn.Parameter(torch.tensor(float(k)))
        self.classes = classes

    def forward(self, x, task_id=None):
        d, h, w = x.shape[2:]
        r = (torch.arange(d, device=x.device).view(d, 1, 1) * 0.37 + torch.arange(h, device=x.device).view(1, h, 1)
             * 0.11 - torch.arange(w, device=x.device).view(1, 1, w) * 0.05)
        outs = [x[:, 0] * torch.sin(r * (c + 1) * 0.1) * self.k + 0.1 * c for c in range(self.classes)]
        return torch.stack(outs, 1)


def _ref(nets, image, tile, classes, tta):
    def pred_fn(t):
        with torch.no_grad():
            xs = torch.from_numpy(np.ascontiguousarray(t)).float().cuda()
            outs = [n(xs, None) for n in nets]
            outs = [o[0] if isinstance(o, (tuple, list)) else o for o in outs]
            return (sum(outs) / len(outs)).double().cpu().numpy()
    return O.predict_sliding(pred_fn, image, tile, classes, tta=tta)


@pytest.mark.parametrize("shape,tile,tta,nnets", [
    ((2, 1, 20, 40, 36), (16, 24, 24), False, 1),
    ((1, 1, 23, 37, 50), (16, 24, 24), True, 2),
    ((1, 1, 16, 24, 24), (16, 24, 24), True, 1),      # one tile covering the volume
    ((1, 1, 64, 40, 40), (16, 24, 32), False, 1),     # anisotropic tile, many depth steps
])
def test_predict_sliding_ramp(gpu, shape, tile, tta, nnets):
    import evaluate_amos as E
    rng = np.random.default_rng(0)
    image = rng.standard_normal(shape).astype(np.float32)
    nets = [_RampNet(3, k=1.0 + 0.5 * i).cuda() for i in range(nnets)]
    with torch.no_grad():
        out = E.predict_sliding(None, nets, image, list(tile), 3, None, tta=tta)
    torch.cuda.synchronize()
    ref = _ref(nets, image, tile, 3, tta)
    got = out.double().cpu().numpy()
    assert got.shape == ref.shape
    assert np.isfinite(got).all()
    np.testing.assert_allclose(got, ref, atol=WIN_TOL * np.abs(ref).max(), rtol=0)


def test_predict_sliding_baseline_model(gpu):
    """The native UNet3D baseline as the per-tile network, two nets averaged, flip TTA."""
    import unet3D
    import evaluate_amos as E
    from oracle.weights_recipe import apply_recipe
    nets = []
    for seed in (0, 1):
        m = unet3D.unet3D_baseline([1, 2, 2, 2, 2], num_classes=4, weight_std=True)
        apply_recipe(m, seed=seed)
        nets.append(m.cuda().eval())
    rng = np.random.default_rng(3)
    image = rng.standard_normal((1, 1, 24, 48, 40)).astype(np.float32)
    tile = (16, 32, 32)
    with torch.no_grad():
        out = E.predict_sliding(None, nets, image, list(tile), 4, None, tta=True)
        ref = _ref(nets, image, tile, 4, True)
    got = out.double().cpu().numpy()
    np.testing.assert_allclose(got, ref, atol=WIN_TOL * np.abs(ref).max(), rtol=0)



class _StandIn(torch.nn.Module):
    """The deterministic network of fixture G13 (tests/golden/gen_golden.py g13): tanh(conv3d 3^3 + bias)."""

    def __init__(self, w, b):
        super().__init__()
        self.w = torch.nn.Parameter(torch.from_numpy(w))
        self.b = torch.nn.Parameter(torch.from_numpy(b))

    def forward(self, x, task_id=None):
        return torch.tanh(torch.nn.functional.conv3d(x, self.w, padding=1) + self.b.view(1, -1, 1, 1, 1))


@pytest.mark.parametrize("tag", ["a", "b", "c"])
def test_predict_sliding_vs_reference_fixture(gpu, tag):
    """evaluate_amos.predict_sliding on the device against the REFERENCE's own predict_sliding output (G13: ragged
    volume without TTA; two nets with the 8-flip TTA; a one-tile volume), same stand-in networks: <= WIN_TOL of the
    volume's max |probability| (fp32 device accumulation vs the reference's float64 host arrays)."""
    from conftest import golden
    from evaluate_amos import predict_sliding
    g = golden("g13_predict_sliding.npz")
    nets = [_StandIn(w, b).to(gpu).eval() for w, b in zip(g[f"{tag}_w"], g[f"{tag}_b"])]
    tile = tuple(int(v) for v in g[f"{tag}_tile"])
    ref = g[f"{tag}_full"]
    with torch.no_grad():
        out = predict_sliding(None, nets, g[f"{tag}_img"], tile, ref.shape[1], 0, tta=bool(g[f"{tag}_tta"]))
    err = np.abs(out.double().cpu().numpy() - ref).max()
    assert err <= WIN_TOL * np.abs(ref).max(), err


def test_predict_sliding_full_tiles_bf16_vs_fp32(gpu):
    """BASELINE configs[4] at its real tile size: two overlapping 64 x 192 x 192 tiles (1 x 1 x 64 x 192 x 240
    volume, stride 144 along W) of unet3D_baseline(16) through predict_sliding, the bf16 native path (autocast, as
    the bench's inference mode) against the fp32 native path (pinned to the reference forward by G5).

    The reference's "fp16" for this config computes fp32: evaluate_amos.py:594-601 (--FP16 selects a checkpoint
    branch identical to the other) and the forward is never autocast. Tolerance as for the bf16 training forward
    (test_gpu_fullsize.py: ~40 rounded stages, sqrt(40) x 2^-8 = 2.5e-2): relative L2 of the accumulated
    probabilities <= 5e-2, and the arg-max label agrees on >= 97% of the voxels where the fp32 top-2 margin
    exceeds 5% of the logit scale."""
    import time
    import unet3D
    import evaluate_amos as E
    from oracle.weights_recipe import apply_recipe, input_volume
    m = unet3D.unet3D_baseline([1, 2, 2, 2, 2], num_classes=16, weight_std=True)
    apply_recipe(m, seed=0)
    m = m.to(gpu).eval()
    image = input_volume((1, 1, 64, 192, 240), seed=71, kind="ct")
    tile = [64, 192, 192]
    assert len(E.tile_plan(image.shape, tile)) == 2
    outs, ms = {}, {}
    for mode in ("fp32", "bf16"):
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16, enabled=mode == "bf16"):
            E.predict_sliding(None, [m], image, tile, 16, None)  # warm-up (weight packs, workspaces)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            outs[mode] = E.predict_sliding(None, [m], image, tile, 16, None)
            torch.cuda.synchronize()
            ms[mode] = (time.perf_counter() - t0) * 1e3
    a, b = outs["fp32"].double(), outs["bf16"].double()
    assert torch.isfinite(b).all()
    rel = ((b - a).norm() / a.norm()).item()
    top2 = a.topk(2, dim=1).values
    sure = (top2[:, 0] - top2[:, 1]) > 0.05 * a.abs().max()
    agree = (a.argmax(1) == b.argmax(1))[sure].double().mean().item()
    print(f"2 x 64x192x192 tiles: fp32 {ms['fp32']:.1f} ms, bf16 {ms['bf16']:.1f} ms; rel L2 {rel:.3e}, "
          f"arg-max agreement {agree:.4f} on {sure.double().mean().item():.3f} of the voxels")
    assert rel <= 5e-2, rel
    assert agree >= 0.97, agree
