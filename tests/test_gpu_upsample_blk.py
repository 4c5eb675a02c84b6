"""Trilinear x2 backward with 2 x 2 input rows per thread (up_bwd_blk_kernel, u3d_upsample2x_bwd's choice for grids of >= 1024 workgroups)
against the one-row gather (option UP_BWD_BLK=0, itself checked against torch autograd in test_gpu_parity.py). Same taps,
weights and add order per output: bitwise equal. Odd d / h (a half-empty row pair), size-1 dims, accumulate, fp32 and
bf16. Reference: nn.Upsample(scale_factor=2, mode='trilinear') (unet3D.py:1646)."""

import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [(2, 48, 48, 48, 32), (2, 24, 24, 24, 64), (1, 5, 7, 9, 16), (2, 3, 4, 6, 8), (1, 1, 1, 1, 8),
          (1, 1, 3, 2, 16), (3, 6, 5, 12, 64), (1, 7, 1, 4, 32)]


def _bwd(dy, shape, prev, blk):
    from u3d import ops
    with ops.option("UP_BWD_BLK", 1 if blk else 0):
        dx = ops.upsample2x_bwd(dy, shape, dx=None if prev is None else prev.clone(), accumulate=prev is not None)
        torch.cuda.synchronize()
    return dx


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("acc", [False, True], ids=["set", "acc"])
def test_upsample_bwd_blocked_bitwise(gpu, shape, dtype, acc):
    n, d, h, w, c = shape
    torch.manual_seed(11)
    dy = torch.randn((n, 2 * d, 2 * h, 2 * w, c), device=gpu).to(dtype)
    prev = torch.randn(shape, device=gpu).to(dtype) if acc else None
    a = _bwd(dy, shape, prev, True)
    b = _bwd(dy, shape, prev, False)
    assert torch.isfinite(a.float()).all()
    iv = torch.int32 if dtype == torch.float32 else torch.int16
    assert torch.equal(a.view(iv), b.view(iv)), f"max diff {(a.float() - b.float()).abs().max().item()}"
