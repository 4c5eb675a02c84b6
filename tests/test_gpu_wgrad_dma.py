"""The 16 x 16-tile weight-gradient ring with LDS-DMA staging (wgrad_ring.hip, wgrad_ring_dma_kernel — since round 5
the only 16 x 16 form) against the halo-brick weight gradient (the other stride-1 kernel, a different tiling and
summation order: fp32 sums of the same bf16 products) and against fp64 on the same bf16 operands; two runs bitwise
equal. Cases: the bench levels (2 x 96^3 x 32, 2 x 48^3 x 64), partial plane tiles (h, w not multiples of 16: rows
past the volume come from out-of-range DMAs), several channel tiles, odd depths and sample counts, GroupNorm prologue
on and off (the off form has no in-place transform; its padding rows are the DMA's zero fill). Reference: autograd of
F.conv3d in Conv3d.forward (unet3D.py:27)."""
import pytest
import torch

from test_gpu_fullsize import _act, _bf, _operands

pytestmark = pytest.mark.gpu

CASES = [(2, 32, 32, (96, 96, 96), True), (2, 64, 64, (48, 48, 48), True), (1, 32, 32, (7, 40, 40), True),
         (3, 32, 64, (5, 20, 36), False), (2, 64, 32, (9, 16, 48), True), (1, 96, 64, (6, 33, 17), True),
         (2, 32, 32, (11, 16, 16), False), (1, 48, 24, (4, 18, 30), True)]


@pytest.mark.parametrize("n,cin,cout,dims,use_gn", CASES, ids=lambda v: str(v))
def test_wgrad_dma_ring_vs_brick_and_fp64(gpu, n, cin, cout, dims, use_gn):
    from u3d import ops
    x, _, gn = _operands(gpu, n, cin, cout, dims, 41)
    gn = gn if use_gn else None
    dy = (torch.randn((n,) + dims + (cout,), device=gpu) * 0.7).to(torch.bfloat16)
    with ops.option("WR_TILE16", 1):
        p_dma, _ = ops.conv_wgrad(dy, x, 3, 1, gn, brick="ring")
        p_dma2, _ = ops.conv_wgrad(dy, x, 3, 1, gn, brick="ring")
    p_brk, _ = ops.conv_wgrad(dy, x, 3, 1, gn, brick=True)
    torch.cuda.synchronize()
    assert torch.equal(p_dma, p_dma2), "DMA ring not deterministic"
    dw = p_dma.sum(0).double()[:, :cout, :cin]
    db = p_brk.sum(0).double()[:, :cout, :cin]
    err = ((dw - db).norm() / db.norm()).item()
    assert err <= 5e-4, err  # fp32 reassociation (and the GN prologue's bf16 roundings, computed in another order)
    if max(dims) <= 48:
        a = _act(x, gn, torch.float64) if gn is not None else _bf(x.cpu()).permute(0, 4, 1, 2, 3)
        ref = torch.nn.grad.conv3d_weight(a, (cout, cin, 3, 3, 3), _bf(dy.cpu()).permute(0, 4, 1, 2, 3), padding=1)
        ref = ref.reshape(cout, cin, 27).permute(2, 0, 1)
        assert ((dw.cpu() - ref).norm() / ref.norm()).item() <= 1e-3
