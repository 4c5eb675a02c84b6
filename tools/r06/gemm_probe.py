"""round 6 probe: the small-level weight gradient as a library GEMM (27 batched dy^T @ im2col(x)) vs the in-tree
weight-gradient kernels + their slab sum (timing only)."""
import os
import sys
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "multimodal-pl_amd"),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")]
import torch  # noqa: E402
from kbench import t_  # noqa: E402
from u3d import ops  # noqa: E402

dev = torch.device("cuda:0")
for s in (12, 6):
    n, c = 2, 256
    V = n * s ** 3
    dy = torch.randn(V, c, device=dev).to(torch.bfloat16)
    xcol = torch.randn(V, 27 * c, device=dev).to(torch.bfloat16)
    A = dy.t().unsqueeze(0).expand(27, c, V)
    B = xcol.view(V, 27, c).permute(1, 0, 2)
    out = torch.empty(27, c, c, device=dev)
    for dt in ("bf16out", "f32out"):
        if dt == "f32out":
            try:
                f = lambda: torch.bmm(A, B, out_dtype=torch.float32)
                f()
            except Exception as e:
                print("bmm out_dtype fails:", str(e)[:200]); continue
        else:
            f = lambda: torch.bmm(A, B)
        us = t_(f)
        print(f"{s}^3 bmm {dt}: {us:.1f} us  {2.0 * V * 27 * c * c / us / 1e6:.1f} TFLOP/s")
    # one flat GEMM [c x V] @ [V x 27c] then a permute copy
    f = lambda: torch.mm(dy.t(), xcol, out_dtype=torch.float32)
    try:
        us = t_(f)
        print(f"{s}^3 mm f32out flat: {us:.1f} us")
    except Exception as e:
        print("mm out_dtype fails:", str(e)[:200])
    # in-tree weight gradient + slab sum
    x = torch.randn(n, s, s, s, c, device=dev).to(torch.bfloat16)
    dyv = dy.view(n, s, s, s, c)
    g = (ops.gn_stats(x, 16), torch.ones(c, device=dev), torch.zeros(c, device=dev), 16)

    def cur():
        p, ns = ops.conv_wgrad(dyv, x, 3, 1, g)
        ops.sum_slabs(p, ns, c, c)
    print(f"{s}^3 in-tree wgrad + slab sum: {t_(cur):.1f} us; splits {ops.conv_wgrad(dyv, x, 3, 1, g)[1]}")
    def cur0():
        ops.conv_wgrad(dyv, x, 3, 1, g)
    print(f"{s}^3 in-tree wgrad alone: {t_(cur0):.1f} us")
