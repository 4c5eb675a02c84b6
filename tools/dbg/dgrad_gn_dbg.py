"""Debug: the fused ring dgrad + GN-backward partials vs the separate passes, intermediate by intermediate."""
import os, sys
REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path[:0] = [os.path.join(REPO, "multimodal-pl_amd"), REPO]
import torch
from u3d import ops
from u3d._lib import call, query
dev = torch.device("cuda:0")
torch.manual_seed(11)
n, dims = 2, (12, 10, 32)
x = (torch.randn((n,) + dims + (32,), device=dev) * 1.5 + 0.3).to(torch.bfloat16)
w = torch.randn(32, 32, 3, 3, 3, device=dev)
st = ops.gn_stats(x, 16)
ga = 1 + 0.1 * torch.randn(32, device=dev)
be = 0.1 * torch.randn(32, device=dev)
_, pd, _ = ops.wstd_fwd(w, torch.bfloat16, True)
dy = torch.randn((n,) + dims + (32,), device=dev).to(torch.bfloat16)
d, h, w_ = dims
dA = torch.empty_like(x)
ws = torch.zeros(64 * 256 + 64 * 16, device=dev)
call("u3d_conv32_ring_dgrad_gn", dy.data_ptr(), n, d, h, w_, pd.data_ptr(), x.data_ptr(), st.data_ptr(),
     ga.data_ptr(), be.data_ptr(), 16, dA.data_ptr(), ws.data_ptr(), ops._stream())
dA2 = ops.conv_dgrad(dy, pd, 32, x.shape[:4], 3, 1)
torch.cuda.synchronize()
print("dA equal:", torch.equal(dA, dA2), "nan in ws:", torch.isnan(ws).sum().item(), "nan dA:", torch.isnan(dA).sum().item())
coef = torch.empty((n, 5, 32), device=dev)
call("u3d_conv32_ring_gn_bwd_coef", ws.data_ptr(), n, d, h, w_, 16, st.data_ptr(), ga.data_ptr(), be.data_ptr(),
     coef.data_ptr(), None, None, 0, ops._stream())
torch.cuda.synchronize()
print("nan coef:", torch.isnan(coef).sum().item(), coef[0, :, :4])
# reference partial sums
xf, af = x.float(), dA2.float()
g = torch.arange(32, device=dev) // 2
mu, rs = st[:, g, 0], st[:, g, 1]
sc = rs * ga
sh = be - mu * sc
m = (xf * sc.view(n, 1, 1, 1, 32) + sh.view(n, 1, 1, 1, 32)) > 0
gd = torch.where(m, af, torch.zeros_like(af))
xh = (xf - mu.view(n, 1, 1, 1, 32)) * rs.view(n, 1, 1, 1, 32)
s1 = gd.sum((1, 2, 3)); s2 = (gd * xh).sum((1, 2, 3))
import math
pps = math.ceil(h / 8) * math.ceil(w_ / 32) * d
wps0 = max(1, min(pps, 256 // n)); per = -(-pps // wps0); wps = -(-pps // per)
part = ws[: n * wps * 64].view(n, wps, 32, 2).sum(1)
print("wps", wps, "s1 err", (part[..., 0] - s1).abs().max().item(), "s2 err", (part[..., 1] - s2).abs().max().item())
pw = ws[: n * wps * 64].view(n, wps, 32, 2)
bad = torch.isnan(pw)
print("nan (n, wg, ch, k):", bad.nonzero()[:20].tolist())
print("nan channels:", sorted(set(bad.nonzero()[:, 2].tolist())), "wgs:", sorted(set(bad.nonzero()[:, 1].tolist())))
