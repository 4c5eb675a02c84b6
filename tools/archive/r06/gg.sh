#!/bin/bash
# round 6: stride-2 GroupNorm-backward pair with incremental coordinates: bitwise vs libu3d_ab.so, tests, kernel A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06gg; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_conv1x1.py tests/test_gpu_fullsize.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for L in "" "$R/multimodal-pl_amd/u3d/libu3d_ab.so"; do
U3D_LIB=$L timeout -k 10 100 python - <<'PY' >> $O/bits.log 2>&1 || exit 1
import sys, torch, hashlib
sys.path.insert(0, "multimodal-pl_amd")
from u3d import ops
g = torch.Generator().manual_seed(5)
for (n, c, dims) in [(2, 32, (96, 96, 96)), (2, 64, (48, 48, 48)), (1, 128, (7, 9, 11)), (3, 256, (5, 6, 4)), (2, 64, (10, 12, 13))]:
    x = torch.randn((n,) + dims + (c,), generator=g).to(torch.bfloat16).cuda()
    da = torch.randn((n,) + dims + (c,), generator=g).to(torch.bfloat16).cuda()
    cd = tuple((s - 1) // 2 + 1 for s in dims)
    da2c = torch.randn((n,) + cd + (c,), generator=g).to(torch.bfloat16).cuda()
    st = ops.gn_stats(x, 16)
    ga, be = (torch.rand(c, generator=g) + 0.5).cuda(), (torch.randn(c, generator=g) * 0.1).cuda()
    dx = torch.randn((n,) + dims + (c,), generator=g).to(torch.bfloat16).cuda()
    dps = [(torch.zeros(c, device="cuda"), torch.zeros(c, device="cuda")) for _ in range(2)]
    out = ops.gn_bwd2(da, da2c, x, st, (ga, be), (ga * 0.7, be + 0.05), 16, dx=dx, accumulate=True, dparams1=dps[0], dparams2=dps[1], da2_s2=True)
    h = hashlib.sha1(out.view(torch.int16).cpu().numpy().tobytes() + torch.cat([t for p in dps for t in p]).cpu().numpy().tobytes()).hexdigest()
    print(dims, c, h)
PY
done
cat $O/bits.log | grep -v amdgpu
bash tools/kab.sh r06gg 2 gnbwd2s96 gnbwd2s48 gnbwd2s24
