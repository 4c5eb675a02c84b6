#!/bin/bash
# round 6: loss forward with three tiles in flight (static rotation) vs one: tests, bitwise vs the old build, kernel A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06z; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_head_loss.py tests/test_gpu_parity.py tests/test_gpu_head_oracle.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for L in "" "$R/multimodal-pl_amd/u3d/libu3d_ab.so"; do
U3D_LIB=$L timeout -k 10 100 python - <<'PY' >> $O/bits.log 2>&1 || exit 1
import sys, torch
sys.path.insert(0, "multimodal-pl_amd")
from u3d import ops
g = torch.Generator().manual_seed(3)
for dims in [(2, 96, 96, 96), (2, 7, 9, 11), (1, 33, 5, 3)]:
    lg = (torch.randn(dims + (16,), generator=g) * 3).cuda()
    lab = torch.randint(0, 16, dims, generator=g).float().cuda()
    wt = (torch.rand(16, generator=g) < 0.7).float().cuda()
    l, s = ops.partial_loss_fwd(lg, lab, wt, True, True)
    print(dims, l.item().hex(), s.double().sum().item().hex())
PY
done
cat $O/bits.log
bash tools/kab.sh r06z 3 loss96
