#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r02ak; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_s2.py > $O/pytest1.log 2>&1 || { tail -40 $O/pytest1.log; exit 1; }
tail -2 $O/pytest1.log
for cfg in "U3D_S2_FWD=0" "U3D_S2_FWD=1 U3D_S2_FWD_MIN_W=1"; do
  echo "== $cfg" | tee -a $O/k.txt
  env $cfg timeout -k 10 100 python tools/kbench.py fwd_s2_96 fwd_s2_48 fwd_s2_24 fwd_s2_12 2>&1 | grep -v amdgpu.ids | tee -a $O/k.txt || exit 1
done
