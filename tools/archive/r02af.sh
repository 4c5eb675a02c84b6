#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r02af; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv1x1.py > $O/pytest1.log 2>&1 || { tail -40 $O/pytest1.log; exit 1; }
tail -2 $O/pytest1.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bf16.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py > $O/pytest2.log 2>&1 || { tail -40 $O/pytest2.log; exit 1; }
tail -2 $O/pytest2.log
C="c1_s2_96 c1_s2_48 c1_s2_24 c1_s2_12 c1_48 c1_24 c1_12 c1_6 dc1_48 dc1_24 dc1_12 dc1_6"
for cfg in "U3D_CONV1X1=1"; do
  echo "== $cfg" | tee -a $O/k.txt
  env $cfg timeout -k 10 100 python tools/kbench.py $C 2>&1 | grep -v amdgpu.ids | tee -a $O/k.txt || exit 1
done
bash tools/ab.sh r02af "U3D_CONV1X1=0" "U3D_CONV1X1=1" 3
