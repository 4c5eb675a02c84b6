#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r02as; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_epistats.py tests/test_gpu_bf16.py tests/test_gpu_parity.py -k "upsample or up_ or g3 or g1" > $O/pytest1.log 2>&1 || { tail -40 $O/pytest1.log; exit 1; }
tail -2 $O/pytest1.log
for cfg in "U3D_UP_BLK=0" "U3D_UP_BLK=1"; do
  echo "== $cfg" | tee -a $O/k.txt
  env $cfg timeout -k 10 100 python tools/kbench.py upf96 upf48 upb96 upb48 2>&1 | grep -v amdgpu.ids | tee -a $O/k.txt || exit 1
done
bash tools/ab.sh r02as "U3D_UP_BLK=0" "U3D_UP_BLK=1" 3
