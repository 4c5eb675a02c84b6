#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r02an; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bf16.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py > $O/pytest1.log 2>&1 || { tail -40 $O/pytest1.log; exit 1; }
tail -2 $O/pytest1.log
timeout -k 10 100 python tools/kbench.py dec24_c1 dec24_c2 ddec24_c1 ddec24_c2 fwd24 dgrad24 2>&1 | grep -v amdgpu.ids | tee -a $O/k.txt || exit 1
bash tools/ab.sh r02an "U3D_CONVG_CO32=0" "U3D_CONVG_CO32=-1" 3
