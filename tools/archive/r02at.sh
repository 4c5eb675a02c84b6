#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r02at; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_bf16.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_conv1x1.py tests/test_gpu_ddp.py > $O/pytest1.log 2>&1 || { tail -40 $O/pytest1.log; exit 1; }
tail -2 $O/pytest1.log
bash tools/ab.sh r02at "U3D_GN_SPLIT=0" "U3D_GN_SPLIT=1" 3
