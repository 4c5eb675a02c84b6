#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r02ag; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv1x1.py > $O/pytest1.log 2>&1 || { tail -40 $O/pytest1.log; exit 1; }
tail -2 $O/pytest1.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_ddp.py tests/test_gpu_graph.py > $O/pytest2.log 2>&1 || { tail -40 $O/pytest2.log; exit 1; }
tail -2 $O/pytest2.log
bash tools/ab.sh r02ag "U3D_S2_COMPACT=0" "U3D_S2_COMPACT=1" 3
