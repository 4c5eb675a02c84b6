#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r02ai; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv1x1.py tests/test_gpu_parity.py -k "gn or g3 or block" > $O/pytest1.log 2>&1 || { tail -40 $O/pytest1.log; exit 1; }
tail -2 $O/pytest1.log
bash tools/ab.sh r02ai "U3D_LIB=$R/tools/ab_lib/libu3d_a.so" "U3D_LIB=" 3
bash tools/ab.sh r02ai_dgn "U3D_DGRAD_GN=0" "U3D_DGRAD_GN=1" 3
