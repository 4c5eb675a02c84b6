#!/bin/bash
# r03: ring conv staging loads two planes ahead (PF=2, in-tree) vs one (libu3d_ab.so, -DU3D_RING_PF=1)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03n
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_bf16.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/kab.sh r03n/kab 2 fwd96 fwd96_nores dgrad96 wgrad96 wgrad48 wgrad24 || exit 1
bash tools/ab.sh r03n/ab "U3D_NONE=0" "U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_ab.so" 3 || exit 1
