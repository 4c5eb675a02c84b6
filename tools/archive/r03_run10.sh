#!/bin/bash
# r03: persistent brick weight staging with 4 lanes per 64-B row segment (in-tree) vs chunk-major (libu3d_ab.so)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03s
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pbrick.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/kab.sh r03s/kab 2 fwd48 dgrad48 fwd24 dgrad24 || exit 1
bash tools/ab.sh r03s/ab "U3D_NONE=0" "U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_ab.so" 3 || exit 1
