#!/bin/bash
# r03: stem conv1 with a scalar-loaded weight table (tests, kernel A/B vs libu3d_ab.so = the pre-stem tree, step A/B)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03l
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bf16.py -k 'stem or wgrad' > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/kab.sh r03l/kab 2 stem96 || exit 1
bash tools/ab.sh r03l/ab "U3D_NONE=0" "U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_ab.so" 3 || exit 1
