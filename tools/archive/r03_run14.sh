#!/bin/bash
# r03: brick weight gradients on branch-free buffer loads (in-tree) vs branched 64-bit loads (libu3d_ab.so)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03x
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bf16.py tests/test_gpu_fullsize.py -k "wgrad or 2gib or 1x1 or head" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/kab.sh r03x/kab 2 wgrad_s2_96 wgrad_s2_48 wgrad_s2_24 wgrad6 wgrad1_96 wgrad1_s2_96 || exit 1
bash tools/ab.sh r03x/ab "U3D_NONE=0" "U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_ab.so" 3 || exit 1
