#!/bin/bash
# r03: conv1 stem stores through a per-wave LDS transpose + stride-2 data gradient on branch-free buffer loads
# + conv_small on buffer loads (in-tree) vs direct 16-B stores + branched loads (libu3d_ab.so)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03w
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bf16.py tests/test_gpu_fullsize.py -k "stem or s2 or dgrad or small or fwd" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/kab.sh r03w/kab 2 stem96 dgrad_s2_96 dgrad_s2_48 dgrad_s2_24 dgrad_s2_12 fwd12 dgrad12 fwd6 dgrad6 || exit 1
bash tools/ab.sh r03w/ab "U3D_NONE=0" "U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_ab.so" 3 || exit 1
