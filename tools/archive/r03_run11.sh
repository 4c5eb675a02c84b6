#!/bin/bash
# r03: weight-gradient ring staging interleaved with the MFMA chain (in-tree) vs before it (libu3d_ab.so)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03t
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_bf16.py tests/test_gpu_queue.py -k "wgrad or step or queue or 2gib" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/kab.sh r03t/kab 2 wgrad96 wgrad48 wgrad24 fwd96 || exit 1
bash tools/ab.sh r03t/ab "U3D_NONE=0" "U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_ab.so" 4 || exit 1
