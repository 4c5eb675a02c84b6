#!/bin/bash
# r03: spill-free kernels check + two step A/Bs (per-conv slab flush; this tree vs the round-2 library)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03i
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pbrick.py tests/test_gpu_bf16.py > $O/pytest1.log 2>&1 || { tail -30 $O/pytest1.log; exit 1; }
tail -1 $O/pytest1.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/ab.sh r03i/flush "U3D_FLUSH_EACH=0" "U3D_FLUSH_EACH=1" 3 || exit 1
bash tools/ab.sh r03i/lib "U3D_NONE=0" "U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_ab.so" 3 || exit 1
