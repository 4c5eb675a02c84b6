#!/bin/bash
# GN statistics from the persistent brick's epilogue: tests (stats vs the pass, bitwise outputs, bench-size step),
# step A/B via U3D_BRICK_STATS, kernel split.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02s3_bst
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pbrick.py tests/test_gpu_fullsize.py tests/test_gpu_ddp.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/ab.sh r02s3_bst/ab "U3D_BRICK_STATS=1" "U3D_BRICK_STATS=0" 3 || exit 1
