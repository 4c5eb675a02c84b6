#!/bin/bash
# GN-backward partials in the persistent brick's data-gradient epilogue: tests (vs separate passes, bench-size step,
# DDP), step A/B via U3D_BRICK_DGRAD_GN.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02s3_bg
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pbrick.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
U3D_BRICK_DGRAD_GN=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fullsize.py -k "step or yardstick" tests/test_gpu_ddp.py tests/test_gpu_parity.py > $O/pytest2.log 2>&1 || { tail -30 $O/pytest2.log; exit 1; }
tail -1 $O/pytest2.log
bash tools/ab.sh r02s3_bg/ab "U3D_BRICK_DGRAD_GN=1" "U3D_BRICK_DGRAD_GN=0" 3 || exit 1
