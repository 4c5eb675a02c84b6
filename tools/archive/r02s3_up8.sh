#!/bin/bash
# Upsample forward with 2x2x2 outputs per thread: tests, micro-benchmark and step A/B via U3D_UP8.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02s3_up8
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bf16.py tests/test_gpu_parity.py -k "upsample or up_ or g3 or g4 or g5" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/ab.sh r02s3_up8/ab "U3D_UP8=1" "U3D_UP8=0" 3 || exit 1
