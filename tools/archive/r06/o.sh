#!/bin/bash
# round 6: head GN-partials fusion — head/loss tests + full-size parity, then step A/B (fused vs separate partial pass)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out/r06o
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_head_loss.py tests/test_gpu_fullsize.py > gpurun_out/r06o/tests.log 2>&1 || { tail -30 gpurun_out/r06o/tests.log; exit 1; }
tail -3 gpurun_out/r06o/tests.log
bash tools/ab.sh r06o "U3D_HEAD_GN_PARTS=1" "U3D_HEAD_GN_PARTS=0" 3
