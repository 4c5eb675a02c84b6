#!/bin/bash
# round 6: stride-2 forward ring with two staged planes in flight (in-tree) vs one (libu3d_ab.so); its parity tests
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06u; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_s2ring.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/kab.sh r06u 3 fwds2ring
