#!/bin/bash
# r06: the ring's normalised side output (xn) — parity, then a step + kernel A/B of U3D_RING_XN
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06_b; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_ring_xn.py tests/test_gpu_fullsize.py > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/env_ab.sh r06_b "wgrad_ring_dma|conv32_ring" "U3D_RING_XN=1" "U3D_RING_XN=0"
