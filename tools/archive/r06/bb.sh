#!/bin/bash
# round 6: conv1 (stem) forward with its 27 window loads issued up front: tests, kernel A/B vs libu3d_ab.so
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06bb; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bf16.py -k "stem" tests/test_gpu_epi_stats.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/kab.sh r06bb 3 stem96st stem96 stemw96
