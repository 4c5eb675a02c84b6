#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r02ar; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_fullsize.py -k "2gib" > $O/pytest1.log 2>&1 || { tail -40 $O/pytest1.log; exit 1; }
tail -2 $O/pytest1.log
