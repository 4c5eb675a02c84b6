#!/bin/bash
# round 6: upsample + skip (+ statistics): skip loads issued with the input loads, 192-thread blocks — tests, kernel A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06x; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bf16.py -k "upsample" tests/test_gpu_epi_stats.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/kab.sh r06x 3 up96st up48st up96
