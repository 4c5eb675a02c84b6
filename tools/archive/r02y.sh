#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r02y; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fullsize.py -k "trunk and s2" tests/test_gpu_bf16.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 150 python tools/kbench.py fwd_s2_96 fwd_s2_48 fwd_s2_24 fwd_s2_12 2>&1 | grep -v amdgpu.ids | tee $O/s2.txt || exit 1
bash tools/gn_prof.sh r02y || exit 1
bash tools/prof_bench.sh r02y
