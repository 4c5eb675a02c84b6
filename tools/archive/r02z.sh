#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r02z; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_bf16.py tests/test_gpu_epistats.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/gn_prof.sh r02z || exit 1
bash tools/ab.sh r02z "U3D_IGEMM_AUTO=0" "U3D_IGEMM_AUTO=1" 3
