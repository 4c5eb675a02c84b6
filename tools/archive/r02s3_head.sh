#!/bin/bash
# Transposed-MFMA head (vector stores, LDS GN table): bitwise + parity tests, kernel times and step A/B via U3D_HEAD_TR.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02s3_head
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bf16.py -k "head" tests/test_gpu_parity.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for t in 1 0; do U3D_HEAD_TR=$t timeout -k 10 120 python tools/kbench.py head96 2>/dev/null | sed "s/^/tr=$t /"; done | tee $O/kbench.log
bash tools/ab.sh r02s3_head/ab "U3D_HEAD_TR=1" "U3D_HEAD_TR=0" 3 || exit 1
