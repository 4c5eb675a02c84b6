#!/bin/bash
# Default choice of the trilinear backward (blocked at >= 1024 workgroups): bitwise tests, upsample parity, kernels.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02s3_upblk2
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_upsample_blk.py tests/test_gpu_parity.py tests/test_gpu_bf16.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python tools/kbench.py upb96 upb48 2>>$O/kb.err | tee -a $O/kbench.log
