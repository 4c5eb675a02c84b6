#!/bin/bash
# r04: 2x2-output upsample (UP_QUAD=1 vs 0): bitwise test, kernel A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_m
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -k "upsample or wstd" tests/test_gpu_upsample_blk.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  for v in 1 0; do
    echo "== UP_QUAD=$v" >> $O/kab.log
    U3D_UP_QUAD=$v timeout -k 10 120 python tools/kbench.py up96 up48 upb96 upb48 >> $O/kab.log 2>&1 || { tail $O/kab.log; exit 1; }
  done
done
grep -v amdgpu.ids $O/kab.log
