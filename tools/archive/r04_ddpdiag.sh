#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_ddpdiag
mkdir -p $O
cd $R
for v in "U3D_X=0" "U3D_WR_DMA=0" "U3D_GN_BWD_FUSED_BRICK=0" "U3D_GN_BWD_FUSED=0"; do
  echo "== $v" | tee -a $O/log
  env $v timeout -k 10 200 python -u -m pytest tests/test_gpu_ddp.py -k rccl -q -s --timeout 150 --timeout-method thread 2>&1 | grep -E "worst|passed|failed" | tee -a $O/log
done
