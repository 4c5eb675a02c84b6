#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r02ap; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bf16.py tests/test_gpu_parity.py tests/test_gpu_ddp.py tests/test_gpu_optim.py -k "wstd or g3 or g1 or g2 or ddp or sgd or optim" > $O/pytest1.log 2>&1 || { tail -40 $O/pytest1.log; exit 1; }
tail -2 $O/pytest1.log
bash tools/ab.sh r02ap "U3D_WSTD_ROW=0" "U3D_WSTD_ROW=1" 3
