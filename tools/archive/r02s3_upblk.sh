#!/bin/bash
# Blocked trilinear backward: bitwise tests, micro-benchmarks (U3D_UP_BWD_BLK 1 / 0), step A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02s3_upblk
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_upsample_blk.py tests/test_gpu_parity.py -k "upsample or up" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for b in 1 0; do U3D_UP_BWD_BLK=$b timeout -k 10 120 python tools/kbench.py upb96 upb48 2>>$O/kb.err | sed "s/^/blk=$b /" | tee -a $O/kbench.log || exit 1; done
bash tools/ab.sh r02s3_upblk/ab "U3D_UP_BWD_BLK=1" "U3D_UP_BWD_BLK=0" 3
