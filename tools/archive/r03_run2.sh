#!/bin/bash
# r03: full-tile sliding-window test; split-K width of the weight-gradient kernels (fp32 slab bytes vs occupancy)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/r03j
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_gpu_window.py -k full_tiles > gpurun_out/r03j/pytest.log 2>&1 || { tail -30 gpurun_out/r03j/pytest.log; exit 1; }
grep -E "tiles:|passed" gpurun_out/r03j/pytest.log
bash tools/env_ab.sh r03j/wr "wgrad|sum_slabs|wstd" "U3D_WR_WGS=256" "U3D_WR_WGS=128" || exit 1
bash tools/env_ab.sh r03j/wb "wgrad|sum_slabs|wstd" "U3D_WB_WGS=256" "U3D_WB_WGS=128" || exit 1
