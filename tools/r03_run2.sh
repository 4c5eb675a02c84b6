#!/bin/bash
# r03: split-K width of the weight-gradient kernels (fp32 slab bytes vs occupancy)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/env_ab.sh r03j/wr "wgrad|sum_slabs|wstd" "U3D_WR_WGS=256" "U3D_WR_WGS=128" || exit 1
bash tools/env_ab.sh r03j/wb "wgrad|sum_slabs|wstd" "U3D_WB_WGS=256" "U3D_WB_WGS=128" || exit 1
