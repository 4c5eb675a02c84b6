#!/bin/bash
# Grid-target sweeps (step A/B, 2 rounds each): implicit-GEMM split-K target, wgrad ring / brick workgroup targets.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/ab.sh r02s3_grid/ig256 "U3D_IGEMM_TARGET=512" "U3D_IGEMM_TARGET=256" 2 || exit 1
bash tools/ab.sh r02s3_grid/ig1024 "U3D_IGEMM_TARGET=512" "U3D_IGEMM_TARGET=1024" 2 || exit 1
bash tools/ab.sh r02s3_grid/wr512 "U3D_WR_WGS=256" "U3D_WR_WGS=512" 2 || exit 1
bash tools/ab.sh r02s3_grid/wr128 "U3D_WR_WGS=256" "U3D_WR_WGS=128" 2 || exit 1
bash tools/ab.sh r02s3_grid/wb512 "U3D_WB_WGS=256" "U3D_WB_WGS=512" 2 || exit 1
bash tools/ab.sh r02s3_grid/wb128 "U3D_WB_WGS=256" "U3D_WB_WGS=128" 2 || exit 1
