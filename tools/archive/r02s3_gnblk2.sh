#!/bin/bash
# GroupNorm reduction blocks below the default: U3D_GN_MAXBLK 256 / 128 / 64 on the 48^3..6^3 levels.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02s3_gnblk2
mkdir -p $O
cd $R
for m in 256 128 64; do
  U3D_GN_MAXBLK=$m timeout -k 10 120 python tools/kbench.py gnstats96 gnbwd96 gnstats48 gnbwd48 gnbwd248 gnstats24 gnbwd24 gnbwd224 gnstats12 gnbwd12 gnstats6 gnbwd6 2>>$O/kb.err | sed "s/^/blk=$m /" | tee -a $O/kbench.log || exit 1
done
