#!/bin/bash
# GroupNorm reduction block count: U3D_GN_MAXBLK 256 (default) / 512 / 1024, micro-benchmarks then step A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02s3_gnblk
mkdir -p $O
cd $R
for m in 256 512 1024; do
  U3D_GN_MAXBLK=$m timeout -k 10 120 python tools/kbench.py gnstats96 gnbwd96 gnbwd296 gnstats48 gnbwd48 gnstats24 gnbwd24 2>>$O/kb.err | sed "s/^/blk=$m /" | tee -a $O/kbench.log || exit 1
done
bash tools/ab.sh r02s3_gnblk "U3D_GN_MAXBLK=256" "U3D_GN_MAXBLK=512" 3
