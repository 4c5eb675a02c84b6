#!/bin/bash
# GroupNorm reduction grid (U3D_GN_MAXBLK: blocks over all samples for the big tensors): step A/B 256 / 512 / 1024.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/ab.sh r02s3_gnblk/a "U3D_GN_MAXBLK=256" "U3D_GN_MAXBLK=512" 3 || exit 1
bash tools/ab.sh r02s3_gnblk/b "U3D_GN_MAXBLK=256" "U3D_GN_MAXBLK=1024" 3 || exit 1
