#!/bin/bash
# round 6: GroupNorm reduction blocks (U3D_GN_MAXBLK, default 256): step A/B against 512 and 1024
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
bash tools/ab.sh r06v "U3D_GN_MAXBLK=256" "U3D_GN_MAXBLK=512" 3 && bash tools/ab.sh r06v2 "U3D_GN_MAXBLK=256" "U3D_GN_MAXBLK=1024" 3
