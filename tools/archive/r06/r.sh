#!/bin/bash
# round 6: step A/B of the head's fused GN partials (U3D_HEAD_GN_PARTS)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
bash tools/ab.sh r06r "U3D_HEAD_GN_PARTS=1" "U3D_HEAD_GN_PARTS=0" 4
