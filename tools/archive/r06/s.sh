#!/bin/bash
# round 6: slab sum with wave-contiguous columns (in-tree) vs the 16-lane-slice mapping (libu3d_ab.so)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
bash tools/kab.sh r06s 2 slabsum96 slabsum48 slabsum24 slabsum12
