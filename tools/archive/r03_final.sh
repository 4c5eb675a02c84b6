#!/bin/bash
# r03 closing call: GroupNorm-backward partial / paired partial / paired apply with deeper load rounds (in-tree) vs
# the previous rounds (libu3d_ab.so), then the
# round-end measurements of the in-tree library (tools/round_end_r03.sh)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/lib_ab.sh r03z "gn_" tests/test_gpu_parity.py tests/test_gpu_bf16.py -k "gn or g3 or g4" || exit 1
bash tools/round_end_r03.sh
