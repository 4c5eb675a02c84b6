#!/bin/bash
# Ring v2 sweep on the GPU box: parity of the ring tests, then kbench of the 96^3 ring launches for v1 and v2 configs.
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_bf16.py \
  -k "multi_plane or c32to32 or ring or gn_apply or conv_fwd or conv_dgrad" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for cfg in "$@"; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python tools/kbench.py fwd96 fwd96_nores dgrad96 fwd96_plain 2>&1 | grep -v amdgpu.ids | tee -a $O/kbench.log || exit 1
done
