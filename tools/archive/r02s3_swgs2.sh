#!/bin/bash
# conv_small split-K target: 128 vs 256 (the new default), parity at 256, step A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02s3_swgs2
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bf16.py tests/test_gpu_fullsize.py -k "small or trunk_conv or c256" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for t in 128 256; do U3D_SMALL_WGS=$t timeout -k 10 120 python tools/kbench.py fwd12 dgrad12 fwd6nogn 2>/dev/null | sed "s/^/wgs=$t /"; done | tee $O/kbench.log
bash tools/ab.sh r02s3_swgs2/ab "U3D_SMALL_WGS=256" "U3D_SMALL_WGS=128" 2 || exit 1
