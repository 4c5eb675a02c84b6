#!/bin/bash
# 8-wide persistent bricks at 24^3: bitwise + bench-size parity, micro-benchmarks (both widths via U3D_CONVG_BW8),
# step A/B against the previous build.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02s3_bw8
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pbrick.py tests/test_gpu_fullsize.py -k "pbrick or persistent or trunk_conv_fwd or trunk_conv_dgrad" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for b in 1 0; do U3D_CONVG_BW8=$b timeout -k 10 120 python tools/kbench.py fwd24 dgrad24 2>/dev/null | sed "s/^/bw8=$b /"; done | tee $O/kbench.log
bash tools/ab.sh r02s3_bw8/ab "U3D_NONE=0" "U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_ab.so" 3 || exit 1
