#!/bin/bash
# Persistent brick conv, residual loads issued before the last step.s staging commit: bitwise tests, micro-benchmarks vs the
# previous build (U3D_LIB=libu3d_ab.so), step A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02s3_rv
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pbrick.py tests/test_gpu_fullsize.py -k "pbrick or trunk_conv_fwd or trunk_conv_dgrad or persistent" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python tools/kbench.py fwd48 dgrad48 fwd24 dgrad24 2>/dev/null | tee $O/kbench.log || exit 1
U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_ab.so timeout -k 10 120 python tools/kbench.py fwd48 dgrad48 fwd24 dgrad24 2>/dev/null | sed 's/^/prev: /' | tee -a $O/kbench.log || exit 1
bash tools/ab.sh r02s3_rv/ab "U3D_NONE=0" "U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_ab.so" 3 || exit 1
