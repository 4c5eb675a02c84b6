#!/bin/bash
# Persistent stride-2 data gradient: bitwise test, parity (bench-size trunk dgrads, bf16 paths), micro-benchmarks vs
# the previous build (U3D_LIB=libu3d_ab.so), step A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02s3_ds2
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pbrick.py tests/test_gpu_fullsize.py tests/test_gpu_bf16.py -k "dgrad" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python tools/kbench.py dgrad_s2_96 dgrad_s2_48 dgrad_s2_24 dgrad_s2_12 2>/dev/null | tee $O/kbench.log || exit 1
U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_ab.so timeout -k 10 120 python tools/kbench.py dgrad_s2_96 dgrad_s2_48 dgrad_s2_24 dgrad_s2_12 2>/dev/null | sed 's/^/prev: /' | tee -a $O/kbench.log || exit 1
bash tools/ab.sh r02s3_ds2/ab "U3D_NONE=0" "U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_ab.so" 3 || exit 1
