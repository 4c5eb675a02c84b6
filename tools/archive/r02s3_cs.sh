#!/bin/bash
# conv_small with the LDS GroupNorm table: parity (bf16 paths incl. the forced small-conv route, bench-size trunk
# convs), micro-benchmarks, step A/B against the previous library build (U3D_LIB).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02s3_cs
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bf16.py tests/test_gpu_fullsize.py tests/test_gpu_pbrick.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python tools/kbench.py fwd12 dgrad12 fwd6nogn fwd12nogn 2>/dev/null | tee $O/kbench.log || exit 1
U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_ab.so timeout -k 10 120 python tools/kbench.py fwd12 dgrad12 2>/dev/null | sed 's/^/prev: /' | tee -a $O/kbench.log || exit 1
bash tools/ab.sh r02s3_cs/ab "U3D_NONE=0" "U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_ab.so" 3 || exit 1
