#!/bin/bash
# r06: wider GN-backward parts finalize — parity of the fused GN backward, then a step A/B against the round's first lib
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06_e; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gnfused.py tests/test_gpu_epi_stats.py tests/test_gpu_bf16.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab.sh r06_e "U3D_LIB=" "U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_ab.so" 3
