#!/bin/bash
# r06: spread + interleaved ring schedule (libu3d_ab = -DU3D_RING_SPREAD=1): parity under the variant, kernel A/B, step A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06_f; mkdir -p $O; cd $R
U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_ab.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_gnfused.py tests/test_gpu_epi_stats.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/kab.sh r06_f 3 fwd96 fwd96nr dgrad96gn wgrad96 > /dev/null || exit 1
grep -v amdgpu $O/kab.log
bash tools/ab.sh r06_f "U3D_LIB=" "U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_ab.so" 3
