#!/bin/bash
# r06: separable LDS-tiled upsample backward — parity, kernel and step A/B against the gather kernels
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06_j; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_upsample_sep.py tests/test_gpu_upsample_blk.py tests/test_gpu_parity.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for v in 1 0; do echo "== SEP=$v" >> $O/kb.log; U3D_UP_BWD_SEP=$v timeout -k 10 120 python tools/kbench.py upb96 upb48 >> $O/kb.log 2>&1 || exit 1; done; done
grep -v amdgpu $O/kb.log
bash tools/ab.sh r06_j "U3D_UP_BWD_SEP=1" "U3D_UP_BWD_SEP=0" 3
