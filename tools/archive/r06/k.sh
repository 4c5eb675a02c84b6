#!/bin/bash
# r06: separable upsample backward tile variants (UP_BWD_SEP 1: 2x4x16 / 2: 2x8x16 / 3: 4x4x16 / 4: 4x8x16; 0: gather)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06_k; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_upsample_sep.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for v in 0 1 2 3 4; do echo "== SEP=$v" >> $O/kb.log; U3D_UP_BWD_SEP=$v timeout -k 10 120 python tools/kbench.py upb96 upb48 >> $O/kb.log 2>&1 || exit 1; done; done
grep -v amdgpu $O/kb.log
