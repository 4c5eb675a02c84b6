#!/bin/bash
# r04: stride-2 two-consumer GroupNorm backward — conditional compact loads (COND), 16 vectors per apply thread (APV),
# 4-voxel partial rounds (PR): parity, kernel A/B of in-tree vs gn2old (r3 form) / gn2c (COND) / gn2a (COND+APV)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_p
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv1x1.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
L=$R/multimodal-pl_amd/u3d
for i in 1 2; do
  for v in "" "$L/gn2old.so" "$L/gn2c.so" "$L/gn2a.so"; do
    echo "== ${v:-in-tree}" >> $O/kab.log
    U3D_LIB=$v timeout -k 10 120 python tools/kbench.py gnbwd2s96 gnbwd2s48 gnbwd2s24 gnbwd96 gnbwd2s12 >> $O/kab.log 2>&1 || { tail $O/kab.log; exit 1; }
  done
done
grep -v amdgpu.ids $O/kab.log
