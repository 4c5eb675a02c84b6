#!/bin/bash
# r04: fp32-reciprocal voxel division + size-dependent apply work in the stride-2 two-consumer GN backward vs gn2c
# (conditional compact loads only); per-kernel split from a rocprofv3 kernel-trace of the in-tree 96^3 case
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_q
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv1x1.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
L=$R/multimodal-pl_amd/u3d
for i in 1 2; do
  for v in "" "$L/gn2c.so"; do
    echo "== ${v:-in-tree}" >> $O/kab.log
    U3D_LIB=$v timeout -k 10 120 python tools/kbench.py gnbwd2s96 gnbwd2s48 gnbwd2s24 gnbwd2s12 >> $O/kab.log 2>&1 || { tail $O/kab.log; exit 1; }
  done
done
grep -v amdgpu.ids $O/kab.log
cd /tmp && export TMPDIR=/tmp
for v in "" "$L/gn2c.so"; do
  U3D_LIB=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof${v:+_c} -o run --output-format csv -- python $R/tools/kbench.py gnbwd2s96 > /dev/null 2>&1 || exit 1
  f=$(find $O/prof${v:+_c} -name "*kernel_stats.csv" | head -1)
  echo "== ${v:-in-tree}"; cut -d, -f1-5 $f | grep -i "gn_bwd2" 
done
