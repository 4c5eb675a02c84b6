#!/bin/bash
# Vectorised weight-standardisation statistics / bf16 packs: parity, step A/B vs the previous build, kernel times.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02s3_wp
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bf16.py tests/test_gpu_parity.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/ab.sh r02s3_wp/ab "U3D_NONE=0" "U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_ab.so" 3 || exit 1
for L in "" "$R/multimodal-pl_amd/u3d/libu3d_ab.so"; do
  (cd /tmp && export TMPDIR=/tmp && U3D_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt${L:+_ab} -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --no-roofline > $O/kt${L:+_ab}.log 2>&1) || exit 1
  grep -h "wstd" $(find $O/kt${L:+_ab} -name '*kernel_stats.csv') | cut -d, -f1-5 | sed "s|^|${L:+prev }|"
done
