#!/bin/bash
# Generic A/B of the in-tree library against U3D_LIB=libu3d_ab.so (the previous build of one source):
# tools/lib_ab.sh TAG "KERNEL_REGEX" pytest-args...   -> tests, step A/B (3 rounds), per-kernel stats of both builds.
TAG=$1; KRX=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread "$@" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/ab.sh $TAG/ab "U3D_NONE=0" "U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_ab.so" ${LIB_AB_ROUNDS:-3} || exit 1
for L in "" "$R/multimodal-pl_amd/u3d/libu3d_ab.so"; do
  (cd /tmp && export TMPDIR=/tmp && U3D_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt${L:+_ab} -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --no-roofline > $O/kt${L:+_ab}.log 2>&1) || exit 1
  python3 $R/tools/kstats.py "$KRX" $(find $O/kt${L:+_ab} -name '*kernel_stats.csv') | sed "s|^|${L:+prev }|" | tee -a $O/kernels.csv
done
