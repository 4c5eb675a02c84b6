#!/bin/bash
# round 6: in-step slab-sum duration, in-tree lib vs libu3d_ab.so (kernel trace of the timed replays), twice
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06t; mkdir -p $O; cd $R
for i in 1 2; do for L in A B; do
  D=$O/$L$i; mkdir -p $D
  LIB=""; [ $L = B ] && LIB=$R/multimodal-pl_amd/u3d/libu3d_ab.so
  (cd /tmp && export TMPDIR=/tmp && U3D_LIB=$LIB timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/kt -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu --no-roofline --no-infer --no-mixed > $D/bench.log 2>&1) || { echo "prof failed"; exit 1; }
  f=$(find $D/kt -name '*kernel_trace.csv' | head -1); cp $f $D/
  python3 tools/prof_summary.py $D 10 60 steady > $D/summary.txt 2>&1
  echo "== $L$i $(head -1 $D/summary.txt)"; grep -E "sum_slabs|wstd_grad_row" $D/summary.txt | head -4
done; done
