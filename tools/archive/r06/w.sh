#!/bin/bash
# round 6: weight-standardisation backward row kernel (buffer loads, no per-element division): tests, then in-step
# kernel trace in-tree (A) vs libu3d_ab.so (B), twice
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06w; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bf16.py -k "wstd" tests/test_gpu_slabsum.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do for L in A B; do
  D=$O/$L$i; mkdir -p $D
  LIB=""; [ $L = B ] && LIB=$R/multimodal-pl_amd/u3d/libu3d_ab.so
  (cd /tmp && export TMPDIR=/tmp && U3D_LIB=$LIB timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/kt -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu --no-roofline --no-infer --no-mixed > $D/bench.log 2>&1) || { echo "prof failed"; exit 1; }
  f=$(find $D/kt -name '*kernel_trace.csv' | head -1); cp $f $D/
  python3 tools/prof_summary.py $D 10 60 steady > $D/summary.txt 2>&1
  echo "== $L$i $(head -1 $D/summary.txt)"; grep -E "wstd_grad_row" $D/summary.txt | head -2
done; done
