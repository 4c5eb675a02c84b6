#!/bin/bash
# Stride-2 weight-gradient brick shapes (U3D_WGRAD_S2B 0/1/2): parity at each, micro-benchmarks, step A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02s3_ws2
mkdir -p $O
cd $R
for b in 0 1 2; do
  U3D_WGRAD_S2B=$b timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bf16.py tests/test_gpu_fullsize.py -k "wgrad" > $O/pytest_$b.log 2>&1 || { tail -30 $O/pytest_$b.log; exit 1; }
  echo "s2b=$b $(tail -1 $O/pytest_$b.log)"
  U3D_WGRAD_S2B=$b timeout -k 10 120 python tools/kbench.py wgrad_s2_96 wgrad_s2_48 wgrad_s2_24 2>/dev/null | sed "s/^/s2b=$b /"
done | tee $O/kbench.log
bash tools/ab.sh r02s3_ws2/ab1 "U3D_WGRAD_S2B=0" "U3D_WGRAD_S2B=1" 2 || exit 1
bash tools/ab.sh r02s3_ws2/ab2 "U3D_WGRAD_S2B=0" "U3D_WGRAD_S2B=2" 2 || exit 1
