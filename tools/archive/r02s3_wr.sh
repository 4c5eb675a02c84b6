#!/bin/bash
# wgrad ring 12 x 24 / 12 x 12 plane tiles: parity, micro-benchmarks both ways, step A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02s3_wr
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fullsize.py -k "wgrad" tests/test_gpu_bf16.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for t in 0 1; do
  echo "tile16=$t"; U3D_WR_TILE16=$t timeout -k 10 120 python tools/kbench.py wgrad24 wgrad12 wgrad48 2>/dev/null || exit 1
done | tee $O/kbench.log
bash tools/ab.sh r02s3_wr/ab "U3D_WR_TILE16=0" "U3D_WR_TILE16=1" 3 || exit 1
