#!/bin/bash
# Persistent brick conv: bitwise test vs the one-shot kernel, bf16/full-size parity, micro-benchmarks both ways,
# step A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02s3_pb
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pbrick.py tests/test_gpu_bf16.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for p in 1 0; do
  U3D_CONVG_PERSIST=$p timeout -k 10 120 python tools/kbench.py fwd48 dgrad48 fwd24 dgrad24 > $O/kbench_p$p.log 2>&1 || { tail -5 $O/kbench_p$p.log; exit 1; }
  echo "persist=$p"; cat $O/kbench_p$p.log
done
bash tools/ab.sh r02s3_pb/ab "U3D_CONVG_PERSIST=1" "U3D_CONVG_PERSIST=0" 3 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest_all.log 2>&1 || { tail -30 $O/pytest_all.log; exit 1; }
tail -2 $O/pytest_all.log
