#!/bin/bash
# Persistent brick conv with the LDS GroupNorm table: bitwise test, micro-benchmarks, ablations.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02s3_pb2
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pbrick.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for p in 1 0; do
  echo "persist=$p"; U3D_CONVG_PERSIST=$p timeout -k 10 120 python tools/kbench.py fwd48 dgrad48 fwd24 dgrad24 2>/dev/null || exit 1
done | tee $O/kbench.log
for a in 2 4 6 1; do
  echo -n "abl=$a "; U3D_PB_ABL=$a timeout -k 10 120 python tools/kbench.py fwd48 2>/dev/null | grep fwd48 || exit 1
done | tee $O/abl.log
