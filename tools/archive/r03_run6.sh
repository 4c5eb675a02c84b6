#!/bin/bash
# r03: ring convs with staging loads two planes ahead (in-tree PF=2) vs one (libu3d_ab.so, -DU3D_RING_PF=1);
# persistent brick data gradient on a work queue (bitwise tests, concurrency with CUs held)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03o
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pbrick.py tests/test_gpu_queue.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/kab.sh r03o/kab 2 fwd96 fwd96_nores dgrad96 wgrad96 wgrad48 wgrad24 || exit 1
bash tools/ab.sh r03o/ab "U3D_NONE=0" "U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_ab.so" 3 || exit 1
timeout -k 10 300 python tools/concurrency.py 8 32 > $O/concurrency.json 2> $O/concurrency.err || { tail -20 $O/concurrency.err; exit 1; }
cat $O/concurrency.json
