#!/bin/bash
# round 6: head GN backward with the in-kernel bias-gradient sum: its tests, then a step A/B (A = fused, B = the two
# channel-sum launches, U3D_HEAD_DBIAS_FUSED=0), 4 rounds
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06jj; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_head_loss.py \
  tests/test_gpu_head_oracle.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2 3 4; do for F in 1 0; do
  ms=$(U3D_HEAD_DBIAS_FUSED=$F timeout -k 10 200 python bench.py --no-cpu --no-roofline --steps 30 --warmup 5 2>>$O/ab.err | python -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['ms_per_step'])") || exit 1
  echo "fused=$F $ms" | tee -a $O/ab.log
done; done
