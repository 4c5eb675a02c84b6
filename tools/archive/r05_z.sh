#!/bin/bash
# Round 5 batch z: the loss forward with each voxel's 16 classes over a lane pair (LOSS_PAIR): tests, kernel and step
# A/B against the one-lane form (U3D_LOSS_PAIR=0).
TAG=${1:-r05_z}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_head_loss.py tests/test_gpu_parity.py tests/test_gpu_graph.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in "A=1" "U3D_LOSS_PAIR=0" "A=1" "U3D_LOSS_PAIR=0"; do
  env $v timeout -k 10 120 python tools/kbench.py loss96 > $O/kb.log 2>&1 || { cat $O/kb.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $O/kb.log
done
run() {  # run TAG ENV
  local t=$1; shift; local e=$1; shift
  env $e timeout -k 10 300 python bench.py --no-cpu --no-infer --no-roofline --no-mixed --steps 30 --warmup 5 "$@" > $O/bench_$t.log 2>&1 || { echo "bench $t failed"; grep -v "^frame" $O/bench_$t.log | tail -20; exit 1; }
  grep '^{' $O/bench_$t.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', d['ms_per_step'], d['launch'], d.get('graph_error'))"
}
for i in 1 2; do
  run new$i "A=1" || exit 1
  run onelane$i "U3D_LOSS_PAIR=0" || exit 1
done
