#!/bin/bash
# Round 5 batch v: the fused head + loss backward with the voxel's classes split over a lane pair, and the loss
# forward with two voxels in flight per thread: GPU tests, kernel and step A/B (libu3d_prev.so = before both).
TAG=${1:-r05_v}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_head_loss.py tests/test_gpu_graph.py tests/test_gpu_parity.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for L in libu3d.so libu3d_prev.so; do
  U3D_LIB=$R/multimodal-pl_amd/u3d/$L timeout -k 10 120 python tools/kbench.py headloss96 loss96 lossb96 headloss96 loss96 > $O/kb.log 2>&1 || { cat $O/kb.log; exit 1; }
  echo "== $L"; grep -v amdgpu.ids $O/kb.log
done
run() {  # run TAG ENV
  local t=$1; shift; local e=$1; shift
  env $e timeout -k 10 300 python bench.py --no-cpu --no-infer --no-roofline --no-mixed --steps 30 --warmup 5 "$@" > $O/bench_$t.log 2>&1 || { echo "bench $t failed"; grep -v "^frame" $O/bench_$t.log | tail -20; exit 1; }
  grep '^{' $O/bench_$t.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', d['ms_per_step'], d['launch'], d.get('graph_error'))"
}
for i in 1 2; do
  run new$i "A=1" || exit 1
  run prev$i "U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_prev.so" || exit 1
done
