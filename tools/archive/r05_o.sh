#!/bin/bash
# Round 5 batch o: weight-standardisation backward (coalesced row gather, binary descriptor search): parity, the cold
# end-of-backward batch alone (tools/r05_slab.py) new vs previous library, step A/B.
TAG=${1:-r05_o}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_slabsum.py tests/test_gpu_ddp.py tests/test_gpu_graph.py tests/test_gpu_fullsize.py -k "wstd or slab or ddp or graph or wgrad" -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -cE "PASSED" $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|^E " $O/pytest.log | head -30; exit 1; }
timeout -k 10 200 python tools/r05_slab.py > $O/slab.log 2>&1; grep -v amdgpu.ids $O/slab.log
U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_prev.so timeout -k 10 200 python tools/r05_slab.py > $O/slab_prev.log 2>&1; grep -v amdgpu.ids $O/slab_prev.log | sed 's/^/prev /'
run() {  # run TAG ENV ARGS
  local t=$1; shift; local e=$1; shift
  env $e timeout -k 10 300 python bench.py --no-cpu --no-infer --no-roofline --no-mixed --steps 30 --warmup 5 "$@" > $O/bench_$t.log 2>&1 || { echo "bench $t failed"; grep -v "^frame" $O/bench_$t.log | tail -20; exit 1; }
  grep '^{' $O/bench_$t.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', d['ms_per_step'], d['launch'], d.get('graph_error'))"
}
for i in 1 2; do
  run new$i "A=1" || exit 1
  run prev$i "U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_prev.so" || exit 1
done
