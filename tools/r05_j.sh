#!/bin/bash
# Round 5 batch j: 4-wave 96^3 rings (U3D_RING_NW=4: one wave per SIMD, two h-rows per wave, weights in registers):
# parity under the option, kernel A/B, step A/B.
TAG=${1:-r05_j}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
U3D_RING_NW=4 timeout -k 10 400 python -u -m pytest tests/test_gpu_gnfused.py tests/test_gpu_epi_stats.py tests/test_gpu_fullsize.py tests/test_gpu_bf16.py -k "ring or fused or trunk_conv or stats" -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -cE "PASSED" $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|^E " $O/pytest.log | head -30; exit 1; }
for nw in 8 4; do
  U3D_RING_NW=$nw timeout -k 10 120 python tools/kbench.py fwd96 fwd96_nores dgrad96gn > $O/kb_$nw.log 2>&1 && grep -v amdgpu.ids $O/kb_$nw.log | sed "s/^/nw$nw /"
done
run() {  # run TAG ENV ARGS
  local t=$1; shift; local e=$1; shift
  env $e timeout -k 10 300 python bench.py --no-cpu --no-infer --no-roofline --no-mixed --steps 30 --warmup 5 "$@" > $O/bench_$t.log 2>&1 || { echo "bench $t failed"; grep -v "^frame" $O/bench_$t.log | tail -20; exit 1; }
  grep '^{' $O/bench_$t.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', d['ms_per_step'], d['launch'], d.get('graph_error'))"
}
for i in 1 2; do
  run nw8_$i "U3D_RING_NW=8" || exit 1
  run nw4_$i "U3D_RING_NW=4" || exit 1
done
