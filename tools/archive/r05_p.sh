#!/bin/bash
# Round 5 batch p: persistent-brick unit granularity (CONVG_CO32 / CONVG_BW8 forced) at the 48^3 / 24^3 levels:
# kernel and step A/B.
TAG=${1:-r05_p}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for v in "A=1" "U3D_CONVG_CO32=1" "U3D_CONVG_BW8=1" "U3D_CONVG_CO32=1 U3D_CONVG_BW8=1"; do
  env $v timeout -k 10 120 python tools/kbench.py fwd48st fwd48st_nores dgrad48gn fwd24st dgrad24gn > $O/kb.log 2>&1; echo "== $v"; grep -v amdgpu.ids $O/kb.log
done
run() {  # run TAG ENV ARGS
  local t=$1; shift; local e=$1; shift
  env $e timeout -k 10 300 python bench.py --no-cpu --no-infer --no-roofline --no-mixed --steps 30 --warmup 5 "$@" > $O/bench_$t.log 2>&1 || { echo "bench $t failed"; grep -v "^frame" $O/bench_$t.log | tail -20; exit 1; }
  grep '^{' $O/bench_$t.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', d['ms_per_step'], d['launch'], d.get('graph_error'))"
}
for i in 1 2; do
  run def$i "A=1" || exit 1
  run co32_$i "U3D_CONVG_CO32=1" || exit 1
  run bw8_$i "U3D_CONVG_BW8=1" || exit 1
done
