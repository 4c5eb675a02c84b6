#!/bin/bash
# Round 5 batch g: stride-2 ring stamps, step A/B of the in-launch finalize (now off by default) and the eager slab
# sum restricted to >= 16 slabs.
TAG=${1:-r05_g}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_stamps.so timeout -k 10 120 python tools/stamps.py s2ring96 > $O/stamps_s2.log 2>&1; tail -12 $O/stamps_s2.log
run() {  # run TAG ENV ARGS
  local t=$1; shift; local e=$1; shift
  env $e timeout -k 10 300 python bench.py --no-cpu --no-infer --no-roofline --no-mixed --steps 30 --warmup 5 "$@" > $O/bench_$t.log 2>&1 || { echo "bench $t failed"; grep -v "^frame" $O/bench_$t.log | tail -20; exit 1; }
  grep '^{' $O/bench_$t.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', d['ms_per_step'], d['launch'], d.get('graph_error'))"
}
for i in 1 2 3; do
  run def$i "A=1" || exit 1
  run ff$i "U3D_FUSED_FINALIZE=1" || exit 1
  run slab16_$i "U3D_EAGER_SLAB_SUM=1 U3D_EAGER_SLAB_MIN=16" || exit 1
done
