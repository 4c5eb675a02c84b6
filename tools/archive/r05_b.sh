#!/bin/bash
# Round 5: epilogue GN statistics (stem, upsample) tests + step A/B, then the bucket plans of the forced-bucket step.
TAG=${1:-r05_b}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests/test_gpu_epi_stats.py tests/test_gpu_graph.py tests/test_gpu_gnfused_brick.py tests/test_gpu_ddp.py tests/test_gpu_gnfused_small.py tests/test_gpu_pbrick.py tests/test_gpu_fullsize.py -x -v -s --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
grep -E "PASS|FAIL|err" $O/pytest.log | cut -c1-200
run() {  # run TAG ENV ARGS
  local t=$1; shift; local e=$1; shift
  env $e timeout -k 10 300 python bench.py --no-cpu --no-infer --no-roofline --no-mixed --steps 30 --warmup 5 "$@" > $O/bench_$t.log 2>&1 || { echo "bench $t failed"; grep -v "^frame" $O/bench_$t.log | tail -20; exit 1; }
  grep '^{' $O/bench_$t.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', d['ms_per_step'], d['launch'], d.get('graph_error'))"
}
for i in 1 2 3; do
  run off$i "U3D_STEM_STATS=0 U3D_UP_STATS=0 U3D_SMALL_FUSE=0 U3D_FUSED_FINALIZE=0 U3D_SMALL_GB=0" || exit 1
  run on$i "U3D_STEM_STATS=1 U3D_UP_STATS=1 U3D_SMALL_FUSE=1 U3D_FUSED_FINALIZE=1" || exit 1
done
run fb25_25 "A=1" --force-buckets --bucket-mb 25 --tail-mb 25 || exit 1
run fb40_2 "A=1" --force-buckets --bucket-mb 40 --tail-mb 2 || exit 1
run fb25_2 "A=1" --force-buckets --bucket-mb 25 --tail-mb 2 || exit 1
run fb34_34 "A=1" --force-buckets --bucket-mb 34 --tail-mb 34 || exit 1
run fb100 "A=1" --force-buckets --bucket-mb 100 --tail-mb 100 || exit 1
run plain "A=1" || exit 1
