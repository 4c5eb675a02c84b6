#!/bin/bash
# Round 5: backward side-stream branches (trunk.SIDE_MAX_VOX) and the new bucket plan. Tests, then bench A/B.
TAG=${1:-r05_side}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_ddp.py -x -v -s --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
grep -E "PASS|FAIL|bitwise|worst" $O/pytest.log | cut -c1-250
for i in 1 2; do
  for v in 0 3456 27648 221184; do
    U3D_SIDE_MAX_VOX=$v timeout -k 10 300 python bench.py --no-cpu --no-infer --no-roofline --no-mixed --steps 30 --warmup 5 > $O/bench_${i}_$v.log 2>&1 || { echo "bench $v failed"; tail -20 $O/bench_${i}_$v.log; exit 1; }
    grep '^{' $O/bench_${i}_$v.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('side', $v, d['ms_per_step'], d['launch'])"
  done
  timeout -k 10 300 python bench.py --no-cpu --no-infer --no-roofline --no-mixed --steps 30 --warmup 5 --force-buckets > $O/bench_fb$i.log 2>&1 || { echo "bench fb failed"; tail -20 $O/bench_fb$i.log; exit 1; }
  grep '^{' $O/bench_fb$i.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('fb', d['ms_per_step'], d['launch'], d.get('graph_error'))"
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu --no-roofline --no-infer --no-mixed > $O/bench_kt.log 2>&1) || { echo "prof failed"; tail -20 $O/bench_kt.log; exit 1; }
f=$(find $O/kt -name '*kernel_trace.csv' | head -1); [ -n "$f" ] && cp $(dirname $f)/*.csv $O/
python3 tools/prof_summary.py $O 16 > $O/kernel_summary.txt 2>&1 || true
head -12 $O/kernel_summary.txt
