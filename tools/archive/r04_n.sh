#!/bin/bash
# r04: bench lines after the host-side changes (raw stream accessor, probes out of the timed region): default (graph),
# --eager, --force-buckets, alternating x2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_n
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_ddp.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  for a in "" "--eager" "--force-buckets"; do
    timeout -k 10 300 python bench.py --no-cpu --no-infer $a > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
    grep '^{' $O/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$a', d['launch'], d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r['frac'])" | tee -a $O/lines.log
  done
done
