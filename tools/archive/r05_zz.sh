#!/bin/bash
# Round 5 batch zz: the SGD learning-rate tensor rewritten only on change (no fill launch before every replay):
# graph tests (incl. an LR schedule across replays), one bench line.
TAG=${1:-r05_zz}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_graph.py tests/test_gpu_ddp.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --no-cpu --no-infer --no-roofline --no-mixed --steps 30 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 | cut -c1-200
