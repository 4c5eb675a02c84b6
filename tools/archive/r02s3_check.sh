#!/bin/bash
# Session-3 re-entry check on a fresh box: the GPU suite on the rebuilt tree, the 48^3/24^3 brick-conv micro-benchmarks
# and an SQ pass over them.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02s3_check
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 200 python tools/kbench.py fwd48 dgrad48 fwd24 dgrad24 wgrad48 wgrad24 wgrad12 fwd12nogn dgrad12 > $O/kbench.log 2>&1 || { tail -5 $O/kbench.log; exit 1; }
cat $O/kbench.log
bash tools/pmc_sq.sh r02s3_check/sq fwd48 dgrad48 fwd24 dgrad24 || exit 1
python tools/pmc_summary.py $O/sq/*counter_collection.csv 2>/dev/null | head -40 || true
