#!/bin/bash
# Round-6 closing check, part 1: the whole GPU suite and smoke() on one box (logs under gpurun_out/r06_end)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06_end; mkdir -p $O; cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
