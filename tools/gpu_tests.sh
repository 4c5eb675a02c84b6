#!/bin/bash
# Run selected GPU tests on the box: tools/gpu_tests.sh TAG <pytest args...>   (log: gpurun_out/TAG/pytest.log)
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R && timeout -k 10 1000 python -u -m pytest -v -s --timeout 300 --timeout-method thread "$@" > $O/pytest.log 2>&1
rc=$?
tail -15 $O/pytest.log
exit $rc
