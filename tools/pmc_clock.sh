#!/bin/bash
# Clock / MFMA-busy PMC pass over kbench cases: tools/pmc_clock.sh TAG "ENV=.. ENV2=.." case...
TAG=$1; shift; ENVS=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
env $ENVS timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY --output-format csv -d $O/pmc -o run -- python3 $R/tools/kbench.py "$@" > $O/pmc.log 2>&1
rc=$?
f=$(find $O/pmc -name '*counter_collection.csv' | head -1); [ -n "$f" ] && cp $f $O/
exit $rc
