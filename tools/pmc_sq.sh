#!/bin/bash
# SQ counter pass over kbench cases: tools/pmc_sq.sh TAG case...   (one --pmc pass, <= 8 SQ counters)
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc -o run -- python3 $R/tools/kbench.py "$@" > $O/pmc.log 2>&1
rc=$?
f=$(find $O/pmc -name '*counter_collection.csv' | head -1); [ -n "$f" ] && cp $f $O/
exit $rc
