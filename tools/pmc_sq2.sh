#!/bin/bash
# Pipe-level SQ passes over kbench cases (round 6): tools/pmc_sq2.sh TAG case...  -> gpurun_out/TAG/{a,b}_counter_collection.csv
# pass a: per-pipe active / issue-stall cycles; pass b: instruction counts and LDS queue pressure (<= 8 SQ counters each)
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pa -o run -- python3 $R/tools/kbench.py "$@" > $O/pa.log 2>&1 || exit 1
f=$(find $O/pa -name '*counter_collection.csv' | head -1); [ -n "$f" ] && cp $f $O/a_counter_collection.csv
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_LEVEL_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $O/pb -o run -- python3 $R/tools/kbench.py "$@" > $O/pb.log 2>&1 || exit 1
f=$(find $O/pb -name '*counter_collection.csv' | head -1); [ -n "$f" ] && cp $f $O/b_counter_collection.csv
