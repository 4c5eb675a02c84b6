#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/pmc_sq.sh r02au_sq fwd48 dgrad48 fwd24 wgrad96 dgrad96 > /dev/null 2>&1 || { echo "sq failed"; exit 1; }
python tools/pmc_summary.py gpurun_out/r02au_sq/run_counter_collection.csv
