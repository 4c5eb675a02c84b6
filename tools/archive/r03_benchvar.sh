#!/bin/bash
# r03: bench variance check on one box: default line vs the A/B form, before and after a PMC pass
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03bv
mkdir -p $O
cd $R
b() { timeout -k 10 300 python bench.py "$@" 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['avg_launch_ms'] if d.get('roofline') else '')"; }
echo "default: $(b)" | tee -a $O/log
echo "ab form: $(b --no-cpu --no-roofline --steps 30)" | tee -a $O/log
echo "default: $(b)" | tee -a $O/log
echo "steps30: $(b --no-cpu --steps 30)" | tee -a $O/log
bash tools/pmc_conv32.sh gpurun_out/r03bv/pmc.json > $O/pmc.log 2>&1 || exit 1
echo "after pmc default: $(b)" | tee -a $O/log
echo "after pmc ab form: $(b --no-cpu --no-roofline --steps 30)" | tee -a $O/log
