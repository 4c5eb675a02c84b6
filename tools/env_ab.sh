#!/bin/bash
# Step + kernel A/B of two option settings on one box: tools/env_ab.sh TAG "KERNEL_REGEX" "ENV_A" "ENV_B"
# -> ab.log (3 alternating rounds, ms per step) and kernels.csv (per-kernel stats of one profiled run of each)
TAG=$1; KRX=$2; A=$3; B=$4
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
bash tools/ab.sh $TAG "$A" "$B" 3 || exit 1
for cfg in "$A" "$B"; do
  k=$(echo "$cfg" | tr -c 'A-Za-z0-9\n' '_')
  (cd /tmp && export TMPDIR=/tmp && export $cfg && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$k -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --no-roofline > $O/kt_$k.log 2>&1) || exit 1
  python3 $R/tools/kstats.py "$KRX" $(find $O/kt_$k -name '*kernel_stats.csv') | sed "s|^|$k |" | tee -a $O/kernels.csv
done
