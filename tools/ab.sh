#!/bin/bash
# A/B of bench.py step time on one box: tools/ab.sh TAG "ENV_A" "ENV_B" [rounds]   (alternating runs; ms per step)
TAG=$1; A=$2; B=$3; N=${4:-3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for i in $(seq $N); do
  for cfg in "$A" "$B"; do
    ms=$(env $cfg timeout -k 10 200 python bench.py --no-cpu --no-roofline --steps 30 --warmup 5 2>>$O/ab.err | python -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['ms_per_step'])") || exit 1
    echo "$cfg $ms" | tee -a $O/ab.log
  done
done
