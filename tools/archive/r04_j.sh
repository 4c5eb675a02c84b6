#!/bin/bash
# r04: one-row-per-block weight-standardisation backward (U3D_WSTD_ROW=1 vs 0): parity, step A/B; forced-bucket
# step with the coalesced zero fills (plain vs --force-buckets, alternating)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_j
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_ddp.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
  for v in 1 0; do
    ms=$(U3D_WSTD_ROW=$v timeout -k 10 200 python bench.py --no-cpu --no-roofline --no-infer --steps 30 2>>$O/ab.err | python -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['ms_per_step'])") || exit 1
    echo "wstd_row=$v $ms" | tee -a $O/ab.log
  done
done
for i in 1 2; do
  for a in "" "--force-buckets"; do
    ms=$(timeout -k 10 200 python bench.py --no-cpu --no-roofline --no-infer --steps 30 $a 2>>$O/fb.err | python -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['ms_per_step'])") || exit 1
    echo "plain${a} $ms" | tee -a $O/fb.log
  done
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu --no-roofline --no-infer > $O/bench_kt.log 2>&1) || { echo "prof failed"; exit 1; }
f=$(find $O/kt -name '*kernel_trace.csv' | head -1); [ -n "$f" ] && cp $(dirname $f)/*.csv $O/
python3 tools/prof_summary.py $O 13 > $O/kernel_summary.txt 2>&1 || true
grep -i "wstd\|busy" $O/kernel_summary.txt | head
