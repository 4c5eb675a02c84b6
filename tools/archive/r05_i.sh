#!/bin/bash
# Round 5 batch i: register weight-gradient rings (12 x 24 / 12 x 12 tiles) with the staging interleaved into the MFMA
# sub-steps: parity, kernel times, stamps; step A/B against the previous library (libu3d_prev.so) if present.
TAG=${1:-r05_i}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_bf16.py tests/test_gpu_s2ring.py -k "wgrad or s2" -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -cE "PASSED" $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|^E " $O/pytest.log | head -20; exit 1; }
timeout -k 10 120 python tools/kbench.py wgrad24 wgrad12 fwds2ring > $O/kb.log 2>&1 && grep -v amdgpu.ids $O/kb.log
if [ -f multimodal-pl_amd/u3d/libu3d_prev.so ]; then
  U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_prev.so timeout -k 10 120 python tools/kbench.py wgrad24 wgrad12 fwds2ring > $O/kb_prev.log 2>&1 && grep -v amdgpu.ids $O/kb_prev.log | sed 's/^/prev /'
fi
for c in wgrad24 wgrad12 s2ring96; do
  U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_stamps.so timeout -k 10 120 python tools/stamps.py $c > $O/stamps_$c.log 2>&1; tail -11 $O/stamps_$c.log
done
run() {  # run TAG ENV ARGS
  local t=$1; shift; local e=$1; shift
  env $e timeout -k 10 300 python bench.py --no-cpu --no-infer --no-roofline --no-mixed --steps 30 --warmup 5 "$@" > $O/bench_$t.log 2>&1 || { echo "bench $t failed"; grep -v "^frame" $O/bench_$t.log | tail -20; exit 1; }
  grep '^{' $O/bench_$t.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', d['ms_per_step'], d['launch'], d.get('graph_error'))"
}
if [ -f multimodal-pl_amd/u3d/libu3d_prev.so ]; then
  for i in 1 2; do
    run new$i "A=1" || exit 1
    run prev$i "U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_prev.so" || exit 1
  done
fi
