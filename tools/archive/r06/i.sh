#!/bin/bash
# r06: N>1 rehearsal (two gloo ranks on one GPU), the stride-2 normalise-once path (bf16 step tests), step A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06_i; mkdir -p $O; cd $R
U3D_BENCH_BACKEND=gloo U3D_BENCH_SHARE_GPU=1 timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu --no-infer --no-roofline --no-mixed > $O/bench2.log 2>&1
rc=$?; grep -v amdgpu $O/bench2.log | tail -2 | cut -c1-600; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_graph.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab.sh r06_i "U3D_S2_NORM_ONCE=1" "U3D_S2_NORM_ONCE=0" 3
