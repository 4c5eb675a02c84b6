#!/bin/bash
# round 6: GroupNorm backward from partials in one launch (gn_bwd_apply_parts): tests, kernel A/B (gnb96f etc.), step A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06aa; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gn_apply_parts.py tests/test_gpu_gnfused.py tests/test_gpu_gnfused_brick.py tests/test_gpu_head_loss.py tests/test_gpu_head_oracle.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/kab.sh r06aa 3 gnb96f || exit 1
for i in 1 2 3; do for L in "" "$R/multimodal-pl_amd/u3d/libu3d_ab.so"; do
  ms=$(U3D_LIB=$L timeout -k 10 200 python bench.py --no-cpu --no-roofline --steps 30 --warmup 5 2>>$O/ab.err | python -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['ms_per_step'])") || exit 1
  echo "${L:+B}${L:-A} $ms" | tee -a $O/ab.log
done; done
