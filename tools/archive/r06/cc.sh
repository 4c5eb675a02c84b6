#!/bin/bash
# round 6: conv1 on the matrix cores (stem1_mfma_kernel): stem / stats / full-size tests, kernel A/B, step A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06cc; mkdir -p $O; cd $R
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_bf16.py -k "stem" tests/test_gpu_epi_stats.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/kab.sh r06cc 2 stem96st stem96 || exit 1
for i in 1 2 3; do for L in "" "$R/multimodal-pl_amd/u3d/libu3d_ab.so"; do
  ms=$(U3D_LIB=$L timeout -k 10 200 python bench.py --no-cpu --no-roofline --steps 30 --warmup 5 2>>$O/ab.err | python -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['ms_per_step'])") || exit 1
  echo "${L:+B}${L:-A} $ms" | tee -a $O/ab.log
done; done
