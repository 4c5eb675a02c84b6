#!/bin/bash
# round 6: conv1 weight gradient with branch-free B fragments: tests, kbench (tree = 4-plane bricks, bd2new = 2-plane
# with the new fragments, bd2 = the committed kernel), step A/B tree vs bd2, 3 rounds
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06mm; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bf16.py \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "stem or conv1" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do for L in "" bd2new bd2; do
  echo "== ${L:-tree}" >> $O/kb.log
  U3D_LIB=${L:+$R/multimodal-pl_amd/u3d/libu3d_$L.so} timeout -k 10 120 python tools/kbench.py stemw96 >> $O/kb.log 2>&1 || exit 1
done; done
grep -v amdgpu.ids $O/kb.log | paste - -
for i in 1 2 3; do for L in "" bd2; do
  ms=$(U3D_LIB=${L:+$R/multimodal-pl_amd/u3d/libu3d_$L.so} timeout -k 10 200 python bench.py --no-cpu --no-roofline --steps 30 --warmup 5 2>>$O/ab.err | python -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['ms_per_step'])") || exit 1
  echo "${L:-tree} $ms" | tee -a $O/ab.log
done; done
