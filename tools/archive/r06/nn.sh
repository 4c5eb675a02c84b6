#!/bin/bash
# round 6: stride-2 brick weight gradient with 3-plane output bricks (tree; U3D_WB_S2BD=2 = 2-plane bricks in the same
# library; libu3d_head = the committed kernels): tests, kbench 3 rounds, step A/B 3 rounds
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06nn; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bf16.py \
  tests/test_gpu_wgrad_dma.py tests/test_gpu_slabsum.py -k "wgrad or slab" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fullsize.py \
  -k "wgrad" > $O/tests2.log 2>&1 || { tail -30 $O/tests2.log; exit 1; }
tail -1 $O/tests2.log
for i in 1 2 3; do for V in tree bd2 head; do
  echo "== $V" >> $O/kb.log
  E=""; L=""; [ $V = bd2 ] && E=2; [ $V = head ] && L=$R/multimodal-pl_amd/u3d/libu3d_head.so
  U3D_WB_S2BD=${E:-3} U3D_LIB=$L timeout -k 10 120 python tools/kbench.py wgrad_s2_96 wgrad_s2_48 wgrad_s2_24 >> $O/kb.log 2>&1 || exit 1
done; done
grep -v amdgpu.ids $O/kb.log | paste - - - -
for i in 1 2 3; do for V in tree bd2 head; do
  E=""; L=""; [ $V = bd2 ] && E=2; [ $V = head ] && L=$R/multimodal-pl_amd/u3d/libu3d_head.so
  ms=$(U3D_WB_S2BD=${E:-3} U3D_LIB=$L timeout -k 10 200 python bench.py --no-cpu --no-roofline --steps 30 --warmup 5 2>>$O/ab.err | python -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['ms_per_step'])") || exit 1
  echo "$V $ms" | tee -a $O/ab.log
done; done
