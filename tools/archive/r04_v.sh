#!/bin/bash
# r04: upsample backward one-row gather with two planes of loads per round (in-tree) vs HEAD (libu3d_ab.so); the blocked
# form re-checked against it at 96^3 (UP_BWD_BLK=0/1); loss forward grid 512 (in-tree) vs 1024 (HEAD). Parity first.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_v
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_upsample_blk.py tests/test_gpu_parity.py tests/test_gpu_graph.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
L=$R/multimodal-pl_amd/u3d
for i in 1 2; do
  for v in "U3D_X=0" "U3D_LIB=$L/libu3d_ab.so" "U3D_UP_BWD_BLK=0" ; do
    echo "== $v" >> $O/kab.log
    env $v timeout -k 10 120 python tools/kbench.py upb96 upb48 upb24 upb12 loss96 >> $O/kab.log 2>&1 || { tail $O/kab.log; exit 1; }
  done
done
grep -v amdgpu.ids $O/kab.log
for i in 1 2; do
  for v in "U3D_X=0" "U3D_LIB=$L/libu3d_ab.so"; do
    ms=$(env $v timeout -k 10 200 python bench.py --no-cpu --no-roofline --no-infer --steps 40 2>>$O/ab.err | python -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['ms_per_step'])") || exit 1
    echo "$v $ms" | tee -a $O/ab.log
  done
done
