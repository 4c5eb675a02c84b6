#!/bin/bash
# r04: eager (kernel-by-kernel launches from Python) vs whole-step hipGraph replay of the same step, alternating x3
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_k
mkdir -p $O
cd $R
for i in 1 2 3; do
  for a in "" "--graph"; do
    ms=$(timeout -k 10 200 python bench.py --no-cpu --no-roofline --no-infer --steps 30 $a 2>>$O/ab.err | python -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['ms_per_step'])") || exit 1
    echo "eager${a} $ms" | tee -a $O/ab.log
  done
done
L=$R/multimodal-pl_amd/u3d
for i in 1 2; do
  for v in "U3D_X=0" "U3D_LIB=$L/libu3d_ab46.so" "U3D_LIB=$L/libu3d_abcc.so"; do
    echo "== $v" >> $O/kab.log
    env $v timeout -k 10 120 python tools/kbench.py fwd48st fwd48st_nores fwd24st >> $O/kab.log 2>&1 || { tail $O/kab.log; exit 1; }
  done
done
grep -v amdgpu.ids $O/kab.log
