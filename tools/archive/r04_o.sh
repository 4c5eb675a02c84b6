#!/bin/bash
# r04: padded GN table in the data-gradient ring's GB epilogue (in-tree) vs libu3d_ab.so (HEAD): parity, kernel A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_o
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_gnfused.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
L=$R/multimodal-pl_amd/u3d
for i in 1 2 3; do
  for v in "U3D_X=0" "U3D_LIB=$L/libu3d_ab.so"; do
    echo "== $v" >> $O/kab.log
    env $v timeout -k 10 120 python tools/kbench.py dgrad96gn >> $O/kab.log 2>&1 || { tail $O/kab.log; exit 1; }
  done
done
grep -v amdgpu.ids $O/kab.log
for i in 1 2 3; do
  for v in 256 1024; do
    ms=$(U3D_GN_MAXBLK=$v timeout -k 10 200 python bench.py --no-cpu --no-roofline --no-infer --steps 30 2>>$O/ab.err | python -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['ms_per_step'])") || exit 1
    echo "gn_maxblk=$v $ms" | tee -a $O/ab.log
  done
done
