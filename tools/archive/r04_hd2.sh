#!/bin/bash
# r04: head grid cap 768 (in-tree) vs 2048 (HEAD, libu3d_ab.so): head / parity / DDP tests, smoke, step A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_hd2
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_parity.py tests/test_gpu_ddp.py tests/test_gpu_graph.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
L=$R/multimodal-pl_amd/u3d
for i in 1 2 3; do
  for v in "U3D_X=0" "U3D_LIB=$L/libu3d_ab.so"; do
    ms=$(env $v timeout -k 10 200 python bench.py --no-cpu --no-roofline --no-infer --steps 40 2>>$O/ab.err | python -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['ms_per_step'])") || exit 1
    echo "$v $ms" | tee -a $O/ab.log
  done
done
