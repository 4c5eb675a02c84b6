#!/bin/bash
# r03: fused GroupNorm-backward partials in the ring data gradient: parity tests, then step/kernel A/B vs the
# separate partial pass (U3D_GN_BWD_FUSED=0)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03gf
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_gnfused.py tests/test_gpu_bf16.py tests/test_gpu_parity.py tests/test_gpu_ddp.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/env_ab.sh r03gf "gn_bwd|conv32_ring_kernel<true" U3D_GN_BWD_FUSED=1 U3D_GN_BWD_FUSED=0
