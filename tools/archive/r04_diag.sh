#!/bin/bash
# r04 ring diagnostics on one box: in-kernel clock + phase stamps (-DU3D_STAMPS build), SQ pass and HBM traffic of
# the three 96^3 ring kernels.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_diag
mkdir -p $O
cd $R
for c in wgrad96 dgradgn96 fwd96 wgrad48; do
  U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_stamps.so timeout -k 10 120 python tools/stamps.py $c 2.5 >> $O/stamps.txt 2>&1 || { tail -20 $O/stamps.txt; exit 1; }
done
cat $O/stamps.txt | grep -v amdgpu.ids
for c in wgrad96 dgrad96gn fwd96; do
  bash tools/pmc_sq.sh r04_sq_$c $c > /dev/null 2>&1 || { echo "sq $c failed"; exit 1; }
  python3 tools/pmc_summary.py gpurun_out/r04_sq_$c/run_counter_collection.csv > $O/sq_$c.txt 2>&1
  echo "== SQ $c"; tail -12 $O/sq_$c.txt
done
bash tools/pmc_ring.sh wgrad96 "wgrad_ring_kernel<true, 16, 16>" profiles/r04_pmc_wgrad96.json || exit 1
bash tools/pmc_ring.sh dgrad96gn "conv32_ring_kernel<true, true, false" profiles/r04_pmc_dgrad96gn.json || exit 1
bash tools/pmc_ring.sh fwd96 "conv32_ring_kernel<false, true, true" profiles/r04_pmc_fwd96.json || exit 1
cp profiles/r04_pmc_*.json $O/
