cd ${GRAFT_REPO_ROOT:-$(pwd)}
for sc in 100 9 5 3; do echo "SC=$sc"; U3D_RING_SC=$sc timeout -k 10 120 python tools/concurrency.py 8 2>&1 | tail -1; done
