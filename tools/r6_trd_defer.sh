#!/bin/bash
# k_trd with the rank-2 update deferred into the next column's first hand-off poll (ranges >= 3,
# PODS_TRD_DEFER=1, variants/libpodsgen_defer.so): the eigen tests under it (short limits, verbose),
# pods_syev at n = 4096 against the product in alternating processes (spectra checksums), the
# per-column trace and hop view, and the C3 bench with it against the product.
set -o pipefail
O=${1:-gpurun_out/r6df}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=$GRAFT_REPO_ROOT/pods-digital-filter_amd/podsgen/variants/libpodsgen_defer.so
PODSGEN_LIB=$V timeout -k 10 150 python -u -m pytest -x -v --timeout 60 --timeout-method thread tests/test_gpu_eigen.py -k "test_syev_pod_like and (1025 or 2048 or 2049 or 4096)" > $O/eigen_pod_like_defer.log 2>&1 || exit 2
PODSGEN_LIB=$V timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_eigen.py > $O/eigen_tests_defer.log 2>&1 || exit 3
for i in 1 2; do
  timeout -k 10 120 python -u tools/syev_ab.py 10 > $O/syev_prod_$i.log 2>&1 || exit 4
  PODSGEN_LIB=$V timeout -k 10 120 python -u tools/syev_ab.py 10 > $O/syev_defer_$i.log 2>&1 || exit 5
done
PODSGEN_LIB=$V timeout -k 10 150 python -u tools/trd_trace.py 4096 0 255 > $O/trd_trace_defer.log 2>&1 || exit 6
PODSGEN_LIB=$V timeout -k 10 150 python -u tools/trd_hop.py 4096 > $O/trd_hop_defer.log 2>&1 || exit 7
B="python3 -u bench.py --steps 20 --warmup 5 --no-cpu"
for i in 1 2; do
  timeout -k 10 170 $B > $O/bench_prod_$i.json 2>> $O/err.log || exit 8
  PODSGEN_LIB=$V timeout -k 10 170 $B > $O/bench_defer_$i.json 2>> $O/err.log || exit 9
done
echo defer-done
