#!/bin/bash
# pods_syev with k_larft on a second stream beside the bisection / eigenvectors of T (this build)
# against the previous commit's library (variants/libpodsgen_prev.so): the eigen tests under this
# build, pods_syev at n = 4096 and the C3 bench, alternating processes.
set -o pipefail
O=${1:-gpurun_out/r6lf}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=$GRAFT_REPO_ROOT/pods-digital-filter_amd/podsgen/variants/libpodsgen_prev.so
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_eigen.py > $O/eigen_tests.log 2>&1 || exit 2
B="python3 -u bench.py --steps 20 --warmup 5 --no-cpu"
for i in 1 2; do
  timeout -k 10 120 python -u tools/syev_ab.py 10 > $O/syev_new_$i.log 2>&1 || exit 3
  PODSGEN_LIB=$V timeout -k 10 120 python -u tools/syev_ab.py 10 > $O/syev_prev_$i.log 2>&1 || exit 4
  timeout -k 10 170 $B > $O/bench_new_$i.json 2>> $O/err.log || exit 5
  PODSGEN_LIB=$V timeout -k 10 170 $B > $O/bench_prev_$i.json 2>> $O/err.log || exit 6
done
echo larft-done
