#!/bin/bash
# k_trd change A/B on the box: pods_syev at n = 4096 (this build vs the r5 build, alternating
# processes), the per-column trace of this build, and the eigen test module.
set -o pipefail
O=${1:-gpurun_out/r6c}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=pods-digital-filter_amd/podsgen/variants
for i in 1 2; do
  timeout -k 10 120 python -u tools/syev_ab.py 10 > $O/syev_new_$i.log 2>&1 || exit 2
  PODSGEN_LIB=$V/r5/libpodsgen.so timeout -k 10 120 python -u tools/syev_ab.py 10 > $O/syev_r5_$i.log 2>&1 || exit 3
done
timeout -k 10 200 python -u tools/trd_trace.py 4096 0 255 > $O/trd_trace.log 2>&1 || exit 4
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_eigen.py > $O/eigen_tests.log 2>&1 || exit 5
echo trd-ab-done
