#!/bin/bash
# k_trd A/B on the box (one call): this build vs the r5 build (pods_syev at n = 4096, alternating
# processes), the V-store diagnostic variants (no V stores: wrong vectors; nontemporal V stores),
# traces, and the eigen + syev2 test modules.
set -o pipefail
O=${1:-gpurun_out/r6g}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=pods-digital-filter_amd/podsgen/variants
for i in 1 2; do
  timeout -k 10 120 python -u tools/syev_ab.py 10 > $O/syev_new_$i.log 2>&1 || exit 2
  PODSGEN_LIB=$V/r5/libpodsgen.so timeout -k 10 120 python -u tools/syev_ab.py 10 > $O/syev_r5_$i.log 2>&1 || exit 3
done
timeout -k 10 200 python -u tools/trd_trace.py 4096 0 255 > $O/trd_trace.log 2>&1 || exit 6
timeout -k 10 200 python -u tools/trd_hop.py 4096 > $O/trd_hop.log 2>&1 || exit 7
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_eigen.py tests/test_gpu_syev2.py > $O/eigen_tests.log 2>&1 || exit 8
echo trd-ab2-done
