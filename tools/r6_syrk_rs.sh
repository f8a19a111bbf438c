#!/bin/bash
# SYRK A/B: the product library against the register-staged variant (PODS_SYRK_RS=1,
# variants/libpodsgen_rs.so): exactness tests under the variant, then alternating processes.
set -o pipefail
O=${1:-gpurun_out/r6rs}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=$GRAFT_REPO_ROOT/pods-digital-filter_amd/podsgen/variants/libpodsgen_rs.so
PODSGEN_LIB=$V timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_corr_i8.py > $O/tests_rs.log 2>&1 || exit 2
for i in 1 2 3; do
  timeout -k 10 120 python3 -u tools/corr_i8_ab.py 5 - > $O/prod_$i.log 2>&1 || exit 3
  PODSGEN_LIB=$V timeout -k 10 120 python3 -u tools/corr_i8_ab.py 5 - > $O/rs_$i.log 2>&1 || exit 4
done
echo rs-done
