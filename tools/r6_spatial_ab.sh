#!/bin/bash
# k_spatial_modes variants (register budget / loads per group) against the product at C3, alternating
# processes (tools/spatial_ab.py), then the spatial-mode parity tests under the fastest candidate.
set -o pipefail
O=${1:-gpurun_out/r6sp}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=$GRAFT_REPO_ROOT/pods-digital-filter_amd/podsgen/variants
for i in 1 2; do
  timeout -k 10 120 python -u tools/spatial_ab.py 20 > $O/prod_$i.log 2>&1 || exit 2
  for v in spu4 spc256u4 spc128u4 spc256u8 spxc4w3 spxc4 spxc8; do
    PODSGEN_LIB=$V/libpodsgen_$v.so timeout -k 10 120 python -u tools/spatial_ab.py 20 > $O/${v}_$i.log 2>&1 || exit 3
  done
done
echo sp-done
