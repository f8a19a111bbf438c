#!/bin/bash
# k_residues occupancy cap (amdgpu_waves_per_eu max 3 = product, 4, 5, 8): the whole pods_corr at C3
# (tools/corr_i8_ab.py: residues + SYRK + CRT, C checksum) in alternating processes.
set -o pipefail
O=${1:-gpurun_out/r6res}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=$GRAFT_REPO_ROOT/pods-digital-filter_amd/podsgen/variants
for i in 1 2; do
  timeout -k 10 120 python3 -u tools/corr_i8_ab.py 5 - > $O/prod_$i.log 2>&1 || exit 2
  for w in 4 5 8; do
    PODSGEN_LIB=$V/libpodsgen_res$w.so timeout -k 10 120 python3 -u tools/corr_i8_ab.py 5 - > $O/res${w}_$i.log 2>&1 || exit 3
  done
done
echo res-done
