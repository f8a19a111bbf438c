#!/bin/bash
# The x pass beside the solver's tail at 1 / 1.5 / 2 (product) / 3 workgroups per CU
# (variants/libpodsgen_xc{2,3,6}.so, -DPODS_XPASS_CAP in halves); C3 bench, alternating processes.
set -o pipefail
O=${1:-gpurun_out/r6xc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=$GRAFT_REPO_ROOT/pods-digital-filter_amd/podsgen/variants
B="python3 -u bench.py --steps 20 --warmup 5 --no-cpu"
for i in 1 2; do
  timeout -k 10 170 $B > $O/bench_xc4_$i.json 2>> $O/err.log || exit 2
  for c in 2 3 6; do
    PODSGEN_LIB=$V/libpodsgen_xc$c.so timeout -k 10 170 $B > $O/bench_xc${c}_$i.json 2>> $O/err.log || exit 3
  done
done
echo xcap-done
