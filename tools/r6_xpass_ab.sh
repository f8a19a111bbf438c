#!/bin/bash
# Whole-step A/B at C3: the next step's x pass beside this step's bisection / eigenvectors /
# back-transformation (PODS_XPASS_BESIDE=1, behind pods_syev's tail marker) against the default
# (x pass on the main stream), behind the eigenvalues (=2), and both with 2 workgroups per CU (=3, =4), alternating processes; results (nm, num_valid, N_FC) compared.
set -o pipefail
O=${1:-gpurun_out/r6xp}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 -u bench.py --steps 20 --warmup 5 --no-cpu"
for i in 1 2; do
  timeout -k 10 170 $B > $O/bench_prod_$i.json 2>> $O/err.log || exit 2
  PODS_XPASS_BESIDE=1 timeout -k 10 170 $B > $O/bench_xpass_$i.json 2>> $O/err.log || exit 3
  PODS_XPASS_BESIDE=2 timeout -k 10 170 $B > $O/bench_xpass2_$i.json 2>> $O/err.log || exit 4
  PODS_XPASS_BESIDE=3 timeout -k 10 170 $B > $O/bench_xpass3_$i.json 2>> $O/err.log || exit 5
  PODS_XPASS_BESIDE=4 timeout -k 10 170 $B > $O/bench_xpass4_$i.json 2>> $O/err.log || exit 6
done
echo xpass-done
