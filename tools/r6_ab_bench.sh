#!/bin/bash
# Whole-step A/B on one box: C3 bench with the default engine, with the next step's jump-ahead
# beside the solver's tail (PODS_JUMP_BESIDE=1), with the 4-row spatial-mode kernel
# (PODS_SPATIAL4=1), both; then the parity module with the 4-row kernel.
set -o pipefail
O=${1:-gpurun_out/r6h}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 -u bench.py --steps 20 --warmup 5 --no-cpu"
for i in 1 2; do
  timeout -k 10 200 $B > $O/base_$i.json 2>> $O/err.log || exit 2
  PODS_JUMP_BESIDE=1 timeout -k 10 200 $B > $O/jb_$i.json 2>> $O/err.log || exit 3
  PODS_SPATIAL4=1 timeout -k 10 200 $B > $O/s4_$i.json 2>> $O/err.log || exit 4
  PODS_JUMP_BESIDE=1 PODS_SPATIAL4=1 timeout -k 10 200 $B > $O/both_$i.json 2>> $O/err.log || exit 5
done
PODS_SPATIAL4=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py > $O/parity_s4.log 2>&1 || exit 6
echo ab-bench-done
