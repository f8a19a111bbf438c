#!/bin/bash
# One device: the next step's jump-ahead ahead of its planes beside the late tridiagonalisation
# ranges (PODS_JUMP_WITH_PLANES=1) against beside this step's mean and residues (default); C3
# bench, alternating processes; then the prefetch parity tests under it.
set -o pipefail
O=${1:-gpurun_out/r6jwp}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 -u bench.py --steps 20 --warmup 5 --no-cpu"
for i in 1 2; do
  timeout -k 10 170 $B > $O/bench_prod_$i.json 2>> $O/err.log || exit 2
  PODS_JUMP_WITH_PLANES=1 timeout -k 10 170 $B > $O/bench_jwp_$i.json 2>> $O/err.log || exit 3
done
PODS_JUMP_WITH_PLANES=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "prefetch" > $O/prefetch_tests_jwp.log 2>&1 || exit 4
echo jwp-done
