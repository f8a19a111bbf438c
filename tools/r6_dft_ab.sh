#!/bin/bash
# One device: the speculative Fourier stage beside the spatial pass (PODS_DFT_EARLY=1: its side
# stream waits for T only) against behind it (default); C3 bench, alternating processes; then the
# Fourier parity tests under it.
set -o pipefail
O=${1:-gpurun_out/r6dft}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 -u bench.py --steps 20 --warmup 5 --no-cpu"
for i in 1 2; do
  timeout -k 10 170 $B > $O/bench_prod_$i.json 2>> $O/err.log || exit 2
  PODS_DFT_EARLY=1 timeout -k 10 170 $B > $O/bench_early_$i.json 2>> $O/err.log || exit 3
done
PODS_DFT_EARLY=1 timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "fourier or prefetch or speculative" > $O/tests_early.log 2>&1 || exit 4
echo dft-done
