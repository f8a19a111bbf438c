#!/bin/bash
# One device: the spatial-mode pass on its own stream beside the next step's generation, the steps
# alternating between the two snapshot banks (PODS_OVERLAP_SPATIAL=1) against the default; the
# overlap's parity test first, then the C3 bench, alternating processes.
set -o pipefail
O=${1:-gpurun_out/r6ovl}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "overlapping or prefetch" > $O/tests.log 2>&1 || exit 2
B="python3 -u bench.py --steps 20 --warmup 5 --no-cpu"
for i in 1 2; do
  timeout -k 10 170 $B > $O/bench_prod_$i.json 2>> $O/err.log || exit 3
  PODS_OVERLAP_SPATIAL=1 timeout -k 10 170 $B > $O/bench_ovl_$i.json 2>> $O/err.log || exit 4
done
echo ovl-done
