#!/bin/bash
# One device: the next step's random planes behind tridiagonalisation range 2 (default), 3 or 4
# (PODS_PLANES_AFTER); C3 bench, alternating processes.
set -o pipefail
O=${1:-gpurun_out/r6pl}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 -u bench.py --steps 20 --warmup 5 --no-cpu"
for i in 1 2; do
  for a in 3 4 5; do
    PODS_PLANES_AFTER=$a timeout -k 10 170 $B > $O/bench_after${a}_$i.json 2>> $O/err.log || exit 2
  done
done
echo planes-done
