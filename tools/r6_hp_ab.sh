#!/bin/bash
# One device: the main stream at high priority (PODS_HP_MAIN=1: the solver's persistent kernels get
# the CUs before the generator work beside them) against the default stream; C3 bench, alternating.
set -o pipefail
O=${1:-gpurun_out/r6hp}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 -u bench.py --steps 20 --warmup 5 --no-cpu"
for i in 1 2; do
  timeout -k 10 170 $B > $O/bench_prod_$i.json 2>> $O/err.log || exit 2
  PODS_HP_MAIN=1 timeout -k 10 170 $B > $O/bench_hp_$i.json 2>> $O/err.log || exit 3
done
echo hp-done
