#!/bin/bash
# Check of the current defaults: the prefetch parity tests, the one-GPU pipelined tests, then the
# C3 bench twice.
set -o pipefail
O=${1:-gpurun_out/r6chk}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "prefetch or speculative" tests/test_gpu_dropin.py -k "prefetch or pipelined or one_gpu" > $O/tests.log 2>&1 || exit 2
B="python3 -u bench.py --steps 20 --warmup 5 --no-cpu"
for i in 1 2; do
  timeout -k 10 170 $B > $O/bench_$i.json 2>> $O/err.log || exit 3
done
echo check-done
