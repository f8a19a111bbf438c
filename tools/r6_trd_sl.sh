#!/bin/bash
# k_trd LDS-slot choices for ranges 3-5 (pods_syev at n = 4096, alternating processes against the
# product), the one-GPU pipelined-runner test, and the C3 bench with the one-GPU pipelined runner
# (PODS_N1_PIPELINE=1) against the default.
set -o pipefail
O=${1:-gpurun_out/r6sl}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=$GRAFT_REPO_ROOT/pods-digital-filter_amd/podsgen/variants
for i in 1 2; do
  timeout -k 10 120 python -u tools/syev_ab.py 10 > $O/syev_prod_$i.log 2>&1 || exit 2
  for v in sl3a sl3b sl45; do
    PODSGEN_LIB=$V/libpodsgen_$v.so timeout -k 10 120 python -u tools/syev_ab.py 10 > $O/syev_${v}_$i.log 2>&1 || exit 3
  done
done
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_dropin.py -k one_gpu_pipelined > $O/n1_pipe_test.log 2>&1 || exit 4
B="python3 -u bench.py --steps 20 --warmup 5 --no-cpu"
timeout -k 10 200 $B > $O/bench_default.json 2>> $O/err.log || exit 5
PODS_N1_PIPELINE=1 timeout -k 10 200 $B > $O/bench_n1pipe.json 2>> $O/err.log || exit 6
echo sl-done
