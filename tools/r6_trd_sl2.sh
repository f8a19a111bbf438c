#!/bin/bash
# Whole-step A/B: the product against range 3 with no LDS slot (variants/libpodsgen_sl3b.so) and
# range 2 with 3 LDS slots (libpodsgen_sl2c.so) in alternating bench processes; the one-GPU
# pipelined-runner test; the C3 bench with the one-GPU pipelined runner (PODS_N1_PIPELINE=1).
set -o pipefail
O=${1:-gpurun_out/r6sl2}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=$GRAFT_REPO_ROOT/pods-digital-filter_amd/podsgen/variants
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_dropin.py -k "one_gpu_pipelined or world1" > $O/n1_pipe_test.log 2>&1 || exit 2
for i in 1 2; do
  timeout -k 10 120 python -u tools/syev_ab.py 10 > $O/syev_prod_$i.log 2>&1 || exit 3
  PODSGEN_LIB=$V/libpodsgen_sl2c.so timeout -k 10 120 python -u tools/syev_ab.py 10 > $O/syev_sl2c_$i.log 2>&1 || exit 3
done
B="python3 -u bench.py --steps 20 --warmup 5 --no-cpu"
for i in 1 2; do
  timeout -k 10 200 $B > $O/bench_prod_$i.json 2>> $O/err.log || exit 4
  PODSGEN_LIB=$V/libpodsgen_sl3b.so timeout -k 10 200 $B > $O/bench_sl3b_$i.json 2>> $O/err.log || exit 5
done
PODS_N1_PIPELINE=1 timeout -k 10 200 $B > $O/bench_n1pipe.json 2>> $O/err.log || exit 6
echo sl2-done
