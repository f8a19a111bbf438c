#!/bin/bash
# L2 behaviour of k_syrk_i8 under the tile orders (PODS_CORR_ORDER): TCC hits / misses and the
# fabric read requests, one rocprofv3 pass per order.  bash tools/corr_i8_l2.sh gpurun_out/i8l2
set -o pipefail
OUT=${1:-gpurun_out/i8l2}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for o in i x s; do
  PODS_CORR_ORDER=$o timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --kernel-trace -d $OUT/$o -o run --output-format csv -- python tools/corr_i8_probe.py 256 256 4096 2 > $OUT/$o.log 2>&1 || exit 2
done
echo l2-done
