#!/bin/bash
# One GPU call: exactness of the interleaved-DMA SYRK variants, their A/B, and the PMC passes of
# one of them.  From the repo root on the box:  bash tools/syrk_ilv_round.sh gpurun_out/ilv i5
set -o pipefail
OUT=${1:-gpurun_out/ilv}
PMCV=${2:-i5}
mkdir -p $OUT
for v in i5 i6 i7; do
  PODS_SYRK_I8=$v timeout -k 10 120 python -u -m pytest tests/test_gpu_corr_i8.py -x -q --timeout 100 \
    --timeout-method thread -p no:cacheprovider > $OUT/tests_$v.log 2>&1 || exit 2
  echo "$v: $(tail -1 $OUT/tests_$v.log)"
done
timeout -k 10 400 python -u tools/corr_i8_ab.py 5 PODS_SYRK_I8=i5 PODS_SYRK_I8=i6 PODS_SYRK_I8=i7 PODS_SYRK_I8=i2 PODS_SYRK_I8=i5,PODS_CORR_SPLITS=4 PODS_SYRK_I8=i5,PODS_CORR_SPLITS=1 \
  > $OUT/ab.log 2>&1 || exit 3
tail -6 $OUT/ab.log
export PODS_SYRK_I8=$PMCV
bash tools/corr_i8_pmc.sh $OUT/pmc || exit 4
