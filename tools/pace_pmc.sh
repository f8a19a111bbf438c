#!/bin/bash
# L2 and MFMA counters of the int8 SYRK, persistent XCD-paced (default) against the grid form
# (PODS_SYRK_PACE=0), one rocprofv3 --pmc pass per counter group and variant, from the repo root on
# the box:  bash tools/pace_pmc.sh gpurun_out/pacepmc ; python tools/pmc_summary.py DIR/<variant> syrk
set -o pipefail
OUT=${1:-gpurun_out/pacepmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
RUN="python tools/corr_i8_probe.py 256 256 4096 2"
for v in paced grid; do
  if [ $v = grid ]; then export PODS_SYRK_PACE=0; else unset PODS_SYRK_PACE; fi
  timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $OUT/$v/l2 -o run --output-format csv -- $RUN > $OUT/$v-l2.log 2>&1 || exit 2
  timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --kernel-trace -d $OUT/$v/mfma -o run --output-format csv -- $RUN > $OUT/$v-mfma.log 2>&1 || exit 3
done
echo pace-pmc-done
