#!/bin/bash
# MFMA utilisation and effective clock of the fp64 MFMA kernels (SYRK at C3, the Chebyshev step):
# GRBM_GUI_ACTIVE over the kernel's duration = the clock it ran at; SQ_VALU_MFMA_BUSY_CYCLES /
# (GRBM_GUI_ACTIVE x SIMDs) = MfmaUtil.  From the repo root on the box:
#   bash tools/mfma_util_pmc.sh gpurun_out/mfmautil
set -o pipefail
OUT=${1:-gpurun_out/mfmautil}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
CTR="GRBM_GUI_ACTIVE GRBM_COUNT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_BUSY_CU_CYCLES SQ_CYCLES"
timeout -s KILL 120 rocprofv3 --pmc $CTR --kernel-trace -d $OUT/syrk -o run --output-format csv -- python tools/syrk_probe.py 256 256 4096 3 > $OUT/syrk.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc $CTR --kernel-trace -d $OUT/cheb -o run --output-format csv -- python tools/cheb_bench.py 20 > $OUT/cheb.log 2>&1 || exit 3
echo pmc-done
