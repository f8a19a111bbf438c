#!/bin/bash
# Counters of the int8 correlation kernels (k_residues, k_syrk_i8, k_crt) at C3, one rocprofv3
# --pmc pass per group, from the repo root on the box:  bash tools/corr_i8_pmc.sh gpurun_out/i8pmc
# Summary: python tools/pmc_summary.py gpurun_out/i8pmc i8::
set -o pipefail
OUT=${1:-gpurun_out/i8pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
RUN="python tools/corr_i8_probe.py 256 256 4096 2"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace -d $OUT/p1 -o run --output-format csv -- $RUN > $OUT/p1.log 2>&1 || exit 2
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/p2 -o run --output-format csv -- $RUN > $OUT/p2.log 2>&1 || exit 3
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum --kernel-trace -d $OUT/p3 -o run --output-format csv -- $RUN > $OUT/p3.log 2>&1 || exit 4
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_I8 SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU --kernel-trace -d $OUT/p4 -o run --output-format csv -- $RUN > $OUT/p4.log 2>&1 || exit 5
echo pmc-done
