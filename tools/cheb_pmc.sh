#!/bin/bash
# Counters of the Chebyshev step (k_cheb) at n = 4096, m = 64, one rocprofv3 --pmc pass per
# group (each within the per-block limits), from the repo root on the box:
#   bash tools/cheb_pmc.sh gpurun_out/chebpmc
set -o pipefail
OUT=${1:-gpurun_out/chebpmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT --kernel-trace -d $OUT/p1 -o run --output-format csv -- python tools/cheb_bench.py 20 > $OUT/p1.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/p2 -o run --output-format csv -- python tools/cheb_bench.py 20 > $OUT/p2.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 --kernel-trace -d $OUT/p3 -o run --output-format csv -- python tools/cheb_bench.py 20 > $OUT/p3.log 2>&1 || exit 4
echo pmc-done
