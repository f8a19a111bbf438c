#!/bin/bash
# Wave-stall counters of the generator kernels (k_mt_generate_full, k_filter_x2, k_filter_yz),
# one rocprofv3 --pmc pass per counter group, from the repo root on the box:
#   bash tools/gen_stall_pmc.sh gpurun_out/genstall
set -o pipefail
OUT=${1:-gpurun_out/genstall}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY --kernel-trace -d $OUT/p1 -o run --output-format csv -- python tools/stage_probe.py 256 256 4096 1 > $OUT/p1.log 2>&1 || exit 2
echo pmc-done
