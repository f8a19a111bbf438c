#!/bin/bash
# Stall / issue counters and cache traffic of k_residues at C3 (one rocprofv3 --pmc pass per counter
# group), from the repo root on the box:  bash tools/residues_pmc.sh gpurun_out/respmc [PODS_RES_I8 value]
set -o pipefail
OUT=${1:-gpurun_out/respmc}
mkdir -p $OUT
[ -n "$2" ] && export PODS_RES_I8=$2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
RUN="python tools/corr_i8_probe.py 256 256 4096 1"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --kernel-trace -d $OUT/p1 -o run --output-format csv -- $RUN > $OUT/p1.log 2>&1 || exit 2
timeout -s KILL 150 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $OUT/p2 -o run --output-format csv -- $RUN > $OUT/p2.log 2>&1 || exit 3
echo res-pmc-done
